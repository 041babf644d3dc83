// TEST-ONLY host build of the orchard scene -> OBCA obstacle producer (oge_core.h), same
// batch/result structs as htp_oge_obstacles_batch.  Lets CPU tests pin the device code's logic
// against the Python restatement (path_planner/OGE_OBCA.py) without a GPU.
#include <cstdint>

#define HTP_HD
#include "oge_batch.h"

extern "C" int htp_hostsim_oge(const htp_oge_batch* in, htp_oge_result* out) {
  for (int64_t s = 0; s < in->batch; ++s) htp::oge::run_scene(*in, *out, s);
  return 0;
}
