// TEST-ONLY host build of the classic-turn planner (classic_core.h, serial single-lane context), same
// batch/result structs as htp_classic_turn_batch.  The product never loads it.
#include <cstdint>
#include <vector>

#define HTP_HD
#include "wave_ctx.h"
#include "classic_batch.h"

extern "C" int htp_hostsim_classic(const htp_classic_batch* in, htp_classic_result* out) {
  std::vector<double> scr((size_t)htp::ct::SCR_PER_POINT * (size_t)in->cap_samples);
  std::vector<htp::rs::Path> paths(htp::rs::MAXP);
  std::vector<int> flags(htp::rs::MAXP);
  for (int64_t b = 0; b < in->batch; ++b) {
    htp::HostLane c;
    htp::ct::run_problem(c, *in, *out, b, scr.data(), paths.data(), flags.data());
  }
  return 0;
}
