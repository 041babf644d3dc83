// TEST-ONLY host build of the Reeds-Shepp core (rs_core.h), one query at a
// time, in the same CSR format as htp_rs_all_paths_batch.  Lets tests pin the
// device code's logic bit-for-bit against the reference goldens without a GPU.
#define HTP_HD
#include "rs_host.h"

extern "C" int htp_hostsim_rs(const double* q, int64_t cap_paths, int64_t cap_points, int32_t* n_paths,
                              int64_t* n_points, double* lengths, int8_t* ctypes, double* L, int64_t* point_offsets,
                              double* x, double* y, double* yaw, double* cs, int8_t* dir) {
  return htp::rs::all_paths_host(q, cap_paths, cap_points, n_paths, n_points, lengths, ctypes, L, point_offsets, x, y,
                                 yaw, cs, dir);
}
