// TEST-ONLY host build of the Reeds-Shepp core (rs_core.h), one query at a
// time, in the same CSR format as htp_rs_all_paths_batch.  Lets tests pin the
// device code's logic bit-for-bit against the reference goldens without a GPU.
#include <cmath>
#include <cstdint>
#include <vector>

#define HTP_HD
#include "rs_core.h"

using namespace htp::rs;

extern "C" int htp_hostsim_rs(const double* q, int64_t cap_paths, int64_t cap_points, int32_t* n_paths,
                              int64_t* n_points, double* lengths, int8_t* ctypes, double* L, int64_t* point_offsets,
                              double* x, double* y, double* yaw, double* cs, int8_t* dir) {
  std::vector<Path> slots(MAXP);
  PathSet S{slots.data(), 0, 0};
  generate_paths(q[0], q[1], q[2], q[3], q[4], q[5], q[6], S);
  int status = S.err ? 1 : 0;
  const int np = S.err ? 0 : S.n;
  const double maxc = q[6], step = q[7];
  *n_paths = np;
  int64_t off = 0;
  if (point_offsets && cap_paths >= 0) point_offsets[0] = 0;
  for (int k = 0; k < np; ++k) {
    NullSink ns;
    int n = local_course(S.p[k], maxc, step * maxc, ns);
    if (n < 0) { status = 2; n = 0; }
    if (k < cap_paths) {
      for (int j = 0; j < 5; ++j) {
        lengths[k * 5 + j] = j < S.p[k].nseg ? S.p[k].len[j] / maxc : 0.0;
        ctypes[k * 5 + j] = S.p[k].typ[j];
      }
      L[k] = S.p[k].L / maxc;
      point_offsets[k + 1] = off + n;
      if (n > 0 && off + n <= cap_points) {
        GlobalSink gs{x + off, y + off, yaw + off, cs + off, dir + off, n, q[0], q[1], q[2], cos(-q[2]), sin(-q[2])};
        local_course(S.p[k], maxc, step * maxc, gs);
      }
    }
    off += n;
  }
  *n_points = off;
  return status;
}
