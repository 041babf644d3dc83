// Host (serial) driver of the Reeds-Shepp core for one pose pair, in the CSR
// format of htp_rs_all_paths_batch.  Shared by the CPU build (libhtp_cpu.so:
// the workload generator's fish-tail warm starts, before any GPU call) and the
// test-only host simulation (rs_hostsim.cpp).
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

#include "rs_core.h"

namespace htp {
namespace rs {

// q = [sx, sy, syaw, gx, gy, gyaw, maxc, step]; returns 0, 1 (a word shorter than 0.01: the
// reference's AssertionError) or 2 (sampler overrun).  Arrays are written only while they fit
// (cap_paths / cap_points); n_paths / n_points always receive the full sizes.
inline int all_paths_host(const double* q, int64_t cap_paths, int64_t cap_points, int32_t* n_paths,
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

}  // namespace rs
}  // namespace htp
