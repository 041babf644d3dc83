// TEST-ONLY host build of refpath_core.h (serial single-lane context), same
// inputs/outputs as htp_init_ref_path_batch.  The product never loads it.
#include <cmath>
#include <cstdint>
#include <vector>

#define HTP_HD
#include "../../include/htp.h"
#include "wave_ctx.h"
#include "refpath_core.h"

using namespace htp;

extern "C" int htp_hostsim_init_ref_path(const htp_refpath_batch* in, htp_refpath_result* out) {
  std::vector<double> scr((size_t)rp::SCRATCH_PER_POINT * (size_t)in->cap_points);
  for (int b = 0; b < in->batch; ++b) {
    const int a0 = in->path_off[b], a1 = in->path_off[b + 1];
    const double* prm = in->params + 3 * (int64_t)b;
    rp::Out o{};
    if (a0 < 0 || a1 < a0 || a1 - a0 > in->cap_points || !(prm[2] > 0.0)) {
      o.status = rp::ST_BAD_INPUT;
    } else {
      HostLane c;
      rp::Course<HostLane> K{c, in->xs + a0, in->ys + a0, in->dirs + a0, a1 - a0, prm[0], prm[1], prm[2],
                             scr.data(), in->cap_points};
      K.run(o, out->traj + (int64_t)b * in->cap_rows * 5, in->cap_rows);
    }
    out->status[b] = o.status;
    out->n_rows[b] = o.n_rows;
  }
  return 0;
}
