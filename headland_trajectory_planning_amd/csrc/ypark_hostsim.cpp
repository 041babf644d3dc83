// TEST-ONLY host build of the Y-park grid search core (ypark_core.h), serial
// lane; same inputs/outputs as htp_ypark_search_batch.  The product never
// loads this library.
#include <cmath>
#include <cstdint>
#include <vector>

#define HTP_HD
#include "../../include/htp.h"
#include "wave_ctx.h"
#include "ypark_core.h"

using namespace htp;

extern "C" int htp_hostsim_ypark(const htp_ypark_batch* in, htp_ypark_result* out) {
  std::vector<double> scr((size_t)yp::CH * yp::SCR);
  double body[2 * ha::MAXB];
  int32_t cnt[yp::CH], hit[yp::CH];
  ha::Geo g{in->poly_off, in->vertices, nullptr, nullptr, nullptr};
  for (int b = 0; b < in->batch; ++b) {
    HostLane c;
    yp::Search<HostLane> S(c, in->params + (int64_t)b * HTP_YP_NPARAM, in->desc + (int64_t)b * HTP_YP_NDESC, g,
                           in->axis, scr.data(), body, cnt, hit);
    yp::Out o{};
    S.run(o, out->path + (int64_t)b * in->cap_path * 5, in->cap_path);
    out->status[b] = o.status;
    out->cand[b] = o.cand;
    out->n_path[b] = o.n_path;
    out->params[4 * b] = o.bl;
    out->params[4 * b + 1] = o.fl;
    out->params[4 * b + 2] = o.sb;
    out->params[4 * b + 3] = o.sf;
    if (out->n_pose) out->n_pose[b] = o.n_pose;
  }
  return 0;
}
