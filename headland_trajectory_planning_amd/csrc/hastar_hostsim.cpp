// TEST-ONLY host build of the hybrid A* core (hastar_core.h) with a serial
// single-lane context, same inputs/outputs as htp_hastar_search_batch.  Lets
// tests pin the device code's logic against the oracle without a GPU.  The
// product never loads this library (no CPU fallback).
#include <cmath>
#include <cstdint>
#include <vector>

#define HTP_HD
#include "../../include/htp.h"
#include "wave_ctx.h"
#include "hastar_core.h"

using namespace htp;
using namespace htp::ha;

extern "C" int htp_hostsim_hastar(const htp_hastar_batch* in, htp_hastar_result* out) {
  const int64_t cn = 4 + (int64_t)(in->max_nodes_cap + 1) * MAXMOT + 4;
  int64_t cs = 1;
  while (cs < 2 * cn) cs <<= 1;
  std::vector<Node> nodes((size_t)cn);
  std::vector<Slot> slots((size_t)cs);
  std::vector<double> hval((size_t)cn);
  std::vector<int32_t> hslot((size_t)cn);
  std::vector<double> dub((size_t)DUBW * (CAP_DUB + 16));
  Shared* sh = new Shared();
  Geo g{in->poly_off, in->vertices, in->lane_len, in->guide, in->motions};
  for (int b = 0; b < in->batch; ++b) {
    const double* prm = in->params + (int64_t)b * HTP_HA_NPARAM;
    const int32_t* d = in->desc + (int64_t)b * HTP_HA_NDESC;
    HostLane c;
    Work w{nodes.data(), slots.data(), hval.data(), hslot.data(), (int32_t)cn, (int32_t)cs, dub.data(), CAP_DUB};
    Search<HostLane> S(c, prm, d, g, w, *sh);
    Out o{};
    int32_t* log = out->expanded ? out->expanded + (int64_t)b * in->cap_log * 3 : nullptr;
    S.run(o, log, log ? in->cap_log : 0);
    int n_path = 0;
    if (o.status == ST_FOUND || o.status == ST_NO_PATH || o.status == ST_MAX_NODES) {
      const int64_t off = (int64_t)b * in->cap_path;
      int st = o.status;
      n_path = S.backtrack(w.hslot, w.cap_node, out->x + off, out->y + off, out->yaw + off, out->dir + off,
                           out->k + off, in->cap_path, st);
      o.status = st;
    }
    out->status[b] = o.status;
    out->counter[b] = o.counter;
    out->n_path[b] = n_path;
    if (out->n_expanded) out->n_expanded[b] = o.n_expanded;
    if (out->n_pose) out->n_pose[b] = o.n_pose;
  }
  delete sh;
  return 0;
}
