// One problem of an htp_classic_batch -> its htp_classic_result slots; shared by the gfx950 kernel
// (htp_classic.hip) and the test-only host build (classic_hostsim.cpp).
#pragma once
#include "../../include/htp.h"
#include "classic_core.h"

namespace htp {
namespace ct {

template <class C>
HTP_HD inline void run_problem(C& c, const htp_classic_batch& in, const htp_classic_result& out, int64_t b,
                               double* scr, rs::Path* paths, int* flags) {
  const double* p = in.params + b * HTP_CT_NPARAM;
  Spec sp;
  sp.type = (int)p[HTP_CT_P_TYPE];
  sp.side = (int)p[HTP_CT_P_SIDE];
  for (int j = 0; j < 3; ++j) {
    sp.start[j] = p[HTP_CT_P_SX + j];
    sp.end[j] = p[HTP_CT_P_EX + j];
  }
  sp.wb = p[HTP_CT_P_WB];
  sp.max_steer = p[HTP_CT_P_MAXSTEER];
  sp.radius = p[HTP_CT_P_RADIUS];
  sp.step = p[HTP_CT_P_STEP];
  const int32_t* d = in.desc + 3 * b;
  ha::Footprint fp{};
  fp.g.poly_off = in.poly_off;
  fp.g.vert = in.vertices;
  const int bo = in.poly_off[d[0]];
  fp.body = in.vertices + 2 * (int64_t)bo;
  fp.nb = in.poly_off[d[0] + 1] - bo;
  fp.blk0 = d[1];
  fp.blk1 = d[2];
  fp.field = -1;
  fp.lane0 = 0;
  fp.lane1 = 0;
  Turn<C> T{c, sp, fp, scr, in.cap_samples, out.path + b * (int64_t)in.cap_path * 5, in.cap_path, paths, flags};
  if (fp.nb < 3 || fp.nb > ha::MAXB) T.status = ST_BAD_INPUT;
  else T.run();
  if (c.lane == 0) {
    out.status[b] = T.status;
    out.n_path[b] = T.status == ST_OK ? T.n_out : 0;
  }
}

}  // namespace ct
}  // namespace htp
