// One scene of an htp_oge_batch -> its htp_oge_result slots (polygons + halfspaces); shared by the
// gfx950 kernel (htp_oge.hip) and the test-only host build (oge_hostsim.cpp).
#pragma once
#include "../../include/htp.h"
#include "oge_core.h"

namespace htp {
namespace oge {

static_assert(MAXPOLY == HTP_OGE_MAXPOLY && MAXV == HTP_OGE_MAXV && MAXR == HTP_OGE_MAXROWS, "htp.h OGE caps");

HTP_HD inline void run_scene(const htp_oge_batch& in, const htp_oge_result& out, int64_t s) {
  const double* p = in.params + s * HTP_OGE_NPARAM;
  SceneIn sc;
  sc.nrows = (int)p[HTP_OGE_P_NROWS];
  sc.row_width = p[HTP_OGE_P_ROWW];
  sc.row_length = p[HTP_OGE_P_ROWLEN];
  sc.slope = p[HTP_OGE_P_SLOPE];
  sc.tree_width = p[HTP_OGE_P_TREEW];
  sc.headland_width = p[HTP_OGE_P_HW];
  sc.row_draws = in.row_draws + s * in.max_rows;
  sc.eps_draws = in.eps_draws + s * in.max_rows;
  for (int j = 0; j < 3; ++j) {
    sc.start[j] = p[HTP_OGE_P_SX + j];
    sc.end[j] = p[HTP_OGE_P_EX + j];
  }
  sc.side = (int)p[HTP_OGE_P_SIDE];
  PolyOut po;
  int st = sc.nrows > in.max_rows ? (int)ST_BAD_INPUT : produce(sc, po);
  if (st != OK) po.n = 0;
  out.status[s] = st;
  out.n_poly[s] = po.n;
  const int64_t base = s * MAXPOLY;
  for (int q = 0; q < MAXPOLY; ++q) {
    const int nv = q < po.n ? po.nv[q] : 0;
    out.n_vert[base + q] = nv;
    double* v = out.vertices + (base + q) * MAXV * 2;
    for (int j = 0; j < nv; ++j) { v[2 * j] = po.xy[q][j][0]; v[2 * j + 1] = po.xy[q][j][1]; }
    if (out.n_facet) {
      double* A = out.A + (base + q) * MAXV * 2;
      double* b = out.b + (base + q) * MAXV;
      out.n_facet[base + q] = q < po.n ? halfspaces(po.xy[q], nv, A, b) : 0;
    }
  }
}

}  // namespace oge
}  // namespace htp
