// TEST-ONLY host build of the orchard workload chain (chain_core.h + classic / refpath / oge cores, serial
// single-lane context), the same stage sequence as htp_orchard_chain_device on host arrays.  Lets CPU tests
// compare the device chain's arithmetic with the host generator (synth.make_orchard_instance).
#include <cstdint>
#include <vector>

#define HTP_HD
#include "../../include/htp.h"
#include "wave_ctx.h"
#include "classic_batch.h"
#include "oge_batch.h"
#include "refpath_core.h"
#include "chain_core.h"

using namespace htp;

extern "C" int htp_hostsim_chain(const htp_chain_batch* in) {
  const int B = in->batch, N = in->N, M = in->M, cap = in->turns.cap_path, cr = in->cap_rows;
  chain::Vehicle V{};
  V.npoly = in->n_vpoly;
  for (int k = 0; k < V.npoly; ++k) {
    V.nv[k] = in->vpoly_nv[k];
    for (int j = 0; j < V.nv[k]; ++j) { V.v[k][j][0] = in->vpoly[k][j][0]; V.v[k][j][1] = in->vpoly[k][j][1]; }
  }
  std::vector<int32_t> cst(B), cn(B);
  std::vector<double> cpath((size_t)B * cap * 5), cws((size_t)ct::SCR_PER_POINT * in->turns.cap_samples);
  std::vector<rs::Path> paths(rs::MAXP);
  std::vector<int> flags(rs::MAXP);
  htp_classic_result cres{cst.data(), cn.data(), cpath.data()};
  std::vector<double> xs(cap), ys(cap), dirs(cap), steps(cap), rpw((size_t)rp::SCRATCH_PER_POINT * cap), prm(3);
  std::vector<double> ref((size_t)cr * 5), s(cr);
  static oge::PolyOut po;
  for (int b = 0; b < B; ++b) {
    HostLane c;
    ct::run_problem(c, in->turns, cres, b, cws.data(), paths.data(), flags.data());
    int st = 0;
    if (cst[b] != 0) st = 16 + cst[b];
    rp::Out o{};
    if (st == 0) {
      const int n = cn[b];
      chain::prep(cpath.data() + (size_t)b * cap * 5, n, N, in->dT, in->wheel_base, xs.data(), ys.data(), dirs.data(),
                  steps.data(), prm.data());
      rp::Course<HostLane> K{c, xs.data(), ys.data(), dirs.data(), n, prm[0], prm[1], prm[2], rpw.data(), cap};
      K.run(o, ref.data(), cr);
      if (o.status != 0 || o.n_rows < 2) st = 32 + (o.status ? o.status : 15);
    }
    double* p = const_cast<double*>(in->scenes.params) + (size_t)b * HTP_OGE_NPARAM;
    oge::SceneIn sc;
    oge::Scene S;
    if (st == 0) {
      sc.nrows = (int)p[HTP_OGE_P_NROWS];
      sc.row_width = p[HTP_OGE_P_ROWW];
      sc.row_length = p[HTP_OGE_P_ROWLEN];
      sc.slope = p[HTP_OGE_P_SLOPE];
      sc.tree_width = p[HTP_OGE_P_TREEW];
      sc.row_draws = in->scenes.row_draws + (size_t)b * in->scenes.max_rows;
      sc.eps_draws = in->scenes.eps_draws + (size_t)b * in->scenes.max_rows;
      for (int j = 0; j < 3; ++j) { sc.start[j] = p[HTP_OGE_P_SX + j]; sc.end[j] = p[HTP_OGE_P_EX + j]; }
      sc.side = (int)p[HTP_OGE_P_SIDE];
      oge::make_rows(sc, S);
      p[HTP_OGE_P_HW] = chain::resample_hw(ref.data(), o.n_rows, N, s.data(), in->traj + (size_t)b * N * 5, V, S,
                                           in->margin[b]);
      sc.headland_width = p[HTP_OGE_P_HW];
      const int og = oge::produce(sc, po);
      if (og != 0) st = 48 + og;
    }
    if (st == 0 && chain::pack(po, sc, S, in->traj + (size_t)b * N * 5, N, ref.data(), o.n_rows, V, M,
                               in->obs_A + (size_t)b * M * 8, in->obs_b + (size_t)b * M * 4))
      st = 65;
    in->status[b] = st;
  }
  return 0;
}
