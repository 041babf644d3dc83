// TEST-ONLY: 64-lane wavefront simulation of the solver core on the CPU
// (one std::thread per lane, std::barrier for sync, shared-array reductions),
// to debug lane-parallel logic (races, out-of-bounds via ASan) without a GPU.
#include <barrier>
#include <thread>
#include <vector>

#define HTP_HD
#include "wave_ctx.h"
#include "obca_batch.h"
#include "thread_wave.h"

using namespace htp;


extern "C" int htp_threadsim_obca_solve(const htp_obca_batch* in, htp_obca_result* out, int max_iter) {
  const char* e = nullptr;
  if (check_shape(in, &e)) return -1;
  Options o = default_options();
  if (max_iter >= 0) o.max_iter = max_iter;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  Layout L = make_layout(D);
  BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
              in->init_control, in->init_mu, in->init_lambda};
  for (int p = 0; p < in->batch; ++p) {
    std::vector<double> ws((size_t)L.total, 0.0);
    std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128, 0.0);
    std::vector<int> ilds(2 * NBMAX, 0);
    WaveShared sh;
    std::vector<Result> rr(64);
    std::vector<std::thread> th;
    for (int lane = 0; lane < 64; ++lane)
      th.emplace_back([&, lane]() {
        ThreadWave c{lane, lds.data(), ilds.data(), &sh};
        ProblemIn pin = problem_view(b, D, p);
        ObcaSolver<ThreadWave, MAXE, MAXE> S(c, D, L, o, pin, ws.data());
        S.run(rr[lane]);
      });
    for (auto& t : th) t.join();
    Result r = rr[0];
    for (int q = 0; q < D.n; ++q) out->x[(size_t)p * D.n + q] = ws[L.x + q];
    if (out->objective) out->objective[p] = r.objective;
    if (out->status) out->status[p] = r.status;
    if (out->iterations) out->iterations[p] = r.iters;
    if (out->n_factor) out->n_factor[p] = r.n_factor;
    if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
      if (out->n_resto) out->n_resto[p] = r.n_resto;
  }
  return 0;
}
