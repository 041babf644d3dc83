// TEST-ONLY: the device solver reproduced on the host bit for bit (emu_wave.h): the same ObcaSolver
// instantiation the kernel launches (htp_obca.hip: <4, 4> for all-quadrilateral problems, else <MAXE, MAXE>;
// the point formulation <1, 4> / <1, MAXE>), run by 64 lane threads with the device's reduction and
// matrix-core order.  Built by tests/_hostsim.build_emusim() with clang++ -ffp-contract=on -mfma.
#include <thread>
#include <vector>

#define HTP_HD
#define HTP_EMU_WAVE 1
#include "emu_wave.h"
#include "obca_batch.h"

using namespace htp;

namespace {

template <int EN, int EM, int FORM, class Dm>
void solve_one(const Dm& D, const Layout& L, const Options& o, const BatchView& b, int64_t p, double* x_out,
               Result& res) {
  std::vector<double> ws((size_t)L.total, 0.0);
  std::vector<double> lds(LDS_WAVE_DOUBLES, 0.0);
  std::vector<int> ilds(2 * NBMAX, 0);
  EmuShared sh;
  std::vector<Result> rr(64);
  std::vector<std::thread> th;
  for (int lane = 0; lane < 64; ++lane)
    th.emplace_back([&, lane]() {
      EmuWave c{lane, lds.data(), ilds.data(), &sh};
      EmuWave::self = &c;
      Dm Dl = D;
      ProblemIn pin = problem_view(b, Dl, p);
      ObcaSolver<EmuWave, EN, EM, FORM> S(c, Dl, L, o, pin, ws.data());
      S.run(rr[lane]);
    });
  for (auto& t : th) t.join();
  res = rr[0];
  for (int q = 0; q < D.n; ++q) x_out[q] = ws[L.x + q];
}

void store(htp_obca_result* out, int64_t p, const Result& r) {
  if (out->objective) out->objective[p] = r.objective;
  if (out->status) out->status[p] = r.status;
  if (out->iterations) out->iterations[p] = r.iters;
  if (out->n_factor) out->n_factor[p] = r.n_factor;
  if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
  if (out->n_resto) out->n_resto[p] = r.n_resto;
}

int options(Options& o, const char** names, const double* values, int nopt) {
  o = default_options();
  o.wall_rate = 1e9;
  for (int k = 0; k < nopt; ++k)
    if (set_option(o, names[k], values[k])) return -2;
  o.max_cpu_time = 0.0;   // no clock in the emulation
  return 0;
}

}  // namespace

extern "C" int htp_emusim_obca_solve(const htp_obca_batch* in, htp_obca_result* out, const char** names,
                                     const double* values, int nopt) {
  const char* e = nullptr;
  if (check_shape(in, &e)) return -1;
  Options o;
  if (options(o, names, values, nopt)) return -2;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  Layout L = make_layout(D);
  bool u44 = true;
  for (int m = 0; m < D.M; ++m) u44 = u44 && D.eo[m] == 4;
  for (int k = 0; k < D.K; ++k) u44 = u44 && D.eb[k] == 4;
  BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
              in->init_control, in->init_mu, in->init_lambda};
  for (int64_t p = 0; p < in->batch; ++p) {
    Result r{};
    if (u44) solve_one<4, 4, 0>(D, L, o, b, p, out->x + p * D.n, r);
    else solve_one<MAXE, MAXE, 0>(D, L, o, b, p, out->x + p * D.n, r);
    store(out, p, r);
  }
  return 0;
}

extern "C" int htp_emusim_obca_points_solve(const htp_obca_points_batch* in, htp_obca_result* out,
                                            const char** names, const double* values, int nopt) {
  const char* e = nullptr;
  if (check_shape_points(in, &e)) return -1;
  Options o;
  if (options(o, names, values, nopt)) return -2;
  Dims D;
  make_dims_points(D, in->N, in->M, in->n_vertices, in->obs_edges);
  Layout L = make_layout(D);
  bool u4 = true;
  for (int m = 0; m < D.M; ++m) u4 = u4 && D.eo[m] == 4;
  BatchView b = points_view(in);
  for (int64_t p = 0; p < in->batch; ++p) {
    Result r{};
    if (u4) solve_one<1, 4, 1>(D, L, o, b, p, out->x + p * D.n, r);
    else solve_one<1, MAXE, 1>(D, L, o, b, p, out->x + p * D.n, r);
    store(out, p, r);
  }
  return 0;
}
