// libhtp.so, the orchard workload chain on the device (chain_core.h): classic turn -> init guess ->
// resample + headland width -> obstacle producer -> quads / halfspaces, five launches on one stream with
// every intermediate in HBM (context-owned), one problem per wavefront (the producer: one per thread).
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "classic_batch.h"
#include "oge_batch.h"
#include "refpath_core.h"
#include "chain_core.h"

using namespace htp;

namespace {

struct ChainBufs {
  int32_t *ct_status, *ct_n;
  double* ct_path;                  // [B][cap_path][5]
  double* ct_ws;                    // classic scratch
  double *xs, *ys, *dirs, *steps;   // [B][cap_path]
  double* rp_params;                // [B][3]
  double* rp_ws;                    // refpath scratch [B][SCRATCH_PER_POINT * cap_path]
  int32_t *rp_status, *rp_rows;
  double* rp_traj;                  // [B][cap_rows][5]
  double* s;                        // [B][cap_rows]
  int32_t *og_status, *og_np, *og_nv;
  double* og_v;                     // [B][MAXPOLY][MAXV][2]
};

__global__ __launch_bounds__(64) void k_classic(htp_classic_batch in, double* ws, htp_classic_result out) {
  const int64_t b = blockIdx.x;
  if (b >= in.batch) return;
  __shared__ rs::Path paths[rs::MAXP];
  __shared__ int flags[rs::MAXP];
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  ct::run_problem(c, in, out, b, ws + b * (int64_t)ct::SCR_PER_POINT * in.cap_samples, paths, flags);
}

__global__ __launch_bounds__(64) void k_prep(int B, int N, int cap, double dT, double wb, ChainBufs w) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int n = w.ct_status[b] == 0 ? w.ct_n[b] : 0;
  if (n < 2) return;
  chain::prep(w.ct_path + b * cap * 5, n, N, dT, wb, w.xs + b * cap, w.ys + b * cap, w.dirs + b * cap,
              w.steps + b * cap, w.rp_params + 3 * b);
}

__global__ __launch_bounds__(64) void k_refpath(int B, int cap, int cap_rows, ChainBufs w) {
  const int64_t b = blockIdx.x;
  if (b >= B) return;
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  const int n = w.ct_status[b] == 0 ? w.ct_n[b] : 0;
  rp::Out o{};
  if (n < 2) {
    o.status = rp::ST_BAD_INPUT;
  } else {
    const double* prm = w.rp_params + 3 * b;
    rp::Course<DevWave> K{c, w.xs + b * cap, w.ys + b * cap, w.dirs + b * cap, n, prm[0], prm[1], prm[2],
                          w.rp_ws + b * (int64_t)rp::SCRATCH_PER_POINT * cap, cap};
    K.run(o, w.rp_traj + b * (int64_t)cap_rows * 5, cap_rows);
  }
  if (threadIdx.x == 0) {
    w.rp_status[b] = o.status;
    w.rp_rows[b] = o.n_rows;
  }
}

__global__ __launch_bounds__(64) void k_resample(htp_chain_batch in, ChainBufs w, chain::Vehicle V) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= in.batch) return;
  if (w.ct_status[b] != 0 || w.rp_status[b] != 0 || w.rp_rows[b] < 2) return;
  double* p = const_cast<double*>(in.scenes.params) + b * HTP_OGE_NPARAM;
  oge::SceneIn sc;
  sc.nrows = (int)p[HTP_OGE_P_NROWS];
  sc.row_width = p[HTP_OGE_P_ROWW];
  sc.row_length = p[HTP_OGE_P_ROWLEN];
  sc.slope = p[HTP_OGE_P_SLOPE];
  sc.row_draws = in.scenes.row_draws + b * in.scenes.max_rows;
  oge::Scene S;
  if (sc.nrows < 3 || sc.nrows > in.scenes.max_rows || sc.nrows > oge::MAXR) return;
  oge::make_rows(sc, S);
  const double hw = chain::resample_hw(w.rp_traj + b * (int64_t)in.cap_rows * 5, w.rp_rows[b], in.N,
                                       w.s + b * (int64_t)in.cap_rows, in.traj + b * (int64_t)in.N * 5, V, S,
                                       in.margin[b]);
  p[HTP_OGE_P_HW] = hw;
}

__global__ __launch_bounds__(64) void k_oge(htp_oge_batch in, htp_oge_result out) {
  const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (s >= in.batch) return;
  oge::run_scene(in, out, s);
}

__global__ __launch_bounds__(64) void k_pack(htp_chain_batch in, ChainBufs w, chain::Vehicle V) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= in.batch) return;
  int st = 0;
  if (w.ct_status[b] != 0) st = 16 + w.ct_status[b];
  else if (w.rp_status[b] != 0 || w.rp_rows[b] < 2) st = 32 + (w.rp_status[b] ? w.rp_status[b] : 15);
  else if (w.og_status[b] != 0) st = 48 + w.og_status[b];
  if (st == 0) {
    const double* p = in.scenes.params + b * HTP_OGE_NPARAM;
    oge::SceneIn sc;
    sc.nrows = (int)p[HTP_OGE_P_NROWS];
    sc.row_width = p[HTP_OGE_P_ROWW];
    sc.row_length = p[HTP_OGE_P_ROWLEN];
    sc.slope = p[HTP_OGE_P_SLOPE];
    sc.tree_width = p[HTP_OGE_P_TREEW];
    sc.headland_width = p[HTP_OGE_P_HW];
    sc.row_draws = in.scenes.row_draws + b * in.scenes.max_rows;
    sc.eps_draws = in.scenes.eps_draws + b * in.scenes.max_rows;
    for (int j = 0; j < 3; ++j) { sc.start[j] = p[HTP_OGE_P_SX + j]; sc.end[j] = p[HTP_OGE_P_EX + j]; }
    sc.side = (int)p[HTP_OGE_P_SIDE];
    oge::Scene S;
    oge::make_rows(sc, S);
    oge::PolyOut po;
    po.n = w.og_np[b];
    for (int q = 0; q < po.n; ++q) {
      po.nv[q] = w.og_nv[b * oge::MAXPOLY + q];
      const double* v = w.og_v + (b * oge::MAXPOLY + q) * oge::MAXV * 2;
      for (int j = 0; j < po.nv[q]; ++j) { po.xy[q][j][0] = v[2 * j]; po.xy[q][j][1] = v[2 * j + 1]; }
    }
    if (chain::pack(po, sc, S, in.traj + b * (int64_t)in.N * 5, in.N, w.rp_traj + b * (int64_t)in.cap_rows * 5,
                    w.rp_rows[b], V, in.M, in.obs_A + b * (int64_t)in.M * 8, in.obs_b + b * (int64_t)in.M * 4))
      st = 64 + 1;
  }
  in.status[b] = st;
}

}  // namespace

extern "C" {

int htp_orchard_chain_device(htp_ctx* ctx, const htp_chain_batch* in, void* stream) {
  if (!ctx || !in) return fail(ctx, "chain: null argument");
  const int B = in->batch;
  if (B < 0 || in->N < 2 || in->M < 1 || in->cap_rows < 2 || in->turns.batch != B || in->scenes.batch != B)
    return fail(ctx, "chain: bad sizes");
  if (in->n_vpoly < 1 || in->n_vpoly > 2 || in->vpoly_nv[0] < 3 || in->vpoly_nv[0] > 8 ||
      (in->n_vpoly == 2 && (in->vpoly_nv[1] < 3 || in->vpoly_nv[1] > 8)))
    return fail(ctx, "chain: vehicle polygons");
  if (!in->traj || !in->obs_A || !in->obs_b || !in->status || !in->margin) return fail(ctx, "chain: output missing");
  // the stage kernels' own entry checks (htp_oge.hip, htp_classic.hip check_in): k_resample / k_pack build the
  // scene's rows into fixed [oge::MAXR] arrays, the classic stage needs its scratch and path pools
  if (in->scenes.max_rows < 3 || in->scenes.max_rows > HTP_OGE_MAXROWS || in->scenes.max_rows > oge::MAXR)
    return fail(ctx, "chain: scenes.max_rows out of [3, HTP_OGE_MAXROWS]");
  if (!in->scenes.params || !in->scenes.row_draws || !in->scenes.eps_draws) return fail(ctx, "chain: scene input missing");
  if (in->turns.cap_samples < 16 || in->turns.cap_path < 2) return fail(ctx, "chain: turns.cap_samples / cap_path");
  if (!in->turns.params || !in->turns.desc || !in->turns.poly_off || !in->turns.vertices)
    return fail(ctx, "chain: turn input missing");
  if (B == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const size_t cap = (size_t)in->turns.cap_path, cr = (size_t)in->cap_rows, Bz = (size_t)B;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  size_t off[16];
  const size_t sz[16] = {4 * Bz, 4 * Bz, 40 * Bz * cap, 8 * Bz * ct::SCR_PER_POINT * (size_t)in->turns.cap_samples,
                         8 * Bz * cap, 8 * Bz * cap, 8 * Bz * cap, 8 * Bz * cap, 24 * Bz,
                         8 * Bz * rp::SCRATCH_PER_POINT * cap, 4 * Bz, 4 * Bz, 40 * Bz * cr, 8 * Bz * cr,
                         4 * Bz * (3 + oge::MAXPOLY), 16 * Bz * oge::MAXPOLY * oge::MAXV};
  for (int k = 0; k < 16; ++k) { off[k] = o; o += al(sz[k]); }
  if (order_after(ctx, ctx->ch_ev1, s)) return -1;
  if (ensure(ctx, &ctx->ch_ws, &ctx->ch_ws_bytes, o)) return -1;
  char* d = (char*)ctx->ch_ws;
  ChainBufs w;
  w.ct_status = (int32_t*)(d + off[0]);
  w.ct_n = (int32_t*)(d + off[1]);
  w.ct_path = (double*)(d + off[2]);
  w.ct_ws = (double*)(d + off[3]);
  w.xs = (double*)(d + off[4]);
  w.ys = (double*)(d + off[5]);
  w.dirs = (double*)(d + off[6]);
  w.steps = (double*)(d + off[7]);
  w.rp_params = (double*)(d + off[8]);
  w.rp_ws = (double*)(d + off[9]);
  w.rp_status = (int32_t*)(d + off[10]);
  w.rp_rows = (int32_t*)(d + off[11]);
  w.rp_traj = (double*)(d + off[12]);
  w.s = (double*)(d + off[13]);
  w.og_status = (int32_t*)(d + off[14]);
  w.og_np = w.og_status + B;
  w.og_nv = w.og_np + B;
  w.og_v = (double*)(d + off[15]);
  chain::Vehicle V{};
  V.npoly = in->n_vpoly;
  for (int k = 0; k < V.npoly; ++k) {
    V.nv[k] = in->vpoly_nv[k];
    for (int j = 0; j < V.nv[k]; ++j) { V.v[k][j][0] = in->vpoly[k][j][0]; V.v[k][j][1] = in->vpoly[k][j][1]; }
  }
  const dim3 waves(B), threads_blocks((B + 63) / 64), wave(64);
  HIPCHK(hipEventRecord(ctx->ch_ev0, s));
  htp_classic_result cres{w.ct_status, w.ct_n, w.ct_path};
  hipLaunchKernelGGL(k_classic, waves, wave, 0, s, in->turns, w.ct_ws, cres);
  hipLaunchKernelGGL(k_prep, threads_blocks, wave, 0, s, B, in->N, (int)cap, in->dT, in->wheel_base, w);
  hipLaunchKernelGGL(k_refpath, waves, wave, 0, s, B, (int)cap, (int)cr, w);
  hipLaunchKernelGGL(k_resample, threads_blocks, wave, 0, s, *in, w, V);
  htp_oge_result ores{w.og_status, w.og_np, w.og_nv, w.og_v, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(k_oge, threads_blocks, wave, 0, s, in->scenes, ores);
  hipLaunchKernelGGL(k_pack, threads_blocks, wave, 0, s, *in, w, V);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ch_ev1, s));
  return 0;
}

double htp_chain_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->ch_ev1) return 0.0;
  float ms = 0.f;
  if (hipEventSynchronize(ctx->ch_ev1) != hipSuccess) return 0.0;
  if (hipEventElapsedTime(&ms, ctx->ch_ev0, ctx->ch_ev1) != hipSuccess) return 0.0;
  return (double)ms;
}

}  // extern "C"
