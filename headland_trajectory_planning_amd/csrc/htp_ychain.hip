// libhtp.so: the notebook planner chain on the device (R/path_planner/headland_path_planning.py:124-255):
// Y-type parking search -> heuristic lowering (ychain_core.h) -> hybrid A* search -> joined warm start ->
// get_init_ref_path -> N-row resample, four launches on one stream, every intermediate in HBM.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "refpath_core.h"
#include "chain_core.h"
#include "ychain_core.h"

using namespace htp;

namespace {

static_assert(HTP_YC_MAXWP == yc::MAXWP && HTP_YC_VERT_STRIDE == yc::MAXSEG * yc::CAPV, "htp.h / ychain_core.h");
constexpr int YP_FOUND = 0, HA_FOUND = 0;

// one problem per thread: the search's heuristic inputs into the problem's reserved slots
__global__ __launch_bounds__(64) void k_lower(htp_ychain_batch in) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= in.batch) return;
  const htp_hastar_batch& H = in.hastar;
  int32_t* desc = const_cast<int32_t*>(H.desc) + b * HTP_HA_NDESC;
  double* prm = const_cast<double*>(H.params) + b * HTP_HA_NPARAM;
  int32_t* poly_off = const_cast<int32_t*>(H.poly_off);
  double* verts = const_cast<double*>(H.vertices);
  double* lane_len = const_cast<double*>(H.lane_len);
  double* guide = const_cast<double*>(H.guide);
  const int pbase = in.lane_poly0 + (int)b * HTP_YC_POLY_STRIDE;
  const int vbase = in.lane_vert0 + (int)b * HTP_YC_VERT_STRIDE;
  const int gbase = in.guide0 + (int)b * in.guide_stride;
  desc[HTP_HA_D_LANE0] = pbase;
  desc[HTP_HA_D_LANE1] = pbase;   // invalid (no lane) until the lowering succeeds: the search reports bad input
  int st = 0;
  const int ys = in.ypark_out.status[b];
  const int nr = in.nrows[b];
  if (ys != YP_FOUND) st = 16 + ys;
  else if (nr < 1 || nr > in.max_rows || nr > yc::MAXROWS) st = 32 + yc::ST_BAD_INPUT;
  int cum = 0;
  if (st == 0) {
    const double* goal = in.ypark_out.path + b * (int64_t)in.ypark.cap_path * 5;   // intermediate_pose = y_path[0][:3]
    double wp[yc::MAXWP][2];
    const int nwp = yc::waypoints(in.rows + b * (int64_t)in.max_rows * 4, nr, in.eps + b * (int64_t)in.max_rows,
                                  in.start + 3 * b, goal, in.drive_row_offset, wp);
    if (nwp < 2) {
      st = 32 + yc::ST_TOO_MANY_WAYPOINTS;
    } else {
      const int m = yc::guide(wp, nwp, guide + 4 * (int64_t)gbase, in.guide_stride);
      if (m < 1) st = 32 + yc::ST_GUIDE_OVERFLOW;
      const int nseg = nwp - 1;
      for (int k = 0; k < nseg && st == 0; ++k) {
        double ring[yc::CAPV][2];
        const int nv = yc::capsule(wp[k], wp[k + 1], yc::LANE_HALF_WIDTH, ring);
        if (nv < 3) { st = 32 + yc::ST_RING_OVERFLOW; break; }
        for (int j = 0; j < nv; ++j) {
          verts[2 * (int64_t)(vbase + cum + j)] = ring[j][0];
          verts[2 * (int64_t)(vbase + cum + j) + 1] = ring[j][1];
        }
        cum += nv;
        poly_off[pbase + k + 1] = vbase + cum;
        lane_len[pbase + k] = yc::search_length(k, nseg, prm[HTP_HA_P_DEFLEN]);
      }
      if (st == 0) {
        for (int k = nseg + 1; k < HTP_YC_POLY_STRIDE; ++k) poly_off[pbase + k] = vbase + cum;   // empty slots
        prm[HTP_HA_P_GX] = goal[0];
        prm[HTP_HA_P_GY] = goal[1];
        prm[HTP_HA_P_GYAW] = goal[2];
        desc[HTP_HA_D_LANE1] = pbase + nseg;
        desc[HTP_HA_D_GUIDE0] = gbase;
        desc[HTP_HA_D_GUIDE1] = gbase + m;
      }
    }
  }
  if (st != 0)   // keep the slot's polygon table monotone
    for (int k = 1; k < HTP_YC_POLY_STRIDE; ++k) poly_off[pbase + k] = vbase;
  in.status[b] = st;
}

struct JoinBufs {
  double *xs, *ys, *dirs;   // [B][cap] joined warm start
  double* rp_ws;            // [B][SCRATCH_PER_POINT * cap]
  double* s;                // [B][cap_rows] resample arc length
};

// one problem per wavefront: hybrid A* path + parking manoeuvre -> get_init_ref_path -> N rows
__global__ __launch_bounds__(64) void k_join(htp_ychain_batch in, JoinBufs w, int cap) {
  const int64_t b = blockIdx.x;
  if (b >= in.batch) return;
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  int st = in.status[b];
  const int hs = in.hastar_out.status[b];
  if (st == 0 && hs != HA_FOUND) st = 48 + hs;
  const int nh = st == 0 ? in.hastar_out.n_path[b] : 0, ny = st == 0 ? in.ypark_out.n_path[b] : 0;
  if (st == 0 && (nh > in.hastar.cap_path || ny > in.ypark.cap_path || nh + ny > cap || nh + ny < 2))
    st = 64 + rp::ST_OVERFLOW;
  rp::Out o{};
  if (st == 0) {
    const int64_t hb = b * (int64_t)in.hastar.cap_path, yb = b * (int64_t)in.ypark.cap_path * 5;
    double* xs = w.xs + b * cap;
    double* ys = w.ys + b * cap;
    double* ds = w.dirs + b * cap;
    for (int i = c.lane; i < nh + ny; i += 64) {   // np.concatenate([xs, y_path[:, 0]]), ... dirs from column 4
      if (i < nh) { xs[i] = in.hastar_out.x[hb + i]; ys[i] = in.hastar_out.y[hb + i]; ds[i] = in.hastar_out.dir[hb + i]; }
      else { const double* r = in.ypark_out.path + yb + 5 * (int64_t)(i - nh); xs[i] = r[0]; ys[i] = r[1]; ds[i] = r[4]; }
    }
    c.sync();
    const double* p = in.rp_params + 3 * b;
    rp::Course<DevWave> K{c, xs, ys, ds, nh + ny, p[0], p[1], p[2], w.rp_ws + b * (int64_t)rp::SCRATCH_PER_POINT * cap,
                          cap};
    double* ref = in.ref + b * (int64_t)in.cap_rows * 5;
    K.run(o, ref, in.cap_rows);
    if (o.status != rp::ST_OK) st = 64 + o.status;
    else if (o.n_rows < 2) st = 64 + rp::ST_BAD_INPUT;
    c.sync();
    if (st == 0 && c.lane == 0) chain::resample(ref, o.n_rows, in.N, w.s + b * (int64_t)in.cap_rows, in.traj + b * (int64_t)in.N * 5);
  }
  if (threadIdx.x == 0) {
    in.status[b] = st;
    in.n_ref[b] = st == 0 ? o.n_rows : 0;
  }
}

}  // namespace

extern "C" {

int htp_ypark_hastar_chain_device(htp_ctx* ctx, const htp_ychain_batch* in, void* stream) {
  if (!ctx || !in) return fail(ctx, "ychain: null argument");
  const int B = in->batch;
  if (B < 0 || in->N < 2 || in->cap_rows < in->N || in->ypark.batch != B || in->hastar.batch != B)
    return fail(ctx, "ychain: bad sizes");
  if (in->max_rows < 1 || in->max_rows > yc::MAXROWS || in->guide_stride < 2 || in->lane_poly0 < 0 ||
      in->lane_vert0 < 0 || in->guide0 < 0)
    return fail(ctx, "ychain: bad slot layout");
  if ((int64_t)in->lane_poly0 + (int64_t)B * HTP_YC_POLY_STRIDE > in->hastar.npoly ||
      (int64_t)in->lane_vert0 + (int64_t)B * HTP_YC_VERT_STRIDE > in->hastar.nvert ||
      (int64_t)in->guide0 + (int64_t)B * in->guide_stride > in->hastar.nguide)
    return fail(ctx, "ychain: reserved slots exceed the hybrid A* pools");
  if (in->ypark.cap_path < 1 || in->hastar.cap_path < 1) return fail(ctx, "ychain: path capacities");
  if (!in->rows || !in->nrows || !in->eps || !in->start || !in->rp_params || !in->ref || !in->n_ref || !in->traj ||
      !in->status || !in->ypark_out.status || !in->ypark_out.n_path || !in->ypark_out.path || !in->hastar_out.x ||
      !in->hastar_out.y || !in->hastar_out.dir || !in->hastar_out.status || !in->hastar_out.n_path)
    return fail(ctx, "ychain: array missing");
  // the hybrid A* entry's own host checks, done here before anything is enqueued: k_lower writes into these
  // pools, and a rejected search must not leave the Y-park search and the lowering already queued
  const htp_hastar_batch& ha = in->hastar;
  if (!ha.params || !ha.desc || !ha.poly_off || !ha.vertices || !ha.lane_len || !ha.guide || !ha.motions)
    return fail(ctx, "ychain: hybrid A* pool missing");
  if (ha.npoly < 1 || ha.nvert < 1 || ha.nguide < 1 || ha.nmotion < 1 || ha.max_nodes_cap < 0 ||
      ha.max_nodes_cap > 1000000 || ha.cap_log < 0)
    return fail(ctx, "ychain: hybrid A* pool sizes");
  if (!in->hastar_out.counter || !in->hastar_out.yaw || !in->hastar_out.k)
    return fail(ctx, "ychain: hybrid A* output array missing");
  if (B == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  for (auto& e : ctx->yc_ev)
    if (!e) HIPCHK(hipEventCreate(&e));
  const int cap = in->hastar.cap_path + in->ypark.cap_path;
  const size_t Bz = (size_t)B;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  const size_t sz_j = al(8 * Bz * (size_t)cap), sz_rp = al(8 * Bz * (size_t)rp::SCRATCH_PER_POINT * (size_t)cap),
               sz_s = al(8 * Bz * (size_t)in->cap_rows);
  if (order_after(ctx, ctx->yc_ev[4], s)) return -1;
  if (ensure(ctx, &ctx->yc_ws, &ctx->yc_ws_bytes, 3 * sz_j + sz_rp + sz_s)) return -1;
  char* d = (char*)ctx->yc_ws;
  JoinBufs w{(double*)d, (double*)(d + sz_j), (double*)(d + 2 * sz_j), (double*)(d + 3 * sz_j),
             (double*)(d + 3 * sz_j + sz_rp)};
  htp_ypark_result yo = in->ypark_out;
  htp_hastar_result ho = in->hastar_out;
  HIPCHK(hipEventRecord(ctx->yc_ev[0], s));
  if (htp_ypark_search_batch_device(ctx, &in->ypark, &yo, stream)) return -1;
  HIPCHK(hipEventRecord(ctx->yc_ev[1], s));
  hipLaunchKernelGGL(k_lower, dim3((B + 63) / 64), dim3(64), 0, s, *in);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->yc_ev[2], s));
  if (htp_hastar_search_batch_device(ctx, &in->hastar, &ho, stream)) return -1;
  HIPCHK(hipEventRecord(ctx->yc_ev[3], s));
  hipLaunchKernelGGL(k_join, dim3(B), dim3(64), 0, s, *in, w, cap);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->yc_ev[4], s));
  return 0;
}

int htp_ychain_last_ms(htp_ctx* ctx, double* ms4) {
  if (!ctx || !ms4 || !ctx->yc_ev[4]) return -1;
  if (hipEventSynchronize(ctx->yc_ev[4]) != hipSuccess) return -1;
  for (int k = 0; k < 4; ++k) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->yc_ev[k], ctx->yc_ev[k + 1]) != hipSuccess) return -1;
    ms4[k] = ms;
  }
  return 0;
}

}  // extern "C"
