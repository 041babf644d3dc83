// libhtp.so, hybrid A* batch: one warm-start search per 64-lane wavefront
// (hastar_core.h), every search of the batch in one launch; the hardware
// dispatcher refills a SIMD as soon as a search retires.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "hastar_core.h"

using namespace htp;
using namespace htp::ha;

namespace {


struct Sizes {
  int32_t cap_node, cap_slot;
  size_t per_search;  // bytes
};

Sizes ws_sizes(int max_nodes_cap) {
  Sizes z;
  const int64_t cn = 4 + (int64_t)(max_nodes_cap + 1) * MAXMOT + 4;
  z.cap_node = (int32_t)cn;
  int64_t cs = 1;
  while (cs < 2 * cn) cs <<= 1;
  z.cap_slot = (int32_t)cs;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  z.per_search = al(sizeof(Node) * (size_t)cn) + al(sizeof(Slot) * (size_t)cs) + al(8 * (size_t)cn) + al(4 * (size_t)cn) +
                 al(8 * (size_t)DUBW * (CAP_DUB + 16));
  return z;
}

HTP_HD inline Work work_of(char* base, const Sizes& z, int b) {
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  char* p = base + (size_t)b * z.per_search;
  Work w;
  w.node = (Node*)p; p += al(sizeof(Node) * (size_t)z.cap_node);
  w.slot = (Slot*)p; p += al(sizeof(Slot) * (size_t)z.cap_slot);
  w.hval = (double*)p; p += al(8 * (size_t)z.cap_node);
  w.hslot = (int32_t*)p; p += al(4 * (size_t)z.cap_node);
  w.dub = (double*)p;
  w.cap_node = z.cap_node;
  w.cap_slot = z.cap_slot;
  w.cap_dub = CAP_DUB;
  return w;
}


// One instantiation per motion type (MODE 1 King: Reeds-Shepp goal shots,
// MODE 0 Pawn: Dubins + spline); each launch covers the whole batch and a
// search is run by the instantiation of its own type (searches with an invalid
// type by King's, which reports them as bad input).  MODE 2 is the combined
// kernel (both goal shots in one body, Search::run dispatch): the default, one
// launch for a mixed batch (256 VGPRs, no VGPR spills).  The split pair stays
// selectable (HTP_HA_SPLIT=1) and tests/test_gpu_hastar.py checks that both
// give the same results on a mixed King/Pawn batch.
template <int MODE>
__global__ __launch_bounds__(64) void hastar_kernel(Pools P, int batch, int max_nodes_cap, char* ws, Sizes z,
                                                    htp_hastar_result out, int cap_path, int cap_log) {
  __shared__ Shared sh;
  const int b = blockIdx.x;
  if (b >= batch) return;
  const double* prm = P.params + (int64_t)b * HTP_HA_NPARAM;
  const int32_t* d = P.desc + (int64_t)b * HTP_HA_NDESC;
  constexpr bool KING = MODE == 1;
  if (MODE != 2 && (d[D_KING] != 0) != KING) return;
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  Out o{};
  int n_path = 0;
  if (!valid_search(P, prm, d, max_nodes_cap)) {
    o.status = ST_BAD_INPUT;
  } else {
    Work w = work_of(ws, z, b);
    Search<DevWave> S(c, prm, d, P.g, w, sh);
    int32_t* log = out.expanded ? out.expanded + (int64_t)b * cap_log * 3 : nullptr;
    if constexpr (MODE == 2) S.run(o, log, log ? cap_log : 0);
    else S.template run_t<KING>(o, log, log ? cap_log : 0);
    if (o.status == ST_FOUND || o.status == ST_NO_PATH || o.status == ST_MAX_NODES) {
      const int64_t off = (int64_t)b * cap_path;
      int st = o.status;
      if constexpr (MODE == 2)
        n_path = S.backtrack(w.hslot, w.cap_node, out.x + off, out.y + off, out.yaw + off, out.dir + off, out.k + off,
                             cap_path, st);
      else
        n_path = S.template backtrack_t<KING>(w.hslot, w.cap_node, out.x + off, out.y + off, out.yaw + off,
                                              out.dir + off, out.k + off, cap_path, st);
      o.status = st;
    }
  }
  if (threadIdx.x == 0) {
    out.status[b] = o.status;
    out.counter[b] = o.counter;
    out.n_path[b] = n_path;
    if (out.n_expanded) out.n_expanded[b] = o.n_expanded;
    if (out.n_pose) out.n_pose[b] = o.n_pose;
  }
}

int enqueue(htp_ctx* ctx, const htp_hastar_batch* in, const Pools& P, htp_hastar_result out, hipStream_t s) {
  const Sizes z = ws_sizes(in->max_nodes_cap);
  if (ensure(ctx, &ctx->ha_ws, &ctx->ha_ws_bytes, z.per_search * (size_t)in->batch)) return -1;
  HIPCHK(hipEventRecord(ctx->ha_ev0, s));
  const char* split = getenv("HTP_HA_SPLIT");
  if (!(split && split[0] == '1')) {
    hipLaunchKernelGGL(hastar_kernel<2>, dim3(in->batch), dim3(64), 0, s, P, in->batch, in->max_nodes_cap,
                       (char*)ctx->ha_ws, z, out, in->cap_path, out.expanded ? in->cap_log : 0);
    HIPCHK(hipGetLastError());
  } else {
    hipLaunchKernelGGL(hastar_kernel<1>, dim3(in->batch), dim3(64), 0, s, P, in->batch, in->max_nodes_cap,
                       (char*)ctx->ha_ws, z, out, in->cap_path, out.expanded ? in->cap_log : 0);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(hastar_kernel<0>, dim3(in->batch), dim3(64), 0, s, P, in->batch, in->max_nodes_cap,
                       (char*)ctx->ha_ws, z, out, in->cap_path, out.expanded ? in->cap_log : 0);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ha_ev1, s));
  return 0;
}

int check_in(htp_ctx* ctx, const htp_hastar_batch* in, const htp_hastar_result* out) {
  if (!ctx || !in || !out) return fail(ctx, "hastar: null argument");
  if (in->batch < 0 || in->npoly < 1 || in->nvert < 1 || in->nguide < 1 || in->nmotion < 1)
    return fail(ctx, "hastar: empty pools");
  if (in->max_nodes_cap < 0 || in->max_nodes_cap > 1000000) return fail(ctx, "hastar: max_nodes_cap out of range");
  if (in->cap_path < 0 || in->cap_log < 0) return fail(ctx, "hastar: negative capacity");
  if (!in->params || !in->desc || !in->poly_off || !in->vertices || !in->lane_len || !in->guide || !in->motions)
    return fail(ctx, "hastar: input array missing");
  if (!out->status || !out->counter || !out->n_path) return fail(ctx, "hastar: output array missing");
  if (in->cap_path > 0 && (!out->x || !out->y || !out->yaw || !out->dir || !out->k))
    return fail(ctx, "hastar: path arrays missing");
  return 0;
}

}  // namespace

extern "C" {

int htp_hastar_search_batch_device(htp_ctx* ctx, const htp_hastar_batch* in, htp_hastar_result* out, void* stream) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  Pools P{in->params, in->desc, Geo{in->poly_off, in->vertices, in->lane_len, in->guide, in->motions},
          in->npoly, in->nvert, in->nguide, in->nmotion};
  return enqueue(ctx, in, P, *out, (hipStream_t)stream);
}

int htp_hastar_search_batch(htp_ctx* ctx, const htp_hastar_batch* in, htp_hastar_result* out) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  // host-side range check of the polygon table (the kernel trusts poly_off)
  if (!poly_table_ok(in->poly_off, in->npoly, in->nvert)) return fail(ctx, "hastar: poly_off out of range");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t B = in->batch;
  const int64_t cp = in->cap_path, cl = out->expanded ? in->cap_log : 0;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  const size_t o_prm = o; o += al(8 * HTP_HA_NPARAM * (size_t)B);
  const size_t o_dsc = o; o += al(4 * HTP_HA_NDESC * (size_t)B);
  const size_t o_po = o; o += al(4 * ((size_t)in->npoly + 1));
  const size_t o_v = o; o += al(16 * (size_t)in->nvert);
  const size_t o_ll = o; o += al(8 * (size_t)in->npoly);
  const size_t o_g = o; o += al(32 * (size_t)in->nguide);
  const size_t o_m = o; o += al(16 * (size_t)in->nmotion);
  const size_t o_st = o; o += al(4 * (size_t)B);
  const size_t o_ct = o; o += al(4 * (size_t)B);
  const size_t o_np = o; o += al(4 * (size_t)B);
  const size_t o_ne = o; o += al(4 * (size_t)B);
  const size_t o_npo = o; o += al(8 * (size_t)B);
  const size_t o_path = o; o += al(5 * 8 * (size_t)(B * cp));
  const size_t o_log = o; o += al(12 * (size_t)(B * cl));
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && n && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "hastar: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && dst && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(ctx, "hastar: download");
  };
  H2D(o_prm, in->params, 8 * HTP_HA_NPARAM * (size_t)B);
  H2D(o_dsc, in->desc, 4 * HTP_HA_NDESC * (size_t)B);
  H2D(o_po, in->poly_off, 4 * ((size_t)in->npoly + 1));
  H2D(o_v, in->vertices, 16 * (size_t)in->nvert);
  H2D(o_ll, in->lane_len, 8 * (size_t)in->npoly);
  H2D(o_g, in->guide, 32 * (size_t)in->nguide);
  H2D(o_m, in->motions, 16 * (size_t)in->nmotion);
  Pools P{(const double*)(d + o_prm), (const int32_t*)(d + o_dsc),
          Geo{(const int32_t*)(d + o_po), (const double*)(d + o_v), (const double*)(d + o_ll),
              (const double*)(d + o_g), (const double*)(d + o_m)},
          in->npoly, in->nvert, in->nguide, in->nmotion};
  htp_hastar_result dv{};
  dv.status = (int32_t*)(d + o_st);
  dv.counter = (int32_t*)(d + o_ct);
  dv.n_path = (int32_t*)(d + o_np);
  dv.n_expanded = (int32_t*)(d + o_ne);
  dv.n_pose = (int64_t*)(d + o_npo);
  double* pb = (double*)(d + o_path);
  dv.x = pb; dv.y = pb + B * cp; dv.yaw = pb + 2 * B * cp; dv.dir = pb + 3 * B * cp; dv.k = pb + 4 * B * cp;
  dv.expanded = cl ? (int32_t*)(d + o_log) : nullptr;
  if (rc == 0) rc = enqueue(ctx, in, P, dv, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("hastar kernel: ") + hipGetErrorString(er));
  }
  D2H(out->status, o_st, 4 * (size_t)B);
  D2H(out->counter, o_ct, 4 * (size_t)B);
  D2H(out->n_path, o_np, 4 * (size_t)B);
  D2H(out->n_expanded, o_ne, 4 * (size_t)B);
  D2H(out->n_pose, o_npo, 8 * (size_t)B);
  if (cp) {
    D2H(out->x, o_path, 8 * (size_t)(B * cp));
    D2H(out->y, o_path + 8 * (size_t)(B * cp), 8 * (size_t)(B * cp));
    D2H(out->yaw, o_path + 16 * (size_t)(B * cp), 8 * (size_t)(B * cp));
    D2H(out->dir, o_path + 24 * (size_t)(B * cp), 8 * (size_t)(B * cp));
    D2H(out->k, o_path + 32 * (size_t)(B * cp), 8 * (size_t)(B * cp));
  }
  if (cl) D2H(out->expanded, o_log, 12 * (size_t)(B * cl));
  (void)hipFree(d);
  return rc;
}

double htp_hastar_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->ha_ev1) return 0.0;
  if (hipEventSynchronize(ctx->ha_ev1) != hipSuccess) return 0.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ctx->ha_ev0, ctx->ha_ev1) != hipSuccess) return 0.0;
  return ms;
}

}  // extern "C"
