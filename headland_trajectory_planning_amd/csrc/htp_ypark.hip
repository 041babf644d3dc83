// libhtp.so, Y-type parking grid search: one search per 64-lane wavefront
// (ypark_core.h), the whole batch in one launch.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "ypark_core.h"

using namespace htp;

namespace {

struct Pools {
  const double* params;
  const int32_t* desc;
  const int32_t* poly_off;
  const double* vert;
  const double* axis;
  int32_t npoly, naxis;
};

__device__ bool valid(const Pools& P, const double* prm, const int32_t* d) {
  auto poly_ok = [&](int p) { return p >= 0 && p < P.npoly; };
  if (!poly_ok(d[yp::D_BODY])) return false;
  const int nb = P.poly_off[d[yp::D_BODY] + 1] - P.poly_off[d[yp::D_BODY]];
  if (nb < 3 || nb > ha::MAXB) return false;
  if (d[yp::D_BLK0] < 0 || d[yp::D_BLK1] < d[yp::D_BLK0] || d[yp::D_BLK1] > P.npoly) return false;
  if (d[yp::D_FIELD] != -1 && !poly_ok(d[yp::D_FIELD])) return false;
  for (int a = 0; a < 4; ++a) {
    const int o = d[yp::D_BL0 + 2 * a], n = d[yp::D_BL0 + 2 * a + 1];
    if (o < 0 || n < 1 || o + n > P.naxis) return false;
  }
  const double step = prm[yp::P_STEP];
  if (!(step > 0) || !(prm[yp::P_WB] > 0)) return false;
  for (int a = 0; a < 2; ++a) {  // arc lengths: round(L/step) in [1, MAXARC - 1]
    const int o = d[yp::D_BL0 + 2 * a], n = d[yp::D_BL0 + 2 * a + 1];
    for (int k = 0; k < n; ++k) {
      const double r = rint(P.axis[o + k] / step);
      if (!(r >= 1) || r > yp::MAXARC - 1) return false;
    }
  }
  return true;
}

__global__ __launch_bounds__(64) void ypark_kernel(Pools P, int batch, double* ws, htp_ypark_result out,
                                                   int cap_path) {
  __shared__ double body[2 * ha::MAXB];
  __shared__ int32_t cnt[yp::CH], hit[yp::CH];
  const int b = blockIdx.x;
  if (b >= batch) return;
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  const double* prm = P.params + (int64_t)b * HTP_YP_NPARAM;
  const int32_t* d = P.desc + (int64_t)b * HTP_YP_NDESC;
  yp::Out o{};
  o.cand = -1;
  if (!valid(P, prm, d)) {
    o.status = yp::ST_BAD_INPUT;
  } else {
    ha::Geo g{P.poly_off, P.vert, nullptr, nullptr, nullptr};
    yp::Search<DevWave> S(c, prm, d, g, P.axis, ws + (int64_t)b * yp::CH * yp::SCR, body, cnt, hit);
    S.run(o, out.path + (int64_t)b * cap_path * 5, cap_path);
  }
  if (threadIdx.x == 0) {
    out.status[b] = o.status;
    out.cand[b] = o.cand;
    out.n_path[b] = o.n_path;
    out.params[4 * b] = o.bl;
    out.params[4 * b + 1] = o.fl;
    out.params[4 * b + 2] = o.sb;
    out.params[4 * b + 3] = o.sf;
    if (out.n_pose) out.n_pose[b] = o.n_pose;
  }
}

int enqueue(htp_ctx* ctx, const htp_ypark_batch* in, const Pools& P, const htp_ypark_result& out, hipStream_t s) {
  const size_t need = sizeof(double) * (size_t)yp::CH * yp::SCR * (size_t)in->batch;
  if (ensure(ctx, &ctx->yp_ws, &ctx->yp_ws_bytes, need)) return -1;
  HIPCHK(hipEventRecord(ctx->yp_ev0, s));
  hipLaunchKernelGGL(ypark_kernel, dim3(in->batch), dim3(64), 0, s, P, in->batch, (double*)ctx->yp_ws, out,
                     in->cap_path);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->yp_ev1, s));
  return 0;
}

int check_in(htp_ctx* ctx, const htp_ypark_batch* in, const htp_ypark_result* out) {
  if (!ctx || !in || !out) return fail(ctx, "ypark: null argument");
  if (in->batch < 0 || in->npoly < 1 || in->nvert < 1 || in->naxis < 1) return fail(ctx, "ypark: empty pools");
  if (in->cap_path < 0) return fail(ctx, "ypark: negative capacity");
  if (!in->params || !in->desc || !in->poly_off || !in->vertices || !in->axis)
    return fail(ctx, "ypark: input array missing");
  if (!out->status || !out->cand || !out->n_path || !out->params || (in->cap_path > 0 && !out->path))
    return fail(ctx, "ypark: output array missing");
  return 0;
}

}  // namespace

extern "C" {

int htp_ypark_search_batch_device(htp_ctx* ctx, const htp_ypark_batch* in, htp_ypark_result* out, void* stream) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  Pools P{in->params, in->desc, in->poly_off, in->vertices, in->axis, in->npoly, in->naxis};
  return enqueue(ctx, in, P, *out, (hipStream_t)stream);
}

int htp_ypark_search_batch(htp_ctx* ctx, const htp_ypark_batch* in, htp_ypark_result* out) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  for (int p = 0; p < in->npoly; ++p)
    if (in->poly_off[p] < 0 || in->poly_off[p + 1] < in->poly_off[p] || in->poly_off[p + 1] > in->nvert)
      return fail(ctx, "ypark: poly_off out of range");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t B = in->batch, cp = in->cap_path;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  const size_t o_prm = o; o += al(8 * HTP_YP_NPARAM * (size_t)B);
  const size_t o_dsc = o; o += al(4 * HTP_YP_NDESC * (size_t)B);
  const size_t o_po = o; o += al(4 * ((size_t)in->npoly + 1));
  const size_t o_v = o; o += al(16 * (size_t)in->nvert);
  const size_t o_ax = o; o += al(8 * (size_t)in->naxis);
  const size_t o_st = o; o += al(4 * (size_t)B);
  const size_t o_cd = o; o += al(4 * (size_t)B);
  const size_t o_np = o; o += al(4 * (size_t)B);
  const size_t o_pr = o; o += al(32 * (size_t)B);
  const size_t o_npo = o; o += al(8 * (size_t)B);
  const size_t o_path = o; o += al(40 * (size_t)(B * cp));
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && n && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "ypark: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && dst && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(ctx, "ypark: download");
  };
  H2D(o_prm, in->params, 8 * HTP_YP_NPARAM * (size_t)B);
  H2D(o_dsc, in->desc, 4 * HTP_YP_NDESC * (size_t)B);
  H2D(o_po, in->poly_off, 4 * ((size_t)in->npoly + 1));
  H2D(o_v, in->vertices, 16 * (size_t)in->nvert);
  H2D(o_ax, in->axis, 8 * (size_t)in->naxis);
  Pools P{(const double*)(d + o_prm), (const int32_t*)(d + o_dsc), (const int32_t*)(d + o_po),
          (const double*)(d + o_v), (const double*)(d + o_ax), in->npoly, in->naxis};
  htp_ypark_result dv{(int32_t*)(d + o_st), (int32_t*)(d + o_cd), (int32_t*)(d + o_np), (double*)(d + o_pr),
                      (int64_t*)(d + o_npo), (double*)(d + o_path)};
  if (rc == 0) rc = enqueue(ctx, in, P, dv, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("ypark kernel: ") + hipGetErrorString(er));
  }
  D2H(out->status, o_st, 4 * (size_t)B);
  D2H(out->cand, o_cd, 4 * (size_t)B);
  D2H(out->n_path, o_np, 4 * (size_t)B);
  D2H(out->params, o_pr, 32 * (size_t)B);
  D2H(out->n_pose, o_npo, 8 * (size_t)B);
  D2H(out->path, o_path, 40 * (size_t)(B * cp));
  (void)hipFree(d);
  return rc;
}

double htp_ypark_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->yp_ev1) return 0.0;
  if (hipEventSynchronize(ctx->yp_ev1) != hipSuccess) return 0.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ctx->yp_ev0, ctx->yp_ev1) != hipSuccess) return 0.0;
  return ms;
}

}  // extern "C"
