// libhtp.so, orchard scene -> OBCA obstacles (oge_core.h): one scene per thread, 64 scenes per
// wavefront, the whole batch in one launch; each polygon's halfspace form is computed in the same
// thread so the OBCA input (obs_A, obs_b) never leaves the device.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "oge_batch.h"

using namespace htp;

namespace {

__global__ __launch_bounds__(64) void oge_kernel(htp_oge_batch in, htp_oge_result out) {
  const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (s >= in.batch) return;
  oge::run_scene(in, out, s);
}

int enqueue(htp_ctx* ctx, const htp_oge_batch& in, const htp_oge_result& out, hipStream_t s) {
  HIPCHK(hipEventRecord(ctx->oge_ev0, s));
  hipLaunchKernelGGL(oge_kernel, dim3((in.batch + 63) / 64), dim3(64), 0, s, in, out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->oge_ev1, s));
  return 0;
}

int check_in(htp_ctx* ctx, const htp_oge_batch* in, const htp_oge_result* out) {
  if (!ctx || !in || !out) return fail(ctx, "oge: null argument");
  if (in->batch < 0 || in->max_rows < 3 || in->max_rows > HTP_OGE_MAXROWS) return fail(ctx, "oge: bad sizes");
  if (!in->params || !in->row_draws || !in->eps_draws) return fail(ctx, "oge: input missing");
  if (!out->status || !out->n_poly || !out->n_vert || !out->vertices) return fail(ctx, "oge: output missing");
  if (out->n_facet && (!out->A || !out->b)) return fail(ctx, "oge: n_facet given without A / b");
  return 0;
}

}  // namespace

extern "C" {

int htp_oge_obstacles_batch_device(htp_ctx* ctx, const htp_oge_batch* in, htp_oge_result* out, void* stream) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  return enqueue(ctx, *in, *out, (hipStream_t)stream);
}

int htp_oge_obstacles_batch(htp_ctx* ctx, const htp_oge_batch* in, htp_oge_result* out) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t B = (size_t)in->batch, R = (size_t)in->max_rows, PQ = B * oge::MAXPOLY;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  const size_t o_p = o; o += al(8 * B * HTP_OGE_NPARAM);
  const size_t o_rd = o; o += al(8 * B * R);
  const size_t o_ed = o; o += al(8 * B * R);
  const size_t o_st = o; o += al(4 * B);
  const size_t o_np = o; o += al(4 * B);
  const size_t o_nv = o; o += al(4 * PQ);
  const size_t o_v = o; o += al(16 * PQ * oge::MAXV);
  const size_t o_nf = o; o += al(4 * PQ);
  const size_t o_A = o; o += al(16 * PQ * oge::MAXV);
  const size_t o_b = o; o += al(8 * PQ * oge::MAXV);
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && n && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "oge: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && dst && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(ctx, "oge: download");
  };
  H2D(o_p, in->params, 8 * B * HTP_OGE_NPARAM);
  H2D(o_rd, in->row_draws, 8 * B * R);
  H2D(o_ed, in->eps_draws, 8 * B * R);
  htp_oge_batch din = *in;
  din.params = (const double*)(d + o_p);
  din.row_draws = (const double*)(d + o_rd);
  din.eps_draws = (const double*)(d + o_ed);
  const bool hs = out->n_facet != nullptr;
  htp_oge_result dout{(int32_t*)(d + o_st), (int32_t*)(d + o_np), (int32_t*)(d + o_nv), (double*)(d + o_v),
                      hs ? (int32_t*)(d + o_nf) : nullptr, hs ? (double*)(d + o_A) : nullptr,
                      hs ? (double*)(d + o_b) : nullptr};
  if (rc == 0) rc = enqueue(ctx, din, dout, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("oge kernel: ") + hipGetErrorString(er));
  }
  D2H(out->status, o_st, 4 * B);
  D2H(out->n_poly, o_np, 4 * B);
  D2H(out->n_vert, o_nv, 4 * PQ);
  D2H(out->vertices, o_v, 16 * PQ * oge::MAXV);
  if (hs) {
    D2H(out->n_facet, o_nf, 4 * PQ);
    D2H(out->A, o_A, 16 * PQ * oge::MAXV);
    D2H(out->b, o_b, 8 * PQ * oge::MAXV);
  }
  (void)hipFree(d);
  return rc;
}

double htp_oge_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->oge_ev1) return 0.0;
  float ms = 0.f;
  if (hipEventSynchronize(ctx->oge_ev1) != hipSuccess) return 0.0;
  if (hipEventElapsedTime(&ms, ctx->oge_ev0, ctx->oge_ev1) != hipSuccess) return 0.0;
  return (double)ms;
}

}  // extern "C"
