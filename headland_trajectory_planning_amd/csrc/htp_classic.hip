// libhtp.so, classic headland turns (classic_core.h): one turn per 64-lane wavefront, the whole batch in
// one launch.  Per-wave HBM scratch holds the Dubins samples and spline work of the turn being planned.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "classic_batch.h"

using namespace htp;

namespace {

__global__ __launch_bounds__(64) void classic_kernel(htp_classic_batch in, double* ws, htp_classic_result out) {
  const int64_t b = blockIdx.x;
  if (b >= in.batch) return;
  __shared__ rs::Path paths[rs::MAXP];
  __shared__ int flags[rs::MAXP];
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  ct::run_problem(c, in, out, b, ws + b * (int64_t)ct::SCR_PER_POINT * in.cap_samples, paths, flags);
}

int enqueue(htp_ctx* ctx, const htp_classic_batch& in, const htp_classic_result& out, hipStream_t s) {
  const size_t need = sizeof(double) * ct::SCR_PER_POINT * (size_t)in.cap_samples * (size_t)in.batch;
  if (order_after(ctx, ctx->ct_ev1, s)) return -1;
  if (ensure(ctx, &ctx->ct_ws, &ctx->ct_ws_bytes, need)) return -1;
  HIPCHK(hipEventRecord(ctx->ct_ev0, s));
  hipLaunchKernelGGL(classic_kernel, dim3(in.batch), dim3(64), 0, s, in, (double*)ctx->ct_ws, out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ct_ev1, s));
  return 0;
}

int check_in(htp_ctx* ctx, const htp_classic_batch* in, const htp_classic_result* out) {
  if (!ctx || !in || !out) return fail(ctx, "classic: null argument");
  if (in->batch < 0 || in->cap_path < 1 || in->cap_samples < 16 || in->npoly < 0 || in->nvert < 0)
    return fail(ctx, "classic: bad sizes");
  if (!in->params || !in->desc || !in->poly_off || !in->vertices) return fail(ctx, "classic: input missing");
  if (!out->status || !out->n_path || !out->path) return fail(ctx, "classic: output missing");
  return 0;
}

}  // namespace

extern "C" {

int htp_classic_turn_batch_device(htp_ctx* ctx, const htp_classic_batch* in, htp_classic_result* out,
                                  void* stream) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  return enqueue(ctx, *in, *out, (hipStream_t)stream);
}

int htp_classic_turn_batch(htp_ctx* ctx, const htp_classic_batch* in, htp_classic_result* out) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  const int64_t B = in->batch;
  for (int64_t b = 0; b < B; ++b) {   // polygon ids in range (the kernel trusts them)
    const int32_t* d = in->desc + 3 * b;
    if (d[0] < 0 || d[0] >= in->npoly || d[1] < 0 || d[2] < d[1] || d[2] > in->npoly)
      return fail(ctx, "classic: polygon ids out of range");
  }
  if (in->poly_off[0] != 0 || in->poly_off[in->npoly] != in->nvert) return fail(ctx, "classic: poly_off");
  HIPCHK(hipSetDevice(ctx->device));
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  const size_t o_p = o; o += al(8 * (size_t)B * HTP_CT_NPARAM);
  const size_t o_d = o; o += al(4 * 3 * (size_t)B);
  const size_t o_po = o; o += al(4 * (size_t)(in->npoly + 1));
  const size_t o_v = o; o += al(16 * (size_t)in->nvert);
  const size_t o_st = o; o += al(4 * (size_t)B);
  const size_t o_np = o; o += al(4 * (size_t)B);
  const size_t o_pa = o; o += al(40 * (size_t)B * (size_t)in->cap_path);
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && n && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "classic: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(ctx, "classic: download");
  };
  H2D(o_p, in->params, 8 * (size_t)B * HTP_CT_NPARAM);
  H2D(o_d, in->desc, 12 * (size_t)B);
  H2D(o_po, in->poly_off, 4 * (size_t)(in->npoly + 1));
  H2D(o_v, in->vertices, 16 * (size_t)in->nvert);
  htp_classic_batch din = *in;
  din.params = (const double*)(d + o_p);
  din.desc = (const int32_t*)(d + o_d);
  din.poly_off = (const int32_t*)(d + o_po);
  din.vertices = (const double*)(d + o_v);
  htp_classic_result dout{(int32_t*)(d + o_st), (int32_t*)(d + o_np), (double*)(d + o_pa)};
  if (rc == 0) rc = enqueue(ctx, din, dout, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("classic kernel: ") + hipGetErrorString(er));
  }
  D2H(out->status, o_st, 4 * (size_t)B);
  D2H(out->n_path, o_np, 4 * (size_t)B);
  D2H(out->path, o_pa, 40 * (size_t)B * (size_t)in->cap_path);
  (void)hipFree(d);
  return rc;
}

double htp_classic_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->ct_ev1) return 0.0;
  float ms = 0.f;
  if (hipEventSynchronize(ctx->ct_ev1) != hipSuccess) return 0.0;
  if (hipEventElapsedTime(&ms, ctx->ct_ev0, ctx->ct_ev1) != hipSuccess) return 0.0;
  return (double)ms;
}

}  // extern "C"
