// libhtp.so, warm start -> OBCA initial guess (refpath_core.h): one path per
// 64-lane wavefront, the whole batch in one launch.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "wave_ctx.h"
#include "refpath_core.h"

using namespace htp;

namespace {

__global__ __launch_bounds__(64) void refpath_kernel(htp_refpath_batch in, double* ws, htp_refpath_result out) {
  const int b = blockIdx.x;
  if (b >= in.batch) return;
  DevWave c{(int)threadIdx.x, nullptr, nullptr};
  const int a0 = in.path_off[b], a1 = in.path_off[b + 1];
  const double* prm = in.params + 3 * (int64_t)b;
  rp::Out o{};
  if (a0 < 0 || a1 < a0 || a1 - a0 > in.cap_points || !(prm[2] > 0.0)) {
    o.status = rp::ST_BAD_INPUT;
  } else {
    rp::Course<DevWave> K{c, in.xs + a0, in.ys + a0, in.dirs + a0, a1 - a0, prm[0], prm[1], prm[2],
                          ws + (int64_t)b * rp::SCRATCH_PER_POINT * in.cap_points, in.cap_points};
    K.run(o, out.traj + (int64_t)b * in.cap_rows * 5, in.cap_rows);
  }
  if (threadIdx.x == 0) {
    out.status[b] = o.status;
    out.n_rows[b] = o.n_rows;
  }
}

int enqueue(htp_ctx* ctx, const htp_refpath_batch& in, const htp_refpath_result& out, hipStream_t s) {
  const size_t need = sizeof(double) * rp::SCRATCH_PER_POINT * (size_t)in.cap_points * (size_t)in.batch;
  if (ensure(ctx, &ctx->rp_ws, &ctx->rp_ws_bytes, need)) return -1;
  HIPCHK(hipEventRecord(ctx->rp_ev0, s));
  hipLaunchKernelGGL(refpath_kernel, dim3(in.batch), dim3(64), 0, s, in, (double*)ctx->rp_ws, out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->rp_ev1, s));
  return 0;
}

int check_in(htp_ctx* ctx, const htp_refpath_batch* in, const htp_refpath_result* out) {
  if (!ctx || !in || !out) return fail(ctx, "refpath: null argument");
  if (in->batch < 0 || in->cap_points < 1 || in->cap_rows < 1) return fail(ctx, "refpath: bad sizes");
  if (!in->path_off || !in->xs || !in->ys || !in->dirs || !in->params) return fail(ctx, "refpath: input missing");
  if (!out->status || !out->n_rows || !out->traj) return fail(ctx, "refpath: output missing");
  return 0;
}

}  // namespace

extern "C" {

int htp_init_ref_path_batch_device(htp_ctx* ctx, const htp_refpath_batch* in, htp_refpath_result* out,
                                   void* stream) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  return enqueue(ctx, *in, *out, (hipStream_t)stream);
}

int htp_init_ref_path_batch(htp_ctx* ctx, const htp_refpath_batch* in, htp_refpath_result* out) {
  if (check_in(ctx, in, out)) return -1;
  if (in->batch == 0) return 0;
  const int64_t B = in->batch;
  const int64_t P = in->path_off[B];
  for (int64_t b = 0; b < B; ++b)
    if (in->path_off[b] < 0 || in->path_off[b + 1] < in->path_off[b] || in->path_off[b + 1] > P)
      return fail(ctx, "refpath: path_off not monotone");
  HIPCHK(hipSetDevice(ctx->device));
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  size_t o = 0;
  const size_t o_off = o; o += al(4 * (size_t)(B + 1));
  const size_t o_x = o; o += al(8 * (size_t)P);
  const size_t o_y = o; o += al(8 * (size_t)P);
  const size_t o_d = o; o += al(8 * (size_t)P);
  const size_t o_p = o; o += al(24 * (size_t)B);
  const size_t o_st = o; o += al(4 * (size_t)B);
  const size_t o_nr = o; o += al(4 * (size_t)B);
  const size_t o_tr = o; o += al(40 * (size_t)B * (size_t)in->cap_rows);
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && n && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "refpath: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(ctx, "refpath: download");
  };
  H2D(o_off, in->path_off, 4 * (size_t)(B + 1));
  H2D(o_x, in->xs, 8 * (size_t)P);
  H2D(o_y, in->ys, 8 * (size_t)P);
  H2D(o_d, in->dirs, 8 * (size_t)P);
  H2D(o_p, in->params, 24 * (size_t)B);
  htp_refpath_batch din = *in;
  din.path_off = (const int32_t*)(d + o_off);
  din.xs = (const double*)(d + o_x);
  din.ys = (const double*)(d + o_y);
  din.dirs = (const double*)(d + o_d);
  din.params = (const double*)(d + o_p);
  htp_refpath_result dout{(int32_t*)(d + o_st), (int32_t*)(d + o_nr), (double*)(d + o_tr)};
  if (rc == 0) rc = enqueue(ctx, din, dout, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("refpath kernel: ") + hipGetErrorString(er));
  }
  D2H(out->status, o_st, 4 * (size_t)B);
  D2H(out->n_rows, o_nr, 4 * (size_t)B);
  D2H(out->traj, o_tr, 40 * (size_t)B * (size_t)in->cap_rows);
  (void)hipFree(d);
  return rc;
}

double htp_init_ref_path_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->rp_ev1) return 0.0;
  if (hipEventSynchronize(ctx->rp_ev1) != hipSuccess) return 0.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ctx->rp_ev0, ctx->rp_ev1) != hipSuccess) return 0.0;
  return ms;
}

}  // extern "C"
