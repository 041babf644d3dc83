// libhtp.so: the planner cores' correctly rounded libm (htp_libm.h) evaluated on the device over a batch of
// arguments -- the parity surface that shows the gfx950 build of each function returns the host build's doubles.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "libm_batch.h"

namespace {

__global__ __launch_bounds__(256) void libm_kernel(int fn, const double* __restrict__ x, const double* __restrict__ y,
                                                   double* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = htp::hm::eval(fn, x[i], y ? y[i] : 0.0);
}

}  // namespace

extern "C" int htp_libm_batch_device(htp_ctx* ctx, int32_t fn, const double* x, const double* y, double* out,
                                     int64_t n, void* stream) {
  if (!ctx) return -1;
  if (fn < 0 || fn >= htp::hm::F_COUNT) return fail(ctx, "libm: unknown function id");
  if (n < 0 || (n > 0 && (!x || !out))) return fail(ctx, "libm: bad arguments");
  if ((fn == htp::hm::F_ATAN2 || fn == htp::hm::F_HYPOT || fn == htp::hm::F_POW) && n > 0 && !y)
    return fail(ctx, "libm: two-argument function needs y");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t blocks = (n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192;
  hipLaunchKernelGGL(libm_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, fn, x, y, out, n);
  HIPCHK(hipGetLastError());
  return 0;
}
