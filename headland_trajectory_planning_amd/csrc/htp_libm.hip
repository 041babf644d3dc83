// libhtp.so: the planner cores' correctly rounded libm (htp_libm.h) evaluated on the device over a batch of
// arguments -- the parity surface that shows the gfx950 build of each function returns the host build's doubles --
// and the fp64 matrix-core op on caller tiles, the parity surface of the host model of its rounding.
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

typedef double dbl4 __attribute__((ext_vector_type(4)));

// D = A (16x4) B (4x16) + C, one v_mfma_f64_16x16x4f64 per wavefront, in the operand layout of the solver's
// Riccati tiles (obca_core.h riccati_*_mfma; wave_ctx.h DevWave::mfma16)
__global__ __launch_bounds__(64) void mfma_kernel(const double* __restrict__ A, const double* __restrict__ B,
                                                  const double* __restrict__ C, double* __restrict__ D, int64_t n) {
  const int64_t t = blockIdx.x;
  if (t >= n) return;
  const int l = threadIdx.x, row = l & 15, k = l >> 4;
  const double a = A[t * 64 + row * 4 + k], b = B[t * 64 + k * 16 + row];
  dbl4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (k + 4 * r) * 16 + row];
  const dbl4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[t * 256 + (k + 4 * r) * 16 + row] = d[r];
}

}  // namespace

extern "C" int htp_mfma_f64_probe(htp_ctx* ctx, const double* A, const double* B, const double* C, double* D,
                                  int64_t n, void* stream) {
  if (!ctx) return -1;
  if (n < 0 || (n > 0 && (!A || !B || !C || !D))) return fail(ctx, "mfma probe: bad arguments");
  if (n == 0) return 0;
  if (n > (int64_t)1 << 30) return fail(ctx, "mfma probe: too many tiles");
  HIPCHK(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(mfma_kernel, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream, A, B, C, D, n);
  HIPCHK(hipGetLastError());
  return 0;
}

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
