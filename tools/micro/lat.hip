// EXPERIMENT ONLY: dependent-chain latency of the operations on the stage chain's critical path, one wave:
// v_mfma_f64_16x16x4f64 accumulating into C, the same with its result fed back as the B operand, fp64 division,
// fp64 sqrt, an LDS write -> read round trip.   hipcc --offload-arch=gfx950 -O3 lat.hip -o lat && ./lat
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
__global__ void lat(long long* out, double* sink, double seed) {
  __shared__ double lds[64 * 4];
  const int l = threadIdx.x;
  double a = seed + l * 1e-3, b = 1.0 - l * 1e-4;
  dbl4 acc = {0.1, 0.2, 0.3, 0.4};
  constexpr int R = 256;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < R; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  long long t1 = __builtin_amdgcn_s_memtime();
  double bb = b;
  for (int i = 0; i < R; ++i) { acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0); bb = acc[0] * 1e-9 + b; }
  long long t2 = __builtin_amdgcn_s_memtime();
  double x = a + 2.0;
  for (int i = 0; i < R; ++i) x = (x + 1.0) / (x * 0.5 + 0.25);
  long long t3 = __builtin_amdgcn_s_memtime();
  double y = a + 2.0;
  for (int i = 0; i < R; ++i) y = sqrt(y + 1.5);
  long long t4 = __builtin_amdgcn_s_memtime();
  double z = a;
  for (int i = 0; i < R; ++i) { lds[(l + i) & 255] = z; __builtin_amdgcn_wave_barrier(); z = lds[(l + i + 1) & 255] + 1.0; }
  long long t5 = __builtin_amdgcn_s_memtime();
  double w = a;
  for (int i = 0; i < R; ++i) w = fma(w, 1.0000001, 1e-7);
  long long t6 = __builtin_amdgcn_s_memtime();
  if (l == 0) {
    out[0] = (t1 - t0) / R; out[1] = (t2 - t1) / R; out[2] = (t3 - t2) / R; out[3] = (t4 - t3) / R;
    out[4] = (t5 - t4) / R; out[5] = (t6 - t5) / R;
  }
  sink[l] = acc[0] + acc[1] + acc[2] + acc[3] + x + y + z + w;
}
int main() {
  long long* o; double* s;
  hipMalloc(&o, 64); hipMalloc(&s, 64 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, o, s, 1.0 + rep);
    long long h[6];
    hipMemcpy(h, o, 48, hipMemcpyDeviceToHost);
    printf("cycles per dependent op: mfma acc-chain %lld | mfma via B operand %lld | fp64 div %lld | fp64 sqrt %lld | "
           "lds write+read %lld | fp64 fma %lld\n", h[0], h[1], h[2], h[3], h[4], h[5]);
  }
  return 0;
}
