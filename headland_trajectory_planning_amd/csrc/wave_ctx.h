// Wave context for the solver core: one problem per 64-lane wavefront on
// gfx950 (DevWave), or a single serial lane for the test-only host build
// (HostLane, tests/ only -- never a product fallback).
#pragma once
#include <cmath>

namespace htp {

#if defined(__HIPCC__)
struct DevWave {
  using gd = __attribute__((address_space(1))) double;  // HBM (global) doubles
  using ld = __attribute__((address_space(3))) double;  // LDS doubles
  using li = __attribute__((address_space(3))) int;     // LDS ints
  template <class T>
  using cst = const __attribute__((address_space(4))) T;  // constant (scalar-cached) memory
  static constexpr int width = 64;
  int lane;
  ld* lds;    // per-wave LDS scratch
  li* ildsp;  // per-wave LDS int scratch
  __device__ __forceinline__ void sync() const { __syncthreads(); }
  __device__ __forceinline__ double sum(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
  __device__ __forceinline__ double maxv(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
  }
  __device__ __forceinline__ double minv(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
  }
  __device__ __forceinline__ int isum(int v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
  __device__ __forceinline__ double bcast(double v, int src) const { return __shfl(v, src, 64); }
  __device__ __forceinline__ long long clock() const { return (long long)__builtin_amdgcn_s_memtime(); }
};
#endif

struct HostLane {
  using gd = double;
  using ld = double;
  using li = int;
  template <class T>
  using cst = const T;
  static constexpr int width = 1;
  int lane = 0;
  double* lds;
  int* ildsp;
  void sync() const {}
  double sum(double v) const { return v; }
  double maxv(double v) const { return v; }
  double minv(double v) const { return v; }
  int isum(int v) const { return v; }
  double bcast(double v, int) const { return v; }
  long long clock() const { return 0; }
};

}  // namespace htp
