// Wave context for the solver core: one problem per 64-lane wavefront on
// gfx950 (DevWave), or a single serial lane for the test-only host build
// (HostLane, tests/ only -- never a product fallback).
#pragma once
#include <cmath>

namespace htp {

#if defined(__HIPCC__)
struct DevWave {
  static constexpr int width = 64;
  int lane;
  double* lds;  // per-wave LDS scratch
  int* ildsp;   // per-wave LDS int scratch
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
};
#endif

struct HostLane {
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
};

}  // namespace htp
