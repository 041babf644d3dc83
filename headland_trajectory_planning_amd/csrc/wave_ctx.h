// Wave context for the solver core: one problem per 64-lane wavefront on
// gfx950 (DevWave), or a single serial lane for the test-only host build
// (HostLane, tests/ only -- never a product fallback).
#pragma once
#include <chrono>
#include <cmath>

namespace htp {

#if defined(__HIPCC__)
typedef double dbl4 __attribute__((ext_vector_type(4)));

struct DevWave {
  using gd = __attribute__((address_space(1))) double;  // HBM (global) doubles
  using ld = __attribute__((address_space(3))) double;  // LDS doubles
  using li = __attribute__((address_space(3))) int;     // LDS ints
  template <class T>
  using cst = const __attribute__((address_space(4))) T;  // constant (scalar-cached) memory
  static constexpr int width = 64;
  static constexpr bool kMfma = true;  // v_mfma_f64_16x16x4f64 available (gfx950)
  int lane;
  ld* lds;    // per-wave LDS scratch
  li* ildsp;  // per-wave LDS int scratch
  // The workgroup is a single wavefront: its LDS and global accesses are
  // performed in program order, so cross-lane RAW only needs the compiler not
  // to reorder memory operations -- a wavefront-scope fence (no s_waitcnt
  // vmcnt(0), unlike __syncthreads(), so prefetches and stores stay in flight).
  __device__ __forceinline__ void sync() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // Reduction results are identical in every lane; readfirstlane tells the
  // compiler so (scalar registers, uniform branches instead of exec masks).
  __device__ __forceinline__ static double uni(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  }
  __device__ __forceinline__ double sum(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return uni(v);
  }
  __device__ __forceinline__ double maxv(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return uni(v);
  }
  __device__ __forceinline__ double minv(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return uni(v);
  }
  __device__ __forceinline__ int isum(int v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return __builtin_amdgcn_readfirstlane(v);
  }
  // compaction: this lane's index among the lanes with `pred` set, and (uniform) how many are set
  __device__ __forceinline__ int rank(bool pred, int& total) const {
    const unsigned long long m = __ballot(pred ? 1 : 0);
    total = __builtin_amdgcn_readfirstlane((int)__popcll(m));
    return (int)__popcll(m & ((1ull << lane) - 1ull));
  }
  __device__ __forceinline__ double uniform(double v) const { return uni(v); }
  __device__ __forceinline__ int uniform_i(int v) const { return __builtin_amdgcn_readfirstlane(v); }
  __device__ __forceinline__ double bcast(double v, int src) const { return __shfl(v, src, 64); }
  __device__ __forceinline__ long long clock() const { return (long long)__builtin_amdgcn_s_memtime(); }
  // constant-rate wall clock (hipDeviceAttributeWallClockRate ticks/s), for max_cpu_time
  __device__ __forceinline__ long long wall() const { return (long long)wall_clock64(); }
  // D = A (16x4) B (4x16) + C in fp64 on the matrix core.  Lane l supplies a = A[l&15][l>>4] and
  // b = B[l>>4][l&15]; c/d[r] = C[(l>>4) + 4r][l&15] (MI355X_MICROARCH / cdna_hip_programming f64 map).
  __device__ __forceinline__ static dbl4 mfma16(double a, double b, dbl4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
};

// DevWave whose lane index and LDS bases are values the compiler rematerializes (the work-item id; the addresses
// of module-scope __shared__ arrays, S::d() / S::i()) instead of fields of a context object.  The solver keeps a
// reference to its context inside an object whose address escapes into out-of-line phases, so after every
// wavefront fence (sync) each use of a field was reloaded through two dependent flat loads.  Same values: the
// arithmetic is unchanged.  One 64-lane wavefront per workgroup (the lane is the work-item id).
template <class S>
struct DevWaveR : DevWave {
  struct Lane {
    __device__ __forceinline__ operator int() const { return (int)__builtin_amdgcn_workitem_id_x(); }
  };
  struct Lds {
    __device__ __forceinline__ operator ld*() const { return S::d(); }
  };
  struct ILds {
    __device__ __forceinline__ operator li*() const { return S::i(); }
  };
  Lane lane;
  Lds lds;
  ILds ildsp;
  __device__ __forceinline__ int rank(bool pred, int& total) const {
    const unsigned long long m = __ballot(pred ? 1 : 0);
    total = __builtin_amdgcn_readfirstlane((int)__popcll(m));
    return (int)__popcll(m & ((1ull << (int)lane) - 1ull));
  }
};
#endif

struct HostLane {
  using gd = double;
  using ld = double;
  using li = int;
  template <class T>
  using cst = const T;
  static constexpr int width = 1;
  static constexpr bool kMfma = false;
  int lane = 0;
  double* lds;
  int* ildsp;
  void sync() const {}
  double sum(double v) const { return v; }
  double maxv(double v) const { return v; }
  double minv(double v) const { return v; }
  int isum(int v) const { return v; }
  int rank(bool pred, int& total) const { total = pred ? 1 : 0; return 0; }
  double bcast(double v, int) const { return v; }
  double uniform(double v) const { return v; }
  int uniform_i(int v) const { return v; }
  long long clock() const { return 0; }
  long long wall() const {  // ns (Options::wall_rate = 1e9 on the host builds)
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }
};

}  // namespace htp
