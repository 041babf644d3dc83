// TEST-ONLY: a bit-exact host model of the gfx950 wavefront the solver core runs on (DevWave, wave_ctx.h).
// 64 std::threads play the 64 lanes (std::barrier per c.sync()); every cross-lane operation is evaluated in the
// order the device evaluates it:
//   sum / maxv / minv ... the xor butterfly of DevWave::sum (v op= shfl_xor(v, o), o = 32, 16, .., 1);
//   mfma16 ............. v_mfma_f64_16x16x4f64 on the lanes' operands, D = C + A B as a fused multiply-add chain
//                        over k = 0..3 (the model tests/test_gpu_mfma_model.py pins on the hardware).
// Built with clang (-ffp-contract=on, FMA enabled) like the device translation unit, so every a * b + c of the
// source is fused or not fused alike on both; the solver's libm is the deterministic one on both
// (obca_core.h HTP_SOLVER_DETLIBM: htp_fastm.h's explicit-FMA sin / cos / tan / log, htp_libm.h's pow).  The device solve is then reproduced on the host bit for bit
// (tests/test_gpu_emulation.py) -- the witness that a device / oracle divergence is summation order, not a bug.
// Never part of the product.
#pragma once
#include <barrier>
#include <cmath>

namespace htp {

typedef double dbl4 __attribute__((ext_vector_type(4)));

struct EmuShared {
  std::barrier<> bar{64};
  double red[64];
  int ired[64];
  double ma[64], mb[64];
};

struct EmuWave {
  using gd = double;
  using ld = double;
  using li = int;
  template <class T>
  using cst = const T;
  static constexpr int width = 64;
  static constexpr bool kMfma = true;
  int lane;
  double* lds;
  int* ildsp;
  EmuShared* sh;
  static inline thread_local const EmuWave* self = nullptr;

  void sync() const { sh->bar.arrive_and_wait(); }
  template <class Op>
  double butterfly(double v, Op op) const {
    for (int o = 32; o > 0; o >>= 1) {
      sync();
      sh->red[lane] = v;
      sync();
      v = op(v, sh->red[lane ^ o]);
    }
    sync();
    return v;
  }
  double sum(double v) const { return butterfly(v, [](double a, double b) { return a + b; }); }
  double maxv(double v) const { return butterfly(v, [](double a, double b) { return fmax(a, b); }); }
  double minv(double v) const { return butterfly(v, [](double a, double b) { return fmin(a, b); }); }
  int isum(int v) const {
    sync(); sh->ired[lane] = v; sync();
    int s = 0;
    for (int i = 0; i < 64; ++i) s += sh->ired[i];
    sync();
    return s;
  }
  int rank(bool pred, int& total) const {
    sync(); sh->ired[lane] = pred ? 1 : 0; sync();
    int r = 0, t = 0;
    for (int i = 0; i < 64; ++i) { if (i < lane) r += sh->ired[i]; t += sh->ired[i]; }
    sync();
    total = t;
    return r;
  }
  long long clock() const { return 0; }
  long long wall() const { return 0; }
  double uniform(double v) const { return v; }
  int uniform_i(int v) const { return v; }
  double bcast(double v, int src) const {
    sync(); sh->red[lane] = v; sync();
    const double r = sh->red[src];
    sync();
    return r;
  }
  // lane l supplies a = A[l & 15][l >> 4], b = B[l >> 4][l & 15]; d[r] = D[(l >> 4) + 4 r][l & 15]
  static dbl4 mfma16(double a, double b, dbl4 c) {
    const EmuWave& w = *self;
    EmuShared* s = w.sh;
    w.sync();
    s->ma[w.lane] = a;
    s->mb[w.lane] = b;
    w.sync();
    const int col = w.lane & 15, rg = w.lane >> 4;
    dbl4 d;
    for (int r = 0; r < 4; ++r) {
      const int row = rg + 4 * r;
      double acc = c[r];
      for (int k = 0; k < 4; ++k) acc = std::fma(s->ma[row + 16 * k], s->mb[col + 16 * k], acc);
      d[r] = acc;
    }
    w.sync();
    return d;
  }
};

}  // namespace htp
