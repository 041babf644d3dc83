// TEST-ONLY: a 64-lane wavefront simulated by 64 std::threads (std::barrier per
// sync, shared-array reductions) for the solver cores' lane-parallel code, so
// races and out-of-bounds lane indexing can be hunted on the CPU (ASan/UBSan)
// without a GPU.  Never part of the product.
#pragma once
#include <barrier>
#include <cmath>

namespace htp {
struct WaveShared {
  std::barrier<> bar{64};
  double red[64];
  int ired[64];
};
struct ThreadWave {
  using gd = double;
  using ld = double;
  using li = int;
  template <class T>
  using cst = const T;
  static constexpr int width = 64;
  static constexpr bool kMfma = false;
  int lane;
  double* lds;
  int* ildsp;
  WaveShared* sh;
  void sync() const { sh->bar.arrive_and_wait(); }
  double sum(double v) const {
    sync();
    sh->red[lane] = v;
    sync();
    double s = 0;
    for (int i = 0; i < 64; ++i) s += sh->red[i];
    sync();
    return s;
  }
  double maxv(double v) const {
    sync(); sh->red[lane] = v; sync();
    double s = sh->red[0];
    for (int i = 1; i < 64; ++i) s = fmax(s, sh->red[i]);
    sync();
    return s;
  }
  double minv(double v) const {
    sync(); sh->red[lane] = v; sync();
    double s = sh->red[0];
    for (int i = 1; i < 64; ++i) s = fmin(s, sh->red[i]);
    sync();
    return s;
  }
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
    double r = sh->red[src];
    sync();
    return r;
  }
};
}  // namespace htp
