// TEST-ONLY: the host build of the hybrid A* core (hastar_core.h +
// dubins_core.h + rs_core.h, serial lane, csrc/hastar_hostsim.cpp) as a
// standalone executable built with -fsanitize=address,undefined by
// tests/_hostsim.py::hastar_asan, with exact-size buffers, so an out-of-bounds
// index in the Dubins/spline scratch, the node/slot/heap arrays, the private
// arrays or the shared block, or undefined behaviour on the Pawn or King paths
// aborts the run.  (A 64-thread simulation of the wave does not apply to this
// core: its heap and table updates are executed redundantly by every lane in
// lockstep, which threads cannot reproduce.)  Never part of the product.
#include <cstdlib>
#include "hastar_hostsim.cpp"
// Standalone driver (so the sanitizers are linked into an executable, not
// preloaded into Python): argv[1] = packed batch written by
// tests/_hostsim.py::hastar_asan, argv[2] = result file.
#include <cstdio>
template <class T>
static std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
  return v;
}
template <class T>
static void wr(FILE* f, const std::vector<T>& v) { fwrite(v.data(), sizeof(T), v.size(), f); }

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  auto h = rd<int32_t>(f, 8);
  const int B = h[0], np = h[1], nv = h[2], ng = h[3], nm = h[4];
  auto params = rd<double>(f, (size_t)B * HTP_HA_NPARAM);
  auto desc = rd<int32_t>(f, (size_t)B * HTP_HA_NDESC);
  auto poly_off = rd<int32_t>(f, np + 1);
  auto vert = rd<double>(f, (size_t)nv * 2);
  auto lane_len = rd<double>(f, np);
  auto guide = rd<double>(f, (size_t)ng * 4);
  auto mot = rd<double>(f, (size_t)nm * 2);
  fclose(f);
  htp_hastar_batch in{B, np, nv, ng, nm, params.data(), desc.data(), poly_off.data(), vert.data(),
                      lane_len.data(), guide.data(), mot.data(), h[5], h[6], h[7]};
  std::vector<int32_t> st(B), cnt(B), npth(B), nexp(B), log((size_t)B * h[7] * 3);
  std::vector<int64_t> npose(B);
  std::vector<double> x((size_t)B * h[6]), y(x.size()), yaw(x.size()), dir(x.size()), k(x.size());
  htp_hastar_result out{st.data(), cnt.data(), npth.data(), nexp.data(), npose.data(), x.data(), y.data(),
                        yaw.data(), dir.data(), k.data(), h[7] ? log.data() : nullptr};
  const int rc = htp_hostsim_hastar(&in, &out);
  FILE* o = fopen(argv[2], "wb");
  wr(o, st); wr(o, cnt); wr(o, npth); wr(o, nexp); wr(o, npose);
  wr(o, x); wr(o, y); wr(o, yaw); wr(o, dir); wr(o, k); wr(o, log);
  fclose(o);
  return rc == 0 ? 0 : 3;
}
