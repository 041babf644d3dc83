// libhtp.so: batched OBCA interior-point solver for gfx950 (MI355X) + C ABI.
//
// One 64-lane wavefront (one workgroup) per headland-turn problem; the whole
// IPOPT-restated solve (oracle/ipm.py) runs inside one kernel launch, so
// problems converge independently and the hardware dispatcher refills a CU as
// soon as a wave retires (no host round trip per iteration).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>

#define HTP_HD __host__ __device__
#include "wave_ctx.h"
#include "obca_batch.h"

using namespace htp;

namespace {

constexpr int LDS_D = LDS_WAVE_DOUBLES;  // scratch + filter + Riccati stage ring / pivoted blocks (obca_core.h)

// HTP_ONLY44 (experiment variants, tools/build_variants.py): instantiate only the config A-E solver
// obca_solve_kernel<4, 4, 0> -- one instantiation compiles in a quarter of the time
#ifndef HTP_ONLY44
#define HTP_ONLY44 0
#endif

#ifndef HTP_WAVES_PER_EU
#define HTP_WAVES_PER_EU 1
#endif

// The solver's wave context (wave_ctx.h): DevWaveR (1) keeps the lane index and the LDS bases out of memory;
// DevWave (0) holds them as fields (round 5)
#ifndef HTP_CTX_REG
#define HTP_CTX_REG 0
#endif
#if HTP_CTX_REG
__shared__ double g_solver_lds[LDS_D];
__shared__ int g_solver_ilds[2 * NBMAX];
struct SolverLds {
  __device__ __forceinline__ static DevWave::ld* d() { return (DevWave::ld*)g_solver_lds; }
  __device__ __forceinline__ static DevWave::li* i() { return (DevWave::li*)g_solver_ilds; }
};
using SolverWave = DevWaveR<SolverLds>;
#else
using SolverWave = DevWave;
#endif

// Residency cap (experiment knob): HTP_WG_LDS_BYTES = LDS bytes claimed per problem
// (workgroup), so at most floor(160 KB / that) solver waves share one CU.  The
// kernel never touches the padding.  Unset or 0: no cap (4 waves per CU).
inline unsigned lds_pad_bytes() {
  const char* e = getenv("HTP_WG_LDS_BYTES");
  const long want = e ? atol(e) : 0;
  const long fixed = (long)sizeof(double) * LDS_D + (long)sizeof(int) * 2 * NBMAX;
  if (want <= fixed) return 0;
  return (unsigned)(want > 160 * 1024 ? 160 * 1024 - fixed : want - fixed);
}

// Work source of a solve launch: a static range (ticket t solves problem t, t <
// n_static) or a host work queue (htp_queue_*: ticket t solves items[t] once the
// host has published it).
struct QueueHost {              // pinned, GPU-coherent host memory
  long long avail;              // tickets published (host writes, release)
  int closed;                   // no more tickets will be published
  int pad0;
  long long pad1[6];
  long long claimed;            // claim hint written by the waves (separate line)
  long long pad2[7];
  int items[1];                 // [capacity] problem indices
};
struct WorkSrc {
  unsigned long long* next;     // device ticket counter (agent-scope atomics)
  QueueHost* q;                 // nullptr: static range
  long long n_static;
  long long max_wait;           // device wall-clock ticks a wave may wait for a ticket
};
struct OutView {                // per-ticket outputs (any may be null); x per problem
  double* objective;
  int32_t *status, *iters, *n_factor;
  double* nlp_error;
  int32_t* n_resto;
};

// Next ticket of this wave and its problem index (uniform); false = retire.
__device__ __forceinline__ bool claim(const WorkSrc& w, long long& t, long long& pid) {
  long long v = 0;
  if (threadIdx.x == 0) v = (long long)__hip_atomic_fetch_add(w.next, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __shfl(v, 0, 64);
  if (!w.q) {
    pid = t;
    return t < w.n_static;
  }
  if (threadIdx.x == 0) {  // claimed = max(claimed, t + 1): a monotone hint (compare-and-swap, a PCIe atomic)
    long long cur = __hip_atomic_load(&w.q->claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    while (cur < t + 1 &&
           !__hip_atomic_compare_exchange_strong(&w.q->claimed, &cur, t + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM)) {
    }
  }
  const long long t0 = (long long)wall_clock64();
  int ok = 0;
  for (;;) {
    const long long av = __hip_atomic_load(&w.q->avail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < av) { ok = 1; break; }
    if (__hip_atomic_load(&w.q->closed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) {
      // closed after the last publish: re-read avail once (publish precedes close)
      ok = t < __hip_atomic_load(&w.q->avail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    if ((long long)wall_clock64() - t0 > w.max_wait) break;   // host gone: retire
    __builtin_amdgcn_s_sleep(127);
  }
  ok = __shfl(ok, 0, 64);
  if (!ok) return false;
  int it = 0;
  if (threadIdx.x == 0) it = __hip_atomic_load(&w.q->items[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  pid = __shfl(it, 0, 64);
  return true;
}

// One wavefront per problem at a time; each wave keeps claiming tickets until
// its work source is exhausted, so a long solve holds one wave and never the
// launch (no per-launch tail); the workspace is per wave, not per problem.
// FORM 0: optimizer.py (EN, EM edges of the body / obstacle polytopes); FORM 1: the point
// formulation of optimizer_points.py (lambda-only local blocks, EN unused).
template <int EN, int EM, int FORM>
__global__ __launch_bounds__(64, HTP_WAVES_PER_EU) void obca_solve_kernel(const Shape* __restrict__ shp, BatchView b,
                                                        double* __restrict__ ws_all, int64_t ws_stride,
                                                        Result* __restrict__ res, double* __restrict__ xout,
                                                        WorkSrc src, OutView ov) {
#if !HTP_CTX_REG
  __shared__ double lds_[LDS_D];
  __shared__ int ilds_[2 * NBMAX];
  DevWave::ld* lds = (DevWave::ld*)lds_;
  DevWave::li* ilds = (DevWave::li*)ilds_;
#endif
  using CS = DevWave::cst<Shape>;
  CS* sh = (CS*)shp;
  double* ws = ws_all + (int64_t)blockIdx.x * ws_stride;
  long long t, p;
  while (claim(src, t, p)) {
#if HTP_CTX_REG
    SolverWave c{};
#else
    SolverWave c{(int)threadIdx.x, lds, ilds};
#endif
    ProblemIn in = problem_view(b, sh->D, p);
    ObcaSolver<SolverWave, EN, EM, FORM> S(c, sh->D, sh->L, sh->o, in, ws);
    Result r{};
    S.run(r);
    if (threadIdx.x == 0) {
      if (res) res[t] = r;
      if (ov.objective) ov.objective[t] = r.objective;
      if (ov.status) ov.status[t] = r.status;
      if (ov.iters) ov.iters[t] = r.iters;
      if (ov.n_factor) ov.n_factor[t] = r.n_factor;
      if (ov.nlp_error) ov.nlp_error[t] = r.nlp_error;
      if (ov.n_resto) ov.n_resto[t] = r.n_resto;
    }
    const double* x = ws + sh->L.x;
    const int n = sh->D.n;
    for (int q = threadIdx.x; q < n; q += 64) xout[p * n + q] = x[q];
    c.sync();
  }
}

}  // namespace

#include "htp_ctx.h"

extern "C" {

int htp_obca_sizes(int32_t N, int32_t M, int32_t K, int32_t time_opt, const int32_t* eo, const int32_t* eb,
                   int64_t* n_var, int64_t* n_eq, int64_t* n_ineq, int64_t* ws_doubles) {
  if (N < 2 || M < 1 || M > MAXM || K < 1 || K > MAXK) return -1;
  Dims D;
  make_dims(D, N, M, K, time_opt, eo, eb);
  Layout L = make_layout(D);
  if (n_var) *n_var = D.n;
  if (n_eq) *n_eq = D.mc;
  if (n_ineq) *n_ineq = D.md;
  if (ws_doubles) *ws_doubles = L.total;
  return 0;
}

htp_ctx* htp_create(int32_t device) {
  htp_ctx* c = new htp_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    c->err = "hipSetDevice failed";
    return c;
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    c->wall_rate = 1e3 * (double)khz;
  (void)hipEventCreate(&c->ev0);
  (void)hipEventCreate(&c->ev1);
  (void)hipEventCreate(&c->rs_ev0);
  (void)hipEventCreate(&c->rs_ev1);
  (void)hipEventCreate(&c->ha_ev0);
  (void)hipEventCreate(&c->ha_ev1);
  (void)hipEventCreate(&c->yp_ev0);
  (void)hipEventCreate(&c->yp_ev1);
  (void)hipEventCreate(&c->rp_ev0);
  (void)hipEventCreate(&c->rp_ev1);
  (void)hipEventCreate(&c->oge_ev0);
  (void)hipEventCreate(&c->oge_ev1);
  (void)hipEventCreate(&c->ct_ev0);
  (void)hipEventCreate(&c->ct_ev1);
  (void)hipEventCreate(&c->ch_ev0);
  (void)hipEventCreate(&c->ch_ev1);
  return c;
}

void htp_destroy(htp_ctx* c) {
  if (!c) return;
  if (c->ws) (void)hipFree(c->ws);
  if (c->next) (void)hipFree(c->next);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->shape) (void)hipFree(c->shape);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->rs_scratch) (void)hipFree(c->rs_scratch);
  if (c->rs_ev0) (void)hipEventDestroy(c->rs_ev0);
  if (c->rs_ev1) (void)hipEventDestroy(c->rs_ev1);
  if (c->ha_ws) (void)hipFree(c->ha_ws);
  if (c->ha_ev0) (void)hipEventDestroy(c->ha_ev0);
  if (c->ha_ev1) (void)hipEventDestroy(c->ha_ev1);
  if (c->yp_ws) (void)hipFree(c->yp_ws);
  if (c->yp_ev0) (void)hipEventDestroy(c->yp_ev0);
  if (c->yp_ev1) (void)hipEventDestroy(c->yp_ev1);
  if (c->rp_ws) (void)hipFree(c->rp_ws);
  if (c->rp_ev0) (void)hipEventDestroy(c->rp_ev0);
  if (c->rp_ev1) (void)hipEventDestroy(c->rp_ev1);
  if (c->oge_ev0) (void)hipEventDestroy(c->oge_ev0);
  if (c->oge_ev1) (void)hipEventDestroy(c->oge_ev1);
  if (c->ct_ws) (void)hipFree(c->ct_ws);
  if (c->ct_ev0) (void)hipEventDestroy(c->ct_ev0);
  if (c->ct_ev1) (void)hipEventDestroy(c->ct_ev1);
  if (c->ch_ws) (void)hipFree(c->ch_ws);
  if (c->ch_ev0) (void)hipEventDestroy(c->ch_ev0);
  if (c->ch_ev1) (void)hipEventDestroy(c->ch_ev1);
  if (c->yc_ws) (void)hipFree(c->yc_ws);
  for (auto e : c->yc_ev)
    if (e) (void)hipEventDestroy(e);
  delete c;
}

const char* htp_last_error(htp_ctx* c) { return c ? c->err.c_str() : "null context"; }

int htp_set_option(htp_ctx* ctx, const char* name, double v) {
  if (!ctx || !name) return -1;
  if (set_option(ctx->opt, name, v)) return fail(ctx, std::string("unknown option ") + name);
  return 0;
}

double htp_last_kernel_ms(htp_ctx* c) {
  if (!c || !c->ev1) return 0.0;
  if (hipEventSynchronize(c->ev1) != hipSuccess) return c->last_ms;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->last_ms = ms;
  return c->last_ms;
}

// Diagnostic: per-problem phase cycle counters of the last solve ([batch][6] int64;
// local sweeps, stage assembly, stage chain, KKT solves, total, reserved).
int htp_last_cycles(htp_ctx* ctx, int64_t* out, int32_t batch) {
  if (!ctx || !ctx->scratch) return -1;
  std::vector<Result> r((size_t)batch);
  HIPCHK(hipMemcpy(r.data(), ctx->scratch, sizeof(Result) * (size_t)batch, hipMemcpyDeviceToHost));
  for (int p = 0; p < batch; ++p)
    for (int k = 0; k < 8; ++k) out[(size_t)p * 8 + k] = r[(size_t)p].cyc[k];
  return 0;
}

}  // extern "C"

struct htp_queue {
  htp_ctx* ctx;
  QueueHost* h;                 // hipHostMalloc (coherent)
  unsigned long long* next;     // device ticket counter
  int64_t cap;
  int64_t limit;                // problems resident for the launch (publish checks pid < limit)
};

namespace {

template <int EN, int EM, int FORM = 0>
int resident_waves_t(htp_ctx* ctx, unsigned pad) {
  int per_cu = 0, cus = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)obca_solve_kernel<EN, EM, FORM>, 64, pad));
  HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
  return per_cu * cus > 0 ? per_cu * cus : 1;
}

bool uniform44(const Dims& D) {
  bool u = true;
  for (int m = 0; m < D.M; ++m) u = u && D.eo[m] == 4;
  for (int k = 0; k < D.K; ++k) u = u && D.eb[k] == 4;
  return u;
}

// Shared launch path of the static-range and queue modes.
// The ticket counter, the per-wave workspace and the result scratch belong to the context: a launch is ordered
// after the context's previous one (stream order, or an event wait across streams).  A queue-mode launch whose
// queue is still open never ends by itself, so a launch behind it is rejected loudly instead of waiting forever.
int check_idle(htp_ctx* ctx, hipStream_t s) {
  if (ctx->ev1 && hipEventQuery(ctx->ev1) == hipErrorNotReady) {
    const QueueHost* q = (const QueueHost*)ctx->last_queue;
    if (q && !__atomic_load_n(&q->closed, __ATOMIC_ACQUIRE))
      return fail(ctx, "[OBCA] the previous queue launch of this context is still open (htp_queue_close it first)");
  }
  return order_after(ctx, ctx->ev1, s);
}

int launch_solve(htp_ctx* ctx, const htp_obca_batch* in, const htp_obca_result* out, hipStream_t s, WorkSrc src,
                 int64_t waves, bool keep_results) {
  if (check_idle(ctx, s)) return -1;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  Layout L = make_layout(D);
  const bool u44 = uniform44(D);
  const unsigned pad = lds_pad_bytes();
#if HTP_ONLY44
  if (!u44) return fail(ctx, "[OBCA] experiment build (HTP_ONLY44): 4-edge polytopes only");
  const int cap = resident_waves_t<4, 4>(ctx, pad);
#else
  const int cap = u44 ? resident_waves_t<4, 4>(ctx, pad) : resident_waves_t<MAXE, MAXE>(ctx, pad);
#endif
  if (cap < 0) return -1;
  if (waves <= 0 || waves > cap) waves = cap;
  if (src.q == nullptr && waves > src.n_static) waves = src.n_static;
  if (waves < 1) waves = 1;
  if (ensure(ctx, &ctx->ws, &ctx->ws_bytes, (size_t)L.total * sizeof(double) * (size_t)waves)) return -1;
  if (keep_results && ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, sizeof(Result) * (size_t)in->batch)) return -1;
  if (!ctx->shape) HIPCHK(hipMalloc((void**)&ctx->shape, sizeof(Shape)));
  Shape hs{D, L, ctx->opt};
  hs.o.wall_rate = ctx->wall_rate;
  BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
              in->init_control, in->init_mu, in->init_lambda};
  OutView ov{out->objective, out->status, out->iterations, out->n_factor, out->nlp_error, out->n_resto};
  HIPCHK(hipMemcpyAsync(ctx->shape, &hs, sizeof(Shape), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(src.next, 0, sizeof(unsigned long long), s));
  HIPCHK(hipEventRecord(ctx->ev0, s));
  Result* res = keep_results ? (Result*)ctx->scratch : nullptr;
  if (u44) {
    if (pad) HIPCHK(hipFuncSetAttribute((const void*)obca_solve_kernel<4, 4, 0>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad));
    hipLaunchKernelGGL((obca_solve_kernel<4, 4, 0>), dim3((unsigned)waves), dim3(64), pad, s, (const Shape*)ctx->shape, b,
                       (double*)ctx->ws, (int64_t)L.total, res, out->x, src, ov);
  } else {
#if !HTP_ONLY44
    if (pad) HIPCHK(hipFuncSetAttribute((const void*)obca_solve_kernel<MAXE, MAXE, 0>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad));
    hipLaunchKernelGGL((obca_solve_kernel<MAXE, MAXE, 0>), dim3((unsigned)waves), dim3(64), pad, s,
                       (const Shape*)ctx->shape, b, (double*)ctx->ws, (int64_t)L.total, res, out->x, src, ov);
#endif
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev1, s));
  ctx->last_queue = src.q;
  return 0;
}

}  // namespace

extern "C" {

int32_t htp_obca_resident_waves(htp_ctx* ctx, const htp_obca_batch* in) {
  if (!ctx || !in) return -1;
  const char* e = nullptr;
  if (check_shape(in, &e)) return fail(ctx, e);
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  HIPCHK(hipSetDevice(ctx->device));
#if HTP_ONLY44
  return resident_waves_t<4, 4>(ctx, lds_pad_bytes());
#else
  return uniform44(D) ? resident_waves_t<4, 4>(ctx, lds_pad_bytes()) : resident_waves_t<MAXE, MAXE>(ctx, lds_pad_bytes());
#endif
}

int htp_obca_solve_batch_device(htp_ctx* ctx, const htp_obca_batch* in, htp_obca_result* out, void* stream) {
  if (!ctx || !in || !out) return -1;
  const char* e = nullptr;
  if (check_shape(in, &e)) return fail(ctx, e);
  if (in->batch == 0) return 0;
  if (!out->x) return fail(ctx, "[OBCA] out->x is required");
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->next) HIPCHK(hipMalloc((void**)&ctx->next, 256));
  WorkSrc src{(unsigned long long*)ctx->next, nullptr, (long long)in->batch, 0};
  return launch_solve(ctx, in, out, (hipStream_t)stream, src, 0, true);
}

htp_queue* htp_queue_create(htp_ctx* ctx, int64_t capacity) {
  if (!ctx || capacity < 1 || capacity > (int64_t)1 << 31) return nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
  htp_queue* q = new htp_queue{ctx, nullptr, nullptr, capacity, INT64_MAX};
  const size_t bytes = sizeof(QueueHost) + sizeof(int) * (size_t)capacity;
  if (hipHostMalloc((void**)&q->h, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipMalloc((void**)&q->next, 256) != hipSuccess) {
    ctx->err = "htp_queue_create: allocation failed";
    htp_queue_destroy(q);
    return nullptr;
  }
  std::memset((void*)q->h, 0, bytes);
  return q;
}

void htp_queue_destroy(htp_queue* q) {
  if (!q) return;
  if (q->h) (void)hipHostFree(q->h);
  if (q->next) (void)hipFree(q->next);
  delete q;
}

int htp_queue_publish(htp_queue* q, const int32_t* pids, int64_t n) {
  if (!q || n < 0 || (n && !pids)) return -1;
  if (__atomic_load_n(&q->h->closed, __ATOMIC_ACQUIRE)) return -1;
  const long long av = __atomic_load_n(&q->h->avail, __ATOMIC_RELAXED);
  if (av + n > q->cap) return -1;
  for (int64_t k = 0; k < n; ++k)
    if (pids[k] < 0 || pids[k] >= q->limit) return -1;
  std::memcpy(&q->h->items[av], pids, sizeof(int32_t) * (size_t)n);
  __atomic_store_n(&q->h->avail, av + n, __ATOMIC_RELEASE);
  return 0;
}

int htp_queue_close(htp_queue* q) {
  if (!q) return -1;
  __atomic_store_n(&q->h->closed, 1, __ATOMIC_RELEASE);
  return 0;
}

int64_t htp_queue_published(const htp_queue* q) { return q ? __atomic_load_n(&q->h->avail, __ATOMIC_ACQUIRE) : -1; }
int64_t htp_queue_claimed(const htp_queue* q) { return q ? __atomic_load_n(&q->h->claimed, __ATOMIC_ACQUIRE) : -1; }

int htp_obca_solve_queue_device(htp_ctx* ctx, const htp_obca_batch* in, htp_queue* q, htp_obca_result* out,
                                void* stream, int32_t waves, double max_wait_s) {
  if (!ctx || !in || !q || !out) return -1;
  const char* e = nullptr;
  if (check_shape(in, &e)) return fail(ctx, e);
  if (!out->x) return fail(ctx, "[OBCA] out->x is required");
  if (q->ctx->device != ctx->device) return fail(ctx, "htp_obca_solve_queue_device: queue of another device");
  const int64_t av = htp_queue_published(q);
  for (int64_t t = 0; t < av; ++t)
    if (q->h->items[t] < 0 || q->h->items[t] >= in->batch) return fail(ctx, "[OBCA] queued problem index out of range");
  q->limit = in->batch;
  HIPCHK(hipSetDevice(ctx->device));
  if (!(max_wait_s > 0)) max_wait_s = 60.0;
  WorkSrc src{q->next, (QueueHost*)q->h, 0, (long long)(max_wait_s * ctx->wall_rate)};
  return launch_solve(ctx, in, out, (hipStream_t)stream, src, waves, false);
}

int htp_obca_solve_batch(htp_ctx* ctx, const htp_obca_batch* in, htp_obca_result* out) {
  if (!ctx || !in || !out) return -1;
  const char* e = nullptr;
  if (check_shape(in, &e)) return fail(ctx, e);
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  const int64_t B = in->batch;
  auto bytes = [&](int64_t n) { return (size_t)(n * (int64_t)sizeof(double)); };
  const size_t sz_traj = bytes(B * D.N * NS), sz_A = bytes(B * D.TEo * 2), sz_b = bytes(B * D.TEo);
  const size_t sz_G = bytes(B * D.TEb * 2), sz_g = bytes(B * D.TEb), sz_p = bytes(B * NPARAM);
  const size_t sz_u = in->init_control ? bytes(B * (D.N - 1) * NC) : 0;
  const size_t sz_mu = in->init_mu ? bytes(B * D.N * D.mu_count) : 0;
  const size_t sz_la = in->init_lambda ? bytes(B * D.N * D.lam_count) : 0;
  const size_t sz_x = bytes(B * D.n);
  std::vector<size_t> sizes = {sz_traj, sz_A, sz_b, sz_G, sz_g, sz_p, sz_u, sz_mu, sz_la, sz_x,
                               bytes(B), (size_t)B * 4, (size_t)B * 4, (size_t)B * 4, bytes(B), (size_t)B * 4};
  size_t total = 0;
  std::vector<size_t> off;
  for (size_t s : sizes) { off.push_back(total); total += (s + 255) & ~size_t(255); }
  char* dev = nullptr;
  HIPCHK(hipMalloc((void**)&dev, total));
  const void* srcs[9] = {in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
                         in->init_control, in->init_mu, in->init_lambda};
  for (int k = 0; k < 9; ++k)
    if (sizes[k]) {
      hipError_t er = hipMemcpy(dev + off[k], srcs[k], sizes[k], hipMemcpyHostToDevice);
      if (er != hipSuccess) { (void)hipFree(dev); return fail(ctx, hipGetErrorString(er)); }
    }
  htp_obca_batch din = *in;
  din.traj = (const double*)(dev + off[0]);
  din.obs_A = (const double*)(dev + off[1]);
  din.obs_b = (const double*)(dev + off[2]);
  din.body_G = (const double*)(dev + off[3]);
  din.body_g = (const double*)(dev + off[4]);
  din.params = (const double*)(dev + off[5]);
  din.init_control = sz_u ? (const double*)(dev + off[6]) : nullptr;
  din.init_mu = sz_mu ? (const double*)(dev + off[7]) : nullptr;
  din.init_lambda = sz_la ? (const double*)(dev + off[8]) : nullptr;
  htp_obca_result dout;
  dout.x = (double*)(dev + off[9]);
  dout.objective = (double*)(dev + off[10]);
  dout.status = (int32_t*)(dev + off[11]);
  dout.iterations = (int32_t*)(dev + off[12]);
  dout.n_factor = (int32_t*)(dev + off[13]);
  dout.nlp_error = (double*)(dev + off[14]);
  dout.n_resto = (int32_t*)(dev + off[15]);
  int rc = htp_obca_solve_batch_device(ctx, &din, &dout, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("solve kernel: ") + hipGetErrorString(er));
  }
  if (rc == 0) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) ctx->last_ms = ms;
    struct { void* dst; size_t off, sz; } outs[7] = {{out->x, off[9], sz_x}, {out->objective, off[10], bytes(B)},
                                                     {out->status, off[11], (size_t)B * 4}, {out->iterations, off[12], (size_t)B * 4},
                                                     {out->n_factor, off[13], (size_t)B * 4}, {out->nlp_error, off[14], bytes(B)},
                                                     {out->n_resto, off[15], (size_t)B * 4}};
    for (auto& o : outs)
      if (o.dst && hipMemcpy(o.dst, dev + o.off, o.sz, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(ctx, "copy back");
  }
  (void)hipFree(dev);
  return rc;
}

int htp_obca_points_sizes(int32_t N, int32_t M, int32_t n_vertices, const int32_t* eo, int64_t* n_var,
                          int64_t* n_eq, int64_t* n_ineq, int64_t* ws_doubles) {
  if (N < 2 || M < 1 || M > MAXM || n_vertices < 3 || n_vertices > MAXKV || !eo) return -1;
  Dims D;
  make_dims_points(D, N, M, n_vertices, eo);
  Layout L = make_layout(D);
  if (n_var) *n_var = D.n;
  if (n_eq) *n_eq = D.mc;
  if (n_ineq) *n_ineq = D.md;
  if (ws_doubles) *ws_doubles = L.total;
  return 0;
}

int htp_obca_points_solve_batch_device(htp_ctx* ctx, const htp_obca_points_batch* in, htp_obca_result* out,
                                       void* stream) {
  if (!ctx || !in || !out) return -1;
  const char* e = nullptr;
  if (check_shape_points(in, &e)) return fail(ctx, e);
  if (in->batch == 0) return 0;
  if (!out->x) return fail(ctx, "[OBCA] out->x is required");
  HIPCHK(hipSetDevice(ctx->device));
#if HTP_ONLY44
  return fail(ctx, "[OBCA] experiment build (HTP_ONLY44): no point formulation");
#else
  if (check_idle(ctx, (hipStream_t)stream)) return -1;
  Dims D;
  make_dims_points(D, in->N, in->M, in->n_vertices, in->obs_edges);
  Layout L = make_layout(D);
  bool u4 = true;
  for (int m = 0; m < D.M; ++m) u4 = u4 && D.eo[m] == 4;
  // persistent launch: as many wavefronts as are resident, each claiming problems from the
  // static ticket range (as obca_solve_kernel for optimizer.py), workspace per wavefront
  int cap = u4 ? resident_waves_t<1, 4, 1>(ctx, 0) : resident_waves_t<1, MAXE, 1>(ctx, 0);
  if (cap < 0) return -1;
  const int64_t waves = cap < in->batch ? cap : in->batch;
  if (ensure(ctx, &ctx->ws, &ctx->ws_bytes, (size_t)L.total * sizeof(double) * (size_t)waves)) return -1;
  if (ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, sizeof(Result) * (size_t)in->batch)) return -1;
  if (!ctx->shape) HIPCHK(hipMalloc((void**)&ctx->shape, sizeof(Shape)));
  if (!ctx->next) HIPCHK(hipMalloc((void**)&ctx->next, 256));
  Shape hs{D, L, ctx->opt};
  hs.o.wall_rate = ctx->wall_rate;
  const BatchView b = points_view(in);
  hipStream_t s = (hipStream_t)stream;
  WorkSrc src{(unsigned long long*)ctx->next, nullptr, (long long)in->batch, 0};
  OutView ov{out->objective, out->status, out->iterations, out->n_factor, out->nlp_error, out->n_resto};
  HIPCHK(hipMemcpyAsync(ctx->shape, &hs, sizeof(Shape), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(src.next, 0, sizeof(unsigned long long), s));
  HIPCHK(hipEventRecord(ctx->ev0, s));
  if (u4)
    hipLaunchKernelGGL((obca_solve_kernel<1, 4, 1>), dim3((unsigned)waves), dim3(64), 0, s, (const Shape*)ctx->shape, b,
                       (double*)ctx->ws, (int64_t)L.total, (Result*)ctx->scratch, out->x, src, ov);
  else
    hipLaunchKernelGGL((obca_solve_kernel<1, MAXE, 1>), dim3((unsigned)waves), dim3(64), 0, s,
                       (const Shape*)ctx->shape, b, (double*)ctx->ws, (int64_t)L.total, (Result*)ctx->scratch, out->x,
                       src, ov);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev1, s));
  ctx->last_queue = nullptr;
  return 0;
#endif
}

int htp_obca_points_solve_batch(htp_ctx* ctx, const htp_obca_points_batch* in, htp_obca_result* out) {
  if (!ctx || !in || !out) return -1;
  const char* e = nullptr;
  if (check_shape_points(in, &e)) return fail(ctx, e);
  if (in->batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  Dims D;
  make_dims_points(D, in->N, in->M, in->n_vertices, in->obs_edges);
  const int64_t B = in->batch;
  auto bytes = [&](int64_t n) { return (size_t)(n * (int64_t)sizeof(double)); };
  const size_t sz_in[6] = {bytes(B * D.N * NS), bytes(B * D.TEo * 2), bytes(B * D.TEo), bytes(B * D.KV * 2),
                           bytes(B * NPARAM), in->init_control ? bytes(B * (D.N - 1) * NC) : 0};
  const void* srcs[6] = {in->traj, in->obs_A, in->obs_b, in->vertices, in->params, in->init_control};
  const size_t sz_x = bytes(B * D.n);
  std::vector<size_t> sizes(sz_in, sz_in + 6);
  for (size_t v : {sz_x, bytes(B), (size_t)B * 4, (size_t)B * 4, (size_t)B * 4, bytes(B), (size_t)B * 4}) sizes.push_back(v);
  size_t total = 0;
  std::vector<size_t> off;
  for (size_t v : sizes) { off.push_back(total); total += (v + 255) & ~size_t(255); }
  char* dev = nullptr;
  HIPCHK(hipMalloc((void**)&dev, total));
  for (int k = 0; k < 6; ++k)
    if (sizes[k]) {
      hipError_t er = hipMemcpy(dev + off[k], srcs[k], sizes[k], hipMemcpyHostToDevice);
      if (er != hipSuccess) { (void)hipFree(dev); return fail(ctx, hipGetErrorString(er)); }
    }
  htp_obca_points_batch din = *in;
  din.traj = (const double*)(dev + off[0]);
  din.obs_A = (const double*)(dev + off[1]);
  din.obs_b = (const double*)(dev + off[2]);
  din.vertices = (const double*)(dev + off[3]);
  din.params = (const double*)(dev + off[4]);
  din.init_control = sizes[5] ? (const double*)(dev + off[5]) : nullptr;
  htp_obca_result dout;
  dout.x = (double*)(dev + off[6]);
  dout.objective = (double*)(dev + off[7]);
  dout.status = (int32_t*)(dev + off[8]);
  dout.iterations = (int32_t*)(dev + off[9]);
  dout.n_factor = (int32_t*)(dev + off[10]);
  dout.nlp_error = (double*)(dev + off[11]);
  dout.n_resto = (int32_t*)(dev + off[12]);
  int rc = htp_obca_points_solve_batch_device(ctx, &din, &dout, nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("points solve kernel: ") + hipGetErrorString(er));
  }
  if (rc == 0) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) ctx->last_ms = ms;
    struct { void* dst; size_t off, sz; } outs[7] = {{out->x, off[6], sz_x}, {out->objective, off[7], bytes(B)},
                                                     {out->status, off[8], (size_t)B * 4}, {out->iterations, off[9], (size_t)B * 4},
                                                     {out->n_factor, off[10], (size_t)B * 4}, {out->nlp_error, off[11], bytes(B)},
                                                     {out->n_resto, off[12], (size_t)B * 4}};
    for (auto& o : outs)
      if (o.dst && hipMemcpy(o.dst, dev + o.off, o.sz, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(ctx, "copy back");
  }
  (void)hipFree(dev);
  return rc;
}

}  // extern "C"
