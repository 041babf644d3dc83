// libhtp.so, Reeds-Shepp batch: all admissible paths for a batch of pose pairs
// (R/path_planner/utils/reeds_shepp.py calc_all_paths), CSR output in HBM.
//
// Four launches, no host round trip:
//   rs_generate  one thread per query: the 46 candidate words, de-duplicated,
//                into fixed slots [query][MAXP] (path records, 64 B each)
//   rs_scan      paths per query -> path offsets (single workgroup)
//   rs_count     one thread per path: sample count of generate_local_course
//   rs_scan      samples per path -> point offsets
//   rs_fill      one thread per path: lengths/ctypes/L + the global-frame samples
// Per-path work is sequential in the reference (each sample's origin is the
// previous segment's end), so paths, not samples, are the parallel unit.
#include <hip/hip_runtime.h>

#include <string>

#define HTP_HD __host__ __device__
#include "../../include/htp.h"
#include "htp_ctx.h"
#include "rs_core.h"

using namespace htp::rs;

namespace {

constexpr int SCAN_T = 1024;

struct RsScratch {
  Path* rec;         // [batch][MAXP]
  int32_t* npaths;   // [batch]
  int64_t* path_off; // [batch+1]
  int32_t* cnt;      // [batch*MAXP]
  int64_t* pt_off;   // [batch*MAXP+1]
  int64_t* totals;   // [2]
};

__global__ __launch_bounds__(256) void rs_generate(const double* __restrict__ q, int batch, Path* __restrict__ rec,
                                                   int32_t* __restrict__ npaths, int32_t* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  const double* a = q + (int64_t)i * 8;
  PathSet S{rec + (int64_t)i * MAXP, 0, 0};
  generate_paths(a[0], a[1], a[2], a[3], a[4], a[5], a[6], S);
  npaths[i] = S.err ? 0 : S.n;
  status[i] = S.err ? HTP_RS_ASSERT : HTP_RS_OK;
}

// Exclusive scan of n int32 counts (n from n_dev when given) into out[0..n].
__global__ __launch_bounds__(SCAN_T) void rs_scan(const int32_t* __restrict__ in, const int64_t* n_dev, int64_t n_host,
                                                  int64_t* __restrict__ out, int64_t* total) {
  __shared__ int64_t part[SCAN_T];
  const int64_t n = n_dev ? *n_dev : n_host;
  const int t = threadIdx.x;
  const int64_t chunk = (n + SCAN_T - 1) / SCAN_T;
  const int64_t b = min(n, (int64_t)t * chunk), e = min(n, b + chunk);
  int64_t s = 0;
  for (int64_t k = b; k < e; ++k) s += in[k];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t k = b; k < e; ++k) {
    out[k] = run;
    run += in[k];
  }
  if (t == SCAN_T - 1) {
    out[n] = part[t];
    if (total) *total = part[t];
  }
}

__device__ inline int query_of(const int64_t* __restrict__ path_off, int batch, int64_t g) {
  int lo = 0, hi = batch;  // path_off[lo] <= g < path_off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (path_off[mid] <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void rs_count(const double* __restrict__ q, int batch, const Path* __restrict__ rec,
                                                const int64_t* __restrict__ path_off, int32_t* __restrict__ cnt,
                                                int32_t* __restrict__ status) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= path_off[batch]) return;
  const int i = query_of(path_off, batch, g);
  const Path p = rec[(int64_t)i * MAXP + (g - path_off[i])];
  const double maxc = q[(int64_t)i * 8 + 6], step = q[(int64_t)i * 8 + 7];
  NullSink ns;
  int n = local_course(p, maxc, step * maxc, ns);
  if (n < 0) {
    status[i] = HTP_RS_OVERFLOW;
    n = 0;
  }
  cnt[g] = n;
}

__global__ __launch_bounds__(256) void rs_fill(const double* __restrict__ q, int batch, const Path* __restrict__ rec,
                                               const int64_t* __restrict__ path_off, const int32_t* __restrict__ cnt,
                                               const int64_t* __restrict__ pt_off, htp_rs_paths out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t P = path_off[batch];
  if (g == 0 && out.point_offsets && out.cap_paths >= 0) out.point_offsets[0] = 0;
  if (g >= P) return;
  const int i = query_of(path_off, batch, g);
  const Path p = rec[(int64_t)i * MAXP + (g - path_off[i])];
  const double* a = q + (int64_t)i * 8;
  const double maxc = a[6], step = a[7];
  if (g < out.cap_paths) {
    for (int j = 0; j < 5; ++j) {
      out.lengths[g * 5 + j] = j < p.nseg ? p.len[j] / maxc : 0.0;
      out.ctypes[g * 5 + j] = p.typ[j];
    }
    out.L[g] = p.L / maxc;
    out.point_offsets[g + 1] = pt_off[g + 1];
  }
  const int64_t base = pt_off[g];
  const int n = cnt[g];
  if (n == 0 || base + n > out.cap_points) return;
  GlobalSink gs{out.x + base, out.y + base, out.yaw + base, out.cs + base, out.directions + base, n,
                a[0], a[1], a[2], htp::hm::cos(-a[2]), htp::hm::sin(-a[2])};
  local_course(p, maxc, step * maxc, gs);
}

struct ScratchLayout {
  size_t rec, npaths, path_off, cnt, pt_off, totals, total;
};

ScratchLayout scratch_layout(int64_t batch) {
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  ScratchLayout L{};
  size_t o = 0;
  L.rec = o; o += al(sizeof(Path) * (size_t)batch * MAXP);
  L.npaths = o; o += al(4 * (size_t)batch);
  L.path_off = o; o += al(8 * ((size_t)batch + 1));
  L.cnt = o; o += al(4 * (size_t)batch * MAXP);
  L.pt_off = o; o += al(8 * ((size_t)batch * MAXP + 1));
  L.totals = o; o += al(16);
  L.total = o;
  return L;
}

}  // namespace

static int rs_enqueue(htp_ctx* ctx, int32_t batch, const double* q, htp_rs_paths* out, int64_t* totals,
                      hipStream_t s) {
  const ScratchLayout SL = scratch_layout(batch);
  if (ensure(ctx, &ctx->rs_scratch, &ctx->rs_scratch_bytes, SL.total)) return -1;
  char* b = (char*)ctx->rs_scratch;
  RsScratch W{(Path*)(b + SL.rec), (int32_t*)(b + SL.npaths), (int64_t*)(b + SL.path_off), (int32_t*)(b + SL.cnt),
              (int64_t*)(b + SL.pt_off), (int64_t*)(b + SL.totals)};
  int64_t* tot = totals ? totals : W.totals;
  HIPCHK(hipEventRecord(ctx->rs_ev0, s));
  const int64_t maxpaths = (int64_t)batch * MAXP;
  hipLaunchKernelGGL(rs_generate, dim3((batch + 255) / 256), dim3(256), 0, s, q, batch, W.rec, W.npaths, out->status);
  hipLaunchKernelGGL(rs_scan, dim3(1), dim3(SCAN_T), 0, s, (const int32_t*)W.npaths, (const int64_t*)nullptr,
                     (int64_t)batch, W.path_off, tot);
  const dim3 pg((unsigned)((maxpaths + 255) / 256));
  hipLaunchKernelGGL(rs_count, pg, dim3(256), 0, s, q, batch, (const Path*)W.rec, (const int64_t*)W.path_off, W.cnt,
                     out->status);
  hipLaunchKernelGGL(rs_scan, dim3(1), dim3(SCAN_T), 0, s, (const int32_t*)W.cnt, (const int64_t*)(W.path_off + batch),
                     (int64_t)0, W.pt_off, tot + 1);
  hipLaunchKernelGGL(rs_fill, pg, dim3(256), 0, s, q, batch, (const Path*)W.rec, (const int64_t*)W.path_off,
                     (const int32_t*)W.cnt, (const int64_t*)W.pt_off, *out);
  HIPCHK(hipGetLastError());
  if (out->path_offsets)
    HIPCHK(hipMemcpyAsync(out->path_offsets, W.path_off, 8 * ((size_t)batch + 1), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipEventRecord(ctx->rs_ev1, s));
  return 0;
}

extern "C" {

int htp_rs_all_paths_batch_device(htp_ctx* ctx, int32_t batch, const double* queries, htp_rs_paths* out,
                                  int64_t* totals, void* stream) {
  if (!ctx || !out || batch < 0 || (batch > 0 && !queries) || !out->status) return fail(ctx, "rs: bad arguments");
  if (out->cap_paths > 0 && (!out->lengths || !out->ctypes || !out->L || !out->point_offsets))
    return fail(ctx, "rs: path arrays missing");
  if (out->cap_points > 0 && (!out->x || !out->y || !out->yaw || !out->cs || !out->directions))
    return fail(ctx, "rs: point arrays missing");
  if (batch == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  return rs_enqueue(ctx, batch, queries, out, totals, (hipStream_t)stream);
}

int htp_rs_all_paths_batch(htp_ctx* ctx, int32_t batch, const double* queries, htp_rs_paths* out) {
  if (!ctx || !out || batch < 0 || (batch > 0 && !queries) || !out->status || !out->path_offsets)
    return fail(ctx, "rs: bad arguments");
  out->n_paths = out->n_points = 0;
  if (batch == 0) {
    out->path_offsets[0] = 0;
    return 0;
  }
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t B = batch;
  const int64_t cp = out->cap_paths > 0 ? out->cap_paths : 0, cq = out->cap_points > 0 ? out->cap_points : 0;
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  // device staging: queries, status, path_offsets, totals, path arrays, point arrays
  size_t o = 0;
  const size_t o_q = o; o += al(64 * (size_t)B);
  const size_t o_st = o; o += al(4 * (size_t)B);
  const size_t o_po = o; o += al(8 * ((size_t)B + 1));
  const size_t o_tot = o; o += al(16);
  const size_t o_len = o; o += al(40 * (size_t)cp);
  const size_t o_ct = o; o += al(5 * (size_t)cp);
  const size_t o_L = o; o += al(8 * (size_t)cp);
  const size_t o_pto = o; o += al(8 * ((size_t)cp + 1));
  const size_t o_x = o; o += al(8 * (size_t)cq);
  const size_t o_y = o; o += al(8 * (size_t)cq);
  const size_t o_yaw = o; o += al(8 * (size_t)cq);
  const size_t o_cs = o; o += al(8 * (size_t)cq);
  const size_t o_dir = o; o += al((size_t)cq);
  char* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, o));
  int rc = 0;
  auto H2D = [&](size_t off, const void* src, size_t n) {
    if (rc == 0 && hipMemcpy(d + off, src, n, hipMemcpyHostToDevice) != hipSuccess) rc = fail(ctx, "rs: upload");
  };
  auto D2H = [&](void* dst, size_t off, size_t n) {
    if (rc == 0 && n && hipMemcpy(dst, d + off, n, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(ctx, "rs: download");
  };
  H2D(o_q, queries, 64 * (size_t)B);
  htp_rs_paths dv{};
  dv.cap_paths = cp;
  dv.cap_points = cq;
  dv.path_offsets = (int64_t*)(d + o_po);
  dv.status = (int32_t*)(d + o_st);
  dv.lengths = (double*)(d + o_len);
  dv.ctypes = (int8_t*)(d + o_ct);
  dv.L = (double*)(d + o_L);
  dv.point_offsets = (int64_t*)(d + o_pto);
  dv.x = (double*)(d + o_x);
  dv.y = (double*)(d + o_y);
  dv.yaw = (double*)(d + o_yaw);
  dv.cs = (double*)(d + o_cs);
  dv.directions = (int8_t*)(d + o_dir);
  if (rc == 0) rc = rs_enqueue(ctx, batch, (const double*)(d + o_q), &dv, (int64_t*)(d + o_tot), nullptr);
  if (rc == 0) {
    hipError_t er = hipDeviceSynchronize();
    if (er != hipSuccess) rc = fail(ctx, std::string("rs kernels: ") + hipGetErrorString(er));
  }
  int64_t tot[2] = {0, 0};
  D2H(tot, o_tot, 16);
  D2H(out->status, o_st, 4 * (size_t)B);
  D2H(out->path_offsets, o_po, 8 * ((size_t)B + 1));
  if (rc == 0) {
    out->n_paths = tot[0];
    out->n_points = tot[1];
    if (tot[0] > out->cap_paths || tot[1] > out->cap_points) {
      (void)hipFree(d);
      return HTP_RS_CAPACITY;
    }
    D2H(out->lengths, o_len, 40 * (size_t)tot[0]);
    D2H(out->ctypes, o_ct, 5 * (size_t)tot[0]);
    D2H(out->L, o_L, 8 * (size_t)tot[0]);
    D2H(out->point_offsets, o_pto, 8 * ((size_t)tot[0] + 1));
    D2H(out->x, o_x, 8 * (size_t)tot[1]);
    D2H(out->y, o_y, 8 * (size_t)tot[1]);
    D2H(out->yaw, o_yaw, 8 * (size_t)tot[1]);
    D2H(out->cs, o_cs, 8 * (size_t)tot[1]);
    D2H(out->directions, o_dir, (size_t)tot[1]);
  }
  (void)hipFree(d);
  return rc;
}

double htp_rs_last_ms(htp_ctx* ctx) {
  if (!ctx || !ctx->rs_ev1) return 0.0;
  if (hipEventSynchronize(ctx->rs_ev1) != hipSuccess) return 0.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ctx->rs_ev0, ctx->rs_ev1) != hipSuccess) return 0.0;
  return ms;
}

}  // extern "C"
