// Library context shared by the translation units of libhtp.so (host side).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "htp_common.h"

struct htp_ctx {
  using Options = htp::Options;
  using Shape = htp::Shape;
  int device = 0;
  std::string err;
  Options opt = htp::default_options();
  double wall_rate = 1e8;   // device wall-clock ticks/s (hipDeviceAttributeWallClockRate)
  void* ws = nullptr;
  void* next = nullptr;     // device ticket counter of the solve launch
  size_t ws_bytes = 0;
  void* scratch = nullptr;  // Result array
  size_t scratch_bytes = 0;
  Shape* shape = nullptr;   // device copy of the launch-uniform shape
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_ms = 0.0;
  const void* last_queue = nullptr;   // host queue of the last solve launch (queue mode), else nullptr
  // Reeds-Shepp batch (htp_rs.hip)
  void* rs_scratch = nullptr;
  size_t rs_scratch_bytes = 0;
  hipEvent_t rs_ev0 = nullptr, rs_ev1 = nullptr;
  // Hybrid A* batch (htp_hastar.hip)
  void* ha_ws = nullptr;
  size_t ha_ws_bytes = 0;
  hipEvent_t ha_ev0 = nullptr, ha_ev1 = nullptr;
  // Y-park batch (htp_ypark.hip)
  void* yp_ws = nullptr;
  size_t yp_ws_bytes = 0;
  hipEvent_t yp_ev0 = nullptr, yp_ev1 = nullptr;
  // warm start -> initial guess batch (htp_refpath.hip)
  void* rp_ws = nullptr;
  size_t rp_ws_bytes = 0;
  hipEvent_t rp_ev0 = nullptr, rp_ev1 = nullptr;
  // orchard scene -> OBCA obstacles (htp_oge.hip)
  hipEvent_t oge_ev0 = nullptr, oge_ev1 = nullptr;
  // classic turns (htp_classic.hip)
  void* ct_ws = nullptr;
  size_t ct_ws_bytes = 0;
  hipEvent_t ct_ev0 = nullptr, ct_ev1 = nullptr;
  // orchard workload chain (htp_chain.hip)
  void* ch_ws = nullptr;
  size_t ch_ws_bytes = 0;
  hipEvent_t ch_ev0 = nullptr, ch_ev1 = nullptr;
  // notebook planner chain (htp_ychain.hip): stage boundaries Y-park | lowering | hybrid A* | init guess
  void* yc_ws = nullptr;
  size_t yc_ws_bytes = 0;
  hipEvent_t yc_ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};

static inline int fail(htp_ctx* c, const std::string& m) {
  if (c) c->err = m;
  return -1;
}

#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) return fail(ctx, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// A launch that reuses one of the context's workspaces is ordered after the previous launch that used it
// (`done` = that launch's end event): stream order when both are on one stream, an event wait otherwise.
static inline int order_after(htp_ctx* ctx, hipEvent_t done, hipStream_t s) {
  if (done && hipEventQuery(done) == hipErrorNotReady) HIPCHK(hipStreamWaitEvent(s, done, 0));
  return 0;
}

static inline int ensure(htp_ctx* ctx, void** p, size_t* have, size_t need) {
  if (*have >= need) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  HIPCHK(hipMalloc(p, need));
  *have = need;
  return 0;
}

