// One evaluation of the correctly rounded libm (htp_libm.h) by function id, shared by the device batch
// (htp_libm.hip: htp_libm_batch_device) and the host batch (htp_cpu.cpp: htp_cpu_libm_batch), so the parity
// tests compare the two builds of the same source argument by argument.
#pragma once
#include "htp_fastm.h"
#include "htp_libm.h"

namespace htp {
namespace hm {

enum { F_SIN = 0, F_COS, F_TAN, F_ATAN, F_ATAN2, F_ASIN, F_ACOS, F_HYPOT, F_POW, F_LOG, F_FLOG, F_FSIN, F_FCOS, F_FTAN, F_COUNT };

HTP_HD inline double eval(int fn, double x, double y) {
  switch (fn) {
    case F_SIN: return sin(x);
    case F_COS: return cos(x);
    case F_TAN: return tan(x);
    case F_ATAN: return atan(x);
    case F_ATAN2: return atan2(x, y);   // atan2(y = x[i], x = y[i]): first argument first
    case F_ASIN: return asin(x);
    case F_ACOS: return acos(x);
    case F_HYPOT: return hypot(x, y);
    case F_POW: return pow(x, y);
    case F_LOG: return log(x);
    case F_FLOG: return fm::log(x);   // the solver's fast deterministic functions (htp_fastm.h)
    case F_FSIN: return fm::sin(x);
    case F_FCOS: return fm::cos(x);
    case F_FTAN: return fm::tan(x);
    default: return __builtin_nan("");
  }
}

}  // namespace hm
}  // namespace htp
