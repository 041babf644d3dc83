"""Static code size of the config-D solver kernel (ObcaSolver<DevWave, 4, 4, 0>): instruction mix, registers,
scratch, and the inclusive instruction count of every obca_core.h function over its inlined copies (from the
inline chains of -gline-tables-only).  Used to find phases whose inlined copies dominate the kernel's
instruction footprint (outlined: barrier).

    python tools/code_size.py [csrc_dir] [-- extra hipcc flags]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = r'''
#include <hip/hip_runtime.h>
#define HTP_HD __host__ __device__
#include "wave_ctx.h"
#include "obca_batch.h"
using namespace htp;
__global__ __launch_bounds__(64, 1) void k44(const Shape* shp, BatchView b, double* ws, int64_t stride, Result* res) {
  __shared__ double lds_[LDS_WAVE_DOUBLES];
  __shared__ int ilds_[2 * NBMAX];
  DevWave c{(int)threadIdx.x, (DevWave::ld*)lds_, (DevWave::li*)ilds_};
  using CS = DevWave::cst<Shape>;
  CS* sh = (CS*)shp;
  ProblemIn in = problem_view(b, sh->D, blockIdx.x);
  ObcaSolver<DevWave, 4, 4, 0> S(c, sh->D, sh->L, sh->o, in, ws + blockIdx.x * stride);
  Result r{};
  S.run(r);
  if (threadIdx.x == 0) res[blockIdx.x] = r;
}
'''


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        extra = args[args.index("--") + 1:]
        args = args[:args.index("--")]
    csrc = args[0] if args else os.path.join(ROOT, "headland_trajectory_planning_amd", "csrc")
    d = tempfile.mkdtemp()
    k, s = os.path.join(d, "k44.hip"), os.path.join(d, "k44.s")
    open(k, "w").write(KERNEL)
    p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{csrc}",
                        "-gline-tables-only", "--offload-device-only", "-S", "-o", s, k,
                        "-Rpass-analysis=kernel-resource-usage"] + extra, capture_output=True, text=True)
    if p.returncode:
        sys.exit(p.stderr[-3000:])
    res = {m.group(1).strip(): m.group(2) for m in re.finditer(r"remark:\s+([\w \[\]/]+): (\d+)", p.stderr)}
    src = open(os.path.join(csrc, "obca_core.h")).read().split("\n")
    fn_at, cur = {}, "?"
    for i, line in enumerate(src, 1):
        m = re.match(r"\s+(?:template <[^>]*>\s*)?(?:__attribute__\(\(noinline\)\)\s+|HTP_BARRIER_ATTR\s+)?HTP_HD\s+"
                     r"(?:HTP_FI\s+|HTP_PHASE\s+|static\s+|inline\s+)*(?:[\w:<>*&,\s]+?)\s+\**(\w+)\(", line)
        if m:
            cur = m.group(1)
        fn_at[i] = cur
    mix, incl, loc = collections.Counter(), collections.Counter(), None
    scr_fn, scr_line = collections.Counter(), collections.Counter()   # scratch instructions by function / line
    for line in open(s):
        if line.startswith("\t.loc"):
            loc = line
            continue
        t = line.strip()
        if not t or t[0] in ".;" or t.endswith(":"):
            continue
        op = t.split()[0]
        kind = ("scratch" if op.startswith("scratch_") else "accvgpr" if op.startswith("v_accvgpr") else
                "lane" if op.startswith(("v_readlane", "v_writelane")) else "valu" if op.startswith("v_") else
                "salu" if op.startswith("s_") else "vmem" if op.startswith(("global_", "buffer_")) else
                "lds" if op.startswith("ds_") else "other")
        mix[kind] += 1
        if loc and ";" in loc:
            seen = set()
            chain = re.findall(r"([\w./-]+\.(?:h|hip)):(\d+):\d+", loc.split(";", 1)[1])
            if kind == "scratch" and chain:
                scr_line[f"{os.path.basename(chain[0][0])}:{chain[0][1]}"] += 1
            for f, ln in chain:
                if f.endswith("obca_core.h"):
                    fn = fn_at.get(int(ln), "?")
                    if fn not in seen:
                        seen.add(fn)
                        incl[fn] += 1
                        if kind == "scratch":
                            scr_fn[fn] += 1
    print(f"instructions {sum(mix.values())} {dict(mix)}")
    print("resources", {k: res[k] for k in res if k in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]",
                                                         "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]")})
    print("inclusive instructions per obca_core.h function (all inlined copies):")
    for fn, v in incl.most_common(30):
        print(f"  {fn:28s} {v}")
    print("scratch instructions per obca_core.h function (inclusive):")
    for fn, v in scr_fn.most_common(25):
        print(f"  {fn:28s} {v}")
    print("scratch instructions per source line (innermost):")
    for ln, v in scr_line.most_common(40):
        print(f"  {ln:28s} {v}")


if __name__ == "__main__":
    main()
