"""Build A/B variants of libhtp.so with different compile flags for the OBCA
TU (experiments only; the product library is built by __graft_entry__.build()).

    python tools/build_variants.py name1="-DFOO" name2="-DBAR=2" ...
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "headland_trajectory_planning_amd", "csrc")
PKG = os.path.join(ROOT, "headland_trajectory_planning_amd")
OBJ = os.path.join(ROOT, "build", "obj")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC"]

procs = []
names = []
for arg in sys.argv[1:]:
    name, _, extra = arg.partition("=")
    obj = os.path.join(OBJ, f"htp_obca_{name}.o")
    cmd = [HIPCC] + FLAGS + extra.split() + ["-c", os.path.join(CSRC, "htp_obca.hip"), "-o", obj]
    print(" ".join(cmd), flush=True)
    procs.append(subprocess.Popen(cmd, cwd=CSRC))
    names.append(name)
for p in procs:
    if p.wait() != 0:
        sys.exit("build failed")
for name in names:
    out = os.path.join(PKG, f"libhtp_{name}.so")
    others = [os.path.join(OBJ, f) for f in sorted(os.listdir(OBJ))
              if f.endswith(".hip.o") and f != "htp_obca.hip.o"]
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out,
                           os.path.join(OBJ, f"htp_obca_{name}.o")] + others)
    print("built", out)
