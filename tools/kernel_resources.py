"""Register, spill, scratch and LDS figures of every kernel in a built library, read from the gfx950 code object's
own metadata (the AMDGPU note: .vgpr_count, .agpr_count, .sgpr_count, .vgpr_spill_count, .sgpr_spill_count,
.private_segment_fixed_size, .group_segment_fixed_size) -- the numbers the hardware launches with, not a profiler's
per-dispatch summary (rocprofv3's counter CSV reports the architectural VGPRs only).

    python tools/kernel_resources.py [headland_trajectory_planning_amd/libhtp.so] [name-filter]

The library's .hip_fatbin section is a clang offload bundle: "__CLANG_OFFLOAD_BUNDLE__", an entry count, then per
entry (offset, size, triple length, triple); the hipv4-amdgcn-amd-amdhsa--gfx950 entry is an ELF code object whose
notes llvm-readobj prints as YAML."""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size")


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(d, "x")])
        data = open(fb, "rb").read()
    out = []
    pos = 0
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    while True:
        pos = data.find(magic, pos)
        if pos < 0:
            break
        p = pos + len(magic)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple:
                out.append(data[pos + off:pos + off + size])
        pos = p
    return out


def kernels(lib):
    res = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", f.name], capture_output=True, text=True).stdout
        for block in re.split(r"\n\s+- \.agpr_count", txt)[1:]:
            block = ".agpr_count" + block
            name = re.search(r"\.name:\s+(\S+)", block)
            if not name:
                continue
            vals = {}
            for fld in FIELDS:
                m = re.search(re.escape(fld) + r":\s+(\d+)", block)
                if m:
                    vals[fld.lstrip(".")] = int(m.group(1))
            res[name.group(1)] = vals
    return res


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp.so")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    ks = {k: v for k, v in kernels(lib).items() if filt in k}
    print(json.dumps(ks, indent=1))


if __name__ == "__main__":
    main()
