#!/usr/bin/env python3
"""Register / scratch / LDS use of the built library's gfx950 kernels (from the code object's metadata
notes; CPU only).  Usage: tools/kernel_resources.py [LIB] [SUBSTRING ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def resources(lib):
    with tempfile.TemporaryDirectory() as tmp:
        fb, co = os.path.join(tmp, "fb"), os.path.join(tmp, "co")
        subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, lib, os.path.join(tmp, "c")],
                       check=True)
        subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        t = line.strip()
        m = re.match(r"^(?:- )?\.name:\s+(\S+)", t)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.match(r"^\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"private_segment_fixed_size|group_segment_fixed_size|max_flat_workgroup_size):\s+(\d+)", t)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else \
        os.path.join(ROOT, "trpo-robot-control_amd", "lib", "libtrpo_mi355x.so")
    pats = [a for a in sys.argv[1:] if not a.endswith(".so")] or [""]
    res = resources(lib)
    names = list(res)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    demangle = dict(zip(names, dem)).get
    for name, r in sorted(res.items(), key=lambda kv: demangle(kv[0])):
        d = demangle(name)
        if any(p in d for p in pats):
            print("%-4d vgpr %-3d agpr %-3d sgpr %-3d spill v%d s%d scratch %-5d lds %-6d %s" % (
                r.get("max_flat_workgroup_size", 0), r.get("vgpr_count", 0), r.get("agpr_count", 0),
                r.get("sgpr_count", 0), r.get("vgpr_spill_count", 0), r.get("sgpr_spill_count", 0),
                r.get("private_segment_fixed_size", 0), r.get("group_segment_fixed_size", 0), d[:150]))
