"""Device-code properties of the built library (CPU only: the gfx950 code object is disassembled, not run).

The Makefile compiles the device code without packed fp32 VALU (`NOPK`): beside MFMAs a
`v_pk_*_f32` costs more issue cycles than the two scalar instructions it replaces.  hipcc forms them from
float4 arithmetic by itself, so a build that lost the flag would still pass every numerics test (the
results are bit-identical) and only run slower.  This guards the flag."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "trpo-robot-control_amd", "lib", "libtrpo_mi355x.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TOOLS = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]


def _disassemble(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    if not all(os.access(t, os.X_OK) for t in TOOLS):
        pytest.skip("ROCm LLVM tools not available")
    objcopy, bundler, objdump = TOOLS
    fb, co = tmp_path / "fatbin.bin", tmp_path / "gfx950.co"
    # objcopy writes a stripped copy as its output file; only the dumped section is used
    subprocess.run([objcopy, "--dump-section=.hip_fatbin=%s" % fb, LIB, str(tmp_path / "copy.so")], check=True)
    subprocess.run([bundler, "--unbundle", "--type=o", "--input=%s" % fb,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=%s" % co], check=True)
    return subprocess.run([objdump, "-d", str(co)], check=True, capture_output=True, text=True).stdout


def _functions(dis):
    """{symbol: [mnemonic, ...]} of an llvm-objdump -d listing."""
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None:
            t = line.strip().split()
            if t and re.match(r"^[sv]_|^ds_|^buffer_|^global_", t[0]):
                cur.append(t[0])
    return funcs


def test_cg_iteration_kernels_have_no_packed_fp32(tmp_path):
    funcs = _functions(_disassemble(tmp_path))
    # _Z15fvp_mlp3_kernel...: the small-net FVP / CG-iteration kernels (every MODE, QB and twin)
    mlp3 = {k: v for k, v in funcs.items() if k.startswith("_Z15fvp_mlp3_kernel")}
    assert len(mlp3) >= 8, sorted(funcs)[:20]
    packed = re.compile(r"^v_pk_(fma|mul|add)_f32")
    for name, ops in mlp3.items():
        assert any(o.startswith("v_mfma") for o in ops), name
        bad = [o for o in ops if packed.match(o)]
        assert not bad, "%s: %d packed fp32 instructions (%s)" % (name, len(bad), bad[:3])
