"""C-ABI checks that need no GPU: the library loads, exports every symbol the
public header declares, TRPOparam has the reference layout, host-side error
paths follow the reference (src/TRPO_FVP.c:671-674,732-735)."""
import ctypes as C
import os
import re
import subprocess
import textwrap

import numpy as np
import pytest

import trpo_amd
from trpo_amd import synth


def test_library_exports_every_header_symbol():
    L = trpo_amd.lib()
    syms = trpo_amd.header_symbols()
    for must in ("NumParamsCalc", "FVP", "FVPFast", "CG", "FVP_FPGA", "CG_FPGA", "trpo_ctx_create",
                 "trpo_ctx_cg", "trpo_ctx_fvp", "trpo_ctx_attach_comm"):
        assert must in syms
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_numparams_matches_reference_formula():
    assert trpo_amd.NumParamsCalc([15, 16, 16, 3]) == 582
    assert trpo_amd.NumParamsCalc([15, 64, 64, 3]) == 5382
    assert trpo_amd.NumParamsCalc([376, 64, 64, 17]) == synth.num_params([376, 64, 64, 17])


def test_trpoparam_layout_matches_c(tmp_path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "off.c"
    src.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <stddef.h>
        #include "trpo_mi355x.h"
        int main(void) {
          printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(TRPOparam), offsetof(TRPOparam, NumLayers),
                 offsetof(TRPOparam, LayerSize), offsetof(TRPOparam, NumSamples),
                 offsetof(TRPOparam, CG_Damping), offsetof(TRPOparam, NumBlocks));
          return 0; }
    """))
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    P = trpo_amd.TRPOparam
    assert got == [C.sizeof(P), P.NumLayers.offset, P.LayerSize.offset, P.NumSamples.offset,
                   P.CG_Damping.offset, P.NumBlocks.offset]


def test_missing_files_return_minus_one(capfd):
    prm = trpo_amd.make_param("/nonexistent/model.txt", "/nonexistent/data.txt", [15, 16, 16, 3], "lttl", 10)
    P = 582
    out = np.zeros(P)
    assert trpo_amd.FVPFast(prm, out, np.ones(P), 1) == -1
    assert trpo_amd.CG(prm, out, np.ones(P), 10, 1e-10, 1) == -1
    err = capfd.readouterr().err
    assert "[ERROR] Cannot open Model File [/nonexistent/model.txt]" in err


def test_bad_activation_rejected(tmp_path, capfd):
    th = synth.make_theta([15, 16, 16, 3])
    m, d = tmp_path / "m.txt", tmp_path / "d.txt"
    synth.write_model_file(str(m), th)
    synth.write_data_file(str(d), synth.make_obs(4, 15), np.ones(3))
    prm = trpo_amd.make_param(str(m), str(d), [15, 16, 16, 3], "ltxl", 4)
    assert trpo_amd.FVPFast(prm, np.zeros(582), np.ones(582), 1) == -1
    assert "Unsupported" in capfd.readouterr().err


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    with pytest.raises(trpo_amd.TRPOError):
        trpo_amd.Context([15, 16, 16, 3], "lttl", synth.make_theta([15, 16, 16, 3]), synth.make_obs(8, 15),
                         np.ones(3))


@pytest.mark.parametrize("compiler", [["gcc", "-std=gnu99"], ["g++", "-x", "c++", "-std=c++11"]])
def test_compiled_caller_builds_and_links(compiler, tmp_path):
    """The drop-in caller (tests/c_caller/drop_in_caller.c, the TRPOCpuCode.c pattern) compiles as C and
    as C++ against include/trpo_mi355x.h alone and links with -ltrpo_mi355x; the reference's entry
    points are imported UNMANGLED in the C++ build (extern "C" linkage, build/Makefile.cpuonly:5)."""
    import subprocess
    libdir = os.path.dirname(trpo_amd.LIB_PATH)
    exe = str(tmp_path / "caller")
    src = os.path.join(os.path.dirname(__file__), "c_caller", "drop_in_caller.c")
    subprocess.run(compiler + ["-O1", "-Wall", "-Werror", "-I", os.path.dirname(trpo_amd.HEADER), "-o", exe, src,
                               "-L", libdir, "-ltrpo_mi355x"], check=True)
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for name in ("NumParamsCalc", "FVPFast", "CG", "TRPO_Update"):
        assert re.search(r"\bU %s$" % name, syms, re.M), name


# the seven TRPO.h:81-104 entry points and the Itanium names g++ gives them when TRPO.h is included
# without extern "C" (build/Makefile.cpuonly:5,11 compiles every caller with g++ -std=c++11)
MANGLED = {
    "NumParamsCalc": "_Z13NumParamsCalcPmm",
    "FVP": "_Z3FVP9TRPOparamPdS0_",
    "FVPFast": "_Z7FVPFast9TRPOparamPdS0_m",
    "CG": "_Z2CG9TRPOparamPdS0_mdm",
    "FVP_FPGA": "_Z8FVP_FPGA9TRPOparamPdS0_",
    "CG_FPGA": "_Z7CG_FPGA9TRPOparamPdS0_mdm",
    "TRPO_Update": "_Z11TRPO_Update9TRPOparamPdm",
}

# a caller taking the address of every Part-1 entry point (so each is imported), header chosen by -D
ALL_ENTRY_CALLER = textwrap.dedent("""
    #include <stdio.h>
    #ifdef USE_REFERENCE_HEADER
    #include "TRPO.h"
    #else
    #include "trpo_mi355x.h"
    #endif
    int main(void) {
        void *volatile f[] = {(void *)&NumParamsCalc, (void *)&FVP, (void *)&FVPFast, (void *)&CG,
                     (void *)&FVP_FPGA, (void *)&CG_FPGA, (void *)&TRPO_Update};
        size_t ls[] = {15, 16, 16, 3};
        int all = 1;
        for (int i = 0; i < 7; ++i) all &= f[i] != 0;
        printf("%zu %d\\n", NumParamsCalc(ls, 4), all);
        return NumParamsCalc(ls, 4) == 582 ? 0 : 1;
    }
""")


def test_library_exports_cxx_linkage_twins():
    """Every TRPO.h entry point is exported with C linkage AND with the C++ linkage an unchanged g++-built
    caller of the reference's header imports (csrc/trpo_cxx_abi.cpp)."""
    out = subprocess.run(["nm", "-D", "--defined-only", trpo_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    for c_name, cxx_name in MANGLED.items():
        assert re.search(r" T %s$" % c_name, out, re.M), c_name
        assert re.search(r" T %s$" % cxx_name, out, re.M), cxx_name


def _link_caller(tmp_path, defs, incdir):
    src = tmp_path / "caller.cpp"
    src.write_text(ALL_ENTRY_CALLER)
    exe = str(tmp_path / "caller")
    libdir = os.path.dirname(trpo_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O1", *defs, "-I", incdir, "-o", exe, str(src), "-L", libdir,
                    "-ltrpo_mi355x", "-Wl,-rpath," + libdir], check=True)
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    return exe, und


def test_cxx_linkage_header_switch_links(tmp_path):
    """include/trpo_mi355x.h with TRPO_MI355X_CXX_LINKAGE declares Part 1 as the reference's TRPO.h does;
    the caller imports the mangled names and links against the library with nothing undefined."""
    exe, und = _link_caller(tmp_path, ["-DTRPO_MI355X_CXX_LINKAGE"], os.path.dirname(trpo_amd.HEADER))
    for cxx_name in MANGLED.values():
        assert re.search(r"\bU %s$" % cxx_name, und, re.M), cxx_name
    # NumParamsCalc is pure host code: the mangled twin runs without a GPU
    assert subprocess.run([exe], capture_output=True, text=True).stdout.split() == ["582", "1"]


REF_INC = "/root/reference/src/include"


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF_INC, "TRPO.h")), reason="reference header absent")
def test_unchanged_reference_header_caller_links(tmp_path):
    """a caller compiled exactly as build/Makefile.cpuonly:5 compiles one (g++ -std=c++11
    against the reference's own src/include/TRPO.h, no extern "C") links with -ltrpo_mi355x."""
    exe, und = _link_caller(tmp_path, ["-DUSE_REFERENCE_HEADER"], REF_INC)
    for cxx_name in MANGLED.values():
        assert re.search(r"\bU %s$" % cxx_name, und, re.M), cxx_name
    assert subprocess.run([exe], capture_output=True, text=True).stdout.split() == ["582", "1"]


def test_library_runs_on_the_system_rocm_runtime():
    """conftest.py loads libtrpo_mi355x.so before anything imports torch, so its HIP calls resolve to
    the libamdhip64 it is built and rpath-linked against (lib/build_info.json), not torch's bundled copy."""
    import trpo_amd
    rt = trpo_amd.runtime_path()
    assert trpo_amd.built_runtime_dir() is not None
    assert trpo_amd.runtime_is_built_one(), (rt, trpo_amd.built_runtime_dir())


def test_runtime_dir_compares_whole_components():
    """/opt/rocm_other is not /opt/rocm (the old check was a string prefix)."""
    assert trpo_amd._same_dir("/opt/rocm/lib", "/opt/rocm/lib/")
    assert not trpo_amd._same_dir("/opt/rocm_other/lib", "/opt/rocm/lib")
    assert not trpo_amd._same_dir("/opt/rocm/lib/x", "/opt/rocm/lib")


def test_library_exports_exactly_the_abi():
    """the dynamic symbol table is the header's functions (C linkage) plus the seven
    C++-linkage twins of TRPO.h -- no kernel stubs, no trpo_dev_* / trpo_peer_* internals."""
    out = subprocess.run(["nm", "-D", "--defined-only", trpo_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    got = sorted(line.split()[-1] for line in out.splitlines() if line.strip())
    want = sorted(set(trpo_amd.header_symbols()) | set(MANGLED.values()))
    assert got == want, (sorted(set(got) - set(want))[:20], sorted(set(want) - set(got)))
