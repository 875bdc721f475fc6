"""MI355X: the drop-in from a COMPILED caller.

tests/c_caller/drop_in_caller.c calls NumParamsCalc / FVPFast / CG / TRPO_Update the way the
reference's src/TRPOCpuCode.c:15-135,314-372 calls them -- built as C with gcc and as C++ with g++
(build/Makefile.cpuonly:5 compiles callers with g++) against include/trpo_mi355x.h and linked with
-ltrpo_mi355x (built by __graft_entry__.build(), make -C tests/c_caller).  Run on the reference's
fixture files; its output vectors are checked against the goldens the reference produced, with the
same tolerances as the ctypes parity tests, and its stdout must carry the reference's lines.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("binary", ["drop_in_caller_c", "drop_in_caller_cxx", "drop_in_caller_cxxmangle",
                                    "drop_in_caller_refhdr"])
def test_compiled_caller_on_fixtures(binary, tmp_path):
    """_cxxmangle and _refhdr import the C++-LINKAGE entry points (_Z7FVPFast9TRPOparamPdS0_m, ...):
    _refhdr is compiled against the reference's own src/include/TRPO.h with g++ -std=c++11, as
    build/Makefile.cpuonly:5,11 compiles an unchanged caller; it is built only where /root/reference
    exists (by __graft_entry__.build() in the build container, then shipped with the tree)."""
    exe = os.path.join(HERE, "c_caller", binary)
    if binary == "drop_in_caller_refhdr" and not os.path.exists(exe):
        pytest.skip("built only where the reference's TRPO.h exists (make -C tests/c_caller refhdr)")
    assert os.path.exists(exe), "build the callers first: make -C tests/c_caller (__graft_entry__.build)"
    p = subprocess.run([exe, cases.GOLDEN, str(tmp_path), "3150", "6"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    fvp = np.loadtxt(tmp_path / "fvp.txt")
    cg = np.loadtxt(tmp_path / "cg.txt")
    upd = np.loadtxt(tmp_path / "update.txt")
    assert cases.rel_l2(fvp, cases.expected(cases.case("fix_fvp_n3150"))) <= 1e-5
    assert cases.rel_l2(cg, cases.expected(cases.case("fix_cg_n3150_th1e-10"))) <= 1e-4
    th = cases.fixture_model()
    assert cases.rel_l2(upd - th, cases.expected(cases.case("fix_update_n3150")) - th) <= 1e-4
    out = p.stdout
    iters = re.findall(r"CG Iter\[(\d+)\] Residual Norm=(\S+), Soln Norm=(\S+)", out)
    assert iters and iters[0][0] == "0" and iters[0][1].startswith("9.05595253")
    # CG(10, 1e-10) and TRPO_Update's CG each stop after 8 FVPs on the fixture, as the reference does:
    # 9 "CG Iter[...]" lines each (src/TRPO_CG.c:56 prints before the threshold test)
    assert len(iters) == 18 and [int(i[0]) for i in iters] == list(range(9)) * 2
    assert re.search(r"shs: \S+", out) and re.search(r"lagrange multiplier: \S+, gnorm: \S+", out)
    assert re.search(r"a/e/r \S+ / \S+ / \S+", out)
    assert "[ERROR] Cannot open Model File" in p.stderr          # the bad-path call, reference message
