#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/ref_driver -- the reference's unchanged src/TRPO_FVP.c,
src/TRPO_CG.c, src/TRPO_Util.c and src/TRPO_Update.c compiled by oracle/Makefile (needs
/root/reference; only ever run in the build container, never on the GPU box).

Every case is described in manifest.json so that tests can rebuild the exact
inputs: fixture cases read the reference's own ArmTest*.txt files (copied here
as data), synthetic cases regenerate inputs with trpo_amd.synth (bit-exact).
Outputs are written with %.17g, so they round-trip exactly.

    python tests/golden/make_goldens.py
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "trpo-robot-control_amd"))
sys.path.insert(0, os.path.dirname(HERE))
from trpo_amd import synth  # noqa: E402
from cases import baseline_inputs, synth_update_inputs  # noqa: E402

DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
ARM = [15, 16, 16, 3]
SIGMA3 = [0.6065306597126334, 0.8, 1.3]     # exp(-0.5) and two more, as exact literals
# TRPO_Update with sigma != 1: model LogStd and the data file's Std (= exp(LogStd), literals)
LOGSTD_U = [-0.5, 0.0, 0.25]
SIGMA_U = [0.6065306597126334, 1.0, 1.2840254166877414]

CASES = [
    # --- reference fixtures (build/ArmTest*.txt) ---
    dict(name="fix_fvp_n3150", kind="fvp", src="fixture", n=3150, vin="fvp_col1"),
    dict(name="fix_fvp_n2400", kind="fvp", src="fixture", n=2400, vin="fvp_col1"),
    dict(name="fix_cg_n3150_th1e-10", kind="cg", src="fixture", n=3150, vin="cg_col1", maxiter=10, resth=1e-10),
    dict(name="fix_cg_n3150_th0", kind="cg", src="fixture", n=3150, vin="cg_col1", maxiter=10, resth=0.0),
    dict(name="fix_cg_n2400_th1e-10", kind="cg", src="fixture", n=2400, vin="cg_col1", maxiter=10, resth=1e-10),
    dict(name="fix_fvp_n1", kind="fvp", src="fixture", n=1, vin="fvp_col1"),
    dict(name="fix_fvp_n17", kind="fvp", src="fixture", n=17, vin="fvp_col1"),
    # --- synthetic (trpo_amd.synth, seed 20261015) ---
    dict(name="syn_sigma_fvp", kind="fvp", src="synth", layers=ARM, acfunc="lttl", n=1000, std=SIGMA3, vin="v"),
    dict(name="syn_sigma_cg", kind="cg", src="synth", layers=ARM, acfunc="lttl", n=1000, std=SIGMA3, vin="b",
         maxiter=10, resth=0.0),
    dict(name="syn_acts_fvp", kind="fvp", src="synth", layers=ARM, acfunc="lsto", n=777, std=SIGMA3, vin="v"),
    dict(name="syn_deep_fvp", kind="fvp", src="synth", layers=[15, 32, 16, 8, 3], acfunc="lotsl", n=1000,
         std=[1.0, 1.0, 1.0], vin="v"),
    dict(name="syn_wide_in_fvp", kind="fvp", src="synth", layers=[376, 64, 64, 17], acfunc="lttl", n=600,
         std=[1.0] * 17, vin="v"),
    dict(name="syn_2x64_fvp_n4096", kind="fvp", src="synth", layers=[15, 64, 64, 3], acfunc="lttl", n=4096,
         std=[1.0, 1.0, 1.0], vin="v"),
    dict(name="syn_arm_cg_n50000", kind="cg", src="synth", layers=ARM, acfunc="lttl", n=50000,
         std=[1.0, 1.0, 1.0], vin="b", maxiter=10, resth=0.0),
    dict(name="syn_2x64_cg_n50000", kind="cg", src="synth", layers=[15, 64, 64, 3], acfunc="lttl", n=50000,
         std=[1.0, 1.0, 1.0], vin="b", maxiter=10, resth=0.0),
    # --- TRPO_Update (src/TRPO_Update.c; hard-wired CG 10 / 1e-10, MaxKL 0.01, 10 backtracks) ---
    dict(name="fix_update_n3150", kind="update", src="fixture", n=3150),
    dict(name="syn_update_arm_n20000", kind="update", src="synth", layers=ARM, acfunc="lttl", n=20000,
         logstd=[0.0, 0.0, 0.0], std=[1.0, 1.0, 1.0], adv="normal"),
    dict(name="syn_update_sigma_n5000", kind="update", src="synth", layers=ARM, acfunc="lttl", n=5000,
         logstd=LOGSTD_U, std=SIGMA_U, adv="normal"),
    dict(name="syn_update_2x64_n8192", kind="update", src="synth", layers=[15, 64, 64, 3], acfunc="lttl",
         n=8192, logstd=[0.0, 0.0, 0.0], std=[1.0, 1.0, 1.0], adv="normal"),
    # every backtrack rejected: the reference returns the CG step x itself (:850-852)
    dict(name="syn_update_reject_n5000", kind="update", src="synth", layers=ARM, acfunc="lttl", n=5000,
         logstd=[0.0, 0.0, 0.0], std=[1.0, 1.0, 1.0], adv="neg_abs"),
    # --- value-baseline objective evaluate() (src/TRPO_Baseline.c:29-240) ---
    dict(name="syn_baseline_n3000", kind="baseline", layers=[16, 16, 16, 1], acfunc="lttl", num_ep=20, ep_len=150,
         scale=1.0, pad=0.0),
    dict(name="syn_baseline_n777", kind="baseline", layers=[16, 16, 16, 1], acfunc="lttl", num_ep=7, ep_len=111,
         scale=1.7, pad=0.25),
    dict(name="syn_baseline_lin_n1000", kind="baseline", layers=[16, 32, 16, 1], acfunc="lltl", num_ep=10,
         ep_len=100, scale=0.8, pad=0.0),
    # the reference's own baseline parameters (build/ArmTestBaseline.txt: the [16,16,16,1] theta that
    # src/TRPOCpuCode.c:381 hands to the trainers), zero-padded to 576 as the L-BFGS vector; the
    # fixture's observations, 20 episodes x 150 steps, and its advantage column as regression targets
    dict(name="fix_baseline_armtest", kind="baseline", src="fixture", layers=[16, 16, 16, 1], acfunc="lttl",
         num_ep=20, ep_len=150),
]



def build_inputs(case, tmp):
    """Returns (model_path, data_path, layers, acfunc, vin_vector)."""
    if case["src"] == "fixture":
        layers, acfunc = ARM, "lttl"
        model, data = os.path.join(HERE, "ArmTestModel.txt"), os.path.join(HERE, "ArmTestData.txt")
        P = synth.num_params(layers)
        fname = "ArmTestFVP.txt" if case["vin"] == "fvp_col1" else "ArmTestCG.txt"
        vin = np.loadtxt(os.path.join(HERE, fname))[:P, 0]
        return model, data, layers, acfunc, vin
    layers, acfunc = case["layers"], case["acfunc"]
    P = synth.num_params(layers)
    theta = synth.make_theta(layers)
    obs = synth.make_obs(case["n"], layers[0])
    model, data = os.path.join(tmp, case["name"] + ".model"), os.path.join(tmp, case["name"] + ".data")
    synth.write_model_file(model, theta)
    synth.write_data_file(data, obs, np.asarray(case["std"], dtype=np.float64))
    vin = synth.make_v(P) if case["vin"] == "v" else synth.make_b(P)
    return model, data, layers, acfunc, vin


def run_update_case(case, tmp):
    if case["src"] == "fixture":
        layers, acfunc = ARM, "lttl"
        model, data = os.path.join(HERE, "ArmTestModel.txt"), os.path.join(HERE, "ArmTestData.txt")
    else:
        layers, acfunc = case["layers"], case["acfunc"]
        theta, obs, std, mean, action, adv = synth_update_inputs(case)
        model, data = os.path.join(tmp, case["name"] + ".model"), os.path.join(tmp, case["name"] + ".data")
        synth.write_model_file(model, theta)
        synth.write_data_file(data, obs, std, mean, action, adv)
    out = os.path.join(HERE, case["name"] + ".txt")
    lay = ",".join(str(x) for x in layers)
    cmd = [DRIVER, "update", model, data, str(case["n"]), lay, acfunc, "0.1", out, "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, check=True)
    rec = dict(case)
    rec.update(layers=layers, acfunc=acfunc, damping=0.1, expected=os.path.basename(out))
    hist = re.findall(r"CG Iter\[(\d+)\] Residual Norm=(\S+), Soln Norm=(\S+)", res.stdout)
    rec["rdotr"] = [float(h[1]) for h in hist]
    rec["iters"] = len(hist) - 1
    rec["shs"] = float(re.search(r"shs: (\S+)", res.stdout).group(1))
    m = re.search(r"lagrange multiplier: (\S+), gnorm: (\S+)", res.stdout)
    rec["lagrange"], rec["gnorm"] = float(m.group(1)), float(m.group(2))
    rec["fval"] = float(re.search(r"fval before (\S+)", res.stdout).group(1))
    are = re.findall(r"a/e/r (\S+) / (\S+) / (\S+)", res.stdout)
    rec["ratio"] = [float(a[2]) for a in are]
    last_a, last_r = float(are[-1][0]), float(are[-1][2])
    rec["accepted"] = len(are) - 1 if (last_r > 0.1 and last_a > 0) else -1
    y = np.loadtxt(out)
    rec["norm"] = float(np.linalg.norm(y))
    print("%-24s P=%-5d |theta'|=%.15g accepted=%d" % (case["name"], len(y), rec["norm"], rec["accepted"]),
          flush=True)
    return rec


def run_baseline_case(case, tmp):
    x, obs, target = baseline_inputs(case)
    files = {}
    for key, arr in (("obs", obs.ravel()), ("tgt", target), ("x", x)):
        files[key] = os.path.join(tmp, case["name"] + "." + key)
        synth.write_vector_file(files[key], arr)
    out = os.path.join(HERE, case["name"] + ".txt")
    cmd = [DRIVER, "baseline", ",".join(str(v) for v in case["layers"]), case["acfunc"], str(case["num_ep"]),
           str(case["ep_len"]), files["obs"], files["tgt"], files["x"], out]
    res = subprocess.run(cmd, capture_output=True, text=True, check=True)
    rec = dict(case)
    rec["f"] = float(re.search(r"f (\S+)", res.stdout).group(1))
    rec["padded"] = int(x.size)
    rec["n"] = case["num_ep"] * case["ep_len"]
    rec["expected"] = os.path.basename(out)
    print("%-24s f=%.15g" % (case["name"], rec["f"]), flush=True)
    return rec


def run_case(case, tmp):
    if case["kind"] == "update":
        return run_update_case(case, tmp)
    if case["kind"] == "baseline":
        return run_baseline_case(case, tmp)
    model, data, layers, acfunc, vin = build_inputs(case, tmp)
    vpath = os.path.join(tmp, case["name"] + ".in")
    synth.write_vector_file(vpath, vin)
    out = os.path.join(HERE, case["name"] + ".txt")
    lay = ",".join(str(x) for x in layers)
    if case["kind"] == "fvp":
        cmd = [DRIVER, "fvp", model, data, str(case["n"]), lay, acfunc, "0.1", vpath, out, "1"]
    else:
        cmd = [DRIVER, "cg", model, data, str(case["n"]), lay, acfunc, "0.1", vpath, str(case["maxiter"]),
               repr(case["resth"]), out, "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, check=True)
    rec = dict(case)
    rec.update(layers=layers, acfunc=acfunc, damping=0.1, expected=os.path.basename(out))
    if case["kind"] == "cg":
        hist = re.findall(r"CG Iter\[(\d+)\] Residual Norm=(\S+), Soln Norm=(\S+)", res.stdout)
        rec["rdotr"] = [float(h[1]) for h in hist]
        rec["xnorm"] = [float(h[2]) for h in hist]
        rec["iters"] = len(hist) - 1
    y = np.loadtxt(out)
    rec["norm"] = float(np.linalg.norm(y))
    print("%-24s P=%-5d |out|=%.15g" % (case["name"], len(y), rec["norm"]), flush=True)
    return rec


def main():
    """python tests/golden/make_goldens.py [NAME ...]: all cases, or only the named ones (the other
    records of manifest.json are kept)."""
    if not os.path.exists(DRIVER):
        sys.exit("build the reference first: make -C oracle ref")
    only = set(sys.argv[1:])
    old = {}
    if only and os.path.exists(os.path.join(HERE, "manifest.json")):
        old = {c["name"]: c for c in json.load(open(os.path.join(HERE, "manifest.json")))["cases"]}
    with tempfile.TemporaryDirectory() as tmp:
        recs = [run_case(c, tmp) if (not only or c["name"] in only) else old[c["name"]] for c in CASES]
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_goldens.py", "driver": "oracle/_ref/ref_driver",
                   "seed": synth.SEED, "cases": recs}, f, indent=1)


if __name__ == "__main__":
    main()
