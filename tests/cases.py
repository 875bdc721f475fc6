"""Rebuild the inputs of every golden case in tests/golden/manifest.json."""
from __future__ import annotations

import json
import os

import numpy as np

from trpo_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ARM = [15, 16, 16, 3]


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


def case(name):
    for c in manifest():
        if c["name"] == name:
            return c
    raise KeyError(name)


def _read_table(fname):
    return np.loadtxt(os.path.join(GOLDEN, fname))


_fixture_cache = {}


def fixture_data():
    """ArmTestData.txt -> (obs[3150,15], std[3] of the LAST line), as FVPFast reads it."""
    if "data" not in _fixture_cache:
        t = _read_table("ArmTestData.txt")
        _fixture_cache["data"] = (np.ascontiguousarray(t[:, 6:21]), t[-1, 3:6].copy())
    return _fixture_cache["data"]


def fixture_model():
    if "model" not in _fixture_cache:
        _fixture_cache["model"] = _read_table("ArmTestModel.txt")
    return _fixture_cache["model"]


def inputs(c):
    """Returns dict(layers, acfunc, theta, obs, std, vin, damping) for a manifest case."""
    n = c["n"]
    if c["src"] == "fixture":
        obs, _ = fixture_data()
        obs = obs[:n]
        # FVPFast keeps the Std of the last line it parsed, i.e. line n
        std = _read_table("ArmTestData.txt")[n - 1, 3:6] if n < 3150 else fixture_data()[1]
        theta = fixture_model()
        fname = "ArmTestFVP.txt" if c["vin"] == "fvp_col1" else "ArmTestCG.txt"
        vin = _read_table(fname)[:, 0]
        return dict(layers=ARM, acfunc="lttl", theta=theta, obs=obs, std=np.asarray(std), vin=vin,
                    damping=c["damping"])
    layers = c["layers"]
    P = synth.num_params(layers)
    return dict(layers=layers, acfunc=c["acfunc"], theta=synth.make_theta(layers),
                obs=synth.make_obs(n, layers[0]), std=np.asarray(c["std"], dtype=np.float64),
                vin=synth.make_v(P) if c["vin"] == "v" else synth.make_b(P), damping=c["damping"])


def synth_update_inputs(c):
    """theta, obs, std, mean, action, adv of a synthetic TRPO_Update case."""
    layers, acfunc, n = c["layers"], c["acfunc"], c["n"]
    theta = synth.make_theta(layers)
    theta[-layers[-1]:] = c["logstd"]
    obs = synth.make_obs(n, layers[0])
    std = np.asarray(c["std"], dtype=np.float64)
    mean, action, adv = synth.make_rollout(layers, acfunc, theta, obs, std)
    if c["adv"] == "neg_abs":
        adv = -np.abs(adv)
    return theta, obs, std, mean, action, adv


def update_inputs(c):
    """dict(layers, acfunc, theta, obs, std, mean, action, adv, damping) of an update case."""
    if c["src"] == "fixture":
        t = _read_table("ArmTestData.txt")[: c["n"]]
        A, O = 3, 15
        return dict(layers=ARM, acfunc="lttl", theta=fixture_model(), obs=np.ascontiguousarray(t[:, 2 * A:2 * A + O]),
                    std=t[-1, A:2 * A].copy(), mean=np.ascontiguousarray(t[:, :A]),
                    action=np.ascontiguousarray(t[:, 2 * A + O:3 * A + O]), adv=t[:, 3 * A + O].copy(),
                    damping=c["damping"])
    theta, obs, std, mean, action, adv = synth_update_inputs(c)
    return dict(layers=c["layers"], acfunc=c["acfunc"], theta=theta, obs=obs, std=std, mean=mean, action=action,
                adv=adv, damping=c["damping"])


def baseline_inputs(c):
    """(x, observ, target) of a baseline case; the expected file holds g [padded] then predict [N].
    Fixture case: x = the reference's ArmTestBaseline.txt (561 values) zero-padded to a multiple of 16,
    observations and targets (the advantage column) from the first num_ep * ep_len lines of
    ArmTestData.txt."""
    if c.get("src") == "fixture":
        th = _read_table("ArmTestBaseline.txt")
        x = np.zeros((th.size + 15) // 16 * 16)
        x[:th.size] = th
        n = c["num_ep"] * c["ep_len"]
        t = _read_table("ArmTestData.txt")[:n]
        return x, np.ascontiguousarray(t[:, 6:21]), t[:, 24].copy()
    return synth.make_baseline_problem(c["layers"], c["num_ep"], c["ep_len"], scale=c["scale"], pad_value=c["pad"])


def expected(c):
    return np.loadtxt(os.path.join(GOLDEN, c["expected"]))


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))
