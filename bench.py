#!/usr/bin/env python3
"""Headline benchmark: FVP samples/sec + 10-iteration CG wall time, armDOF_0 policy.

BASELINE.json metric "FVP samples/sec + 10-iter CG wall time, armDOF_0 policy,
1/2/4/8 MI355X".  One STEP = one complete 10-iteration CG solve (ResidualTh=0,
so exactly 10 Fisher-vector products + the fp64 CG vector updates) over a
synthetic armDOF_0 batch of 50 000 samples resident in HBM (SURVEY.md §8d,
configs C3/C4).  With --gpus N the 50 000 samples are split into contiguous
shards, one per rank, and every FVP all-reduces the P-sized partial sum over
RCCL (strong scaling, config C4).

    python bench.py                      # N=1
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  value = 10 * 50 000 / (seconds per solve), the
whole-job FVP throughput; ms_per_step = the CG wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd"), os.path.join(ROOT, "oracle")]

import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402

ARM = [15, 16, 16, 3]
N_TOTAL = 50_000
PEAK_FP64_TFLOPS = 78.6       # MI355X dense fp64 matrix (AMD spec sheet; the guide lists fp32/bf16 only)
CG_ITERS = 10
DAMPING = 0.1
PEAK_FP32_TFLOPS = 157.3     # MI355X dense FP32 (vector = matrix), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def flops_per_sample(L):
    """2(5S - 2 L0 L1) + 7(L1 + L2) + 2 L3, S = sum L_i L_{i+1}."""
    S = sum(L[i] * L[i + 1] for i in range(len(L) - 1))
    return 2 * (5 * S - 2 * L[0] * L[1]) + 7 * sum(L[1:-1]) + 2 * L[-1]


def bytes_per_fvp(L, n):
    """observations read once + v in, Fv out, theta read once (fp32)."""
    return 4 * n * L[0] + 12 * synth.num_params(L)


def flops_per_sample_cached(L):
    """The cached-forward FVP (SURVEY §8d "optional cached-forward variant"): theta is fixed across
    the FVPs of a solve, so y1, y2 are computed once and only the R chains + backward run:
    2(4S - 2 L0 L1) + 7(L1 + L2) + 2 L3 = 3622 for armDOF_0."""
    S = sum(L[i] * L[i + 1] for i in range(len(L) - 1))
    return 2 * (4 * S - 2 * L[0] * L[1]) + 7 * sum(L[1:-1]) + 2 * L[-1]


def bytes_per_fvp_cached(L, n):
    """observations + the cached y1, y2 (fp32) read once, v in, Fv out, theta (188 B/sample armDOF_0)."""
    return 4 * n * (L[0] + sum(L[1:-1])) + 12 * synth.num_params(L)


from trpo_amd.dist import shard_range as shard  # noqa: E402


class Dist:
    """torch.distributed (gloo) only for bootstrap, barriers and the max-over-ranks
    timing; the data path all-reduce is RCCL inside libtrpo_mi355x.so."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.pg is None and self.world > 1:
            self.dist.barrier()

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def make_ctx(L, n_total, dist, device, precision=None):
    theta = synth.make_theta(L)
    obs_all = synth.make_obs(n_total, L[0])
    lo, hi = shard(n_total, dist.rank, dist.world)
    ctx = trpo_amd.Context(L, "lttl", theta, obs_all[lo:hi], np.ones(L[-1]), DAMPING, device=device,
                           precision=precision)
    if dist.world > 1:
        uid = dist.bcast_bytes(trpo_amd.unique_id() if dist.rank == 0 else None)
        ctx.attach_comm(dist.rank, dist.world, uid)
    return ctx, theta, obs_all


def time_steps(ctx, dist, steps, warmup, b):
    ctx.upload_b(b)
    for _ in range(warmup):
        ctx.enqueue_cg(CG_ITERS, 0.0)
    ctx.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.enqueue_cg(CG_ITERS, 0.0)
    ctx.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    return dist.max(t1 - t0)


def cpu_baseline(theta, obs_all, b, gpu_x):
    """The reference's own CG (oracle/_ref, compiled from src/TRPO_FVP.c + TRPO_CG.c with
    the Makefile.cpuonly flags) on 1 host core, full 10-iteration solve at N=50k; falls back
    to the clean-room port (oracle/liboracle.so) when oracle/_ref was not built."""
    import oracle
    n = obs_all.shape[0]
    res = dict(unit="FVP samples/s", cores=1,
               sample="one full 10-iteration CG solve, armDOF_0, N=50000, ResidualTh=0, 1 thread")
    x_ref = None
    if os.path.exists(oracle.REF_DRIVER_FAST):
        with tempfile.TemporaryDirectory() as tmp:
            mf, df, bf, xf = (os.path.join(tmp, f) for f in ("m.txt", "d.txt", "b.txt", "x.txt"))
            synth.write_model_file(mf, theta)
            synth.write_data_file(df, obs_all, np.ones(ARM[-1]))
            synth.write_vector_file(bf, b)
            cmd = [oracle.REF_DRIVER_FAST, "cg", mf, df, str(n), ",".join(map(str, ARM)), "lttl", str(DAMPING), bf,
                   str(CG_ITERS), "0", xf, "1"]
            w0 = time.perf_counter()
            out = subprocess.run(cmd, capture_output=True, text=True)
            wall = time.perf_counter() - w0
            if out.returncode == 0:
                x_ref = np.loadtxt(xf)
                # compute seconds exclude the reference's per-call file parsing: time it separately
                tcmd = [oracle.REF_DRIVER_FAST, "time", mf, df, str(n), ",".join(map(str, ARM)), "lttl",
                        str(DAMPING), bf, str(CG_ITERS), "0", "1"]
                tout = subprocess.run(tcmd, capture_output=True, text=True)
                tj = json.loads(tout.stderr.strip().splitlines()[-1])
                res.update(kind="reference", value=CG_ITERS * n / tj["compute_s"], compute_s=tj["compute_s"],
                           wall_s_incl_file_parse=tj["wall_s"])
    if x_ref is None:
        r = oracle.cg(ARM, "lttl", theta, obs_all, np.ones(ARM[-1]), b, CG_ITERS, 0.0, DAMPING, threads=1)
        x_ref = r["x"]
        res.update(kind="port", value=CG_ITERS * n / r["seconds"], compute_s=r["seconds"])
    try:
        res["cpu_model"] = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if "model name" in l][0]
    except Exception:
        pass
    rel = float(np.linalg.norm(gpu_x - x_ref) / np.linalg.norm(x_ref))
    return res, rel


def bench_update(device, L=ARM, n=N_TOTAL, reps=20, cpu_ref=True):
    """One full TRPO policy update (src/TRPO_Update.c: policy gradient, 10-iteration CG, FVP(x),
    line search) on a synthetic rollout of policy L, host-visible wall time per update (includes the
    host round trips of x / z / the line-search scalars); CPU reference TRPO_Update timed beside it
    (cpu_ref)."""
    import oracle
    theta = synth.make_theta(L)
    obs = synth.make_obs(n, L[0])
    std = np.ones(L[-1])
    mean, action, adv = synth.make_rollout(L, "lttl", theta, obs, std)
    ctx = trpo_amd.Context(L, "lttl", theta, obs, std, DAMPING, device=device)
    ctx.set_rollout(mean, action, adv)
    for _ in range(3):      # warm-up: first-call allocations, CG graph capture
        r = ctx.update()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.update()
    wall = (time.perf_counter() - t0) / reps
    ctx.close()
    out = {"update_ms": 1e3 * wall, "accepted": r["accepted"], "cg_iters": int(r["cg_iters"]),
           "samples": n, "what": "policy gradient (fp32 tile kernel, fp64 sums) + CG(10, 1e-10) + FVP(x) + fp64 line search"}
    if cpu_ref and os.path.exists(oracle.REF_DRIVER_FAST):
        with tempfile.TemporaryDirectory() as tmp:
            mf, df, of = (os.path.join(tmp, f) for f in ("m.txt", "d.txt", "o.txt"))
            synth.write_model_file(mf, theta)
            synth.write_data_file(df, obs, std, mean, action, adv)
            cmd = [oracle.REF_DRIVER_FAST, "update", mf, df, str(n), ",".join(map(str, L)), "lttl", str(DAMPING),
                   of, "1"]
            w0 = time.perf_counter()
            p = subprocess.run(cmd, capture_output=True, text=True)
            if p.returncode == 0:
                ref = np.loadtxt(of)
                tj = json.loads(p.stderr.strip().splitlines()[-1])
                out["cpu_reference_compute_s_1core"] = tj["compute_s"]
                out["cpu_reference_wall_s_1core_incl_parse"] = time.perf_counter() - w0
                out["theta_update_relL2_vs_cpu"] = float(np.linalg.norm((r["theta"] - theta) - (ref - theta))
                                                         / np.linalg.norm(ref - theta))
    return out


def bench_baseline(device, num_ep=20, ep_len=150, reps=50):
    """One value-baseline objective + gradient evaluation (src/TRPO_Baseline.c evaluate(), the
    L-BFGS callback) on the reference's own batch shape (20 episodes x 150 steps, [16,16,16,1]),
    device-resident data; the clean-room CPU port timed beside it (1 core)."""
    import oracle
    L = [16, 16, 16, 1]
    x, obs, tgt = synth.make_baseline_problem(L, num_ep, ep_len)
    with trpo_amd.Baseline(L, "lttl", device=device) as b:
        b.set_data(obs, tgt, num_ep, ep_len)
        b.evaluate(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            f, g = b.evaluate(x)
        dev = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    fo, go, _ = oracle.baseline_evaluate(L, "lttl", x, obs, tgt, num_ep, ep_len)
    cpu = time.perf_counter() - t0
    return {"evaluate_us": 1e6 * dev, "cpu_port_evaluate_us_1core": 1e6 * cpu, "samples": num_ep * ep_len,
            "grad_relL2_vs_cpu": float(np.linalg.norm(g - go) / np.linalg.norm(go)),
            "what": "host-visible wall per L-BFGS callback incl. x upload and g/f download"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra", action="store_true", help="also time the 2x64 configs (C2/C3)")
    args = ap.parse_args()

    dist = Dist()
    if dist.world != args.gpus and dist.rank == 0:
        print("warning: --gpus %d but WORLD_SIZE=%d" % (args.gpus, dist.world), file=sys.stderr)
    device = int(os.environ.get("TRPO_BENCH_DEVICE", dist.local_rank))   # override: testing only

    ctx, theta, obs_all = make_ctx(ARM, N_TOTAL, dist, device)
    P = synth.num_params(ARM)
    b = synth.make_b(P)

    t = time_steps(ctx, dist, args.steps, args.warmup, b)
    ms_per_step = 1e3 * t / args.steps
    value = CG_ITERS * N_TOTAL / (t / args.steps)
    x = ctx.download_x()

    # dominant kernel: the fused FVP kernel, timed with HIP events on the context's stream
    ctx.upload_v(synth.make_v(P))
    reps = 200
    k_ms = ctx.time_ms(0, reps)
    fvp_ms = ctx.time_ms(1, reps)
    n_local = ctx.n
    # the kernel timed is the one 9 of the 10 FVPs of a solve run: the cached-forward variant
    # (MODE 2); its algorithmic work is its own (fewer flops, the cache's bytes counted)
    flops = flops_per_sample_cached(ARM) * n_local
    bytes_alg = bytes_per_fvp_cached(ARM, n_local)
    achieved_tflops = flops / (k_ms * 1e-3) / 1e12
    achieved_gbs = bytes_alg / (k_ms * 1e-3) / 1e9
    hbm_bound = bytes_alg / (PEAK_HBM_GBS * 1e9) >= flops / (PEAK_FP32_TFLOPS * 1e12)

    traffic = None
    tpath = os.environ.get("TRPO_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "r01_fvp_traffic.json"))
    if os.path.exists(tpath) and dist.world == 1:
        # HBM bytes per launch of this kernel at this workload, from the committed rocprofv3 PMC passes
        traffic = json.load(open(tpath))["traffic_bytes"]

    result = {
        "metric": "FVP samples/sec + 10-iter CG wall time, armDOF_0 policy",
        "value": value,
        "unit": "FVP samples/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded splitmix64, SURVEY §8d)",
        "config": {"workload": "cg10_armDOF_0_N50000", "policy": "armDOF_0 [15,16,16,3] lttl",
                   "samples": N_TOTAL, "cg_iters": CG_ITERS, "residual_th": 0.0, "damping": DAMPING,
                   "parallelism": "dp%d (contiguous sample shards, RCCL all-reduce per FVP)" % dist.world,
                   "cg_scalars": "fp64", "fvp_kernel": ctx.kernel_name, "geometry": ctx.geometry},
        "cg_wall_ms": ms_per_step,
        "fvp_ms": fvp_ms,
        "roofline": {"bound": "hbm" if hbm_bound else "mfma",
                     "achieved": achieved_gbs if hbm_bound else achieved_tflops,
                     "peak": PEAK_HBM_GBS if hbm_bound else PEAK_FP32_TFLOPS,
                     "unit": "GB/s" if hbm_bound else "TFLOP/s",
                     "frac": achieved_gbs / PEAK_HBM_GBS if hbm_bound else achieved_tflops / PEAK_FP32_TFLOPS,
                     "traffic": traffic,
                     "kernel": "fvp_mlp3_kernel (MODE 2: cached forward)", "kernel_ms": k_ms,
                     "flops_per_launch": flops, "alg_bytes_per_launch": bytes_alg,
                     "fp32_tflops": achieved_tflops, "fp32_frac": achieved_tflops / PEAK_FP32_TFLOPS,
                     "hbm_gbs_algorithmic": achieved_gbs, "hbm_frac_algorithmic": achieved_gbs / PEAK_HBM_GBS,
                     "full_recompute_equiv_tflops": flops_per_sample(ARM) * n_local / (k_ms * 1e-3) / 1e12},
    }

    if args.extra and dist.world == 1:
        extra = {}
        L2 = [15, 64, 64, 3]
        # C2: repeated FVP calls on one context reuse the forward-activation cache (theta unchanged);
        # a first call after set_theta recomputes the forward pass -- timed too (TRPO_YCACHE=0)
        c2res = {}
        for tag, env in (("", None), ("_recompute", "0")):
            if env is not None:
                os.environ["TRPO_YCACHE"] = env
            c2, th2, obs2 = make_ctx(L2, 4096, dist, device)
            os.environ.pop("TRPO_YCACHE", None)
            c2.upload_v(synth.make_v(synth.num_params(L2)))
            k2 = c2.time_ms(0, reps)
            f2 = c2.time_ms(1, reps)
            fl = flops_per_sample_cached(L2) if env is None else flops_per_sample(L2)
            c2res.update({"fvp_ms" + tag: f2, "kernel_ms" + tag: k2, "fvp_samples_per_s" + tag: 4096 / (f2 * 1e-3),
                          "kernel_tflops" + tag: fl * 4096 / (k2 * 1e-3) / 1e12})
            c2.close()
        extra["C2_fvp_2x64_N4096"] = c2res
        c3, th3, obs3 = make_ctx(L2, N_TOTAL, dist, device)
        t3 = time_steps(c3, dist, 20, 3, synth.make_b(synth.num_params(L2)))
        k3 = c3.time_ms(0, reps)
        extra["C3_cg10_2x64_N50000"] = {"cg_wall_ms": 1e3 * t3 / 20, "fvp_samples_per_s": CG_ITERS * N_TOTAL / (t3 / 20),
                                        "kernel_ms": k3, "kernel": c3.kernel_name + " (cached forward)",
                                        "kernel_tflops": flops_per_sample_cached(L2) * N_TOTAL / (k3 * 1e-3) / 1e12,
                                        "kernel_tflops_recompute_equiv":
                                            flops_per_sample(L2) * N_TOTAL / (k3 * 1e-3) / 1e12}
        c3.close()
        # fp64 precision mode (the reference's arithmetic, fp64 MFMA): same CG(10) workloads
        for key, L in (("C1_cg10_armDOF_0_N50000_fp64", [15, 16, 16, 3]), ("C3_cg10_2x64_N50000_fp64", L2)):
            cf, _, _ = make_ctx(L, N_TOTAL, dist, device, precision="fp64")
            tf = time_steps(cf, dist, 20, 3, synth.make_b(synth.num_params(L)))
            kf = cf.time_ms(0, reps)
            extra[key] = {"cg_wall_ms": 1e3 * tf / 20, "fvp_samples_per_s": CG_ITERS * N_TOTAL / (tf / 20),
                          "kernel": cf.kernel_name + " (cached forward)", "kernel_ms": kf,
                          "kernel_tflops": flops_per_sample_cached(L) * N_TOTAL / (kf * 1e-3) / 1e12,
                          "kernel_tflops_recompute_equiv": flops_per_sample(L) * N_TOTAL / (kf * 1e-3) / 1e12,
                          "peak_fp64_mfma_tflops": PEAK_FP64_TFLOPS}
            cf.close()
        extra["C5_update_armDOF_0_N50000"] = bench_update(device)
        extra["C5_update_2x64_N50000"] = bench_update(device, L=[15, 64, 64, 3], cpu_ref=False)
        extra["C5_baseline_evaluate_N3000"] = bench_baseline(device)
        result["extra"] = extra

    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        cb, rel = cpu_baseline(theta, obs_all, b, x)
        result["cpu_baseline"] = cb
        result["parity"] = {"cg_step_relL2_vs_cpu": rel, "tolerance": 1e-4}
    ctx.close()
    dist.close()
    if dist.rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
