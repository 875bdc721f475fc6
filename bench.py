#!/usr/bin/env python3
"""Headline benchmark: FVP samples/sec + 10-iteration CG wall time, armDOF_0 policy.

BASELINE.json metric "FVP samples/sec + 10-iter CG wall time, armDOF_0 policy,
1/2/4/8 MI355X".  One STEP = one complete 10-iteration CG solve (ResidualTh=0,
so exactly 10 Fisher-vector products + the fp64 CG vector updates) over a
synthetic armDOF_0 batch of 50 000 samples resident in HBM (SURVEY.md §8d,
configs C3/C4).  With --gpus N the 50 000 samples are split into contiguous
shards, one per rank (one process per GPU), and every FVP all-reduces the
P-sized partial sum over xGMI (strong scaling, config C4): by default with the
library's one-shot peer-window exchange (--comm peer; SURVEY §5 / §8e: "prefer
... a custom P2P one-shot all-reduce over IPC buffers" for these 2-43 KB
messages), RCCL's all-reduce timed beside it (extra.C4_rccl_exchange) and taken
instead if the peer exchange fails its setup or self-check (--comm rccl swaps
the two roles).

    python bench.py                      # N=1
    python bench.py --gpus 8             # launches 8 rank processes itself
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  value = 10 * 50 000 / (seconds per solve), the
whole-job FVP throughput; ms_per_step = the CG wall time (max over ranks).
Measured in this order at N = 1: the secondary configs (extra), the dominant kernel's HIP-event
timing (roofline), then the headline's timed region (W untimed solves, exactly K timed ones).  At
N > 1 the headline's collective is set up stage by stage with cross-rank agreement, self-checked and
hash-checked before anything is timed (make_ctx_agreed; comm.verify / comm.fallback in the line), the
headline is timed right after, and the secondary configs follow, each set up and run the same agreed
way; a watchdog prints the line by a deadline whatever they do (Emitter).
At N = 1, after the timed region, roofline.traffic is measured in the same run: two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE, one per child process of this script on the headline workload;
measure_traffic); --no-pmc, or a failed pass, falls back to the newest committed profile.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

ARM = [15, 16, 16, 3]
N_TOTAL = 50_000
CG_ITERS = 10
DAMPING = 0.1
PEAK_FP32_TFLOPS = 157.3     # MI355X dense FP32 (vector = matrix), MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6      # MI355X dense fp64 matrix (AMD spec sheet; the guide lists fp32/bf16 only)
PEAK_HBM_GBS = 8000.0
# the latency crossover of the sharded solve; 6 250 and 500 000 are the per-rank shards of
# the 50k headline and of 4M at 8 GPUs (the one-GPU inputs of DESIGN §6.1's 8-GPU model)
SWEEP_N = (6_250, 500_000, 4_000_000)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a solve takes ~0.1 ms: 500 timed solves (~50 ms) after 50 warm-up solves, so the one-off costs of
    # the timed region (the first graph launch, the closing stream synchronisation, the clock settling
    # after the warm-up) are not booked against the per-solve time (measured: 50 timed solves after 5
    # warm-up ones read ~4 % slower per solve than 500 after 50 on the same box)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # round 6: the peer-window exchange is the headline's default collective at N > 1.  Its one-GPU floor is
    # 3.56 us per exchange (profiles/r05_peer_floor_1gpu.txt) against RCCL's multi-step protocol for the 9-37 KB
    # replica message; RCCL stays the measured A/B (extra.C4_rccl_exchange) and the fallback of the agreed setup
    ap.add_argument("--comm", choices=("rccl", "peer"), default="peer",
                    help="N > 1: collective of the headline solve (peer: the peer-window exchange over xGMI, "
                         "default; rccl: RCCL's all-reduce)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="N = 1: take roofline.traffic from the newest committed profile instead of measuring it")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)   # internal: see measure_traffic
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary configs (C2, C3 2x64, fp64, C5, baseline, N sweep)")
    return ap.parse_args()


def relaunch(args) -> int:
    """--gpus N without a torch.distributed environment: start N rank processes (one per GPU) with
    torch.distributed.run and exit with its code.  Nothing in this process has touched HIP."""
    # --standalone: the rendezvous store binds a free port itself (a port probed here and passed on
    # can be taken by another process on a shared box before torchrun binds it: EADDRINUSE, seen once)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", "--nproc-per-node=%d" % args.gpus, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def flops_per_sample(L):
    """2(5S - 2 L0 L1) + 7(L1 + L2) + 2 L3, S = sum L_i L_{i+1}."""
    S = sum(L[i] * L[i + 1] for i in range(len(L) - 1))
    return 2 * (5 * S - 2 * L[0] * L[1]) + 7 * sum(L[1:-1]) + 2 * L[-1]


def flops_per_sample_cached(L):
    """The cached-forward FVP (SURVEY §8d "optional cached-forward variant"): theta is fixed across
    the FVPs of a solve, so y1, y2 are computed once and only the R chains + backward run:
    2(4S - 2 L0 L1) + 7(L1 + L2) + 2 L3 = 3622 for armDOF_0."""
    S = sum(L[i] * L[i + 1] for i in range(len(L) - 1))
    return 2 * (4 * S - 2 * L[0] * L[1]) + 7 * sum(L[1:-1]) + 2 * L[-1]


def num_params(L):
    return sum(L[i] * L[i + 1] + L[i + 1] for i in range(len(L) - 1)) + L[-1]


def bytes_per_fvp_cached(L, n):
    """observations + the cached y1, y2 (fp32) read once, v in, Fv out, theta (188 B/sample armDOF_0)."""
    return 4 * n * (L[0] + sum(L[1:-1])) + 12 * num_params(L)


def bytes_cg_step(L):
    """The fp64 CG step fused into the CG-iteration kernel, each P-vector touched once: z, p, r, x in,
    p, r, x and the new basis vector out."""
    return 8 * 8 * num_params(L)


class Dist:
    """torch.distributed (gloo) only for bootstrap, barriers and the max-over-ranks timing; the
    data-path all-reduce is RCCL inside libtrpo_mi355x.so."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.group = None           # the group every collective below uses (None: the default group)
        self.broken = False         # a gloo collective raised: the ranks may be out of step, no more of them
        if self.world > 1:
            import datetime
            import torch.distributed as dist
            # every rendezvous / agreement is bounded: a rank that dies makes the others raise, not hang.
            # The headline's setup and timed region use the default group (TRPO_GLOO_TIMEOUT_S); the
            # secondary configs measured after it use a group with a shorter bound, so that their worst
            # case (one rank stuck) ends well inside the driver's lease
            dist.init_process_group("gloo", timeout=datetime.timedelta(
                seconds=int(os.environ.get("TRPO_GLOO_TIMEOUT_S", "600"))))
            self.dist = dist
            self.secondary_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(
                seconds=int(os.environ.get("TRPO_GLOO_SECONDARY_TIMEOUT_S", "90"))))

    def _coll(self, fn):
        if self.broken:
            raise RuntimeError("an earlier gloo collective failed; the ranks may be out of step")
        try:
            return fn()
        except Exception:
            self.broken = True
            raise

    def barrier(self):
        if self.world > 1:
            self._coll(lambda: self.dist.barrier(group=self.group))

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self._coll(lambda: self.dist.broadcast_object_list(obj, src=0, group=self.group))
        return obj[0]

    def allgather_bytes(self, b):
        if self.world == 1:
            return [b]
        out = [None] * self.world
        self._coll(lambda: self.dist.all_gather_object(out, b, group=self.group))
        return out

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self._coll(lambda: self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group))
        return float(t.item())

    def secondary(self):
        """Context manager: the collectives inside use the secondary group (shorter gloo bound)."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            saved = self.group
            if self.world > 1:
                self.group = self.secondary_group
            try:
                yield self
            finally:
                self.group = saved
        return cm()

    def close(self):
        if self.world > 1 and not self.broken:
            self.dist.destroy_process_group()


def make_ctx(L, n_total, dist, device, precision=None, comm="rccl"):
    """This rank's context: all weights, its contiguous shard of the seeded observation stream.
    comm: "rccl" (RCCL communicator) or "peer" (the peer-window exchange over xGMI, csrc/trpo_peer.hip).
    For the secondary configs; the headline context is built by make_ctx_agreed."""
    import numpy as np
    import trpo_amd
    from trpo_amd import synth
    from trpo_amd.dist import shard_range
    theta = synth.make_theta(L)
    lo, hi = shard_range(n_total, dist.rank, dist.world)
    obs = synth.make_obs(hi - lo, L[0], start=lo)
    ctx = trpo_amd.Context(L, "lttl", theta, obs, np.ones(L[-1]), DAMPING, device=device, precision=precision)
    try:
        if dist.world > 1 and comm == "peer":
            handles = dist.allgather_bytes(ctx.peer_handle())
            ctx.attach_peers(dist.rank, dist.world, handles)
        elif dist.world > 1:
            uid = dist.bcast_bytes(trpo_amd.unique_id() if dist.rank == 0 else None)
            ctx.attach_comm(dist.rank, dist.world, uid, COMM_TIMEOUT_MS)
        if dist.world > 1:
            info = ctx.comm_info()
            if info["world"] != dist.world:
                raise RuntimeError("%s communicator has %d ranks, expected %d" % (comm, info["world"], dist.world))
    except BaseException:
        ctx.close()
        raise
    return ctx, theta, obs


COMM_TIMEOUT_MS = int(os.environ.get("TRPO_BENCH_COMM_TIMEOUT_MS", "60000"))   # RCCL init, self-check, solve
STAGES = ("context", "bootstrap", "attach", "verify", "solve", "hash")


class StageFault(RuntimeError):
    pass


def _fault(stage, rank, attempt):
    """TRPO_BENCH_FAULT=<stage>:<rank>[:<attempt>][,...] (testing): make `stage` fail on `rank` in attempt
    `attempt` (default 0).  Stages of the headline's collective setup: STAGES, plus comm-verify /
    comm-hang, which arm the LIBRARY's self-check fault (TRPO_COMM_FAULT) for that attempt.  The
    secondary configs at N > 1 prefix their stages with their name (`sweep4000000.context:1`,
    `update.solve:1`, `sweep500000.timed:1`, ...; see run_secondary); `<name>.hang:R` makes rank R block
    forever inside that secondary (a library call that ignores its bound: the watchdog's case)."""
    spec = os.environ.get("TRPO_BENCH_FAULT", "")
    for one in filter(None, spec.split(",")):
        f = one.split(":")
        if f[0] == stage and int(f[1]) == rank and (int(f[2]) if len(f) > 2 else 0) == attempt:
            return True
    return False


def agreed(dist, what, fn):
    """Run fn() on every rank, then agree (over gloo) that it succeeded everywhere: a failure on any one
    rank raises StageFault on all of them, so no rank enters the next collective alone."""
    err, out = None, None
    try:
        if _fault(what, dist.rank, 0):
            raise StageFault("injected fault (TRPO_BENCH_FAULT)")
        out = fn()
    except Exception as e:              # noqa: BLE001 -- agreed below, every rank moves on together
        err = "%s: %s" % (type(e).__name__, e)
    if dist.max(0.0 if err is None else 1.0) != 0.0:
        raise StageFault(err or "another rank failed at %s" % what)
    return out


def x_digest(x):
    import hashlib
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(x, np.float64).tobytes()).hexdigest()[:16]


def make_ctx_agreed(L, n_total, dist, device, comm, b, plan=None, tag=None):
    """The headline context at N > 1, set up stage by stage with the ranks agreeing (over gloo) after
    EVERY stage, so a failure on one rank alone never leaves the others in a mismatched collective:
      context   create this rank's context (its shard)
      bootstrap the RCCL unique id on rank 0 (then broadcast) / this rank's peer window handle (then
                all-gathered)
      attach    RCCL init bounded by COMM_TIMEOUT_MS / the peer attach (its 3-s exchange bound)
      verify    the library's self-check: one eager all-reduce of a rank-dependent vector, completion
                bounded, the exact sum checked bit for bit (trpo_ctx_comm_verify)
      solve     one graph-replayed sharded 10-iteration CG solve, completion bounded (trpo_ctx_wait)
      hash      x from every rank: identical bits (sha256 all-gathered)
    On a failure anywhere every rank aborts its collective (ncclCommAbort / the peer error flag), closes
    its context and moves to the next backend of `plan` (default: the requested one, the other, the
    requested one again); SystemExit when none passes.  tag: a secondary config's name, prefixed to the
    stage names of TRPO_BENCH_FAULT (`<tag>.<stage>`).
    Returns (ctx, theta, obs, backend, record) -- record = {"verify": ..., "fallback": [...] or None}."""
    pre = tag + "." if tag else ""
    import numpy as np
    import trpo_amd
    from trpo_amd import synth
    from trpo_amd.dist import shard_range
    other = "rccl" if comm == "peer" else "peer"
    failed = []
    for attempt, c in enumerate(plan or (comm, other, comm)):
        ctx, stage, err, attached, digest = None, None, None, False, None
        lib_fault = None
        for kind in ("comm-verify", "comm-hang"):
            if _fault(pre + kind, dist.rank, attempt):
                lib_fault = "%s:%d" % (kind.split("-")[1], dist.rank)
        saved = os.environ.pop("TRPO_COMM_FAULT", None)
        if lib_fault:
            os.environ["TRPO_COMM_FAULT"] = lib_fault
        t0 = time.perf_counter()
        try:
            for stage in STAGES:
                try:
                    if _fault(pre + stage, dist.rank, attempt):
                        raise StageFault("injected fault (TRPO_BENCH_FAULT)")
                    if stage == "context":
                        theta = synth.make_theta(L)
                        lo, hi = shard_range(n_total, dist.rank, dist.world)
                        obs = synth.make_obs(hi - lo, L[0], start=lo)
                        ctx = trpo_amd.Context(L, "lttl", theta, obs, np.ones(L[-1]), DAMPING, device=device)
                    elif stage == "bootstrap":
                        boot = ctx.peer_handle() if c == "peer" else (trpo_amd.unique_id() if dist.rank == 0 else None)
                    elif stage == "attach":
                        if c == "peer":
                            ctx.attach_peers(dist.rank, dist.world, boot)
                        else:
                            ctx.attach_comm(dist.rank, dist.world, boot, COMM_TIMEOUT_MS)
                        attached = True
                        info = ctx.comm_info()
                        if info["world"] != dist.world:
                            raise RuntimeError("%s communicator has %d ranks, expected %d"
                                               % (c, info["world"], dist.world))
                    elif stage == "verify":
                        ctx.comm_verify(COMM_TIMEOUT_MS)
                    elif stage == "solve":
                        ctx.upload_b(b)
                        ctx.enqueue_cg(CG_ITERS, 0.0)
                        ctx.wait(COMM_TIMEOUT_MS)
                        digest = x_digest(ctx.download_x())
                except Exception as e:          # noqa: BLE001 -- agreed below, every rank moves on together
                    err = "%s: %s" % (type(e).__name__, e)
                # agreement after the stage; the collective parts of bootstrap / hash run only if all agree
                if dist.max(0.0 if err is None else 1.0) != 0.0:
                    raise StageFault(err or "another rank failed at stage %s" % stage)
                if stage == "bootstrap":
                    boot = dist.allgather_bytes(boot) if c == "peer" else dist.bcast_bytes(boot)
                elif stage == "hash":
                    digests = dist.allgather_bytes(digest.encode())
                    if len(set(digests)) != 1 or _fault(pre + "hash-mismatch", dist.rank, attempt):
                        err = "x differs across ranks: %s" % sorted(set(d.decode() for d in digests))
                    if dist.max(0.0 if err is None else 1.0) != 0.0:
                        raise StageFault(err or "another rank saw differing x")
            record = {"verify": {"stages": list(STAGES), "eager_allreduce_exact": True, "x_sha256_16": digest,
                                 "x_identical_on_all_ranks": True, "attempt": attempt,
                                 "setup_s": time.perf_counter() - t0},
                      "fallback": ({"requested": comm, "failed": failed} if failed else None)}
            return ctx, theta, obs, c, record
        except StageFault as e:
            if ctx is not None:
                if attached:
                    ctx.comm_abort()
                ctx.close()
            failed.append({"attempt": attempt, "comm": c, "stage": stage, "rank": dist.rank, "error": str(e)})
            print("bench.py: rank %d: %s failed at stage %s (%s)" % (dist.rank, c, stage, e), file=sys.stderr)
        finally:
            os.environ.pop("TRPO_COMM_FAULT", None)
            if saved is not None:
                os.environ["TRPO_COMM_FAULT"] = saved
    raise SystemExit("bench.py: no collective passed setup and self-check: %s" % failed)


def time_steps(ctx, dist, steps, warmup, b, tag="headline"):
    """K timed solves after W warm-up ones, bracketed by barrier + completion on both sides; the wait
    is bounded at N > 1 (trpo_ctx_wait polls the stream, so it costs what a synchronize costs).  The
    barriers are agreements (`agreed`): a rank whose solves fail or time out makes every rank raise
    StageFault together instead of leaving the others in a mismatched collective."""
    wait = ctx.synchronize if dist.world == 1 else (lambda: ctx.wait(COMM_TIMEOUT_MS))

    def warm():
        ctx.upload_b(b)
        for _ in range(warmup):
            ctx.enqueue_cg(CG_ITERS, 0.0)
        wait()

    agreed(dist, tag + ".warmup", warm)               # the barrier in front of the timed region
    err = None
    t0 = time.perf_counter()
    try:
        if _fault(tag + ".timed", dist.rank, 0):
            raise StageFault("injected fault (TRPO_BENCH_FAULT)")
        for _ in range(steps):
            ctx.enqueue_cg(CG_ITERS, 0.0)
        wait()
    except Exception as e:              # noqa: BLE001 -- agreed below
        err = "%s: %s" % (type(e).__name__, e)
    t1 = time.perf_counter()
    agreed(dist, tag + ".timed-check", lambda: _raise(err))   # the barrier behind it
    return dist.max(t1 - t0)


def _raise(err):
    if err is not None:
        raise StageFault(err)


def _cpu_model():
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if "model name" in l][0]
    except Exception:
        return None


CPU_FLAGS = "gcc -O3 -march=x86-64-v3 -fopenmp (Makefile.cpuonly flags, portable -march)"


def _ref_run(mode, mf, df, nn, vec, extra, threads):
    """oracle/_ref/ref_driver_fast: the reference's own TRPO_FVP.c / TRPO_CG.c / TRPO_Update.c."""
    import oracle
    cmd = [oracle.REF_DRIVER_FAST, mode, mf, df, str(nn), ",".join(map(str, ARM)), "lttl", str(DAMPING), vec]
    cmd += extra + [str(threads)]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError("%s failed: %s" % (mode, p.stderr[-400:]))
    return json.loads(p.stderr.strip().splitlines()[-1])


def cpu_reference_cg(theta, obs_all, b):
    """The reference's CG (src/TRPO_CG.c) on all of obs_all, one host core: (headline record, x_ref).
    Falls back to the clean-room port where the reference build is absent (kind "port")."""
    import numpy as np
    import oracle
    from trpo_amd import synth
    n = obs_all.shape[0]
    if not os.path.exists(oracle.REF_DRIVER_FAST):
        r = oracle.cg(ARM, "lttl", theta, obs_all, np.ones(ARM[-1]), b, CG_ITERS, 0.0, DAMPING, threads=1)
        head = dict(value=CG_ITERS * n / r["seconds"], unit="FVP samples/s", cores=1, kind="port",
                    sample="one 10-iteration CG solve, armDOF_0, N=%d, ResidualTh=0, clean-room port, 1 thread" % n,
                    compute_s=r["seconds"], cpu_model=_cpu_model())
        return head, r["x"]
    with tempfile.TemporaryDirectory() as tmp:
        mf, df, bf, xf = (os.path.join(tmp, f) for f in ("m.txt", "d.txt", "b.txt", "x.txt"))
        synth.write_model_file(mf, theta)
        synth.write_data_file(df, obs_all, np.ones(ARM[-1]))
        synth.write_vector_file(bf, b)
        t1 = _ref_run("cg", mf, df, n, bf, [str(CG_ITERS), "0", xf], 1)
        x_ref = np.loadtxt(xf)
    head = dict(value=CG_ITERS * n / t1["compute_s"], unit="FVP samples/s", cores=1, kind="reference",
                sample="one 10-iteration CG solve (the reference's CG, src/TRPO_CG.c), armDOF_0, N=%d, "
                       "ResidualTh=0, NumThreads=1; compute seconds as CG returns them (file parsing excluded)" % n,
                compute_s=t1["compute_s"], wall_s_incl_file_parse=t1["wall_s"], build=CPU_FLAGS,
                cpu_model=_cpu_model())
    return head, x_ref


def cpu_rows(theta, obs_all, b, threads_all):
    """The reference itself (oracle/_ref/ref_driver_fast: src/TRPO_FVP.c + TRPO_CG.c compiled with the
    Makefile.cpuonly flags, -march=x86-64-v3) on this host: returns (headline, rows, x_ref)."""
    import numpy as np
    from trpo_amd import synth
    n = obs_all.shape[0]
    head, x_ref = cpu_reference_cg(theta, obs_all, b)
    rows = []
    if head["kind"] != "reference":
        return head, rows, x_ref
    rows.append(dict(config="C3 CG10 armDOF_0 N=%d" % n, threads=1, compute_s=head["compute_s"],
                     fvp_samples_per_s=head["value"]))
    with tempfile.TemporaryDirectory() as tmp:
        mf, bf = os.path.join(tmp, "m.txt"), os.path.join(tmp, "b.txt")
        synth.write_model_file(mf, theta)
        synth.write_vector_file(bf, b)
        # all host cores: the reference's per-neuron OpenMP fork/join anti-scales, so a
        # bounded sample -- the first 5 000 samples, one 10-iteration solve -- keeps this row to seconds
        ns = min(n, 5000)
        df5 = os.path.join(tmp, "d5.txt")
        synth.write_data_file(df5, obs_all[:ns], np.ones(ARM[-1]))
        ta = _ref_run("time", mf, df5, ns, bf, [str(CG_ITERS), "0"], threads_all)
        rows.append(dict(config="C3 CG10 armDOF_0 N=%d (bounded sample of the N=%d workload)" % (ns, n),
                         threads=threads_all, compute_s=ta["compute_s"],
                         fvp_samples_per_s=CG_ITERS * ns / ta["compute_s"]))
    # C1: the reference's own fixtures (ArmTest{Model,Data,FVP,CG}.txt, N=3150), 1 thread and all cores
    g = os.path.join(ROOT, "tests", "golden")
    mfix, dfix = os.path.join(g, "ArmTestModel.txt"), os.path.join(g, "ArmTestData.txt")
    with tempfile.TemporaryDirectory() as tmp:
        vf, bf2, of = (os.path.join(tmp, f) for f in ("v.txt", "b.txt", "o.txt"))
        synth.write_vector_file(vf, np.loadtxt(os.path.join(g, "ArmTestFVP.txt"))[:, 0])
        synth.write_vector_file(bf2, np.loadtxt(os.path.join(g, "ArmTestCG.txt"))[:, 0])
        for th in (1, threads_all):
            tf = _ref_run("fvp", mfix, dfix, 3150, vf, [of], th)
            tc = _ref_run("time", mfix, dfix, 3150, bf2, ["10", "1e-10"], th)
            rows.append(dict(config="C1 fixture FVPFast N=3150", threads=th, compute_s=tf["compute_s"],
                             fvp_samples_per_s=3150 / tf["compute_s"]))
            rows.append(dict(config="C1 fixture CG(10, 1e-10) N=3150 (8 FVPs)", threads=th,
                             compute_s=tc["compute_s"], fvp_samples_per_s=8 * 3150 / tc["compute_s"]))
    return head, rows, x_ref


def bench_update(device, L=ARM, n=N_TOTAL, reps=20, cpu_ref=True):
    """One full TRPO policy update (src/TRPO_Update.c: policy gradient, 10-iteration CG, FVP(x),
    line search) on a synthetic rollout of policy L, host-visible wall time per update (includes the
    host round trips of x / z / the line-search scalars); CPU reference TRPO_Update timed beside it."""
    import numpy as np
    import oracle
    import trpo_amd
    from trpo_amd import synth
    theta = synth.make_theta(L)
    obs = synth.make_obs(n, L[0])
    std = np.ones(L[-1])
    mean, action, adv = synth.make_rollout(L, "lttl", theta, obs, std)
    ctx = trpo_amd.Context(L, "lttl", theta, obs, std, DAMPING, device=device)
    ctx.set_rollout(mean, action, adv)
    for _ in range(3):      # warm-up: first-call allocations, CG graph capture
        r = ctx.update()
    # the stall guard: an update whose solve it re-ran in fp64 says so (trpo_ctx_cg_status,
    # read by update()); counted over the timed updates so the row shows whether its time includes any
    reruns = 0
    t0 = time.perf_counter()
    for _ in range(reps):
        r = ctx.update()
        reruns += bool(r["fp64_rerun"])
    wall = (time.perf_counter() - t0) / reps
    ctx.close()
    out = {"update_ms": 1e3 * wall, "accepted": r["accepted"], "cg_iters": int(r["cg_iters"]), "samples": n,
           "fp64_reruns": reruns, "updates_timed": reps, "ritz_residual": r["ritz_residual"],
           "what": "policy gradient (fp32 tile kernel, fp64 sums) + CG(10, 1e-10) + FVP(x) + fp64 line search"}
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
    import numpy as np
    import oracle
    import trpo_amd
    from trpo_amd import synth
    L = [16, 16, 16, 1]
    x, obs, tgt = synth.make_baseline_problem(L, num_ep, ep_len)
    from scipy.optimize import fmin_l_bfgs_b
    with trpo_amd.Baseline(L, "lttl", device=device) as b:
        b.set_data(obs, tgt, num_ep, ep_len)
        b.evaluate(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            f, g = b.evaluate(x)
        dev = (time.perf_counter() - t0) / reps
        # a baseline fit under a second driver, scipy's L-BFGS-B (at most 25 iterations) on the device
        # objective; the fit a trainer runs -- the caller's liblbfgs -- is caller_lbfgs_fit below
        fits = []
        for _ in range(3):
            t0 = time.perf_counter()
            xd, fd, info = fmin_l_bfgs_b(lambda v: b.evaluate(v), x, maxiter=25)
            fits.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    fo, go, _ = oracle.baseline_evaluate(L, "lttl", x, obs, tgt, num_ep, ep_len)
    cpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    xo, fo_fit, info_o = fmin_l_bfgs_b(lambda v: oracle.baseline_evaluate(L, "lttl", v, obs, tgt, num_ep, ep_len)[:2],
                                       x, maxiter=25)
    cpu_fit = time.perf_counter() - t0
    return {"evaluate_us": 1e6 * dev, "cpu_port_evaluate_us_1core": 1e6 * cpu, "samples": num_ep * ep_len,
            "grad_relL2_vs_cpu": float(np.linalg.norm(g - go) / np.linalg.norm(go)),
            "what": "host-visible wall per L-BFGS callback incl. x upload and g/f download",
            "scipy_lbfgsb_fit25_ms": 1e3 * sorted(fits)[1], "scipy_lbfgsb_fit25_evals": int(info["funcalls"]),
            "cpu_port_scipy_lbfgsb_fit25_ms_1core": 1e3 * cpu_fit,
            "scipy_fit_x_relL2_vs_cpu_fit": float(np.linalg.norm(xd - xo) / np.linalg.norm(xo)),
            "caller_liblbfgs_fit": caller_lbfgs_fit(device)}


def caller_lbfgs_fit(device, reps=5):
    """The baseline fit with the CALLER's optimiser (liblbfgs 1.10, src/lbfgs.c, as
    src/TRPO_Lightweight.c:676 calls it) on the device evaluate, and on the reference's CPU evaluate
    beside it: tests/lbfgs_fit_child.py (test infrastructure, like the CPU baseline) in a child process,
    which also checks that both fits end at the same point.  None where oracle/_ref is not built."""
    child = os.path.join(ROOT, "tests", "lbfgs_fit_child.py")
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_lbfgs.so")):
        return {"error": "oracle/_ref/libref_lbfgs.so not built (make -C oracle ref)"}
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", str(device)))
    p = subprocess.run([sys.executable, child, str(reps)], capture_output=True, text=True, timeout=180, env=env)
    if p.returncode != 0:
        return {"error": "lbfgs_fit_child exited %d: %s" % (p.returncode, p.stderr[-400:])}
    return json.loads(p.stdout.strip().splitlines()[-1])


def c5_iteration(u, bl):
    """One training iteration's learning step: TRPO_Update + the baseline fit by the caller's liblbfgs
    (the trainer's own optimiser; scipy's L-BFGS-B fit is reported in the baseline row only)."""
    fit = bl.get("caller_liblbfgs_fit") or {}
    if "device_evaluate_fit_ms" not in fit:
        return {"error": "no caller-liblbfgs fit timing: %s" % fit.get("error")}
    cpu_u = u.get("cpu_reference_compute_s_1core")
    return {"device_ms": u["update_ms"] + fit["device_evaluate_fit_ms"], "fp64_reruns": u.get("fp64_reruns"),
            "cpu_reference_ms_1core": (1e3 * cpu_u + fit["reference_cpu_evaluate_fit_ms_1core"]
                                       if cpu_u is not None else None),
            "what": "TRPO_Update (N=50000, device) + the value-baseline fit by the caller's liblbfgs 1.10 "
                    "(max 25 iterations, 20x150 batch) on the device evaluate; CPU: the reference's "
                    "TRPO_Update + the same liblbfgs on the reference's evaluate, 1 core; rollouts not included"}


def _guarded(extra, key, fn, lock=None):
    """extra[key] = fn(), or {"error": ...} if it raised: a secondary config never ends the run."""
    try:
        val = fn()
    except (Exception, SystemExit) as e:        # noqa: BLE001 -- recorded; the headline line still prints
        val = {"error": "%s: %s" % (type(e).__name__, e)}
    if lock is not None:
        with lock:
            extra[key] = val
    else:
        extra[key] = val
    return val


def extras_single(device, dist, reps, lock=None):
    """Secondary configs at N=1 (SURVEY §8d C2, C3 for the 2x64 MLP, the fp64 mode, C5), each guarded:
    a failing one is recorded as {"error": ...} and the rest still run."""
    from trpo_amd import synth
    extra = {}
    L2 = [15, 64, 64, 3]

    def c2():
        c2res = {}
        for tag, env in (("", None), ("_recompute", "0")):
            # C2: repeated FVP calls on one context reuse the forward-activation cache (theta unchanged);
            # a first call after set_theta recomputes the forward pass -- timed too (TRPO_YCACHE=0)
            if env is not None:
                os.environ["TRPO_YCACHE"] = env
            try:
                ctx, _, _ = make_ctx(L2, 4096, dist, device)
            finally:
                os.environ.pop("TRPO_YCACHE", None)
            try:
                ctx.upload_v(synth.make_v(num_params(L2)))
                k2 = ctx.time_ms(0, reps)
                f2 = ctx.time_ms(1, reps)
            finally:
                ctx.close()
            fl = flops_per_sample_cached(L2) if env is None else flops_per_sample(L2)
            c2res.update({"fvp_ms" + tag: f2, "kernel_ms" + tag: k2, "fvp_samples_per_s" + tag: 4096 / (f2 * 1e-3),
                          "kernel_tflops" + tag: fl * 4096 / (k2 * 1e-3) / 1e12})
        return c2res

    def c3(L, prec):
        ctx, _, _ = make_ctx(L, N_TOTAL, dist, device, precision=prec)
        try:
            K3 = 100                                 # 100 solves after 10 (as the headline: a steady-state rate)
            t3 = time_steps(ctx, dist, K3, 10, synth.make_b(num_params(L)), tag="c3")
            if prec is None and ctx.kernel_name.endswith(" coop"):
                # fp32 cooperative path: the CG step runs over slices (cg_dots / cg_axpy), so the
                # per-iteration tile kernel is the standalone cached-forward FVP kernel (MODE 3)
                ctx.upload_v(synth.make_v(num_params(L)))
                k3 = ctx.time_ms(0, 50)
                kdesc = " (FVP kernel, cached forward; per iteration + slab reduce with the CG dots (one rank) + cg_axpy)"
            else:
                k3 = ctx.time_ms(3, 10, CG_ITERS)
                kdesc = " (CG-iteration kernel, cached forward)"
            name = ctx.kernel_name
        finally:
            ctx.close()
        return {"cg_wall_ms": 1e3 * t3 / K3, "fvp_samples_per_s": CG_ITERS * N_TOTAL / (t3 / K3),
                "cg_iter_kernel_ms": k3, "kernel": name + kdesc,
                "kernel_tflops": flops_per_sample_cached(L) * N_TOTAL / (k3 * 1e-3) / 1e12,
                "kernel_tflops_recompute_equiv": flops_per_sample(L) * N_TOTAL / (k3 * 1e-3) / 1e12,
                "peak_tflops": PEAK_FP64_TFLOPS if prec == "fp64" else PEAK_FP32_TFLOPS}

    _guarded(extra, "C2_fvp_2x64_N4096", c2, lock)
    for key, L, prec in (("C3_cg10_2x64_N50000", L2, None),
                         ("C3_cg10_armDOF_0_N50000_fp64", ARM, "fp64"), ("C3_cg10_2x64_N50000_fp64", L2, "fp64")):
        _guarded(extra, key, lambda: c3(L, prec), lock)
    u = _guarded(extra, "C5_update_armDOF_0_N50000", lambda: bench_update(device), lock)
    _guarded(extra, "C5_update_2x64_N50000", lambda: bench_update(device, L=L2, cpu_ref=False), lock)
    bl = _guarded(extra, "C5_baseline_evaluate_N3000", lambda: bench_baseline(device), lock)
    if "update_ms" in u and "evaluate_us" in bl:
        _guarded(extra, "C5_iteration_armDOF_0", lambda: c5_iteration(u, bl), lock)
    return extra


def extras_multi(device, dist, b, x_ref, comm="rccl", out=None, lock=None):
    """N > 1, measured AFTER the headline: the same sharded solve with the other collectives in place of
    the headline's (A/B on the driver's multi-GPU node): RCCL or the peer-window exchange (tagged granules,
    the default form since round 5), and the peer exchange in its flag hand-off form (TRPO_PEER_PROTO=1,
    the default through round 4: one more xGMI trip per exchange); and one sharded TRPO update (config C5)
    under the headline's collective.
    Every one goes through run_secondary (agreed setup, agreed steps, abort + close in `finally`);
    results go into `out` as they complete (under `lock`: the watchdog may serialise it meanwhile)."""
    out = {} if out is None else out
    other = "rccl" if comm == "peer" else "peer"
    runs = (("C4_%s_exchange" % other, "other", other, _solve_body(dist, b, x_ref), None),
            ("C4_peer_flag_exchange", "flag", "peer", _solve_body(dist, b, x_ref), {"TRPO_PEER_PROTO": "1"}),
            ("C5_update_armDOF_0_N50000", "update", comm, _update_body(dist), None))
    for key, tag, backend, body, env in runs:
        if dist.broken:                          # a gloo bound expired: the ranks may be out of step
            out[key] = {"error": "skipped: an earlier secondary's gloo collective failed"}
            continue
        _guarded(out, key, lambda: run_secondary(dist, device, tag, backend, N_TOTAL, b, body, env=env), lock)
    return out


def run_secondary(dist, device, tag, backend, n, b, body, env=None):
    """One secondary config at N > 1: its context through make_ctx_agreed (plan = this backend only:
    per-stage agreement, the collective's self-check, the x-hash), then body(ctx, record) whose steps
    are agreed too; the context is closed in `finally`, its collective aborted first when anything
    failed.  Collectives run on the secondary gloo group (shorter bound).  Faults: TRPO_BENCH_FAULT
    stages `<tag>.<stage>` (make_ctx_agreed), `<tag>.body` (any rank raising inside the body), and
    `<tag>.hang` (a rank blocking forever inside the body: only the watchdog ends that)."""
    ctx, ok = None, False
    old = {k: os.environ.get(k) for k in (env or {})}
    with dist.secondary():
        try:
            os.environ.update(env or {})
            try:
                ctx, _, _, _, rec = make_ctx_agreed(ARM, n, dist, device, backend, b, plan=(backend,), tag=tag)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            if _fault(tag + ".hang", dist.rank, 0):
                while True:
                    time.sleep(3600)
            agreed(dist, tag + ".body", lambda: None)
            res = body(ctx, rec, tag)
            ok = True
            return res
        finally:
            if ctx is not None:
                if not ok:
                    ctx.comm_abort()
                ctx.close()


def _solve_body(dist, b, x_ref):
    """The headline's sharded solve on this context, timed like the headline (50 after 5)."""
    import numpy as np

    def body(ctx, rec, tag):
        t = time_steps(ctx, dist, 50, 5, b, tag=tag)
        x = agreed(dist, tag + ".result", ctx.download_x)
        return {"ms_per_step": 1e3 * t / 50, "fvp_samples_per_s": CG_ITERS * N_TOTAL / (t / 50),
                "backend": ctx.comm_backend, "n_gpus": dist.world, "verify": rec["verify"],
                "x_relL2_vs_headline": float(np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref))}
    return body


def _update_body(dist):
    """C5: one TRPO policy update over the sharded rollout (policy-gradient / FVP / surrogate all-reduces)."""
    import numpy as np
    from trpo_amd import synth
    from trpo_amd.dist import shard_range

    def body(ctx, rec, tag):
        theta = synth.make_theta(ARM)
        obs_all = synth.make_obs(N_TOTAL, ARM[0])
        mean, action, adv = synth.make_rollout(ARM, "lttl", theta, obs_all, np.ones(ARM[-1]))
        lo, hi = shard_range(N_TOTAL, dist.rank, dist.world)
        agreed(dist, tag + ".rollout", lambda: ctx.set_rollout(mean[lo:hi], action[lo:hi], adv[lo:hi]))
        r = None
        for _ in range(3):
            r = agreed(dist, tag + ".warmup-update", ctx.update)
        reruns = 0
        t0 = time.perf_counter()
        for _ in range(20):
            r = agreed(dist, tag + ".update", ctx.update)
            reruns += bool(r["fp64_rerun"])
        wall = dist.max((time.perf_counter() - t0) / 20)
        return {"update_ms": 1e3 * wall, "accepted": r["accepted"], "cg_iters": int(r["cg_iters"]),
                "fp64_reruns": reruns, "updates_timed": 20,
                "samples": N_TOTAL, "n_gpus": dist.world, "comm": ctx.comm_backend,
                "what": "sharded rollout; all-reduces of the policy gradient, every FVP and the surrogate sums; "
                        "host-visible wall per update (max over ranks; each update followed by a cross-rank "
                        "agreement, as a trainer's step would be)"}
    return body


def sweep(device, dist, steps=10, comm="rccl", out=None, lock=None):
    """C4's N sweep: the same sharded 10-iteration solve at larger batches (whole-job rates).  At one
    rank each row also carries the CG-iteration kernel's roofline at that N (HIP events, same units as
    the headline `roofline`): the 50k headline is latency-bound, these rows show the kernel's
    throughput regime.  At N > 1 ranks a weak-scaling row (50k samples per rank) is added, and every
    row goes through run_secondary.  Each row is guarded: one that fails is recorded as an error."""
    from trpo_amd import synth
    out = {} if out is None else out
    b = synth.make_b(num_params(ARM))
    ns = list(SWEEP_N) + ([N_TOTAL * dist.world] if dist.world > 1 else [])

    def row_multi(n):
        def body(ctx, rec, tag):
            t = time_steps(ctx, dist, steps, 2, b, tag=tag)
            row = {"ms_per_step": 1e3 * t / steps, "fvp_samples_per_s": CG_ITERS * n / (t / steps),
                   "n_gpus": dist.world, "backend": ctx.comm_backend}
            if n == N_TOTAL * dist.world:
                row["scaling"] = "weak (50000 samples per rank)"
            return row
        return run_secondary(dist, device, "sweep%d" % n, comm, n, b, body)

    def row_single(n):
        ctx, _, _ = make_ctx(ARM, n, dist, device)
        try:
            t = time_steps(ctx, dist, steps, 2, b, tag="sweep%d" % n)
            row = {"ms_per_step": 1e3 * t / steps, "fvp_samples_per_s": CG_ITERS * n / (t / steps),
                   "n_gpus": dist.world}
            k3 = ctx.time_ms(3, 5, CG_ITERS)
            bytes_alg = bytes_per_fvp_cached(ARM, ctx.n) + bytes_cg_step(ARM)
            row.update({"cg_iter_kernel_ms": k3, "alg_bytes_per_launch": bytes_alg,
                        "hbm_frac_algorithmic": bytes_alg / (k3 * 1e-3) / 1e9 / PEAK_HBM_GBS,
                        "fp32_frac": flops_per_sample_cached(ARM) * ctx.n / (k3 * 1e-3) / 1e12 / PEAK_FP32_TFLOPS})
            return row
        finally:
            ctx.close()

    for n in ns:
        _guarded(out, "cg10_armDOF_0_N%d" % n, (lambda n=n: row_multi(n)) if dist.world > 1 else (lambda n=n: row_single(n)),
                 lock)
        if dist.broken:
            break
    return out


def latest_traffic_json():
    """profiles/rNN_cgiter_traffic.json of the highest round present (None if there is none)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_cgiter_traffic.json")))
    return files[-1] if files else None


PMC_KERNEL = "fvp_mlp3_kernel<1, 1, 1, 1, 5, 3"       # the CG-iteration kernel (MODE 3, every QB variant)
N_SIMDS = 1024                                        # 256 CUs x 4 SIMDs (MI355X)
N_XCDS = 8


def pmc_child(device):
    """--pmc-child: the headline workload (armDOF_0, the seeded batch of TRPO_PMC_N samples -- 50k unless
    set --, b) for a few CG solves, run by pmc_pass under rocprofv3's counter collection; nothing printed
    on stdout."""
    from trpo_amd import synth
    n = int(os.environ.get("TRPO_PMC_N", N_TOTAL))
    ctx, _, _ = make_ctx(ARM, n, _OneRank(), device)
    ctx.upload_b(synth.make_b(num_params(ARM)))
    for _ in range(5 if n <= 500_000 else 2):
        ctx.enqueue_cg(CG_ITERS, 0.0)
    ctx.synchronize()
    ctx.close()


class _OneRank:
    rank, world, local_rank = 0, 1, 0


def pmc_median(path, counter, kernel=PMC_KERNEL):
    """(median over dispatches of `kernel` of the counter's per-dispatch total, dispatch count) from a
    rocprofv3 counter_collection.csv (one row per counter instance), or None if no dispatch matched."""
    import csv
    import statistics
    per = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return (statistics.median(per.values()), len(per)) if per else None


def pmc_pass(device, counters, n=N_TOTAL, limit=90):
    """One rocprofv3 counter pass (its own child process of this script, --pmc-child, on the headline
    workload at n samples, under its own hard time limit): {counter: (median per dispatch of the
    CG-iteration kernel, dispatches)}, or (None, reason).  The counters of one pass must fit the
    hardware's slots (MI355X_MICROARCH.md: SQ 8, TCC 4 with FETCH_SIZE = 3 and WRITE_SIZE = 2, GRBM 2)."""
    import shutil
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if not prof:
        return None, "rocprofv3 not found"
    with tempfile.TemporaryDirectory(prefix="trpo_pmc_") as tmp:
        cmd = ["timeout", "-s", "KILL", str(limit), prof, "--pmc", *counters, "--output-format", "csv", "-d", tmp,
               "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--pmc-child"]
        env = dict(os.environ, TRPO_BENCH_DEVICE=str(device), TRPO_PMC_N=str(n))
        try:
            r = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                               timeout=limit + 30)
        except (OSError, subprocess.SubprocessError) as e:      # no `timeout` binary, a stuck child, ...
            return None, "rocprofv3 --pmc %s: %s: %s" % (" ".join(counters), type(e).__name__, e)
        if r.returncode != 0:
            return None, "rocprofv3 --pmc %s exited %d: %s" % (" ".join(counters), r.returncode, r.stderr[-300:].strip())
        files = [os.path.join(dp, fn) for dp, _, fns in os.walk(tmp) for fn in fns
                 if fn.endswith("counter_collection.csv")]
        if not files:
            return None, "no counter_collection.csv from the %s pass" % " ".join(counters)
        med = {}
        for c in counters:
            m = pmc_median(files[0], c)
            if m is None:
                return None, "no %s dispatches of %s" % (c, PMC_KERNEL)
            med[c] = m
        return med, None


def measure_traffic(device):
    """roofline.traffic measured in this run (N = 1): two counter passes (pmc_pass) as MI355X_MICROARCH.md's
    HBM section prescribes (FETCH_SIZE, then WRITE_SIZE, each in its own run, kernel dispatches serialised
    by the profiler); per-launch HBM bytes of the CG-iteration kernel = 2 x median FETCH_SIZE (the gfx950
    wide-read undercount) + median WRITE_SIZE, KiB -> bytes.  The parent is idle meanwhile (after its
    timed region).  Returns (bytes, source) or (None, reason)."""
    med = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        m, why = pmc_pass(device, (counter,))
        if m is None:
            return None, why
        med.update(m)
    fetch = 2.0 * med["FETCH_SIZE"][0] * 1024
    write = med["WRITE_SIZE"][0] * 1024
    return fetch + write, {"measured": "in this run", "fetch_bytes": fetch, "write_bytes": write,
                           "dispatches": [med["FETCH_SIZE"][1], med["WRITE_SIZE"][1]],
                           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount) + WRITE_SIZE"}


MFMA_COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
                 "GRBM_GUI_ACTIVE")


PEAK_CLOCK_GHZ = 2.4                                  # MI355X peak engine clock (MI355X_MICROARCH.md)


def mfma_from_counters(med, kernel_ms=None):
    """MFMA utilisation of the CG-iteration kernel from one counter pass (medians per dispatch):
    SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over every SIMD) / (1 024 SIMDs x GRBM_GUI_ACTIVE / 8), the
    dispatch's GPU-active cycles per XCD (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is the sum over the 8 XCDs,
    and reads high on dispatches shorter than ~0.3 ms, so at 50k this is a lower bound)."""
    busy, grbm = med["SQ_VALU_MFMA_BUSY_CYCLES"][0], med["GRBM_GUI_ACTIVE"][0]
    grbm_frac = busy / (N_SIMDS * grbm / N_XCDS) if grbm > 0 else None
    out = {"mfma_busy_frac": grbm_frac, "mfma_busy_frac_grbm": grbm_frac,
           "mfma_busy_denominator": "1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs (the dispatch's GPU-active cycles, "
                                    "per dispatch of the CG-iteration kernel, medians)",
           "counters": {c: m[0] for c, m in med.items()}, "dispatches": med["GRBM_GUI_ACTIVE"][1]}
    if kernel_ms:
        # the same busy cycles over the kernel's HIP-event time at the peak clock (the clock under load is at
        # most 2.4 GHz, so a lower bound).  GRBM_GUI_ACTIVE reads high on dispatches shorter than ~0.3 ms
        # (MI355X_MICROARCH.md), which dilutes the GRBM form at 50k (0.075 there against 0.14 here, round 6);
        # at 4M the two agree (0.54 / 0.50).  So this form is the line's mfma_busy_frac when the event time is
        # known.
        out["mfma_busy_frac_at_peak_clock"] = busy / (N_SIMDS * kernel_ms * 1e-3 * PEAK_CLOCK_GHZ * 1e9)
        out["mfma_busy_frac"] = out["mfma_busy_frac_at_peak_clock"]
        out["mfma_busy_denominator"] = ("1024 SIMDs x the kernel's HIP-event time x 2.4 GHz (peak clock: a lower "
                                        "bound); mfma_busy_frac_grbm: over GRBM_GUI_ACTIVE / 8 XCDs instead")
        out["kernel_ms_events"] = kernel_ms
    if med.get("SQ_WAVE_CYCLES", (0,))[0] > 0:
        out["wait_inst_any_frac"] = med["SQ_WAIT_INST_ANY"][0] / med["SQ_WAVE_CYCLES"][0]
    return out


def measure_mfma(device, n=N_TOTAL, kernel_ms=None):
    """roofline.mfma_busy_frac: one counter pass (5 SQ + 1 GRBM slots) at n samples;
    kernel_ms: the kernel's HIP-event time from this run, for the peak-clock form."""
    med, why = pmc_pass(device, MFMA_COUNTERS, n=n, limit=150 if n > 500_000 else 90)
    if med is None:
        return {"error": why}
    return dict(mfma_from_counters(med, kernel_ms), measured="in this run", samples=n)


def main():
    args = parse_args()
    if args.pmc_child:
        sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
        pmc_child(int(os.environ.get("TRPO_BENCH_DEVICE", "0")))
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd"), os.path.join(ROOT, "oracle")]
    import numpy as np
    from trpo_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:                       # before any rendezvous or device use
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    # stdout carries exactly one line (rank 0's JSON): what RCCL, gloo and the runtimes print to fd 1
    # (RCCL's version banner, gloo's connection notice) goes to stderr from here on
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import trpo_amd
    trpo_amd.lib()                               # the system ROCm runtime before torch's (Dist)
    dist = Dist()
    device = int(os.environ.get("TRPO_BENCH_DEVICE", dist.local_rank))   # override: testing only

    P = num_params(ARM)
    b = synth.make_b(P)
    emitter = Emitter(json_fd, dist.rank)
    if dist.world > 1:
        ctx, theta, obs_local, args.comm, setup = make_ctx_agreed(ARM, N_TOTAL, dist, device, args.comm, b)
    else:
        (ctx, theta, obs_local), setup = make_ctx(ARM, N_TOTAL, dist, device), {"verify": None, "fallback": None}
    comm = ctx.comm_info()

    # Order of the measurements.  N = 1: the secondary configs first, then the dominant kernel's event
    # timing, then the headline's timed region LAST.  A 20-solve region (2 ms) right after a cold start
    # caught the GPU before its clock had settled: per solve 0.1035 ms at K=20/W=5 against 0.0982 ms at
    # K=500/W=50 on one box, 0.1020 ms with the 2 ms of kernel timing in front (profiles/r04_warm_ab.log);
    # measured last, the headline sees the steady state a trainer's repeated updates run in.  N > 1: the
    # headline's timed region comes right after its agreed setup, and the secondary configs (each with
    # its own agreed setup, shorter gloo bound, abort + close on failure) only after it, under a
    # watchdog that prints the headline line by the deadline whatever a secondary does.
    # The timed region itself is the same in both: W untimed solves, then exactly K full solves between
    # barriers.
    extra = {} if not args.no_extra else None
    if extra is not None and dist.world == 1:
        extra.update(extras_single(device, dist, 200))
        extra["C4_sweep"] = sweep(device, dist, comm=args.comm)

    # the dominant kernel: the fused CG-iteration kernel (9 of the 10 launches of a solve), timed alone
    # with HIP events on the context's stream, averaged over the iterations K_1..K_9 of a solve
    reps = 20
    k3 = ctx.time_ms(3, reps, CG_ITERS)
    ctx.upload_v(synth.make_v(P))
    k2 = ctx.time_ms(0, 200)                     # the standalone FVP kernel (no CG step), secondary

    t = time_steps(ctx, dist, args.steps, args.warmup, b)
    ms_per_step = 1e3 * t / args.steps
    value = CG_ITERS * N_TOTAL / (t / args.steps)
    x = ctx.download_x()

    n_local = ctx.n
    flops = flops_per_sample_cached(ARM) * n_local
    bytes_alg = bytes_per_fvp_cached(ARM, n_local) + bytes_cg_step(ARM)
    achieved_gbs = bytes_alg / (k3 * 1e-3) / 1e9
    achieved_tflops = flops / (k3 * 1e-3) / 1e12
    hbm_bound = bytes_alg / (PEAK_HBM_GBS * 1e9) >= flops / (PEAK_FP32_TFLOPS * 1e12)

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
                   "samples": N_TOTAL, "samples_per_rank": n_local, "cg_iters": CG_ITERS, "residual_th": 0.0,
                   "damping": DAMPING,
                   "parallelism": "dp%d (contiguous sample shards, %s all-reduce per FVP)"
                                  % (dist.world, "RCCL" if args.comm == "rccl" else "peer-window"),
                   "cg_scalars": "fp64", "fvp_kernel": ctx.kernel_name, "geometry": ctx.geometry},
        "comm": {"backend": comm["backend"], "ranks": comm["world"],
                 "replicas_per_fvp": comm["replicas"], "hip_runtime": trpo_amd.runtime_path(),
                 "verify": setup["verify"], "fallback": setup["fallback"]},
        "cg_wall_ms": ms_per_step,
        "roofline": {"bound": "hbm" if hbm_bound else "mfma",
                     "achieved": achieved_gbs if hbm_bound else achieved_tflops,
                     "peak": PEAK_HBM_GBS if hbm_bound else PEAK_FP32_TFLOPS,
                     "unit": "GB/s" if hbm_bound else "TFLOP/s",
                     "frac": achieved_gbs / PEAK_HBM_GBS if hbm_bound else achieved_tflops / PEAK_FP32_TFLOPS,
                     "traffic": None, "traffic_source": None,
                     "kernel": "fvp_mlp3_kernel MODE 3 (CG-iteration kernel: fp64 CG step + cached-forward FVP)",
                     "kernel_ms": k3, "flops_per_launch": flops, "alg_bytes_per_launch": bytes_alg,
                     "fp32_tflops": achieved_tflops, "fp32_frac": achieved_tflops / PEAK_FP32_TFLOPS,
                     "hbm_gbs_algorithmic": achieved_gbs, "hbm_frac_algorithmic": achieved_gbs / PEAK_HBM_GBS,
                     "full_recompute_equiv_tflops": flops_per_sample(ARM) * n_local / (k3 * 1e-3) / 1e12,
                     "secondary_fvp_kernel_mode2_ms": k2},
    }
    if extra is not None:
        result["extra"] = extra

    if dist.world > 1 and not args.no_cpu_baseline:
        # the sharded solve's step against the reference's CG over the WHOLE batch (rank 0 regenerates
        # the seeded 50k observations; the other ranks wait at the agreement)
        def parity():
            if dist.rank == 0:
                obs_all = synth.make_obs(N_TOTAL, ARM[0])
                _, x_ref = cpu_reference_cg(theta, obs_all, b)
                rel = float(np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref))
                result["parity"] = {"cg_step_relL2_vs_cpu": rel, "tolerance": 1e-4,
                                    "what": "x of the %d-rank sharded solve vs the reference CG on all %d samples"
                                            % (dist.world, N_TOTAL)}
        try:
            agreed(dist, "parity", parity)
        except Exception as e:                  # noqa: BLE001 -- recorded; the line still prints
            result["parity"] = {"error": "%s: %s" % (type(e).__name__, e)}

    # the headline is measured: from here the line is printed by the deadline whatever follows does
    emitter.arm(result)

    if extra is not None and dist.world > 1:
        extras_multi(device, dist, b, x, args.comm, out=extra, lock=emitter.lock)
        if not dist.broken:
            with emitter.lock:
                extra["C4_sweep"] = {}
            sweep(device, dist, comm=args.comm, out=extra["C4_sweep"], lock=emitter.lock)

    if dist.world == 1:
        traffic, tsrc = None, None
        if not args.no_pmc and os.environ.get("TRPO_TRAFFIC_JSON") is None:
            traffic, tsrc = measure_traffic(device)
            mf = measure_mfma(device, kernel_ms=k3)
            with emitter.lock:
                result["roofline"]["mfma_busy_frac"] = mf.get("mfma_busy_frac")
                result["roofline"]["mfma"] = mf
            row4m = (extra or {}).get("C4_sweep", {}).get("cg10_armDOF_0_N4000000")
            if isinstance(row4m, dict) and "error" not in row4m:
                mf4 = measure_mfma(device, 4_000_000, kernel_ms=row4m.get("cg_iter_kernel_ms"))
                with emitter.lock:
                    row4m["mfma_busy_frac"] = mf4.get("mfma_busy_frac")
                    row4m["mfma"] = mf4
        if traffic is None:
            # fallback: HBM bytes per launch of this kernel at this workload from the newest committed
            # rocprofv3 PMC passes (tools/profile_round.sh: FETCH_SIZE x2 + WRITE_SIZE, separate passes)
            why = tsrc
            tpath = os.environ.get("TRPO_TRAFFIC_JSON") or latest_traffic_json()
            if tpath and os.path.exists(tpath):
                traffic = json.load(open(tpath))["traffic_bytes"]
                tsrc = {"measured": "profile file " + os.path.relpath(tpath, ROOT), "why_not_live": why}
        with emitter.lock:
            result["roofline"]["traffic"], result["roofline"]["traffic_source"] = traffic, tsrc

    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        threads_all = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        head, rows, x_ref = cpu_rows(theta, obs_local, b, threads_all)
        head["rows"] = rows
        rel = float(np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref))
        with emitter.lock:
            result["cpu_baseline"] = head
            result["parity"] = {"cg_step_relL2_vs_cpu": rel, "tolerance": 1e-4}

    if dist.world > 1 and not dist.broken:
        try:
            dist.barrier()
        except Exception:                       # noqa: BLE001 -- the line still prints
            pass
    if dist.broken:
        ctx.comm_abort()                        # a rank may be stuck: do not wait on the collective
        # the exit status stays 0 (the headline was measured and verified before any secondary ran); the
        # line itself says that a secondary's gloo collective failed, as do the secondaries'
        # own error records
        with emitter.lock:
            result["dist_broken"] = True
    ctx.close()
    emitter.emit(result)
    if dist.broken:
        # a gloo collective timed out: tearing its process group down can abort in its destructor
        # (std::terminate), so leave without interpreter teardown once the line is out
        sys.stderr.flush()
        os._exit(0)
    dist.close()


class Emitter:
    """Prints rank 0's one JSON line exactly once: from the main thread at the end, or -- once the
    headline has been measured (arm) -- from a watchdog thread at the deadline, which then ends the
    process (os._exit(0), on every rank) so that no secondary config, however it fails, can cost the
    driver its headline line.  Deadline: TRPO_BENCH_DEADLINE_S (default 420) after the process started,
    and at least TRPO_BENCH_GRACE_S (default 60) after the headline.  `lock` guards the result dict
    against the watchdog's serialisation while the main thread adds secondary results."""

    def __init__(self, fd, rank):
        import threading
        self.fd, self.rank, self.lock, self.done = fd, rank, threading.RLock(), False
        self.t_start = time.monotonic()

    def emit(self, result, note=None):
        with self.lock:
            if self.done:
                return False
            self.done = True
            if note is not None:
                result = dict(result, watchdog=note)
            line = json.dumps(result) + "\n"
        sys.stdout.flush()
        if self.rank == 0:
            os.write(self.fd, line.encode())
        return True

    def arm(self, result):
        import threading
        deadline = max(self.t_start + float(os.environ.get("TRPO_BENCH_DEADLINE_S", "420")),
                       time.monotonic() + float(os.environ.get("TRPO_BENCH_GRACE_S", "60")))

        def run():
            while time.monotonic() < deadline:
                time.sleep(min(1.0, max(0.0, deadline - time.monotonic())))
            note = ("deadline reached after %.0f s: the line was printed by the watchdog; secondary configs "
                    "still running were abandoned" % (time.monotonic() - self.t_start))
            if self.emit(result, note):
                print("bench.py: rank %d: %s" % (self.rank, note), file=sys.stderr)
                sys.stderr.flush()
                os._exit(0)

        threading.Thread(target=run, name="bench-watchdog", daemon=True).start()


if __name__ == "__main__":
    main()
