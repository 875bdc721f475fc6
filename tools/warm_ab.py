"""Is the driver's short headline run (--steps 20 --warmup 5: 0.5 ms of warm-up) slower per solve than a
long one because of one-off costs inside the timed region?  Each trial is a fresh process (as the
driver's) that builds the headline context and times K solves after W warm-up ones, optionally after
`pre` ms of the CG-iteration kernel's event timing (what bench.py does for the roofline).
usage: python tools/warm_ab.py [trials]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, time
sys.path[:0] = [%r, %r]
import bench
import trpo_amd
trpo_amd.lib()
from trpo_amd import synth
K, W, pre = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
d = bench.Dist()
ctx, _, _ = bench.make_ctx(bench.ARM, bench.N_TOTAL, d, 0)
b = synth.make_b(bench.num_params(bench.ARM))
ctx.upload_b(b)
if pre:
    ctx.time_ms(3, 20, 10)
t = bench.time_steps(ctx, d, K, W, b)
print(json.dumps({"ms": 1e3 * t / K}))
''' % (ROOT, os.path.join(ROOT, "trpo-robot-control_amd"))

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 3
configs = ((20, 5, 0, ""), (20, 5, 1, ""), (500, 50, 0, ""), (20, 50, 0, ""), (100, 5, 0, ""))
if len(sys.argv) > 2 and sys.argv[2] == "graph":       # CG graph vs eager launches (TRPO_NO_GRAPH)
    configs = ((20, 5, 0, ""), (20, 5, 0, "TRPO_NO_GRAPH=1"), (500, 50, 0, ""), (500, 50, 0, "TRPO_NO_GRAPH=1"))
res = {}
for t in range(trials):
    for K, W, pre, env in configs:
        e = dict(os.environ)
        if env:
            k, v = env.split("=")
            e[k] = v
        p = subprocess.run([sys.executable, "-c", CHILD, str(K), str(W), str(pre)], capture_output=True, text=True,
                           timeout=120, env=e)
        ms = json.loads(p.stdout.strip().splitlines()[-1])["ms"] if p.returncode == 0 else None
        res.setdefault("K%d W%d pre%d %s" % (K, W, pre, env), []).append(ms)
        print("trial %d K=%d W=%d pre=%d %s: %s ms" % (t, K, W, pre, env, ms), flush=True)
for k, v in res.items():
    print(k, " ".join("%.4f" % x for x in v if x))
