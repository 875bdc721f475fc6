"""Floor of one peer-window exchange (csrc/trpo_peer.hip) measured on ONE GPU: two in-process ranks
(contexts on contiguous halves of the armDOF_0 N = 50k batch, windows joined by pointer), each
running SOLVES 10-iteration CG solves in its own thread.  Run under
  rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- python3 tools/peer_floor.py
The rank that reaches an exchange second finds the other's data and flag already there, so its
exchange kernel's duration is the exchange itself (local replica sum, the two pushes, release, flag,
acquire, rank-order sum) with no waiting: the lower half of the kernel-duration distribution.  What
it does not contain is the xGMI round trip of the remote stores and flag (both ranks share one HBM)."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402

L = [15, 16, 16, 3]
N = int(os.environ.get("N", "50000"))
SOLVES = int(os.environ.get("SOLVES", "200"))
th, obs = synth.make_theta(L), synth.make_obs(N, 15)
b = synth.make_b(synth.num_params(L))
half = N // 2
ctxs = [trpo_amd.Context(L, "lttl", th, obs[lo:hi], np.ones(3)) for lo, hi in ((0, half), (half, N))]
for c in ctxs:
    c.cg(b, 10, 0.0)                       # size the lazily allocated buffers before attaching
    c.peer_handle()
out = [None, None]
err = [None, None]


def work(r):
    try:
        ctxs[r].attach_peers_local(r, ctxs)
        for _ in range(SOLVES):
            x = ctxs[r].cg(b, 10, 0.0)
        out[r] = x
    except BaseException as e:             # noqa: BLE001 -- reported below
        err[r] = e


ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(2)]
for t in ts:
    t.start()
for t in ts:
    t.join(300)
assert not any(t.is_alive() for t in ts), "a rank did not finish"
for e in err:
    if e is not None:
        raise e
assert np.array_equal(out[0], out[1]), "ranks disagree"
print("ok: %d solves per rank, x identical on both ranks, backend %s" % (SOLVES, ctxs[0].comm_info()["backend"]))
for c in ctxs:
    c.close()
