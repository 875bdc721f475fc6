"""TEST HELPER (CPU, no GPU): one rank of bench.py's N > 1 path with the device library replaced by
fake contexts, so tests/test_bench_secondaries.py can run the real bench.main() -- real gloo
agreements, real fault hooks, real watchdog -- as two processes on the CPU.  The fakes do no compute:
x is a fixed vector, every collective is a no-op, and the timings are small constants.
    WORLD_SIZE=2 RANK=r LOCAL_RANK=r MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/bench_fake_rank.py <bench args>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "trpo-robot-control_amd")]

import numpy as np  # noqa: E402

import trpo_amd  # noqa: E402


class FakeContext:
    def __init__(self, layers, acfunc, theta, obs, std, damping=0.1, device=-1, precision=None):
        self.layers, self.n, self.backend = list(layers), int(np.asarray(obs).shape[0]), "none"
        L = self.layers
        self.P = sum(L[i] * L[i + 1] + L[i + 1] for i in range(len(L) - 1)) + L[-1]
        self.world = 1
        self.closed = False

    def peer_handle(self):
        return b"h" * trpo_amd.PEER_HANDLE_BYTES

    def attach_peers(self, rank, world, handles):
        self.backend, self.world = "peer", world

    def attach_comm(self, rank, world, uid, timeout_ms=0):
        self.backend, self.world = "rccl", world

    def comm_info(self):
        return dict(rank=0, world=self.world, replicas=2, backend=self.backend)

    @property
    def comm_backend(self):
        return self.backend

    def comm_verify(self, timeout_ms=0):
        pass

    def comm_abort(self):
        sys.stderr.write("fake: comm_abort\n")

    def upload_b(self, b):
        pass

    def upload_v(self, v):
        pass

    def enqueue_cg(self, *a):
        pass

    def wait(self, timeout_ms=0):
        pass

    def synchronize(self):
        pass

    def time_ms(self, *a):
        return 0.01

    def download_x(self):
        return np.linspace(1.0, 2.0, self.P)

    def set_rollout(self, mean, action, adv):
        pass

    def update(self, *a, **k):
        return dict(accepted=True, cg_iters=10, fp64_rerun=False)

    @property
    def kernel_name(self):
        return "fake"

    @property
    def geometry(self):
        return dict(blocks=1, threads=1, lds_bytes=0)

    def close(self):
        self.closed = True


def main():
    trpo_amd.Context = FakeContext
    trpo_amd.lib = lambda: None
    trpo_amd.runtime_path = lambda: "fake"
    trpo_amd.unique_id = lambda: b"u" * 128
    import bench
    bench.SWEEP_N = (4000, 6000)                 # small rows: the fakes do no work, the shapes are synthesised
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()


if __name__ == "__main__":
    main()
