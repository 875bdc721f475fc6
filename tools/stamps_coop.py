"""Phase profile of the cooperative kernel (fvp_coop_kernel, 2x64 policies) from the stamps build
(make -C trpo-robot-control_amd stamps): wave 0 and wave 4 (the first waves of the two lane groups) of
every block accumulate the shader-clock cycles
(s_memtime) of each phase of its tile steps.  Phases (round 5, the segments of
fvp_coop_kernel's tile step): 0 S0 layer 0 (incl. the wait for the tile's inputs), 1 the barrier wait
before S1, 2 S1 (y1/r1 rows read, layer 1, the layer-2 partial), 3 the wait before S2, 4 S2 (partials
summed, G3, RGW2, G2), 5 the wait before S3, 6 S3's G1, 7 S3's RGW1 + RGW0; 8 = the whole tile loop.  Prints the median over blocks of the
cycles per tile step.   usage: python tools/stamps_coop.py [N ...]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TRPO_LIB", os.path.join(ROOT, "trpo-robot-control_amd/lib/libtrpo_mi355x_stamps.so"))
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd  # noqa: E402
from trpo_amd import synth  # noqa: E402

L = trpo_amd.lib()
L.trpo_dev_read_stamps.restype = C.c_int
L.trpo_dev_read_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
NAMES = ["S0 layer0", "wait > S1", "S1 layer1+2", "wait > S2", "S2 g3/RGW2/G2", "wait > S3", "S3 G1", "S3 RGW1+0"]
layers = [15, 64, 64, 3]
for n in [int(a) for a in sys.argv[1:]] or [4096, 50000]:
    th = synth.make_theta(layers)
    P = synth.num_params(layers)
    with trpo_amd.Context(layers, "lttl", th, synth.make_obs(n, 15), np.ones(3)) as ctx:
        ctx.upload_v(synth.make_v(P))
        for _ in range(6):                       # the first call writes the forward cache; then cached
            ctx.enqueue_fvp_kernel()
        ctx.synchronize()
        G = ctx.geometry["blocks"]
        buf = (C.c_ulonglong * (1024 * 32))()
        L.trpo_dev_read_stamps(buf, 1024 * 32)
        full = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 32)[:G].astype(np.float64)
        meds = []
        for o in (0, 16):                        # wave 0 (group 0) and the first wave of group 1
            a = full[:, o:o + 10]
            steps = np.maximum(a[:, 9], 1)
            meds.append(np.median(a[:, :9] / steps[:, None], axis=0))
        print("2x64 N=%d blocks=%d steps=%d kernel %s; cycles per tile step (median over blocks), "
              "group 0 wave 0 | group 1 wave 0:" % (n, G, int(np.median(steps)), ctx.kernel_name))
        for k in range(8):
            print("  %-12s %7.0f  (%4.1f %%) | %7.0f  (%4.1f %%)" % (NAMES[k], meds[0][k], 100 * meds[0][k] / meds[0][8],
                                                              meds[1][k], 100 * meds[1][k] / meds[1][8]))
        print("  %-12s %7.0f | %7.0f" % ("loop", meds[0][8], meds[1][8]))
        pro, epi = np.median(full[:, 10]), np.median(full[:, 11])
        print("  prologue (entry -> loop) %.0f cycles, epilogue (loop -> slab stored) %.0f cycles, loop total %.0f"
              % (pro, epi, np.median(full[:, 8])))
        print("  kernel_us(events) %.2f" % (ctx.time_ms(0, 50) * 1e3))
