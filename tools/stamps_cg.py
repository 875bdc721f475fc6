"""Phase stamps of the LAST fused CG-iteration kernel of a CG solve (make stamps).
Slots: 0 entry, 7 loads+LDS staged, 1 after fused update + v pack, 13/14/2 first tile layers 0/1/2,
15 first tile G2, 3 first tile,
4 tiles done, 5 wave combine done, 6 end."""
import ctypes as C, os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TRPO_LIB"] = os.path.join(ROOT, "trpo-robot-control_amd/lib/libtrpo_mi355x_stamps.so")
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
L = trpo_amd.lib()
L.trpo_dev_read_stamps.restype = C.c_int
L.trpo_dev_read_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
order = [0, 7, 8, 9, 10, 11, 12, 1, 13, 14, 2, 15, 3, 4, 5, 6]
NS = [int(x) for x in os.environ.get("NS", "50000").split(",")]
cfgs = [("arm", [15,16,16,3], n, g, r) for n in NS for g in os.environ.get("GRIDS", "0").split(",") for r in os.environ.get("REPL", "8").split(",")]
if os.environ.get("WIDE", "1") == "1":
    cfgs += [("2x64", [15,64,64,3], 50000, "0", "8")]
for name, layers, n, grid, repl in cfgs:
    os.environ["TRPO_REPLICAS"] = repl
    if grid != "0": os.environ["TRPO_FVP_BLOCKS"] = grid
    else: os.environ.pop("TRPO_FVP_BLOCKS", None)
    th = synth.make_theta(layers); P = synth.num_params(layers)
    with trpo_amd.Context(layers, "lttl", th, synth.make_obs(n, 15), np.ones(3)) as ctx:
        ctx.upload_b(synth.make_b(P))
        for rep in range(20):
            ctx.enqueue_cg(10, 0.0)
        ctx.synchronize()
        G = ctx.geometry["blocks"]
        buf = (C.c_ulonglong * (1024 * 32))()
        L.trpo_dev_read_stamps(buf, 1024 * 32)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 32)[:G].astype(np.int64)
        t = a[:, order]
        rel = (t - t[:, 0].min()) * 10 / 1000.0
        d = np.diff(rel, axis=1)
        print("%s N=%d G=%d R=%s cg10_us=%.1f" % (name, n, G, repl, ctx.time_ms(2, 20, 10, 0.0) * 1e3))
        print("   entry min/med/max %.2f %.2f %.2f  end min/med/max %.2f %.2f %.2f" % (
            rel[:, 0].min(), np.median(rel[:, 0]), rel[:, 0].max(), rel[:, -1].min(), np.median(rel[:, -1]), rel[:, -1].max()))
        print("   median phases  load>staged %.2f  zwait %.2f  red1 %.2f  red2 %.2f  stage %.2f  bar %.2f  gather %.2f | L0 %.2f  L1 %.2f  L2 %.2f  G2 %.2f  tile1 %.2f  rest %.2f  combine %.2f  write %.2f" % tuple(np.median(d, axis=0)))
