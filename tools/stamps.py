"""Per-phase timing of the FVP kernel from the diagnostic stamps build (make stamps).
Phases (block-local, thread 0): 0 entry, 1 weights staged, 2 first tile forward done,
3 first tile done, 4 tile loop done, 5 cross-wave tree done, 6 slab written."""
import ctypes as C, os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TRPO_LIB"] = os.path.join(ROOT, "trpo-robot-control_amd/lib/libtrpo_mi355x_stamps.so")
sys.path[:0] = [os.path.join(ROOT, "trpo-robot-control_amd")]
import trpo_amd
from trpo_amd import synth
L = trpo_amd.lib()
L.trpo_dev_read_stamps.restype = C.c_int
L.trpo_dev_read_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
for name, layers, n in [("arm", [15,16,16,3], 16), ("arm", [15,16,16,3], 50000), ("2x64", [15,64,64,3], 16), ("2x64", [15,64,64,3], 50000)]:
    th = synth.make_theta(layers); P = synth.num_params(layers)
    with trpo_amd.Context(layers, "lttl", th, synth.make_obs(n, 15), np.ones(3)) as ctx:
        ctx.upload_v(synth.make_v(P))
        for rep in range(int(os.environ.get("WARM", "5"))):
            ctx.enqueue_fvp_kernel()
        ctx.synchronize()
        G = ctx.geometry["blocks"]
        buf = (C.c_ulonglong * (1024 * 32))()
        L.trpo_dev_read_stamps(buf, 1024 * 32)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 32)[:G, :7].astype(np.int64)
        t0 = a[:, 0].min()
        rel = (a - t0) * 10 / 1000.0   # us
        print("%s N=%d G=%d  block0 phases (us): %s" % (name, n, G, " ".join("%.2f" % x for x in rel[0])))
        print("   entry  min/med/max %.2f %.2f %.2f   exit(6) min/med/max %.2f %.2f %.2f" % (
            rel[:,0].min(), np.median(rel[:,0]), rel[:,0].max(), rel[:,6].min(), np.median(rel[:,6]), rel[:,6].max()))
        d = np.diff(rel, axis=1)
        print("   median phase durations 0>1 1>2 2>3 3>4 4>5 5>6: %s" % " ".join("%.2f" % x for x in np.median(d, axis=0)))
        cyc = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 32)[:G, 16:23].astype(np.int64)
        clk = (cyc[:, 6] - cyc[:, 0]) / np.maximum(1, (a[:, 6] - a[:, 0])) * 100.0   # MHz
        print("   shader clock (MHz) median %.0f  min %.0f  max %.0f" % (np.median(clk), clk.min(), clk.max()))
        print("   kernel_us(events) %.2f" % (ctx.time_ms(0, 50) * 1e3))
