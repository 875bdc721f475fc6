"""Fit / check the fp32 tanh used by the tile kernel (csrc/trpo_kernels.hip tanh_fast): degree-4
Chebyshev-node least squares for tanh(x)/x on |x| < 0.625, fp32-emulated max relative error."""
import numpy as np
thr=0.625
u=np.linspace(1e-12, thr*thr, 20001)
x=np.sqrt(u)
f=(np.tanh(x)/x - 1)/u   # Q(u)
for deg in [3,4,5]:
    # Chebyshev-weighted LS fit -> close to minimax
    t=np.cos(np.pi*(np.arange(400)+0.5)/400)*0.5*thr*thr+0.5*thr*thr
    xx=np.sqrt(t); ff=(np.tanh(xx)/xx-1)/t
    c=np.polyfit(t, ff, deg)
    # evaluate in fp32 emulation
    xs=np.linspace(-thr,thr,200001).astype(np.float32)
    u32=(xs*xs).astype(np.float32)
    q=np.float32(c[0])
    for cc in c[1:]:
        q=(q*u32+np.float32(cc)).astype(np.float32)
    y=(xs + (xs*u32).astype(np.float32)*q).astype(np.float32)
    ref=np.tanh(xs.astype(np.float64))
    rel=np.abs(y-ref)/np.maximum(np.abs(ref),1e-30)
    print(deg, rel.max(), [float(np.float32(v)) for v in c])
# big branch check
xs=np.linspace(thr,12,200001).astype(np.float32)
e=np.exp2((xs*np.float32(2*1.4426950408889634)).astype(np.float32)).astype(np.float32)
t=(np.float32(1)-np.float32(2)*(np.float32(1)/(e+np.float32(1))).astype(np.float32)).astype(np.float32)
ref=np.tanh(xs.astype(np.float64)); print('big', (np.abs(t-ref)/ref).max())
