"""numpy emulation of where fp32 FVP error comes from inside CG (2x64 TRPO_Update case):
fp32 per-sample math vs fp64, and rounding only the CG direction p to fp32.  CPU only."""
import sys; sys.path[:0]=['oracle','tests','trpo-robot-control_amd']
import numpy as np, oracle
from trpo_amd import synth
L=[15,64,64,3]; n=8192
th=synth.make_theta(L); obs=synth.make_obs(n,15); P=synth.num_params(L); v=synth.make_v(P)
std=np.ones(3)
ref,_=oracle.fvp(L,'lttl',th,obs,std,v)
def unpack(t, dt):
    Ws=[];Bs=[];pos=0
    for i in range(3):
        W=t[pos:pos+L[i]*L[i+1]].reshape(L[i],L[i+1]).astype(dt); pos+=L[i]*L[i+1]
        B=t[pos:pos+L[i+1]].astype(dt); pos+=L[i+1]; Ws.append(W); Bs.append(B)
    return Ws,Bs
def fvp(dt, acc_dt, tile=16):
    W,B=unpack(th,dt); VW,VB=unpack(v,dt); x=obs.astype(dt)
    y1=np.tanh(x@W[0]+B[0]); rx1=x@VW[0]+VB[0]; ry1=rx1*(1-y1*y1)
    y2=np.tanh(y1@W[1]+B[1]); rx2=ry1@W[1]+y1@VW[1]+VB[1]; ry2=rx2*(1-y2*y2)
    rx3=ry2@W[2]+y2@VW[2]+VB[2]; g3=rx3/(std.astype(dt)**2)
    g2=(g3@W[2].T)*(1-y2*y2); g1=(g2@W[1].T)*(1-y1*y1)
    # accumulate outer products over samples in tiles of `tile` (fp dt), then acc_dt across tiles
    out=[]
    for (a,g) in [(x,g1),(y1,g2),(y2,g3)]:
        acc=np.zeros((a.shape[1],g.shape[1]),acc_dt)
        for s in range(0,n,tile):
            acc+= (a[s:s+tile].T@g[s:s+tile]).astype(acc_dt)
        out.append((acc, g.sum(0,dtype=acc_dt)))
    res=[]
    for i in range(3):
        res.append(out[i][0].ravel().astype(np.float64)); res.append(out[i][1].astype(np.float64))
    r=np.concatenate(res)/n
    r=np.concatenate([r, 2*v[-3:]]) + 0.1*v
    return r
for dt,acc in [(np.float64,np.float64),(np.float32,np.float64),(np.float32,np.float32)]:
    r=fvp(dt,acc)
    print(dt.__name__, acc.__name__, np.linalg.norm(r-ref)/np.linalg.norm(ref))
import cases
c=cases.case('syn_update_2x64_n8192'); X=cases.update_inputs(c)
th=X['theta']; obs=X['obs']; std=X['std']
b,_=oracle.policy_grad(L,'lttl',th,obs,X['mean'],X['action'],X['adv'])
ref=oracle.update(L,'lttl',th,obs,X['mean'],X['action'],X['adv'],std)
def cg(fv, b, iters=10, th_=1e-10):
    x=np.zeros_like(b); r=b.copy(); p=b.copy(); rr=r@r
    for it in range(iters):
        if rr<th_: break
        z=fv(p); a=rr/(p@z); x+=a*p; r-=a*z; nr=r@r; p=r+nr/rr*p; rr=nr
    return x
for dt,acc in [(np.float64,np.float64),(np.float32,np.float64),(np.float32,np.float32)]:
    def fv(p):
        global v
        v=p; return fvp(dt,acc)
    x=cg(fv,b)
    print('CG', dt.__name__, acc.__name__, np.linalg.norm(x-ref['x'])/np.linalg.norm(ref['x']))
print('--- decomposition')
f32=lambda a: a.astype(np.float32).astype(np.float64)
def fv_vround(p):
    global v
    v=f32(p); return fvp(np.float64,np.float64)
x=cg(fv_vround,b); print('v rounded only', np.linalg.norm(x-ref['x'])/np.linalg.norm(ref['x']))
th_s, obs_s = th, obs
th=f32(th_s); obs=f32(obs_s)
def fv64(p):
    global v
    v=p; return fvp(np.float64,np.float64)
x=cg(fv64,b); print('theta/obs rounded only', np.linalg.norm(x-ref['x'])/np.linalg.norm(ref['x']))
th=th_s; obs=obs_s
