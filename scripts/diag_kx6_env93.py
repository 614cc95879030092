"""The kx6 divergence, traced on the oracle (CPU): env 93 of the 96-env, N = 5
instance workload (seed 36, synthetic actions seed 5) before and after step 5.  Compares the oracle's
body-5 velocity change with the one implied by the GPU's positions (scripts/diag_instance.py output,
profiles/r05/fault/kx6_state_divergence_b96.jsonl): the press impulse has the right direction and the
wrong length, and the one near-midpoint square of that step (dx = -34.6387..., glibc path) is the only
square that can explain it -- the GPU's implied dx^2 is 1028.349..., what scripts/kx6_table_repro.cpp
computes with the miscompiled table.  TEST / DIAGNOSTIC INFRASTRUCTURE (uses the oracle)."""
import sys, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'gym-futbol_amd')
from helpers import O
import rng_tape as R
n,B=5,96; seed=36
ora=O.V1Vec(B,N=n,seed=seed,portable=True); ora.reset()
def acts(t): return np.stack([R.synthetic_actions_vec(5, np.arange(B), t, j, 5) for j in range(2*n)],1).astype(np.int32)
E=93
for t in range(5): ora.step(acts(t))
e=ora.envs[E]
g=lambda f,k: getattr(e,f)[k]
pre={f:[g(f,k) for k in range(11)] for f in ("px","py","vx","vy","bx","by")}
print("left acts", acts(5)[E])
ora.step(acts(5))
post={f:[g(f,k) for k in range(11)] for f in ("px","py","vx","vy","bx","by")}
k=5
vact_o=((post['px'][k]-pre['px'][k])/0.1-pre['bx'][k], (post['py'][k]-pre['py'][k])/0.1-pre['by'][k])
gp=(86.7657898124569,18.52665300582688)
vact_g=((gp[0]-pre['px'][k])/0.1-pre['bx'][k], (gp[1]-pre['py'][k])/0.1-pre['by'][k])
print("pre v5", pre['vx'][k], pre['vy'][k], "pre b5", pre['bx'][k], pre['by'][k])
print("v_act oracle", vact_o, "gpu", vact_g, "diff", np.subtract(vact_g,vact_o))
d_oracle=np.subtract(vact_o,(pre['vx'][k],pre['vy'][k])); d_gpu=np.subtract(vact_g,(pre['vx'][k],pre['vy'][k]))
print("impulse/m oracle", d_oracle, np.hypot(*d_oracle), "gpu", d_gpu, np.hypot(*d_gpu))
ball=(pre['px'][10],pre['py'][10]); pl=(pre['px'][k],pre['py'][k])
u=np.subtract(ball,pl); print("ball-player dir", u/np.hypot(*u), "dist", np.hypot(*u))
for j in range(11): print(j, pre['px'][j], pre['py'][j], pre['vx'][j], pre['vy'][j])
import math
dx=pre['px'][10]-pre['px'][5]; dy=pre['py'][10]-pre['py'][5]
def near(x):
    from fractions import Fraction as F
    h=x*x; l=float(F(x)*F(x)-F(h))
    import struct
    eb=struct.unpack('<Q',struct.pack('<d',h))[0]&0x7ff0000000000000
    if h==0: return False
    nr=struct.unpack('<d',struct.pack('<Q',eb-(53<<52)))[0]*(1-2**-5)
    return not(abs(l)<nr)
print("dx",dx,"near",near(dx),"dy",dy,"near",near(dy))
mg=2*math.hypot(dx,dy)/2.129838935140013
print("gpu mag^2", mg*mg, "dx^2",dx*dx,"dy^2",dy*dy, "implied other", mg*mg-dx*dx, mg*mg-dy*dy)
sq=[]
for j in range(10):
    sq+= [(pre['px'][10]-pre['px'][j])**2, (pre['py'][10]-pre['py'][j])**2]
sq+=[(105-pre['px'][10])**2,(0-pre['px'][10])**2,(34-pre['py'][10])**2]
import itertools
best=sorted(((abs(a+b-mg*mg),i,j) for (i,a),(j,b) in itertools.product(enumerate(sq),enumerate(sq))))[:5]
print(best)
for j in range(10):
    for q,x in ((0,pre['px'][10]-pre['px'][j]),(1,pre['py'][10]-pre['py'][j])):
        if near(x): print("near-midpoint square: player",j,"axis",q,x)
