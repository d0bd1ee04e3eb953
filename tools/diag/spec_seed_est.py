"""Diagnostic (numpy, CPU): how close a speculative band limit — the j-th best score of a strided 1/frac sample of
the table — lies to the exact K-th, after the margin that keeps a failure rate p.  usage: python tools/diag/spec_seed_est.py [cfg2]"""
import sys, time, numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0]=[R, os.path.join(R,'audio-compression_amd')]
from oracle import fractal_oracle as O
from fwav import synth
cfg=sys.argv[1] if len(sys.argv)>1 else 'cfg2'
sig,sr,_=synth.make_config_signal(cfg, seed=0)
tile={'cfg2':2048,'cfg3':2048}.get(cfg,2048)
rs,step=O.geometry(tile)
t=time.time(); pool=O.domain_pool(sig,tile,rs,step); E=O.embed(pool).astype(np.float32); print('embed',E.shape,time.time()-t,flush=True)
nd=len(E); nr=-(-len(sig)//rs)
rng=np.random.default_rng(0)
qs=rng.choice(nr,600,replace=False)
Q=E[(qs*rs)//step]
K=64
S=Q@E.T  # 600 x nd
srt=-np.sort(-S,axis=1)
kth=srt[:,K-1]
print('kth mean %.4f sd %.4f'%(kth.mean(),kth.std()))
for frac,j in ((16,4),(16,2),(8,8),(8,4),(32,2),(4,16)):
    # strided chunk sample: every frac-th chunk of 256 domains
    ch=np.arange(nd)//256
    m=(ch%frac)==0
    ss=-np.sort(-S[:,m],axis=1)
    est=ss[:,j-1]
    d=kth-est   # positive = estimate below K-th (valid-ish)
    # margin so that seed=est-m <= kth - 0.006 (3 delta) for all but p of queries
    for p in (0.0,0.002,0.01):
        need=np.quantile(-d,1-p) if p>0 else (-d).max()
        mgn=max(0,need)+0.006
        gap=(kth-(est-mgn))
        print(f'frac 1/{frac} j={j} p={p}: margin {mgn:.4f} mean gap {gap.mean():.4f} (median {np.median(gap):.4f})')
