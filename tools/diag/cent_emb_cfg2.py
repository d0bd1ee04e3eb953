import sys, time, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'audio-compression_amd')
from oracle import fractal_oracle as O
from fwav import synth
sig,_,_ = synth.make_config_signal("cfg2")
t=time.time()
pool = O.domain_pool(sig, 2048, 8, 2)
print('pool', pool.shape, time.time()-t, flush=True)
t=time.time()
emb = O.embed(pool)
print('emb', emb.shape, time.time()-t, flush=True)
np.save('/tmp/cfg2_emb.npy', emb)
