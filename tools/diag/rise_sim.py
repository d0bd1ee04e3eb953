"""Rising band limit of the fp16 search, simulated on the real cfg2 table (f32 scores as the s16 proxy): appends and
compactions per query of one whole-table pass (plan P = 1) for the product policy (compact when the two-ended
buffer of C = 256 passes 224; limit = K-th − 2δ; seed = K-th of the own window ±64 − 2δ) and for variants.
Table: /tmp/cfg2_emb.npy (tools/diag/cent_emb_cfg2.py).  usage: python tools/diag/rise_sim.py [n_queries]"""
import sys
import numpy as np

E = np.load('/tmp/cfg2_emb.npy')
nd = len(E)
K, C, D = 64, 256, 2e-3


def run(q, policy):
    s_all = E @ E[q]
    w = s_all[max(0, q - 64):q + 64]
    thf = np.sort(w)[-K] - 2 * D
    buf = []
    app = comp = 0
    step = policy.get('step')
    lvl = None
    cnt = 0
    for a in range(0, nd, 1024):  # one group of 4 chunks: the limit is applied per tile; per group is close enough
        s = s_all[a:a + 1024]
        idx = np.nonzero(s > thf)[0]
        if len(idx) == 0:
            continue
        new = s[idx]
        app += len(new)
        buf.extend(new.tolist())
        if step is not None:
            if lvl is None:
                lvl = thf + 2 * D + step
            cnt += int((new > lvl).sum())
            while cnt >= K:  # K collected entries above lvl: K-th ≥ lvl
                thf = max(thf, lvl - 2 * D)
                lvl = thf + 2 * D + step
                cnt = 0 if policy.get('reset') else sum(1 for x in buf if x > lvl)
        if len(buf) > policy.get('trig', C - 32):
            comp += 1
            b = np.array(buf)
            T = np.sort(b)[-K] if len(b) >= K else -np.inf
            thf = max(thf, T - 2 * D)
            buf = b[b > thf].tolist()
            if step is not None:
                lvl = thf + 2 * D + step
                cnt = 0 if policy.get('reset') else sum(1 for x in buf if x > lvl)
    b = np.array(buf)
    T = np.sort(b)[-K]
    band = int((b > T - 2 * D).sum())
    return app, comp, band


n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rng = np.random.default_rng(3)
qs = rng.choice(330750, n, replace=False)
for name, pol in [('product (trig 224)', {}), ('trig 128', {'trig': 128}), ('trig 96', {'trig': 96}),
                  ('counter step 2e-3', {'step': 2e-3}), ('counter step 1e-3', {'step': 1e-3}),
                  ('counter step 4e-3', {'step': 4e-3}), ('counter reset 2e-3', {'step': 2e-3, 'reset': 1}),
                  ('counter reset 4e-3', {'step': 4e-3, 'reset': 1}), ('counter reset 8e-3', {'step': 8e-3, 'reset': 1})]:
    r = np.array([run(int(q), pol) for q in qs])
    print(f"{name:22s} appends/query {r[:, 0].mean():7.1f}  compactions {r[:, 1].mean():5.2f}  final band {r[:, 2].mean():6.1f}",
          flush=True)
