"""Diagnostic: the host side of a tie resolution on this box — numpy's argpartition/argsort on one exact score row
(cfg2 / cfg3 widths) and the device→host copy of that row (pageable vs pinned), serial and with a thread pool."""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

for nd in (1321977, 6613977):
    rng = np.random.default_rng(0)
    rows = [(1.9 + rng.random(nd, dtype=np.float32) * 0.1).astype(np.float32) for _ in range(8)]
    f = lambda s: (lambda p: p[np.argsort(s[p])[::-1]])(np.argpartition(s, -64)[-64:])  # noqa: E731
    f(rows[0])
    t = time.perf_counter()
    for r in rows:
        f(r)
    ser = (time.perf_counter() - t) / len(rows) * 1e3
    for nt in (2, 4, 8):
        with ThreadPoolExecutor(nt) as ex:
            t = time.perf_counter()
            list(ex.map(f, rows))
            par = (time.perf_counter() - t) / len(rows) * 1e3
        print(f"nd {nd}: numpy top-64 serial {ser:.2f} ms/row, {nt} threads {par:.2f} ms/row", flush=True)
    d = torch.from_numpy(rows[0]).cuda()
    pin = torch.empty(nd, dtype=torch.float32, pin_memory=True)
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        h = d.cpu()
        a = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        pin.copy_(d)
        torch.cuda.synchronize()
        b = (time.perf_counter() - t) * 1e3
    print(f"nd {nd}: D2H pageable {a:.2f} ms, pinned {b:.2f} ms", flush=True)
