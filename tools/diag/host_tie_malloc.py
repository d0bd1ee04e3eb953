"""Diagnostic: numpy's argpartition on exact score rows, with glibc's default mmap of large blocks (a fresh 8-byte
index array per call: page faults) vs mallopt(M_MMAP_MAX=0) + no trimming (the index arrays reuse heap pages),
serial and threaded; and a process pool for comparison."""
import ctypes
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def top64(s):
    p = np.argpartition(s, -64)[-64:]
    return p[np.argsort(s[p])[::-1]]


def bench(label):
    for nd in (1321977, 6613977):
        rng = np.random.default_rng(0)
        rows = [(1.9 + rng.random(nd, dtype=np.float32) * 0.1).astype(np.float32) for _ in range(16)]
        top64(rows[0])
        t = time.perf_counter()
        for r in rows:
            top64(r)
        ser = (time.perf_counter() - t) / len(rows) * 1e3
        out = [f"{label} nd {nd}: serial {ser:.2f} ms/row"]
        for nt in (4, 8, 16):
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(top64, rows[:nt]))
                t = time.perf_counter()
                list(ex.map(top64, rows))
                out.append(f"{nt} thr {(time.perf_counter() - t) / len(rows) * 1e3:.2f}")
        print(", ".join(out), flush=True)


if __name__ == "__main__":
    bench("default")
    libc = ctypes.CDLL("libc.so.6")
    M_TRIM_THRESHOLD, M_MMAP_MAX = -1, -4
    print("mallopt", libc.mallopt(M_MMAP_MAX, 0), libc.mallopt(M_TRIM_THRESHOLD, 1 << 40), flush=True)
    bench("no-mmap")
