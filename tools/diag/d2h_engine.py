#!/usr/bin/env python3
"""How a tied row's exact scores reach the host: 20 device→page-locked copies of one cfg2 score row (1,321,977
floats, 5.3 MB), timed with HIP events, while a long kernel may run on another stream — run under
`rocprofv3 --kernel-trace` to see whether the runtime moves them with a blit kernel (`__amd_rocclr_copyBuffer`, which
takes CUs from the search) or a DMA engine, and compare the HIP runtime's copy settings (GPU_FORCE_BLIT_COPY_SIZE …).
usage: python tools/diag/d2h_engine.py"""
from __future__ import annotations

import torch


def main():
    n = 1_321_977
    src = torch.randn(n, device="cuda")
    dst = torch.empty(n, dtype=torch.float32, pin_memory=True)
    side = torch.cuda.Stream()
    ms = []
    for i in range(21):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record()
            dst.copy_(src, non_blocking=True)
            e1.record()
        torch.cuda.synchronize()
        if i:
            ms.append(e0.elapsed_time(e1))
    ms.sort()
    print(f"5.3 MB device->pinned copy: median {ms[len(ms) // 2] * 1e3:.1f} us, {n * 4 / (ms[len(ms) // 2] * 1e-3) / 1e9:.1f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
