"""How long a pinned host allocation of a map set takes when the previous set was
released vs still held: torch's pinned allocator, and the library's host cache
(comap_host_alloc via _native.host_empty):  python scripts/pinned_probe.py"""
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from comapreduce_amd import _native as N  # noqa: E402


def main():
    torch.cuda.init()
    dev = torch.device('cuda', 0)
    src = torch.zeros((4, 4, 230400), dtype=torch.float64, device=dev)
    for mode in ('release', 'hold', 'cache-release', 'cache-hold'):
        ts = []
        held = []
        for _ in range(6):
            t0 = time.perf_counter()
            if mode.startswith('cache'):
                h = torch.from_numpy(N.host_empty(tuple(src.shape)))
            else:
                h = torch.empty(src.shape, dtype=torch.float64, pin_memory=True)
            t1 = time.perf_counter()
            h.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            a = h.numpy()
            if mode.endswith('hold'):
                held.append(a)
            del h, a
            ts.append((t1 - t0) * 1e3)
        t0 = time.perf_counter()
        h = torch.from_numpy(N.host_empty(tuple(src.shape))) if mode.startswith('cache') else \
            torch.empty(src.shape, dtype=torch.float64, pin_memory=True)
        h.copy_(src, non_blocking=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(mode, 'copy enqueue ms %.3f, copy %.3f ms' % ((t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
        print(mode, 'alloc ms', [round(t, 3) for t in ts], flush=True)


if __name__ == '__main__':
    main()
