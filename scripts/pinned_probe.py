"""How long torch's pinned host allocation of a map set takes when the previous set was
released (cached) vs still held (fresh hipHostMalloc):  python scripts/pinned_probe.py"""
import time

import torch


def main():
    torch.cuda.init()
    dev = torch.device('cuda', 0)
    src = torch.zeros((4, 4, 230400), dtype=torch.float64, device=dev)
    held = []
    for mode in ('release', 'hold'):
        ts = []
        for _ in range(6):
            t0 = time.perf_counter()
            h = torch.empty(src.shape, dtype=torch.float64, pin_memory=True)
            t1 = time.perf_counter()
            h.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            a = h.numpy()
            if mode == 'hold':
                held.append(a)
            del h, a
            ts.append((t1 - t0) * 1e3)
        print(mode, 'alloc ms', [round(t, 3) for t in ts], flush=True)


if __name__ == '__main__':
    main()
