"""comap_prep_auto_rms alone at the chain's size (19 feeds x 4 bands x 180 000 samples,
the Level-2 rows read_comap_data weights by), timed with HIP events:
    python scripts/prep_rms_probe.py [reps]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from comapreduce_amd import _native as N  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    F, B, T = 19, 4, 180_000
    x = torch.randn((F, B, T), dtype=torch.float64, device=dev)
    rows = torch.arange(F * B, dtype=torch.int32, device=dev)
    scale = torch.ones(F * B, dtype=torch.float64, device=dev)
    rms = torch.empty(F * B, dtype=torch.float64, device=dev)
    c = N.ctx(0)
    N.bind_stream(c, dev)

    def run():
        N.check(N.lib().comap_prep_auto_rms(c, N.dptr(x), T, N.dptr(rows), N.dptr(scale), F * B, T, N.dptr(rms)), c,
                'comap_prep_auto_rms')
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    ref = np.array([np.nanstd(r[1:] - r[0]) / np.sqrt(2) for r in x.reshape(F * B, T).cpu().numpy()[:4]])
    print(json.dumps({'ms_per_call': ms, 'GBs_2pass': 2 * F * B * T * 8 / (ms * 1e-3) / 1e9,
                      'max_rel_vs_numpy_first4': float(np.max(np.abs(rms[:4].cpu().numpy() - ref) / ref))}),
          flush=True)


if __name__ == '__main__':
    main()
