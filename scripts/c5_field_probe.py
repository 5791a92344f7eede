"""Round-5 probe: why the rounds 2-4 C5 field never converged.

C5 per-GPU size (8 obs x 19 feeds x 180k samples, L = 50, 480 x 480 1' CAR), one band,
the reference's stopping rule (threshold 1e-6, at most 100 iterations), per-iteration
delta = rr / rr0 recorded with the DeviceOps pieces (cg_solve's order, one rank):
  a. the old field: +-4.2 deg Lissajous on the +-4.0 deg map (~37 % of samples off-map,
     pixel -1: not binned, but the projection gathers m[-1] -- Destriper.py:206-213);
  b. the same pointing with the off-map samples' weights set to 0 (no m[-1] reads);
  c. the new default field, +-3.8 deg (every sample on-map).
Then the native solve's ms per iteration for c (1 and 4 bands).
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from comapreduce_amd import synthetic  # noqa: E402
from comapreduce_amd.mapmaking.destriper import DeviceDestriper  # noqa: E402


def history(pix, tod, w, L=50, npix=480 * 480, niter=100, thr=1e-6):
    ops = DeviceDestriper(pix, tod, w, L, npix, device=0).ops
    h, _, nnum = ops.local_maps()
    NO = ops.n_offsets
    x, r, q = ops.zeros(NO), ops.zeros(NO), ops.zeros(NO)
    ops.project(None, nnum, h, r)
    p = ops.copy(r)
    rr0, rr, pq, rrn = ops.scalar(), ops.scalar(), ops.scalar(), ops.scalar()
    ops.dot(r, r, rr0)
    rr.copy_(rr0)
    t0 = float(rr0.item())
    num = ops.zeros(npix)
    deltas = []
    for i in range(niter):
        ops.bin(p, 0, num)
        ops.project(p, num, h, q, pq)
        ops.cg_update(rr, pq, x, r, p, q, rrn)
        ops.cg_direction(rrn, rr, p, r)
        rr.copy_(rrn)
        d = float(rrn.item()) / t0
        deltas.append(d)
        if np.isnan(d) or d < thr:
            break
    xn = ops.natural(x)
    return {'iters': len(deltas), 'delta_first10': deltas[:10], 'delta_last': deltas[-1],
            'delta_min': min(deltas), 'max_abs_x': float(xn.abs().max().item()),
            'pq_sign_flips': int(sum(1 for a, b in zip(deltas, deltas[1:]) if b > a))}


def main():
    out = {}
    pix, tod, w = synthetic.destriper_inputs_device(8, device=0, seed=1000, amp=4.2)
    off = pix < 0
    out['a_amp4.2'] = dict(history(pix, tod, w), offmap_fraction=float(off.double().mean().item()))
    w0 = torch.where(off, torch.zeros_like(w), w)
    out['b_amp4.2_offmap_w0'] = history(pix, tod, w0)
    del pix, tod, w, w0, off
    torch.cuda.empty_cache()
    pix, tod, w = synthetic.destriper_inputs_device(8, device=0, seed=1000)
    out['c_amp3.8'] = dict(history(pix, tod, w), offmap_fraction=float((pix < 0).double().mean().item()))
    for nb in (1, 4):
        if nb == 4:
            pix, tod, w = synthetic.destriper_inputs_device(8, device=0, seed=1000, n_bands=4)
        dd = DeviceDestriper(pix, tod, w, 50, 480 * 480, device=0)
        dd.solve(0.0, 3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = dd.solve(0.0, 100)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        conv = dd.solve(1e-6, 100)
        out[f'c_native_{nb}band'] = {'ms_per_iter': dt / 100 * 1e3, 'converged_iters': conv['iters'],
                                     'nnz': dd.nnz(), 'sell_entries': dd.sell_entries()}
        print(json.dumps({f'c_native_{nb}band': out[f'c_native_{nb}band']}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == '__main__':
    main()
