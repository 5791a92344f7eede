"""Round-5 probe for the CG pair's gather locality.

scripts/micro/gather_probe.hip showed the scattered 32-B map gathers cost what the 64
lanes of one load instruction touch in distinct cache lines (the same 21 M gathers: 181 us
uniformly random, 91 us along Lissajous-like tracks, 25 us all lanes on one pixel).  Here
the C5 problem's pixel ids are relabelled onto a 2-D tiled layout before the set-up --
tiles of T x T pixels, tiles row-major, pixels inside a tile row-major or in Morton order
-- which (a) puts 2-D neighbours on the same map cache lines and (b) makes the set-up's
spatial offset order (first pixel id) cluster offsets by tile instead of by map row.
Prints ms per CG iteration (fixed 100 iterations) per layout, 1 and 4 bands, and checks
that the maps map back to the row-major solve (weight / hits identical, map <= 1e-9).
"""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from comapreduce_amd import synthetic  # noqa: E402
from comapreduce_amd.mapmaking.destriper import DeviceDestriper  # noqa: E402

NX = NY = 480


def morton2(x, y, bits):
    z = torch.zeros_like(x)
    for b in range(bits):
        z |= ((x >> b) & 1) << (2 * b)
        z |= ((y >> b) & 1) << (2 * b + 1)
    return z


def tiled_ids(T, order):
    """int64 [NY * NX]: internal id of every row-major pixel, and the padded map size."""
    p = torch.arange(NX * NY, device='cuda', dtype=torch.int64)
    y, x = p // NX, p % NX
    ntx, nty = (NX + T - 1) // T, (NY + T - 1) // T
    tx, ty, ix, iy = x // T, y // T, x % T, y % T
    if order == 'morton':
        inner = morton2(ix, iy, max(1, (T - 1).bit_length()))
    else:
        inner = iy * T + ix
    return (ty * ntx + tx) * T * T + inner, ntx * nty * T * T


def run(pix, tod, w, nb, T, order, niter=100):
    if T == 0:
        ids, npix = None, NX * NY
        pp = pix
    else:
        ids, npix = tiled_ids(T, order)
        pp = ids[pix.long()].to(torch.int32)
    dd = DeviceDestriper(pp, tod, w, 50, npix, device=0)
    dd.solve(0.0, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = dd.solve(0.0, niter)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / niter * 1e3
    conv = dd.solve(1e-6, 100)
    maps = {k: (v.reshape(nb, -1) if nb > 1 else v.reshape(1, -1)) for k, v in res['maps'].items()}
    if ids is not None:
        maps = {k: v[:, ids] for k, v in maps.items()}
    return ms, conv['iters'], maps


def main():
    out = {}
    for nb in (1, 4):
        pix, tod, w = synthetic.destriper_inputs_device(8, device=0, seed=1000, n_bands=nb)
        ref = None
        for T, order in ((0, 'row'), (2, 'row'), (4, 'row'), (4, 'morton'), (8, 'morton'), (16, 'row'),
                         (16, 'morton'), (32, 'morton'), (64, 'morton')):
            ms, its, maps = run(pix, tod, w, nb, T, order)
            key = f'{nb}band_T{T}_{order}'
            rec = {'ms_per_iter': ms, 'converged_iters': its}
            if ref is None:
                ref = maps
            else:
                rec['weight_hits_equal'] = bool(torch.equal(maps['weight'], ref['weight']) and
                                                torch.equal(maps['hits'], ref['hits']))
                d = (maps['map'] - ref['map']).abs().max() / ref['map'].abs().max()
                rec['map_rel'] = float(d)
            out[key] = rec
            print(json.dumps({key: rec}), flush=True)
        del pix, tod, w
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
