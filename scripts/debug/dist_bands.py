"""Debug: multi-rank destriper pieces with 4 batched bands vs the 1-band problem of band 0."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_gpu_destriper import _bands_problem, L, NPIX
from comapreduce_amd.mapmaking.destriper import DeviceOps

p, tods, ws, keep = _bands_problem(4)
o4 = DeviceOps(p, tods, ws, L, NPIX, keep=keep)
o1 = DeviceOps(p, tods[0], ws[0], L, NPIX)
for ops in (o1, o4):
    nb = ops.nb
    h0, _, n0 = ops.local_maps()
    NO = ops.n_offsets
    x, r, q = ops.zeros(NO * nb), ops.zeros(NO * nb), ops.zeros(NO * nb)
    num = ops.zeros(ops.npix * nb)
    ops.project(None, n0, h0, r)
    p_ = ops.copy(r)
    scal = ops.zeros(4 * nb + 1)
    ops.dot(r, r, scal[0:nb])
    scal[nb:2 * nb].copy_(scal[0:nb])
    scal[4 * nb] = 1e-6
    flags = torch.zeros(2 + 2 * nb, dtype=torch.int32, device=ops.dev)
    print('nb', nb, 'r[:4]', r[:4 * nb:nb].tolist(), 'scal', scal.tolist())
    for it in range(3):
        ops.dist_bin(p_, num, flags)
        print(' num band0 sum', float(num[0::nb].sum()))
        ops.dist_project(p_, num, h0, q, scal, flags)
        print(' q band0 [:4]', q[0:4 * nb:nb].tolist(), 'scal', scal.tolist())
        ops.dist_update(scal, x, r, p_, q, flags)
        print(' upd scal', scal.tolist())
        ops.dist_direction(scal, p_, r, flags)
        print(' dir scal', scal.tolist(), 'flags', flags.tolist())
