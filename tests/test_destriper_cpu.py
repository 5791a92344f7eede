"""Destriper: oracle pinned to the reference golden run, and the product's
distributed CG driver (comapreduce_amd.mapmaking.destriper.cg_solve) checked
on 2 CPU ranks (gloo) with the oracle's NumPy shard operators."""
import json
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from comapreduce_amd import synthetic
from oracle import destriper as od

L = 50
NPIX = 60 * 60


@pytest.fixture(scope='module')
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, 'golden_destriper.npz'))


@pytest.fixture(scope='module')
def problem(golden_dir):
    meta = json.load(open(os.path.join(golden_dir, 'golden_meta.json')))['destriper_inputs']
    p, t, w = synthetic.destriper_inputs()
    assert [synthetic.sha256(a) for a in (p, t, w)] == meta['sha256']
    return p, t, w


def test_oracle_destriper_bit_exact(problem, golden):
    p, t, w = problem
    maps, x, it = od.destriper_iteration(p, t, w, L, NPIX, threshold=1e-6, niter=100)
    assert np.array_equal(x, golden['destriper_offsets'])
    for k in ('map', 'naive', 'weight', 'hits'):
        assert np.array_equal(maps[k], golden[f'destriper_{k}']), k


def test_oracle_destriper_fixed_iterations(problem, golden):
    p, t, w = problem
    maps, x, it = od.destriper_iteration(p, t, w, L, NPIX, threshold=0.0, niter=5)
    assert it == 5
    assert np.array_equal(x, golden['destriper_offsets_niter5'])
    assert np.array_equal(maps['map'], golden['destriper_map_niter5'])


def test_cg_driver_single_rank_matches_oracle(problem):
    from comapreduce_amd.mapmaking.destriper import cg_solve
    p, t, w = problem
    ops = od.ShardOps(p, t, w, L, NPIX)
    x, it, h, nnum = cg_solve(ops, lambda a: a, threshold=1e-6, niter=100)
    _, xr, itr = od.destriper_iteration(p, t, w, L, NPIX, threshold=1e-6, niter=100)
    assert it == itr
    assert np.max(np.abs(x - xr)) <= 1e-9 * np.max(np.abs(xr))


def _rank(rank, world, port, p, t, w, q):
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import cg_solve
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.size // L
    lo, hi = (no * rank // world) * L, (no * (rank + 1) // world) * L   # whole offsets per rank

    def allreduce(a):
        dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM)
        return a

    ops = od.ShardOps(p[lo:hi], t[lo:hi], w[lo:hi], L, NPIX)
    x, it, h, nnum = cg_solve(ops, allreduce, threshold=1e-6, niter=100)
    num = np.zeros(NPIX)
    ops.bin(x, 1, num)
    allreduce(num)
    m = np.zeros(NPIX)
    ops.div_map(num, h, m)
    q.put((rank, x, it, m))
    dist.barrier()
    dist.destroy_process_group()


def test_cg_driver_two_ranks_gloo(problem):
    p, t, w = problem
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_rank, args=(r, 2, port, p, t, w, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    maps, xr, itr = od.destriper_iteration(p, t, w, L, NPIX, threshold=1e-6, niter=100)
    x = np.concatenate([res[0][1], res[1][1]])
    assert res[0][2] == res[1][2] == itr
    assert np.max(np.abs(x - xr)) <= 1e-9 * np.max(np.abs(xr))
    scale = np.max(np.abs(maps['map']))
    assert np.max(np.abs(res[0][3] - maps['map'])) <= 1e-9 * scale


def _compact_rank(rank, world, port, p, t, w, npix, q):
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import cg_solve, compact_pixels
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.size // L
    lo, hi = (no * rank // world) * L, (no * (rank + 1) // world) * L

    def allreduce(a):
        dist.all_reduce(torch.from_numpy(a) if isinstance(a, np.ndarray) else a, op=dist.ReduceOp.SUM)
        return a

    comp, idx = compact_pixels(torch.from_numpy(p[lo:hi].astype(np.int64)), npix, allreduce)
    out = []
    for pix, n in ((comp.numpy().astype(np.int64), int(idx.numel())), (p[lo:hi], npix)):
        ops = od.ShardOps(pix, t[lo:hi], w[lo:hi], L, n)
        x, it, h, nnum = cg_solve(ops, allreduce, threshold=1e-6, niter=60)
        num = np.zeros(n)
        ops.bin(x, 1, num)
        allreduce(num)
        m = np.zeros(n)
        ops.div_map(num, h, m)
        out.append((x, it, m))
    full = np.zeros(npix)
    full[idx.numpy()] = out[0][2]
    q.put((rank, idx.numpy(), out[0][0], out[0][1], full, out[1]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('wrap', [False, True])
def test_compacted_map_allreduce_two_ranks_gloo(problem, wrap):
    """compact_pixels (DeviceDestriper's multi-rank default): the map all-reduce over
    the union of the pixels the operator touches, relabelled monotonically, gives the
    same offsets and map as the full map, bit for bit (2 gloo ranks, oracle operators,
    the golden pointing placed in a 200x200 map).  wrap: the off-map samples carry
    negative ids below -1, which op_Z reads as m[npix + p] (numpy's wrap,
    Destriper.py:206-213): the union keeps those pixels and the relabelled ids stay
    negative and read the same pixel."""
    p0, t, w = problem
    big = 200
    p = np.where(p0 >= 0, (p0 // 60 + 70) * big + (p0 % 60 + 70), -1).astype(np.int64)
    if wrap:
        off = p < 0
        p[off] = -np.random.default_rng(4).integers(1, big * big + 1, int(off.sum()))
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 28500 + os.getpid() % 1000 + (7 if wrap else 0)
    procs = [ctx.Process(target=_compact_rank, args=(r, 2, port, p, t, w, big * big, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    read = np.unique(np.where(p >= 0, p, p + big * big))          # every pixel a sample bins or reads
    for rank, idx, xc, itc, mc, (xu, itu, mu) in res:
        assert np.array_equal(idx, res[0][1])                       # one union on every rank
        assert np.array_equal(idx, read) and np.all(np.diff(idx) > 0)
        assert idx.size < 0.3 * big * big
        assert itc == itu and np.array_equal(xc, xu) and np.array_equal(mc, mu), rank


def test_tiled_layout_is_a_permutation():
    """tiled_layout's internal ids (T x T tiles, Morton order inside) are distinct and
    below the padded size for power-of-two tiles on ragged maps; any other T is refused
    (its Morton code would exceed T*T - 1 and merge pixels of neighbouring tiles)."""
    import torch
    from comapreduce_amd.mapmaking.destriper import tiled_layout
    for ny, nx in ((480, 480), (37, 53), (1, 9)):
        for T in (1, 2, 8, 16):
            ids, nt = tiled_layout(ny, nx, T, torch.device('cpu'))
            assert ids.unique().numel() == ny * nx and int(ids.max()) < nt and int(ids.min()) >= 0, (ny, nx, T)
    for T in (3, 12):
        with pytest.raises(ValueError):
            tiled_layout(48, 48, T, torch.device('cpu'))


def test_device_destriper_rejects_non_power_of_two_tile(monkeypatch):
    """COMAP_DS_TILE must be 0 or a power of two: checked before any device
    work."""
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    monkeypatch.setenv('COMAP_DS_TILE', '12')
    with pytest.raises(ValueError, match='power of two'):
        DeviceDestriper(np.zeros(100, np.int32), np.zeros(100), np.ones(100), 50, 16, map_shape=(4, 4))
