"""GPU destriper vs the reference golden run (Destriper.destriper_iteration on
2 feeds x 20k samples, 60x60 map, L = 50).  Weight and hit maps are summed in
binValues' sample order -> bit-exact; offsets and maps within 1e-5 relative
(north_star), measured against max |value| since destriped maps are ~0-mean."""
import os

import numpy as np
import pytest

from comapreduce_amd import synthetic

pytestmark = pytest.mark.gpu
L = 50
NPIX = 3600


@pytest.fixture(scope='module')
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, 'golden_destriper.npz'))


def rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def test_run_destriper_matches_reference(golden):
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper, run_destriper
    p, t, w = synthetic.destriper_inputs()
    maps = run_destriper(p, t, w, L, np.arange(NPIX), threshold=1e-6, niter=100)['All']
    assert np.array_equal(maps['weight'], golden['destriper_weight'])
    assert np.array_equal(maps['hits'], golden['destriper_hits'])
    assert np.array_equal(maps['naive'], golden['destriper_naive'])
    assert rel(maps['map'], golden['destriper_map']) < 1e-5
    res = DeviceDestriper(p, t, w, L, NPIX).solve(1e-6, 100)
    assert rel(res['x'].cpu().numpy(), golden['destriper_offsets']) < 1e-5


def test_destriper_fixed_iterations_iterates(golden):
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, t, w = synthetic.destriper_inputs()
    res = DeviceDestriper(p, t, w, L, NPIX).solve(0.0, 5)
    assert res['iters'] == 5
    assert rel(res['x'].cpu().numpy(), golden['destriper_offsets_niter5']) < 1e-9
    assert rel(res['maps']['map'].cpu().numpy(), golden['destriper_map_niter5']) < 1e-9


def test_python_cg_driver_matches_native(golden):
    """The RCCL-path driver (cg_solve over DeviceOps) == the native C++ loop."""
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve
    p, t, w = synthetic.destriper_inputs()
    ops = DeviceOps(p, t, w, L, NPIX)
    x, it, h, nnum = cg_solve(ops, lambda a: a, threshold=1e-6, niter=100)
    xn, itn, _ = ops.solve_native(1e-6, 100)
    assert [it] == itn
    assert np.array_equal(ops.natural(x).cpu().numpy(), xn.cpu().numpy())


@pytest.mark.parametrize('threshold,niter', [(1e-6, 100), (0.0, 37)])
def test_batched_cg_driver_matches_native(threshold, niter):
    """The multi-rank driver (cg_solve_batched: device stop flag, 16 iterations per
    host check) == the native loop, including a count that stops mid-batch."""
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve_batched
    p, t, w = synthetic.destriper_inputs()
    ops = DeviceOps(p, t, w, L, NPIX)
    x, it, h, nnum = cg_solve_batched(ops, lambda a: a, threshold=threshold, niter=niter)
    xn, itn, _ = ops.solve_native(threshold, niter)
    assert it == itn
    assert np.array_equal(ops.natural(x).cpu().numpy(), xn.cpu().numpy())


@pytest.mark.parametrize('L,threshold,niter', [(250, 1.0, 100), (250, 0.0, 7), (50, 0.0, 37), (100, 1e-6, 100)])
def test_destriper_offset_lengths_vs_oracle(L, threshold, niter):
    """Calibrator offsets (L = 250, threshold 1: run_destriper.py:142-144), L = 100, and
    iteration counts that are not a multiple of the device graph batch, against the
    NumPy restatement of destriper_iteration (oracle/destriper.py)."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper, DeviceOps, cg_solve
    p, t, w = synthetic.destriper_inputs()
    ref, xr, itr = od.destriper_iteration(p, t, w, L, NPIX, threshold=threshold, niter=niter)
    res = DeviceDestriper(p, t, w, L, NPIX).solve(threshold, niter)
    assert res['iters'] == itr
    assert rel(res['x'].cpu().numpy(), xr) < 1e-9
    m = {k: v.cpu().numpy() for k, v in res['maps'].items()}
    assert np.array_equal(m['weight'], ref['weight'])
    assert np.array_equal(m['hits'], ref['hits'])
    assert rel(m['map'], ref['map']) < 1e-9
    # the per-call (RCCL-path) driver reproduces the graph-batched native loop exactly
    ops = DeviceOps(p, t, w, L, NPIX)
    x, it, _, _ = cg_solve(ops, lambda a: a, threshold=threshold, niter=niter)
    assert it == itr
    assert np.array_equal(ops.natural(x).cpu().numpy(), res['x'].cpu().numpy())


def _gloo_rank(rank, world, port, p, t, w, q):
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ["COMAP_DS_RANKS"] = "shard"    # the sharded CG (the default; "auto" may gather small problems)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.size // L
    lo, hi = (no * rank // world) * L, (no * (rank + 1) // world) * L   # whole offsets per rank
    res = DeviceDestriper(p[lo:hi], t[lo:hi], w[lo:hi], L, NPIX, device=0).solve(1e-6, 100)
    q.put((rank, res['x'].cpu().numpy(), res['iters'], {k: v.cpu().numpy() for k, v in res['maps'].items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_destriper_two_ranks_distributed_path(golden):
    """DeviceDestriper's multi-rank path (cg_solve over DeviceOps, map numerator,
    weights, hits and CG scalars all-reduced every iteration) on 2 ranks sharing
    cuda:0 over gloo -- the same code the RCCL run executes, with the samples
    split at an offset boundary; the joined offsets and the maps must match the
    reference golden as the single-rank solve does."""
    import torch.multiprocessing as mp
    p, t, w = synthetic.destriper_inputs()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, p, t, w, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    x = np.concatenate([res[0][1], res[1][1]])
    assert res[0][2] == res[1][2]
    assert rel(x, golden['destriper_offsets']) < 1e-5
    m = res[0][3]
    assert rel(m['weight'], golden['destriper_weight']) < 1e-12   # two partial sums, then the all-reduce
    assert np.array_equal(m['hits'], golden['destriper_hits'])
    assert rel(m['map'], golden['destriper_map']) < 1e-5
    assert rel(m['naive'], golden['destriper_naive']) < 1e-5


def _compact_rank(rank, world, port, p, t, w, npix, q, shape=None):
    """Solve this rank's half with the map all-reduces compacted to the hit pixels
    (DeviceDestriper's default across ranks) and without (COMAP_DS_COMPACT=0)."""
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ["COMAP_DS_RANKS"] = "shard"    # the sharded CG (the default; "auto" may gather small problems)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.shape[-1] // L
    lo, hi = (no * rank // world) * L, (no * (rank + 1) // world) * L
    out = []
    for compact in ('1', '0'):
        os.environ['COMAP_DS_COMPACT'] = compact
        prob = DeviceDestriper(p[lo:hi], t[..., lo:hi], w[..., lo:hi], L, npix, device=0, map_shape=shape)
        res = prob.solve(1e-6, 60)
        out.append((prob.hit_index is not None, res['x'].cpu().numpy(), res['iters'],
                    {k: v.cpu().numpy() for k, v in res['maps'].items()}))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('nb,wrap,tile', [(1, False, False), (4, False, False), (4, True, False), (4, True, True)])
def test_two_ranks_compacted_map_allreduce_bit_identical(nb, wrap, tile):
    """Across ranks the map numerator is all-reduced over the union of the pixels the
    operator touches only (a monotone relabelling; the pixels unbinned samples read,
    m[npix + p], are kept): on a 200x200 map the golden pointing covers ~9%, and
    offsets, iteration counts and every map equal the uncompacted solve bit for bit,
    on 2 gloo ranks.  wrap: off-map ids spread over [-npix, -1]; tile: both solves on the
    2-D tiled pixel layout (map_shape), maps returned in the caller's order."""
    import torch.multiprocessing as mp
    p0, tods, ws, _ = _bands_problem(4)
    big = 200
    p = np.where(p0 >= 0, (p0 // 60 + 70) * big + (p0 % 60 + 70), -1).astype(np.int64)
    if wrap:
        off = p < 0
        p[off] = -np.random.default_rng(9).integers(1, big * big + 1, int(off.sum()))
    t, w = (tods, ws) if nb == 4 else (tods[0], ws[0])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 190 + (3 if wrap else 0) + nb + (7 if tile else 0)
    shape = (big, big) if tile else None
    procs = [ctx.Process(target=_compact_rank, args=(r, 2, port, p, t, w, big * big, q, shape)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    for rank, ((on, xc, ic, mc), (off, xu, iu, mu)) in res:
        assert on and not off
        assert ic == iu
        assert np.array_equal(xc, xu), rank
        for k in mu:
            assert mc[k].shape == mu[k].shape and np.array_equal(mc[k], mu[k]), (rank, k)
    assert np.count_nonzero(res[0][1][0][3]['hits']) < 0.25 * big * big * (4 if nb == 4 else 1)


def _uneven_rank(rank, world, port, p, t, w, frac, q):
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ["COMAP_DS_RANKS"] = "shard"    # the sharded CG (the default; "auto" may gather small problems)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.shape[-1] // L
    cut = int(no * frac) * L
    lo, hi = (0, cut) if rank == 0 else (cut, t.shape[-1])
    res = DeviceDestriper(p[lo:hi], t[..., lo:hi], w[..., lo:hi], L, NPIX, device=0).solve(1e-6, 100)
    q.put((rank, res['x'].cpu().numpy(), res['iters'], {k: v.cpu().numpy() for k, v in res['maps'].items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('nb', [1, 4])
def test_two_ranks_uneven_split_matches_single_rank(nb):
    """The multi-rank CG all-reduces the p.q / r.r block partials (native kernels, no
    final-sum launches); ranks with different grids (80 / 20 % of the offsets) must
    clear the partial slots they do not write.  Offsets and maps == the single-rank
    native solve to 1e-9, same iteration counts."""
    import torch.multiprocessing as mp
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, tods, ws, _ = _bands_problem(4)
    t, w = (tods, ws) if nb == 4 else (tods[0], ws[0])
    ref = DeviceDestriper(p, t, w, L, NPIX).solve(1e-6, 100)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29300 + os.getpid() % 190
    procs = [ctx.Process(target=_uneven_rank, args=(r, 2, port, p, t, w, 0.8, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    assert res[0][2] == res[1][2] == ref['iters']
    x = np.concatenate([res[0][1], res[1][1]], axis=-1)
    assert rel(x, ref['x'].cpu().numpy()) < 1e-9
    for k in ('map', 'naive', 'weight', 'hits'):
        assert rel(res[0][3][k], ref['maps'][k].cpu().numpy()) < 1e-9, k


def _gather_rank(rank, world, port, p, t, w, keep, policy, q):
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['COMAP_DS_RANKS'] = policy
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    no = t.shape[-1] // L
    lo, hi = (no * rank // world), (no * (rank + 1) // world)
    k = None if keep is None else keep[:, lo:hi]
    prob = DeviceDestriper(p[lo * L:hi * L], t[..., lo * L:hi * L], w[..., lo * L:hi * L], L, NPIX, device=0, keep=k)
    res = prob.solve(1e-6, 100)
    q.put((rank, prob.gathered is not None, None if prob.plan is None else prob.plan['mode'], res['x'].cpu().numpy(),
           res['iters'], {kk: v.cpu().numpy() for kk, v in res['maps'].items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('nb,policy', [(1, 'auto'), (4, 'auto'), (3, 'gather')])
def test_two_ranks_gathered_solve_equals_single_rank(nb, policy):
    """A problem the rank model (mapmaking/rankplan.py) finds latency-bound across ranks
    -- the golden pointing, 40k samples -- is gathered to rank 0 and solved there alone:
    every rank's offsets and the maps equal the single-rank native solve bit for bit
    (same operator, same order), on 2 gloo ranks; 3 bands exercise the padded band."""
    import torch.multiprocessing as mp
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, tods, ws, keep = _bands_problem(4)
    if nb == 1:
        t, w, keep = tods[0], ws[0], None
    else:
        t, w, keep = tods[:nb], ws[:nb], keep[:nb].astype(np.uint8)
    ref = DeviceDestriper(p, t, w, L, NPIX, keep=keep).solve(1e-6, 100)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29100 + os.getpid() % 190
    procs = [ctx.Process(target=_gather_rank, args=(r, 2, port, p, t, w, keep, policy, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    for rank, gathered, mode, x, it, maps in res:
        assert gathered, rank
        if policy == 'auto':
            assert mode == 'gather'
        assert it == ref['iters']
        for k in ('map', 'naive', 'weight', 'hits'):
            assert np.array_equal(maps[k], ref['maps'][k].cpu().numpy()), (rank, k)
    x = np.concatenate([res[0][3], res[1][3]], axis=-1)
    assert np.array_equal(x, ref['x'].cpu().numpy())


# ---------------------------------------------------------------- batched bands
def _bands_problem(nb=4, seed=11):
    """The golden problem's pointing with nb sidebands: per-band tod and weight
    scales, and per-band offsets whose weights are all zero (what each band's
    read_comap_data would drop, COMAPData.py:550-568)."""
    p, t, w = synthetic.destriper_inputs()
    rng = np.random.default_rng(seed)
    NO = t.size // L
    tods = np.stack([t * (1.0 + 0.1 * b) + 0.01 * b * rng.standard_normal(t.size) for b in range(nb)])
    ws = np.stack([w * rng.uniform(0.5, 1.5) for b in range(nb)])
    keep = np.ones((nb, NO), dtype=bool)
    for b in range(1, nb):
        drop = rng.choice(NO, 25 * b, replace=False)
        keep[b, drop] = False
        ws[b].reshape(NO, L)[drop] = 0.0
    return p, tods, ws, keep


@pytest.mark.parametrize('nb,threshold,niter', [(4, 1e-6, 100), (4, 0.0, 37), (2, 1e-6, 100), (3, 1e-8, 60)])
def test_batched_bands_vs_per_band_oracle(nb, threshold, niter):
    """nb sidebands solved as one batched system == each band solved alone (on its
    own kept samples) by the oracle's destriper_iteration: weight / hits / naive
    bit-exact, offsets and map <= 1e-9, the same iteration count per band."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, tods, ws, keep = _bands_problem(nb)
    res = DeviceDestriper(p, tods, ws, L, NPIX, keep=keep).solve(threshold, niter)
    assert len(res['iters']) == nb
    for b in range(nb):
        sel = np.repeat(keep[b], L)
        ref, xr, itr = od.destriper_iteration(p[sel], tods[b][sel], ws[b][sel], L, NPIX, threshold=threshold,
                                              niter=niter)
        assert res['iters'][b] == itr, (b, res['iters'], itr)
        m = {k: v[b].cpu().numpy() for k, v in res['maps'].items()}
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(m[k], ref[k]), (b, k)
        assert rel(m['map'], ref['map']) < 1e-9, b
        x = res['x'][b].cpu().numpy()
        assert rel(x[keep[b]], xr) < 1e-9, b
        assert not x[~keep[b]].any()


def test_batched_bands_multirank_driver_matches_native():
    """The multi-rank driver (cg_solve_batched, per-band device stop flags) on a
    batched 4-band problem == its native graph-batched solve, bit for bit."""
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve_batched
    p, tods, ws, keep = _bands_problem(4)
    ops = DeviceOps(p, tods, ws, L, NPIX, keep=keep)
    x, it, _, _ = cg_solve_batched(ops, lambda a: a, threshold=1e-6, niter=100)
    xn, itn, _ = ops.solve_native(1e-6, 100)
    assert it == itn
    assert np.array_equal(ops.natural(x).cpu().numpy(), xn.cpu().numpy())


@pytest.mark.parametrize('niter', [37, 100])
def test_graph_driver_matches_batched(niter):
    """The captured-graph multi-rank driver (kernels + collectives of 16 iterations
    per replay) == the eager batched driver, bit for bit (one rank, identity sums)."""
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve_batched, cg_solve_graph
    p, tods, ws, keep = _bands_problem(4)
    ops = DeviceOps(p, tods, ws, L, NPIX, keep=keep)
    xg, itg, _, _ = cg_solve_graph(ops, lambda a: a, threshold=1e-6, niter=niter)
    xb, itb, _, _ = cg_solve_batched(ops, lambda a: a, threshold=1e-6, niter=niter)
    assert itg == itb
    assert np.array_equal(xg.cpu().numpy(), xb.cpu().numpy())


def test_library_calls_after_capture_on_another_stream():
    """After the graph driver's capture (library temporaries may be freed while the stream
    is capturing: their reuse event is null), calls bound to a different stream take fresh
    or safely reusable blocks and leave no stale HIP error behind for the next launch check
    (capi.hip make_safe / comap_upload clear the error of a failed query)."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper, DeviceOps, cg_solve_graph
    from comapreduce_amd.tools.medfilt import medfilt_batch
    import oracle
    p, tods, ws, keep = _bands_problem(4)
    ops = DeviceOps(p, tods, ws, L, NPIX, keep=keep)
    cg_solve_graph(ops, lambda a: a, threshold=1e-6, niter=20)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        N.bind_stream(N.ctx(0), torch.device('cuda', 0))
        x = np.random.default_rng(2).standard_normal(5000)
        got = medfilt_batch([x], 401, reflect=True)[0]
        z = np.concatenate((x[::-1], x, x[::-1]))
        assert np.array_equal(got, oracle.medfilt(z, 401)[x.size:2 * x.size])
        r = DeviceDestriper(p, tods[0], ws[0], L, NPIX).solve(1e-6, 100)
        assert r['iters'] > 0
    torch.cuda.synchronize()
    N.bind_stream(N.ctx(0), torch.device('cuda', 0))


def _nccl_graph_rank(port, q):
    """One-rank RCCL process group: the graph driver captures real ncclAllReduce calls."""
    import torch
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve_batched, cg_solve_graph
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))

    def ar(t):
        dist.all_reduce(t)
        return t
    p, tods, ws, keep = _bands_problem(4)
    ops = DeviceOps(p, tods, ws, L, NPIX, keep=keep)
    xg, itg, _, _ = cg_solve_graph(ops, ar, threshold=1e-6, niter=48)
    xb, itb, _, _ = cg_solve_batched(ops, ar, threshold=1e-6, niter=48)
    q.put((itg, itb, bool(np.array_equal(xg.cpu().numpy(), xb.cpu().numpy()))))
    dist.destroy_process_group()


def test_graph_driver_captures_rccl_allreduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29900 + os.getpid() % 90
    pr = ctx.Process(target=_nccl_graph_rank, args=(port, q))
    pr.start()
    itg, itb, same = q.get(timeout=240)
    pr.join(timeout=60)
    assert itg == itb and same


@pytest.mark.parametrize('form,nb', [('count', 1), ('count', 4), ('count', 2), ('full', 1), ('full', 4),
                                     ('nonuniform', 1), ('nonuniform', 4), ('sell-count', 1), ('sell-count', 4),
                                     ('sell-count', 2), ('sell-full', 1), ('sell-full', 4)])
def test_entry_forms_vs_oracle(form, nb, monkeypatch):
    """The operator's two entry forms against the oracle: the count form (uint8
    non-zero-sample counts per band, s_e = wbar_o c_e; chosen when every offset's
    non-zero weights are one value per band, as COMAP's per-(feed, band) weights with
    zeroed cuts are), the f64 weight sums (COMAP_DS_CF=0), and weights that vary inside
    an offset (the set-up falls back to the f64 form by itself).  Same solve to 1e-9,
    weight / hits bit-exact, the same iteration counts.  sell-*: the projection on the
    sliced-ELLPACK copy of the offset rows (COMAP_DS_SELL=1), both entry forms."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    if form.startswith('sell-'):
        monkeypatch.setenv('COMAP_DS_SELL', '1')
        form = form[5:]
    if form == 'full':
        monkeypatch.setenv('COMAP_DS_CF', '0')
    p, tods, ws, keep = _bands_problem(max(nb, 2))
    tods, ws, keep = tods[:nb], ws[:nb], keep[:nb]
    if form == 'nonuniform':
        ws = ws * np.random.default_rng(5).uniform(0.5, 2.0, ws.shape)
    want_bytes = 4 + nb if form == 'count' else 4 + 8 * nb
    if nb == 1:
        dd = DeviceDestriper(p, tods[0], ws[0], L, NPIX)
        assert dd.entry_bytes() == want_bytes
        res = dd.solve(1e-6, 100)
        ref, xr, itr = od.destriper_iteration(p, tods[0], ws[0], L, NPIX, threshold=1e-6, niter=100)
        assert res['iters'] == itr
        assert rel(res['x'].cpu().numpy(), xr) < 1e-9
        m = {k: v.cpu().numpy() for k, v in res['maps'].items()}
        assert np.array_equal(m['weight'], ref['weight']) and np.array_equal(m['hits'], ref['hits'])
        assert rel(m['map'], ref['map']) < 1e-9
        return
    dd = DeviceDestriper(p, tods, ws, L, NPIX, keep=keep)
    assert dd.entry_bytes() == want_bytes
    res = dd.solve(1e-6, 100)
    for b in range(nb):
        sel = np.repeat(keep[b], L)
        ref, xr, itr = od.destriper_iteration(p[sel], tods[b][sel], ws[b][sel], L, NPIX, threshold=1e-6, niter=100)
        assert res['iters'][b] == itr
        m = {k: v[b].cpu().numpy() for k, v in res['maps'].items()}
        assert np.array_equal(m['weight'], ref['weight']) and np.array_equal(m['hits'], ref['hits'])
        assert rel(m['map'], ref['map']) < 1e-9, b
        assert rel(res['x'][b].cpu().numpy()[keep[b]], xr) < 1e-9, b


@pytest.mark.parametrize('nb,sell', [(1, '0'), (1, '1'), (4, '0'), (4, '1')])
def test_negative_pixel_ids_wrap_vs_oracle(nb, sell, monkeypatch):
    """op_Z reads m[pointing] (Destriper.py:206-213): a negative pixel id p in [-npix, -1]
    is never binned (binValues skips it, binFuncs.pyx:28) but its sample's projection
    reads m[npix + p] -- numpy's wrap, not only m[-1].  The golden problem's off-map
    samples get random ids in [-npix, -1]; CSR and sliced-ELLPACK projections, 1 and 4
    bands, against the oracle (plain NumPy indexing): weight / hits bit-exact, offsets
    and map <= 1e-9, equal iteration counts.  Ids below -npix raise IndexError, as
    numpy does."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    monkeypatch.setenv('COMAP_DS_SELL', sell)
    p, tods, ws, keep = _bands_problem(max(nb, 2))
    p = p.copy()
    off = p < 0
    assert off.sum() > 100
    p[off] = -np.random.default_rng(8).integers(1, NPIX + 1, int(off.sum()))
    if nb == 1:
        res = DeviceDestriper(p, tods[0], ws[0], L, NPIX).solve(1e-6, 100)
        ref, xr, itr = od.destriper_iteration(p, tods[0], ws[0], L, NPIX, threshold=1e-6, niter=100)
        assert res['iters'] == itr
        assert rel(res['x'].cpu().numpy(), xr) < 1e-9
        m = {k: v.cpu().numpy() for k, v in res['maps'].items()}
        assert np.array_equal(m['weight'], ref['weight']) and np.array_equal(m['hits'], ref['hits'])
        assert rel(m['map'], ref['map']) < 1e-9
        # the old behaviour (every negative id reads m[-1]) is a different operator
        _, xo, _ = od.destriper_iteration(np.where(p < 0, -1, p), tods[0], ws[0], L, NPIX, threshold=1e-6, niter=100)
        assert rel(xo, xr) > 1e-6
    else:
        res = DeviceDestriper(p, tods[:nb], ws[:nb], L, NPIX, keep=keep[:nb]).solve(1e-6, 100)
        for b in range(nb):
            sel = np.repeat(keep[b], L)
            ref, xr, itr = od.destriper_iteration(p[sel], tods[b][sel], ws[b][sel], L, NPIX, threshold=1e-6,
                                                  niter=100)
            assert res['iters'][b] == itr
            m = {k: v[b].cpu().numpy() for k, v in res['maps'].items()}
            assert np.array_equal(m['weight'], ref['weight']) and np.array_equal(m['hits'], ref['hits'])
            assert rel(m['map'], ref['map']) < 1e-9, b
            assert rel(res['x'][b].cpu().numpy()[keep[b]], xr) < 1e-9, b
    bad = p.copy()
    bad[7] = -NPIX - 1
    with pytest.raises(IndexError):
        DeviceDestriper(bad, tods[0], ws[0], L, NPIX)


@pytest.mark.parametrize('nb,wrap', [(1, False), (4, False), (3, True)])
def test_tiled_layout_equals_row_major(nb, wrap, monkeypatch):
    """map_shape: the operator on the 2-D tiled internal pixel order (T x T tiles, Morton
    inside) -- a relabelling, so the sample-level maps (weight / hits / naive) are equal
    bit for bit, offsets and map <= 1e-9 (other summation orders), the same iteration
    counts, and the maps come back in the caller's row-major order (device and to_host
    paths).  wrap: negative ids below -1 read the same pixel through the relabel."""
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, tods, ws, keep = _bands_problem(4)
    p = p.copy()
    if wrap:
        off = p < 0
        p[off] = -np.random.default_rng(12).integers(1, NPIX + 1, int(off.sum()))
    if nb == 1:
        args, kw = (p, tods[0], ws[0], L, NPIX), {}
    else:
        args, kw = (p, tods[:nb], ws[:nb], L, NPIX), {'keep': keep[:nb]}
    monkeypatch.setenv('COMAP_DS_TILE', '0')
    ref = DeviceDestriper(*args, map_shape=(60, 60), **kw)
    assert ref.layout is None
    r0 = ref.solve(1e-6, 100)
    for T in ('8', '16'):
        monkeypatch.setenv('COMAP_DS_TILE', T)
        dd = DeviceDestriper(*args, map_shape=(60, 60), **kw)
        assert dd.layout is not None and dd.npix_full >= NPIX
        res = dd.solve(1e-6, 100)
        assert res['iters'] == r0['iters']
        m = {k: v.cpu().numpy() for k, v in res['maps'].items()}
        m0 = {k: v.cpu().numpy() for k, v in r0['maps'].items()}
        for k in ('weight', 'hits', 'naive'):
            assert m[k].shape == m0[k].shape and np.array_equal(m[k], m0[k]), (T, k)
        assert rel(m['map'], m0['map']) < 1e-9
        assert rel(res['x'].cpu().numpy(), r0['x'].cpu().numpy()) < 1e-9
        hres = dd.solve(1e-6, 100, to_host=True)
        for k in ('weight', 'hits', 'naive', 'map'):
            assert np.array_equal(np.asarray(hres['maps'][k]), m[k]), (T, k)
    with pytest.raises(ValueError):
        DeviceDestriper(*args, map_shape=(60, 61), **kw)


@pytest.mark.parametrize('ny,nx,T', [(37, 53, 8), (480, 480, 8), (480, 480, 16), (64, 1, 4), (9, 130, 2)])
def test_relabel_tiled_equals_table(ny, nx, T):
    """comap_relabel_pixels_tiled (the layout's ids computed per id) == comap_relabel_pixels
    through tiled_layout's table, for ids in range, negative ids and out-of-range ids."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd.mapmaking.destriper import tiled_layout
    npix = ny * nx
    ids, nt = tiled_layout(ny, nx, T, torch.device('cuda', 0))
    rng = np.random.default_rng(4)
    p = rng.integers(-npix - 40, npix + 40, 100_003).astype(np.int32)
    p[:4] = [0, npix - 1, -1, -npix]
    pd = torch.from_numpy(p).cuda()
    a, b = torch.empty_like(pd), torch.empty_like(pd)
    c = N.ctx(0)
    N.bind_stream(c, torch.device('cuda', 0))
    N.check(N.lib().comap_relabel_pixels(c, N.dptr(pd), pd.numel(), N.dptr(ids), npix, nt, N.dptr(a)), c, 'lut')
    N.check(N.lib().comap_relabel_pixels_tiled(c, N.dptr(pd), pd.numel(), nx, ny, T, N.dptr(b)), c, 'tiled')
    assert torch.equal(a, b)


def test_relabel_pixels_kernel():
    """comap_relabel_pixels (the tiled layout's one-pass relabel) against its numpy
    statement: ids in [0, npix) through the table, ids in [-npix, 0) to the negative id
    that reads the same internal pixel, anything else to n_internal."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd.mapmaking.destriper import tiled_layout
    ny, nx, T = 37, 53, 8
    npix = ny * nx
    ids, nt = tiled_layout(ny, nx, T, torch.device('cuda', 0))
    rng = np.random.default_rng(3)
    p = rng.integers(-npix - 40, npix + 40, 200_003).astype(np.int32)
    p[:4] = [0, npix - 1, -1, -npix]
    pd = torch.from_numpy(p).cuda()
    out = torch.empty_like(pd)
    c = N.ctx(0)
    N.bind_stream(c, torch.device('cuda', 0))
    N.check(N.lib().comap_relabel_pixels(c, N.dptr(pd), pd.numel(), N.dptr(ids), npix, nt, N.dptr(out)), c, 'relabel')
    lut = ids.cpu().numpy().astype(np.int64)
    q = p.astype(np.int64)
    want = np.where((q >= npix) | (q < -npix), nt,
                    np.where(q >= 0, lut[np.clip(q, 0, npix - 1)], lut[np.clip(q + npix, 0, npix - 1)] - nt))
    assert np.array_equal(out.cpu().numpy().astype(np.int64), want)


@pytest.mark.parametrize('nb', [1, 3, 4])
def test_solve_to_host_equals_device_maps(nb):
    """solve(to_host=True) -- naive / weight / hits copied during the CG on a copy
    stream, the map after it -- returns bit for bit what solve() + maps_to_host do."""
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper, maps_to_host
    p, tods, ws, keep = _bands_problem(max(nb, 2))
    if nb == 1:
        args = (p, tods[0], ws[0], L, NPIX)
        kw = {}
    else:
        args = (p, tods[:nb], ws[:nb], L, NPIX)
        kw = {'keep': keep[:nb]}
    dev = DeviceDestriper(*args, **kw).solve(1e-6, 100)
    want = maps_to_host(dev['maps'])
    got = DeviceDestriper(*args, **kw).solve(1e-6, 100, to_host=True)
    assert got['iters'] == dev['iters']
    assert np.array_equal(got['x'].cpu().numpy(), dev['x'].cpu().numpy())
    assert set(got['maps']) == set(want)
    for k, v in want.items():
        assert got['maps'][k].shape == v.shape, k
        assert np.array_equal(got['maps'][k], v), k


@pytest.mark.parametrize('case,Lc,nb', [('walk', 50, 4), ('payload', 50, 4), ('walk', 100, 1), ('walk', 250, 2),
                                        ('heavy', 50, 4), ('heavy', 100, 2), ('noprefetch', 50, 4), ('xcd', 50, 4),
                                        ('zeros', 50, 4), ('nonfinite', 50, 1), ('nonfinite', 50, 4)])
def test_sample_maps_set_up_paths(case, Lc, nb, monkeypatch):
    """The set-up's sample-level maps (weight, hits, naive: binValues' sample order, so
    bit-exact) on each of its paths against the oracle: the member-mask walk (default;
    member masks of 1, 2 and 4 words for L = 50, 100, 250), the sorted-sample payload walk
    (COMAP_DS_WALK=0), the walk with most rows taken from its heavy-row list first
    (COMAP_DS_HEAVY=2), without the record prefetch (COMAP_DS_WPF=0), with the rows dealt to
    the XCDs in contiguous ranges (COMAP_DS_WXCD=1), kept offsets holding all-zero-weight pixel
    groups (their hits come
    from the count pass's integer adds), and non-finite tod on zero-weight samples (the
    set-up falls back to the payload walk, whose NaN reaches the naive map as
    binValues' does; the solve itself is not compared there)."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    if case == 'payload':
        monkeypatch.setenv('COMAP_DS_WALK', '0')
    if case == 'heavy':
        monkeypatch.setenv('COMAP_DS_HEAVY', '2')
    if case == 'noprefetch':
        monkeypatch.setenv('COMAP_DS_WPF', '0')
    if case == 'xcd':
        monkeypatch.setenv('COMAP_DS_WXCD', '1')
    p, tods, ws, keep = _bands_problem(max(nb, 2))
    tods, ws, keep = tods[:nb].copy(), ws[:nb].copy(), keep[:nb]
    if Lc != L:                       # whole offsets of the new length, no band drops
        n = p.size // Lc * Lc
        p, tods, ws = p[:n], tods[:, :n], ws[:, :n]
        keep = np.ones((nb, n // Lc), dtype=bool)
        ws[ws == 0] = 1.0
    rng = np.random.default_rng(3)
    if case in ('zeros', 'nonfinite'):
        zero = rng.choice(p.size, p.size // 20, replace=False)
        ws[:, zero] = 0.0
    if case == 'nonfinite':
        tods[:, zero[:7]] = np.nan
        tods[:, zero[7:9]] = np.inf
    dd = DeviceDestriper(p, tods if nb > 1 else tods[0], ws if nb > 1 else ws[0], Lc, NPIX,
                         keep=keep if nb > 1 else None)
    finite = case != 'nonfinite'
    res = dd.solve(1e-6 if finite else 0.0, 100 if finite else 2)
    for b in range(nb):
        sel = np.repeat(keep[b], Lc)
        ref, xr, itr = od.destriper_iteration(p[sel], tods[b][sel], ws[b][sel], Lc, NPIX,
                                              threshold=1e-6 if finite else 0.0, niter=100 if finite else 2)
        m = {k: (v[b] if nb > 1 else v).cpu().numpy() for k, v in res['maps'].items()}
        assert np.array_equal(m['weight'], ref['weight']), (case, b)
        assert np.array_equal(m['hits'], ref['hits']), (case, b)
        assert np.array_equal(m['naive'], ref['naive'], equal_nan=True), (case, b)
        if finite:
            assert (res['iters'][b] if nb > 1 else res['iters']) == itr
            assert rel(m['map'], ref['map']) < 1e-9, (case, b)


def test_pixel_out_of_range_raises():
    """A pixel index >= npix is an error (the reference's binning would index past the
    map); the set-up's count pass finds it on the device."""
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    p, t, w = synthetic.destriper_inputs()
    p = p.copy()
    p[1234] = NPIX
    with pytest.raises(IndexError):
        DeviceDestriper(p, t, w, L, NPIX)


@pytest.mark.parametrize('L,nx,ny,n_off', [(50, 480, 480, 1000), (64, 37, 53, 300), (100, 60, 60, 257), (1, 9, 7, 130)])
def test_offset_centroid_keys_vs_numpy(L, nx, ny, n_off):
    """comap_offset_centroid_keys (the LDS-staged kernel for L <= 64, the wave-per-offset one
    above) against NumPy: lut[round(mean y) nx + round(mean x)] over an offset's on-map
    samples (0 <= p < nx ny; round half up), n_internal for an offset with none."""
    import torch
    from comapreduce_amd import _native as N
    rng = np.random.default_rng(L + nx)
    npix = nx * ny
    pix = rng.integers(-3, npix + 3, size=n_off * L).astype(np.int32)
    pix[:L] = -1                                            # an offset with no on-map sample
    pix[L:2 * L] = npix - 1
    lut = rng.permutation(npix).astype(np.int32)
    n_internal = npix + 5
    dev = torch.device('cuda', 0)
    tp, tl = torch.from_numpy(pix).to(dev), torch.from_numpy(lut).to(dev)
    keys = torch.empty(n_off, dtype=torch.int32, device=dev)
    c = N.ctx(0)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_offset_centroid_keys(c, N.dptr(tp), pix.size, L, nx, ny, N.dptr(tl), n_internal,
                                               N.dptr(keys)), c, 'comap_offset_centroid_keys')
    got = keys.cpu().numpy()
    want = np.full(n_off, n_internal, dtype=np.int64)
    for o in range(n_off):
        p = pix[o * L:(o + 1) * L].astype(np.int64)
        p = p[(p >= 0) & (p < npix)]
        if p.size:
            c_ = p.size
            yi = (2 * (p // nx).sum() + c_) // (2 * c_)
            xi = (2 * (p % nx).sum() + c_) // (2 * c_)
            want[o] = lut[yi * nx + xi]
    assert np.array_equal(got, want)
