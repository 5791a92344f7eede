"""Full-size C2 parity (BASELINE configs[1]): the 19-feed x 4 x 1024 x 180,000
observation (56 GB f32, generated on device exactly as bench.py does) reduced
by the three device stages, checked against the CPU oracle (oracle/l1.py,
pinned to the reference goldens) on (feed, scan) units that cover the first,
a middle and the last feed and the first, middle and last scans:

  * vane Tsys / gain of each checked feed: bit-exact (VaneCalibration.py:67-198);
  * atmosphere fit of each unit: <= 1e-5 relative (Level1Averaging.py:197-227);
  * averaged_tod tod / tod_original / weights of each unit: <= 1e-5 relative
    (Level1Averaging.py:792-872, north_star tolerance);
  * shapes and the finite / zero pattern of every averaged_tod array.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
RTOL = 1e-5
F, T = 19, 180_000


def relmax(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), 'NaN pattern differs'
    return np.max(np.abs(a[fin] - b[fin])) / max(np.max(np.abs(b[fin])), 1e-300)


@pytest.fixture(scope='module')
def c2():
    import torch
    import bench
    from comapreduce_amd.pipeline.datahandling import to_host
    data, sh = bench.build_observation(F, T, obs_id=1, device=0)
    level2 = bench.reduce_step(data, 0)
    torch.cuda.synchronize()
    host = {k: to_host(level2[k]) for k in ('vane/system_temperature', 'vane/system_gain', 'atmosphere/fit_values',
                                            'averaged_tod/tod', 'averaged_tod/tod_original',
                                            'averaged_tod/weights')}
    host['averaged_tod/scan_edges'] = np.asarray(level2['averaged_tod/scan_edges'])
    yield data, sh, host
    del data, level2
    torch.cuda.empty_cache()


def test_c2_shapes_and_patterns(c2):
    data, sh, h = c2
    edges = h['averaged_tod/scan_edges']
    S = len(edges)
    assert S >= 10
    assert h['vane/system_temperature'].shape == (1, F, 4, 1024)
    assert h['atmosphere/fit_values'].shape == (S, F, 4, 2, 1024)
    inside = np.zeros(T, dtype=bool)
    for s, e in edges:
        inside[s:e] = True
    for k in ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
        a = h[k]
        assert a.shape == (F, 4, T), k
        assert np.isfinite(a).all(), k
        assert not a[..., ~inside].any(), k          # samples outside every scan stay 0
        assert (a[..., inside] != 0).mean() > 0.999, k
    fit = h['atmosphere/fit_values']
    fitted = np.zeros(1024, dtype=bool)
    fitted[10:1014] = True
    fitted[510:515] = False                          # Level1Averaging.py:201-202
    assert np.isfinite(fit[..., fitted]).all()
    assert np.isnan(fit[..., ~fitted]).all()
    # every scan's weights are constant per (feed, band, scan) (1/auto_rms^2)
    w = h['averaged_tod/weights']
    for s, e in edges:
        seg = w[..., s:e]
        assert np.array_equal(seg, np.broadcast_to(seg[..., :1], seg.shape))


@pytest.mark.parametrize('f,which', [(0, 'first'), (9, 'middle'), (18, 'last'), (5, 'first'), (13, 'middle')])
def test_c2_units_vs_oracle(c2, f, which):
    import oracle.l1 as ol1
    data, sh, h = c2
    edges = h['averaged_tod/scan_edges']
    s = {'first': 0, 'middle': len(edges) // 2, 'last': len(edges) - 1}[which]
    t0, t1 = (int(v) for v in edges[s])
    tod_f = data['spectrometer/tod'][f].cpu().numpy()
    ba_f = data['spectrometer/band_average'][f].cpu().numpy()
    el = np.asarray(data['spectrometer/pixel_pointing/pixel_el'])[f]
    A = 1.0 / np.sin(el * np.pi / 180.0)
    # vane (event 0) of this feed: bit-exact
    tsys, gain = ol1.measure_system_temperature(tod_f[None], ba_f[None], data.features, data.vane_temperature)
    assert np.array_equal(h['vane/system_temperature'][:, f], tsys[:, 0])
    assert np.array_equal(h['vane/system_gain'][:, f], gain[:, 0])
    # atmosphere fit of the unit
    fit = np.stack([np.stack(ol1.fit_atmosphere(A[t0:t1], tod_f[b, :, t0:t1])) for b in range(4)])
    assert relmax(h['atmosphere/fit_values'][s, f], fit) < RTOL
    # the unit's Level-2 TOD
    r, o, w, _ = ol1.reduce_scan(tod_f[..., t0:t1].copy(), A[t0:t1], h['atmosphere/fit_values'][s, f],
                                 tsys[0, 0], gain[0, 0], is_first_scan=(s == 0))
    assert relmax(h['averaged_tod/tod'][f, :, t0:t1], r) < RTOL
    assert relmax(h['averaged_tod/tod_original'][f, :, t0:t1], o) < RTOL
    assert relmax(h['averaged_tod/weights'][f, :, t0:t1], np.broadcast_to(w[:, None], (4, t1 - t0))) < RTOL


# ---------------------------------------------------------------- C3: the 8-way (feed, scan) split
C3_WORLD = 8


def c3_ranks(edges):
    """Rank 0, the first middle rank whose first feed is cut between it and the rank
    before (its first unit is not scan 0), and the last rank of the 8-way split."""
    from comapreduce_amd.pipeline.sharding import shard_for
    mid = next(r for r in range(1, C3_WORLD - 1) if int(shard_for(edges, F, r, C3_WORLD).units[0, 1]) != 0)
    return {'first': 0, 'cut': mid, 'last': C3_WORLD - 1}


@pytest.mark.parametrize('which', ['first', 'cut', 'last'])
def test_c3_shard_bit_identical(c2, which):
    """C3 (BASELINE configs[2]): one rank's shard of the 8-way (feed, scan) split of the
    full C2 observation, generated and reduced alone exactly as bench.py --gpus 8 does
    on that rank (its feeds only, its units only, no collective).  Its owned slices of
    averaged_tod/*, atmosphere/fit_values and the vane of every feed it holds equal the
    unsharded run's bit for bit (sharding.assemble semantics; run_average.py:38-39 split
    files, this splits one observation's units)."""
    import torch
    import bench
    from comapreduce_amd.pipeline.datahandling import to_host
    _, _, h = c2
    r = c3_ranks(h['averaged_tod/scan_edges'])[which]
    data, sh = bench.build_observation(F, T, obs_id=1, device=0, rank=r, world=C3_WORLD)
    assert sh.units.size and sh.n_feeds < F
    if which == 'cut':
        assert int(sh.units[0, 1]) != 0            # its first feed's earlier scans belong to rank r - 1
    level2 = bench.reduce_step(data, 0)
    torch.cuda.synchronize()
    got = {k: to_host(level2[k]) for k in ('vane/system_temperature', 'vane/system_gain', 'atmosphere/fit_values',
                                           'averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights')}
    del data, level2
    torch.cuda.empty_cache()
    for f, s, t0, n in sh.units:
        fl = f - sh.f_lo
        for k in ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights'):
            assert np.array_equal(got[k][fl, :, t0:t0 + n], h[k][f, :, t0:t0 + n]), (r, f, s, k)
        assert np.array_equal(got['atmosphere/fit_values'][s, fl], h['atmosphere/fit_values'][s, f],
                              equal_nan=True), (r, f, s)
    for k in ('vane/system_temperature', 'vane/system_gain'):
        assert np.array_equal(got[k], h[k][:, sh.f_lo:sh.f_hi]), (r, k)


# ---------------------------------------------------------------- C4 / C5 destriper parity
def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.fixture(scope='module')
def c4(c2):
    """C4 inputs: COMAPData.read_comap_data (band 0, 19 feeds, L = 50, 480x480 CAR) on
    the C2 observation's Level-2 output -- the device-median prep the bench times."""
    import bench
    from comapreduce_amd.mapmaking import comapdata as CD
    data, _, h = c2
    store = bench.level2_store(h, data, obsid=1)
    res = CD.read_comap_data(list(store), bench.c4_map_info(), iband=0, offset_length=50, store=store, device=0)
    return store, res


def test_c4_prep_device_matches_oracle(c4):
    """The device data prep at C4 size (COMAPData.py:471-577: 19 feeds x ~178k scan
    samples, weights, Sun / az-el / scan-edge cuts, the 400-sample high-pass, the
    empty-offset cut, CAR pixel ids) == oracle/comapdata.py (the NumPy + medianFilter.cpp
    restatement pinned to the reference golden) on every output bit for bit, except the
    Sun-centric coordinates (trigonometric leaves, <= 1e-12 relative)."""
    import bench
    from oracle import comapdata as oc
    store, dev = c4
    ref = oc.read_comap_data(list(store), store, bench.c4_map_info(), iband=0, offset_length=50)
    assert dev[0].size > 1_500_000 and dev[0].size % 50 == 0
    names = ('tod', 'weights', 'pointing', 'remapping_array', 'az', 'el', 'ra', 'dec', 'feedid', 'obsids')
    for k, a, b in zip(names, dev, ref):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, k
        if k in ('ra', 'dec'):
            assert np.max(np.abs(a - b)) <= 1e-12 * np.max(np.abs(b)), k
        else:
            assert np.array_equal(a, b), k


def test_c4_destriper_vs_oracle(c4):
    """C4 solve (threshold 0, 20 CG iterations) against oracle/destriper.py
    (Destriper.py:155-263, 402-453): weight / hits / naive bit-exact, offsets and
    map <= 1e-5 relative (north_star)."""
    import oracle.destriper as od
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    _, (tod, w, pix) = c4[0], c4[1][:3]
    npix = 480 * 480
    res = DeviceDestriper(pix, tod, w, 50, npix, device=0).solve(threshold=0.0, niter=20)
    ref, xr, itr = od.destriper_iteration(np.asarray(pix, np.int64), tod, w, 50, npix, threshold=0.0, niter=20)
    assert res['iters'] == itr == 20
    m = {k: v.cpu().numpy() for k, v in res['maps'].items()}
    for k in ('weight', 'hits', 'naive'):
        assert np.array_equal(m[k], ref[k]), k
    assert rel(m['map'], ref['map']) < 1e-5
    assert rel(res['x'].cpu().numpy(), xr) < 1e-5


def test_c4_four_bands_batched_vs_oracle(c4):
    """All 4 sidebands of C4 (read_comap_data_bands -> one batched solve) == each band
    prepared and solved alone by the oracle path (its own kept offsets)."""
    import bench
    import oracle.destriper as od
    from comapreduce_amd.mapmaking import comapdata as CD
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    store = c4[0]
    npix, niter = 480 * 480, 8
    r = CD.read_comap_data_bands(list(store), bench.c4_map_info(), bands=(0, 1, 2, 3), offset_length=50,
                                 store=store, device=0)
    res = DeviceDestriper(r['pointing'], r['tod'], r['weights'], 50, npix, device=0, keep=r['keep']).solve(0.0, niter)
    for b in range(4):
        tb, wb, pb = CD.read_comap_data(list(store), bench.c4_map_info(), iband=b, offset_length=50, store=store,
                                        device=0)[:3]
        ref, xr, itr = od.destriper_iteration(np.asarray(pb, np.int64), tb, wb, 50, npix, threshold=0.0, niter=niter)
        assert res['iters'][b] == itr
        m = {k: v[b].cpu().numpy() for k, v in res['maps'].items()}
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(m[k], ref[k]), (b, k)
        assert rel(m['map'], ref['map']) < 1e-5, b
        x = res['x'][b].cpu().numpy()
        assert rel(x[r['keep'][b].astype(bool)], xr) < 1e-5, b


def test_chain_as_timed_vs_oracle(c2):
    """The north_star chain exactly as bench.py times it (chain_fn: Level-2 left in HBM
    by the three stages -> level2_store_device -> prep.precompute_pointing on a side
    stream -> read_comap_data_bands(device_outputs=True, pointing=...) -> ONE batched
    solve to the reference's stopping rule, threshold 1e-6 / at most 100 iterations,
    maps copied to the host while the CG runs), run twice (the second run reuses the
    process caches the timed runs use), against the oracle per band: read_comap_data
    (COMAPData.py:471-577) on the host Level-2 of the same observation, then
    destriper_iteration (Destriper.py:402-453, run_destriper.py:146-189).
    weight / hits / naive bit-exact, map <= 1e-5 relative, equal iteration counts."""
    from concurrent.futures import ThreadPoolExecutor
    import bench
    import oracle.destriper as od
    from oracle import comapdata as oc
    data, _, h = c2
    chain = bench.chain_fn(data, 0)
    runs = [chain(False), chain(False)]
    for k in ('map', 'naive', 'weight', 'hits'):
        assert np.array_equal(runs[0]['maps'][k], runs[1]['maps'][k]), k
    assert runs[0]['iters'] == runs[1]['iters']
    got, iters = runs[1]['maps'], runs[1]['iters']
    assert got['map'].shape == (4, 480 * 480)
    obsid = int(data.obsid) if data.obsid > 0 else 1
    store = bench.level2_store(h, data, obsid=obsid)
    npix = 480 * 480

    def ref_band(b):
        tb, wb, pb = oc.read_comap_data(list(store), store, bench.c4_map_info(), iband=b, offset_length=50)[:3]
        return od.destriper_iteration(np.asarray(pb, np.int64), tb, wb, 50, npix, threshold=1e-6, niter=100)
    with ThreadPoolExecutor(4) as ex:
        refs = list(ex.map(ref_band, range(4)))
    for b, (ref, _, itr) in enumerate(refs):
        assert iters[b] == itr, (b, iters, itr)
        assert 1 < itr < 100, itr                  # converged by the threshold, not the cap
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(got[k][b], ref[k]), (b, k)
        assert rel(got['map'][b], ref['map']) < 1e-5, b


def test_c5_two_observations_two_bands_vs_oracle():
    """Reduced C5: 2 observations x 19 feeds x 180,000 samples (6.8 M samples, 137k
    offsets, 480x480 CAR), 2 sidebands batched, 12 CG iterations, against the oracle
    per band."""
    import torch
    import oracle.destriper as od
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    L, npix, niter = 50, 480 * 480, 12
    pix, tod, w = synthetic.destriper_inputs_device(2, offset_length=L, device=0, seed=1000, n_bands=2)
    res = DeviceDestriper(pix, tod, w, L, npix, device=0).solve(threshold=0.0, niter=niter)
    p, t, ww = pix.cpu().numpy().astype(np.int64), tod.cpu().numpy(), w.cpu().numpy()
    del pix, tod, w
    torch.cuda.empty_cache()
    assert p.size == 2 * 19 * 180_000
    for b in range(2):
        ref, xr, itr = od.destriper_iteration(p, t[b], ww[b], L, npix, threshold=0.0, niter=niter)
        assert res['iters'][b] == itr == niter
        m = {k: v[b].cpu().numpy() for k, v in res['maps'].items()}
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(m[k], ref[k]), (b, k)
        assert rel(m['map'], ref['map']) < 1e-5, b
        assert rel(res['x'][b].cpu().numpy(), xr) < 1e-5, b


@pytest.mark.parametrize('nb', [1, 4])
def test_c5_converged_vs_oracle(nb):
    """C5 at the bench's per-GPU size (BASELINE configs[4]: 64 observations over 8 GPUs
    -> 8 observations x 19 feeds x 180,000 samples per GPU, 27.4 M samples, 547k
    offsets, 480x480 CAR; the +-3.8 deg field keeps every sample on the map), solved to
    the reference's stopping rule (threshold 1e-6, at most 100 iterations:
    run_destriper.py:96-97, Destriper.py:85-152), 1 band and all 4 sidebands as one
    batched system, against oracle/destriper.py per band (Destriper.py:155-263,
    402-453): weight / hits / naive bit-exact, offsets and map <= 1e-5 relative
    (north_star), equal iteration counts, converged by the threshold (not the cap)."""
    from concurrent.futures import ThreadPoolExecutor
    import torch
    import oracle.destriper as od
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    L, npix = 50, 480 * 480
    pix, tod, w = synthetic.destriper_inputs_device(8, offset_length=L, device=0, seed=1000, n_bands=nb)
    assert int((pix < 0).sum().item()) == 0                 # the field lies inside the map
    res = DeviceDestriper(pix, tod, w, L, npix, device=0).solve(threshold=1e-6, niter=100)
    p = pix.cpu().numpy().astype(np.int64)
    t, ww = tod.cpu().numpy().reshape(nb, -1), w.cpu().numpy().reshape(nb, -1)
    got = {k: v.cpu().numpy().reshape(nb, -1) for k, v in res['maps'].items()}
    x = res['x'].cpu().numpy().reshape(nb, -1)
    iters = res['iters'] if nb > 1 else [res['iters']]
    del pix, tod, w, res
    torch.cuda.empty_cache()
    assert p.size == 8 * 19 * 180_000
    with ThreadPoolExecutor(nb) as ex:
        refs = list(ex.map(lambda b: od.destriper_iteration(p, t[b], ww[b], L, npix, threshold=1e-6, niter=100),
                           range(nb)))
    for b, (ref, xr, itr) in enumerate(refs):
        assert iters[b] == itr, (b, iters, itr)
        assert 1 < itr < 100, itr
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(got[k][b], ref[k]), (b, k)
        assert rel(got['map'][b], ref['map']) < 1e-5, b
        assert rel(x[b], xr) < 1e-5, b


def _c5_shard_rank(rank, world, port, q):
    """One rank of the sharded C5 solve: its 4 of the 8 observations (whole offsets), the
    map numerator compacted to the union of hit pixels and all-reduced with the p.q / r.r
    block partials every iteration (the path rankplan.plan() picks for C5)."""
    import os
    import torch
    import torch.distributed as dist
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['COMAP_DS_RANKS'] = 'shard'
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    L, npix = 50, 480 * 480
    import bench
    pix, tod, w = synthetic.destriper_inputs_device(8, offset_length=L, device=0, seed=1000, n_bands=4)
    # bench.py's work-balanced split of the (obs, feed) series (uneven: the early
    # observations scan faster and hold more entries per sample)
    ranges, _, _ = bench.field_split(8, world, device=0)
    ns = pix.numel() // (8 * 19)
    lo, hi = ranges[rank][0] * ns, ranges[rank][1] * ns
    prob = DeviceDestriper(pix[lo:hi].contiguous(), tod[:, lo:hi].contiguous(), w[:, lo:hi].contiguous(), L, npix,
                           device=0)
    res = prob.solve(threshold=1e-6, niter=100)
    q.put((rank, res['x'].cpu().numpy(), res['iters'], {k: v.cpu().numpy() for k, v in res['maps'].items()},
           int(prob.hit_index.numel()) if prob.hit_index is not None else -1))
    dist.barrier()
    dist.destroy_process_group()


def test_c5_two_ranks_sharded_field_scale():
    """The sharded multi-rank solve at field scale (C5 per-GPU size: 8 obs x 19 feeds x
    180k samples, 4 bands, 547k offsets, 480x480 CAR), its (obs, feed) series split over 2
    gloo ranks sharing cuda:0 by bench.field_split's work balance (not 4 + 4 observations) (Destriper.py:61-82, 183-204: partial maps and CG sums
    over ranks), solved to the reference's stopping rule (threshold 1e-6, <= 100
    iterations).  Offsets and maps <= 1e-9 of the single-rank solve, hits bit-exact,
    equal iteration counts; the compacted union is exactly the hit pixels, which on the
    +-3.8 deg field is a strict subset of the 480 x 480 map."""
    import os
    import torch
    import torch.multiprocessing as mp
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceDestriper
    L, npix = 50, 480 * 480
    pix, tod, w = synthetic.destriper_inputs_device(8, offset_length=L, device=0, seed=1000, n_bands=4)
    ref = DeviceDestriper(pix, tod, w, L, npix, device=0).solve(threshold=1e-6, niter=100)
    rx = ref['x'].cpu().numpy()
    rm = {k: v.cpu().numpy() for k, v in ref['maps'].items()}
    rit = list(ref['iters'])
    del pix, tod, w, ref
    torch.cuda.empty_cache()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29100 + os.getpid() % 190
    procs = [ctx.Process(target=_c5_shard_rank, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=600) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=120)
    assert list(res[0][2]) == list(res[1][2]) == rit
    assert all(1 < i < 100 for i in rit), rit
    x = np.concatenate([res[0][1], res[1][1]], axis=-1)
    assert x.shape == rx.shape == (4, 8 * 19 * 180_000 // L)
    # two partial sums per all-reduce instead of one sequential sum: rounding-level
    # differences only (north_star allows 1e-5)
    for b in range(4):
        assert rel(x[b], rx[b]) < 1e-9, b
    for k in ('map', 'naive', 'weight', 'hits'):
        assert res[0][3][k].shape == rm[k].shape, k
        for b in range(4):
            assert rel(res[0][3][k][b], rm[k][b]) < 1e-9, (k, b)
        assert np.array_equal(res[0][3][k], res[1][3][k]), k          # every rank holds the same maps
    assert np.array_equal(res[0][3]['hits'], rm['hits'])
    nhit = int(np.count_nonzero(rm['hits'].sum(axis=0)))
    assert res[0][4] == res[1][4] == nhit                # no unbinned samples: the union is the hit pixels
    assert nhit < 0.95 * npix, nhit                      # ... a strict subset of the map (about (3.8/4)^2)
