"""run_destriper driver: .ini parsing (pinned to the reference Parser's output
on tests/golden/params_case.ini), FITS map files, and the end-to-end
read_comap_data -> destriper -> write_map chain on the GPU."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))


def test_parser_matches_reference(golden_dir):
    from comapreduce_amd.tools.parser import Parser, sex2deg
    ref = json.load(open(os.path.join(golden_dir, 'golden_meta.json')))['parser_case']
    p = Parser(os.path.join(golden_dir, 'params_case.ini'))
    assert p.infodict == ref['parsed']
    got = [sex2deg('11:20:00', hours=True), sex2deg('+52:00:00'), sex2deg('-00:30:36'),
           sex2deg('05:32:00.3', hours=True)]
    assert got == ref['sex2deg']
    with pytest.raises(AttributeError):
        p['Missing']


def test_fits_roundtrip(tmp_path):
    from comapreduce_amd.mapmaking.fits import read_image_hdus
    from comapreduce_amd.mapmaking.run_destriper import write_map
    from comapreduce_amd.mapmaking.comapdata import map_info_from
    mi = map_info_from([170.0, 52.0], [-1 / 60., 1 / 60.], [10, 8], ['RA---CAR', 'DEC--CAR'], 20, 16)
    rng = np.random.default_rng(0)
    v = {'map': rng.standard_normal(320), 'naive': rng.standard_normal(320),
         'weight': rng.uniform(0, 2, 320), 'hits': rng.integers(0, 9, 320).astype(float)}
    v['weight'][3] = 0.0
    write_map('case', {'All': v}, mi, str(tmp_path), 2)
    hdus = read_image_hdus(str(tmp_path / 'All_case_Band02.fits'))
    assert [h.get('EXTNAME') for h, _ in hdus] == [None, 'Naive', 'Noise', 'Hits']
    h0, m = hdus[0]
    assert h0['SIMPLE'] is True and h0['BITPIX'] == -64 and h0['CTYPE1'] == 'RA---CAR'
    assert h0['CRPIX1'] == 10.0 and h0['CDELT2'] == 1 / 60.
    assert np.array_equal(m, v['map'].reshape(16, 20))
    assert np.array_equal(hdus[1][1], v['naive'].reshape(16, 20))
    with np.errstate(divide='ignore'):
        assert np.array_equal(hdus[2][1], np.sqrt(1. / v['weight']).reshape(16, 20))
    assert np.array_equal(hdus[3][1], v['hits'].reshape(16, 20))
    assert os.path.getsize(tmp_path / 'All_case_Band02.fits') % 2880 == 0


@pytest.mark.gpu
def test_run_destriper_main_end_to_end(tmp_path):
    """main() on the COMAPData fixture files vs the oracle chain
    (oracle.comapdata -> oracle.destriper.destriper_iteration)."""
    import comapdata_case as cc
    from comapreduce_amd.mapmaking.run_destriper import main
    from comapreduce_amd.mapmaking.fits import read_image_hdus
    from oracle import comapdata as oc, destriper as od
    store, names = cc.store()
    names = names[:2]                                   # Field00 files (non-calibrator mode)
    m = cc.CASES['car']['map']
    out = main(names, offset_length=50, prefix='t', output_dir=str(tmp_path), feeds=cc.FEEDS,
               nxpix=m['nxpix'], nypix=m['nypix'], crval=m['crval'], crpix=m['crpix'], ctype=m['ctype'],
               cdelt=m['cdelt'], use_gain_filter=True, calibration=False, threshold=1e-6, niter=50,
               bands=(0,), store=store)
    from comapreduce_amd.mapmaking.comapdata import map_info_from
    mi = map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])
    tod, w, pix, *_ = oc.read_comap_data(names, store, mi, iband=0, offset_length=50, feeds=cc.FEEDS)
    npix = m['nxpix'] * m['nypix']
    ref, _, _ = od.destriper_iteration(pix, tod, w, 50, npix, threshold=1e-6, niter=50)
    got = out[0]['All']
    for k in ('weight', 'hits', 'naive'):
        a, b = np.nan_to_num(got[k]), np.nan_to_num(ref[k])
        bad = np.nonzero(a != b)[0]
        assert bad.size == 0, (k, bad.size, bad[:5].tolist(), a[bad[:5]].tolist(), b[bad[:5]].tolist(),
                               ref['weight'][bad[:5]].tolist())
    fin = np.isfinite(ref['map']) & (ref['weight'] > 0)
    scale = np.max(np.abs(ref['map'][fin]))
    assert np.max(np.abs(got['map'][fin] - ref['map'][fin])) <= 1e-6 * scale
    hdus = read_image_hdus(str(tmp_path / 'All_t_Band00.fits'))
    assert np.array_equal(np.nan_to_num(hdus[0][1].ravel()), np.nan_to_num(got['map']))


@pytest.mark.gpu
def test_run_destriper_main_bands_batched(tmp_path):
    """main() with the 4 bands batched (read_comap_data_bands + one batched
    device solve) == the oracle chain run band by band."""
    import comapdata_case as cc
    from comapreduce_amd.mapmaking.run_destriper import main
    from comapreduce_amd.mapmaking.comapdata import map_info_from
    from oracle import comapdata as oc, destriper as od
    store, names = cc.store()
    names = names[:2]
    m = cc.CASES['car']['map']
    out = main(names, offset_length=50, prefix='t', output_dir=str(tmp_path), feeds=cc.FEEDS,
               nxpix=m['nxpix'], nypix=m['nypix'], crval=m['crval'], crpix=m['crpix'], ctype=m['ctype'],
               cdelt=m['cdelt'], use_gain_filter=True, calibration=False, threshold=1e-6, niter=50,
               bands=(0, 1, 2, 3), store=store)
    mi = map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])
    npix = m['nxpix'] * m['nypix']
    for b in range(4):
        tod, w, pix, *_ = oc.read_comap_data(names, store, mi, iband=b, offset_length=50, feeds=cc.FEEDS)
        ref, _, _ = od.destriper_iteration(pix, tod, w, 50, npix, threshold=1e-6, niter=50)
        got = out[b]['All']
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(np.nan_to_num(got[k]), np.nan_to_num(ref[k])), (b, k)
        fin = np.isfinite(ref['map']) & (ref['weight'] > 0)
        scale = np.max(np.abs(ref['map'][fin]))
        assert np.max(np.abs(got['map'][fin] - ref['map'][fin])) <= 1e-6 * scale, b
        assert os.path.exists(tmp_path / f'All_t_Band{b:02d}.fits')


@pytest.mark.gpu
@pytest.mark.parametrize('batch', [False, True])
def test_run_destriper_main_healpix(tmp_path, batch):
    """healpix=True: RING nside-4096 pixels (read_pixels_healpix, COMAPData.py:429-469),
    compacted to the union of hit pixels (:572-573), pixel_edges = arange(max + 1)
    (run_destriper.py:159-161), partial HEALPix files (write_map_healpix, :53-77).
    The data prep is otherwise unchanged (tod / weights equal the CAR read's), and the
    maps equal the oracle destriper on the compact pointing; the file holds the union
    pixels with (map, naive, sqrt(1/weight)).  healpy parity itself is unpinned."""
    import comapdata_case as cc
    from comapreduce_amd.mapmaking import comapdata as CD, healpix as H
    from comapreduce_amd.mapmaking.run_destriper import main
    from oracle import destriper as od
    store, names = cc.store()
    names = names[:2]
    m = cc.CASES['car']['map']
    geo = dict(nxpix=m['nxpix'], nypix=m['nypix'], crval=m['crval'], crpix=m['crpix'], ctype=m['ctype'],
               cdelt=m['cdelt'])
    bands = (0, 1) if batch else (0,)
    out = main(names, offset_length=50, prefix='h', output_dir=str(tmp_path), feeds=cc.FEEDS,
               use_gain_filter=True, calibration=False, threshold=1e-6, niter=50, bands=bands, store=store,
               healpix=True, batch_bands=batch, **geo)
    mi = CD.map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])
    for b in bands:
        tod_c, w_c, _, _, *_ = CD.read_comap_data(names, mi, iband=b, offset_length=50, feeds=cc.FEEDS, store=store)
        tod, w, pix, remap, *_ = CD.read_comap_data(names, mi, iband=b, offset_length=50, feeds=cc.FEEDS,
                                                    store=store, healpix=True)
        assert np.array_equal(tod, tod_c) and np.array_equal(w, w_c)
        assert pix.min() >= 0 and pix.max() < remap.size and np.all(np.diff(remap) > 0)
        assert remap.max() < H.nside2npix(4096)
        ref, _, _ = od.destriper_iteration(pix, tod, w, 50, remap.size, threshold=1e-6, niter=50)
        got = out[b]['All']
        for k in ('weight', 'hits', 'naive'):
            assert np.array_equal(np.nan_to_num(got[k]), np.nan_to_num(ref[k])), (b, k)
        fin = np.isfinite(ref['map']) & (ref['weight'] > 0)
        assert np.max(np.abs(got['map'][fin] - ref['map'][fin])) <= 1e-6 * np.max(np.abs(ref['map'][fin]))
        hdr, rec = H.read_map_partial(str(tmp_path / f'All_h_Band{b:02d}.fits'))
        assert hdr['NSIDE'] == 4096 and hdr['ORDERING'] == 'RING'
        assert np.array_equal(rec['PIXEL'], remap)
        assert np.array_equal(rec['TEMPERATURE'], got['map'], equal_nan=True)
        assert np.array_equal(rec['Q_POLARISATION'], got['naive'], equal_nan=True)


def _rank_files_worker(rank, world, port, q):
    import os
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden'))
    import comapdata_case as cc
    from comapreduce_amd.mapmaking import comapdata as C
    from comapreduce_amd.mapmaking.run_destriper import _rank_files
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    store, names = cc.store()
    m = cc.CASES['car']['map']
    mi = C.map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])
    files = _rank_files(np.array(names), rank, world, 50, cc.FEEDS, mi, False, C._opener(store))
    q.put((rank, [str(f) for f in files]))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_files_balanced_on_work():
    """run_destriper's file split on 2 gloo ranks: the mapped set stays the reference's
    (the first len // size x size files, run_destriper.py:131-138), dealt in contiguous
    ranges that minimise the largest rank's CG work (operator entries + offsets, weighed
    from each file's pointing) instead of equal counts."""
    import os
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden'))
    import comapdata_case as cc
    from comapreduce_amd.mapmaking import comapdata as C
    from comapreduce_amd.mapmaking import rankplan
    from comapreduce_amd.mapmaking.run_destriper import _file_work
    store, names = cc.store()
    m = cc.CASES['car']['map']
    mi = C.map_info_from(m['crval'], m['cdelt'], m['crpix'], m['ctype'], m['nxpix'], m['nypix'])
    opener = C._opener(store)
    weights = [_file_work(opener(f), 50, cc.FEEDS, mi, False) for f in names[:2]]
    assert all(w > 0 for w in weights)
    want = rankplan.balanced_ranges(weights, 2)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29400 + os.getpid() % 190
    procs = [ctx.Process(target=_rank_files_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert res[0] + res[1] == list(names[:2])            # the reference's mapped set, in order
    for r in range(2):
        a, b = want[r]
        assert res[r] == list(names[a:b]), r
