"""HEALPix RING pixelisation and partial maps (mapmaking/healpix.py) for the
destriper's healpix mode (COMAPData.py:429-469, run_destriper.py:53-77).
healpy is not in the image, so parity with it is unpinned; these tests pin the
restatement to the scheme's own invariants: every pixel centre maps back to its
pixel, known pixel centres, equal areas, ring ordering, the pole branches, and the
partial-map file layout."""
import os

import numpy as np
import pytest

from comapreduce_amd.mapmaking import healpix as H


@pytest.mark.parametrize('nside', [1, 2, 4, 8, 16, 64, 4096])
def test_pixel_centres_map_back(nside):
    npix = H.nside2npix(nside)
    pix = np.arange(npix) if npix <= 50_000 else np.unique(np.concatenate([
        np.arange(20_000), npix - 1 - np.arange(20_000), np.random.default_rng(1).integers(0, npix, 50_000)]))
    th, ph = H.pix2ang_ring(nside, pix)
    assert np.array_equal(H.ang2pix(nside, th, ph), pix)
    # phi wrapped by +-2pi lands on the same pixel
    assert np.array_equal(H.ang2pix(nside, th, ph + 2 * np.pi), pix)
    assert np.array_equal(H.ang2pix(nside, th, ph - 2 * np.pi), pix)


def test_known_pixels():
    assert H.ang2pix(1, 0.0, 0.0) == 0
    assert H.ang2pix(1, np.pi, 0.0) == 8                       # phi = 0 opens the south ring
    th, ph = H.pix2ang_ring(1, [0, 4, 11])
    assert np.allclose(th, [np.arccos(2 / 3), np.pi / 2, np.arccos(-2 / 3)])
    assert np.allclose(ph, [np.pi / 4, 0.0, 7 * np.pi / 4])
    # near the poles: the first pixels of the polar rings (sin(theta) branch)
    n = 4096
    assert H.ang2pix(n, 1e-9, 0.1) == 0 and H.ang2pix(n, np.pi - 1e-9, 0.1) == H.nside2npix(n) - 4


def test_equal_area():
    rng = np.random.default_rng(7)
    m = 2_000_000
    th = np.arccos(rng.uniform(-1, 1, m))
    ph = rng.uniform(0, 2 * np.pi, m)
    cnt = np.bincount(H.ang2pix(4, th, ph), minlength=H.nside2npix(4))
    mean = m / cnt.size
    assert cnt.min() > mean - 6 * np.sqrt(mean) and cnt.max() < mean + 6 * np.sqrt(mean)


def test_ring_order_follows_colatitude():
    nside = 32
    th, _ = H.pix2ang_ring(nside, np.arange(H.nside2npix(nside)))
    assert np.all(np.diff(th) >= -1e-15)                       # RING: pixels ordered by ring, north first


def test_index_replace_reference_semantics():
    a = np.array([50, 7, 19, 3])
    b = np.array([19, 3, 3, 50, 7])
    assert np.array_equal(H.index_replace(a, b), [2, 3, 3, 0, 1])
    u = np.unique(b)
    assert np.array_equal(H.index_replace(u, b), np.searchsorted(u, b))


def test_partial_map_file(tmp_path):
    nside = 16
    npix = H.nside2npix(nside)
    m = np.zeros((3, npix)) + H.UNSEEN
    pix = np.array([0, 5, 77, npix - 1])
    m[0, pix] = [1.0, -2.0, 3.5, 4.0]
    m[1, pix] = [0.1, 0.2, 0.3, 0.4]
    m[2, pix] = [np.inf, 1.0, 2.0, 3.0]
    f = str(tmp_path / 'hp.fits')
    H.write_map_partial(f, m, nside)
    hdr, rec = H.read_map_partial(f)
    assert hdr['XTENSION'] == 'BINTABLE' and hdr['PIXTYPE'] == 'HEALPIX' and hdr['ORDERING'] == 'RING'
    assert hdr['NSIDE'] == nside and hdr['INDXSCHM'] == 'EXPLICIT' and hdr['OBJECT'] == 'PARTIAL'
    assert hdr['TTYPE1'] == 'PIXEL' and hdr['TTYPE2'] == 'TEMPERATURE' and hdr['TFORM2'] == 'D'
    assert np.array_equal(rec['PIXEL'], pix)
    assert np.array_equal(rec['TEMPERATURE'], m[0, pix]) and np.array_equal(rec['U_POLARISATION'], m[2, pix])
    assert (tmp_path / 'hp.fits').stat().st_size % 2880 == 0


def _remap_rank(rank, world, port, pix, q):
    import torch.distributed as dist
    from comapreduce_amd.mapmaking.comapdata import find_unique_values
    from comapreduce_amd.mapmaking.run_destriper import _healpix_edges
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mine = pix[rank]
    remap = find_unique_values(np.unique(mine))
    pointing = H.index_replace(remap, mine)
    edges = _healpix_edges(pointing)
    q.put((rank, remap, pointing, edges))
    dist.destroy_process_group()


def test_multirank_healpix_remapping_gloo():
    """COMAPData.py:570-574 + run_destriper.py:159-161 on 2 gloo ranks: every rank
    gets the same union of hit pixels (find_unique_values), its pointing becomes
    positions in that union, and pixel_edges spans the union on both ranks."""
    import multiprocessing as mp
    rng = np.random.default_rng(3)
    npix = H.nside2npix(4096)
    pix = [rng.integers(0, npix // 2, 5000), np.concatenate([rng.integers(npix // 4, npix, 3000), [npix - 1]])]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 27500 + os.getpid() % 1000
    procs = [ctx.Process(target=_remap_rank, args=(r, 2, port, pix, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    union = np.unique(np.concatenate(pix))
    for r in range(2):
        remap, pointing, edges = res[r]
        assert np.array_equal(remap, union)
        assert np.array_equal(union[pointing], pix[r])
        assert np.array_equal(edges, np.arange(union.size))
