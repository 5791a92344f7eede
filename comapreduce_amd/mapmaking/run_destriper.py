"""Map-making driver: mirror of reference comancpipeline/MapMaking/run_destriper.py.

    python run_destriper.py parameters.ini
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 run_destriper.py parameters.ini

One process per GPU (torch.distributed over RCCL, RANK/WORLD_SIZE from the
environment) replaces mpi4py.  The 4 sidebands together: read_comap_data_bands
(the whole data prep on the device: weights, cuts, pixel ids, the 400-sample
high-pass) -> one batched device destriper solve (per-iteration SUM all-reduce of
the map numerator across ranks) -> rank 0 writes each band's FITS maps.

Reference behaviours kept: files lacking averaged_tod/tod are dropped; the
source of the FIRST file decides calibrator mode (offset_length 250,
threshold 1); files are split in blocks of ``len // size`` per rank, so the
``len % size`` trailing files are not mapped (run_destriper.py:131-138).
"""
from __future__ import annotations

import os

import numpy as np

from . import comapdata as COMAPData
from .destriper import run_destriper, run_destriper_bands
from .fits import write_image_hdus
from ..tools.parser import Parser, sex2deg

CALIBRATORS = COMAPData.CALIBRATORS


def _rank_size():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def write_map(prefix, maps, map_info, output_dir, iband, postfix=''):
    """run_destriper.write_map (run_destriper.py:19-50)."""
    os.makedirs(output_dir, exist_ok=True)
    wcs, nx, ny = map_info['wcs'], map_info['nxpix'], map_info['nypix']
    cards = wcs.to_header()
    for k, v in maps.items():
        images = [(None, np.reshape(v['map'], (ny, nx)))]
        if 'naive' in v:
            images.append(('Naive', np.reshape(v['naive'], (ny, nx))))
        if 'weight' in v:
            with np.errstate(divide='ignore'):
                images.append(('Noise', np.reshape(np.sqrt(1. / v['weight']), (ny, nx))))
        if 'hits' in v:
            images.append(('Hits', np.reshape(v['hits'], (ny, nx))))
        fname = '{}/{}_{}_Band{:02d}.fits'.format(output_dir, k, prefix, iband)
        write_image_hdus(fname, images, cards)


def write_map_healpix(prefix, maps, remapping_array, map_info, output_dir, iband, postfix='', nside=4096):
    """run_destriper.write_map_healpix (run_destriper.py:53-77): per map set a
    partial HEALPix file of (map, naive, sqrt(1/weight)) on the union pixels."""
    from .healpix import UNSEEN, nside2npix, write_map_partial
    os.makedirs(output_dir, exist_ok=True)
    for k, v in maps.items():
        m = np.zeros((3, nside2npix(nside))) + UNSEEN
        m[0, remapping_array] = v['map']
        m[1, remapping_array] = v['naive']
        with np.errstate(divide='ignore'):
            m[2, remapping_array] = np.sqrt(1. / v['weight'])
        fname = '{}/{}_{}_Band{:02d}.fits'.format(output_dir, k, prefix, iband)
        write_map_partial(fname, m, nside)


def _healpix_edges(pointing):
    """run_destriper.py:159-161: pixel_edges = arange(max over ranks of pointing + 1)."""
    import torch.distributed as dist
    mx = int(np.max(pointing)) if np.size(pointing) else -1
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        import torch
        dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else 'cpu'
        t = torch.tensor([mx], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mx = int(t.item())
    return np.arange(mx + 1, dtype=int)


def _file_work(f, offset_length, feeds, map_info, healpix):
    """The CG work one file brings a rank: its operator entries -- the (offset, pixel run)
    pairs of its scan pointing (rankplan.offset_pixel_runs) -- plus FILE_KAPPA x its offsets
    (per-offset CG vector work in entries-equivalent units, as bench.py's field split)."""
    from . import rankplan
    fi, _ = COMAPData.GetFeeds(f['spectrometer/feeds'], feeds)
    datasize = int(COMAPData.countDataSize(f, len(fi), offset_length)['datasize'])
    if datasize == 0 or len(fi) == 0:
        return 0
    read = COMAPData.read_pixels_healpix if healpix else COMAPData.read_pixels
    pix = np.asarray(read(f, datasize, offset_length, feeds, map_info))[:len(fi), :datasize]
    entries = int(rankplan.offset_pixel_runs(pix.astype(np.int64), offset_length, groups=pix.shape[0]).sum())
    return entries + int(FILE_KAPPA * pix.size // offset_length)


FILE_KAPPA = 6.5


def _rank_files(filelist, rank, size, offset_length, feeds, map_info, healpix, open_file):
    """This rank's files.  The mapped set is the reference's: the first (len // size) x size
    files (run_destriper.py:131-138 drops the remainder); the reference then deals them in
    equal counts.  Here (COMAP_DS_SPLIT=work, the default) they are dealt in contiguous
    ranges balanced on each file's CG work (_file_work; every rank weighs its own
    equal-count share, the weights are all-gathered): a sharded CG iteration waits for its
    slowest rank, whose time follows its operator entries, not its file count.  The maps do
    not depend on which rank holds a file.  COMAP_DS_SPLIT=count: the reference's split."""
    step = filelist.size // size
    lo, hi = step * rank, min(step * (rank + 1), filelist.size)
    if size == 1 or step == 0 or os.environ.get('COMAP_DS_SPLIT', 'work') == 'count':
        return filelist[lo:hi]
    import torch.distributed as dist
    from . import rankplan
    mine = [_file_work(open_file(f), offset_length, feeds, map_info, healpix) for f in filelist[lo:hi]]
    parts = [None] * size
    dist.all_gather_object(parts, mine)
    weights = [w for p in parts for w in p]
    a, b = rankplan.balanced_ranges(weights, size)[rank]
    return filelist[:step * size][a:b]


def main(filelistname, offset_length=50, feed_weights=None, prefix='fg9', output_dir='maps/fg9/', obsid_cuts=[],
         feeds=[1, 2, 3, 5, 6, 9, 11, 12, 13, 14, 15, 16, 17, 18, 19], nxpix=480, nypix=480,
         crval=['05:32:00.3', '+12:30:28.0'], crpix=[240, 240], ctype=['RA---CAR', 'DEC--CAR'],
         cdelt=[-0.016666, 0.016666], use_gain_filter=True, calibration=True, calibrator='TauA', threshold=1e-6,
         niter=100, healpix=False, bands=(0, 1, 2, 3), store=None, device=None, batch_bands=True):
    """run_destriper.main (run_destriper.py:79-189).  ``store`` (tests) maps
    filename -> (datasets, attrs) instead of reading files; ``device`` is the
    rank's GPU (default: torch's current device, LOCAL_RANK under torchrun).
    ``batch_bands``: the bands share the pointing, so they are read with one
    batched median call and solved as ONE batched device system
    (read_comap_data_bands + run_destriper_bands); False runs the reference's
    per-band loop.  The maps are the same either way."""
    rank, size = _rank_size()
    if device is None:
        import torch
        device = torch.cuda.current_device()
    input_filelist = np.loadtxt(filelistname, dtype=str, ndmin=1) if isinstance(filelistname, str) \
        else np.asarray(filelistname)
    open_file = COMAPData._opener(store)
    filelist, source = [], None
    for i, f in enumerate(input_filelist):
        h = open_file(f)
        if i == 0:
            source = h.attrs('comap')['source'].split(',')[0]
        if 'averaged_tod/tod' in h:
            filelist.append(f)
    filelist = np.array(filelist)
    if isinstance(crval[0], str):
        crval = [sex2deg(c, hours=hr) for c, hr in zip(crval, [True, False])]
    map_info = COMAPData.map_info_from(crval, cdelt, crpix, ctype, nxpix, nypix)
    filelist = _rank_files(filelist, rank, size, offset_length, feeds, map_info, healpix, open_file)
    if source in CALIBRATORS:
        offset_length = 250
        threshold = 1
    out = {}
    if batch_bands and len(bands) > 1:
        r = COMAPData.read_comap_data_bands(filelist, map_info, bands=bands, offset_length=offset_length, feeds=feeds,
                                            use_gain_filter=use_gain_filter, calibration=calibration,
                                            calibrator=calibrator, healpix=healpix, store=store, device=device)
        pixel_edges = _healpix_edges(r['pointing']) if healpix else np.arange(nxpix * nypix)
        res = run_destriper_bands(r['pointing'], r['tod'], r['weights'], offset_length, pixel_edges, keep=r['keep'],
                                  threshold=threshold, niter=niter, device=device,
                                  map_shape=None if healpix else (nypix, nxpix))
        for iband, maps in zip(bands, res):
            maps = {'All': maps['All']}
            if rank == 0:
                if healpix:
                    write_map_healpix(prefix, maps, r['remapping_array'], map_info, output_dir, iband)
                else:
                    write_map(prefix, maps, map_info, output_dir, iband)
            out[iband] = maps
        return out
    for iband in bands:
        tod, weights, pointing, remap, az, el, ra, dec, feedid, obsids = COMAPData.read_comap_data(
            filelist, map_info, feed_weights=feed_weights, offset_length=offset_length, iband=iband, feeds=feeds,
            use_gain_filter=use_gain_filter, calibration=calibration, calibrator=calibrator, healpix=healpix,
            store=store, device=device)
        pixel_edges = _healpix_edges(pointing) if healpix else np.arange(nxpix * nypix)
        maps = run_destriper(pointing, tod, weights, offset_length, pixel_edges, az, el, ra, dec, feedid, obsids,
                             obsid_cuts, threshold=threshold, niter=niter, chi2_cutoff=20,
                             device=device, map_shape=None if healpix else (nypix, nxpix))
        if rank == 0:
            if healpix:
                write_map_healpix(prefix, maps, remap, map_info, output_dir, iband)
            else:
                write_map(prefix, maps, map_info, output_dir, iband)
        out[iband] = maps
    return out


def cli(argv):
    """``__main__`` block of run_destriper.py (:191-212): everything from [Inputs]
    except use_gain_filter / calibration / calibrator from [ReadData]."""
    p = Parser(argv[0])
    params = p['Inputs']
    feeds = params['feeds']
    feeds = [int(f) for f in (feeds if isinstance(feeds, list) else [feeds])]
    as_list = lambda v: v if isinstance(v, list) else [v]  # noqa: E731
    return main(params['filelistname'], offset_length=int(params['offset_length']), prefix=params['prefix'],
                output_dir=params['output_dir'], feeds=feeds, feed_weights=params['feed_weights'],
                nxpix=int(params['nxpix']), nypix=int(params['nypix']), crval=as_list(params['crval']),
                crpix=as_list(params['crpix']), ctype=as_list(params['ctype']), cdelt=as_list(params['cdelt']),
                use_gain_filter=p['ReadData']['use_gain_filter'], calibration=p['ReadData']['calibration'],
                calibrator=p['ReadData']['calibrator'], threshold=10 ** float(params['threshold']),
                niter=int(params['niter']), healpix=params['healpix'])
