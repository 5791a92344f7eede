#!/usr/bin/env python3
"""bench.py -- COMAP Level-1 -> Level-2 reduction throughput on MI355X.

Metric (BASELINE.json): TOD samples x channels / s for the L1 -> L2 reduction
(MeasureSystemTemperature -> AtmosphereRemoval -> Level1AveragingGainCorrection)
of the full 19-feed x 4 x 1024-channel x 180,000-sample synthetic observation
(configs[1], C2: 56 GB f32 resident in HBM), plus the destriper's CG
iterations / s on that observation's Level-2 TOD (configs[3], C4) and on a
multi-observation HBM-resident field (configs[4], C5).

One step = one complete reduction of the observation (every kernel of the
three stages; the plan/airmass set-up happens once per observation, like
opening the file).

N GPUs (``--gpus N``; the script launches its own N ranks through
torch.distributed.run when started without WORLD_SIZE, one process per GPU):
  --mode shard (default)  configs[2], C3: ONE observation's (feed, scan) units
                          are split over the ranks (pipeline/sharding.py), each
                          rank generates and holds only its feeds, and reduces
                          its units with no collective -> "scaling": "strong";
                          value = the observation's samples x channels per step
                          / the slowest rank's time.
  --mode obs              one whole observation per rank (the reference's
                          file-level MPI split) -> "scaling": "weak".
The C5 destriper leg is weak-scaled (8 observations per GPU) with an RCCL
all-reduce of the map numerator and CG scalars every iteration.

    python bench.py [--gpus N --steps K --warmup W --mode shard|obs]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALGO_BYTES_PER_SAMPCH_PASS = 4      # one f32 read of the cube per streaming pass
SURVEY_BYTES_PER_SAMPCH = 16        # 4 passes (A, B, C, D) x 4 B
# this design streams the cube 3 times: A (moments), B (band means + every per-sample
# output sum, band_sums) and C (regression sums, regress); B and C read only the
# median_filter channels
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
DESTRIPER_BYTES_PER_SAMPLE = 24     # per CG iteration
DESTRIPER_BYTES_PER_OFFSET = 80


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--mode', choices=('shard', 'obs'), default='shard',
                    help='N > 1: shard one observation over the ranks (C3, strong) or one observation per rank (weak)')
    ap.add_argument('--feeds', type=int, default=19)
    ap.add_argument('--samples', type=int, default=180_000)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-destriper', action='store_true')
    ap.add_argument('--destriper-iters', type=int, default=100)
    ap.add_argument('--c5-obs', type=int, default=8, help='observations per GPU in the C5 destriper leg (0: skip)')
    ap.add_argument('--c5-field-obs', type=int, default=64,
                    help='observations of the C5 field solved as ONE system over all ranks (configs[4]; 0: skip)')
    ap.add_argument('--check', action='store_true', help='compare one unit against the CPU oracle')
    ap.add_argument('--no-e2e', action='store_true', help='skip the host-cube -> host-Level-2 leg')
    ap.add_argument('--no-chain', action='store_true', help='skip the L1 -> L2 -> maps chain leg')
    ap.add_argument('--shard-of', type=int, default=0,
                    help='measurement aid: reduce only rank 0\'s C3 shard of an N-way split, in this one process')
    return ap.parse_args()


# ---------------------------------------------------------------- N-GPU launch
def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Run this script on n ranks (one process per GPU) via torch.distributed.run
    and return its exit code.  Called before anything touches the GPU; the ranks
    are child processes (no exec)."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------- observation
def build_observation(F, T, obs_id, device, rank=0, world=1):
    """Device-resident synthetic Level-1 observation; with
    world > 1 only this rank's shard: the feeds its (feed, scan) units touch,
    generated on device with the same samples the full cube holds, and the
    unit filter that restricts the reduction to its units.
    Returns (COMAPLevel1, Shard)."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd import synthetic
    from comapreduce_amd.pipeline.datahandling import COMAPLevel1
    from comapreduce_amd.pipeline.sharding import shard_for, slice_feeds
    cfg = synthetic.SyntheticConfig(n_feeds=F, n_samples=T, obs_id=obs_id)
    meta, attrs, level, mult, hot = synthetic.level1_metadata(cfg)
    full = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in meta.items():
        full[k] = v
    for p, a in attrs.items():
        for k, v in a.items():
            full.set_attrs(p, k, v)
    sh = shard_for(full.scan_edges, F, rank, world)
    lo, hi = sh.f_lo, sh.f_hi
    if hi <= lo:
        raise RuntimeError(f'rank {rank}: no unit to reduce (world {world} > units)')
    Fs = hi - lo
    dev = torch.device('cuda', device)
    lv = torch.from_numpy(np.ascontiguousarray(level[lo:hi])).to(dev)
    mu = torch.from_numpy(np.ascontiguousarray(mult[lo:hi])).to(dev)
    ho = torch.from_numpy(np.ascontiguousarray(hot[lo:hi])).to(dev)
    tod = torch.empty((Fs, 4, 1024, T), dtype=torch.float32, device=dev)
    ba = torch.empty((Fs, 4, T), dtype=torch.float32, device=dev)
    c = N.ctx(device)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_synth_tod(c, Fs, lo, T, 1000 + obs_id, N.dptr(lv), N.dptr(mu), N.dptr(ho), N.dptr(tod),
                                    N.dptr(ba)), c, 'comap_synth_tod')
    torch.cuda.synchronize(dev)
    del lv, mu, ho
    full['spectrometer/tod'] = tod
    full['spectrometer/band_average'] = ba
    if world == 1:
        return full, sh
    # the shard's feeds: tod/band_average already hold only them
    part = slice_feeds(full, lo, hi, sh.local_filter())
    part['spectrometer/tod'] = tod
    part['spectrometer/band_average'] = ba
    return part, sh


def reduce_step(data, device, timing=None, device_outputs=True):
    """One full L1 -> L2 reduction (outputs stay on the device unless
    device_outputs=False, the Runner's host arrays).  ``timing`` (a dict) collects
    host wall time per stage call (enqueue + host work)."""
    from comapreduce_amd import Analysis as A
    from comapreduce_amd.pipeline.datahandling import COMAPLevel2
    level2 = COMAPLevel2(filename='/nonexistent/level2.hd5')
    for cls in (A.MeasureSystemTemperature, A.AtmosphereRemoval, A.Level1AveragingGainCorrection):
        t0 = time.perf_counter()
        st = cls(level2=level2, device=device, device_outputs=device_outputs)
        if not st(data, level2):
            raise RuntimeError(f'{cls.__name__} stopped the file')
        level2.update(st)
        if timing is not None:
            timing[cls.__name__] = timing.get(cls.__name__, 0.0) + (time.perf_counter() - t0) * 1e3
    return level2


# ---------------------------------------------------------------- CPU baselines
def cpu_baseline(level2=None, data=None):
    """The CPU oracle (a NumPy/C restatement of the reference, 'port') timed on
    this host on a bounded sample -- the C1 observation (1 feed x 4 x 1024 x
    30,000) -- next to the reference itself ('reference'), which cannot travel
    to the GPU box and was timed in the build container by
    tests/golden/make_golden.py (tests/golden/golden_meta.json).  Destriper: the
    oracle's CG iterations / s on this observation's C4 problem (a few timed
    iterations) and the reference's, timed likewise in the build container."""
    from threadpoolctl import threadpool_limits
    import oracle.l1 as ol1
    from comapreduce_amd import synthetic
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000, obs_id=1))
    with threadpool_limits(1):
        t0 = time.perf_counter()
        ol1.reduce_level1(gen['data'])
        dt = time.perf_counter() - t0
    n = 1 * 4 * 1024 * 30_000
    out = {'value': n / dt, 'unit': 'samples*channels/s', 'cores': 1, 'kind': 'port',
           'sample': f'C1 observation 1x4x1024x30000 ({n} samp*ch), full vane+atmosphere+L2 reduce, '
                     f'{dt:.2f} s on 1 host core of the GPU box (oracle/l1.py)'}
    meta = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'golden_meta.json')))
    tr = meta.get('reference_timings_s_c1')
    if tr:
        rs = float(sum(tr.values()))
        nref = int(meta.get('reference_samples_channels_c1', n))
        out['reference'] = {
            'value': nref / rs, 'unit': 'samples*channels/s', 'cores': 1, 'kind': 'reference',
            'sample': f'the reference v0.9.1 itself (MeasureSystemTemperature + AtmosphereRemoval + '
                      f'Level1AveragingGainCorrection, PNG writing on) on the same C1 observation: {rs:.2f} s, '
                      f'1 process, 8-core Xeon build container (no GPU box: the reference never travels); '
                      f'tests/golden/golden_meta.json reference_timings_s_c1'}
    rcb = meta.get('reference_cpu_baseline')
    if rcb:
        # SURVEY §8(d) / BASELINE.md §3: the reference as its MPI file split runs it, one
        # observation per process on the build container's cores, one BLAS thread each
        k8 = next((k for k in rcb if k.endswith('_processes_png_written')), None)
        k8s = next((k for k in rcb if k.endswith('_processes_savefig_stubbed')), None)
        for key, name in ((k8, 'reference_mpi_split'), (k8s, 'reference_mpi_split_savefig_stubbed'),
                          ('one_process_savefig_stubbed', 'reference_one_core_savefig_stubbed')):
            if key and key in rcb:
                r = rcb[key]
                procs = r['processes']
                out[name] = {
                    'value': r['samples_channels_per_s'], 'unit': 'samples*channels/s', 'cores': procs,
                    'kind': 'reference',
                    'sample': f"the reference v0.9.1 on {procs} C1 observation(s) ({procs} process(es), one "
                              f"observation and one BLAS thread each, run_average.py:38-39 file split; "
                              f"{'savefig stubbed' if 'stubbed' in key else 'PNG files written'}): "
                              f"{r.get('wall_s', r.get('seconds')):.1f} s wall, {rcb['host']}; "
                              'tests/golden/golden_meta.json reference_cpu_baseline'}
    dref = meta.get('reference_destriper_c4')
    if dref:
        out['destriper_reference'] = {
            'value': dref['iters_per_s'], 'unit': 'CG iterations/s', 'cores': 1, 'kind': 'reference',
            'sample': f"reference Destriper.cgm on {dref.get('inputs', 'a C4-size problem')} ({dref['n_samples']} "
                      f"samples, {dref['n_offsets']} offsets, 480x480 map, L=50): {dref['iters']} iterations in "
                      f"{dref['seconds']:.1f} s (3 matvecs/iteration as shipped), build container; "
                      'tests/golden/golden_meta.json reference_destriper_c4'}
    return out


def cpu_destriper_port(tod, w, pix, L, npix, iters=3):
    """The oracle's destriper (NumPy + C binValues, one matvec per iteration) on the
    C4 problem: a few fixed iterations (bounded sample)."""
    from threadpoolctl import threadpool_limits
    import oracle.destriper as od
    p = np.asarray(pix, dtype=np.int64)
    t = np.asarray(tod, dtype=np.float64)
    ww = np.asarray(w, dtype=np.float64)
    with threadpool_limits(1):
        A = lambda x: od.op_Ax(x, p, ww, L, npix)          # noqa: E731
        b = od.op_Ax(t, p, ww, L, npix, extend=False)
        t0 = time.perf_counter()
        od.cgm(A, b, threshold=0.0, niter=iters)
        dt = time.perf_counter() - t0
    return {'value': iters / dt, 'unit': 'CG iterations/s', 'cores': 1, 'kind': 'port',
            'sample': f'oracle/destriper.py cgm, {iters} iterations on the C4 problem ({t.size} samples), '
                      f'{dt:.2f} s on 1 host core of the GPU box'}


def check_against_oracle(data, level2, device):
    """Full-size parity: one (feed, scan) unit of the device cube reduced by the oracle."""
    import oracle.l1 as ol1
    from comapreduce_amd.pipeline.datahandling import to_host
    obs = data._gpu_observation
    f, s, t0, n = (int(v) for v in obs.units[len(obs.units) // 2])
    tod_f = data['spectrometer/tod'][f].cpu().numpy()
    A = 1.0 / np.sin(np.asarray(data['spectrometer/pixel_pointing/pixel_el'])[f] * np.pi / 180.0)
    fit = ol1.fit_atmosphere(A[t0:t0 + n], tod_f[0, :, t0:t0 + n])
    tsys0 = to_host(level2['vane/system_temperature'])[0, f]
    gain0 = to_host(level2['vane/system_gain'])[0, f]
    fitv = to_host(level2['atmosphere/fit_values'])[s, f]
    r, o, w, _ = ol1.reduce_scan(tod_f[..., t0:t0 + n].copy(), A[t0:t0 + n], fitv, tsys0, gain0, is_first_scan=(s == 0))
    g = to_host(level2['averaged_tod/tod'])[f, :, t0:t0 + n]
    err = float(np.max(np.abs(g - r)) / np.max(np.abs(r)))
    ferr = float(np.nanmax(np.abs(fitv[0, 0] - fit[0])) / np.nanmax(np.abs(fit[0])))
    return {'unit': [f, s, t0, n], 'tod_rel_err': err, 'fit_rel_err': ferr}


# ---------------------------------------------------------------- destriper legs
def level2_store(level2, data, obsid):
    """The Level-2 'file' read_comap_data reads (COMAPData.py:247-427), built from a
    reduced observation: {filename: (datasets, attrs)} on the host."""
    from comapreduce_amd.pipeline.datahandling import to_host
    F = int(np.asarray(to_host(data['spectrometer/feeds'])).size)
    ds = {'averaged_tod/tod': to_host(level2['averaged_tod/tod']),
          'averaged_tod/tod_original': to_host(level2['averaged_tod/tod_original']),
          'averaged_tod/weights': to_host(level2['averaged_tod/weights']),
          'averaged_tod/scan_edges': np.asarray(to_host(level2['averaged_tod/scan_edges'])),
          'spectrometer/feeds': np.asarray(to_host(data['spectrometer/feeds'])),
          'spectrometer/MJD': np.asarray(to_host(data['spectrometer/MJD']))}
    for k in ('ra', 'dec', 'az', 'el'):
        ds[f'spectrometer/pixel_pointing/pixel_{k}'] = np.asarray(to_host(data[f'spectrometer/pixel_pointing/pixel_{k}']))
    attrs = {'comap': {'source': 'Field00', 'obsid': obsid, 'bad_observation': np.zeros(max(20, F + 1), np.int64)}}
    name = f'comap-{obsid:07d}-2020-06-01-000000_Level2Cont.hd5'
    return {name: (ds, attrs)}


def c4_map_info():
    """480 x 480 CAR map at 1' on the synthetic field centre."""
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.comapdata import map_info_from
    return map_info_from([synthetic.FIELD_RA, synthetic.FIELD_DEC], [-1.0 / 60.0, 1.0 / 60.0], [240, 240],
                         ['RA---CAR', 'DEC--CAR'], 480, 480)


def _timed_solve(prob, threshold, niter):
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = prob.solve(threshold=threshold, niter=niter)
    torch.cuda.synchronize()
    return res, time.perf_counter() - t0


def _timed_setup(*args, **kw):
    """DeviceDestriper set-up on device-resident inputs (comap_destripe_create_bands:
    spatial order, offset rows, pixel-major transpose, sample-level maps)."""
    import torch
    from comapreduce_amd.mapmaking import destriper as D
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prob = D.DeviceDestriper(*args, **kw)
    torch.cuda.synchronize()
    return prob, time.perf_counter() - t0


def operator_bytes(prob, NO, n_bands):
    """HBM bytes one CG iteration of the batched operator must move: the
    offset-major and pixel-major entries streamed once each (4 B index + NB count
    bytes in the count form, else + 8 NB B of weights), the row pointers, and the
    offset vectors of 8 NB B (bin gather source excluded as cache resident, like
    SURVEY's map): project x / ws / y (+ wbar), update x r p q in + x r out,
    direction p r in + p out (+ wbar in, pt out)."""
    nb = 4 if n_bands == 3 else n_bands
    nnz, nnzp = prob.nnz()
    eb = prob.entry_bytes()
    nvec = 13 + (3 if eb == 4 + nb else 0)
    return (nnz + nnzp) * eb + 8 * (NO + 1) + nvec * NO * 8 * nb


def _iters(res):
    it = res['iters']
    return max(it) if isinstance(it, (list, tuple)) else it


def destriper_leg(level2, data, niter, device, want_cpu=False):
    """C4: COMAPData.read_comap_data (host prep + batched device w=400 median) on this
    observation's Level-2 output (band 0, 19 feeds, L = 50, 480x480 CAR), then the
    device destriper: set-up on device-resident inputs, the reference's own stopping
    rule (threshold 1e-6, run_destriper.py:96-97, Destriper.py:134-141) timed to
    convergence with the final maps, and CG iterations / s over a fixed niter with
    early exit disabled (single rank)."""
    import torch
    from comapreduce_amd.mapmaking import comapdata as CD
    dev = torch.device('cuda', device)
    store = level2_store(level2, data, obsid=int(data.obsid) if data.obsid > 0 else 1)
    t0 = time.perf_counter()
    tod, w, pix = CD.read_comap_data(list(store), c4_map_info(), iband=0, offset_length=50, store=store,
                                     device=device)[:3]
    prep = time.perf_counter() - t0
    td, wd, pd = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (tod, w, pix.astype(np.int32)))
    _timed_setup(pd, td, wd, 50, 480 * 480, device=device, map_shape=(480, 480))   # warm (module load, allocations)
    prob, setup = _timed_setup(pd, td, wd, 50, 480 * 480, device=device, map_shape=(480, 480))
    prob.solve(threshold=0.0, niter=3)   # warm
    conv, conv_s = _timed_solve(prob, 1e-6, 100)
    res, dt = _timed_solve(prob, 0.0, niter)
    out = {'config': 'C4: read_comap_data (band 0, 19 feeds) -> destriper, L=50, 480x480 CAR, '
                     f'{niter} CG iterations (no early exit), single rank',
           'cg_iters_per_s': res['iters'] / dt, 'iters': res['iters'], 'n_samples': int(tod.size),
           'n_offsets': int(tod.size // 50), 'prep_s': prep, 'setup_ms': setup * 1e3, 'nnz': prob.nnz(),
           'converged': {'threshold': 1e-6, 'iters': conv['iters'], 'solve_ms': conv_s * 1e3,
                         'setup_plus_solve_ms': (setup + conv_s) * 1e3}}
    # all 4 sidebands: one batched read (one device median call) and ONE batched solve
    t0 = time.perf_counter()
    r = CD.read_comap_data_bands(list(store), c4_map_info(), bands=(0, 1, 2, 3), offset_length=50, store=store,
                                 device=device)
    prep4 = time.perf_counter() - t0
    t4, w4, p4, k4 = (torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                      for a in (r['tod'], r['weights'], r['pointing'].astype(np.int32), r['keep']))
    _timed_setup(p4, t4, w4, 50, 480 * 480, device=device, keep=k4, map_shape=(480, 480))   # warm (first use)
    prob4, setup4 = _timed_setup(p4, t4, w4, 50, 480 * 480, device=device, keep=k4, map_shape=(480, 480))
    prob4.solve(threshold=0.0, niter=3)
    conv4, conv4_s = _timed_solve(prob4, 1e-6, 100)
    res4, dt4 = _timed_solve(prob4, 0.0, niter)
    it4 = max(res4['iters'])
    out['bands4'] = {'config': 'C4, all 4 sidebands batched (read_comap_data_bands -> one batched solve)',
                     'band_iters_per_s': 4 * it4 / dt4, 'cg_iters_per_s': it4 / dt4, 'iters': res4['iters'],
                     'n_samples_union': int(r['pointing'].size), 'prep_s': prep4, 'setup_ms': setup4 * 1e3,
                     'converged': {'threshold': 1e-6, 'iters': conv4['iters'], 'solve_ms': conv4_s * 1e3,
                                   'setup_plus_solve_ms': (setup4 + conv4_s) * 1e3}}
    if want_cpu:
        out['cpu_port'] = cpu_destriper_port(tod, w, pix, 50, 480 * 480)
    return out


def destriper_c5_leg(n_obs, niter, device, world, rank, n_bands=1):
    """C5: the destriper on n_obs synthetic observations' Level-2 TOD
    (19 feeds x 180,000 samples each, L = 50, 480x480 1' CAR map) per GPU, weak-scaled:
    every rank holds its own observations; with several ranks the map numerator and
    the CG scalars are summed over RCCL every iteration.  n_bands > 1: that many
    sidebands on the same pointing as one batched system.  Roofline on SURVEY
    §8(d)'s algorithmic bytes: 24 B per sample + 80 B per offset per band-iteration."""
    import torch
    import torch.distributed as dist
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    L, npix = 50, 480 * 480
    pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=L, device=device, seed=1000 + rank,
                                                    n_bands=n_bands)
    _timed_setup(pix, tod, w, L, npix, device=device, map_shape=(480, 480))        # warm (first use of these sizes)
    prob, setup = _timed_setup(pix, tod, w, L, npix, device=device, map_shape=(480, 480))
    prob.solve(threshold=0.0, niter=3)   # warm (graph capture, RCCL communicators)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    conv, conv_s = _timed_solve(prob, 1e-6, 100)
    if world > 1:
        dist.barrier()
    res, dt = _timed_solve(prob, 0.0, niter)
    if world > 1:
        e = torch.tensor([dt], device='cuda', dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dt = float(e.item())
    N = int(pix.numel())
    NO = N // L
    it = max(max(res['iters']) if n_bands > 1 else res['iters'], 1)
    algo = DESTRIPER_BYTES_PER_SAMPLE * N + DESTRIPER_BYTES_PER_OFFSET * NO     # per band-iteration
    ms = dt / it * 1e3
    ms_band = ms / n_bands
    op_bytes = operator_bytes(prob, NO, n_bands)
    comm = None
    if world > 1:       # the measured per-iteration all-reduce time and bytes (rankplan's alpha / beta)
        ta = D.TimedAllreduce()
        prob.solve(threshold=0.0, niter=20, allreduce=ta)
        comm = ta.summary(20)
    return {'comm_rank0': comm, 'config': f'C5: {n_obs} obs x 19 feeds x 180000 samples per GPU, {n_bands} band(s) per solve, L={L}, '
                      f'480x480 CAR, {niter} CG iterations (no early exit), {world} rank(s)',
            'cg_iters_per_s': it / dt, 'band_iters_per_s': n_bands * it / dt, 'ms_per_iter': ms,
            'ms_per_band_iter': ms_band, 'iters': res['iters'],
            'n_samples_per_gpu': N, 'n_offsets_per_gpu': NO, 'nnz': prob.nnz(), 'setup_ms': setup * 1e3,
            'converged': {'threshold': 1e-6, 'iters': conv['iters'], 'solve_ms': conv_s * 1e3,
                          'setup_plus_solve_ms': (setup + conv_s) * 1e3},
            # SURVEY §8(d) prices a band-iteration at 24 B/sample + 80 B/offset; the batched
            # operator never moves those bytes (entries fold samples, bands share the pixel
            # stream), so their ratio to the operator's own bytes is a work saving, not a
            # bandwidth; the roofline is operator_roofline_frac below
            'survey_bytes_per_band_iter_per_gpu': algo,
            'work_saving_vs_survey_bytes': algo * n_bands / max(op_bytes, 1),
            'operator_bytes_per_iter': op_bytes, 'entry_bytes': prob.entry_bytes(),
            'sell_entries': prob.sell_entries(),
            'operator_roofline_frac': op_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def allreduce_probe(dev, sizes, reps=30):
    """Measured RCCL all-reduce cost on this node at the CG's message sizes (bytes): per
    size the mean of ``reps`` back-to-back collectives between device syncs, then the
    least-squares alpha (us) + bytes / beta (GB/s) line that mapmaking/rankplan.py's
    cost model takes (scripts/rankplan_calibrate.py turns these fields of the SCALE runs
    into its table).  Collective: every rank calls it."""
    import torch
    import torch.distributed as dist
    pts = []
    for b in sizes:
        t = torch.zeros(max(1, int(b) // 8), dtype=torch.float64, device=dev)
        for _ in range(3):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / reps * 1e6
        e = torch.tensor([us], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        pts.append({'bytes': int(t.numel() * 8), 'us': float(e.item())})
    x = np.array([p['bytes'] for p in pts], float)
    y = np.array([p['us'] for p in pts], float)
    A = np.stack([np.ones_like(x), x], axis=1)
    (alpha, slope), *_ = np.linalg.lstsq(A, y, rcond=None)
    return {'n_ranks': dist.get_world_size(), 'backend': dist.get_backend(), 'reps': reps, 'points': pts,
            'alpha_us': float(alpha), 'beta_GBs': float(1e-3 / slope) if slope > 0 else None}


FIELD_KAPPA = 6.5     # entries-equivalent CG work of one offset (rankplan.balanced_ranges weights)


def field_split(n_obs, world, n_feeds=19, kappa=FIELD_KAPPA, device='cpu'):
    """The field's (obs, feed) series dealt to ``world`` ranks as contiguous ranges balanced
    on the CG work each rank takes on: its operator entries (the (offset, pixel run) pairs
    of its pointing) + kappa x its offsets (rankplan.balanced_ranges).  Equal observation
    counts (run_destriper.py:131-138's len // size split) left rank 0 with 1.32 / 1.63 /
    1.86 x the mean entries at 2 / 4 / 8 ranks: the synthetic scan slows down with the
    observation index.  COMAP_FIELD_SPLIT=obs restores the equal split.  Returns
    ([(lo, hi)] series ranges, per-series entries, offsets per series)."""
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import rankplan
    ent, no = synthetic.field_series_work(n_obs, n_feeds=n_feeds, device=device)
    if os.environ.get('COMAP_FIELD_SPLIT', 'work') == 'obs':
        return [(n_feeds * (n_obs * r // world), n_feeds * (n_obs * (r + 1) // world)) for r in range(world)], ent, no
    w = np.round(ent + kappa * no).astype(np.int64)
    return rankplan.balanced_ranges(w, world), ent, no


def destriper_c5_field_leg(n_obs, niter, device, world, rank, n_bands=4):
    """configs[4] as stated: n_obs (64) synthetic observations x 19 feeds x 180,000 samples
    co-added into ONE 480 x 480 1' CAR field map and solved as one system (run_destriper.py:
    131-189 puts every rank's files into one map).  On N ranks the (obs, feed) series are
    dealt in contiguous ranges balanced on CG work (field_split), so total work is fixed
    ("scaling": strong): the map numerator (compacted to the hit pixels) and the CG block
    partials are all-reduced over RCCL every iteration.  Reports the set-up, ms per CG
    iteration (fixed niter, no early exit; the max over ranks) and the converged solve
    (threshold 1e-6); with N > 1 also, per rank, the entries, samples, set-up ms and the
    rank's own compute ms per CG iteration (its local operator solved alone, no
    collectives), the measured per-iteration all-reduce time and bytes (TimedAllreduce)
    and the RCCL alpha / beta probe at the CG's message sizes."""
    import torch
    import torch.distributed as dist
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    from comapreduce_amd.mapmaking import rankplan
    L, npix = 50, 480 * 480
    ranges, ent, no = field_split(n_obs, world, device=device)
    lo, hi = ranges[rank]
    pix, tod, w = synthetic.destriper_inputs_device(0, offset_length=L, device=device, seed=5000,
                                                    n_bands=n_bands, series=(lo, hi))
    _timed_setup(pix, tod, w, L, npix, device=device, map_shape=(480, 480))          # warm (first use of these sizes)
    prob, setup = _timed_setup(pix, tod, w, L, npix, device=device, map_shape=(480, 480))
    N_local = int(pix.numel())
    del pix, tod, w
    prob.solve(threshold=0.0, niter=3)   # warm
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    conv, conv_s = _timed_solve(prob, 1e-6, 100)
    if world > 1:
        dist.barrier()
    res, dt = _timed_solve(prob, 0.0, niter)
    it = max(max(res['iters']) if n_bands > 1 else res['iters'], 1)
    local = {'nnz': int(prob.nnz()[0]), 'n_samples': N_local, 'setup_ms': setup * 1e3}
    times = [dt, setup, conv_s]
    if world > 1:
        e = torch.tensor(times, device='cuda', dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        times = [float(v) for v in e.tolist()]
    dt, setup, conv_s = times
    N = N_local
    if world > 1:
        nt = torch.tensor([N_local], device='cuda', dtype=torch.int64)
        dist.all_reduce(nt)
        N = int(nt.item())
    w_ranks = [float(ent[a:b].sum() + FIELD_KAPPA * no * (b - a)) for a, b in ranges]
    out = {'config': f'configs[4]: {n_obs} obs x 19 feeds x 180000 samples co-added into ONE 480x480 CAR field map, '
                     f'{n_bands} bands batched, L={L}, split over {world} rank(s) by CG work (strong scaling), '
                     f'{niter} CG iterations (no early exit)',
           'n_samples_per_band': N, 'n_offsets': N // L, 'n_samples_rank0': N_local,
           'setup_ms': setup * 1e3, 'ms_per_iter': dt / it * 1e3, 'cg_iters_per_s': it / dt,
           'band_iters_per_s': n_bands * it / dt, 'iters': res['iters'],
           'converged': {'threshold': 1e-6, 'iters': conv['iters'], 'solve_ms': conv_s * 1e3,
                         'setup_plus_solve_ms': (setup + conv_s) * 1e3},
           'scaling': 'strong', 'nnz_rank0': prob.nnz(), 'entry_bytes': prob.entry_bytes(),
           'split': {'policy': os.environ.get('COMAP_FIELD_SPLIT', 'work'), 'kappa': FIELD_KAPPA,
                     'series_ranges': [list(map(int, r)) for r in ranges],
                     'modelled_work_max_over_mean': max(w_ranks) / (sum(w_ranks) / len(w_ranks)),
                     'entries_max_over_mean': rankplan.imbalance(ent, ranges)}}
    if world == 1:
        op_bytes = operator_bytes(prob, N // L, n_bands)
        out['operator_bytes_per_iter'] = op_bytes
        out['operator_roofline_frac'] = op_bytes / (dt / it) / 1e9 / HBM_PEAK_GBS
    else:
        ta = D.TimedAllreduce()
        prob.solve(threshold=0.0, niter=20, allreduce=ta)
        out['comm_rank0'] = ta.summary(20)
        nb = 4 if n_bands == 3 else n_bands
        nmap = int(prob.hit_index.numel()) if prob.hit_index is not None else npix
        out['allreduce_probe'] = allreduce_probe(torch.device('cuda', device),
                                                 [8 * nb, 8 * nb * 1024, 8 * nb * nmap, 1 << 20])
        # each rank's own compute per CG iteration: its local operator solved alone (no
        # collectives) -- the imbalance the sharded iteration waits on, and what remains
        # once the all-reduce cost (comm_rank0) is known
        prob.ops.solve_native(0.0, 3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prob.ops.solve_native(0.0, niter)
        torch.cuda.synchronize()
        local['local_ms_per_iter'] = (time.perf_counter() - t0) / niter * 1e3
        vec = torch.tensor([local['nnz'], local['n_samples'], local['setup_ms'], local['local_ms_per_iter']],
                           dtype=torch.float64, device='cuda')
        parts = [torch.zeros_like(vec) for _ in range(world)]
        dist.all_gather(parts, vec)
        rows = [p.tolist() for p in parts]
        out['per_rank'] = {'nnz': [int(r[0]) for r in rows], 'n_samples': [int(r[1]) for r in rows],
                           'setup_ms': [r[2] for r in rows], 'local_ms_per_iter': [r[3] for r in rows]}
        lm = [r[3] for r in rows]
        out['per_rank']['local_iter_max_over_mean'] = max(lm) / (sum(lm) / len(lm))
    del prob, res, conv
    torch.cuda.empty_cache()
    return out


def pointing_device(data, dev):
    """The observation's pixel pointing resident in HBM beside the Level-1 cube (input
    data of the chain, uploaded before its timed region as the cube is)."""
    import torch
    out = {}
    for k in ('ra', 'dec', 'az', 'el'):
        v = data[f'spectrometer/pixel_pointing/pixel_{k}']
        out[k] = (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v, np.float64))).to(dev)
    return out


def level2_store_device(level2, data, obsid, dev, pointing=None):
    """level2_store with the Level-2 TOD left where the stages wrote it (HBM) and the
    pointing resident beside the Level-1 cube: the in-memory hand-off of the chain leg."""
    from comapreduce_amd.pipeline.datahandling import to_host
    pointing = pointing if pointing is not None else pointing_device(data, dev)
    F = int(np.asarray(to_host(data['spectrometer/feeds'])).size)
    ds = {'averaged_tod/tod': level2['averaged_tod/tod'],
          'averaged_tod/tod_original': level2['averaged_tod/tod_original'],
          'averaged_tod/weights': level2['averaged_tod/weights'],
          'averaged_tod/scan_edges': np.asarray(to_host(level2['averaged_tod/scan_edges'])),
          'spectrometer/feeds': np.asarray(to_host(data['spectrometer/feeds'])),
          'spectrometer/MJD': np.asarray(to_host(data['spectrometer/MJD']))}
    for k in ('ra', 'dec', 'az', 'el'):
        ds[f'spectrometer/pixel_pointing/pixel_{k}'] = pointing[k]
    attrs = {'comap': {'source': 'Field00', 'obsid': obsid, 'bad_observation': np.zeros(max(20, F + 1), np.int64)}}
    name = f'comap-{obsid:07d}-2020-06-01-000000_Level2Cont.hd5'
    return {name: (ds, attrs)}


def chain_leg(data, device, l1_bytes, reps=3):
    """north_star end to end on one GPU (BASELINE.json): the resident C2
    Level-1 cube -> the three stages (Level-2 TOD kept in HBM) -> read_comap_data_bands
    (device prep of all 4 sidebands, run_destriper.py:146-189 reading the files the
    reduction wrote) -> one batched destriper solve to the reference's stopping rule
    (threshold 1e-6, at most 100 iterations: run_destriper.py:96-97, Destriper.py:134-141)
    -> the 4 bands' maps (map, naive, weight, hits) copied to the host.

    Timed as one host wall clock per chain, no synchronisation between the phases: the
    pointing-only part of the prep (az / el percentiles, prep.precompute_pointing) is
    enqueued on a side stream as soon as the reduction's last stage has been queued, so
    it runs beside the reduction's tail.  The median of ``reps`` chains; 5 extra chains
    with a device sync at every phase boundary give the phase breakdown (per-phase median).  Roofline: the
    L1 passes' design bytes + the operator bytes of every CG iteration, over the wall."""
    import torch
    chain = chain_fn(data, device)
    chain(False)                                   # warm the prep / set-up paths
    # per-phase median of 5 synced chains: one synced chain's prep phase moved 2.4 - 5.7 ms
    # with the host's scheduling (r05ab3)
    synced = []
    for _ in range(5):
        ph = chain(True)
        ph.pop('maps')
        synced.append(ph)
    phases = {k: (float(np.median([p[k] for p in synced])) if k.endswith('_ms') else v) for k, v in synced[-1].items()}
    walls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = chain(False)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        # the job's output is consumed (checked) before the next job starts, so its pinned
        # host block returns to torch's host cache; a map set still held when the next
        # solve starts costs that solve a fresh 29 MB pinned allocation (~2.5 ms)
        assert np.isfinite(info.pop('maps')['map']).all(), 'chain maps not finite'
    wall = sorted(walls)[len(walls) // 2]
    algo = l1_bytes + info['op_bytes'] * max(info['iters'])
    return {'config': 'north_star chain, 1 GPU: C2 resident cube -> vane + atmosphere + L1AveragingGainCorrection -> '
                      'read_comap_data_bands (4 sidebands, device prep) -> batched destriper to threshold 1e-6 '
                      '(max 100 it), L=50, 480x480 CAR -> 4 bands of maps on the host',
            'reps': reps, 'wall_ms': wall, 'wall_ms_all': walls, 'iters': info['iters'],
            'phases_synced_ms': {k: v for k, v in phases.items() if k.endswith('_ms')},
            'phases_note': 'per-phase median of 5 extra chains with a device sync at every phase boundary (no overlap)',
            'algo_bytes': algo, 'achieved_GBs': algo / (wall * 1e-3) / 1e9,
            'roofline_frac': algo / (wall * 1e-3) / 1e9 / HBM_PEAK_GBS,
            'roofline_note': 'algorithmic bytes = the 3 L1 streaming passes (design bytes) + the batched operator '
                             'bytes x CG iterations; prep, set-up and map copy move ~1.5 GB and count as overhead'}


def chain_fn(data, device):
    """The chain of chain_leg as a callable ``chain(sync) -> info`` (sync: a device
    sync and a wall-clock mark at every phase boundary)."""
    import torch
    from comapreduce_amd.mapmaking import comapdata as CD
    from comapreduce_amd.mapmaking import destriper as D
    from comapreduce_amd.mapmaking import prep as P
    dev = torch.device('cuda', device)
    obsid = int(data.obsid) if data.obsid > 0 else 1
    pointing = pointing_device(data, dev)          # resident input, like the cube
    side = torch.cuda.Stream(dev)

    def chain(sync):
        ph = {}
        t = [time.perf_counter()]

        def mark(k):
            if sync:
                torch.cuda.synchronize()
                now = time.perf_counter()
                ph[k] = (now - t[0]) * 1e3
                t[0] = now
        level2 = reduce_step(data, device)
        mark('l1_ms')
        store = level2_store_device(level2, data, obsid, dev, pointing)
        with torch.cuda.stream(side):      # the pointing has been resident since before the chain
            pp = P.precompute_pointing([CD.Level2File(*store[k], k) for k in store], list(store),
                                       [i + 1 for i in range(19)], device)
        r = CD.read_comap_data_bands(list(store), c4_map_info(), bands=(0, 1, 2, 3), offset_length=50, store=store,
                                     device=device, device_outputs=True, pointing=pp)
        mark('prep_ms')
        prob = D.DeviceDestriper(r['pointing'].to(torch.int32), r['tod'], r['weights'], 50, 480 * 480,
                                 device=device, keep=r['keep'], map_shape=(480, 480))
        mark('setup_ms')
        res = prob.solve(threshold=1e-6, niter=100, to_host=True)    # maps copied to the host
        mark('solve_and_maps_ms')
        ph['maps'] = res['maps']           # checked by the caller, outside the timed region
        ph['iters'] = res['iters']
        ph['op_bytes'] = operator_bytes(prob, int(r['tod'].shape[1]) // 50, 4)
        ph['n_samples_union'] = int(r['tod'].shape[1])
        return ph
    return chain


def e2e_leg(F, T, device):
    """C2 from host memory, the Runner path (Running.py:120-153): the Level-1 cube is
    a pageable host NumPy array (as read from a file), the stages upload it
    (gpu.upload: pinned double-buffered chunks on a copy stream), reduce, and hand
    back host Level-2 arrays.  Timed: upload + the three stages + outputs to host."""
    import torch
    from comapreduce_amd.gpu import gpu_observation
    from comapreduce_amd.pipeline.datahandling import COMAPLevel1
    dev_data, _ = build_observation(F, T, obs_id=1, device=device)
    host = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in dev_data.items():
        host[k] = v.cpu().numpy() if hasattr(v, 'cpu') else v
    for p, a in dev_data.items(attr=True):
        for k, v in a.items():
            host.set_attrs(p, k, v)
    del dev_data
    torch.cuda.empty_cache()
    nbytes = host['spectrometer/tod'].nbytes
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gpu_observation(host, device)                  # upload (what the first stage does)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t0
    level2 = reduce_step(host, device, device_outputs=False)
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    assert isinstance(level2['averaged_tod/tod'], np.ndarray)
    sampch = F * 4 * 1024 * T
    del host, level2
    torch.cuda.empty_cache()
    return {'config': f'C2 from a host (pageable) cube: upload + 3 stages + host Level-2 outputs, {F} feeds',
            'value': sampch / t_all, 'unit': 'samples*channels/s', 'seconds': t_all, 'upload_s': t_up,
            'upload_GBs': nbytes / t_up / 1e9, 'reduce_and_outputs_s': t_all - t_up}


# ---------------------------------------------------------------- main
def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one rank per GPU; COMAP_DIST_BACKEND=gloo with more ranks than GPUs is a rehearsal
    # mode only (ranks share devices; RCCL refuses duplicate GPUs)
    backend = os.environ.get('COMAP_DIST_BACKEND', 'nccl')
    device = local % max(torch.cuda.device_count(), 1) if backend == 'gloo' else local
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', device))
        else:
            dist.init_process_group(backend)
    F, T = args.feeds, args.samples
    shard = args.mode == 'shard' and world > 1
    if shard:
        data, sh = build_observation(F, T, obs_id=1, device=device, rank=rank, world=world)
    elif args.shard_of > 1:
        data, sh = build_observation(F, T, obs_id=1, device=device, rank=0, world=args.shard_of)
    else:
        data, sh = build_observation(F, T, obs_id=rank + 1, device=device)
    cube_sampch = F * 4 * 1024 * T                 # one observation's cube
    job_sampch = cube_sampch if shard else world * cube_sampch

    for _ in range(max(args.warmup, 1)):       # the first step also creates the plan
        level2 = reduce_step(data, device)
    obs = data._gpu_observation
    # timed region: HIP events around the three streaming passes only (the roofline's
    # kernel); the per-kernel breakdown comes from extra untimed steps below
    obs.profile(1)
    obs.profile_collect()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_ms = {}
    for _ in range(args.steps):
        level2 = reduce_step(data, device, host_ms)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    prof = obs.profile_collect()
    obs.profile(2)
    n_kprof = max(1, min(args.steps, 3))
    for _ in range(n_kprof):
        level2 = reduce_step(data, device)
    kprof = obs.profile_collect()
    obs.profile(False)
    rank_ms = None
    if world > 1:
        e = torch.tensor([elapsed], device='cuda', dtype=torch.float64)
        parts = [torch.zeros_like(e) for _ in range(world)]
        dist.all_gather(parts, e)               # every rank's own step time (the shard balance)
        rank_ms = [float(p.item()) / args.steps * 1e3 for p in parts]
        elapsed = max(float(p.item()) for p in parts)

    frac = obs.pass_fractions()
    vane_search_ms = getattr(obs, 'last_vane_search_ms', None)
    check = check_against_oracle(data, level2, device) if (args.check and rank == 0) else None
    dstr = None
    if not args.no_destriper and not shard:
        dstr = destriper_leg(level2, data, args.destriper_iters, device,
                             want_cpu=(rank == 0 and world == 1 and not args.no_cpu_baseline))
        if world > 1:
            v = torch.tensor([dstr['cg_iters_per_s']], device='cuda', dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
            dstr['cg_iters_per_s_min_over_ranks'] = float(v.item())

    chain = None
    if not args.no_destriper and not shard and world == 1 and not args.no_chain:
        scan_sc0 = sh.samples_x_channels()
        l1_bytes = sum(ALGO_BYTES_PER_SAMPCH_PASS * scan_sc0 * frac[k] for k in type_streaming())
        chain = chain_leg(data, device, l1_bytes)

    c5 = None
    if not args.no_destriper and args.c5_obs > 0:
        del data, level2, obs
        torch.cuda.empty_cache()
        c5 = destriper_c5_leg(args.c5_obs, args.destriper_iters, device, world, rank)
        torch.cuda.empty_cache()
        c5['bands4'] = destriper_c5_leg(args.c5_obs, args.destriper_iters, device, world, rank, n_bands=4)
    c5f = None
    if not args.no_destriper and args.c5_field_obs > 0:
        if c5 is None:
            del data, level2, obs
        torch.cuda.empty_cache()
        c5f = destriper_c5_field_leg(args.c5_field_obs, args.destriper_iters, device, world, rank)

    e2e = None
    if not args.no_e2e and world == 1:
        e2e = e2e_leg(F, T, device)

    if rank == 0:
        value = job_sampch * args.steps / elapsed
        scan_sc = sh.samples_x_channels()
        stream = {k: prof[k] for k in type_streaming()}
        pass_bytes = {k: ALGO_BYTES_PER_SAMPCH_PASS * scan_sc * frac[k] for k in type_streaming()}
        dom = max(stream, key=lambda k: stream[k][0])
        ms_avg = stream[dom][0] / max(stream[dom][1], 1)
        algo_bytes = pass_bytes[dom] * args.steps / max(stream[dom][1], 1)
        achieved = algo_bytes / (ms_avg * 1e-3) / 1e9
        design_bytes = sum(pass_bytes.values())
        # roofline.traffic is NOT measured in this run: PMC counters need their own
        # rocprofv3 passes (profiles/profile.sh); it is the committed per-launch HBM
        # bytes of the same kernel from the run named in traffic_source
        traffic, traffic_src = None, None
        tpath = os.path.join(ROOT, 'profiles', 'traffic_latest.json')
        if os.path.exists(tpath) and world == 1:
            tj = json.load(open(tpath))
            traffic = tj.get(dom)
            traffic_src = (f"committed rocprofv3 PMC measurement profiles/{tj.get('_source', 'r02q')}_traffic.json "
                           '(2 x FETCH_SIZE + WRITE_SIZE, separate passes), not measured in this run')
        step_ms = elapsed / args.steps * 1e3
        rank0_ms = (t1 - t0) / args.steps * 1e3
        if shard:
            workload = (f'C3: one {F}-feed x 4 x 1024 ch x {T}-sample L1 observation sharded by (feed, scan) units '
                        f'over {world} GPUs, no collectives (rank 0: feeds {sh.f_lo}..{sh.f_hi - 1}, '
                        f'{len(sh.units)} units)')
            par = f'(feed, scan)-sharded x{world}'
        else:
            workload = (f'C2: {F}-feed x 4 x 1024 ch x {T} samples L1 observation per GPU '
                        f'({cube_sampch * 4 / 1e9:.1f} GB f32 resident in HBM), vane + atmosphere + '
                        'L1AveragingGainCorrection')
            par = f'observation-parallel x{world}'
        line = {
            'metric': 'TOD samples x channels / s (L1 -> L2 reduction)',
            'value': value,
            'unit': 'samples*channels/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': step_ms,
            'higher_is_better': True,
            'scaling': 'strong' if shard else 'weak',
            'vs_baseline': None,
            'dtype': 'f32 in, f64 accumulate',
            'data': 'synthetic (SURVEY.md §8d spec, generated on device)',
            'config': {'workload': workload, 'parallelism': par},
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic, 'traffic_source': traffic_src,
                         'algo_bytes_per_launch': algo_bytes, 'avg_launch_ms': ms_avg},
            'l1_step_roofline': {'passes': len(type_streaming()), 'design_bytes': design_bytes,
                                 'rank0_ms_per_step': rank0_ms,
                                 'achieved_GBs': design_bytes / (rank0_ms * 1e-3) / 1e9,
                                 'frac': design_bytes / (rank0_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                 'pass_channel_fraction': frac,
                                 # SURVEY §8(d) prices 4 streaming passes; this design does the
                                 # same reduction in 3 (a work saving, not a bandwidth figure)
                                 'survey_4pass_bytes': SURVEY_BYTES_PER_SAMPCH * scan_sc,
                                 'work_saving_vs_survey_4pass': SURVEY_BYTES_PER_SAMPCH * scan_sc / design_bytes},
            'kernel_ms_per_step': {k: v[0] / n_kprof for k, v in kprof.items()},
            'kernel_ms_note': f'HIP events around every kernel, {n_kprof} extra steps after the timed region',
            'host_stage_ms_per_step': {k: v / args.steps for k, v in host_ms.items()},
            'host_vane_search_ms': vane_search_ms,
            'pass_GBs': {k: pass_bytes[k] / (stream[k][0] / args.steps * 1e-3) / 1e9
                         for k in type_streaming() if stream[k][1] > 0},
            'launches_per_step': {k: stream[k][1] / args.steps for k in type_streaming()},
        }
        if dstr is not None:
            line['destriper'] = dstr
        if c5 is not None:
            line['destriper_c5'] = c5
        if c5f is not None:
            line['destriper_c5_field'] = c5f
        if rank_ms is not None:
            line['rank_ms_per_step'] = rank_ms
        if chain is not None:
            line['chain_l1_to_maps'] = chain
        if e2e is not None:
            line['end_to_end_host'] = e2e
        if check is not None:
            line['check'] = check
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline()
            if dstr is not None and 'cpu_port' in dstr:
                cb['destriper_port'] = dstr.pop('cpu_port')
            line['cpu_baseline'] = cb
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def type_streaming():
    from comapreduce_amd.gpu import GPUObservation
    return GPUObservation.STREAMING


if __name__ == '__main__':
    main()
