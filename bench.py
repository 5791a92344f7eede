#!/usr/bin/env python3
"""bench.py -- COMAP Level-1 -> Level-2 reduction throughput on MI355X.

Metric (BASELINE.json): TOD samples x channels / s for the L1 -> L2 reduction
(MeasureSystemTemperature -> AtmosphereRemoval -> Level1AveragingGainCorrection)
of the full 19-feed x 4 x 1024-channel x 180,000-sample synthetic observation
(configs[1], 56 GB f32 resident in HBM) per GPU, plus the destriper's CG
iterations / s on the resulting band-0 Level-2 TOD.

One step = one complete reduction of one observation (every kernel of the
three stages; the plan/airmass set-up happens once per observation, like
opening the file).  N GPUs: one process per GPU (torch.distributed.run), each
reducing its own observation (obs_id = rank + 1) with no collective in the
reduction -- the reference's file-level MPI parallelism -- so scaling is
"weak"; the driver derives efficiency from the per-N values.

    python bench.py [--gpus N --steps K --warmup W]
"""
import argparse
import json
import os
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--feeds', type=int, default=19)
    ap.add_argument('--samples', type=int, default=180_000)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-destriper', action='store_true')
    ap.add_argument('--destriper-iters', type=int, default=100)
    ap.add_argument('--c5-obs', type=int, default=8, help='observations per GPU in the C5 destriper leg (0: skip)')
    ap.add_argument('--check', action='store_true', help='compare one unit against the CPU oracle')
    return ap.parse_args()


def build_observation(F, T, obs_id, device):
    """Device-resident synthetic Level-1 observation."""
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd import synthetic
    from comapreduce_amd.pipeline.datahandling import COMAPLevel1
    cfg = synthetic.SyntheticConfig(n_feeds=F, n_samples=T, obs_id=obs_id)
    meta, attrs, level, mult, hot = synthetic.level1_metadata(cfg)
    dev = torch.device('cuda', device)
    lv = torch.from_numpy(level).to(dev)
    mu = torch.from_numpy(mult).to(dev)
    ho = torch.from_numpy(hot).to(dev)
    tod = torch.empty((F, 4, 1024, T), dtype=torch.float32, device=dev)
    ba = torch.empty((F, 4, T), dtype=torch.float32, device=dev)
    c = N.ctx(device)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_synth_tod(c, F, T, 1000 + obs_id, N.dptr(lv), N.dptr(mu), N.dptr(ho), N.dptr(tod),
                                    N.dptr(ba)), c, 'comap_synth_tod')
    torch.cuda.synchronize(dev)
    del lv, mu, ho
    data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in meta.items():
        data[k] = v
    data['spectrometer/tod'] = tod
    data['spectrometer/band_average'] = ba
    for p, a in attrs.items():
        for k, v in a.items():
            data.set_attrs(p, k, v)
    return data


def reduce_step(data, device, timing=None):
    """One full L1 -> L2 reduction (outputs stay on the device).  ``timing``
    (a dict) collects host wall time per stage call (enqueue + host work)."""
    from comapreduce_amd import Analysis as A
    from comapreduce_amd.pipeline.datahandling import COMAPLevel2
    level2 = COMAPLevel2(filename='/nonexistent/level2.hd5')
    for cls in (A.MeasureSystemTemperature, A.AtmosphereRemoval, A.Level1AveragingGainCorrection):
        t0 = time.perf_counter()
        st = cls(level2=level2, device=device, device_outputs=True)
        if not st(data, level2):
            raise RuntimeError(f'{cls.__name__} stopped the file')
        level2.update(st)
        if timing is not None:
            timing[cls.__name__] = timing.get(cls.__name__, 0.0) + (time.perf_counter() - t0) * 1e3
    return level2


def cpu_baseline():
    """The CPU oracle (a NumPy/C restatement of the reference, 'port') on a
    bounded sample: the C1 observation (1 feed x 4 x 1024 x 30,000)."""
    from threadpoolctl import threadpool_limits
    import oracle.l1 as ol1
    from comapreduce_amd import synthetic
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000, obs_id=1))
    with threadpool_limits(1):
        t0 = time.perf_counter()
        ol1.reduce_level1(gen['data'])
        dt = time.perf_counter() - t0
    n = 1 * 4 * 1024 * 30_000
    return {'value': n / dt, 'unit': 'samples*channels/s', 'cores': 1, 'kind': 'port',
            'sample': f'C1 observation 1x4x1024x30000 ({n} samp*ch), full vane+atmosphere+L2 reduce, '
                      f'{dt:.2f} s on 1 host core (oracle/l1.py)'}


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


def destriper_leg(level2, data, niter, device):
    """Destriper CG iterations/s on the band-0 Level-2 TOD of this observation
    (C4-like: 19 feeds, L=50, 480x480 CAR map at 1'), single rank."""
    import torch
    from comapreduce_amd.mapmaking import destriper as D
    tod, w, pix = D.level2_to_destriper_inputs(level2, data, band=0, offset_length=50)
    t0 = time.perf_counter()
    prob = D.DeviceDestriper(pix, tod, w, 50, 480 * 480, device=device)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    prob.solve(threshold=0.0, niter=3)   # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = prob.solve(threshold=0.0, niter=niter)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {'cg_iters_per_s': res['iters'] / dt, 'iters': res['iters'], 'n_samples': int(tod.numel()),
            'n_offsets': int(tod.numel() // 50), 'setup_s': setup, 'nnz': prob.nnz()}


def destriper_c5_leg(n_obs, niter, device, world, rank):
    """C5: the destriper on n_obs synthetic observations' Level-2 TOD
    (19 feeds x 180,000 samples each, one band, L = 50, 480x480 1' CAR map) per GPU,
    weak-scaled: every rank holds its own observations; with several ranks the map
    numerator and the CG scalars are summed over RCCL every iteration.  Roofline on
    SURVEY §8(d)'s algorithmic bytes: 24 B per sample + 80 B per offset per iteration."""
    import torch
    import torch.distributed as dist
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    L, npix = 50, 480 * 480
    pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=L, device=device, seed=1000 + rank)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prob = D.DeviceDestriper(pix, tod, w, L, npix, device=device)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    prob.solve(threshold=0.0, niter=3)   # warm (graph capture, RCCL communicators)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = prob.solve(threshold=0.0, niter=niter)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([dt], device='cuda', dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        dt = float(e.item())
    N = int(tod.numel())
    NO = N // L
    it = max(res['iters'], 1)
    algo = 24 * N + 80 * NO
    ms = dt / it * 1e3
    return {'config': f'C5: {n_obs} obs x 19 feeds x 180000 samples per GPU, L={L}, 480x480 CAR, '
                      f'{niter} CG iterations (no early exit)',
            'cg_iters_per_s': it / dt, 'ms_per_iter': ms, 'iters': res['iters'],
            'n_samples_per_gpu': N, 'n_offsets_per_gpu': NO, 'nnz': prob.nnz(), 'setup_s': setup,
            'algo_bytes_per_iter_per_gpu': algo, 'achieved_GBs_per_gpu': algo / (ms * 1e-3) / 1e9,
            'roofline_frac': algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one rank per GPU (the driver's torchrun); COMAP_DIST_BACKEND=gloo with more ranks than
    # GPUs is a rehearsal mode only (ranks share devices; RCCL refuses duplicate GPUs)
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
    data = build_observation(F, T, obs_id=rank + 1, device=device)
    samp_ch = F * 4 * 1024 * T

    for _ in range(max(args.warmup, 1)):       # the first step also creates the plan
        level2 = reduce_step(data, device)
    obs = data._gpu_observation
    obs.profile(True)
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
    obs.profile(False)
    if world > 1:
        e = torch.tensor([elapsed], device='cuda', dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    check = check_against_oracle(data, level2, device) if (args.check and rank == 0) else None
    dstr = None
    if not args.no_destriper:
        dstr = destriper_leg(level2, data, args.destriper_iters, device)
        if world > 1:
            v = torch.tensor([dstr['cg_iters_per_s']], device='cuda', dtype=torch.float64)
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
            dstr['cg_iters_per_s_min_over_ranks'] = float(v.item())

    c5 = None
    if not args.no_destriper and args.c5_obs > 0:
        c5 = destriper_c5_leg(args.c5_obs, args.destriper_iters, device, world, rank)

    if rank == 0:
        value = world * samp_ch * args.steps / elapsed
        scan_sc = obs.scan_samples() * 4096
        stream = {k: prof[k] for k in obs.STREAMING}
        # bytes each pass must read: A all 1024 channels, B the median_filter channels with a
        # finite 1/rms, C those channels in the bands the median filter did not skip
        frac = obs.pass_fractions()
        pass_bytes = {k: ALGO_BYTES_PER_SAMPCH_PASS * scan_sc * frac[k] for k in obs.STREAMING}
        dom = max(stream, key=lambda k: stream[k][0])
        ms_avg = stream[dom][0] / max(stream[dom][1], 1)
        # passes B and C run as one launch per unit group (pipelined with the median)
        algo_bytes = pass_bytes[dom] * args.steps / max(stream[dom][1], 1)
        achieved = algo_bytes / (ms_avg * 1e-3) / 1e9
        design_bytes = sum(pass_bytes.values())
        traffic = None
        tpath = os.path.join(ROOT, 'profiles', 'traffic_latest.json')
        if os.path.exists(tpath):
            traffic = json.load(open(tpath)).get(dom)
        step_ms = elapsed / args.steps * 1e3
        line = {
            'metric': 'TOD samples x channels / s (L1 -> L2 reduction)',
            'value': value,
            'unit': 'samples*channels/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': step_ms,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32 in, f64 accumulate',
            'data': 'synthetic (SURVEY.md §8d spec, generated on device)',
            'config': {'workload': f'C2: {F}-feed x 4 x 1024 ch x {T} samples L1 observation per GPU '
                                   f'({samp_ch * 4 / 1e9:.1f} GB f32 resident in HBM), vane + atmosphere + '
                                   'L1AveragingGainCorrection', 'parallelism': f'observation-parallel x{world}'},
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'algo_bytes_per_launch': algo_bytes, 'avg_launch_ms': ms_avg},
            'l1_step_roofline': {'passes': len(obs.STREAMING), 'design_bytes': design_bytes,
                                 'achieved_GBs': design_bytes / (step_ms * 1e-3) / 1e9,
                                 'frac': design_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                 'pass_channel_fraction': frac,
                                 'survey_4pass_bytes': SURVEY_BYTES_PER_SAMPCH * scan_sc,
                                 'survey_4pass_equiv_frac':
                                     SURVEY_BYTES_PER_SAMPCH * scan_sc / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            'kernel_ms_per_step': {k: v[0] / args.steps for k, v in prof.items()},
            'host_stage_ms_per_step': {k: v / args.steps for k, v in host_ms.items()},
            'host_vane_search_ms': getattr(obs, 'last_vane_search_ms', None),
            'pass_GBs': {k: pass_bytes[k] / (stream[k][0] / args.steps * 1e-3) / 1e9
                         for k in obs.STREAMING if stream[k][1] > 0},
            'launches_per_step': {k: stream[k][1] / args.steps for k in obs.STREAMING},
        }
        if dstr is not None:
            line['destriper'] = dstr
        if c5 is not None:
            line['destriper_c5'] = c5
        if check is not None:
            line['check'] = check
        if not args.no_cpu_baseline and world == 1:
            line['cpu_baseline'] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
