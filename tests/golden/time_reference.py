#!/usr/bin/env python3
"""Time the REFERENCE (COMAPreduce v0.9.1) Level-1 -> Level-2 reduction on CPU cores,
the CPU baseline SURVEY.md §8(d) / BASELINE.md §3 prescribe, in the build container.

Test infrastructure like make_golden.py (whose reference build and import stand-ins it
reuses): it runs only where /root/reference exists and never travels to the GPU box;
the numbers land in tests/golden/golden_meta.json ('reference_cpu_baseline'), which
bench.py reports under cpu_baseline.reference.

Cases, all on C1-shaped synthetic observations (1 feed x 4 x 1024 x 30,000, obs ids
1..8, MeasureSystemTemperature -> AtmosphereRemoval -> Level1AveragingGainCorrection):
  * 1 process, matplotlib's savefig stubbed to a no-op (the figures are still drawn);
  * 8 processes at once, one observation each -- run_average.py:38-39's file split
    over 8 MPI ranks on the container's 8 cores -- as shipped (PNG files written);
  * the same 8 processes with savefig stubbed.
Each worker is a fresh interpreter with one BLAS / OpenMP thread (one core per rank,
as the reference's MPI layout assumes).

Usage:  python tests/golden/time_reference.py [--procs 8]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

SAMPCH = 1 * 4 * 1024 * 30_000


def worker(obs_id, stub_savefig, figdir):
    """One rank: the reference's three stages on observation obs_id; prints the seconds."""
    import make_golden as mg
    mg.install_stubs()
    import numpy as np
    import matplotlib
    matplotlib.use('Agg')
    if stub_savefig:
        from matplotlib import figure, pyplot
        pyplot.savefig = lambda *a, **k: None
        figure.Figure.savefig = lambda *a, **k: None
    from comancpipeline.Analysis.DataHandling import COMAPLevel1, COMAPLevel2
    from comancpipeline.Analysis.VaneCalibration import MeasureSystemTemperature
    from comancpipeline.Analysis.Level1Averaging import AtmosphereRemoval, Level1AveragingGainCorrection
    from comapreduce_amd import synthetic
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(n_feeds=1, n_samples=30_000, obs_id=obs_id))
    data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
    for k, v in gen['data'].items():
        data[k] = mg.CopyOnSlice(v) if k == 'spectrometer/tod' else v
    for k, v in gen['attrs']['comap'].items():
        data.set_attrs('comap', k, v)
    level2 = COMAPLevel2(filename=os.path.join(figdir, 'does_not_exist.hd5'))
    t0 = time.perf_counter()
    for cls in (MeasureSystemTemperature, AtmosphereRemoval, Level1AveragingGainCorrection):
        stage = cls(level2=level2, figure_directory=figdir)
        assert stage(data, level2), cls.__name__
        level2.update(stage)
    dt = time.perf_counter() - t0
    assert np.isfinite(np.asarray(level2['averaged_tod/tod'])).any()
    print(json.dumps({'obs_id': obs_id, 'seconds': dt}), flush=True)


def run_group(n, stub):
    """n workers at once (observations 1..n); returns (wall seconds, per-worker seconds)."""
    env = dict(os.environ, OMP_NUM_THREADS='1', OPENBLAS_NUM_THREADS='1', MKL_NUM_THREADS='1',
               PYTHONHASHSEED='0')
    with tempfile.TemporaryDirectory() as figdir:
        t0 = time.perf_counter()
        procs = [subprocess.Popen([sys.executable, __file__, '--worker', str(i + 1), '--stub', str(int(stub)),
                                   '--figdir', os.path.join(figdir, f'r{i}')], env=env, stdout=subprocess.PIPE,
                                  cwd=REPO) for i in range(n)]
        outs = [p.communicate()[0] for p in procs]
        wall = time.perf_counter() - t0
        if any(p.returncode for p in procs):
            raise RuntimeError('a reference worker failed')
    per = [json.loads(o.decode().strip().splitlines()[-1])['seconds'] for o in outs]
    return wall, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--worker', type=int, default=0)
    ap.add_argument('--stub', type=int, default=0)
    ap.add_argument('--figdir', default='')
    ap.add_argument('--procs', type=int, default=8)
    a = ap.parse_args()
    if a.worker:
        os.makedirs(a.figdir, exist_ok=True)
        worker(a.worker, bool(a.stub), a.figdir)
        return
    import make_golden as mg
    if not os.path.isdir(os.path.join(mg.SCRATCH, 'comancpipeline')):
        mg.build_reference_helpers()
    res = {'config': 'C1 observations (1 feed x 4 x 1024 x 30000) through the reference v0.9.1 '
                     'MeasureSystemTemperature + AtmosphereRemoval + Level1AveragingGainCorrection',
           'samples_channels_per_obs': SAMPCH, 'host': f'build container, {os.cpu_count()} cores',
           'threads_per_process': 1}
    wall1, per1 = run_group(1, True)
    res['one_process_savefig_stubbed'] = {'processes': 1, 'seconds': per1[0], 'wall_s': wall1,
                                          'samples_channels_per_s': SAMPCH / per1[0]}
    for stub in (False, True):
        wall, per = run_group(a.procs, stub)
        key = f'{a.procs}_processes_' + ('savefig_stubbed' if stub else 'png_written')
        res[key] = {'processes': a.procs, 'wall_s': wall, 'per_process_s': per,
                    'samples_channels_per_s': a.procs * SAMPCH / wall}
        print(key, json.dumps(res[key]), flush=True)
    path = os.path.join(HERE, 'golden_meta.json')
    meta = json.load(open(path))
    meta['reference_cpu_baseline'] = res
    with open(path, 'w') as f:
        json.dump(meta, f, indent=1, default=str)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
