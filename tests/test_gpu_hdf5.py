"""The reference's file-driven path on the GPU: Runner.run_tod over a real HDF5
Level-1 file (Running.py:120-153) -- the cube stays a lazy dataset and is staged
from the file into pinned buffers on its way to HBM (gpu.upload) -- writing the
Level-2 HDF5 file after every stage, which is read back and compared with the
reference golden of the same C1 observation (tests/golden/golden_l1_c1.npz)."""
import json
import os

import numpy as np
import pytest

from comapreduce_amd import synthetic
from comapreduce_amd.pipeline import h5file as H
from comapreduce_amd.pipeline.datahandling import COMAPLevel2, HDF5Data

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not H.available(), reason='libcomap_h5.so not built')]
RTOL = 1e-5


def relmax(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), 'NaN pattern differs'
    return np.max(np.abs(a[fin] - b[fin])) / max(np.max(np.abs(b[fin])), 1e-300)


def test_runner_hdf5_level1_to_level2(golden_dir, tmp_path):
    from comapreduce_amd import Analysis as A
    from comapreduce_amd.pipeline.running import Runner
    meta = json.load(open(os.path.join(golden_dir, 'golden_meta.json')))
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**meta['l1_c1_config']))
    l1 = str(tmp_path / 'comap-0000001-2021-01-01-000000.hd5')
    w = HDF5Data(name='writer')
    for k, v in gen['data'].items():
        w[k] = v
    for p, a in gen['attrs'].items():
        for k, v in a.items():
            w.set_attrs(p, k, v)
    w.write_data_file(l1)
    del w

    runner = Runner()
    runner.filelist = [l1]
    runner.level2_data_dir = str(tmp_path)
    runner.processes = {A.MeasureSystemTemperature: {}, A.AtmosphereRemoval: {},
                        A.Level1AveragingGainCorrection: {}}
    runner.run_tod()
    out = str(tmp_path / ('Level2_' + os.path.basename(l1)))
    assert os.path.exists(out)
    with H.H5File(out) as f:                    # a real HDF5 file
        names = dict(f.visit())
    for k in ('vane/system_temperature', 'atmosphere/fit_values', 'averaged_tod/tod', 'averaged_tod/weights'):
        assert names.get(k) == 'dataset', k

    l2 = COMAPLevel2(filename=out)
    g = np.load(os.path.join(golden_dir, 'golden_l1_c1.npz'))
    assert np.array_equal(l2['vane/system_temperature'], g['vane__system_temperature'])
    assert np.array_equal(l2['vane/system_gain'], g['vane__system_gain'])
    assert relmax(l2['atmosphere/fit_values'], g['atmosphere__fit_values']) < RTOL
    assert np.array_equal(l2['averaged_tod/scan_edges'], g['averaged_tod__scan_edges'])
    for k in ('tod', 'tod_original', 'weights'):
        assert relmax(l2[f'averaged_tod/{k}'], g[f'averaged_tod__{k}']) < RTOL, k
