"""run_average.py's TOML process list (reference run_average.py:43-48): stage
names resolve in comapreduce_amd.Analysis; a stage outside this build's scope
fails with a clear error before any file is touched."""
import os

import pytest

import run_average


def _cfg(tmp_path, processes):
    fl = tmp_path / 'files.txt'
    fl.write_text('obs1.hd5\nobs2.hd5\n')
    return {'Global': {'level2_data': str(tmp_path / 'l2'), 'level2_figures': str(tmp_path / 'fig'),
                       'level1_filelist': str(fl), 'log_file': str(tmp_path / 'log.log'),
                       'processes': processes},
            'Level1AveragingGainCorrection': {'overwrite': True, 'gain_subtraction_name': 'gain_subtraction_fit'}}


def test_shipped_stage_list_resolves(tmp_path):
    from comapreduce_amd import Analysis as A
    procs = ['MeasureSystemTemperature', 'AtmosphereRemoval', 'Level1AveragingGainCorrection',
             'Level2FitPowerSpectrum', 'Spikes', 'NoiseStatistics']
    runner = run_average.create_tod_processing(_cfg(tmp_path, procs), rank=1, size=2, device=0)
    names = [c.__name__ for c in runner.processes]
    assert names[:2] == ['CheckLevel1File', 'AssignLevel1Data'] and names[2:] == procs
    assert runner.processes[A.Level1AveragingGainCorrection]['gain_subtraction_name'] == 'gain_subtraction_fit'
    assert list(runner.filelist) == ['obs2.hd5']          # rank 1 of 2 takes its block


def test_out_of_scope_stage_is_a_clear_error(tmp_path):
    with pytest.raises(NotImplementedError, match='SkyDip'):
        run_average.create_tod_processing(_cfg(tmp_path, ['MeasureSystemTemperature', 'SkyDip']))
