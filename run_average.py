#!/usr/bin/env python3
"""TOML-driven L1 -> L2 reduction (mirror of the reference run_average.py:19-121).

    python run_average.py configuration.toml
    python -m torch.distributed.run --nproc-per-node 8 run_average.py configuration.toml

[Global] keys: level2_data, level2_figures, level1_filelist, log_file,
log_level, processes; one [StageName] section of dataclass kwargs per stage.
Each rank (one per GPU) takes its contiguous block of the file list and
reduces it with no communication (run_average.py:38-39).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def create_tod_processing(configuration, rank=0, size=1, device=0):
    from comapreduce_amd import Analysis
    from comapreduce_amd.pipeline.running import split_filelist
    g = configuration['Global']
    os.makedirs(g['level2_figures'], exist_ok=True)
    os.makedirs(g['level2_data'], exist_ok=True)
    filelist = np.loadtxt(g['level1_filelist'], dtype=str, ndmin=1)
    runner = Analysis.Runner()
    processes = {Analysis.CheckLevel1File: {'overwrite': True},
                 Analysis.AssignLevel1Data: {'overwrite': False, 'write': True}}
    for name in g['processes']:
        cls = getattr(Analysis, name, None)
        if cls is None:
            raise NotImplementedError(
                f"stage {name!r} is not provided by comapreduce_amd (outside the L1->L2 / noise-QA scope of "
                f"DESIGN.md; available: {', '.join(Analysis.STAGES)}); remove it from [Global] processes")
        kw = dict(configuration.get(name, {}))
        kw['figure_directory'] = g['level2_figures']
        if 'device' in getattr(cls, '__dataclass_fields__', {}):
            kw['device'] = device
        processes[cls] = kw
    runner.level2_data_dir = g['level2_data']
    runner.filelist = split_filelist(filelist, rank, size)
    runner.processes = processes
    return runner


def main(argv=None):
    import tomli
    argv = sys.argv[1:] if argv is None else argv
    with open(argv[0], 'rb') as f:
        configuration = tomli.load(f)
    from comapreduce_amd.pipeline.running import set_logging
    rank = int(os.environ.get('RANK', 0))
    size = int(os.environ.get('WORLD_SIZE', 1))
    device = int(os.environ.get('LOCAL_RANK', 0))
    set_logging(configuration['Global']['log_file'], configuration['Global'].get('log_level', 'INFO'))
    create_tod_processing(configuration, rank, size, device).run_tod()


if __name__ == '__main__':
    main()
