"""Stage protocol and runner (reference comancpipeline/Analysis/Running.py:30-180).

``PipelineFunction`` keeps the reference's plugin contract: a dataclass with
``name``, ``groups`` (Level-2 top-level groups it produces), ``overwrite``,
``STATE``, ``write``, ``figure_directory``, ``level2``; ``__call__(data,
level2) -> bool``; ``save_data -> (datasets, attrs)``; ``pre_init``;
``bad_data``.  ``Runner.run_tod`` loads each Level-1 file, skips stages whose
groups already exist in the Level-2 file (per-stage resume), runs the rest,
updates and rewrites the Level-2 file after every stage and stops the file
when a stage returns False.

Parallelism is one process per GPU: each rank takes its contiguous block of
the file list (``np.sort(np.mod(arange, size)) == rank``, run_average.py:38-39)
and never communicates during the reduction.  The reference's
``time.sleep(rank*15)`` staggering is not reproduced.
"""
from __future__ import annotations

import logging
import os
import socket
import sys
import traceback
from dataclasses import dataclass, field
from datetime import datetime
from os import path

import numpy as np

from .datahandling import COMAPLevel1, COMAPLevel2, HDF5Data

_STARTED = datetime.now().strftime('%Y-%m-%d-%H-%M-%S')


def dist_rank_size():
    """(rank, size) from torch.distributed when initialised, else the launcher env."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except ImportError:  # pragma: no cover
        pass
    return int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1))


def set_logging(logfilename: str, loglevel: str = 'INFO'):
    """One log file per rank: <dir>/<base>_<time>_<host>_PID<pid>_rank<NN>.log."""
    rank, _ = dist_rank_size()
    d = os.path.dirname(logfilename) or '.'
    base = os.path.basename(logfilename).split('.')[0]
    os.makedirs(d, exist_ok=True)
    logging.basicConfig(level=getattr(logging, loglevel),
                        format='%(asctime)s %(name)-12s %(levelname)-8s %(message)s', datefmt='%m-%d %H:%M',
                        filename=f'{d}/{base}_{_STARTED}_{socket.gethostname()}_PID{os.getpid()}_rank{rank:02d}.log',
                        filemode='w')

    def hook(etype, value, tb):
        frame = traceback.extract_tb(tb)[-1] if tb else None
        logging.info(f'{etype.__name__}: {value}')
        if frame:
            logging.info(f'Error on line {frame.lineno} in {frame.filename}')
        sys.__excepthook__(etype, value, tb)
    sys.excepthook = hook


@dataclass
class PipelineFunction:
    """Minimum interface of a pipeline stage."""
    name: str = 'PipelineFunction'
    STATE: bool = True
    level2: COMAPLevel2 = None
    write: bool = True
    figure_directory: str = 'figures'
    overwrite: bool = False
    groups: list = field(default_factory=list)

    @property
    def save_data(self):
        return {}, {}

    def bad_data(self):
        return False

    def pre_init(self, data: HDF5Data):
        pass

    def __call__(self, data: HDF5Data, level2_data: COMAPLevel2 = None) -> bool:
        return self.STATE


class Runner:
    """Runs a dict {stage class: kwargs} over a list of Level-1 files."""

    def __init__(self):
        self._filelist = []
        self._processes = {}
        self.level2_data = None
        self.level2_data_dir = '.'
        self.level2_prefix = 'Level2_'
        self.level1_loader = None     # optional callable(filename) -> COMAPLevel1

    @property
    def filelist(self):
        return self._filelist

    @filelist.setter
    def filelist(self, v):
        self._filelist = list(v)

    @property
    def processes(self):
        return self._processes

    @processes.setter
    def processes(self, v):
        self._processes = v

    def is_level2_file(self, filename: str) -> bool:
        return self.level2_prefix in filename

    def data_path(self, filename: str, level2_prefix: str) -> str:
        return f'{self.level2_data_dir}/{level2_prefix}{path.basename(filename)}'

    def load(self, filename):
        if self.level1_loader is not None:
            return self.level1_loader(filename)
        if self.is_level2_file(filename):
            data = COMAPLevel2(filename=filename, overwrite=False, large_datasets=['spectrometer/tod'])
            self.level2_prefix = 'temp_'
        else:
            data = COMAPLevel1(overwrite=False, large_datasets=['spectrometer/tod'])
            data.read_data_file(filename)
        return data

    def run_tod(self):
        for filename in self._filelist:
            logging.info(f'PROCESSING {path.basename(filename)}')
            data = self.load(filename)
            self.level2_data = COMAPLevel2(filename=self.data_path(filename, self.level2_prefix))
            stages = [cls(level2=self.level2_data, **kw) for cls, kw in self.processes.items()]
            for stage in stages:
                logging.info(f'INITIALISING {stage.name}')
                stage.pre_init(data)
                if (not self.level2_data.contains(stage)) or stage.overwrite or stage.bad_data():
                    logging.info(f'RUNNING {stage.name}')
                    if not stage(data, self.level2_data):
                        logging.info(f'{stage.name} has stopped processing file')
                        break
                    self.level2_data.update(stage)
                    if stage.write:
                        self.level2_data.write_data_file(
                            f'{self.level2_data_dir}/Level2_{path.basename(filename)}')


def split_filelist(filelist, rank: int, size: int):
    """Contiguous block per rank (run_average.py:38-39)."""
    filelist = np.asarray(filelist, dtype=str).reshape(-1)
    idx = np.sort(np.mod(np.arange(filelist.size), size))
    return filelist[np.where(idx == rank)[0]]
