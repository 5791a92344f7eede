"""Level-2 statistics stages (drop-in for comancpipeline/Analysis/Statistics.py).

``Spikes`` (Statistics.py:31-105): spike mask of the Level-2 band-averaged
TOD -- per (feed, band) auto-rms of the non-zero samples, per scan a
medfilt(100) high-pass, |x| > 10 rms, each run dilated by fit_spikes' window.
The whole mask is one device call (``comap_spikes``, spikes_kernels.hip).
Its output ``spikes/spike_mask`` zeroes destriper weights (COMAPData.py:332-334).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from .. import _native as N
from ..gpu import _torch, to_device
from ..pipeline.datahandling import CALIBRATOR_LIST, COMAPLevel2, to_host
from ..pipeline.running import PipelineFunction


def spike_mask(tod, scan_edges, medfilt_window=100, step=100, threshold=10.0, device=0):
    """Device spike mask of a Level-2 TOD [F, B, T] (NumPy or CUDA tensor) -> CUDA bool [F, B, T]."""
    torch = _torch()
    dev = torch.device('cuda', device)
    t = to_device(tod, torch.float64, dev)
    F, B, T = t.shape
    edges = np.ascontiguousarray(np.asarray(to_host(scan_edges), dtype=np.int64).reshape(-1, 2))
    mask = torch.empty((F, B, T), dtype=torch.uint8, device=dev)
    c = N.ctx(device)
    N.bind_stream(c, dev)
    N.check(N.lib().comap_spikes(c, N.dptr(t), F * B, T, N.hptr(edges, ctypes.c_int64), edges.shape[0],
                                 int(medfilt_window), int(step), float(threshold), N.dptr(mask)), c, 'comap_spikes')
    return mask.bool()


@dataclass
class Spikes(PipelineFunction):
    name: str = 'Spikes'
    overwrite: bool = False
    STATE: bool = True
    MEDIAN_FILTER_STEP: int = 100
    SPIKE_THRESHOLD: float = 10
    device: int = 0
    device_outputs: bool = False
    data: dict = field(default_factory=lambda: {'spikes/spike_mask': np.empty(1)})

    def __post_init__(self):
        self.groups = list(np.unique([s.split('/')[0] for s in self.data.keys()]))

    @property
    def save_data(self):
        return self.data, {}

    def __call__(self, data, level2_data: COMAPLevel2 = None):
        level2_data = level2_data if level2_data is not None else self.level2
        if data.source_name not in CALIBRATOR_LIST:
            self.run_fit_spikes(data, level2_data)
        return self.STATE

    def run_fit_spikes(self, data, level2_data):
        m = spike_mask(level2_data['averaged_tod/tod'], level2_data.scan_edges, self.MEDIAN_FILTER_STEP, 100,
                       self.SPIKE_THRESHOLD, self.device)
        self.data['spikes/spike_mask'] = m if self.device_outputs else m.cpu().numpy()
