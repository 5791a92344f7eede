"""How many ranks a destriper problem should run on.

Across ranks every CG iteration all-reduces the compacted map numerator and two
block-partial vectors (Destriper.py:183-204 sums the map over MPI every matvec), so
the per-iteration cost on n ranks is

    t_iter(n) = a + b_NB * N / n + 3 * alpha(n) + map_bytes * 2 (n - 1) / n / beta

(a: the 4 launches' latency floor; b_NB: the streaming part per sample for NB bands;
N: the problem's total samples; alpha(n): one small RCCL all-reduce; beta: the ring's
bus bandwidth), and the set-up costs s0_NB + s1_NB * N / n.  Gathering the inputs to
one rank instead costs bytes / (gather bandwidth) once, then the single-rank times.
plan() compares the two for the expected iteration count and returns the faster.

The a / b / s constants are fitted to this build's single-GPU measurements (bench.py
C4 and C5 legs, count-form operator, tiled pixel layout, round 5: 1 band 21.8 / 124 us per
iteration at 1.76 M / 27.36 M samples, 4 bands 29.9 / 275 us; set-up 1 band 2.58 ms and 4
bands 3.21 / 22.0 ms at 27.36 M / 218.9 M samples (profiles/r05/r05x_bench.log) -- the
64-observation field, whose iteration, 1.47 ms, the per-sample model overestimates: its
pointing holds fewer entries per sample).
alpha and beta cannot be measured on the one-GPU box (it cannot run two RCCL ranks; a
one-rank all-reduce costs 10 us of host enqueue, profiles/r03/r03n_rccl_one_rank.log).
Until a multi-GPU run has measured them, alpha(n) = 10 us + 2 (n - 1) x 1.5 us per ring
hop and beta = 100 GB/s are assumptions for 8 MI355X on xGMI (7 links x ~153 GB/s per
GPU).  bench.py measures both on every N > 1 run (``allreduce_probe``: the all-reduce
time at the CG's message sizes, fitted to alpha + bytes / beta, and ``comm_rank0``: the
all-reduce time per CG iteration inside the solve); scripts/rankplan_calibrate.py writes
them from the driver's SCALE records into rankplan_measured.json beside this file, and
CostModel() then uses the measured alpha(n) / beta(n) for the rank counts it covers.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

MEASURED = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'rankplan_measured.json')


def _load_measured(path=MEASURED):
    """{'alpha_us': {n: us}, 'beta_GBs': {n: GB/s}} from a calibration file, or empty."""
    try:
        with open(path) as f:
            m = json.load(f)
    except (OSError, ValueError):
        return {}, {}
    a = {int(k): float(v) for k, v in m.get('alpha_us', {}).items()}
    b = {int(k): float(v) for k, v in m.get('beta_GBs', {}).items() if v}
    return a, b


@dataclass
class CostModel:
    a_us: float = 14.0                                   # per-iteration latency floor
    b_us_per_msample: dict = field(default_factory=lambda: {1: 3.99, 2: 6.5, 4: 9.57})
    setup0_ms: dict = field(default_factory=lambda: {1: 0.24, 2: 0.38, 4: 0.53})
    setup1_ms_per_msample: dict = field(default_factory=lambda: {1: 0.086, 2: 0.092, 4: 0.098})
    alpha0_us: float = 10.0                              # one all-reduce: enqueue / protocol floor
    alpha_hop_us: float = 1.5                            # per ring step (2 (n - 1) steps)
    beta_gbs: float = 100.0                              # all-reduce bus bandwidth
    gather_gbs: float = 150.0                            # inputs gathered to one rank (7 links in parallel)
    # measured per rank count (rankplan_measured.json, scripts/rankplan_calibrate.py); None:
    # load the file beside this module when it exists
    alpha_measured: dict = None
    beta_measured: dict = None

    def __post_init__(self):
        if self.alpha_measured is None or self.beta_measured is None:
            a, b = _load_measured()
            self.alpha_measured = a if self.alpha_measured is None else self.alpha_measured
            self.beta_measured = b if self.beta_measured is None else self.beta_measured

    def alpha_us(self, n):
        if n <= 1:
            return 0.0
        if n in self.alpha_measured:
            return self.alpha_measured[n]
        return self.alpha0_us + 2 * (n - 1) * self.alpha_hop_us

    def beta(self, n):
        return self.beta_measured.get(n, self.beta_gbs)

    def measured(self, n):
        return n in self.alpha_measured

    def iter_us(self, n_samples, nb, n, map_bytes):
        nb = 4 if nb == 3 else nb
        t = self.a_us + self.b_us_per_msample[nb] * n_samples / 1e6 / n
        if n > 1:
            # alpha + bytes / beta per all-reduce (the probe's fit already holds the ring's
            # 2 (n - 1) / n factor in a MEASURED beta; the assumed bus bandwidth does not)
            ring = 1.0 if n in self.beta_measured else 2 * (n - 1) / n
            t += 3 * self.alpha_us(n) + map_bytes * ring / (self.beta(n) * 1e3)
        return t

    def setup_ms(self, n_samples, nb, n):
        nb = 4 if nb == 3 else nb
        return self.setup0_ms[nb] + self.setup1_ms_per_msample[nb] * n_samples / 1e6 / n


def input_bytes(n_samples, nb, offset_length=50):
    """Bytes of one problem's inputs: int32 pixel + f64 tod and weight per band and
    sample, the uint8 keep mask per band and offset."""
    return n_samples * (4 + 16 * nb) + nb * n_samples // max(offset_length, 1)


def plan(n_samples, nb, world, n_hit_pixels=31_000, iters=25, model=None):
    """Shard (every rank solves its own samples, RCCL all-reduces per iteration) or
    gather (the inputs go to rank 0, which solves alone).  Returns a dict with the
    choice and both modelled times (ms), plus the per-iteration model for 1/2/4/8 ranks."""
    m = model or CostModel()
    nbb = 4 if nb == 3 else nb
    map_bytes = 8 * nbb * n_hit_pixels
    t_shard = m.setup_ms(n_samples, nb, world) + iters * m.iter_us(n_samples, nb, world, map_bytes) / 1e3
    t_gather = (input_bytes(n_samples, nbb) * (world - 1) / world / (m.gather_gbs * 1e6) +
                m.setup_ms(n_samples, nb, 1) + iters * m.iter_us(n_samples, nb, 1, map_bytes) / 1e3)
    per_iter = {n: m.iter_us(n_samples, nb, n, map_bytes) for n in (1, 2, 4, 8)}
    mode = 'gather' if world > 1 and t_gather < t_shard else 'shard'
    return {'mode': mode, 'shard_ms': t_shard, 'gather_ms': t_gather, 'iters': iters,
            'iter_us_by_ranks': per_iter}


# ---------------------------------------------------------------- work-balanced splits
# A sharded CG iteration waits for its slowest rank, and a rank's operator time follows its
# sparse operator's entries -- the distinct (offset, pixel) pairs of its samples -- not its
# sample count: a slow scan crosses fewer pixels per offset.  The reference splits the file
# list into equal counts (run_destriper.py:131-138); the map it solves is the same whichever
# rank holds a file, so the files can be dealt by work instead.


def offset_pixel_runs(pix, offset_length, groups=1):
    """Per group (``pix`` holds ``groups`` equal contiguous blocks of whole offsets, e.g. one
    per observation): the number of (offset, pixel run) pairs -- 1 + the pixel changes
    inside each offset.  That is the operator's entry count when no offset revisits a
    pixel after leaving it (a scan track moves on), and an upper bound otherwise.  NumPy
    or torch input (any device); returns int64 NumPy [groups]."""
    L = int(offset_length)
    if type(pix).__module__.startswith('torch'):                    # a torch tensor (any device)
        p = pix.reshape(int(groups), -1, L)
        runs = (p[:, :, 1:] != p[:, :, :-1]).sum(dim=(1, 2)) + p.shape[1]
        return runs.cpu().numpy().astype(np.int64)
    p = np.asarray(pix).reshape(int(groups), -1, L)
    return ((p[:, :, 1:] != p[:, :, :-1]).sum(axis=(1, 2)) + p.shape[1]).astype(np.int64)


def balanced_ranges(weights, world):
    """Contiguous [(lo, hi)] index ranges, one per rank, minimising the largest rank's total
    weight (the optimal contiguous partition of pipeline/sharding.partition_units); the
    concatenation in rank order keeps the caller's order."""
    from ..pipeline.sharding import partition_units
    return partition_units(np.asarray(weights, dtype=np.int64), int(world))


def imbalance(weights, ranges):
    """max / mean of the ranks' total weights."""
    w = np.asarray(weights, dtype=np.float64)
    tot = np.array([w[a:b].sum() for a, b in ranges])
    return float(tot.max() / max(tot.mean(), 1e-300))
