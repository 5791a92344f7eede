"""C3 (BASELINE configs[2]): one observation's (feed, scan) units sharded over
ranks with no collective (comapreduce_amd/pipeline/sharding.py).

CPU checks of the host side: the balanced contiguous unit partition, the
feed slices a rank holds, and -- on 2 gloo ranks -- that reducing each shard
(here with the CPU oracle, oracle/l1.py) and assembling the owned unit slices
gives bit-identical Level-2 arrays to the unsharded reduction.  The device
path's own 1-vs-N-shard identity is tests/test_gpu_l1.py::test_shards_bit_identical."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from comapreduce_amd import synthetic
from comapreduce_amd.pipeline import sharding
from comapreduce_amd.pipeline.datahandling import level1_from_dict

# 3 feeds (one numbered > 19) x 2 short scans: 6 units, so 2 ranks share a feed
F3 = dict(n_feeds=3, n_samples=16_000, obs_id=5, feed_numbers=(1, 2, 20), scan_len=6500, scan_gap=500, min_last=5000)


def _best_bound(w, world):
    """Brute-force optimum of the largest contiguous run (DP), small cases."""
    n = len(w)
    c = np.concatenate(([0], np.cumsum(w)))
    INF = float('inf')
    dp = [[INF] * (n + 1) for _ in range(world + 1)]
    dp[0][0] = 0
    for k in range(1, world + 1):
        for i in range(n + 1):
            for j in range(i + 1):
                dp[k][i] = min(dp[k][i], max(dp[k - 1][j], c[i] - c[j]))
    return dp[world][n]


def test_partition_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    for U, world in [(209, 8), (209, 1), (5, 8), (57, 3), (1, 2), (0, 4), (9, 3), (12, 4), (7, 2)]:
        w = rng.integers(100, 20000, U)
        parts = sharding.partition_units(w, world)
        assert len(parts) == world
        assert parts[0][0] == 0 and parts[-1][1] == U
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        if U:
            loads = [int(w[lo:hi].sum()) for lo, hi in parts]
            assert max(loads) <= int(np.ceil(w.sum() / world)) + int(w.max())
            if U <= 12:
                assert max(loads) == _best_bound(w, world)   # optimal contiguous split


def test_c2_shards_cover_units_once():
    cfg = synthetic.SyntheticConfig(n_feeds=19, n_samples=180_000, obs_id=1)
    meta, attrs, *_ = synthetic.level1_metadata(cfg)
    edges = synthetic.scan_edges_from_status(meta['hk/antenna0/deTracker/lissajous_status'])
    units = sharding.unit_table(edges, 19)
    for world in (1, 2, 4, 8):
        shards = [sharding.shard_for(edges, 19, r, world) for r in range(world)]
        got = np.concatenate([s.units for s in shards])
        assert np.array_equal(got, units)
        for s in shards:
            assert np.all((s.units[:, 0] >= s.f_lo) & (s.units[:, 0] < s.f_hi))
        loads = [s.units[:, 3].sum() for s in shards]
        if world == 8:
            # (feed, scan) granularity: within one unit of perfect balance (7.7x)
            assert max(loads) - units[:, 3].sum() / world <= units[:, 3].max()


def test_slice_feeds_and_filter():
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**F3))
    data = level1_from_dict(gen)
    sh, part = sharding.shard_level1(data, 1, 2)
    assert part['spectrometer/tod'].shape[0] == sh.n_feeds
    assert np.array_equal(part['spectrometer/feeds'], gen['data']['spectrometer/feeds'][sh.f_lo:sh.f_hi])
    assert np.array_equal(part.scan_edges, data.scan_edges)
    assert np.array_equal(part.unit_filter, sh.local_filter())
    assert np.array_equal(part['spectrometer/tod'], gen['data']['spectrometer/tod'][sh.f_lo:sh.f_hi])


def _oracle_shard(data_dict, sh):
    import oracle.l1 as ol1
    sub = {k: (v[sh.f_lo:sh.f_hi] if k in sharding.FEED_AXIS_PATHS else v) for k, v in data_dict.items()}
    return ol1.reduce_level1(sub)


def _rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**F3))
    sh, _ = sharding.shard_level1(level1_from_dict(gen), rank, world)
    out = _oracle_shard(gen['data'], sh)          # no collective during the reduction
    keep = ('averaged_tod/tod', 'averaged_tod/tod_original', 'averaged_tod/weights', 'atmosphere/fit_values',
            'vane/system_temperature', 'vane/system_gain')
    parts = [None] * world
    dist.gather_object(({k: out[k] for k in keep}, sh), parts if rank == 0 else None, dst=0)   # once, at the end
    if rank == 0:
        q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_bit_identical_to_unsharded():
    import oracle.l1 as ol1
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29400 + os.getpid() % 300
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    gen = synthetic.generate_level1(synthetic.SyntheticConfig(**F3))
    full = ol1.reduce_level1(gen['data'])
    shards = [s for _, s in parts]
    assert shards[0].f_hi > shards[1].f_lo, 'the F=3 split should share a feed between the ranks'
    S = len(full['averaged_tod/scan_edges'])
    got = sharding.assemble(shards, [o for o, _ in parts], 3, S, F3['n_samples'])
    for k, v in got.items():
        assert np.array_equal(v, full[k], equal_nan=True), k
    # feed 20 (> 19) is skipped by the reducer (Level1Averaging.py:817-818)
    assert not got['averaged_tod/tod'][2].any()
