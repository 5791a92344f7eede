"""The multi-rank destriper model (mapmaking/rankplan.py): it reproduces the
single-GPU measurements it is fitted to, and chooses to gather a single observation
(C4) to one rank and to shard the C5 field."""
import pytest

from comapreduce_amd.mapmaking import rankplan


@pytest.mark.parametrize('n,nb,us', [(1.76e6, 1, 21.8), (27.36e6, 1, 124.0), (1.76e6, 4, 29.9), (27.36e6, 4, 275.0)])
def test_single_rank_iteration_matches_measurement(n, nb, us):
    # bench.py r05c / ds_tiling_probe: C4 45.8k it/s (1 band) and 134k band-it/s (4 bands),
    # C5 (8 obs, tiled layout) 0.124 / 0.275 ms per iteration
    assert rankplan.CostModel().iter_us(n, nb, 1, 0) == pytest.approx(us, rel=0.06)


def test_c4_is_gathered_c5_is_sharded():
    for world in (2, 4, 8):
        for nb in (1, 4):
            assert rankplan.plan(1.76e6, nb, world)['mode'] == 'gather'
            assert rankplan.plan(27.36e6 * world, nb, world)['mode'] == 'shard'
    assert rankplan.plan(1.76e6, 4, 1)['mode'] == 'shard'      # one rank: nothing to gather


def test_sharded_iteration_time_shape():
    m = rankplan.CostModel()
    t = rankplan.plan(27.36e6 * 8, 4, 8)['iter_us_by_ranks']
    assert t[8] < t[4] < t[2] < t[1]                               # a big field scales
    c4 = rankplan.plan(1.76e6, 4, 8)['iter_us_by_ranks']
    assert c4[8] > c4[1]                                           # one observation does not
    assert m.alpha_us(1) == 0.0 and m.alpha_us(8) > m.alpha_us(2)


def test_measured_alpha_beta_replace_the_assumptions(tmp_path):
    """scripts/rankplan_calibrate.py turns bench.py's N > 1 allreduce_probe fields into
    rankplan_measured.json; CostModel then uses the measured alpha / beta for those rank
    counts and keeps the assumptions for the others."""
    import json
    import subprocess
    import sys
    rec = {'parsed': {'destriper_c5_field': {'allreduce_probe': {
        'n_ranks': 4, 'points': [{'bytes': 32, 'us': 31.0}, {'bytes': 1 << 20, 'us': 52.0}],
        'alpha_us': 31.0, 'beta_GBs': 50.0}, 'comm_rank0': {'allreduce_ms_per_iter': 0.12}}}}
    src = tmp_path / 'SCALE_test.json'
    src.write_text(json.dumps([rec]))
    out = rankplan.MEASURED
    saved = open(out).read() if __import__('os').path.exists(out) else None
    try:
        subprocess.run([sys.executable, 'scripts/rankplan_calibrate.py', str(src)], check=True, capture_output=True,
                       cwd=__import__('os').path.dirname(__import__('os').path.dirname(__file__)))
        m = rankplan.CostModel()
        assert m.alpha_us(4) == 31.0 and m.beta(4) == 50.0 and m.measured(4)
        assert not m.measured(8) and m.alpha_us(8) == m.alpha0_us + 14 * m.alpha_hop_us
        t = m.iter_us(1e6, 1, 4, 1e6)
        assert t == pytest.approx(m.a_us + m.b_us_per_msample[1] / 4 + 3 * 31.0 + 1e6 / 50e3)
    finally:
        if saved is None:
            __import__('os').remove(out)
        else:
            open(out, 'w').write(saved)


@pytest.fixture(scope='module')
def field_work():
    """Per-series work of bench.py's configs[4] field (64 obs x 19 feeds), from the
    pointing alone (CPU)."""
    import torch
    from comapreduce_amd import synthetic
    torch.set_num_threads(min(8, torch.get_num_threads()))
    return synthetic.field_series_work(64, device='cpu')


def test_field_work_counts_the_operator_entries(field_work):
    """The (offset, pixel run) pairs of the field's pointing are its operator entries up to
    the few offsets that revisit a pixel: 86,704,202 entries on one GPU (bench r05,
    destriper_c5_field nnz)."""
    ent, no = field_work
    assert ent.size == 64 * 19 and no == 3600
    assert 0 <= ent.sum() - 86_704_202 < 1000


def test_field_split_balances_work(field_work, monkeypatch):
    """bench.field_split deals the field's (obs, feed) series to 2 / 4 / 8 ranks in
    contiguous ranges balanced on CG work (entries + FIELD_KAPPA x offsets): the slowest
    rank's modelled work is within 2 % of the mean, and its entries within 15 %; equal
    observation counts (run_destriper.py:131-138, rounds 2-5) gave rank 0 1.32 / 1.63 /
    1.86 x the mean entries.  The ranges cover every series once, in order."""
    import numpy as np
    import bench
    ent, no = field_work
    w = ent + bench.FIELD_KAPPA * no
    for world, obs_imb in ((2, 1.32), (4, 1.63), (8, 1.86)):
        monkeypatch.setenv('COMAP_FIELD_SPLIT', 'obs')
        eq, _, _ = bench.field_split(64, world)
        assert rankplan.imbalance(ent, eq) == pytest.approx(obs_imb, abs=0.01)
        monkeypatch.delenv('COMAP_FIELD_SPLIT')
        r, _, _ = bench.field_split(64, world)
        assert r[0][0] == 0 and r[-1][1] == ent.size and all(a[1] == b[0] for a, b in zip(r, r[1:]))
        assert rankplan.imbalance(w, r) < 1.02, world
        assert rankplan.imbalance(ent, r) < 1.15, world
        assert np.all(np.diff([a for a, _ in r]) > 0)
