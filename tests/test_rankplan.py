"""The multi-rank destriper model (mapmaking/rankplan.py): it reproduces the
single-GPU measurements it is fitted to, and chooses to gather a single observation
(C4) to one rank and to shard the C5 field."""
import pytest

from comapreduce_amd.mapmaking import rankplan


@pytest.mark.parametrize('n,nb,us', [(1.76e6, 1, 22.0), (27.36e6, 1, 152.0), (1.76e6, 4, 34.0), (27.36e6, 4, 339.0)])
def test_single_rank_iteration_matches_measurement(n, nb, us):
    # bench.py r03d: C4 45.4k / 29.5k it/s (1 / 4 bands), C5 0.152 / 0.339 ms per iteration
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
