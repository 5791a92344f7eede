"""Dump the bench's C4 destriper problem (read_comap_data band 0 of the reduced C2
observation: pointing, tod, weights -- what bench.py's C4 leg solves) to an .npz, so the
reference's own destriper can be timed on exactly that problem in the build container
(tests/golden/make_golden.py --only-timing --c4-npz).  GPU box only.

    python scripts/dump_c4_problem.py gpurun_out/c4_problem.npz
"""
import sys

import numpy as np

sys.path.insert(0, '.')


def main(path):
    import bench
    from comapreduce_amd.mapmaking import comapdata as CD
    data, _ = bench.build_observation(19, 180_000, obs_id=1, device=0)
    level2 = bench.reduce_step(data, 0)
    store = bench.level2_store(level2, data, obsid=1)
    tod, w, pix = CD.read_comap_data(list(store), bench.c4_map_info(), iband=0, offset_length=50, store=store,
                                     device=0)[:3]
    np.savez_compressed(path, pointing=np.asarray(pix, np.int32), tod=np.asarray(tod, np.float64),
                        weights=np.asarray(w, np.float64))
    print(path, int(np.asarray(tod).size), 'samples')


if __name__ == '__main__':
    main(sys.argv[1])
