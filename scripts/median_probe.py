"""Median kernels alone, for kernel traces and PMC passes: the chain's data-prep shape
(912 reflect-padded series of ~15 k samples, w = 400) and a C2-like shape (w = 6000),
each filtered `reps` times through comap_medfilt_batch_f64; prints wall ms per call.
    python scripts/median_probe.py [reps]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from comapreduce_amd.tools.medfilt import medfilt_batch  # noqa: E402


def series(n, length, seed):
    g = np.random.default_rng(seed)
    out = []
    for i in range(n):
        m = length + int(g.integers(-600, 600))
        out.append(np.cumsum(g.normal(0, 1e-3, m)) + g.normal(0, 1e-2, m) + 1.0)
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    res = {}
    for name, n, length, w in (('prep_w400', 912, 15_000, 400), ('c2_w6000', 304, 14_500, 6000)):
        s = series(n, length, 1)
        medfilt_batch(s, w, reflect=True)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = medfilt_batch(s, w, reflect=True)
            t.append((time.perf_counter() - t0) * 1e3)
        digest = hashlib.sha1(b''.join(o.tobytes() for o in out)).hexdigest()[:16]
        res[name] = {'series': n, 'samples': int(sum(x.size for x in s)), 'w': w, 'wall_ms': sorted(t)[len(t) // 2],
                     'sha1': digest}
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
