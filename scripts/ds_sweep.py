"""Launch-shape sweep of the destriper CG kernels at C5 (one process): the same
synthetic problem (bench.destriper_c5_leg's inputs) solved for a fixed number of
iterations under each COMAP_DS_* setting (read when a problem is created); prints
one JSON line per (bands, setting) with ms per iteration and the iterate's checksum
(so a variant that changes the answer beyond rounding shows).
    python scripts/ds_sweep.py [n_obs] [iters] [bands ...] [set=layout|heavy]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SETS = {}
SETS['layout'] = [
    {},
    {'COMAP_DS_OKEY': 'first'},                  # offsets ordered by their first pixel (rounds 2-5)
    {'COMAP_DS_TILE': '0'},                      # row-major internal pixel order
    {'COMAP_DS_TILE': '16'},
    {'COMAP_DS_PB': '1024'},
    {'COMAP_DS_SELL': '0'},
]
SETS['heavy'] = [{'COMAP_DS_HEAVY': v} for v in ('0', '256', '1024', '4096')]   # walk: heavy rows first
SETS['cg'] = [{}, {'COMAP_DS_BL': '32'}, {'COMAP_DS_BL': '64'}, {'COMAP_DS_BL': '8'}, {'COMAP_DS_BU': '8'},
             {'COMAP_DS_PB': '4096'}, {'COMAP_DS_PB': '8192'}]
SETS['cg2'] = [{}, {'COMAP_DS_BU': '8'}, {'COMAP_DS_PB': '8192'}, {'COMAP_DS_BU': '8', 'COMAP_DS_PB': '8192'},
              {'COMAP_DS_BL': '64', 'COMAP_DS_BU': '8', 'COMAP_DS_PB': '8192'}, {}]
SETS['cg3'] = [{}, {'COMAP_DS_PU': '8'}, {'COMAP_DS_BL': '32'}, {'COMAP_DS_PB': '4096'}, {}]
SETS['walk'] = [{}, {'COMAP_DS_WXCD': '0'}, {'COMAP_DS_HEAVY': '0'}, {'COMAP_DS_WXCD': '0', 'COMAP_DS_HEAVY': '0'}]
# knobs the current kernels read (the removed variants' knobs are gone with them)
KEYS = ('COMAP_DS_PG', 'COMAP_DS_PU', 'COMAP_DS_PB', 'COMAP_DS_BU', 'COMAP_DS_BL', 'COMAP_DS_SELL', 'COMAP_DS_TILE',
        'COMAP_DS_OKEY', 'COMAP_DS_HEAVY', 'COMAP_DS_WXCD')


def main():
    import torch
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    n_obs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    bands = [int(b) for b in sys.argv[3:] if not b.startswith('set=')] or [1, 4]
    which = ([a[4:] for a in sys.argv[3:] if a.startswith('set=')] or ['layout'])[0]
    torch.cuda.set_device(0)
    for nb in bands:
        pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=50, device=0, seed=1000, n_bands=nb)
        for st in SETS[which]:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(st)
            setup = None
            for _ in range(2):           # the second build is timed (the first warms the caches)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                prob = D.DeviceDestriper(pix, tod, w, 50, 480 * 480, device=0, map_shape=(480, 480))
                torch.cuda.synchronize()
                setup = (time.perf_counter() - t0) * 1e3
            prob.solve(threshold=0.0, niter=3)
            best = None
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = prob.solve(threshold=0.0, niter=iters)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / iters * 1e3
                best = dt if best is None else min(best, dt)
            x = res['x']
            print(json.dumps({'bands': nb, 'setting': st, 'ms_per_iter': best, 'setup_ms': setup,
                              'x_sum': float(x.double().sum()), 'x_abs': float(x.double().abs().sum())}), flush=True)
            del prob, res
        for k in KEYS:
            os.environ.pop(k, None)
        del pix, tod, w
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
