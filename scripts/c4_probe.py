"""C4-size destriper solve timing (one synthetic observation, 1 and 4 bands): 100
fixed CG iterations and the converged solve, median of reps -- for A/B runs of two
library builds on one box (COMAP_HIP_LIB).
    python scripts/c4_probe.py [reps]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get('PROBE_ROOT') or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    torch.cuda.set_device(0)
    out = {'lib': os.environ.get('COMAP_HIP_LIB', 'in-tree')}
    for nb in (1, 4):
        pix, tod, w = synthetic.destriper_inputs_device(1, offset_length=50, device=0, seed=7, n_bands=nb)
        prob = D.DeviceDestriper(pix, tod, w, 50, 480 * 480, device=0)
        prob.solve(threshold=0.0, niter=3)
        for name, thr, nit in (('fixed100', 0.0, 100), ('converged', 1e-6, 100)):
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                prob.solve(threshold=thr, niter=nit)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            out[f'nb{nb}_{name}_ms'] = round(statistics.median(ts), 4)
        del prob
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
