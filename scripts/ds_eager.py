"""Cost of the multi-rank CG driver: cg_solve_batched (identity sums, one rank)
against the native graph-batched solve on the same problem.
usage: python scripts/ds_eager.py [n_obs] [n_bands] [niter]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking.destriper import DeviceOps, cg_solve_batched
    n_obs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    niter = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    torch.cuda.set_device(0)
    pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=50, device=0, seed=7, n_bands=nb)
    ops = DeviceOps(pix, tod, w, 50, 480 * 480)
    out = {'n_obs': n_obs, 'bands': nb, 'niter': niter, 'offsets': ops.n_offsets}
    ops.solve_native(0.0, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.solve_native(0.0, niter)
    torch.cuda.synchronize()
    out['native_ms_per_iter'] = (time.perf_counter() - t0) / niter * 1e3
    cg_solve_batched(ops, lambda a: a, threshold=0.0, niter=3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cg_solve_batched(ops, lambda a: a, threshold=0.0, niter=niter)
    torch.cuda.synchronize()
    out['batched_ms_per_iter'] = (time.perf_counter() - t0) / niter * 1e3
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
