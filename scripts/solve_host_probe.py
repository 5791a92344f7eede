"""Host-side timing of DeviceOps.solve_native_host's steps (the chain's solve with maps to
the host): where the GPU-idle gap before the CG's first kernel comes from.
    python scripts/solve_host_probe.py [n_obs] [reps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from comapreduce_amd import _native as N
    from comapreduce_amd import synthetic
    from comapreduce_amd.mapmaking import destriper as D
    n_obs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    torch.cuda.set_device(0)
    pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=50, device=0, seed=7, n_bands=4)
    prob = D.DeviceDestriper(pix, tod, w, 50, 480 * 480, device=0)
    ops = prob.ops
    prob.solve(threshold=1e-6, niter=100, to_host=True)        # warm
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = {}
        t0 = time.perf_counter()

        def mark(k):
            t[k] = (time.perf_counter() - t0) * 1e3
        nb, npix, nbo = ops.nb, ops.npix, ops.n_bands
        cur = torch.cuda.current_stream(ops.dev)
        m = torch.empty((4, npix * nb), dtype=torch.float64, device=ops.dev)
        nn = ops.zeros(npix * nb)
        mark('alloc')
        ops._c('comap_destripe_local_maps', ops.h, N.dptr(m[2]), N.dptr(m[3]), N.dptr(nn))
        ops._c('comap_destripe_div_map', ops.h, N.dptr(nn), None, N.dptr(m[1]))
        mark('local_maps')
        bands = m.view(4, npix, nb).permute(0, 2, 1)[:, :nbo]
        static = bands[1:].contiguous()
        mark('static')
        host_np = N.host_empty((4, nbo, npix))
        mark('host_empty')
        host = torch.from_numpy(host_np)
        mark('from_numpy')
        ready = torch.cuda.Event()
        ready.record(cur)
        cs = torch.cuda.Stream(ops.dev) if not hasattr(ops, '_probe_cs') else ops._probe_cs
        ops._probe_cs = cs
        cs.wait_event(ready)
        mark('event')
        with torch.cuda.stream(cs):
            host[1:].copy_(static, non_blocking=True)
        mark('copy_enqueue')
        x = ops.zeros(ops.n_offsets * nb)
        it = (ctypes.c_int32 * nb)()
        ops._c('comap_destripe_solve', ops.h, 1e-6, 100, N.dptr(x), N.dptr(m[0]), None, None, None,
               ctypes.cast(it, ctypes.POINTER(ctypes.c_int32)))
        mark('solve_enqueue')
        host[0].copy_(bands[0], non_blocking=True)
        mark('map_copy_enqueue')
        cur.synchronize()
        cs.synchronize()
        mark('done')
        out.append({k: round(v, 3) for k, v in t.items()})
        del host_np, host
    print(json.dumps({'n_samples': int(pix.numel()), 'steps_ms': out}), flush=True)


if __name__ == '__main__':
    main()
