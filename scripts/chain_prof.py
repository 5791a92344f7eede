"""The north_star chain leg (bench.chain_leg) alone, with the device prep's phase
breakdown (COMAP_PREP_PROFILE=1) and the destriper's first-solve vs repeat-solve
time, for kernel traces of the chain's non-L1 part:
    python scripts/chain_prof.py [feeds]
    python scripts/chain_prof.py --cprofile OUT.txt   (host cProfile of one unsynced chain)
    python scripts/chain_prof.py --plain              (3 unsynced chains, for a kernel trace)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if '--cprofile' not in sys.argv and '--plain' not in sys.argv:
    os.environ.setdefault('COMAP_PREP_PROFILE', '1')
import bench  # noqa: E402


def host_profile(path, profile=True):
    """cProfile one unsynced chain (after two warm ones): where the host spends the
    wall clock the GPU timeline does not account for."""
    import cProfile
    import io
    import pstats
    import torch
    torch.cuda.set_device(0)
    data, sh = bench.build_observation(19, 180_000, obs_id=1, device=0)
    chain = bench.chain_fn(data, 0)
    for _ in range(2):
        chain(False)
    torch.cuda.synchronize()
    walls = []
    pr = cProfile.Profile()
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if i == 2 and profile:
            pr.enable()
        chain(False)
        torch.cuda.synchronize()
        if i == 2 and profile:
            pr.disable()
        walls.append((time.perf_counter() - t0) * 1e3)
    if not profile:
        print(json.dumps({'walls_ms': walls}), flush=True)
        return
    buf = io.StringIO()
    st = pstats.Stats(pr, stream=buf)
    st.sort_stats('cumulative').print_stats(60)
    st.sort_stats('tottime').print_stats(40)
    with open(path, 'w') as f:
        f.write(f'walls_ms {walls}\n')
        f.write(buf.getvalue())
    print(json.dumps({'walls_ms': walls}), flush=True)


def main():
    import torch
    if len(sys.argv) > 2 and sys.argv[1] == '--cprofile':
        return host_profile(sys.argv[2])
    if len(sys.argv) > 1 and sys.argv[1] == '--plain':
        return host_profile(None, profile=False)
    from comapreduce_amd.mapmaking import comapdata as CD
    from comapreduce_amd.mapmaking import destriper as D
    from comapreduce_amd.mapmaking import prep
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 19
    torch.cuda.set_device(0)
    data, sh = bench.build_observation(F, 180_000, obs_id=1, device=0)
    level2 = bench.reduce_step(data, 0)
    level2 = bench.reduce_step(data, 0)
    dev = torch.device('cuda', 0)
    out = {}
    pointing = bench.pointing_device(data, dev)
    for rep in range(3):
        store = bench.level2_store_device(level2, data, 1, dev, pointing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = CD.read_comap_data_bands(list(store), bench.c4_map_info(), bands=(0, 1, 2, 3), offset_length=50,
                                     store=store, device=0, device_outputs=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        prob = D.DeviceDestriper(r['pointing'].to(torch.int32), r['tod'], r['weights'], 50, 480 * 480, device=0,
                                 keep=r['keep'])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = prob.solve(threshold=1e-6, niter=100)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        res = prob.solve(threshold=1e-6, niter=100)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        out[f'rep{rep}'] = {'prep_ms': (t1 - t0) * 1e3, 'prep_phases_ms': {k: v * 1e3 for k, v in prep.last_phases.items()},
                            'setup_ms': (t2 - t1) * 1e3, 'first_solve_ms': (t3 - t2) * 1e3,
                            'repeat_solve_ms': (t4 - t3) * 1e3, 'iters': res['iters']}
        del prob, res, r, store
    out['chain'] = bench.chain_leg(data, 0, 1.6e11, reps=2)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
