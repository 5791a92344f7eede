"""Median unsynced chain wall time over many repetitions in ONE process (for A/B runs of
two library builds on the same box: COMAP_HIP_LIB=... python scripts/chain_ab.py TAG)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get('COMAP_HIP_LIB', 'default')
    torch.cuda.set_device(0)
    data, sh = bench.build_observation(19, 180_000, obs_id=1, device=0)
    chain = bench.chain_fn(data, 0)
    for _ in range(3):
        chain(False)
    torch.cuda.synchronize()
    walls, synced = [], []
    for _ in range(15):
        t0 = time.perf_counter()
        chain(False)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
    for _ in range(8):
        info = chain(True)
        synced.append({k: round(v, 3) for k, v in info.items() if k.endswith('_ms')})
    print(tag, 'chain median %.3f ms min %.3f' % (statistics.median(walls), min(walls)), flush=True)
    for k in synced[0]:
        v = [x[k] for x in synced]
        print(tag, 'synced', k, 'median %.3f' % statistics.median(v), v, flush=True)


if __name__ == '__main__':
    main()
