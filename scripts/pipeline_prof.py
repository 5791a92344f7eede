"""The pipelined multi-observation chain (bench.chain_pipeline_fn) alone, for a kernel
trace: two warm observations, then n timed ones; prints the delivery intervals.
    python scripts/pipeline_prof.py [n]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.cuda.set_device(0)
    data, _ = bench.build_observation(19, 180_000, obs_id=1, device=0)
    run = bench.chain_pipeline_fn(data, 0)
    run(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    maps, iters, t_done = run(n)
    torch.cuda.synchronize()
    print(json.dumps({'wall_ms': (time.perf_counter() - t0) * 1e3,
                      'intervals_ms': [(b - a) * 1e3 for a, b in zip(t_done, t_done[1:])],
                      'first_ms': (t_done[0] - t0) * 1e3}), flush=True)


if __name__ == '__main__':
    main()
