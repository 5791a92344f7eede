"""RCCL all-reduce latency of the destriper's per-iteration payloads on ONE rank
(DESIGN §8 multi-rank model): the compacted map numerator (n_hit x NB f64) and the
two block-partial vectors (1024 x NB f64 = 32 KB for 4 bands), eager (host enqueue,
back to back) and captured into a HIP graph (16 per replay, as cg_solve_graph does).
A one-rank communicator moves no bytes over xGMI: this is the launch / protocol floor
the model adds to the per-hop terms.

    python scripts/rccl_latency.py        (on the GPU box; one process, world size 1)
"""
import json
import os
import time


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    out = {}
    for name, n in (('map_c4_4band', 31_000 * 4), ('map_c4_1band', 31_000), ('partials_4band', 4096),
                     ('partials_1band', 1024), ('scalar', 4)):
        t = torch.zeros(n, dtype=torch.float64, device='cuda')
        for _ in range(20):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        reps = 200
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(50):
            dist.all_reduce(t)
            torch.cuda.synchronize()
        synced = (time.perf_counter() - t0) / 50 * 1e6
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            dist.all_reduce(t)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(16):
                    dist.all_reduce(t)
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / (20 * 16) * 1e6
        out[name] = {'bytes': n * 8, 'eager_us': eager, 'eager_synced_us': synced, 'graph_us': graph}
    print(json.dumps({'rccl_one_rank_allreduce': out}), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
