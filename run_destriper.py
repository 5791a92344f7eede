#!/usr/bin/env python3
"""Map-making entry point (mirror of the reference MapMaking/run_destriper.py).

    python run_destriper.py parameters.ini
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        run_destriper.py parameters.ini

Each rank binds GPU LOCAL_RANK and joins the nccl (RCCL) process group; the
destriper's per-iteration map all-reduce runs over xGMI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', 1))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', 0)))
        dist.init_process_group('nccl')
    from comapreduce_amd.mapmaking.run_destriper import cli
    try:
        cli(argv)
    finally:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()


if __name__ == '__main__':
    main()
