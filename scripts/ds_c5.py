"""C5 destriper alone (bench.destriper_c5_leg), for rocprofv3 kernel traces and PMC passes:
    python scripts/ds_c5.py [n_obs] [n_bands] [niter] [field]
("field": bench.destriper_c5_field_leg, the configs[4] field solved as one system)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    n_obs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    niter = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    torch.cuda.set_device(0)
    leg = bench.destriper_c5_field_leg if 'field' in sys.argv[4:] else bench.destriper_c5_leg
    print(json.dumps(leg(n_obs, niter, 0, 1, 0, n_bands=nb)), flush=True)


if __name__ == '__main__':
    main()
