"""File -> HBM staging rate of a Level-1 cube in an HDF5 file (gpu.upload over
comap_h5_read_flat) vs the same cube from a pageable host array.  The file is
written to $TMPDIR first, so its read is page-cache hot: this measures the
native read + pinned staging pipeline, not the disk.
usage: python scripts/h5_upload.py [n_feeds] [n_samples]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from comapreduce_amd import gpu
    from comapreduce_amd.pipeline.h5file import H5File
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 180_000
    path = os.path.join(os.environ.get('TMPDIR', '/tmp'), f'h5_upload_{os.getpid()}.hd5')
    x = np.empty((F, 4, 1024, T), dtype=np.float32)
    rng = np.random.default_rng(0)
    for f in range(F):
        x[f] = rng.standard_normal((4, 1024, T), dtype=np.float32)
    t0 = time.perf_counter()
    with H5File(path, 'w') as h:
        h.write('spectrometer/tod', x)
    t_write = time.perf_counter() - t0
    dev = torch.device('cuda', 0)
    gb = x.nbytes / 1e9
    res = {'feeds': F, 'samples': T, 'GB': gb, 'file_write_s': t_write}
    try:
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a = gpu.upload(x, dev)
            torch.cuda.synchronize()
            res[f'pageable_GBs_{rep}'] = gb / (time.perf_counter() - t0)
            del a
            with H5File(path) as h:
                d = h.dataset('spectrometer/tod')
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                b = gpu.to_device(d, torch.float32, dev)
                torch.cuda.synchronize()
                res[f'hdf5_GBs_{rep}'] = gb / (time.perf_counter() - t0)
            if rep == 1:
                assert torch.equal(b[F - 1, 3, 1000, -5:].cpu(), torch.from_numpy(x[F - 1, 3, 1000, -5:]))
            del b
    finally:
        os.remove(path)
    print(res, flush=True)


if __name__ == '__main__':
    main()
