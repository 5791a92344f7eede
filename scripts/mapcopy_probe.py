"""Does the maps' device -> host copy on the side stream overlap the main stream's work?
(the chain trace shows the CG's first kernel starting only after the 395 us copy ends).
Times the host call of copy_(non_blocking=True) into the library's page-locked block
and into torch's pinned allocator, and a main-stream matmul issued right after it.
    python scripts/mapcopy_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from comapreduce_amd import _native as N  # noqa: E402
from comapreduce_amd.mapmaking.destriper import copy_stream  # noqa: E402


def probe(kind, src, work):
    dev = src.device
    cur = torch.cuda.current_stream(dev)
    if kind == 'lib':
        host = torch.from_numpy(N.host_empty(tuple(src.shape)))
    else:
        host = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
    cs = copy_stream(dev)
    torch.cuda.synchronize()
    e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    ready = torch.cuda.Event()
    ready.record(cur)
    cs.wait_event(ready)
    t0 = time.perf_counter()
    with torch.cuda.stream(cs):
        e0.record(cs)
        host.copy_(src, non_blocking=True)
        e1.record(cs)
    t1 = time.perf_counter()
    e2.record(cur)
    for _ in range(8):
        work = work @ work
        work /= work.norm()
    e3.record(cur)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    return dict(kind=kind, pinned=bool(host.is_pinned()), host_copy_call_us=(t1 - t0) * 1e6,
                host_work_enqueue_us=(t2 - t1) * 1e6, copy_us=e0.elapsed_time(e1) * 1e3,
                work_us=e2.elapsed_time(e3) * 1e3, work_start_after_copy_start_us=e0.elapsed_time(e2) * 1e3)


def main():
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    src = torch.randn(3, 4, 230400, dtype=torch.float64, device=dev)
    work = torch.randn(2048, 2048, device=dev)
    for _ in range(2):
        for kind in ('lib', 'torch'):
            print(probe(kind, src, work), flush=True)


if __name__ == '__main__' and '--chain' not in sys.argv:
    main()


def chain_probe():
    """The chain's solve_native_host with host timestamps around the side-stream copy and
    the library solve call (the trace shows the solve's first copy waiting for the maps'
    copy on the side stream)."""
    import bench
    from comapreduce_amd.mapmaking import destriper as D
    orig_copy = torch.Tensor.copy_
    marks = []

    def copy_(self, src, non_blocking=False):
        t0 = time.perf_counter()
        out = orig_copy(self, src, non_blocking=non_blocking)
        if self.device.type == 'cpu' and src.device.type == 'cuda':
            marks.append(('d2h', t0, time.perf_counter(), tuple(src.shape)))
        return out

    orig_c = D.DeviceOps._c

    def _c(self, name, *a):
        t0 = time.perf_counter()
        out = orig_c(self, name, *a)
        if name == 'comap_destripe_solve':
            marks.append(('solve', t0, time.perf_counter(), None))
        return out

    torch.Tensor.copy_ = copy_
    D.DeviceOps._c = _c
    torch.cuda.set_device(0)
    data, sh = bench.build_observation(19, 180_000, obs_id=1, device=0)
    chain = bench.chain_fn(data, 0)
    for rep in range(4):
        marks.clear()
        t0 = time.perf_counter()
        chain(False)
        torch.cuda.synchronize()
        z = marks[0][1] if marks else 0.0
        print(rep, 'chain ms %.2f' % ((time.perf_counter() - t0) * 1e3),
              [(k, round((a - z) * 1e6), round((b - z) * 1e6), sh) for k, a, b, sh in marks], flush=True)


if __name__ == '__main__' and '--chain' in sys.argv:
    chain_probe()
