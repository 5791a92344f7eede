"""Pixel-row lengths (entries = distinct (offset, pixel) pairs per pixel) of the destriper
field problem (bench's configs[4] inputs), to size the CG bin's and the set-up walk's tails:
    python scripts/row_length_probe.py [n_obs]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from comapreduce_amd import synthetic
    n_obs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    torch.cuda.set_device(0)
    pix, tod, w = synthetic.destriper_inputs_device(n_obs, offset_length=50, device=0, seed=1000, n_bands=1)
    del tod, w
    npix = 480 * 480
    L = 50
    n = pix.numel() // L * L
    p = pix[:n].to(torch.int64)
    off = torch.arange(n, device=p.device, dtype=torch.int64) // L
    on = (p >= 0) & (p < npix)
    key = torch.unique(off[on] * npix + p[on])
    rows = torch.bincount(key % npix, minlength=npix)
    samp = torch.bincount(p[on], minlength=npix)
    r = rows.double()
    nz = r[r > 0]
    out = {'n_obs': n_obs, 'entries': int(rows.sum()), 'nonempty_rows': int(nz.numel()),
           'mean_nonempty': float(nz.mean()), 'max_row': int(rows.max()), 'max_row_samples': int(samp.max()),
           'quantiles': {str(q): float(torch.quantile(nz.float()[:1 << 24], q)) for q in (0.5, 0.9, 0.99, 0.999)}}
    for t in (1024, 2048, 4096, 8192, 16384):
        m = rows > t
        out[f'rows_gt_{t}'] = int(m.sum())
        out[f'entries_in_rows_gt_{t}'] = int(rows[m].sum())
        out[f'samples_in_rows_gt_{t}'] = int(samp[m].sum())
    top = torch.topk(rows, 10)
    out['top10'] = [int(v) for v in top.values]
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
