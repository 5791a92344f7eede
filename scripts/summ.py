"""Summarise a GPU pass: kernel stats of ds runs and the bench line (usage: python scripts/summ.py TAG)."""
import csv
import json
import os
import sys

T = sys.argv[1]
for tag in ('ds1', 'ds4'):
    f = f'gpurun_out/{T}_{tag}/run_kernel_stats.csv'
    if not os.path.exists(f):
        continue
    print(f)
    for r in list(csv.DictReader(open(f)))[:6]:
        n = r['Name'][:60]
        print(f"  {n:62s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.1f}us")
f = f'gpurun_out/{T}_bench.log'
if os.path.exists(f):
    d = json.loads([ln for ln in open(f) if ln.startswith('{')][0])
    print('value', f"{d['value']:.4g}", 'ms', round(d['ms_per_step'], 3), 'frac', round(d['roofline']['frac'], 4))
    print('kernel ms', {k: round(v, 3) for k, v in d['kernel_ms_per_step'].items() if v > 0.05})
    if 'destriper' in d:
        print('C4 it/s', round(d['destriper']['cg_iters_per_s']), 'C4 4-band band-it/s',
              round(d['destriper']['bands4']['band_iters_per_s']))
    if 'destriper_c5' in d:
        c5 = d['destriper_c5']
        b = c5['bands4']
        print('C5 1b ms/it', round(c5['ms_per_iter'], 4), 'frac', round(c5['roofline_frac'], 3), '| 4b ms/band-it',
              round(b['ms_per_band_iter'], 4), 'frac', round(b['roofline_frac'], 3))
    if 'end_to_end_host' in d:
        print('e2e', {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d['end_to_end_host'].items()})
