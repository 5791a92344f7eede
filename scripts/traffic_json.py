"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
separate runs, MI355X_MICROARCH.md's counter limits), with the guide's gfx950 correction:
FETCH_SIZE counts half of a wide streaming read, so bytes = 2 x FETCH_SIZE + WRITE_SIZE.
Writes profiles/<tag>_traffic.json and profiles/traffic_latest.json (bench.py's
roofline.traffic source).
    python scripts/traffic_json.py TAG FETCH_DIR WRITE_DIR"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    n = n.split('(')[0]
    n = re.sub(r'^k_', '', n)
    return n.replace(' ', '')


def per_kernel(d, counter):
    f = (glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
         + glob.glob(d.rstrip('/') + '*/*counter_collection.csv'))[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] == counter:
            acc[short(r['Kernel_Name'])].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag, fdir, wdir = sys.argv[1:4]
    fe, wr = per_kernel(fdir, 'FETCH_SIZE'), per_kernel(wdir, 'WRITE_SIZE')
    out, latest = {}, {}
    for k in sorted(set(fe) | set(wr)):
        b = (2 * fe.get(k, 0.0) + wr.get(k, 0.0)) * 1024
        out[k] = {'hbm_bytes_per_launch': b, 'fetch_size_kb': fe.get(k), 'write_size_kb': wr.get(k)}
        latest[k] = b
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    json.dump(out, open(os.path.join(root, 'profiles', f'{tag}_traffic.json'), 'w'), indent=1)
    latest['_source'] = tag
    json.dump(latest, open(os.path.join(root, 'profiles', 'traffic_latest.json'), 'w'), indent=1)
    for k in ('moments', 'band_sums', 'regress'):
        if k in out:
            print(k, round(out[k]['hbm_bytes_per_launch'] / 1e9, 2), 'GB')


if __name__ == '__main__':
    main()
