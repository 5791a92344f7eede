#!/usr/bin/env python3
"""Summarise a profiles/profile.sh run into profiles/<tag>_*.{csv,json}.

kernel stats  : average duration per kernel (rocprofv3 --stats)
traffic       : per-kernel HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024
                (gfx950 FETCH_SIZE under-reports wide coalesced reads by 2x,
                MI355X_MICROARCH.md §HBM), averaged over launches.
Writes <out>/summary/{<tag>_kernel_stats.csv,<tag>_traffic.json,traffic_latest.json}
(under gpurun_out/, which is what travels back from the GPU box); copy them
into profiles/ to commit -- bench.py reads profiles/traffic_latest.json for
roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

KERNEL_RE = re.compile(r'\bk_(\w+)\s*(<[^()]*>)?\s*(?:\(|$)')


def short(name):
    """'k_regress_avg(float const*, ...)' -> 'regress_avg' (the bench's kernel key);
    templates keep their arguments: 'k_ds_project<16, 4>(...)' -> 'ds_project<16,4>'."""
    m = KERNEL_RE.search(name.strip())
    if not m:
        return None
    return m.group(1) + (m.group(2).replace(' ', '') if m.group(2) else '')


def counter_bytes(d, counter):
    per = {}
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get('Counter_Name') != counter:
                continue
            k = short(row.get('Kernel_Name', ''))
            if k is None:
                continue
            per.setdefault(k, {}).setdefault(row['Dispatch_Id'], 0.0)
            per[k][row['Dispatch_Id']] += float(row['Counter_Value'])
    return {k: sum(v.values()) / max(len(v), 1) for k, v in per.items()}


def main():
    out, tag = sys.argv[1], sys.argv[2]
    latest = '--no-latest' not in sys.argv[3:]
    here = os.path.join(out, 'summary')
    os.makedirs(here, exist_ok=True)
    stats = glob.glob(os.path.join(out, 'trace', '**', '*kernel_stats.csv'), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(here, f'{tag}_kernel_stats.csv'))
    fetch = counter_bytes(os.path.join(out, 'fetch'), 'FETCH_SIZE')
    write = counter_bytes(os.path.join(out, 'write'), 'WRITE_SIZE')
    traffic = {}
    for k in set(fetch) | set(write):
        traffic[k] = {'hbm_bytes_per_launch': (2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024,
                      'fetch_size_kb': fetch.get(k), 'write_size_kb': write.get(k)}
    json.dump(traffic, open(os.path.join(here, f'{tag}_traffic.json'), 'w'), indent=1)
    if latest:
        json.dump(dict({k: v['hbm_bytes_per_launch'] for k, v in traffic.items()}, _source=tag),
                  open(os.path.join(here, 'traffic_latest.json'), 'w'), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == '__main__':
    main()
