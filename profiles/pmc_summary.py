"""Per-kernel averages of rocprofv3 --pmc passes (run_counter_collection.csv), merged
over several pass directories:
    python profiles/pmc_summary.py OUT.json DIR [DIR ...] [--match SUBSTR ...]
Kernels are keyed by the name up to the first '(' (templates kept); values are the
mean over dispatches of each counter, plus the mean dispatch duration (ns) and grid /
VGPR / LDS of the first dispatch.  FETCH_SIZE / WRITE_SIZE (KB) are also given as
bytes, FETCH doubled per MI355X_MICROARCH.md's gfx950 correction."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kname(n):
    n = n.replace('(anonymous namespace)::', '')
    depth, out = 0, []
    for ch in n:
        if ch == '(' and depth == 0:
            break
        depth += ch == '<'
        depth -= ch == '>'
        out.append(ch)
    return ''.join(out).replace('void ', '').strip()


def main():
    args = sys.argv[1:]
    match = []
    if '--match' in args:
        i = args.index('--match')
        match = args[i + 1:]
        args = args[:i]
    out_path, dirs = args[0], args[1:]
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r['Kernel_Name'])
                if match and not any(m in k for m in match):
                    continue
                acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
                acc[k]['_dur_ns'].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
                meta.setdefault(k, {'grid': int(r['Grid_Size']), 'wg': int(r['Workgroup_Size']),
                                    'vgpr': int(r['VGPR_Count']), 'lds': int(r['LDS_Block_Size'])})
    res = {}
    for k, cs in acc.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e['_dispatches'] = len(cs['_dur_ns'])
        if 'FETCH_SIZE' in e:
            e['fetch_bytes_x2'] = e['FETCH_SIZE'] * 1024 * 2
        if 'WRITE_SIZE' in e:
            e['write_bytes'] = e['WRITE_SIZE'] * 1024
        if 'TCC_HIT_sum' in e and 'TCC_MISS_sum' in e:
            e['l2_hit_rate'] = e['TCC_HIT_sum'] / max(1.0, e['TCC_HIT_sum'] + e['TCC_MISS_sum'])
        e.update(meta[k])
        res[k] = e
    json.dump(res, open(out_path, 'w'), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda kv: -kv[1]['_dur_ns'] * kv[1]['_dispatches']):
        print(k[:60], {c: round(v, 3) if isinstance(v, float) else v for c, v in e.items() if not c.startswith('TCC_')})


if __name__ == '__main__':
    main()
