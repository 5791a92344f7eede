#!/usr/bin/env python3
"""Per-kernel averages of every counter in gpurun_out/pmc_<tag>/ (sum over instances per dispatch)."""
import csv, glob, re, sys
from collections import defaultdict
d = sys.argv[1]
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'\bk_(\w+)\s*(?:<[^()]*>)?\s*\(', r['Kernel_Name'])
        k = m.group(1) if m else r['Kernel_Name'][:30]
        per[k][r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
for k, cs in sorted(per.items()):
    print(k.ljust(24), '  '.join(f'{c}={sum(v.values())/len(v):.4g}' for c, v in sorted(cs.items())))
