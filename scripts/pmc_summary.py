"""Per-kernel means of a rocprofv3 --pmc counter_collection.csv:
    python scripts/pmc_summary.py OUT_DIR name1,name2,..."""
import csv,sys,collections
d=sys.argv[1]; pats=sys.argv[2].split(',')
import glob
f=(glob.glob(d+"/**/*counter_collection.csv",recursive=True)+glob.glob(d+"*/*counter_collection.csv"))[0]
rows=list(csv.DictReader(open(f)))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in rows:
    k=r['Kernel_Name']
    if not any(p in k for p in pats): continue
    kk=next(p for p in pats if p in k)
    agg[kk][r['Counter_Name']]+=float(r['Counter_Value'])
    n[(kk,r['Counter_Name'])]+=1
for kk,v in agg.items():
    print(kk)
    for c,x in sorted(v.items()): print(f'   {c:32s} {x/n[(kk,c)]:.4g}  (per dispatch)')
