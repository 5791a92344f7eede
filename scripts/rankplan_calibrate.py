"""Replace rankplan.py's assumed all-reduce alpha / beta with the driver's measurement.

Reads SCALE / BENCH JSON records (any nesting: every dict holding bench.py's
``allreduce_probe`` -- n_ranks, points [{bytes, us}], alpha_us, beta_GBs -- is taken, and
every ``comm_rank0`` beside it) and writes comapreduce_amd/mapmaking/rankplan_measured.json:
{"alpha_us": {n: us}, "beta_GBs": {n: GB/s}, "comm_ms_per_iter": {n: ms}, "source": [...]}.
rankplan.CostModel() loads that file when present.

    python scripts/rankplan_calibrate.py SCALE_r05.json [more.json ...]
"""
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'comapreduce_amd', 'mapmaking',
                   'rankplan_measured.json')


def walk(o, found):
    if isinstance(o, dict):
        pr = o.get('allreduce_probe')
        if isinstance(pr, dict) and pr.get('n_ranks', 1) > 1:
            found.append((pr, o.get('comm_rank0')))
        for v in o.values():
            walk(v, found)
    elif isinstance(o, list):
        for v in o:
            walk(v, found)
    elif isinstance(o, str) and o.lstrip().startswith('{'):
        try:
            walk(json.loads(o), found)
        except ValueError:
            pass


def main(paths):
    found = []
    for p in paths:
        with open(p) as f:
            txt = f.read()
        try:
            walk(json.loads(txt), found)
        except ValueError:              # a log: one JSON object per line
            for line in txt.splitlines():
                if line.lstrip().startswith('{'):
                    walk(line, found)
    if not found:
        sys.exit('no allreduce_probe with n_ranks > 1 in ' + ', '.join(paths))
    out = {'alpha_us': {}, 'beta_GBs': {}, 'comm_ms_per_iter': {}, 'source': [os.path.basename(p) for p in paths]}
    for pr, comm in found:
        n = str(int(pr['n_ranks']))
        out['alpha_us'][n] = max(float(pr['alpha_us']), 0.0)
        if pr.get('beta_GBs'):
            out['beta_GBs'][n] = float(pr['beta_GBs'])
        if comm:
            out['comm_ms_per_iter'][n] = float(comm['allreduce_ms_per_iter'])
    with open(OUT, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(sys.argv[1:])
