"""Kernel-trace timeline of one chain (rocprofv3 --kernel-trace run_kernel_trace.csv):
kernels in dispatch order with their durations and the idle gap before each, between two
marker kernels (default: from the first k_ds / prep kernel after the last L1 pass to the
end).  Prints a compact table and the sums (busy, idle).
    python scripts/trace_gaps.py TRACE.csv [--after NAME] [--last N]"""
import csv
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    depth, out = 0, []
    for ch in n:
        if ch == '(' and depth == 0:
            break
        depth += ch == '<'
        depth -= ch == '>'
        out.append(ch)
    return ''.join(out)[:70]


def main():
    path = sys.argv[1]
    after = sys.argv[sys.argv.index('--after') + 1] if '--after' in sys.argv else 'k_regress'
    last = int(sys.argv[sys.argv.index('--last') + 1]) if '--last' in sys.argv else 1
    rows = list(csv.DictReader(open(path)))
    ev = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name'])) for r in rows))
    # the window: after the last-but-(last-1) occurrence of `after` to the end of the trace
    idx = [i for i, e in enumerate(ev) if after in e[2]]
    if not idx:
        sys.exit(f'no kernel named {after}')
    i0 = idx[-last] + 1
    # stop at the next occurrence (if any) of the first L1 kernel after i0
    i1 = len(ev)
    for j in range(i0, len(ev)):
        if 'k_moments' in ev[j][2]:
            i1 = j
            break
    busy = idle = 0
    prev = ev[i0 - 1][1]
    agg = {}
    for s, e, n in ev[i0:i1]:
        gap = max(0, s - max(prev, 0))
        print(f'{gap / 1e3:9.1f} gap {(e - s) / 1e3:9.1f} us  {n}')
        busy += e - s
        idle += gap
        prev = max(prev, e)
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    print(f'window: {(prev - ev[i0 - 1][1]) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle gaps {idle / 1e3:.1f} us, '
          f'{i1 - i0} kernels')
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f'  {c:4d} x  {t / 1e3:9.1f} us  {n}')


if __name__ == '__main__':
    main()
