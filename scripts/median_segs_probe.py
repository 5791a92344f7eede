"""Round-5 probe: wavelet-matrix walk segments per median plan (COMAP_MEDIAN_WMSEGS).
The walk runs one workgroup per segment with ~85 KB of LDS at ~15 k outputs (one per CU),
so 912 series make 3.6 rounds on 256 CUs; splitting series into more, shorter segments
packs 2-3 workgroups per CU (each re-reads its job's sorted sources).  Runs bench.py's L1
step + chain per value in a child process and prints the L1 median kernel time and the
chain's synced prep phase.
    python scripts/median_segs_probe.py [targets or KEY=VAL,KEY=VAL specs...]"""
import json
import os
import subprocess
import sys


def main():
    specs = sys.argv[1:] or ['128', '1024', '2048', '4096']
    for t in specs:
        extra = dict(kv.split('=') for kv in t.split(',')) if '=' in t else {'COMAP_MEDIAN_WMSEGS': t}
        env = dict(os.environ, **extra)
        out = subprocess.run([sys.executable, 'bench.py', '--steps', '3', '--warmup', '1', '--no-e2e',
                              '--no-cpu-baseline', '--c5-obs', '0', '--c5-field-obs', '0'],
                             env=env, capture_output=True, text=True, timeout=280)
        line = next((l for l in out.stdout.splitlines() if l.startswith('{')), None)
        if line is None:
            print(json.dumps({'target': t, 'rc': out.returncode, 'err': out.stderr[-500:]}), flush=True)
            continue
        d = json.loads(line)
        print(json.dumps({'target': t, 'l1_median_ms': d['kernel_ms_per_step'].get('median'),
                          'step_ms': d['ms_per_step'], 'chain_ms': d['chain_l1_to_maps']['wall_ms'],
                          'phases': d['chain_l1_to_maps']['phases_synced_ms']}), flush=True)


if __name__ == '__main__':
    main()
