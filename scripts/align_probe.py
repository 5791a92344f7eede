"""Pass-rate probe: bench.py's L1 leg with the synthetic scans' start shifted by S samples
(SCAN_START = 1500 + S), so the scans' first samples sit at another offset inside a 16-B
chunk -- does pass A's rate depend on its rows' alignment?
    python scripts/align_probe.py S [bench args...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from comapreduce_amd import synthetic
    shift = int(sys.argv[1])
    synthetic.SCAN_START = 1500 + shift
    import bench
    sys.argv = ['bench.py'] + (sys.argv[2:] or ['--steps', '5', '--warmup', '2', '--no-cpu-baseline', '--no-e2e',
                                                '--no-chain', '--no-destriper'])
    bench.main()


if __name__ == '__main__':
    main()
