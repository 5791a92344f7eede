#!/bin/bash
# Collects the rocprofv3 evidence committed under profiles/ (run on the GPU box):
#   1. kernel trace + stats of bench.py (per-kernel average durations)
#   2. HBM traffic per kernel from PMC counters, in SEPARATE passes
#      (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no trace
#      domains are combined with --pmc).  MI355X_MICROARCH.md §HBM: on gfx950
#      FETCH_SIZE reports half the bytes of a wide coalesced streaming read,
#      so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is exact for
#      16-B streaming stores.
# Usage: bash profiles/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}
shift || true
ARGS=${*:---steps 2 --warmup 1 --no-cpu-baseline --no-destriper}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/bench_write.log" 2>&1
python3 profiles/summarize.py "$OUT" "$TAG"
