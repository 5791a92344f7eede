#!/bin/bash
# rocprofv3 evidence for the destriper at C5 (scripts/ds_c5.py: n_obs observations x 19 feeds x
# 180,000 samples, n_bands batched, niter CG iterations, one GPU): kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate passes (see profile.sh for the gfx950 correction).
# Usage: bash profiles/profile_ds.sh <tag> [n_obs n_bands niter]
set -euo pipefail
TAG=${1:-r02_c5}
shift || true
ARGS=${*:-8 4 30}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 scripts/ds_c5.py $ARGS > "$OUT/ds_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 scripts/ds_c5.py $ARGS > "$OUT/ds_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 scripts/ds_c5.py $ARGS > "$OUT/ds_write.log" 2>&1
python3 profiles/summarize.py "$OUT" "$TAG" --no-latest
