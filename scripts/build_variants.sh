#!/bin/bash
# Build tuning variants of libcomap_hip.so into exp/<name>/ (git-ignored; they travel with gpurun).
# usage: scripts/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "..." ...
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -C comapreduce_amd/csrc -j8 OUTDIR=$PWD/exp/$name OBJDIR=/tmp/comap_obj_$name EXTRA="$flags"
  echo "built exp/$name ($flags)"
done
