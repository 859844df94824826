#!/bin/bash
# r05 A/B under rocprofv3 (kernel stats of a short default bench per build).
# usage: scripts/r05_ab.sh <tag> <libdir> [<libdir> ...]   (a directory listed twice shows the spread)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/r05/ab_$tag
i=0
for d in "$@"; do
  i=$((i+1))
  t=$(basename "$(dirname "$d")")_$(basename "$d")_$i
  KFP16_LIBDIR=$(realpath "$d") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/ab_$tag/$t -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra $BENCH_ARGS > gpurun_out/r05/ab_$tag/$t.log 2>&1 || exit $?
  echo "$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/ab_$tag/$t.log)"
done
