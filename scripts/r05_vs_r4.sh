#!/bin/bash
# Same-box comparison of the r4 build (ab_r4/: its bench.py and libraries) with this tree:
# scripts/r05_vs_r4.sh <tag> [extra bench flags for this tree]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
mkdir -p gpurun_out/r05/vs_$tag
for rep in 1 2; do
  (cd ab_r4 && timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline) > gpurun_out/r05/vs_$tag/r4_$rep.log 2>&1 || exit $?
  echo "r4 $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05/vs_$tag/r4_$rep.log | head -1)"
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline "$@" > gpurun_out/r05/vs_$tag/r5_$rep.log 2>&1 || exit $?
  echo "r5 $rep $(python3 scripts/bline.py gpurun_out/r05/vs_$tag/r5_$rep.log)"
done
