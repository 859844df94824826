#!/bin/bash
# A/B of bench.py flag sets on one box (no profiler): scripts/r05_abflags.sh <tag> "<flags A>" "<flags B>" ...
# ("-" = no extra flags). Each run: --steps 20 --warmup 5 (the driver's) --no-extra --no-cpu-baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
mkdir -p gpurun_out/r05/abf_$tag
i=0
for f in "$@"; do
  i=$((i+1))
  [ "$f" = "-" ] && f=""
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $f > gpurun_out/r05/abf_$tag/$i.log 2>&1 || exit $?
  echo "$i [$f] $(python3 scripts/bline.py gpurun_out/r05/abf_$tag/$i.log)"
done
