#!/bin/bash
# A/B of KF_EXPT experiment bits under rocprofv3 (one build; the r5 experiment builds read KF_EXPT,
# the committed code has no bits left): scripts/r05_abenv.sh <tag> v1 v2 ...
# (a value listed twice shows the spread; BENCH_ARGS adds bench flags)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/r05/ab_$tag
i=0
for v in "$@"; do
  i=$((i+1))
  t=e${v}_$i
  KF_EXPT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/ab_$tag/$t -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra $BENCH_ARGS > gpurun_out/r05/ab_$tag/$t.log 2>&1 || exit $?
  echo "$t $(python3 scripts/bline.py gpurun_out/r05/ab_$tag/$t.log)"
done
