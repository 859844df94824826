#!/bin/bash
# rocprofv3 kernel stats of bench.py flag sets on one box: scripts/r05_abprof.sh <tag> "<flags A>" "<flags B>" ...
# ("-" = no extra flags; 5 timed + 2 warmup steps, no per-launch events)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/r05/abp_$tag
i=0
for f in "$@"; do
  i=$((i+1))
  [ "$f" = "-" ] && f=""
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/abp_$tag/p$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra $f > gpurun_out/r05/abp_$tag/p$i.log 2>&1 || exit $?
  echo "p$i [$f] $(python3 scripts/bline.py gpurun_out/r05/abp_$tag/p$i.log)"
done
