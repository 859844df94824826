#!/bin/bash
# Same-box A/B of the libraries in ab_prev/lib (another build of this tree, KFP16_LIBDIR)
# against this tree's: scripts/r05_vs_prev.sh <tag> [bench flags]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
mkdir -p gpurun_out/r05/vp_$tag
for rep in 1 2; do
  KFP16_LIBDIR=$PWD/ab_prev/lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline "$@" > gpurun_out/r05/vp_$tag/prev_$rep.log 2>&1 || exit $?
  echo "prev $rep $(python3 scripts/bline.py gpurun_out/r05/vp_$tag/prev_$rep.log | cut -c1-60)"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline "$@" > gpurun_out/r05/vp_$tag/cur_$rep.log 2>&1 || exit $?
  echo "cur  $rep $(python3 scripts/bline.py gpurun_out/r05/vp_$tag/cur_$rep.log | cut -c1-60)"
done
