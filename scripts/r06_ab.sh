#!/bin/bash
# Same-box A/B (r6): the bench step of a baseline build (ab_r6a, KFP16_LIBDIR) against this
# tree, alternating.
# usage: bash scripts/r06_ab.sh [reps] ; BENCH_ARGS adds bench flags
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
reps=${1:-2}
for i in $(seq 1 $reps); do
  for v in ab_r6a cur; do
    unset KFP16_LIBDIR
    [ $v = ab_r6a ] && export KFP16_LIBDIR=$(realpath ab_r6a)
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra $BENCH_ARGS > gpurun_out/ab/r06_bench_${v}_$i.log 2>&1 || exit $?
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/r06_bench_${v}_$i.log | head -1) $(grep -o '"den_ms_per_step": [0-9.]*' gpurun_out/ab/r06_bench_${v}_$i.log)"
  done
done
