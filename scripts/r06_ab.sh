#!/bin/bash
# Same-box A/B (r6): the bench step of several variants, alternating, in one call.
# usage: bash scripts/r06_ab.sh [reps]
#   VARIANTS (default "ab_r6a@ab_r6a cur"): space-separated tokens label[@libdir][%VAR=VALUE][+ARG],
#     libdir: another build's lib directory (KFP16_LIBDIR), VAR=VALUE: one environment setting,
#     ARG: one extra bench flag (e.g. +--no-prof)
#   BENCH_ARGS adds bench flags
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
reps=${1:-2}
variants=${VARIANTS:-"ab_r6a@ab_r6a cur"}
for i in $(seq 1 $reps); do
  for tok in $variants; do
    label=${tok%%[@%+]*}
    lib=""; envs=""; arg=""
    case "$tok" in *+*) arg=${tok#*+}; tok=${tok%%+*};; esac
    case "$tok" in *@*) lib=${tok#*@}; lib=${lib%%%*};; esac
    case "$tok" in *%*) envs=${tok#*%};; esac
    ( unset KFP16_LIBDIR
      [ -n "$lib" ] && export KFP16_LIBDIR=$(realpath "$lib")
      [ -n "$envs" ] && export "$envs"
      timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra $BENCH_ARGS $arg \
          > gpurun_out/ab/r06_bench_${label}_$i.log 2>&1 ) || exit $?
    echo "$label $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/r06_bench_${label}_$i.log | head -1) $(grep -o '"den_ms_per_step": [0-9.]*' gpurun_out/ab/r06_bench_${label}_$i.log)"
  done
done
