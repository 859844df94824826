#!/bin/bash
# Round-6 evidence on one GPU box (outputs under gpurun_out/r06e/, copied into profiles/ by hand):
#   scripts/r06_evidence.sh A -> full GPU suite, the default bench line, and a rocprofv3 kernel
#                                trace of exactly the driver's command (`python3 bench.py`) with
#                                the fused-class check of its timed window
#   scripts/r06_evidence.sh B -> PMC HBM traffic and utilisation passes, step timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r06e
mkdir -p $out
case "$1" in
A)
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
      > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
  tail -3 $out/gpu_tests.txt
  timeout -k 10 400 python3 bench.py > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
  python3 scripts/bench_summary.py $out/bench_default.log | head -3
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
      python3 bench.py > $out/bench_rocprof.log 2>&1 || { tail -20 $out/bench_rocprof.log; exit 1; }
  tr=$(ls $out/prof/*/run_kernel_trace.csv 2>/dev/null || ls $out/prof/run_kernel_trace.csv)
  python3 scripts/fused_class_check.py $tr $out/bench_rocprof.log > $out/fused_class_check.json || exit 1
  cat $out/fused_class_check.json
  gzip -f $tr
  ;;
B)
  scripts/pmc_traffic.sh > /dev/null && cp gpurun_out/pmc/traffic.json $out/pmc_traffic.json || exit 1
  scripts/pmc_util.sh > /dev/null && cp gpurun_out/pmc_util/util.json $out/pmc_util.json || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tl -o run -- \
      python3 bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 2 > $out/tl_bench.log 2>&1 || exit 1
  python3 scripts/step_timeline.py $(ls $out/tl/*/run_kernel_trace.csv 2>/dev/null || ls $out/tl/run_kernel_trace.csv) \
      > $out/step_timeline.txt || exit 1
  tail -12 $out/step_timeline.txt
  ;;
esac
