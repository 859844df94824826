#!/bin/bash
# Round-5 evidence on one GPU box, in two parts (each well inside gpurun's limit):
#   scripts/r04_evidence.sh A  -> full GPU suite, default bench line, rocprofv3 kernel stats
#   scripts/r04_evidence.sh B  -> PMC utilisation + HBM traffic, drop-in profile, den trace,
#                                 other configurations
# Outputs under gpurun_out/r05e/ (copied into profiles/ by hand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r05e
mkdir -p $out
case "$1" in
A)
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
      > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
  tail -3 $out/gpu_tests.txt
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
  python3 scripts/bench_summary.py $out/bench_default.log | head -3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
      python3 bench.py --no-cpu-baseline --no-extra > $out/bench_rocprof.log 2>&1 || { tail -20 $out/bench_rocprof.log; exit 1; }
  tail -1 $out/bench_rocprof.log | cut -c1-300
  ;;
B)
  scripts/pmc_util.sh > /dev/null && cp gpurun_out/pmc_util/util.json $out/pmc_util.json || exit 1
  scripts/pmc_traffic.sh > /dev/null && cp gpurun_out/pmc/traffic.json $out/pmc_traffic.json || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/dropin -o run -- \
      python3 scripts/dropin_prof.py > $out/dropin.log 2>&1 || exit 1
  grep -o '"dropin_per_op_abi_ms[^,]*' $out/dropin.log
  timeout -k 10 200 python3 scripts/den_trace.py > $out/den_trace.log 2>&1 || exit 1
  scripts/configs_run.sh && cp gpurun_out/cfg/*.log $out/ || exit 1
  ;;
esac
