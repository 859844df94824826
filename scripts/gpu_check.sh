#!/bin/bash
# One gpurun session: GPU parity tests, a short bench, a rocprofv3 kernel-stats
# profile. Every GPU step has its own time limit; a crash / fault / timeout
# (exit >= 124 or signal) ends the script, plain test failures (rc 1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 900 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = slow ]; then
    step pytest_gpu_slow 900 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 300 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3}
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra
fi
echo "== done"
