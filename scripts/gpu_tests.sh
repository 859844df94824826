#!/bin/bash
# The GPU test suite on the box, one pytest process, per-test time limits.
# usage: scripts/gpu_tests.sh <log name> [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
log=gpurun_out/r04/$1.log
shift
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > "$log" 2>&1
rc=$?
tail -5 "$log"
exit $rc
