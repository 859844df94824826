#!/bin/bash
# GPU tests on the box, one pytest process, per-test limits: scripts/r05_tests.sh <log> [pytest args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
log=gpurun_out/r05/$1.log; shift
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > "$log" 2>&1
rc=$?
tail -4 "$log"
exit $rc
