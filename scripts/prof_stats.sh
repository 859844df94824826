#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench step (7 timed steps).
# usage: scripts/prof_stats.sh <name> [bench args...]  ->  gpurun_out/prof/<name>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1
shift
mkdir -p gpurun_out/prof/$name
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$name -o run -- \
    python3 bench.py --steps 7 --warmup 2 --no-cpu-baseline --no-extra --no-prof "$@" > gpurun_out/prof/$name/bench.log 2>&1
rc=$?
tail -c 600 gpurun_out/prof/$name/bench.log
exit $rc
