#!/bin/bash
# A/B/A/B of a presence-switched knob (set vs unset) on bench.py --no-prof --no-extra,
# 5 steps, with rocprofv3 kernel stats per run; usage: scripts/ab_presence.sh VAR [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
var=$1; shift
for v in on off on2 off2; do
  if [ "${v#on}" != "$v" ]; then export $var=1; else unset $var; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp/$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra "$@" > gpurun_out/abp/$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp/$v.log | head -1)"
done
