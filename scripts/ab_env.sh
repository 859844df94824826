#!/bin/bash
# A/B a kernel-selection env knob under rocprofv3: scripts/ab_env.sh VAR v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
var=$1; shift
for v in "$@"; do
  env $var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$var$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof > gpurun_out/ab/$var$v.log 2>&1 || exit $?
  echo "$var=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$var$v.log)"
done
