#!/bin/bash
# A/B of an env knob under rocprofv3: scripts/ab_env.sh VAR valA valB [bench args]
# (one in-tree build; each run: kernel stats of a short bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
var=$1; va=$2; vb=$3; shift 3
for v in "$va" "$vb"; do
  tag=${var}_$v
  env "$var=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra "$@" > gpurun_out/ab/$tag.log 2>&1 || exit $?
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$tag.log)"
done
