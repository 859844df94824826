#!/bin/bash
# A/B of two in-tree builds under rocprofv3: scripts/ab_lib.sh <libdir_a> <libdir_b> [bench args]
# (KFP16_LIBDIR selects the build; each run: kernel stats of a short bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
a=$1; b=$2; shift 2
for d in "$a" "$b"; do
  tag=$(basename "$d")
  KFP16_LIBDIR=$(realpath "$d") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra "$@" > gpurun_out/ab/$tag.log 2>&1 || exit $?
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$tag.log)"
done
