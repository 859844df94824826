#!/bin/bash
# A/B of in-tree builds under rocprofv3: scripts/ab_lib.sh <libdir> [<libdir> ...]
# (KFP16_LIBDIR selects the build; each run: kernel stats of a short bench.py; list a
# directory twice, e.g. A B A B, to see the run-to-run spread; BENCH_ARGS adds bench flags)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
i=0
for d in "$@"; do
  i=$((i+1))
  tag=$(basename "$d")_$i
  KFP16_LIBDIR=$(realpath "$d") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra $BENCH_ARGS > gpurun_out/ab/$tag.log 2>&1 || exit $?
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$tag.log)"
done
