#!/bin/bash
# rocprofv3 kernel summaries of the 3072 model's train step, fp16 and MXFP8 forward,
# 5 timed steps each (bench.py --no-prof --no-extra). usage: scripts/fp8_prof.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-fp8}
mkdir -p gpurun_out/prof gpurun_out/r04
export TMPDIR=/tmp
for v in fp16 fp8; do
  f=""; [ $v = fp8 ] && f=--fp8
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${tag}_$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra --xconfig cnn_tdnn_17f_3072.xconfig $f \
    > gpurun_out/r04/${tag}_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/r04/${tag}_$v.log | cut -c1-200
done
