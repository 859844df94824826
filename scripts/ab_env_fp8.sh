#!/bin/bash
# A/B of an environment switch on the 3072 MXFP8 train step (bench.py --no-prof --no-extra,
# 5 steps), A/B/A/B; usage: scripts/ab_env_fp8.sh VAR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abf8
var=$1
for v in on off on2 off2; do
  if [ "${v#on}" != "$v" ]; then export $var=1; else unset $var; fi
  timeout -k 10 240 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra \
    --xconfig cnn_tdnn_17f_3072.xconfig --fp8 > gpurun_out/abf8/$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abf8/$v.log | head -1)"
done
