#!/bin/bash
# A/B of GEMM tile families within one box: KF_GEMM_BIG=0 (128-wide, 4 waves),
# 1 (256x256, 8 waves), 2 (256x128, 8 waves). Each setting: kernel parity
# tests, the micro-benchmark, then a short bench.py.
set -e
mkdir -p gpurun_out/ab
for big in ${BIGS:-1 2 0}; do
  export KF_GEMM_BIG=$big
  timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/ab/test_$big.log 2>&1
  timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/ab/gemm_$big.log 2>&1
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/ab/bench_$big.log 2>&1
  echo "big=$big done"; tail -1 gpurun_out/ab/bench_$big.log | cut -c1-200
done
