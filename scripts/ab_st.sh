set -e
mkdir -p gpurun_out/st
for st in 2 3 4; do
  export KF_GEMM_ST=$st
  timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/st/gemm_$st.log 2>&1
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/st/bench_$st.log 2>&1
  echo "st=$st"; grep -v amdgpu gpurun_out/st/gemm_$st.log; tail -1 gpurun_out/st/bench_$st.log | cut -c1-190
done
