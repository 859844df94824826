cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for big in 1 0; do
KF_GEMM_BIG=$big timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/big$big -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof > gpurun_out/ab/big$big.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/big$big.log
done
