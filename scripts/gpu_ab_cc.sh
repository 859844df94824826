# GPU tests named in $TESTS (default: the row-subsampling, data-parallel, network, stream-order,
# lifecycle and train-step tests), a same-box A/B of $VARIANTS, and one step's launches
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cc && \
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_row_subsampling.py tests/test_gpu_dp.py tests/test_gpu_nnet.py tests/test_gpu_wgrad_order.py tests/test_gpu_lifecycle.py tests/test_gpu_train_step.py} > gpurun_out/cc/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/cc/tests.txt; [ $rc = 0 ] && \
VARIANTS="${VARIANTS:-head@ab_r6b cur}" bash scripts/r06_ab.sh 2 && \
timeout -k 10 200 python3 scripts/step_launches.py --rsub --one-stream > gpurun_out/cc/launches.txt 2>&1; grep -n "halo\|#" gpurun_out/cc/launches.txt | head -40
