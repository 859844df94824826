# full GPU suite; the split-K fused tiles (KF_SPLITK=2) under the network parity tests; A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sk && export TMPDIR=/tmp && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/sk/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/sk/tests.txt; [ $rc = 0 ] && \
KF_SPLITK=2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_row_subsampling.py tests/test_gpu_nnet.py tests/test_gpu_wgrad_order.py tests/test_gpu_train_step.py > gpurun_out/sk/tests_sk.txt 2>&1; rc=$?; tail -3 gpurun_out/sk/tests_sk.txt; [ $rc = 0 ] && \
REPS=3 VARIANTS="cur sk2%KF_SPLITK=2" bash scripts/r06_ab.sh 3
