# GPU tests named in $TESTS, then a same-box A/B of $VARIANTS (scripts/r06_ab.sh tokens)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cc && \
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_row_subsampling.py} > gpurun_out/cc/tests.txt 2>&1; rc=$?; tail -2 gpurun_out/cc/tests.txt; [ $rc = 0 ] && \
bash scripts/r06_ab.sh ${REPS:-2}
