# quick GPU check: the full GPU suite (or the files given in $TESTS), a headline bench line
# without sub-results, and the per-class launch sums of one row-subsampled step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cc && \
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/cc/tests.txt 2>&1; rc=$?; tail -5 gpurun_out/cc/tests.txt; [ $rc = 0 ] && \
timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/cc/bench.log 2>&1 && python3 scripts/bench_summary.py gpurun_out/cc/bench.log > gpurun_out/cc/sum.txt; grep -o '"hip_pending_log[^}]*' gpurun_out/cc/bench.log; head -3 gpurun_out/cc/sum.txt; \
timeout -k 10 200 python3 scripts/step_launches.py --rsub --one-stream --quiet > gpurun_out/cc/launches.txt 2>&1; tail -6 gpurun_out/cc/launches.txt
