# default bench line (its hip_pending_log) and the per-class launch sums of one step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bd && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bd/bench.log 2>&1; rc=$?; grep -o '"hip_pending_log": "[^"]*"' gpurun_out/bd/bench.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bd/bench.log | head -1; [ $rc = 0 ] && \
timeout -k 10 200 python3 scripts/step_launches.py --rsub > gpurun_out/bd/launches.txt 2>&1; grep -E "c1|# " gpurun_out/bd/launches.txt | head; tail -8 gpurun_out/bd/launches.txt
