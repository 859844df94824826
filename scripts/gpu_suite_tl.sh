# full GPU suite, then a kernel trace of 3 headline steps and its per-stream timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/st && export TMPDIR=/tmp && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/st/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/st/tests.txt; [ $rc = 0 ] && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st/tl -o run -- python3 bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/st/tl_bench.log 2>&1 && \
python3 scripts/step_timeline.py $(ls gpurun_out/st/tl/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/st/tl/run_kernel_trace.csv) > gpurun_out/st/step_timeline.txt && cat gpurun_out/st/step_timeline.txt
