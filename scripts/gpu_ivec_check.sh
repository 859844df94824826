# row-subsampling parity (incl. the ivector topology), the ivector config's bench, and the
# default bench's per-step times
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/iv && \
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_row_subsampling.py > gpurun_out/iv/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/iv/tests.txt; [ $rc = 0 ] && \
timeout -k 10 300 python3 bench.py --xconfig cnn_tdnn_17f_ivec.xconfig --no-extra --no-cpu-baseline > gpurun_out/iv/ivec.log 2>&1 && \
python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/iv/ivec.log') if x.startswith('{\"metric\"')][0]; print('ivec', l['value'], l['ms_per_step'], l['config']['rows'][:20], l['objf_per_frame'])" && \
for i in 1 2; do timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > gpurun_out/iv/def$i.log 2>&1 || exit 1; python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/iv/def$i.log') if x.startswith('{\"metric\"')][0]; print('default', l['value'], l['ms_per_step'], l['step_ms'][:4], l.get('hip_pending_log'))"; done
