# the default bench's per-step times (first timed steps after the warm-up), two runs
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fs && \
for i in 1 2; do timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > gpurun_out/fs/def$i.log 2>&1 || exit 1; python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/fs/def$i.log') if x.startswith('{\"metric\"')][0]; print('default', l['value'], l['ms_per_step'], l['ms_per_step_mean'], l['step_ms'][:4], l.get('hip_pending_log'))"; done
