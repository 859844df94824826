# full GPU suite, then the first-step probe and the Kaldi-topology bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fc && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/fc/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/fc/tests.txt; [ $rc = 0 ] && \
run() { n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/fc/$n.log 2>&1 || exit 1; python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/fc/$n.log') if x.startswith('{\"metric\"')][0]; print('$n', l['value'], l['ms_per_step'], l['ms_per_step_mean'], l['step_ms'][:5], l['config'].get('rows','')[:14], l.get('hip_pending_log'))"; } && \
run w5 python3 bench.py --no-extra --no-cpu-baseline --warmup 5 --steps 20 && \
run kaldi python3 bench.py --no-extra --no-cpu-baseline --xconfig cnn_tdnn_17f_kaldi.xconfig
