# first timed steps: warm-up length and the copy engine
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wp && \
run() { n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/wp/$n.log 2>&1 || exit 1; python3 -c "import json; l=[json.loads(x) for x in open('gpurun_out/wp/$n.log') if x.startswith('{\"metric\"')][0]; print('$n', l['ms_per_step'], l['ms_per_step_mean'], l['step_ms'][:6])"; }
run w3 python3 bench.py --no-extra --no-cpu-baseline --no-prof --warmup 3 --steps 12
run w10 python3 bench.py --no-extra --no-cpu-baseline --no-prof --warmup 10 --steps 12
run noh2d python3 bench.py --no-extra --no-cpu-baseline --no-prof --warmup 3 --steps 12 --no-h2d
HSA_ENABLE_SDMA=0 run nosdma python3 bench.py --no-extra --no-cpu-baseline --no-prof --warmup 3 --steps 12
