cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/cfg
run() { name=$1; shift; timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra "$@" > gpurun_out/cfg/$name.log 2>&1 || exit $?; echo "$name $(tail -1 gpurun_out/cfg/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
run fwd --mode forward
run ivec --xconfig cnn_tdnn_17f_ivec.xconfig
run kaldi --xconfig cnn_tdnn_17f_kaldi.xconfig
run att --xconfig cnn_tdnn_17f_att.xconfig
run m3072 --xconfig cnn_tdnn_17f_3072.xconfig
run m3072fwd8 --xconfig cnn_tdnn_17f_3072.xconfig --mode forward --fp8
run m3072fp8 --xconfig cnn_tdnn_17f_3072.xconfig --fp8
