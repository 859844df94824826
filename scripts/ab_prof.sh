cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/abd
i=0
for d in ab/A ab/D ab/A ab/D; do
  i=$((i+1)); tag=$(basename $d)_$i
  KFP16_LIBDIR=$(realpath $d) timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/abd/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/abd/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], d['chain']['den_ms_per_step'])"
done
