# A/B of GEMM knobs on the GPU box: parity under each knob set, gemm microbench, bench step.
# usage: bash scripts/ab_run.sh "ENV1=.. ENV2=.." "ENV=.." ...   (first arg "" = defaults)
set -e
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "== [$i] $cfg"
  env $cfg timeout -k 10 240 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_$i.log 2>&1 || { tail -30 gpurun_out/ab/pytest_$i.log; exit 1; }
  tail -1 gpurun_out/ab/pytest_$i.log
  env $cfg timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/ab/gemm_$i.log 2>&1
  grep -v amdgpu gpurun_out/ab/gemm_$i.log
  env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_$i.log 2>&1
  tail -1 gpurun_out/ab/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d['chain'])"
done
