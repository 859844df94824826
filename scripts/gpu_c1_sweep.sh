# k_conv_c1_wgrad time per workgroup count (rocprofv3 kernel stats of 3 train steps)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c1 && export TMPDIR=/tmp
for nb in 2048 768 1536 4096; do
  KF_C1_NBLK=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1/n$nb -o run -- python3 scripts/step_launches.py --rsub --quiet --steps 3 > gpurun_out/c1/n$nb.log 2>&1 || exit 1
  echo "nblk $nb: $(grep -h c1_wgrad $(ls gpurun_out/c1/n$nb/*/run_kernel_stats.csv gpurun_out/c1/n$nb/run_kernel_stats.csv 2>/dev/null) | cut -d, -f2-4)"
done
