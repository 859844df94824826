#!/bin/bash
# PMC passes over the chain kernels (den_g_sweep child): L2 hit/miss, wave stall
# buckets, LDS bank conflicts. One counter group per pass, kernel trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcden
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcden/p$i -o run -- python3 scripts/den_g_sweep.py child > gpurun_out/pmcden/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcden/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob("gpurun_out/pmcden/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for key in ("k_den_fwd", "k_den_bwd", "k_den_post", "k_num_fb"):
            if key in k:
                agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[key][r["Counter_Name"]] += 1
for k, d in agg.items():
    print(k, {c: round(v / max(cnt[k][c], 1), 1) for c, v in sorted(d.items())})
PY
