#!/bin/bash
# Issue / MFMA / LDS counters per kernel class, one rocprofv3 --pmc pass (8 SQ + 1 GRBM
# slots, MI355X_MICROARCH.md §rocprofv3 PMC slots), kernel trace only, the program
# directly after --. Writes gpurun_out/pmc_util/util.json (scripts/pmc_util_summarize.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_util
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-prof --no-extra $*"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/pmc_util/run -o run -- $CMD > gpurun_out/pmc_util/run.log 2>&1 || exit $?
python3 scripts/pmc_util_summarize.py gpurun_out/pmc_util/run > gpurun_out/pmc_util/util.json && cat gpurun_out/pmc_util/util.json
