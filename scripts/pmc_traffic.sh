#!/bin/bash
# HBM traffic per kernel class from rocprofv3 PMC counters, collected as
# MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots prescribe: FETCH_SIZE and
# WRITE_SIZE in separate passes (they do not fit one TCC pass), kernel trace only,
# FETCH_SIZE doubled on gfx950. Writes gpurun_out/pmc/traffic.json; copy it to
# profiles/ to have bench.py report it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-prof --no-extra"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/fetch -o run -- $CMD > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/write -o run -- $CMD > gpurun_out/pmc/write.log 2>&1 || exit $?
python3 scripts/pmc_summarize.py gpurun_out/pmc > gpurun_out/pmc/traffic.json && cat gpurun_out/pmc/traffic.json
