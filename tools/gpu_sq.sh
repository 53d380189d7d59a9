#!/bin/bash
# One SQ counter pass over a short C4 run (eager launches): LDS bank conflicts and wave stall
# breakdown per kernel (MI355X_MICROARCH.md PMC table: at most 8 SQ counters per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c4}; TAG=${TAG:-sq}
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --iters 10 --no-cpu-baseline > "$R/gpurun_out/pmc_${TAG}_${CFG}.log" 2>&1; rc=$?
echo "sq rc=$rc"; [ $rc -ne 0 ] && tail -5 "$R/gpurun_out/pmc_${TAG}_${CFG}.log"
exit $rc
