#!/bin/bash
# VALU-side counters of the local step (the hyperelastic prox is compute-bound):
# two SQ passes (at most 8 SQ counters each) over a short eager C4 run; per-kernel rows in the CSV.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c4}; TAG=${TAG:-valu}
cd /tmp && export TMPDIR=/tmp
PASS_A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS GRBM_GUI_ACTIVE"
PASS_B="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
i=0
for P in "$PASS_A" "$PASS_B"; do
  i=$((i + 1))
  AA_ADMM_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$i" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --iters ${ITERS:-10} --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/pmc_${TAG}_${CFG}_$i.log" 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_${TAG}_${CFG}_$i.log"; exit $rc; }
done
exit 0
