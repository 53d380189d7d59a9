#!/bin/bash
# Wave-state split (issuing / parked on waitcnt / issue-stalled) per kernel for each library in LIBS
# (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES), one SQ pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c4}
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  tag=$(basename "$lib" .so)
  AA_ADMM_LIB="$R/$lib" AA_ADMM_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/stall_${CFG}_$tag" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --iters ${ITERS:-10} --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/stall_${CFG}_$tag.log" 2>&1; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/stall_${CFG}_$tag.log"; exit $rc; }
done
exit 0
