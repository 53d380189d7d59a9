#!/bin/bash
# HBM traffic of the dominant kernels (MI355X_MICROARCH.md HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE
# in separate passes -- TCC slots; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950).
# GRAPH=1 (default) profiles the production path (the step replayed as one hipGraph); GRAPH=0 launches
# eagerly (AA_ADMM_NO_GRAPH=1; round 2's eager FETCH_SIZE passes crashed the profiled process).
# AA_DUMP_MAPS writes the process's library map next to the log (resolves a crash's frames).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c4}; TAG=${TAG:-r3}; CTRS=${CTRS:-FETCH_SIZE WRITE_SIZE}
cd /tmp && export TMPDIR=/tmp
EAGER=""; [ "${GRAPH:-1}" = "0" ] && EAGER="AA_ADMM_NO_GRAPH=1"
for ctr in $CTRS; do
  export AA_DUMP_MAPS="$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr.maps"
  [ -n "$EAGER" ] && export AA_ADMM_NO_GRAPH=1
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --iters ${ITERS:-10} --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr.log" 2>&1; rc=$?
  echo "$ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr.log"; exit $rc; }
done
ls -R "$R/gpurun_out/pmc_${TAG}_${CFG}_FETCH_SIZE" | head
exit 0
