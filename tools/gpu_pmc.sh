#!/bin/bash
# HBM traffic of the dominant kernels (MI355X_MICROARCH.md HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE
# in separate passes -- TCC slots; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950).
# Round 2: the profiled process crashed under --pmc (SIGSEGV in the host launch path, three runs, with
# and without the GPU setup factor -- AA_DENSE_GPU); bench.py then reads the round-1 passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c4}; TAG=${TAG:-r1}
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  AA_ADMM_NO_GRAPH=1 timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --iters ${ITERS:-10} --no-cpu-baseline > "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr.log" 2>&1; rc=$?
  echo "$ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_${TAG}_${CFG}_$ctr.log"; exit $rc; }
done
ls -R "$R/gpurun_out/pmc_${TAG}_${CFG}_FETCH_SIZE" | head
exit 0
