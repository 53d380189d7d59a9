#!/bin/bash
# round 3 call e: partition tests (per-part factorization), bunny tests + bench, graph-mode
# kernel traces of the timed steps with and without the work-queue lookahead
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_elastic.py -k "partition or bunny" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_r3e.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --mesh bunny --steps 5 --warmup 1 --no-cpu-baseline --eps-steps 5 --no-secondary > gpurun_out/bench_r3e_bunny.log 2> gpurun_out/bench_r3e_bunny.err; rc=$?
echo "bunny bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3e_bunny.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for ah in 0 1; do
  AA_LQ_AHEAD=$ah timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3e_ah$ah" -o run -- python3 "$R/bench.py" --steps 3 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3e_ah$ah.log" 2>&1; rc=$?
  echo "prof ahead=$ah rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/prof_r3e_ah$ah.log"; exit $rc; }
done
exit 0
