#!/bin/bash
# round 3 call i (session 2 checkpoint): full GPU suite, the driver's bench command, kernel-trace summary of C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3i.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3i.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3i.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r3i.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3i_c4.log 2> gpurun_out/bench_r3i_c4.err; rc=$?
echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_r3i_c4.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3i_c4.err; exit $rc; }
exit 0
