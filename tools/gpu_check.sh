#!/bin/bash
# One GPU session: GPU tests, bench, rocprofv3 kernel-trace summary. Each GPU step runs under
# its own time limit; a fault / abort / timeout (rc 124, 134, 137, 139) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench_rc=$rc"; tail -2 gpurun_out/bench.log; fatal $rc bench
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1; rc=$?
  echo "prof_rc=$rc"; fatal $rc rocprof
fi
