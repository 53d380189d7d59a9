#!/bin/bash
# Round checkpoint: full GPU test suite, then every config's bench line (with its CPU baseline),
# then rocprofv3 kernel-trace summaries of C4 and C2 (eager launches). Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
TAG=${TAG:-r1}
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; fatal $rc pytest
fi
for cfg in ${CFGS:-c4 c2 c3 c5}; do
  timeout -k 10 600 python -u bench.py --config $cfg > gpurun_out/bench_${TAG}_$cfg.log 2>&1; rc=$?
  echo "bench $cfg rc=$rc"; grep -h '^{' gpurun_out/bench_${TAG}_$cfg.log | cut -c1-200; fatal $rc bench-$cfg
done
cd /tmp && export TMPDIR=/tmp
for cfg in ${PROF_CFGS:-c4 c2}; do
  AA_ADMM_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_$cfg" -o run -- python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_${TAG}_$cfg.log" 2>&1; rc=$?
  echo "prof $cfg rc=$rc"; fatal $rc prof-$cfg
done
exit 0
