#!/bin/bash
# bench.py + rocprofv3 kernel-trace summary for one config (each GPU step under its own limit).
#   CFG=c3 TAG=r1_c3 bash tools/gpu_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c2}; TAG=${TAG:-$CFG}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit $1;; esac; }
timeout -k 10 ${T:-600} python -u bench.py --config $CFG ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1; rc=$?
echo "bench_rc=$rc"; tail -3 gpurun_out/bench_$TAG.log; fatal $rc bench
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  AA_ADMM_NO_GRAPH=${PROF_NO_GRAPH:-0} timeout -k 10 ${T:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS} > "$R/gpurun_out/prof_$TAG.log" 2>&1; rc=$?
  echo "prof_rc=$rc"; fatal $rc rocprof
  f=$(ls "$R"/gpurun_out/prof_$TAG/*/run_kernel_stats.csv "$R"/gpurun_out/prof_$TAG/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && head -25 "$f" | cut -c1-220
fi
exit 0
