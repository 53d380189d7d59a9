#!/bin/bash
# C4 bench with and without the hipGraph, then a rocprofv3 kernel-trace summary (eager launches:
# the 100-iteration C4 graph crashed rocprofv3's kernel tracer).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
TAG=${TAG:-c4}
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_graph.log 2>&1; rc=$?
echo "graph rc=$rc"; grep -h '^{' gpurun_out/bench_${TAG}_graph.log | cut -c1-400; fatal $rc bench-graph
AA_ADMM_NO_GRAPH=1 timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_eager.log 2>&1; rc=$?
echo "eager rc=$rc"; grep -h '^{' gpurun_out/bench_${TAG}_eager.log | cut -c1-400; fatal $rc bench-eager
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --config c4 --steps 1 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc rocprof
f=$(ls "$R"/gpurun_out/prof_$TAG/*/run_kernel_stats.csv "$R"/gpurun_out/prof_$TAG/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && head -30 "$f" | cut -c1-200
exit 0
