#!/bin/bash
# Round-6 final measurements: GPU suite, smoke, kernel-trace profile of C4, the default bench line
# and the other configs' lines (tools/gpu.sh steps; logs under gpurun_out/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
bash tools/gpu.sh tests smoke "prof c4 r6" || exit $?
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err; rc=$?
cut -c1-300 gpurun_out/bench_default.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_default.err; exit $rc; }
bash tools/gpu.sh "bench c3 5 1" "bench c5 5 1" "bench c2 20 5"
