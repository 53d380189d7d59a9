#!/bin/bash
# Round-6 measurement run: the default bench line (as the driver runs it), the rho0 variant test,
# a kernel-trace profile of C4 and the two HBM-traffic --pmc passes (tools/gpu.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err; rc=$?
cut -c1-400 gpurun_out/bench_default.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_default.err; exit $rc; }
bash tools/gpu.sh "tests rho0_variant" "prof c4 r6" "pmc c4 r6 FETCH_SIZE;WRITE_SIZE"
