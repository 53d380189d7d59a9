#!/bin/bash
# round 3 call b: WRITE_SIZE pass (graph mode), the C4 bench with the new run-to-eps legs, then
# the round-2 eager FETCH_SIZE crash reproduced once with the library map dumped (last: it ends the call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
CTRS=WRITE_SIZE bash tools/gpu_pmc.sh || exit $?
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r3b_c4.log 2> gpurun_out/bench_r3b_c4.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_r3b_c4.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3b_c4.err; exit $rc; }
GRAPH=0 TAG=r3eager CTRS=FETCH_SIZE bash tools/gpu_pmc.sh; echo "eager pmc rc=$?"
exit 0
