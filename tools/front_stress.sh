#!/bin/bash
# tools/front_stress.hip on the GPU (see its header): the backend's sequence alone, then each
# library call alone, with 1, 2 and 4 processes on the GPU at once, and one checking process beside
# a non-library aggressor.
#   /usr/local/graft/bin/gpurun -- bash tools/front_stress.sh [rounds] [f] [p]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
R=${1:-30}; F=${2:-2844}; P=${3:-1422}
X=tools/bin/front_stress
for mode in ${MODES:-full potrf gemm}; do
  for np in 1 2 4; do
    echo "== $mode, $np process(es)"
    pids=()
    for k in $(seq 1 $np); do timeout -k 10 300 $X $R $F $P $k $mode > gpurun_out/stress_${mode}_${np}_$k.log 2>&1 & pids+=($!); done
    for pid in "${pids[@]}"; do wait $pid; done
    tail -q -n 1 gpurun_out/stress_${mode}_${np}_*.log; grep -h -m1 "max relative" gpurun_out/stress_${mode}_${np}_*.log | head -2
  done
done
echo "== full beside a streaming-copy aggressor (no library calls)"
timeout -k 10 300 $X $((R * 10)) $F $P 9 noise > gpurun_out/stress_noise.log 2>&1 &
na=$!
timeout -k 10 300 $X $R $F $P 1 full > gpurun_out/stress_victim.log 2>&1
wait $na
tail -n 1 gpurun_out/stress_noise.log gpurun_out/stress_victim.log; grep -m1 "max relative" gpurun_out/stress_victim.log
