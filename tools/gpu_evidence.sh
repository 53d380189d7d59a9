#!/bin/bash
# Round evidence: GPU parity suite, every config's bench line (with its CPU baseline), a rocprofv3
# kernel trace + stats of C4, the FETCH_SIZE / WRITE_SIZE passes of C4, and the partitioned bench
# path with 2 ranks on this one GPU (host transport). Each step has its own limit; a failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
TAG=${TAG:-r2}
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2"; exit $1;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; fatal $rc pytest
fi
for cfg in ${CFGS:-c4 c2 c3 c5}; do
  timeout -k 10 600 python -u bench.py --config $cfg > gpurun_out/bench_${TAG}_$cfg.log 2>&1; rc=$?
  echo "bench $cfg rc=$rc"; grep -h '^{' gpurun_out/bench_${TAG}_$cfg.log | cut -c1-160; fatal $rc bench-$cfg
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --partition host --same-device --steps 2 --warmup 1 --no-secondary --eps-steps 1 > gpurun_out/bench_${TAG}_part2.log 2>&1; rc=$?
echo "bench part2 rc=$rc"; grep -h '^{' gpurun_out/bench_${TAG}_part2.log | cut -c1-200; fatal $rc bench-part2
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_c4" -o run -- python3 "$R/bench.py" --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --eps-steps 0 > "$R/gpurun_out/prof_${TAG}_c4.log" 2>&1; rc=$?
echo "prof c4 rc=$rc"; fatal $rc prof-c4
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
cd "$R" && TAG=$TAG CFG=c4 bash tools/gpu_pmc.sh; rc=$?; fatal $rc pmc
exit 0
