#!/bin/bash
# Partitioned-solver rehearsals on ONE GPU: (1) C4 over 2 ranks sharing the GPU through the
# host transport; (2) C4 on a one-rank RCCL communicator under torchrun (torch imported, gloo
# rendezvous) -- the exact RCCL code path of an N-GPU run with an identity all-reduce.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-c4}; EXTRA=${EXTRA:-}
run() {  # name, nproc, args...
  local name=$1 np=$2; shift 2
  timeout -k 10 ${T:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node=$np --master-addr=127.0.0.1 \
    --master-port=$((29500 + RANDOM % 1000)) bench.py --config $CFG --no-cpu-baseline $EXTRA "$@" > gpurun_out/part_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep -h '^{' gpurun_out/part_$name.log | cut -c1-900
  case $rc in 0) ;; *) tail -20 gpurun_out/part_$name.log; exit $rc;; esac
}
run rccl1 1 --partition rccl --steps 3 --warmup 1
run host2 2 --partition host --same-device --steps 2 --warmup 1
