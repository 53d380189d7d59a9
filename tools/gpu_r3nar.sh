#!/bin/bash
# Round 3 (late): narrow backward tiles -- GPU tests + smoke on the in-tree build, bit-identity of
# ab/lib_nar.so against ab/lib_head.so on four scenes, C4 / C5 / C3 A/B, then a fused-subtree sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2; stopping"; exit $1;; esac; }
bash tools/gpu_tests.sh; fatal $? pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; fatal $rc smoke
for sc in drop40 c4small pq cloth; do
  for l in head nar; do
    AA_ADMM_LIB=$PWD/ab/lib_$l.so timeout -k 10 300 python tools/ab_dump.py gpurun_out/ab_${sc}_$l.npz $sc > gpurun_out/abd_${sc}_$l.log 2>&1; fatal $? "ab_dump $sc $l"
  done
  echo -n "$sc: "; python tools/ab_dump.py --compare gpurun_out/ab_${sc}_head.npz gpurun_out/ab_${sc}_nar.npz
done
for cfg in c4 c5 c3; do
  LIBS="ab/lib_head.so ab/lib_nar.so ab/lib_head.so ab/lib_nar.so" CFG=$cfg bash tools/gpu_ab.sh; fatal $? "ab $cfg"
done
BENCH_ARGS="--eps-steps 0 --no-secondary" SWEEP="AA_SOLVE_MIN_SUBTREES=512,AA_SUB_BLOCK=512 AA_SOLVE_MIN_SUBTREES=512,AA_SUB_BLOCK=1024 AA_SUB_BLOCK=512 AA_SOLVE_MIN_SUBTREES=256" bash tools/gpu_sweep.sh
