#!/bin/bash
# Round 3 (late), one box: bit-identity of ab/lib_tri.so (narrow backward tiles + their zero upper
# triangle skipped) and ab/lib_fwd.so (+ forward tiles' padding rows / upper triangle skipped)
# against ab/lib_head.so, the C4 A/B of head / nar / tri / fwd, then the GPU suite + smoke on the
# in-tree build (= fwd).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2; stopping"; exit $1;; esac; }
for sc in drop40 pq; do
  for l in head tri fwd; do
    AA_ADMM_LIB=$PWD/ab/lib_$l.so timeout -k 10 300 python tools/ab_dump.py gpurun_out/ab_${sc}_$l.npz $sc > gpurun_out/abd_${sc}_$l.log 2>&1; fatal $? "ab_dump $sc $l"
  done
  for l in tri fwd; do echo -n "$sc $l: "; python tools/ab_dump.py --compare gpurun_out/ab_${sc}_head.npz gpurun_out/ab_${sc}_$l.npz; done
done
LIBS="ab/lib_head.so ab/lib_nar.so ab/lib_tri.so ab/lib_fwd.so ab/lib_head.so ab/lib_nar.so ab/lib_tri.so ab/lib_fwd.so" CFG=c4 bash tools/gpu_ab.sh; fatal $? "ab c4"
T=500 bash tools/gpu_tests.sh > gpurun_out/tests_r3nar3.txt 2>&1; rc=$?; tail -3 gpurun_out/tests_r3nar3.txt; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; fatal $rc smoke
