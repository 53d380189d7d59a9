#!/bin/bash
# Round 3 (late): backward tiles -- ab/lib_nar.so (narrow <= 64-column blocks, padding lanes masked)
# and ab/lib_tri.so (+ zero upper triangle skipped) against ab/lib_head.so: bit-identity of
# lib_tri on four scenes, then C4 (three-way) and C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in $2; stopping"; exit $1;; esac; }
for sc in drop40 c4small pq cloth; do
  for l in head tri; do
    AA_ADMM_LIB=$PWD/ab/lib_$l.so timeout -k 10 300 python tools/ab_dump.py gpurun_out/ab_${sc}_$l.npz $sc > gpurun_out/abd_${sc}_$l.log 2>&1; fatal $? "ab_dump $sc $l"
  done
  echo -n "$sc tri: "; python tools/ab_dump.py --compare gpurun_out/ab_${sc}_head.npz gpurun_out/ab_${sc}_tri.npz
done
LIBS="ab/lib_head.so ab/lib_nar.so ab/lib_tri.so ab/lib_head.so ab/lib_nar.so ab/lib_tri.so" CFG=c4 bash tools/gpu_ab.sh; fatal $? "ab c4"
LIBS="ab/lib_head.so ab/lib_nar.so ab/lib_tri.so ab/lib_head.so ab/lib_nar.so ab/lib_tri.so" CFG=c3 bash tools/gpu_ab.sh; fatal $? "ab c3"
# + forward tiles: padding rows load nothing, zero upper triangle skipped per lane (ab/lib_fwd.so)
if [ -f ab/lib_fwd.so ]; then
  for sc in drop40 pq; do
    AA_ADMM_LIB=$PWD/ab/lib_fwd.so timeout -k 10 300 python tools/ab_dump.py gpurun_out/ab_${sc}_fwd.npz $sc > gpurun_out/abd_${sc}_fwd.log 2>&1; fatal $? "ab_dump $sc fwd"
    echo -n "$sc fwd: "; python tools/ab_dump.py --compare gpurun_out/ab_${sc}_head.npz gpurun_out/ab_${sc}_fwd.npz
  done
  LIBS="ab/lib_tri.so ab/lib_fwd.so ab/lib_tri.so ab/lib_fwd.so" CFG=c4 bash tools/gpu_ab.sh; fatal $? "ab c4 fwd"
fi
