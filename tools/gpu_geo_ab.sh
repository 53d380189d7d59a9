#!/bin/bash
# A/B of geometry library builds (ab/lib_<tag>.so): PQ-scene bit-identity of every build against
# the first, then the C5 / C3 bench lines with their per-phase times.
#   TAGS="h0s0 h50s1 h50s1+AA_CP_QUEUE=0" CFGS="c5 c3" bash tools/gpu_geo_ab.sh
# (a tag `lib+VAR=val` runs ab/lib_<lib>.so with VAR=val in the environment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
envof() { case $1 in *+*) echo "${1#*+}";; esac; }
set -- $TAGS; base=$1
for v in $TAGS; do
  env $(envof $v) AA_ADMM_LIB=$PWD/ab/lib_${v%%+*}.so timeout -k 10 120 python -u tools/ab_dump.py gpurun_out/ab_pq_$v.npz ${DUMP:-pq} > gpurun_out/ab_pq_$v.log 2>&1 || { echo "dump $v failed"; tail -5 gpurun_out/ab_pq_$v.log; exit 1; }
  [ $v != $base ] && { echo -n "$v vs $base: "; python tools/ab_dump.py --compare gpurun_out/ab_pq_$base.npz gpurun_out/ab_pq_$v.npz || exit 1; }
done
for cfg in ${CFGS:-c5 c3}; do
  for v in $TAGS; do
    env $(envof $v) AA_ADMM_LIB=$PWD/ab/lib_${v%%+*}.so timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0 > gpurun_out/ab_${cfg}_$v.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench $cfg $v rc=$rc"; tail -5 gpurun_out/ab_${cfg}_$v.log; exit $rc; }
    python - $cfg $v gpurun_out/ab_${cfg}_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[1], sys.argv[2], "value", d["value"], "phases", d["roofline"].get("phase_us_per_iter"))
PY
  done
done
exit 0
