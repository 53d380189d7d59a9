#!/bin/bash
# round 3 call u: non-temporal Anderson history loads (A/B builds), top amalgamation budget (AA_TOP_ROWS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
for sc in drop40 pq; do
  for lib in ant0 ant1; do
    AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 200 python3 tools/ab_dump.py gpurun_out/dump_${sc}_$lib.npz $sc > gpurun_out/dump_${sc}_$lib.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "dump $sc $lib rc=$rc"; tail -5 gpurun_out/dump_${sc}_$lib.log; exit $rc; }
  done
  echo "$sc ant0 vs ant1: $(python3 tools/ab_dump.py --compare gpurun_out/dump_${sc}_ant0.npz gpurun_out/dump_${sc}_ant1.npz)"
done
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c4 c5 c3; do
for v in "ant0" "ant1" "ant1 AA_TOP_ROWS=6500" "ant1 AA_FACTOR_NT_ROWS=0" "ant0" "ant1" "ant1 AA_TOP_ROWS=6500" "ant1 AA_FACTOR_NT_ROWS=0"; do
  set -- $v; lib=$1; shift; tag=$(echo "$v" | tr ' =' '__')_$cfg
  env $@ AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3u_$tag.log 2> gpurun_out/ab_r3u_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3u_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];p=r.get('phase_us_per_iter') or r.get('phase_us_per_launch');print(d['value'],r['avg_launch_us'],r['frac'],'aa',p.get('aa'),'nnz',d['config']['nnz_factor'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3u_$tag.err; exit $rc; }
done; done
exit 0
