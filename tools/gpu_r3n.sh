#!/bin/bash
# round 3 call n: whole-workgroup tile reductions -- bit-identity of the A/B builds, C4/C3 A/B, tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
for sc in drop40 c4small pq; do
  for lib in rw0 rw1; do
    AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 200 python3 tools/ab_dump.py gpurun_out/dump_${sc}_$lib.npz $sc > gpurun_out/dump_${sc}_$lib.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "dump $sc $lib rc=$rc"; tail -5 gpurun_out/dump_${sc}_$lib.log; exit $rc; }
  done
  echo "$sc: $(python3 tools/ab_dump.py --compare gpurun_out/dump_${sc}_rw0.npz gpurun_out/dump_${sc}_rw1.npz)"
done
B="--steps 5 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary"
for cfg in c4 c3; do
for lib in rw1 rw0 rw1 rw0; do
  tag=${lib}_$cfg
  AA_ADMM_LIB="$R/ab/lib_$lib.so" timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3n_$tag.log 2> gpurun_out/ab_r3n_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3n_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r.get('phase_us_per_iter') or r.get('phase_us_per_launch'))")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3n_$tag.err; exit $rc; }
done; done
cd /tmp && export TMPDIR=/tmp
AA_ADMM_LIB="$R/ab/lib_rw1.so" AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3n" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3n.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3n.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3n" -name "*kernel_trace.csv" | head -1); python3 "$R/tools/solve_levels.py" "$f" 6 > "$R/gpurun_out/prof_r3n_levels.txt"; cat "$R/gpurun_out/prof_r3n_levels.txt"

AA_ADMM_LIB="$R/ab/lib_rw1.so" AA_SUB_TIMING=2 AA_ADMM_NO_GRAPH=1 timeout -k 10 200 python3 -u "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/subtiming_r3n.log" 2>&1; rc=$?
echo "subtiming rc=$rc"; grep "sub timing" "$R/gpurun_out/subtiming_r3n.log" | head -8
exit 0
