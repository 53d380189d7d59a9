#!/bin/bash
# round 3 call v: plain boundary-row gathers + nt rows rule (lib_fr = the tree), top amalgamation budget sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
B="--steps 4 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0"
for cfg in c4 c3 c2 c5; do
for v in "AA_TOP_ROWS=2048" "AA_TOP_ROWS=4096" "AA_TOP_ROWS=6500" "AA_TOP_ROWS=10000" "AA_TOP_ROWS=2048" "AA_TOP_ROWS=6500"; do
  tag=$(echo "$v" | tr ' =' '__')_$cfg
  env $v timeout -k 10 300 python3 -u bench.py --config $cfg $B > gpurun_out/ab_r3v_$tag.log 2> gpurun_out/ab_r3v_$tag.err; rc=$?
  echo "$tag rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3v_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],'nnz',d['config']['nnz_factor'],'setup',d['config']['setup_ms'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3v_$tag.err; exit $rc; }
done; done
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3v" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3v.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3v.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3v" -name "*kernel_trace.csv" | head -1); python3 "$R/tools/solve_levels.py" "$f" 6 > "$R/gpurun_out/prof_r3v_levels.txt"; cat "$R/gpurun_out/prof_r3v_levels.txt"
exit 0
