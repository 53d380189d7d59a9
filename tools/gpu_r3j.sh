#!/bin/bash
# round 3 call j: streamed tile levels -- GPU suite, C4 A/B (stream on/off, lookahead queue on/off),
# kernel trace of the streamed solve
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_elastic.py -k "streamed" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r3j_stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_r3j_stream.log | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3j.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3j.log; [ $rc -ne 0 ] && exit $rc
B="--steps 5 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary"
for v in "AA_SOLVE_STREAM=1 AA_SOLVE_STATS=1" "AA_SOLVE_STREAM=0" "AA_SOLVE_STREAM=1 AA_LQ_AHEAD=0" "AA_SOLVE_STREAM=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 -u bench.py $B > gpurun_out/ab_r3j_$tag.log 2> gpurun_out/ab_r3j_$tag.err; rc=$?
  echo "$v rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_r3j_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['phase_us_per_launch'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_r3j_$tag.err; exit $rc; }
done
grep "\[solve\]" gpurun_out/ab_r3j_AA_SOLVE_STREAM_1_AA_SOLVE_STATS_1.err | head -40
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3j" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3j.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3j.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3j" -name "*kernel_trace.csv" | head -1); python3 "$R/tools/solve_levels.py" "$f" 6 > "$R/gpurun_out/prof_r3j_levels.txt"; cat "$R/gpurun_out/prof_r3j_levels.txt"
exit 0
