#!/bin/bash
# round 3 call d: packed split-K tiles + lookahead work queue -- GPU suite, A/B bench, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
T=600 bash tools/gpu_tests.sh || exit $?
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eps-steps 0 --no-secondary > gpurun_out/ab_$tag.log 2> gpurun_out/ab_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/ab_$tag.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['phase_us_per_launch'])")"
  return $rc
}
run p1a1 AA_SOLVE_PACKED=1 AA_LQ_AHEAD=1 && run p0a0 AA_SOLVE_PACKED=0 AA_LQ_AHEAD=0 && run p1a0 AA_SOLVE_PACKED=1 AA_LQ_AHEAD=0 \
  && run p1a1r48 AA_LQ_REFILL=48 && run p1a1r32 AA_LQ_REFILL=32 && run p1a1m03 AA_LQ_MARGIN=0.3 && run p1a1b AA_SOLVE_PACKED=1 || exit $?
cd /tmp && export TMPDIR=/tmp
AA_ADMM_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3d_c4" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --iters 10 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3d_c4.log" 2>&1; echo "prof rc=$?"
cd "$R" && python3 tools/solve_levels.py gpurun_out/prof_r3d_c4/run_kernel_trace.csv 6 && python3 tools/solve_levels.py gpurun_out/prof_r3d_c4/run_kernel_trace.csv 3
exit 0
