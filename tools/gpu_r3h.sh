#!/bin/bash
# round 3 call h: solve suite after the clean-up, kernel traces (eager, host sync every 10
# iterations: the profiler's dispatch interception crashes on ~4.5k kernels per host sync) A/B
# lookahead over whole 100-iteration steps, partitioned setup with / without per-part factoring
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_elastic.py tests/test_gpu_geom.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3h.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3h.log; [ $rc -ne 0 ] && exit $rc
for P in 2 4; do for pf in 1 0; do
  AA_PART_FACTOR=$pf AA_SETUP_TIMES=1 timeout -k 10 400 python3 -u bench.py --gpus $P --partition host --same-device --steps 2 --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary > gpurun_out/part_r3h_P${P}_pf$pf.log 2> gpurun_out/part_r3h_P${P}_pf$pf.err; rc=$?
  echo "P=$P partfactor=$pf rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/part_r3h_P${P}_pf$pf.log') if l.startswith('{')][-1]);print(d['n_gpus'],d['value'],d['config']['setup_ms'],d['config']['parallelism'])")"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/part_r3h_P${P}_pf$pf.err; exit $rc; }
done; done
cd /tmp && export TMPDIR=/tmp
for ah in 0 1; do
  AA_LQ_AHEAD=$ah AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3h_ah$ah" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3h_ah$ah.log" 2>&1; rc=$?
  echo "prof ahead=$ah rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3h_ah$ah.log" | tail -5; exit $rc; }
done
exit 0
