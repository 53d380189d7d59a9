#!/bin/bash
# round 3 final evidence (after the narrow backward tiles): GPU suite, smoke, C4 FETCH/WRITE PMC passes, C4 kernel-trace summary,
# kernel-trace summary of C4, FETCH/WRITE PMC passes (graph mode), C2 / C5 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r3f.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3f.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_r3f.log; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  AA_SOLVE_STATS=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_r3f_c4_$ctr" -o run -- python3 "$R/bench.py" --config c4 --steps 1 --warmup 0 --iters 10 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/pmc_r3f_c4_$ctr.log" 2>&1; rc=$?
  echo "pmc $ctr rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/pmc_r3f_c4_$ctr.log" | tail -5; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_r3f_c4" "$R/gpurun_out/r3f_c4_pmc.json" | tail -5
python3 "$R/tools/pmc_solve_table.py" "$R/gpurun_out/pmc_r3f_c4" "$R/gpurun_out/pmc_r3f_c4_FETCH_SIZE.log" > "$R/gpurun_out/r3f_c4_solve_pmc_table.txt" 2>&1; tail -3 "$R/gpurun_out/r3f_c4_solve_pmc_table.txt"
cp "$R/gpurun_out/r3f_c4_pmc.json" "$R/profiles/r3_c4_pmc.json"
for ctr in FETCH_SIZE WRITE_SIZE; do find "$R/gpurun_out/pmc_r3f_c4_$ctr" -name "*.csv" -size +2M -exec gzip -f {} \; ; done
AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r3f" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/prof_r3f.log" 2>&1; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/prof_r3f.log" | tail -5; exit $rc; }
f=$(find "$R/gpurun_out/prof_r3f" -name "*kernel_trace.csv" | head -1); python3 "$R/tools/solve_levels.py" "$f" 6 > "$R/gpurun_out/prof_r3f_levels.txt"; tail -1 "$R/gpurun_out/prof_r3f_levels.txt"; gzip -f "$f"
cd "$R"
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3f_c4.log 2> gpurun_out/bench_r3f_c4.err; rc=$?
echo "bench c4 rc=$rc"; cut -c1-250 gpurun_out/bench_r3f_c4.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3f_c4.err; exit $rc; }
for cfg in ${EXTRA_CFGS:-}; do
  timeout -k 10 600 python3 -u bench.py --config $cfg --steps 10 --warmup 3 > gpurun_out/bench_r3f_$cfg.log 2> gpurun_out/bench_r3f_$cfg.err; rc=$?
  echo "bench $cfg rc=$rc"; cut -c1-200 gpurun_out/bench_r3f_$cfg.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3f_$cfg.err; exit $rc; }
done
exit 0
