#!/bin/bash
# round 3 call c: geometry run-to-eps (test + C3 bench leg), elastic eps curves of the small drop,
# then the round-2 eager --pmc crash reproduced with a 500-iteration eager step (last: may end the call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_geom.py -x -v --timeout 120 --timeout-method thread -k "run_to_eps or deterministic" > gpurun_out/pytest_r3c.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_r3c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r3c_c3.log 2> gpurun_out/bench_r3c_c3.err; rc=$?
echo "bench c3 rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r3c_c3.err; exit $rc; }
timeout -k 10 300 python3 -u tools/elastic_eps_curves.py --gpu --tets 20,8,10 --steps 20 --out gpurun_out/r3_eps_gpu_drop20x8x10.json 2> gpurun_out/eps_gpu.err; rc=$?
echo "eps curves rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/eps_gpu.err; exit $rc; }
# eager FETCH_SIZE over one 500-iteration step (~20k dispatches without a host sync)
export AA_ADMM_NO_GRAPH=1 AA_DUMP_MAPS="$R/gpurun_out/pmc_r3crash.maps"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_r3crash" -o run -- python3 "$R/bench.py" --config c4 --steps 1 --warmup 0 --iters 10 --no-cpu-baseline --eps-steps 1 --no-secondary > "$R/gpurun_out/pmc_r3crash.log" 2>&1; echo "eager 500-iteration pmc rc=$?"
exit 0
