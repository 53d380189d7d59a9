cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_elastic.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1; rc=$?; echo pytest_rc=$rc; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_c4.log | tail -30; \
case $rc in 124|134|137|139) exit $rc;; esac; \
CFG=c4 TAG=r1_c4 BENCH_ARGS="--steps 2 --warmup 1" PROF_ARGS="--tets 100,40,50" bash tools/gpu_bench.sh
