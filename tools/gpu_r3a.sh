#!/bin/bash
# round 3, first GPU call: the parity suite, then one FETCH_SIZE pass in graph mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=600 bash tools/gpu_tests.sh && CTRS=FETCH_SIZE bash tools/gpu_pmc.sh
