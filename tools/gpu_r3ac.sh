#!/bin/bash
# SQ counters of the geometry z kernels (C5, C3), summarised on the box; raw CSVs removed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for cfg in c5 c3; do
  CFG=$cfg TAG=geo ITERS=10 bash tools/gpu_valu.sh || exit 1
  python tools/valu_summary.py gpurun_out/pmc_geo_$cfg gpurun_out/valu_geo_$cfg.json > gpurun_out/valu_geo_$cfg.txt || exit 1
  rm -rf gpurun_out/pmc_geo_${cfg}_1 gpurun_out/pmc_geo_${cfg}_2
  cat gpurun_out/valu_geo_$cfg.txt
done
exit 0
