#!/bin/bash
# A/B of library builds on one box: the same bench line per build (AA_ADMM_LIB), phases printed.
#   LIBS="ab/lib_head.so ab/lib_v1.so" CFG=c4 bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-c4}
for lib in $LIBS; do
  tag=$(basename "$lib" .so)
  AA_ADMM_LIB="$PWD/$lib" timeout -k 10 ${T:-300} python -u bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary ${BENCH_ARGS} > gpurun_out/ab_${CFG}_$tag.log 2>&1; rc=$?
  echo "== $tag rc=$rc"
  case $rc in 0) ;; *) tail -5 gpurun_out/ab_${CFG}_$tag.log; exit $rc;; esac
  python - "$tag" gpurun_out/ab_${CFG}_$tag.log <<'EOF'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], "value", d["value"], "ms/step", d["ms_per_step"], "phases", d["roofline"].get("phase_us_per_launch"))
EOF
done
exit 0
