#!/bin/bash
# round 3 call aa: per-rank rehearsals with this round's kernels -- block C4 at P = 2 / 4 / 8 (rank 0),
# the voxelised bunny at P = 8 (all ranks: partition balance on an irregular mesh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
run() {  # tag, args...
  tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --steps 3 --warmup 1 > gpurun_out/reh_r3_$tag.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -5 gpurun_out/reh_r3_$tag.log; exit $rc; }
  python3 - gpurun_out/reh_r3_$tag.log "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"] or {}
p = r.get("phase_us_per_launch") or {}
print(sys.argv[2], "us/iter", d["rehearsal"]["us_per_iter"], "solve", p.get("solve"), "aa", p.get("aa"), "grad", p.get("grad"),
      "rhs", p.get("rhs"), "prim", p.get("prim"), "elements", d["config"].get("partition"))
PY
}
for P in 2 4 8; do run block_P${P}_r0 --rehearse $P --rehearse-rank 0; done
run block_P8_r7 --rehearse 8 --rehearse-rank 7
for r in 0 1 2 3 4 5 6 7; do run bunny_P8_r$r --mesh bunny --rehearse 8 --rehearse-rank $r; done
exit 0
