#!/bin/bash
# Per-rank cost of a P-GPU mesh-partitioned C4 run, measured on ONE GPU: rank R of a P-way
# partition alone (bench.py --rehearse P, aa_comm_create_solo), dense top (default) and the
# round-1 replicated top (AA_TOP_DENSE=0). Each step has its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for P in ${PS:-2 4 8}; do
  for TD in ${TDS:-1 0}; do
    for R in ${RANKS:-0}; do
      env AA_TOP_DENSE=$TD ${ENVS//,/ } timeout -k 10 300 python -u bench.py --config ${CFG:-c4} --rehearse $P --rehearse-rank $R --steps ${STEPS:-3} --warmup 1 > gpurun_out/rehearse_${CFG:-c4}_P${P}_td${TD}_r$R.log 2>&1; rc=$?
      echo "P=$P top_dense=$TD rank=$R [${ENVS}] rc=$rc"
      case $rc in 0) ;; *) tail -5 gpurun_out/rehearse_${CFG:-c4}_P${P}_td${TD}_r$R.log; exit $rc;; esac
      python - gpurun_out/rehearse_${CFG:-c4}_P${P}_td${TD}_r$R.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"] or {}
print("  us/iter", d["rehearsal"]["us_per_iter"], "phases", r.get("phase_us_per_launch"),
      "elements", d["config"].get("partition"))
PY
    done
  done
done
exit 0
