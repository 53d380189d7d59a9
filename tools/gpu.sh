#!/bin/bash
# The one GPU-box runner (replaces round 1-3's one-off tools/gpu_*.sh): each argument is a step,
# run in order, each under its own time limit; the first failing step (fault, abort, timeout,
# non-zero exit) ends the script -- nothing else touches the GPU after it.
#
#   /usr/local/graft/bin/gpurun -- bash tools/gpu.sh tests smoke "bench c4 20 5" "ab c4 ab/lib_head.so,ab/lib_new.so"
#
# steps (fields separated by spaces inside one quoted argument):
#   tests [K+EXPR]                 pytest -m gpu [-k 'K EXPR'] (log gpurun_out/pytest_gpu.log)
#   smoke                          __graft_entry__.smoke()
#   bench CFG [STEPS] [WARMUP] [bench args]   full bench line -> gpurun_out/bench_CFG.log
#   ab CFG LIB1,LIB2,.. [bench args]          short bench per build (AA_ADMM_LIB), phases printed;
#                                  a build may carry env settings: lib.so+VAR=v+VAR2=w
#   dump SCENE LIB1,LIB2,..        tools/ab_dump.py trajectories per build, each compared
#                                  bit-for-bit with the first (scenes: drop40 c4small cloth pq wire)
#   pmc CFG TAG COUNTER[,COUNTER]  one rocprofv3 --pmc pass per comma group (graph mode)
#   prof CFG TAG [bench args]      rocprofv3 --kernel-trace --stats of a short eager run
#   rehearse CFG P RANK [ENV=V,..] [bench args]   bench.py --rehearse P --rehearse-rank RANK
#   eps TETS STEPS TAG             tools/elastic_eps_curves.py --gpu (per-step curves + npz)
#   geps CFG N TAG                 tools/ref_geom_curve.py --gpu on a (reduced) geometry scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
fatal() { case $1 in 0) ;; *) echo "fatal rc=$1 in [$2]; stopping"; exit $1;; esac; }
libenv() {   # "ab/lib_x.so+A=1+B=2" -> AA_ADMM_LIB=<abs> A=1 B=2
  local spec=$1 lib=${1%%+*} rest=""
  [ "$spec" != "$lib" ] && rest=${spec#*+} && rest=${rest//+/ }
  echo "AA_ADMM_LIB=$R/$lib $rest"
}
summ() {   # one-line summary of a bench log
  python3 - "$1" "$2" <<'PY'
import json, sys
ls = [l for l in open(sys.argv[2]) if l.startswith("{")]
if not ls:
    sys.exit(sys.argv[1] + ": no JSON line")
d = json.loads(ls[-1])
r = d.get("roofline") or {}
print(sys.argv[1], "value", d["value"], "ms/step", d["ms_per_step"], "frac", r.get("frac"),
      "phases", r.get("phase_us_per_launch") or r.get("phase_us_per_iter"))
PY
}
for step in "$@"; do
  set -- $step
  kind=$1; shift
  echo "== step [$step]"
  case $kind in
    tests)   # "tests" or "tests a+or+b" (a -k expression, '+' for spaces)
      kx=(); [ -n "${1:-}" ] && kx=(-k "${1//+/ }")
      timeout -k 10 ${T_TESTS:-1200} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${kx[@]}" \
        > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -8; fatal $rc tests ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -2 gpurun_out/smoke.log; fatal $rc smoke ;;
    bench)
      cfg=$1; st=${2:-20}; wu=${3:-5}; shift; shift; shift
      timeout -k 10 ${T_BENCH:-900} python3 -u bench.py --config $cfg --steps $st --warmup $wu "$@" \
        > gpurun_out/bench_$cfg.log 2> gpurun_out/bench_$cfg.err; rc=$?
      cut -c1-300 gpurun_out/bench_$cfg.log; [ $rc -ne 0 ] && tail -20 gpurun_out/bench_$cfg.err; fatal $rc "bench $cfg" ;;
    ab)
      cfg=$1; libs=$2; shift; shift; i=0
      for spec in ${libs//,/ }; do
        i=$((i+1)); log=gpurun_out/ab_${cfg}_$i.log
        env $(libenv $spec) timeout -k 10 ${T_AB:-300} python -u bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 \
          --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0 "$@" > $log 2>&1; rc=$?
        [ $rc -ne 0 ] && tail -5 $log; fatal $rc "ab $cfg $spec"
        summ "$i:$spec" $log
      done ;;
    dump)
      sc=$1; libs=$2; first=""
      for spec in ${libs//,/ }; do
        tag=$(basename "${spec%%+*}" .so)${spec#${spec%%+*}}; out=gpurun_out/dump_${sc}_${tag//[+=]/_}.npz
        env $(libenv $spec) timeout -k 10 300 python -u tools/ab_dump.py $out $sc > ${out%.npz}.log 2>&1; fatal $? "dump $sc $spec"
        if [ -z "$first" ]; then first=$out; else echo -n "$sc $spec vs first: "; python3 tools/ab_dump.py --compare $first $out; fatal $? "compare $sc $spec"; fi
      done ;;
    pmc)
      cfg=$1; tag=$2; ctrs=$3; shift; shift; shift
      for grp in ${ctrs//;/ }; do
        d="$R/gpurun_out/pmc_${tag}_${cfg}_${grp//,/_}"
        [ -n "${PMC_KERNEL:-}" ] && d="/tmp/pmc_${tag}_${cfg}_${grp//,/_}"   # raw CSVs stay on the box
        (cd /tmp && TMPDIR=/tmp timeout -k 10 -s KILL 300 rocprofv3 --pmc ${grp//,/ } --output-format csv -d "$d" -o run -- \
          python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --iters ${ITERS:-10} --no-cpu-baseline --eps-steps 0 \
          --no-secondary --geom-eps-solves 0 "$@" > "$d.log" 2>&1); rc=$?
        echo "pmc $grp rc=$rc"; [ $rc -ne 0 ] && grep -v "^ *@" "$d.log" | tail -5; fatal $rc "pmc $grp"
        [ -n "${PMC_KERNEL:-}" ] && python3 tools/pmc_sum.py "$d" "$PMC_KERNEL" "gpurun_out/pmc_${tag}_${cfg}.json"
      done ;;
    prof)
      cfg=$1; tag=$2; shift; shift; d="$R/gpurun_out/prof_${tag}_$cfg"
      (cd /tmp && AA_ADMM_NO_GRAPH=1 AA_EAGER_SYNC=10 TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$d" -o run -- python3 "$R/bench.py" --config $cfg --steps ${STEPS:-2} --warmup 0 \
        --no-cpu-baseline --eps-steps 0 --no-secondary --geom-eps-solves 0 "$@" > "$d.log" 2>&1); rc=$?
      echo "prof rc=$rc"; [ $rc -ne 0 ] && grep -v "^ *@" "$d.log" | tail -5; fatal $rc "prof $cfg"
      f=$(find "$d" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-160
      nrs=3; [ "$cfg" = c4 ] && nrs=6   # the Z variant's two-set solve; the others solve one set
      t=$(find "$d" -name "*kernel_trace.csv" | head -1); [ -n "$t" ] && python3 tools/solve_levels.py "$t" $nrs > "$d.levels.txt" 2>&1; [ -n "$t" ] && gzip -f "$t" ;;
    rehearse)   # rehearse CFG P RANK [ENV=V,ENV2=V] [bench args]
      cfg=$1; P=$2; rk=$3; envs=${4:-}; shift; shift; shift; [ $# -gt 0 ] && shift
      log=gpurun_out/rehearse_${cfg}_P${P}_r${rk}_${envs//[,=]/_}.log
      env ${envs//,/ } timeout -k 10 300 python -u bench.py --config $cfg --rehearse $P --rehearse-rank $rk --steps ${STEPS:-3} \
        --warmup 1 "$@" > $log 2>&1; rc=$?
      [ $rc -ne 0 ] && tail -5 $log; fatal $rc "rehearse $cfg $P $rk"
      python3 - $log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"] or {}
print("  us/iter", d["rehearsal"]["us_per_iter"], "phases", r.get("phase_us_per_launch"), "part", d["config"].get("partition"))
PY
      ;;
    eps)
      tets=$1; st=$2; tag=$3
      timeout -k 10 ${T_EPS:-900} python -u tools/elastic_eps_curves.py --gpu --tets $tets --steps $st \
        --out gpurun_out/eps_$tag.json --npz gpurun_out/eps_$tag.npz > gpurun_out/eps_$tag.log 2>&1; rc=$?
      tail -3 gpurun_out/eps_$tag.log; fatal $rc "eps $tag" ;;
    geps)
      cfg=$1; n=$2; tag=$3
      timeout -k 10 ${T_EPS:-900} python -u tools/ref_geom_curve.py --gpu --config $cfg --nx $n --iters ${ITERS:-2000} --out gpurun_out/geps_$tag.json \
        > gpurun_out/geps_$tag.log 2>&1; rc=$?
      tail -3 gpurun_out/geps_$tag.log; fatal $rc "geps $tag" ;;
    *) echo "unknown step [$step]"; exit 2 ;;
  esac
done
exit 0
