#!/bin/bash
# C4 timeline in graph mode: kernel trace of a short bench run (per-iteration busy vs wall,
# gated reject-branch launches), plus the bench line's Anderson reject count
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_r3ad" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --eps-steps 0 --no-secondary > "$R/gpurun_out/tl_r3ad.log" 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -ne 0 ] && { grep -v "^ *@" "$R/gpurun_out/tl_r3ad.log" | tail -5; exit $rc; }
grep '^{' "$R/gpurun_out/tl_r3ad.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'rejects', d.get('anderson_rejects'))"
f=$(find "$R/gpurun_out/tl_r3ad" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline.py" "$f" > "$R/gpurun_out/tl_r3ad.txt"; cat "$R/gpurun_out/tl_r3ad.txt"
gzip -f "$f"
exit 0
