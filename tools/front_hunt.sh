#!/bin/bash
# Run the partition tests that factor GPU fronts under several ranks (the front check throws on a
# wrong factorization); afterwards replay every dumped front on the host (CPU only) into
# gpurun_out/front_replay.json, and drop the dumps (f x f doubles each).
#   /usr/local/graft/bin/gpurun -- bash tools/front_hunt.sh [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; rm -rf /tmp/aa_front_dump; mkdir -p /tmp/aa_front_dump
K=${1:-block1m}
timeout -k 10 900 python -u -m pytest tests/test_gpu_partition.py -x -v --timeout 600 --timeout-method thread -k "$K" \
  > gpurun_out/front_hunt.log 2>&1; rc=$?
grep -E "PASSED|FAILED|front-check" gpurun_out/front_hunt.log | cut -c1-600 | tail -20
ls /tmp/aa_front_dump | head
n=$(ls /tmp/aa_front_dump/*_kept.bin 2>/dev/null | wc -l)
if [ "$n" -gt 0 ]; then
  timeout -k 10 600 python3 tools/front_replay.py /tmp/aa_front_dump/*_kept.bin > gpurun_out/front_replay.json 2>&1
  head -c 3000 gpurun_out/front_replay.json
fi
rm -rf /tmp/aa_front_dump
exit $rc
