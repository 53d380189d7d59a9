#!/bin/bash
# nested-dissection leaf size (AA_ND_LEAF) on one GPU and at a P=8 rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for lf in ${LEAVES:-32 64 128}; do
  CASES="ab/lib_l.so|AA_ND_LEAF=$lf" bash tools/gpu_ab_env.sh || exit 1
  PS=8 TDS=1 ENVS=AA_ND_LEAF=$lf bash tools/gpu_rehearse.sh || exit 1
done
exit 0
