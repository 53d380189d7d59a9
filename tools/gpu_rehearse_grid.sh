set -e
for cfg in "8 32 0" "8 32 1024" "8 32 2048" "8 32 4096" "8 16 2048" "4 64 0" "4 64 2048" "4 64 4096"; do
  set -- $cfg
  PS=$1 TDS=1 ENVS=AA_SOLVE_MIN_SUBTREES=$2,AA_PART_TOP_ROWS=$3 bash tools/gpu_rehearse.sh
done
