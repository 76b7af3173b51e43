# Bench lines for a list of argument sets (comma-separated args; ';' between sets), each once:
#   bash tools/gpu_sched_ab.sh "<args1>;<args2>;..."
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/sched; mkdir -p $OUT
IFS=';' read -ra SETS <<< "$1"
i=0
for a in "${SETS[@]}"; do
  i=$((i+1))
  args=$(echo "$a" | tr ',' ' ')
  timeout -k 10 400 env $ENVV python bench.py $args --no-cpu-baseline > $OUT/run$i.log 2>&1 || { tail $OUT/run$i.log; exit 1; }
  echo "[$args] $(grep -o '"value": [0-9.]*' $OUT/run$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/run$i.log)"
done
