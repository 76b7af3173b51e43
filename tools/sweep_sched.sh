# schedule sweep of bench.py (depth x table CUs x chunk); one line per config:
#   bash tools/sweep_sched.sh "<bench args>" ...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "== $cfg"
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $cfg 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stages_ms'])" || exit 1
done
