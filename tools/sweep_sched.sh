# schedule sweep of bench.py (depth x table CUs); one JSON line per config
set -o pipefail
mkdir -p gpurun_out
for cfg in "--depth 1 --table-cus 64" "--depth 2 --table-cus 64" "--depth 3 --table-cus 64" "--depth 2 --table-cus 32" "--depth 2 --table-cus 128" "--no-overlap"; do
  echo "== $cfg"
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $cfg | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stages_ms'])" || exit 1
done
