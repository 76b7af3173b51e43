#!/bin/bash
# configs[4] (K = 4096) lane layouts: the code tables are the long stage there
set -o pipefail
for cfg in "--lanes 2 --elanes 1" "--lanes 3 --elanes 0" "--lanes 3 --elanes 1"; do
  echo -n "$cfg: "
  timeout -k 10 300 python bench.py --config k4096 --steps 20 --warmup 3 --no-cpu-baseline $cfg 2>&1 | grep '^{' | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stages_ms'])" || exit 1
done
