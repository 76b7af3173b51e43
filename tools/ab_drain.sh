#!/bin/bash
# A/B of the last batch's tree builder (--drain-trees wave | lane) at the driver's 20 steps
set -o pipefail
for r in 1 2 3 4 5 6; do
  for d in wave; do
    echo -n "drain=$d: "
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --drain-trees $d 2>&1 | grep '^{' | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['host_issue_max_gap_ms'], d['stages_ms'])" || exit 1
  done
done
