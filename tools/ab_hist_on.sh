#!/bin/bash
# A/B of the histogram's stream (diagnostic): --hist-on assign (default) vs lanes, 20 and 200 steps
set -o pipefail
for r in 1 2; do
  for h in assign lanes; do
    for k in 20 200; do
      echo -n "hist-on=$h steps=$k: "
      timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu-baseline --hist-on $h 2>&1 | grep '^{' | \
        python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stages_ms'])" || exit 1
    done
  done
done
