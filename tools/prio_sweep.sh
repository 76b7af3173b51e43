#!/bin/bash
# Wave-priority sweep of the default bench (pqh_prio knobs PQH_PRIO_<KERNEL>): one 200-step
# run per setting, the JSON line's value and stage times into gpurun_out/prio/.
set -e
mkdir -p gpurun_out/prio
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 120 python bench.py --steps 200 --warmup 5 --no-cpu-baseline \
        > gpurun_out/prio/$name.log 2>&1
    python - "$name" <<'PY'
import json, sys
n = sys.argv[1]
l = [x for x in open(f"gpurun_out/prio/{n}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(n, d["value"], d["ms_per_step"], d["stages_ms"], flush=True)
PY
}
run default
run hist3 PQH_PRIO_HIST=3
run assign2 PQH_PRIO_ASSIGN=2
run lat1_assign2_hist3 PQH_PRIO_TREES=1 PQH_PRIO_LUTS=1 PQH_PRIO_DECODE=1 PQH_PRIO_ASSIGN=2 PQH_PRIO_HIST=3
run all0 PQH_PRIO_TREES=0 PQH_PRIO_LUTS=0 PQH_PRIO_DECODE=0
run enc3 PQH_PRIO_ENCODE=3
run assign1_hist2 PQH_PRIO_ASSIGN=1 PQH_PRIO_HIST=2
