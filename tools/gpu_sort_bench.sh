#!/bin/bash
# The reference's default sort+context mode: bench line + rocprofv3 kernel stats (sort kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/sort_${1:-x}; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python bench.py --sort --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT/bench.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(d["value"], d["ms_per_step"], d["stages_ms"], "bits/vec", d["bits_per_vector"], "cpu", d["cpu_baseline"]["value"])
PY
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/bench.py" --sort --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { tail "$OUT/kt.log"; exit 1; }
cut -d, -f1-7 "$OUT"/kt/kt_kernel_stats.csv | head -20
