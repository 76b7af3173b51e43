#!/bin/bash
# GPU-box step runner (diagnostic): bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Each step runs under its own time limit; the first failing step ends the call.
#   assign[:cfg]   tools/bench_assign.py 50 <cfg> twice          (default cfg sift)
#   assignvar:<a,b> tools/bench_assign.py with each lib/variants/<v>/libpqh.so
#   micro:<bin>    a built tools/micro diagnostic
#   bench          bench.py --steps 20 --warmup 5 (the driver's), no CPU baseline
#   bench200       bench.py --steps 200 --warmup 20
#   benchargs:<a,b> bench.py with the comma-separated arguments
#   benchcfg:<c>   bench.py --config <c> --steps 100 --warmup 10
#   tests[:<f,g>]  pytest -m gpu on tests/ (or the comma-separated files)
#   kt:<cmd...>    not supported here (profiles/collect.sh owns the profiles)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
for s in "$@"; do
  case "$s" in
    assignvar:*) for v in $(echo "${s#assignvar:}" | tr ',' ' '); do
        for i in 1 2; do
          echo -n "$v: "; PQH_LIB=$R/pq_huffman_amd/lib/variants/$v/libpqh.so \
            timeout -k 10 200 python "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids \
            | tee -a "$OUT/assignvar.log" || exit 1
        done
      done ;;
    micro:*) b=${s#micro:}
      timeout -k 10 120 "$R/tools/micro/$b" 2>&1 | grep -v amdgpu.ids | tee "$OUT/micro_$b.log" || exit 1 ;;
    assign*) cfg=${s#assign}; cfg=${cfg#:}; cfg=${cfg:-sift}
      for i in 1 2; do
        timeout -k 10 200 python "$R/tools/bench_assign.py" 50 "$cfg" 2>&1 | grep -v amdgpu.ids \
          | tee -a "$OUT/assign_$cfg.log" || exit 1
      done ;;
    bench) timeout -k 10 300 python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench20.log" 2>&1 || { tail "$OUT/bench20.log"; exit 1; }
      grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$OUT/bench20.log" ;;
    benchargs:*) a=$(echo "${s#benchargs:}" | tr ',' ' '); tag=$(echo "$a" | tr -c 'a-z0-9' '_')
      timeout -k 10 300 python "$R/bench.py" $a --no-cpu-baseline > "$OUT/bench_$tag.log" 2>&1 \
        || { tail "$OUT/bench_$tag.log"; exit 1; }
      echo -n "$a: "; grep -o '"value": [0-9.]*' "$OUT/bench_$tag.log" ;;
    bench200) timeout -k 10 300 python "$R/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/bench200.log" 2>&1 \
        || { tail "$OUT/bench200.log"; exit 1; }
      grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$OUT/bench200.log" ;;
    benchcfg:*) c=${s#benchcfg:}
      timeout -k 10 300 python "$R/bench.py" --config "$c" --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/bench_$c.log" 2>&1 \
        || { tail "$OUT/bench_$c.log"; exit 1; }
      grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$OUT/bench_$c.log" ;;
    tests*) f=${s#tests}; f=${f#:}; f=${f:-tests}; f=$(echo "$f" | tr ',' ' ')
      (cd "$R" && timeout -k 10 900 python -u -m pytest $f -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/tests.log" 2>&1) || { tail -40 "$OUT/tests.log"; exit 1; }
      tail -2 "$OUT/tests.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_run done"
