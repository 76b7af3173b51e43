set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/sweep_sched.sh "--depth 3 --chunk 8 --table-cus 256" "--no-overlap --chunk 8" || exit 1
timeout -k 10 120 python tools/bench_assign.py 30 2>&1 | grep -v amdgpu.ids
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_b -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --depth 3 --chunk 8 --table-cus 256 > gpurun_out/kt_b.log 2>&1
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/kt_b/kt_kernel_stats.csv')))[:14]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
