set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pq.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pq.log 2>&1 || { tail -30 gpurun_out/gpu_pq.log; exit 1; }
tail -3 gpurun_out/gpu_pq.log
timeout -k 10 120 python tools/bench_assign.py 20 2>&1 | grep -v amdgpu.ids
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_assign -o kt --output-format csv -- python3 tools/bench_assign.py 10 > gpurun_out/kt_assign.log 2>&1
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/kt_assign/kt_kernel_stats.csv')))[:6]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
