set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for d in 2 3; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --depth $d 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stages_ms'])"
done
timeout -k 10 120 python tools/bench_decode.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/bench_encode.py 2>&1 | grep -v amdgpu.ids
