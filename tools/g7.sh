set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_pq.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pq.log 2>&1 || { tail -30 gpurun_out/gpu_pq.log; exit 1; }
tail -1 gpurun_out/gpu_pq.log
PQH_LIB=pq_huffman_amd/lib/variants/stamps/libpqh.so timeout -k 10 120 python tools/assign_stamps.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/bench_assign.py 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 2>&1 | grep -v amdgpu.ids | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stages_ms'])"
