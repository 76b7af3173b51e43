# decoder A/B: GPU decode tests, then bench_encdec and bench lines at PQH_DEC_CHAINS=2 / 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dec
timeout -k 10 600 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_parts.py tests/test_gpu_lds_poison.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dec/tests.log 2>&1 || { tail -40 gpurun_out/dec/tests.log; exit 1; }
tail -1 gpurun_out/dec/tests.log
for c in 2 1; do
  for cfg in sift deep; do
    PQH_DEC_CHAINS=$c timeout -k 10 200 python tools/bench_encdec.py --config $cfg 2>&1 | grep -v amdgpu.ids | sed "s/^/chains=$c /" || exit 1
  done
done
for rep in 1 2; do
for c in 2 1; do
  for a in "--steps 200 --warmup 20" "--config deep --steps 100 --warmup 10"; do
    PQH_DEC_CHAINS=$c timeout -k 10 300 python bench.py $a --no-cpu-baseline > gpurun_out/dec/b.log 2>&1 || { tail gpurun_out/dec/b.log; exit 1; }
    echo "chains=$c [$a] $(grep -o '"value": [0-9.]*' gpurun_out/dec/b.log) $(grep -o '"stages_ms": {[^}]*}' gpurun_out/dec/b.log)"
  done
done
done
