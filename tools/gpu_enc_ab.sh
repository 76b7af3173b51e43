set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/enc
timeout -k 10 600 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_parts.py tests/test_gpu_lds_poison.py tests/test_gpu_zz_shard.py tests/test_gpu_configs.py tests/test_tree.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/enc/tests.log 2>&1 || { tail -40 gpurun_out/enc/tests.log; exit 1; }
tail -2 gpurun_out/enc/tests.log
for impl in tiled onepass; do
  for cfg in sift deep; do
    PQH_ENC_IMPL=$impl timeout -k 10 200 python tools/bench_encdec.py --config $cfg 2>&1 | grep -v amdgpu.ids | sed "s/^/$impl /" || exit 1
  done
  PQH_ENC_IMPL=$impl timeout -k 10 300 python tools/bench_encdec.py --config sift --rows 16000000 --reps 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$impl /" || exit 1
done
for impl in tiled onepass; do
  PQH_ENC_IMPL=$impl timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/enc/b200_$impl.log 2>&1 || { tail gpurun_out/enc/b200_$impl.log; exit 1; }
  echo "$impl $(grep -o '"value": [0-9.]*' gpurun_out/enc/b200_$impl.log) $(grep -o '"stages_ms": {[^}]*}' gpurun_out/enc/b200_$impl.log)"
done
