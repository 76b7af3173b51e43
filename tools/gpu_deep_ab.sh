# Deep (configs[3]) A/B: the in-tree build against lib/variants/<v>: PQ parity tests, the
# assignment alone (tools/bench_assign.py) and the bench at 100 steps, two rounds
#   bash tools/gpu_deep_ab.sh <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/deepab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pq.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
V=(in-tree "$@")
for i in 1 2; do
  for v in "${V[@]}"; do
    L=""; [ "$v" != in-tree ] && L=$GRAFT_REPO_ROOT/pq_huffman_amd/lib/variants/$v/libpqh.so
    env ${L:+PQH_LIB=$L} timeout -k 10 200 python tools/bench_assign.py 20 deep 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
    env ${L:+PQH_LIB=$L} timeout -k 10 300 python bench.py --config deep --steps 100 --warmup 10 --no-cpu-baseline > $OUT/$v.$i.log 2>&1 || { tail $OUT/$v.$i.log; exit 1; }
    echo "$v bench $(grep -o '"value": [0-9.]*' $OUT/$v.$i.log) $(grep -o '"alone_avg_ms": [0-9.]*' $OUT/$v.$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/$v.$i.log)"
  done
done
