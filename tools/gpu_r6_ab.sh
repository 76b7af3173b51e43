set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/ab1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_configs.py tests/test_gpu_huffman.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
 for v in new asm; do
  L=""; [ $v = asm ] && L=pq_huffman_amd/lib/variants/asm/libpqh.so
  PQH_LIB=${L:-pq_huffman_amd/lib/libpqh.so} timeout -k 10 120 python tools/bench_assign.py 50 sift > $O/ba_$v.$r.log 2>&1 || { tail $O/ba_$v.$r.log; exit 1; }
  echo "$v $(tail -1 $O/ba_$v.$r.log)"
  PQH_LIB=${L:-pq_huffman_amd/lib/libpqh.so} timeout -k 10 120 python tools/bench_assign.py 30 deep > $O/bd_$v.$r.log 2>&1 || { tail $O/bd_$v.$r.log; exit 1; }
  echo "$v $(tail -1 $O/bd_$v.$r.log)"
  for K in 20 200; do
   PQH_LIB=${L:-pq_huffman_amd/lib/libpqh.so} timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline > $O/b_$v.$K.$r.log 2>&1 || { tail $O/b_$v.$K.$r.log; exit 1; }
   echo "$v K=$K $(grep -o '"value": [0-9.]*' $O/b_$v.$K.$r.log)"
  done
 done
done
