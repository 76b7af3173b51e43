set -o pipefail
O=gpurun_out/g10; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_huffman.py tests/test_gpu_configs.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for c in sift deep; do
  timeout -k 10 120 python tools/bench_hist.py $c 2>&1 | grep hist || exit 1
  PQH_HIST_IMPL=thread timeout -k 10 120 python tools/bench_hist.py $c 2>&1 | grep hist || exit 1
done
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > $O/sift.log 2>&1 || { tail $O/sift.log; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > $O/sift20.log 2>&1 || { tail $O/sift20.log; exit 1; }
timeout -k 10 200 python bench.py --config deep --no-cpu-baseline > $O/deep.log 2>&1 || { tail $O/deep.log; exit 1; }
for f in sift sift20 deep; do python -c "
import json,sys
for l in open('$O/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['stages_ms'])"; done
