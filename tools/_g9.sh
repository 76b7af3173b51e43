set -o pipefail
mkdir -p gpurun_out/g9
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_huffman.py tests/test_gpu_configs.py > gpurun_out/g9/t.log 2>&1 || { tail -30 gpurun_out/g9/t.log; exit 1; }
tail -2 gpurun_out/g9/t.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_fullsize.py -k "k4096 or deep" > gpurun_out/g9/f.log 2>&1 || { tail -30 gpurun_out/g9/f.log; exit 1; }
tail -2 gpurun_out/g9/f.log
timeout -k 10 200 python bench.py --config deep --no-cpu-baseline > gpurun_out/g9/deep.log 2>&1 || { tail gpurun_out/g9/deep.log; exit 1; }
timeout -k 10 200 python bench.py --config k4096 --steps 40 --no-cpu-baseline > gpurun_out/g9/k3.log 2>&1 || { tail gpurun_out/g9/k3.log; exit 1; }
timeout -k 10 200 python bench.py --config k4096 --steps 40 --lanes 5 --no-cpu-baseline > gpurun_out/g9/k5.log 2>&1 || { tail gpurun_out/g9/k5.log; exit 1; }
timeout -k 10 200 python tools/bench_assign.py 20 k4096 > gpurun_out/g9/a4k.log 2>&1 || { tail gpurun_out/g9/a4k.log; exit 1; }
for f in deep k3 k5; do python -c "
import json,sys
for l in open('gpurun_out/g9/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['stages_ms'])"; done
cat gpurun_out/g9/a4k.log | grep -v amdgpu
