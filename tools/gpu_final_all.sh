# Round-end checks on the final code, as the driver runs them: the whole -m gpu suite, smoke(),
# then the driver's bench command (N = 1, 20 steps, 5 warm-up) -> gpurun_out/r6/final/
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.out 2> $O/driver.err || { tail $O/driver.err; exit 1; }
grep -o '"value": [0-9.]*' $O/driver.out
