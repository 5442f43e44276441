#!/bin/bash
# One GPU iteration: -m gpu parity tests, bench (no CPU baseline) at the default steps in flight,
# and a rocprofv3 kernel trace with one step in flight (per-kernel durations at the full running set:
# python tools/trace_full.py gpurun_out/TAG/prof/run_kernel_trace.csv).
# usage: tools/gpu_perf.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-perf}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],1), 'h/s', round(d['ms_per_step'],1), 'ms/step', 'iters', d['config']['mean_iters'], d['config']['max_iters'], 'conv', d['config']['converged_frac'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --inflight 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python tools/trace_full.py $OUT/prof/run_kernel_trace.csv
