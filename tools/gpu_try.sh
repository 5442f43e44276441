#!/bin/bash
# One iteration on the GPU: -m gpu tests, then the bench (no CPU baseline, no extras) at the given
# steps-in-flight counts.  usage: tools/gpu_try.sh TAG [skip-tests] [INFLIGHT ...]
set -o pipefail
TAG=${1:-try}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
else
  shift
fi
for I in "${@:-2}"; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --inflight $I > $OUT/bench_if$I.json 2> $OUT/bench_if$I.err || { tail -20 $OUT/bench_if$I.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_if$I.json').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('inflight $I', round(d['value'],1), 'h/s', round(d['ms_per_step'],1), 'ms/step', 'iters', round(d['config']['mean_iters'],2), {a: round(b,1) for a,b in k.items()})"
done
