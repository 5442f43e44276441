#!/bin/bash
# Stage stamps of the current build, then the bench at 2/3/4 steps in flight (no CPU baseline, no extras).
# usage: tools/gpu_sweep.sh TAG
set -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python -u tools/diag_stamps.py 2048 > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
tail -22 $OUT/stamps.txt
for I in 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --inflight $I > $OUT/bench_if$I.json 2> $OUT/bench_if$I.err || { tail -20 $OUT/bench_if$I.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_if$I.json').read().strip().splitlines()[-1]); print('inflight $I', round(d['value'],1), 'h/s', round(d['ms_per_step'],1), 'ms/step')"
done
