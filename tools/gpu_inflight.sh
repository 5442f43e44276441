#!/bin/bash
# Throughput against the number of independent steps in flight (bench.py --inflight), plus one
# rocprofv3 kernel trace with a single step in flight (kernel durations not shared with another step).
# usage: tools/gpu_inflight.sh TAG "1 2 3 4"
set -o pipefail
TAG=${1:-inflight}; LIST=${2:-"1 2 3 4"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for k in $LIST; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --inflight $k > $OUT/bench_if$k.json 2> $OUT/bench_if$k.err || { echo "bench inflight $k failed"; tail -20 $OUT/bench_if$k.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_if$k.json').read().strip().splitlines()[-1]); print('inflight', $k, round(d['value'],1), 'h/s', round(d['ms_per_step'],1), 'ms/step')"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --inflight 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
echo done
