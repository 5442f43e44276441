#!/bin/bash
# One GPU call: steps in flight x hardware queues (16-step runs, no extras).  usage: tools/gpu_queues.sh TAG
set -o pipefail
TAG=${1:-queues}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CFGS=${CFGS:-"4,4 8,4 8,8 6,8"}
for cfg in ${CFGS}; do
  cfg=${cfg/,/ }
  set -- $cfg
  timeout -k 10 300 python -u bench.py --hw-queues $2 --steps 16 --warmup 1 --inflight $1 --no-cpu-baseline --no-extra > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { echo "bench $cfg failed"; tail -5 $OUT/b_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$1_$2.json'));print('inflight $1 queues $2', round(d['value'],1), round(d['ms_per_step'],1))"
done
