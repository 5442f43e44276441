#!/bin/bash
# One GPU call: per-kernel breakdown of small batches (1 and 1024 horizons, one step in flight), the
# first-solve probe and the generic-solver throughput.  usage: tools/gpu_small.sh TAG
set -o pipefail
TAG=${1:-small}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for B in 1 1024; do
  timeout -k 10 300 python -u bench.py --batch $B --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-extra > $OUT/bench_$B.json 2> $OUT/bench_$B.err || { echo "bench $B failed"; tail -20 $OUT/bench_$B.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$B.json'));print($B, round(d['value'],1), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()}, d['config']['mean_iters'], d['config']['max_iters'])"
done
timeout -k 10 300 python -u tools/first_solve_probe.py 8192 > $OUT/first_solve.log 2>&1 && cat $OUT/first_solve.log
timeout -k 10 600 python -u tools/generic_bench.py --batch 1024 > $OUT/generic.json 2> $OUT/generic.err || { echo "generic bench failed"; tail -20 $OUT/generic.err; exit 1; }
cut -c1-2000 $OUT/generic.json
