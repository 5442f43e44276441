#!/bin/bash
# A/B of the Riccati kernel variants: parity tests, then the bench at 32 and 64 lanes per horizon, then
# a rocprof kernel-stats run of the default (32).  usage: tools/gpu_ab_kkt.sh TAG
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "kkt_two or headline or pilz6_batch" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -4 $OUT/pytest.log
for L in 32 64; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra --kkt-lanes $L > $OUT/bench_$L.json 2> $OUT/bench_$L.err || { echo "bench $L failed"; tail -30 $OUT/bench_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$L.json'));print($L, round(d['value'],1), {k:round(v,1) for k,v in d['roofline']['kernel_ms'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --inflight 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-6
