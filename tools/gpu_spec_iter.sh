#!/bin/bash
# One GPU call while iterating on the specialised solver: its GPU tests (parity + MPC), a short bench at one step
# in flight (per-kernel HIP-event split) and the default 4-in-flight bench line.   usage: tools/gpu_spec_iter.sh TAG
set -o pipefail
TAG=${1:-speciter}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-extra > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench1 failed"; tail -20 $OUT/bench1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench1.json'));print('solo', round(d['value'],1), round(d['ms_per_step'],1), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()}, d['config']['mean_iters'])"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $OUT/bench4.json 2> $OUT/bench4.err || { echo "bench4 failed"; tail -20 $OUT/bench4.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench4.json'));print('inflight4', round(d['value'],1), round(d['ms_per_step'],1), d['config']['mean_iters'], d['config']['max_iters'])"
