#!/bin/bash
# One GPU call for the round's numbers: smoke, -m gpu tests, the bench line (with the CPU baseline),
# a rocprofv3 kernel-trace summary of the bench and the PMC traffic passes (tools/pmc_traffic.sh).
# usage: tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --inflight 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
bash tools/pmc_traffic.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -30 $OUT/pmc.log; exit 1; }
echo done
