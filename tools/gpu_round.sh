#!/bin/bash
# One GPU call: -m gpu tests, the bench line, a rocprofv3 kernel-trace summary of the bench.
# usage: tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 720 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest.log; exit 1; }
  tail -3 $OUT/gputest.log
fi
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
echo done
