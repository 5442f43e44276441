#!/bin/bash
# One GPU call: generic-solver kernel profile (rocprofv3 kernel stats at a fixed iteration count), the
# per-iteration latency of one horizon, and the first homotopy stage's status / iteration histogram.
# usage: tools/gpu_gprof.sh TAG [full]
set -o pipefail
TAG=${1:-gprof}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/generic_prof.py --batch 1024 --iters 12 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
grep generic_prof $OUT/prof.log
cat $OUT/prof/run_kernel_stats.csv | cut -d, -f1-6 | head -12
timeout -k 10 300 python3 -u tools/generic_prof.py --batch 1 --iters 12 > $OUT/b1.log 2>&1 || { echo "b1 failed"; tail -20 $OUT/b1.log; exit 1; }
grep generic_prof $OUT/b1.log
if [ "$2" == "full" ]; then
  timeout -k 10 400 python3 -u tools/generic_prof.py --batch 1024 --iters 12 --cases c3 --full > $OUT/full.log 2>&1 || { echo "full failed"; tail -20 $OUT/full.log; exit 1; }
  grep generic_prof $OUT/full.log
fi
