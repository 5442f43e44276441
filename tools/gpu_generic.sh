#!/bin/bash
# One GPU call: generic-solver throughput (C3 shared budget N=100, C4 N=50) and its rocprofv3 kernel stats.
# usage: tools/gpu_generic.sh TAG [BATCH]
set -o pipefail
TAG=${1:-gen}; B=${2:-1024}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/generic_bench.py --batch $B > $OUT/generic.json 2> $OUT/generic.err || { echo "generic bench failed"; tail -20 $OUT/generic.err; exit 1; }
cut -c1-1500 $OUT/generic.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/generic_bench.py --batch $B --sample 0 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
