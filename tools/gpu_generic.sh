#!/bin/bash
# One GPU call: generic-solver figures (C3 shared budget N=100 with the bench's homotopy caps, C4 N=50; GPU vs
# the host IPM on 2 horizons) and the rocprofv3 kernel stats of a fixed-iteration probe (tools/generic_prof.py).
# usage: tools/gpu_generic.sh TAG [BATCH]
set -o pipefail
TAG=${1:-gen}; B=${2:-1024}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/generic_bench.py --batch $B --caps 150,300,1000 > $OUT/generic.json 2> $OUT/generic.err || { echo "generic bench failed"; tail -20 $OUT/generic.err; exit 1; }
cut -c1-1500 $OUT/generic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/generic_prof.py --batch $B --iters 12 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cut -d, -f1-6 $OUT/prof/run_kernel_stats.csv | cut -c1-160 | head -14
