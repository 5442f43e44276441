#!/bin/bash
# rocprofv3 kernel trace + stats of the bench with one step in flight (the solo-step kernel durations
# bench.py reports), then the stage stamps.  usage: tools/gpu_prof1.sh TAG
set -o pipefail
TAG=${1:-prof1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --inflight 1 > $OUT/prof.json 2> $OUT/prof.log || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python tools/trace_full.py $OUT/prof/run_kernel_trace.csv
timeout -k 10 200 python -u tools/diag_stamps.py 2048 > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
tail -22 $OUT/stamps.txt
