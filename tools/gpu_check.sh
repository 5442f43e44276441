#!/bin/bash
# One GPU call: parity tests, smoke, bench (with CPU baseline), rocprof kernel stats.
# usage: tools/gpu_check.sh TAG [BATCH]
set -o pipefail
TAG=${1:-run}; B=${2:-8192}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --batch $B > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --batch $B --steps 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
ls -R $OUT/prof > $OUT/prof_files.txt
python tools/prof_summary.py "$OUT/prof/**/*.db" $OUT/rocprof_summary.md "bench.py --batch $B --steps 2 --warmup 1 ($TAG)" || true
bash tools/pmc_traffic.sh $TAG/traffic $B > $OUT/traffic.log 2>&1 || { echo "traffic passes failed"; tail -20 $OUT/traffic.log; exit 1; }
tail -12 $OUT/traffic.log
