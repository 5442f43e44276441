#!/bin/bash
# GPU parity tests then the solve probe at the given batch sizes.  usage: tools/gpu_quick.sh TAG [B ...]
set -o pipefail
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | head -40
[ $rc -ne 0 ] && { tail -40 $OUT/pytest.log; exit 1; }
for B in "$@"; do
  timeout -k 10 300 python -u tools/solve_probe.py $B > $OUT/probe_$B.log 2>&1 || { cat $OUT/probe_$B.log | tail -20; exit 1; }
  cat $OUT/probe_$B.log
done
