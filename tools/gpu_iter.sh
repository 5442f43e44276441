#!/bin/bash
# Quick GPU iteration: parity tests, phase stamps at 1024, probe at the given batch sizes.
# usage: tools/gpu_iter.sh TAG [B ...]
set -o pipefail
TAG=${1:-it}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/diag_stamps.py 1024 > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
for B in "$@"; do
  timeout -k 10 300 python -u tools/solve_probe.py $B > $OUT/probe_$B.log 2>&1 || { tail -20 $OUT/probe_$B.log; exit 1; }
  grep -v amdgpu.ids $OUT/probe_$B.log
done
