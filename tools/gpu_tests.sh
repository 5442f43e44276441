#!/bin/bash
# One GPU call: the -m gpu parity tests (all of them, no -x) and smoke.
# usage: tools/gpu_tests.sh TAG ["pytest -k expression"]
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out/$TAG; mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/gputest.log 2>&1
rc=$?
tail -15 $OUT/gputest.log
[ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
