#!/bin/bash
# One GPU call while iterating on the generic solver: its GPU tests, the phase stamps (C3 shared batch 1
# and 1024, C4 1024) and the per-iteration probe.   usage: tools/gpu_gen_iter.sh TAG
set -o pipefail
TAG=${1:-geniter}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_generic.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "generic gpu tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/gdiag_stamps.py 1 12 c3 > $OUT/c3_1.txt 2>&1 && timeout -k 10 200 python3 -u tools/gdiag_stamps.py 1024 12 c3 > $OUT/c3_1024.txt 2>&1 && timeout -k 10 200 python3 -u tools/gdiag_stamps.py 1024 12 c4 > $OUT/c4_1024.txt 2>&1 || { echo "stamps failed"; tail $OUT/*.txt; exit 1; }
cat $OUT/c3_1.txt $OUT/c3_1024.txt $OUT/c4_1024.txt
timeout -k 10 300 python3 -u tools/generic_prof.py --batch 1024 --iters 12 > $OUT/prof.log 2>&1 && timeout -k 10 300 python3 -u tools/generic_prof.py --batch 1 --iters 12 >> $OUT/prof.log 2>&1 || { echo "prof failed"; tail $OUT/prof.log; exit 1; }
grep generic_prof $OUT/prof.log
