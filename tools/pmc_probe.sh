#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/solve_probe.py.  usage: tools/pmc_probe.sh TAG B "grp1" "grp2" ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; B=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for grp in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/solve_probe.py $B > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/pmc$i.log; exit 1; }
  i=$((i+1))
done
find $OUT -name "*counter_collection*.csv" > $OUT/files.txt
