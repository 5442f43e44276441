#!/bin/bash
# HBM traffic of the headline IPOPT-mode kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over
# tools/traffic_run_ipopt.py, summarised with the copy calibration into profiles/pmc_traffic_ipopt.json.
# usage: tools/pmc_traffic_ipopt.sh TAG [B [ITERS]]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-traffic_ipopt}; B=${2:-8192}; IT=${3:-30}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/traffic_run_ipopt.py $B $IT $OUT/nodes.json > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/traffic_run_ipopt.py $B $IT > $OUT/write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/write.log; exit 1; }
F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic_ipopt.py "$F" "$W" $OUT/nodes.json $OUT/pmc_traffic_ipopt.json > $OUT/summary.log
