#!/bin/bash
# HBM traffic of the solver kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over
# tools/traffic_run.py, plus a pass of FP64 VALU instruction counts, summarised (with the copy
# calibration) into pmc_traffic.json.
# usage: tools/pmc_traffic.sh TAG [B]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-traffic}; B=${2:-8192}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/traffic_run.py $B $OUT/nodes.json > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/traffic_run.py $B > $OUT/write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/write.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVES -d $OUT/fp64 -o run --output-format csv -- python3 tools/traffic_run.py $B > $OUT/fp64.log 2>&1 || { echo "fp64 pass failed"; tail -20 $OUT/fp64.log; exit 1; }
F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
P=$(find $OUT/fp64 -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" $OUT/pmc_traffic.json "$P" $OUT/nodes.json
