#!/bin/bash
# Solve probe per library variant (MF_LIB) after the parity tests of the default library.
# usage: tools/variant_probe.sh TAG B lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; B=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for L in "$@"; do
  echo "== $L"
  MF_LIB=$L timeout -k 10 300 python -u tools/solve_probe.py $B > $OUT/probe_$L.log 2>&1 || { tail -20 $OUT/probe_$L.log; exit 1; }
  grep -v amdgpu.ids $OUT/probe_$L.log
done
