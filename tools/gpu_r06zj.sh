set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zj; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err
