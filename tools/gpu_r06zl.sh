set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zl; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --no-generic --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
