set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zm; mkdir -p $OUT
timeout -k 10 900 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
