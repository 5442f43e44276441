set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zb; mkdir -p $OUT
for f in 2 3 4; do
timeout -k 10 400 python -u bench.py --inflight $f --no-extra --no-cpu-baseline > $OUT/bench_if$f.json 2> $OUT/bench_if$f.err || exit 1
done
