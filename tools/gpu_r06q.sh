set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 900 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
