set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06n; mkdir -p $OUT
timeout -k 10 60 ./tools/bk_bench.bin > $OUT/bk_bench.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1100 --cstamps --verbose 0 > $OUT/cst_1100.json 2> $OUT/cst_1100.err
