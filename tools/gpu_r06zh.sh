set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zh; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1100 --cstamps --verbose 0 > $OUT/cst_1100.json 2> $OUT/cst_1100.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --cstamps --verbose 0 > $OUT/cst_8192.json 2> $OUT/cst_8192.err
