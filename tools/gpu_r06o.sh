set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06o; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bk.py -q --timeout 200 --timeout-method thread > $OUT/bk.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1100 --cstamps --verbose 0 > $OUT/cst_1100.json 2> $OUT/cst_1100.err
