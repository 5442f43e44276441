set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06m; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
MF_CHAIN_KKT=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_nochain.json 2> $OUT/probe_nochain.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_generic.py -k "headline or record or sixteen or elastic or 15nm or G1 or G3" -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --cstamps --verbose 0 > $OUT/cst_8192.json 2> $OUT/cst_8192.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1100 --cstamps --verbose 0 > $OUT/cst_1100.json 2> $OUT/cst_1100.err
