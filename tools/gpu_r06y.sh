set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06y; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_generic.py tests/test_gpu_bk.py -k "headline or record or sixteen or elastic or 15nm or chain or concurrent or bunch" -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
