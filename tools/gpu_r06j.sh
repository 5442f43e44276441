set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06j; mkdir -p $OUT
MF_CHAIN_EVAL=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_old.json 2> $OUT/probe_old.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_new.json 2> $OUT/probe_new.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_generic.py -k "headline or record or sixteen or elastic or 15nm or G1 or G3" -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
