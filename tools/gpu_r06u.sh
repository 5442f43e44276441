set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06u; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
MF_CHAIN_RSPEC=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_norspec.json 2> $OUT/probe_norspec.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_generic.py -k "headline or record or sixteen or elastic or 15nm or chain or concurrent" -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
# the round-5 fault command on the stamps build without its diagnostic factorisation path (item 7)
timeout -k 10 300 python -u tools/gdiag_stamps.py 1 400 c3 ipopt > $OUT/gstamps_c3_b1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gdiag_stamps.py 64 400 c3 ipopt > $OUT/gstamps_c3_b64.txt 2>&1
