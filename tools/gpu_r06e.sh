set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06e; mkdir -p $OUT
MF_CHAIN_KKT=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --counters > $OUT/probe_generic.json 2> $OUT/probe_generic.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --counters > $OUT/probe_chain.json 2> $OUT/probe_chain.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -k headline -x -v -s --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1
