set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06g; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 --counters > $OUT/probe_chain.json 2> $OUT/probe_chain.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_headline.py -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
