set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_runtime.py tests/test_gpu_generic.py -k "headline or runtime or sixteen or elastic or 15nm" -x -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
timeout -k 10 700 python -u bench.py --no-generic > $OUT/bench.json 2> $OUT/bench.err || exit 1
exit $rc
