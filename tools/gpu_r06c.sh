set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_runtime.py tests/test_gpu_generic.py -k "headline or runtime or sixteen or elastic or 15nm" -v --timeout 400 --timeout-method thread -s > $OUT/pytest.log 2>&1
