set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
