set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06p; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputests.txt 2>&1
