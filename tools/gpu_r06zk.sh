set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zk; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
