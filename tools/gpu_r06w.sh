set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06w; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
timeout -k 10 300 python -u tools/gdiag_stamps.py 64 400 c3 ipopt > $OUT/gstamps_c3_b64.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputests.txt 2>&1
