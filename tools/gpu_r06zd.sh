set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zd; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
timeout -k 10 400 python -u bench.py --no-extra --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
