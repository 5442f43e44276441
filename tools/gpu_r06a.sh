set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c2 --output-format csv -- python3 -u tools/c2_ipopt_probe.py 8192 --counters > $OUT/probe.json 2> $OUT/probe.err
