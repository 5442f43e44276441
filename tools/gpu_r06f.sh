set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06f; mkdir -p $OUT
MF_CHAIN_KKT=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_generic.json 2> $OUT/probe_generic.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_chain.json 2> $OUT/probe_chain.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c2 --output-format csv -- python3 -u tools/c2_ipopt_probe.py 8192 --verbose 0 > $OUT/prof.json 2> $OUT/prof.err
