set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zi; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe.json 2> $OUT/probe.err || exit 1
MF_GKKT_OCC=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_nokktocc.json 2> $OUT/probe_nokktocc.err || exit 1
MF_GLS_OCC=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_nolsocc.json 2> $OUT/probe_nolsocc.err || exit 1
MF_GKKT_OCC=0 MF_GLS_OCC=0 timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 > $OUT/probe_noocc.json 2> $OUT/probe_noocc.err
