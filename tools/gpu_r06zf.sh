set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zf; mkdir -p $OUT
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 8192 --timing --verbose 0 --no-spec > $OUT/probe_nospec.json 2> $OUT/probe_nospec.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1024 --timing --verbose 0 --no-spec > $OUT/probe1024_nospec.json 2> $OUT/probe1024_nospec.err || exit 1
timeout -k 10 300 python -u tools/c2_ipopt_probe.py 1024 --timing --verbose 0 > $OUT/probe1024.json 2> $OUT/probe1024.err
