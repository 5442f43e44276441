set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06za; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-extra --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
