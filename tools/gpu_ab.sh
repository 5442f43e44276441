#!/bin/bash
# A/B of library variants on one box: -m gpu tests on the default library, then the bench (no CPU
# baseline, no extras) per library in the order given, twice (ABAB), and a WRITE_SIZE/FETCH_SIZE pass
# of the default library.  usage: tools/gpu_ab.sh TAG lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
MF_LIB=${TEST_LIB:-libmpcfatigue.so} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for R in 1 2; do
  for L in "$@"; do
    MF_LIB=$L timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra > $OUT/bench_${L}_$R.json 2> $OUT/bench_${L}_$R.err || { tail -20 $OUT/bench_${L}_$R.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_${L}_$R.json').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$L', round(d['value'],1), 'h/s', round(d['ms_per_step'],1), 'ms/step', 'iters', round(d['config']['mean_iters'],2), {a: round(b,1) for a,b in k.items()})"
  done
done
if [ -n "$PMC" ]; then MF_LIB=${PMC_LIB:-libmpcfatigue.so} bash tools/pmc_traffic.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -30 $OUT/pmc.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/pmc/pmc_traffic.json')); print({k: (round(v['read_bytes_per_launch']/1e6,1), round(v['write_bytes_per_launch']/1e6,1)) for k,v in d.items() if isinstance(v,dict) and 'read_bytes_per_launch' in v})"
fi
