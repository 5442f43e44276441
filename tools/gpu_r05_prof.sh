#!/bin/bash
# Round-5 profile of the headline bench command: rocprofv3 kernel trace + stats (csv), the bench line of the same
# command (its HIP-event eval-phase time), summarised per kernel.  usage: tools/gpu_r05_prof.sh TAG
set -o pipefail
TAG=${1:-r05prof}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --no-generic --inflight 1 > $OUT/bench.json 2> $OUT/prof.log || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
tail -c 400 $OUT/bench.json
python3 - "$OUT" <<'PY'
import csv, json, sys
out = sys.argv[1]
rows = list(csv.reader(open(f"{out}/prof/run_kernel_stats.csv")))
tot = sum(float(r[2]) for r in rows[1:])
with open(f"{out}/rocprof_summary.md", "w") as f:
    f.write("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|\n")
    for r in rows[1:16]:
        n = r[0]
        n = n[:n.find("(")] if "(" in n else n
        f.write(f"| `{n[:80]}` | {r[1]} | {float(r[2]) / 1e6:.2f} | {float(r[3]) / 1e3:.2f} | {100 * float(r[2]) / tot:.1f} |\n")
print(open(f"{out}/rocprof_summary.md").read())
PY
