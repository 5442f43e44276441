"""Per-kernel durations from a rocprofv3 kernel trace (csv), split by launch grid: median duration of
the launches at the full running set (largest grid) and the total over all launches.
usage: python tools/trace_full.py gpurun_out/TAG/prof/run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "mf::" not in n:
        continue
    nm = n.split("(")[0].replace("void ", "")
    d[nm].append((int(r["Grid_Size_X"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
tot_all = sum(x[1] for v in d.values() for x in v)
print(f"{'kernel':34s} {'calls':>6s} {'full':>5s} {'med_full_us':>11s} {'total_ms':>9s} {'share':>6s}")
for k, v in sorted(d.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
    g = max(x[0] for x in v)
    full = sorted(x[1] for x in v if x[0] == g)
    tot = sum(x[1] for x in v)
    print(f"{k:34s} {len(v):6d} {len(full):5d} {full[len(full) // 2]:11.1f} {tot / 1e3:9.1f} {tot / tot_all:6.3f}")
