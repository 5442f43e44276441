"""Sum rocprofv3 counter_collection CSVs per kernel (short name) and print derived ratios.
usage: python tools/pmc_summary.py file.csv [file.csv ...]"""
import csv
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
dur = defaultdict(dict)
meta = {}
for fn in sys.argv[1:]:
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("mf::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][(fn, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"], r["Workgroup_Size"])
for k, c in tot.items():
    if k.startswith("__amd"):
        continue
    print(f"== {k}  vgpr/agpr/lds/scratch/wg = {meta[k]}  dispatches(per pass) ~{len(dur[k]) // max(1, len(sys.argv) - 1)}")
    for n, v in sorted(c.items()):
        print(f"   {n:24s} {v:16.4g}")
    w = c.get("SQ_WAVES", 0)
    if w:
        print(f"   VALU insts/wave {c.get('SQ_INSTS_VALU', 0) / w:10.1f}   LDS insts/wave {c.get('SQ_INSTS_LDS', 0) / w:8.1f}")
    if c.get("SQ_INSTS_VALU_FMA_F64") is not None and w:
        f64 = c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) + c.get("SQ_INSTS_VALU_ADD_F64", 0)
        print(f"   f64 insts/wave {f64 / w:10.1f}  (fma {c.get('SQ_INSTS_VALU_FMA_F64', 0) / w:.0f})")
