"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs,
MI355X_MICROARCH.md HBM section), calibrated on the copy kernel of tools/traffic_run.py (known
512 MiB read + 512 MiB written), written to profiles/pmc_traffic.json for bench.py.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV [OUT_JSON [FP64_CSV [NODES_JSON]]]
NODES_JSON (written by tools/traffic_run.py) adds per-node-evaluation totals for k_eval_node, the
unit bench.py scales by its own node-evaluation count (launch sizes vary with the running set).
FP64_CSV (SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 pass) adds executed FP64 flops per launch:
64 lanes x (2 FMA + MUL + ADD) per wave instruction, an upper bound (masked lanes count).
"""
import csv
import json
import sys
from collections import defaultdict

COPY_BYTES = 64 * 1024 * 1024 * 8


def load(fn, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(fn)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        base = k.split("<")[0].replace("mf::", "")
        if base == "k_eval_node" and "<" in k:  # one launch per direction class: keep them apart
            base += "[q]" if k.rstrip(">").split(",")[-1].strip() == "0" else "[qd]"
        per[base].append(float(r["Counter_Value"]))
    return per


def add_eval_phase(res, node_evals=None):
    """k_eval_node as the solver's phase 0: the q-class and qd-class launches of one iteration
    (one each per iteration), summed -- the unit bench.py's HIP-event timing uses."""
    # the q directions run as k_eval_q (one wavefront per direction x 64 nodes) since 2ceaaeb
    q, qd = res.get("k_eval_q") or res.get("k_eval_node[q]"), res.get("k_eval_node[qd]")
    if not q or not qd:
        return
    ph = {"launches": q["launches"], "note": "phase = k_eval_q<..> (q directions) + k_eval_node<..,1> (qd directions), "
          "per-iteration sum"}
    for f in ("read_bytes_per_launch", "write_bytes_per_launch", "hbm_bytes_per_launch", "fp64_flops_per_launch"):
        if f in q and f in qd:
            ph[f] = q[f] + qd[f]
    if node_evals:
        ph["node_evals"] = node_evals
        for f, g in (("hbm_bytes_per_launch", "hbm_bytes_per_node_eval"),
                     ("read_bytes_per_launch", "read_bytes_per_node_eval"),
                     ("write_bytes_per_launch", "write_bytes_per_node_eval"),
                     ("fp64_flops_per_launch", "fp64_flops_per_node_eval")):
            if f in ph:
                ph[g] = ph[f] * ph["launches"] / node_evals
    res["k_eval_node"] = ph


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out_path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    flops = {}
    if len(sys.argv) > 4:
        fma, mul, add = (load(sys.argv[4], c) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                        "SQ_INSTS_VALU_ADD_F64"))
        for k in fma:
            n = max(len(fma[k]), 1)
            flops[k] = 64.0 * (2.0 * sum(fma[k]) + sum(mul.get(k, [])) + sum(add.get(k, []))) / n
    # calibration: the largest elementwise (copy) dispatch moved exactly COPY_BYTES each way
    cal_keys = [k for k in fetch if "elementwise" in k or "copy" in k.lower()]
    fr = max(v for k in cal_keys for v in fetch[k])
    wr = max(v for k in cal_keys for v in write.get(k, [0.0]))
    f_scale, w_scale = COPY_BYTES / fr, COPY_BYTES / wr
    res = {"calibration": {"copy_bytes_each_way": COPY_BYTES, "fetch_counter": fr, "write_counter": wr,
                           "bytes_per_fetch_unit": f_scale, "bytes_per_write_unit": w_scale}}
    for k in fetch:
        if k in cal_keys or k.startswith("__amd"):
            continue
        fv, wv = fetch[k], write.get(k, [])
        n = max(len(fv), 1)
        rd = sum(fv) * f_scale / n
        wt = sum(wv) * w_scale / max(len(wv), 1)
        res[k] = {"launches": len(fv), "read_bytes_per_launch": rd, "write_bytes_per_launch": wt,
                  "hbm_bytes_per_launch": rd + wt}
        if k in flops:
            res[k]["fp64_flops_per_launch"] = flops[k]
    nodes = json.load(open(sys.argv[5]))["node_evals"] if len(sys.argv) > 5 else None
    add_eval_phase(res, nodes)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
