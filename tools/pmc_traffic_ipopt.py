"""HBM traffic of the headline (IPOPT-mode, generic chain-family) kernels from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM section), calibrated on tools/traffic_run_ipopt.py's copy kernel
(512 MiB read + 512 MiB written), written to profiles/pmc_traffic_ipopt.json, which bench.py reads for the roofline's
`traffic` (the eval phase: k_geval_chain<q> + k_geval_chain<qd> + k_gasm, per device-counted node evaluation).

usage: python tools/pmc_traffic_ipopt.py FETCH_CSV WRITE_CSV NODES_JSON [OUT_JSON]
"""
import csv
import json
import sys
from collections import defaultdict

COPY_BYTES = 64 * 1024 * 1024 * 8
NODE_BYTES = 952  # SURVEY.md s.8(d) algorithmic bytes per node evaluation (bench.py)


def load(fn, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(fn)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        base = k.split("<")[0].replace("mf::", "")
        if base == "k_geval_chain":
            base += "[q]" if k.rstrip(">").split(",")[-1].strip() == "0" else "[qd]"
        per[base].append(float(r["Counter_Value"]))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    nodes = json.load(open(sys.argv[3]))
    out_path = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic_ipopt.json"
    cal = [k for k in fetch if "elementwise" in k or "copy" in k.lower()]
    fr = max(v for k in cal for v in fetch[k])
    wr = max(v for k in cal for v in write.get(k, [0.0]))
    fs, ws = COPY_BYTES / fr, COPY_BYTES / wr
    res = {"calibration": {"copy_bytes_each_way": COPY_BYTES, "fetch_counter": fr, "write_counter": wr,
                           "bytes_per_fetch_unit": fs, "bytes_per_write_unit": ws},
           "workload": nodes}
    kern = {}
    for k in fetch:
        if k in cal or k.startswith("__amd"):
            continue
        fv, wv = fetch[k], write.get(k, [])
        kern[k] = {"launches": len(fv), "read_bytes_total": sum(fv) * fs, "write_bytes_total": sum(wv) * ws}
        kern[k]["hbm_bytes_per_launch"] = (kern[k]["read_bytes_total"] + kern[k]["write_bytes_total"]) / max(1, len(fv))
    res["kernels"] = kern
    ev = [k for k in ("k_geval_chain[q]", "k_geval_chain[qd]", "k_gasm") if k in kern]
    tot = sum(kern[k]["read_bytes_total"] + kern[k]["write_bytes_total"] for k in ev)
    ne = nodes["node_evals"]
    res["eval_phase_kernels"] = ev
    res["eval_hbm_bytes_per_node_eval"] = tot / ne
    res["eval_read_bytes_per_node_eval"] = sum(kern[k]["read_bytes_total"] for k in ev) / ne
    res["eval_write_bytes_per_node_eval"] = sum(kern[k]["write_bytes_total"] for k in ev) / ne
    res["eval_traffic_over_algorithmic"] = tot / ne / NODE_BYTES
    iters = nodes["eval_launches"]
    res["iteration"] = {"hbm_bytes_per_iteration": sum(v["read_bytes_total"] + v["write_bytes_total"]
                                                       for v in kern.values()) / iters,
                        "per_kernel_bytes_per_iteration": {k: (v["read_bytes_total"] + v["write_bytes_total"]) / iters
                                                           for k, v in kern.items()},
                        "note": "full-batch iterations (the solve capped at the profiled iteration count)"}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
