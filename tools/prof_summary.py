"""Summarise a rocprofv3 --kernel-trace --stats output (the sqlite database, or the kernel_stats.csv of
--output-format csv) into profiles/ (markdown)."""
import csv
import glob
import sqlite3
import sys


def main(db_glob: str, out: str, title: str):
    db = sorted(glob.glob(db_glob, recursive=True))[0]
    if db.endswith(".csv"):
        rows = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                 float(r["Percentage"])) for r in csv.DictReader(open(db))]
    else:
        c = sqlite3.connect(db)
        rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w") as f:
        f.write(f"# {title}\n\nSource: `{db}` (rocprofv3 --kernel-trace --stats), durations in microseconds.\n\n")
        f.write("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|\n")
        ev = []
        for name, calls, tot, avg, pct in rows:
            short = name.split("(")[0].replace("void ", "")
            if any(k in short for k in ("k_eval_node<", "k_eval_q<", "k_eval_dir<")):  # the direction classes
                ev.append((calls, tot, avg, pct))
            if len(short) > 80:
                short = short[:77] + "..."
            f.write(f"| `{short}` | {calls} | {tot:.1f} | {avg:.3f} | {pct:.2f} |\n")
        if len(ev) == 2:
            # the solver's phase 0 is one launch of each direction class per iteration
            f.write(f"| **k_eval_node phase** (q + qd direction launches) | {ev[0][0]} | {ev[0][1] + ev[1][1]:.1f} | "
                    f"{ev[0][2] + ev[1][2]:.3f} | {ev[0][3] + ev[1][3]:.2f} |\n")
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel summary")
