"""Kernel statistics (calls, total / average duration, share) from a rocprofv3 rocpd database (ROCm 7 writes
`<dir>/<name>_results.db` by default), in the layout of rocprofv3's --stats kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/r04h_prof/run_results.db [--md title] > profiles/<round>_....csv|md
"""
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"SELECT {name}, start, end FROM kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3  # ns -> us
    tot = sum(v[1] for v in agg.values())
    return sorted(((n, v[0], v[1], v[1] / v[0], 100.0 * v[1] / tot) for n, v in agg.items()), key=lambda r: -r[2])


if __name__ == "__main__":
    out = stats(sys.argv[1])
    if "--md" in sys.argv:
        print(f"# {sys.argv[sys.argv.index('--md') + 1]}\n")
        print("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|")
        for n, k, t, a, p in out:
            short = n if len(n) < 90 else n[:87] + "..."
            print(f"| `{short}` | {k} | {t:.1f} | {a:.3f} | {p:.2f} |")
    else:
        print('"Name","Calls","TotalDurationUs","AverageUs","Percentage"')
        for n, k, t, a, p in out:
            print(f'"{n}",{k},{t:.3f},{a:.3f},{p:.2f}')
