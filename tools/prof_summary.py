"""Dev tool: kernel-time summary (name, calls, total/avg us, %) from a rocprofv3 output
(either the rocpd SQLite .db or the *_kernel_stats.csv), written as CSV for profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, calls, tot, avg, pct in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
            yield name, int(calls), float(tot), float(avg), float(pct)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]), float(r["Percentage"])


def main(src, dst):
    if os.path.isdir(src):
        cand = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True) or \
            glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = cand[0]
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for name, calls, tot, avg, pct in rows_from(src):
            short = name if len(name) < 160 else name[:157] + "..."
            w.writerow([short, calls, round(tot / 1e3, 3), round(avg / 1e3, 3), round(pct, 3)])
    print(open(dst).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
