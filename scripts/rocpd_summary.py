"""Summarise a rocprofv3 rocpd SQLite database (default output format) as a kernel-stats CSV:
python scripts/rocpd_summary.py <run_results.db> [out.csv]"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0] if not name.startswith("void at::") else name[:120]


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([short(name), calls, tot, round(avg, 1), round(100.0 * tot / total, 3), mn, mx])


if __name__ == "__main__":
    main()
