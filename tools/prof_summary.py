"""Per-kernel summary (calls, total, average, share) from a rocprofv3 output:
either a rocpd SQLite database (*_results.db) or a *_kernel_stats.csv."""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    return [(n, k, s, a, lo, hi) for n, k, s, a, lo, hi in rows]


def main(src, dst):
    rows = from_db(src)
    tot = sum(r[2] for r in rows)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, k, s, a, lo, hi in rows:
            w.writerow([n, k, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
