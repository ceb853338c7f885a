"""Per-(kernel, grid) duration summary of a rocprofv3 SQLite result (rocprofv3 -d DIR -o run
without --output-format csv writes DIR/run_results.db).

    python tools/rocpd_stats.py gpurun_out/prof_b256/run_results.db [--match decode] [--csv out.csv]

Prints calls, total / mean / min duration (us) and share of the summed kernel time, largest
first; --csv writes the same table.
"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default=None, help="only kernels whose name contains this")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    q = ("select name, grid_x, grid_y, grid_z, count(*), sum(duration), avg(duration), min(duration) "
         "from kernels group by name, grid_x, grid_y, grid_z order by sum(duration) desc")
    rows = [r for r in cur.execute(q).fetchall() if a.match is None or a.match in r[0]]
    tot = sum(r[5] for r in rows) or 1
    out = csv.writer(open(a.csv, "w", newline="")) if a.csv else None
    hdr = ["kernel", "grid", "calls", "total_us", "mean_us", "min_us", "share"]
    if out:
        out.writerow(hdr)
    print("\t".join(hdr))
    for name, gx, gy, gz, n, s, m, mn in rows:
        line = [name[:110], f"{gx}x{gy}x{gz}", n, round(s / 1e3, 1), round(m / 1e3, 2), round(mn / 1e3, 2),
                round(s / tot, 4)]
        if out:
            out.writerow([name] + line[1:])
        print("\t".join(map(str, line)))


if __name__ == "__main__":
    sys.exit(main())
