"""Summarise a rocprofv3 .db (kernel dispatch table) into per-kernel stats."""
import glob
import sqlite3
import sys


def summary(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    rows = cur.execute("""
      select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end-d.start), max(d.end-d.start)
      from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
      group by s.kernel_name order by sum(d.end - d.start) desc""").fetchall()
    total = sum(r[2] for r in rows)
    out = ["%-70s %7s %12s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct")]
    for name, n, tot, avg, mn, mx in rows:
        out.append("%-70s %7d %12.1f %10.2f %10.2f %10.2f %6.2f" % (name[:70], n, tot / 1e3, avg / 1e3, mn / 1e3, mx / 1e3, 100.0 * tot / total))
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for f in glob.glob(p, recursive=True):
            print(f)
            print(summary(f))
