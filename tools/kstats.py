#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 results database (rocpd SQLite):
name, calls, average / min / max microseconds. Usage: kstats.py run_results.db"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    q = """select ks.display_name, count(*), avg(k.end-k.start), min(k.end-k.start), max(k.end-k.start)
           from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol ks on k.kernel_id = ks.id
           group by ks.display_name order by sum(k.end-k.start) desc"""
    rows = c.execute(q).fetchall()
    print(f"{'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9}  kernel")
    for name, n, a, lo, hi in rows:
        print(f"{n:6d} {a/1e3:9.2f} {lo/1e3:9.2f} {hi/1e3:9.2f}  {name[:110]}")


if __name__ == "__main__":
    try:
        main(sys.argv[1])
    except BrokenPipeError:      # `| head` closed the pipe
        pass
