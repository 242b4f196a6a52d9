#!/usr/bin/env python3
"""Summarise rocprofv3 rocpd databases (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes) as text.

usage: prof_summary.py <dir with prof/ [pmc_fetch/ pmc_write/]> > profiles/<round>/summary.txt
FETCH_SIZE is doubled for wide coalesced streaming reads on gfx950 (MI355X_MICROARCH.md, HBM section);
the raw value is printed next to it."""
import os
import sqlite3
import sys


def rows(db, q):
    c = sqlite3.connect(db)
    try:
        return list(c.execute(q))
    finally:
        c.close()


def main(d):
    db = os.path.join(d, "prof", "run_results.db")
    print("# rocprofv3 --kernel-trace --stats (%s)" % db)
    print("%-90s %8s %14s %12s %7s" % ("kernel", "calls", "total_us", "avg_us", "pct"))
    for name, calls, tot, avg, pct in rows(db, "select name,total_calls,total_duration,average,percentage "
                                               "from top_kernels order by total_duration desc"):
        print("%-90s %8d %14.1f %12.3f %7.2f" % (name[:90], calls, tot / 1.0, avg, pct))
    for cn, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        p = os.path.join(d, sub, "run_results.db")
        if not os.path.exists(p):
            continue
        print("\n# rocprofv3 --pmc %s (%s): per-dispatch average, MB (1e6 B)" % (cn, p))
        q = ("select kernel_name, count(*), avg(value), avg(duration) from counters_collection "
             "where counter_name='%s' group by kernel_name order by avg(duration) desc" % cn)
        for name, n, v, dur in rows(p, q):
            mb = v * 1024 / 1e6
            extra = "  (x2 gfx950 streaming-read correction: %.1f MB)" % (2 * mb) if cn == "FETCH_SIZE" else ""
            print("%-90s n=%-5d %10.2f MB  dur %9.1f us%s" % (name[:90], n, mb, dur / 1000.0, extra))


if __name__ == "__main__":
    main(sys.argv[1])
