#!/usr/bin/env python3
"""Per-kernel average of every PMC counter in a rocprofv3 --pmc run: pmc_summary.py <run_results.db>"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) from counters_collection "
                 "group by kernel_name, counter_name order by avg(duration) desc").fetchall()
for name, cn, n, v, dur in rows:
    print("%-90s %-24s n=%-4d avg %16.1f  dur %10.1f us" % (name[:90], cn, n, v, dur / 1000.0))
