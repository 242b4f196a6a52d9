#!/usr/bin/env python3
"""Print the rocprofv3 --kernel-trace --stats summary (top kernels) of a run directory: prof_kernels.py <db>"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
print("%-100s %7s %12s %11s %6s" % ("kernel", "calls", "total_us", "avg_us", "pct"))
for name, calls, tot, avg, pct in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels "
                                            "order by total_duration desc limit 25"):
    print("%-100s %7d %12.1f %11.2f %6.2f" % (name[:100], calls, tot / 1.0, avg, pct))
