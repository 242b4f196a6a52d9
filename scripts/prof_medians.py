#!/usr/bin/env python3
"""Median / min / mean duration (us) and launch count of the kernels matching each substring in a rocprofv3
--kernel-trace database: prof_medians.py <run_results.db> <substring> [<substring> ...]"""
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, start, end from kernels order by start"))
for sub in sys.argv[2:]:
    d = np.array([(e - s) / 1e3 for n, s, e in rows if sub in n])
    if len(d):
        print("    %-16s n=%-3d p50 %8.1f us  min %8.1f  mean %8.1f" % (sub, len(d), np.median(d), d.min(), d.mean()))
