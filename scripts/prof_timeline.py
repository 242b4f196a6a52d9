#!/usr/bin/env python3
"""One config-4 query's device timeline from a rocprofv3 --kernel-trace --memory-copy-trace database: the kernels
and memory copies of the last query (after the last COUNT pass), in start order, with gaps.
usage: prof_timeline.py <results.db>"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
kv = next(t for t in tables if t.lower() in ("kernels", "rocpd_kernel_dispatch")) if any(
    t.lower() in ("kernels",) for t in tables) else None
rows = []
if "kernels" in tables:
    for name, s, e in c.execute("select name, start, end from kernels"):
        rows.append((s, e, "K " + name[:90]))
if "memory_copies" in tables:
    cols = [r[1] for r in c.execute("pragma table_info(memory_copies)")]
    sz = "size" if "size" in cols else None
    for r in c.execute("select start, end, %s from memory_copies" % (sz or "0")):
        rows.append((r[0], r[1], "C %d bytes" % (r[2] or 0)))
rows.sort()
marks = [i for i, r in enumerate(rows) if "GB_COUNT" in r[2] or "k_group_query<2" in r[2] or "k_group_ring" in r[2]]
# the last three queries' windows (each from its ring / COUNT pass to the next one)
starts = marks[-3:] if marks else [max(0, len(rows) - 40)]
for wi, first in enumerate(starts):
    last = starts[wi + 1] if wi + 1 < len(starts) else len(rows)
    prev = rows[first][0]
    t0 = prev
    print("---- query window %d" % wi)
    for s, e, what in rows[first:last]:
        print("%9.1f us  gap %8.1f  dur %8.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, what))
        prev = e
print("tables:", ", ".join(tables))
