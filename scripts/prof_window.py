#!/usr/bin/env python3
"""Per-launch durations of one kernel inside the bench's timed window, from a rocprofv3 --kernel-trace database.

    prof_window.py <run_results.db> <kernel-substring> <warmup> <steps> [<launches per step>]

bench.py launches the kernel `launches per step` times per step: the W warm-up steps first, then the K timed steps,
then the timing pass. The launches [W * L, (W + K) * L) are the timed window: their mean / p50 duration (the same
window bench.py's ms_per_step covers) and the gaps between consecutive launches' end and next start (host time per
step the device sat idle) are printed as one JSON line."""
import json
import sqlite3
import sys

import numpy as np

db, sub, W, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
L = int(sys.argv[5]) if len(sys.argv) > 5 else 1
c = sqlite3.connect(db)
rows = [(s, e) for n, s, e in c.execute("select name, start, end from kernels order by start") if sub in n]
win = rows[W * L:(W + K) * L]
if len(win) < K * L:
    sys.exit("only %d launches of %r (need %d)" % (len(rows), sub, (W + K) * L))
dur = np.array([(e - s) / 1e6 for s, e in win])
gaps = np.array([(win[i + 1][0] - win[i][1]) / 1e6 for i in range(len(win) - 1)])
span = (win[-1][1] - win[0][0]) / 1e6
print(json.dumps({"kernel": sub, "launches": len(win), "mean_ms": float(dur.mean()), "p50_ms": float(np.median(dur)),
                  "min_ms": float(dur.min()), "max_ms": float(dur.max()), "first": [round(float(x), 4) for x in dur[:8]],
                  "gap_mean_ms": float(gaps.mean()) if len(gaps) else 0.0,
                  "gap_p50_ms": float(np.median(gaps)) if len(gaps) else 0.0,
                  "window_span_ms": span, "span_per_step_ms": span / K}))
