#!/usr/bin/env python3
"""HBM bytes per launch from two rocprofv3 PMC passes of the same bench command -> profiles/traffic_<workload>.json,
which bench.py reports as roofline.traffic only while the HIP sources still hash to what was measured.

  pmc_traffic.py <workload> <fetch run_results.db> <write run_results.db>

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE reports half of
the bytes of a wide coalesced streaming read on gfx950, so it is doubled; WRITE_SIZE is taken as read.
config2: the k_scan_query launch. config4: the group-by pipeline of one query (every k_group_query / k_partition_*
launch, each once per query) summed, matching bench.py's "group_by_pipeline" timed region."""
import json
import os
import re
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_hash  # noqa: E402

PIPELINE = {"config2": ("k_scan_query",),
            "config4": ("k_group_query", "k_pad_counts", "k_partition_starts", "k_partition_split", "k_partition_reduce",
                        "k_group_ring", "k_ring_reduce"),
            "lds": ("k_group_query",)}
NAME = {"config2": "k_scan_query", "config4": "group_by_pipeline", "lds": "k_group_query_lds"}


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, count(*), avg(value) from counters_collection where counter_name = ? "
                     "group by kernel_name", (counter,)).fetchall()
    return {name: (n, v * 1024.0) for name, n, v in rows}


def main():
    workload, fdb, wdb = sys.argv[1:4]
    fetch, write = per_kernel(fdb, "FETCH_SIZE"), per_kernel(wdb, "WRITE_SIZE")
    parts, total = {}, 0.0
    for name, (n, fb) in sorted(fetch.items()):
        m = re.search(r"::(k_\w+)(<[^>]*>)?\(", name)  # e.g. "void pinot::(anonymous namespace)::k_group_query<6, 3, 512>(..."
        if not m or m.group(1) not in PIPELINE[workload]:
            continue
        wb = write.get(name, (0, 0.0))[1]
        key = m.group(1) + (m.group(2) or "")
        parts[key] = {"dispatches": n, "fetch_bytes_raw": fb, "fetch_bytes_x2": 2 * fb, "write_bytes": wb}
        total += 2 * fb + wb
    out = {"kernel_source_hash": kernel_source_hash(workload), "workload": workload,
           "bytes_per_launch": {NAME[workload]: total}, "parts": parts,
           "_note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of the same bench command; "
                    "FETCH x2 (gfx950 wide-streaming correction; the guide calibrates it for 16-B-per-lane streaming "
                    "reads — the config-4 record reads are 8 B per lane, uncalibrated: fetch_bytes_raw is the bound "
                    "from below), KiB -> bytes"}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "traffic_%s.json" % workload)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
