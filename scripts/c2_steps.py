"""Config-2 per-step breakdown: wall time of each step vs. its kernel time (HIP events, timing=1) and the host-phase
split (debug.host_phases=1 on stderr), to attribute the time outside the kernel (item: query-level >= 70 %)."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--config", default="")
ap.add_argument("--sleep-us", type=float, default=0.0, help="host idle between steps")
args = ap.parse_args()

import torch  # noqa: E402
from pinot_amd import GpuEngine, ServerQueryExecutor  # noqa: E402

torch.cuda.set_device(0)
eng = GpuEngine(0, args.config or None)
ex = ServerQueryExecutor(eng)
segs = [eng.register_synthetic("fact_%d" % i, 125_000_000, bench.COLUMNS, bench.BASE_SEED + i) for i in range(8)]
eng.synchronize()
q = ex.prepare(bench.QUERY)
for _ in range(5):
    ex.process_query(q, segs)
for timing in (0, 1):
    eng.set_config("timing=%d" % timing)
    wall, abi, kern = [], [], []
    for _ in range(args.steps):
        if args.sleep_us:
            t = time.perf_counter() + args.sleep_us / 1e6
            while time.perf_counter() < t:
                pass
        t0 = time.perf_counter()
        res, st = ex.process_query(q, segs)
        wall.append((time.perf_counter() - t0) * 1e3)
        abi.append(st.host_ms)
        kern.append(eng.last_kernel_ms(0)[0] if timing else st.device_ms)
    wall, abi, kern = map(np.array, (wall, abi, kern))
    print("timing=%d wall p50 %.4f mean %.4f min %.4f max %.4f | abi p50 %.4f | kernel(%s) p50 %.4f mean %.4f min %.4f "
          "max %.4f | wall-kernel p50 %.4f" % (timing, np.median(wall), wall.mean(), wall.min(), wall.max(),
                                             np.median(abi), "events" if timing else "device clock", np.median(kern),
                                             kern.mean(), kern.min(), kern.max(), np.median(wall - kern)))
    print("   walls", " ".join("%.3f" % x for x in wall[:20]))
    print("   kerns", " ".join("%.3f" % x for x in kern[:20]))
