#!/usr/bin/env python3
"""Benchmark: rows scanned/s per query on synthetic dict-encoded fact segments (BASELINE.json metric).

Headline workload (BASELINE.json configs[1]): 8 segments x 125,000,000 docs per GPU
(1B rows), 10 fixed-bit dictionary-encoded INT columns d0..d9 with cardinalities
{16, 100, 1000, 4096, 10000, 65536, 1000, 1000, 2^20, 1000} (bits {4,7,10,12,14,16,10,10,20,10}),
generated in HBM (seeded splitmix64), query
    SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1, 3, 5, 7)
The same run also measures BASELINE.json configs[3] on the same segments and embeds it as "config4" in the line:
the 1M-key scan-filter-group-by the north star's >= 70 % target names,
    SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d6, d7 TOP 10
(num.groups.limit = 1,000,000 so no group is dropped). --workload config4 makes it the headline instead.

One step = one query over all of the job's segments, results back on the host. GPUs (weak scaling, 8 segments per
GPU, global segment i on GPU i mod N — config 5 at N = 8):
  * N = 1 (default): one engine (pinot_gpu_aggregate / _group_by); --path server runs the same query through the
    multi-GPU server with one GPU instead.
  * --gpus N without WORLD_SIZE: ONE process serving N GPUs (pinot_gpu_server_create over devices 0..N-1: one
    engine per GPU, RCCL communicators inside the library, the merge on the devices).
  * under torch.distributed.run (WORLD_SIZE = N = --gpus): one process per GPU, each a rank of the library's
    server (pinot_gpu_server_create_rank; the communicator id is shared through a gloo process group, which also
    carries the barriers and the max-over-ranks timing); the merge runs over RCCL inside the library.
The merge's own time (all-gathers, reduce-scatter, gather) is reported per phase in "merge_phases_ms".

Prints ONE JSON line (rank 0).
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))

COLUMNS = [("d0", 16), ("d1", 100), ("d2", 1000), ("d3", 4096), ("d4", 10000), ("d5", 65536), ("d6", 1000),
           ("d7", 1000), ("d8", 1 << 20), ("d9", 1000)]
QUERY = "SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1, 3, 5, 7)"
CONFIG4 = "SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM fact WHERE d2 < 800 GROUP BY d6, d7 TOP 10"
CONFIG4_BYTES_PER_ROW = (10 + 10 + 10 + 20 + 16) / 8  # d2 filter + d6, d7 keys + d8 SUM/AVG + d5 HLL
# the small-key-space group-by (1,600 groups): per-block LDS-privatised accumulators, one launch (GB_LDS)
LDS_QUERY = "SELECT COUNT(*), SUM(d8), AVG(d8) FROM fact WHERE d2 < 800 GROUP BY d0, d1 TOP 10"
LDS_BYTES_PER_ROW = (10 + 4 + 7 + 20) / 8  # d2 filter + d0, d1 keys + d8 SUM/AVG
BASE_SEED = 0x5EED0000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (8.0 TB/s spec)
BITS = {n: max(1, (c - 1).bit_length()) for n, c in COLUMNS}
# device sources each workload's kernels are built from (a PMC traffic profile is reported only for these exact bytes)
KERNEL_SOURCES = {
    "config2": ("fused.hip", "scan.hip", "kernels.hip", "fused_common.h", "common.h", "device.h", "kernels.h"),
    "config4": ("fused_group.hip", "group_ring.hip", "group_lq.h", "groupby.hip", "kernels.hip", "fused_common.h",
                "common.h", "device.h", "kernels.h"),
    "lds": ("fused_group.hip", "group_lq.h", "groupby.hip", "fused_common.h", "common.h", "device.h", "kernels.h"),
}
WORKLOAD_QUERY = {"config2": QUERY, "config4": CONFIG4, "lds": LDS_QUERY}


def algorithmic_bytes(num_docs):
    """Per-segment algorithmic HBM bytes of each kernel class, summed over its launches:
    k_leaf: d2 leaf (d2 stream + bitset write) and d0 leaf AND-ed in (d0 stream + bitset read + write);
    k_colagg: d8 stream + bitset read. Query minimum: the three packed streams only (4.25 B/row)."""
    bitset = (num_docs + 63) // 64 * 8
    filt = (num_docs * BITS["d2"] + 7) // 8 + bitset + (num_docs * BITS["d0"] + 7) // 8 + 2 * bitset
    agg = (num_docs * BITS["d8"] + 7) // 8 + bitset
    query = sum((num_docs * BITS[c] + 7) // 8 for c in ("d0", "d2", "d8"))
    return filt, agg, query


def host_cpu_info():
    """The host the CPU baseline runs on: CPUs this process may use (cgroup CPU quota, else the affinity mask —
    what Java's availableProcessors() reports), the machine's count, and the CPU model (lscpu's 'Model name')."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["model"] = model
    info["available_processors"] = min(x for x in (quota, info["affinity"]) if x)
    return info


def cpu_baseline(threads, segs, docs, min_seconds=10.0):
    """Reference-faithful C executor (oracle/faithful.c) on a bounded sample of the same workload.

    The sample (segs x docs rows of the same synthetic table) is queried repeatedly until at least
    `min_seconds` of CPU work have been timed; the median run is reported."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import faithful
    from concurrent.futures import ThreadPoolExecutor
    faithful.load()
    t0 = time.time()
    # generate the sample columns in parallel (ctypes releases the GIL)
    table = faithful.SyntheticTable(COLUMNS, docs, 0, BASE_SEED, needed=set())
    jobs = {}
    with ThreadPoolExecutor(min(threads, 32)) as ex:
        for s in range(segs):
            for i, (name, card) in enumerate(COLUMNS):
                if name in ("d0", "d2", "d8"):
                    jobs[(s, name)] = ex.submit(faithful.synth_column, BASE_SEED + s, i, card, docs)
    table.segments = [{n: jobs[(s, n)].result() for n in ("d0", "d2", "d8")} for s in range(segs)]
    gen_s = time.time() - t0
    leaves = [("d2", ("RANGE", 100, 600)), ("d0", ("IN", [1, 3, 5, 7]))]
    rows = segs * docs
    out = {}
    for optimized in (False, True):
        faithful.run_and_count_sum(table, leaves, "d8", threads, optimized)  # warm-up (page-in)
        times = []
        t_start = time.time()
        while len(times) < 3 or time.time() - t_start < min_seconds:
            t0 = time.time()
            cnt, sm = faithful.run_and_count_sum(table, leaves, "d8", threads, optimized)
            times.append(time.time() - t0)
        times.sort()
        med = times[len(times) // 2]
        what = ("oracle/faithful.c pinot_fast_run: optimised CPU executor (64-doc batch unpack from big-endian words, "
                "word-mask predicates, exact integer sums, 64K-doc ranges over the threads)" if optimized else
                "oracle/faithful.c per-doc iterator executor (reference-faithful C restatement: the Java executor "
                "cannot run here, no JVM)")
        out["optimized" if optimized else "faithful"] = {
            "value": rows / med, "unit": "rows/s", "cores": host_cpu_info()["available_processors"],
            "threads": threads, "kind": "port",
            "sample": "%d segments x %d docs of the same synthetic table and query, %d runs over %.1fs of CPU work "
                      "(median %.3fs; data generated in %.1fs); %s" % (segs, docs, len(times), sum(times), med, gen_s,
                                                                       what),
            "check": {"count": cnt, "sum": sm}}
    assert out["optimized"]["check"] == out["faithful"]["check"], out
    res = dict(out["faithful"])
    res["optimized"] = out["optimized"]
    return res


def cpu_baseline_config4(threads, segs, docs, min_seconds=10.0, workload="config4"):
    """Reference-faithful group-by (oracle/faithful.c: per-doc readInt, INT_MAP group ids, double / AvgPair /
    HyperLogLog holders per group, then the CombineGroupByOperator merge) on a bounded sample of the config-4
    workload (or the LDS one: GROUP BY d0, d1, no HLL), repeated until `min_seconds` of CPU work; the median run
    is reported."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import faithful
    from concurrent.futures import ThreadPoolExecutor
    faithful.load()
    c4 = workload == "config4"
    g0, g1, hcol = ("d6", "d7", "d5") if c4 else ("d0", "d1", None)
    need = ("d2", "d8", g0, g1) + ((hcol,) if hcol else ())
    t0 = time.time()
    table = faithful.SyntheticTable(COLUMNS, docs, 0, BASE_SEED, needed=set())
    jobs = {}
    with ThreadPoolExecutor(min(threads, 32)) as ex:
        for s in range(segs):
            for i, (name, card) in enumerate(COLUMNS):
                if name in need:
                    jobs[(s, name)] = ex.submit(faithful.synth_column, BASE_SEED + s, i, card, docs)
    table.segments = [{n: jobs[(s, n)].result() for n in need} for s in range(segs)]
    gen_s = time.time() - t0
    leaves = [("d2", ("RANGE", 0, 800))]
    times = []
    t_start = time.time()
    while len(times) < 2 or time.time() - t_start < min_seconds:
        t0 = time.time()
        groups, cnt, sm = faithful.run_group_by(table, leaves, g0, g1, "d8", hcol, threads)
        times.append(time.time() - t0)
    times.sort()
    med = times[len(times) // 2]
    rows = segs * docs
    return {"value": rows / med, "unit": "rows/s", "cores": host_cpu_info()["available_processors"], "threads": threads,
            "kind": "port",
            "sample": "%d segments x %d docs of the same synthetic table and %s query, %d runs over %.1fs "
                      "(median %.3fs, %d groups; data generated in %.1fs); oracle/faithful.c per-doc INT_MAP "
                      "group-by + CombineGroupByOperator merge (reference-faithful C restatement: no JVM here)" %
                      (segs, docs, workload, len(times), sum(times), med, groups, gen_s)}


def kernel_source_hash(workload="config2"):
    """Hash of the device code a workload's kernels are built from (KERNEL_SOURCES): the PMC traffic figures are
    reported only while the sources still hash to the ones they were measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(REPO, "incubator-pinot_amd", "csrc")
    for f in sorted(KERNEL_SOURCES[workload]):
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + fh.read())
    return h.hexdigest()[:16]


def measured_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from profiles/traffic_<workload>.json, written by
    scripts/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE passes; None unless that file was measured on
    exactly these kernel sources."""
    path = os.path.join(REPO, "profiles", "traffic_%s.json" % workload)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("kernel_source_hash") != kernel_source_hash(workload):
        return None
    return t.get("bytes_per_launch", {}).get(kernel)


class Job:
    """The GPUs and segments of this process, and how one query runs over them."""

    def __init__(self, args, world, rank, local_rank):
        from pinot_amd import GpuEngine, GpuServer, ServerExecutor, ServerQueryExecutor
        cfg = args.engine_config or None
        self.world, self.rank = world, rank
        self.server = None
        self.dist = None
        if world > 1:
            # control plane only (communicator id, barriers, max-over-ranks timing); the merge is RCCL in the .so
            import torch
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist
            from pinot_amd import GpuServer as GS
            uid = torch.tensor(list(GS.unique_id()) if rank == 0 else [0] * 128, dtype=torch.uint8)
            dist.broadcast(uid, 0)
            self.server = GpuServer.rank(local_rank, world, rank, bytes(uid.tolist()), cfg)
            self.path = "rank"
        elif args.gpus > 1 or args.path == "server":
            self.server = GpuServer(list(range(args.gpus)), cfg)
            self.path = "server"
        else:
            self.engine = GpuEngine(0, cfg)
            self.path = "engine"
        if self.server is not None:
            self.engines = self.server.engines
            self.ex = ServerExecutor(self.server, num_groups_limit=1_000_000)
        else:
            self.engines = [self.engine]
            self.ex = ServerQueryExecutor(self.engine, num_groups_limit=1_000_000)
        self.n_gpus = world if world > 1 else len(self.engines)
        self.segs = []
        t0 = time.time()
        local = len(self.engines)
        for s in range(args.segments * local):
            gidx = s * world + rank  # global segment i is served by rank i mod world
            eng = self.engines[s % local]  # ... and by engine i mod N within one process
            self.segs.append(eng.register_synthetic("fact_%d" % gidx, args.docs, COLUMNS, BASE_SEED + gidx))
        for e in self.engines:
            e.synchronize()
        self.load_s = time.time() - t0
        self.total_rows = self.n_gpus * args.segments * args.docs

    def step_fn(self, query_text, group_by):
        q = self.ex.prepare(query_text)  # compiled + marshalled once; every step still prunes, plans and runs
        if not group_by:
            return lambda: self.ex.process_query(q, self.segs)
        # what the server hands the broker: the group-by trimmed on the device (CombineGroupByOperator's
        # AggregationGroupByTrimmingService, TOP 10 -> 5,000 groups per function; on the multi-GPU server each rank
        # trims its own key range before the gather to rank 0) serialized as DataTable bytes, handed on as a view of
        # the native buffer (as a transport would send it; no Python-side copy)
        return lambda: self.ex.process_query_datatable(q, self.segs, trim=True, zero_copy=True)

    def set_config(self, cfg):
        for e in self.engines:
            e.set_config(cfg)

    def synchronize(self):
        for e in self.engines:
            e.synchronize()

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.barrier()
        if self.server is not None:
            self.server.close()
        if self.dist:
            self.dist.destroy_process_group()


def timed_steps(job, step, steps, warmup, warmup_s=0.0):
    """W untimed warm-ups (continued, still untimed, until they have run warmup_s seconds: the GPU's clocks ramp over
    the first few hundred ms of work on some boxes), then exactly K steps bracketed by barrier + device sync; max over
    ranks. Returns the extra warm-up steps too."""
    import torch
    # the harness's own collector pauses stay out of the timed steps (the C-ABI call has none); collected before the
    # warm-ups so the timed steps follow them with no idle gap on the device
    gc.collect()
    gc.disable()
    tw = time.perf_counter()
    for _ in range(warmup):
        step()
    # the extra count from the W warm-ups' pace, the same on every rank (a step may hold collectives)
    extra = 0
    if warmup > 0:
        spent = time.perf_counter() - tw
        extra = int(min(5000.0, job.max_over_ranks(max(0.0, (warmup_s - spent) / (spent / warmup)))) + 0.999)
    for _ in range(extra):
        step()
    job.barrier()
    torch.cuda.synchronize()
    job.synchronize()
    t0 = time.perf_counter()
    step_ms, abi_ms, dev_ms = [], [], []
    res = st = None
    for _ in range(steps):
        ts = time.perf_counter()
        res, st = step()  # synchronous: results are on the host when it returns
        step_ms.append((time.perf_counter() - ts) * 1e3)
        abi_ms.append(st.host_ms)
        dev_ms.append(st.device_ms)
    job.synchronize()
    torch.cuda.synchronize()
    job.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    timed_steps.extra_warmup = extra
    return job.max_over_ranks(elapsed), (step_ms, dev_ms), abi_ms, res, st


def kernel_pass(job, step, reps):
    """Per-kernel device time (HIP events on engine 0's own stream) and the server's merge phases, in a separate
    pass with timing=1."""
    job.set_config("timing=1")
    kt = {0: [0.0, 0], 1: [0.0, 0]}
    phases = {}
    eng = job.engines[0]
    for _ in range(reps):
        step()
        for k in (0, 1):
            ms, n = eng.last_kernel_ms(k)
            kt[k][0] += ms
            kt[k][1] += n
        if job.server is not None:
            for k, v in job.server.last_phases().items():
                phases[k] = phases.get(k, 0.0) + v / reps
    job.set_config("timing=0")
    return kt, phases


def measure(job, args, workload):
    gb = workload != "config2"  # a group-by workload (config 4, or the LDS-privatised small-key-space one)
    c4 = workload == "config4"
    text = WORKLOAD_QUERY[workload]
    step = job.step_fn(text, gb)
    steps = args.steps if workload == args.workload else args.c4_steps
    elapsed, (step_ms, dev_ms), abi_ms, res, st = timed_steps(job, step, steps, args.warmup, args.warmup_seconds)
    ms_per_step = elapsed * 1000.0 / steps
    value = job.total_rows * steps / elapsed
    reps = max(3, min(steps, 10))
    kt, phases = kernel_pass(job, step, reps)
    segs_here = args.segments  # per GPU: engine 0's share
    kern = {}
    if c4:
        alg = segs_here * args.docs * CONFIG4_BYTES_PER_ROW
        # the group-by pipeline of one query on engine 0, one timed region: the ring plan (k_group_ring ->
        # k_ring_reduce) or the counted plan (COUNT -> scan -> EMIT2 -> k_partition_reduce), as `plan` says
        names = ((1, "group_by_pipeline", alg),)
        query_b = alg
    elif gb:
        alg = segs_here * args.docs * LDS_BYTES_PER_ROW
        names = ((1, "k_group_query_lds", alg),)  # ONE launch over every segment: LDS accumulators per block
        query_b = alg
    else:
        filt_b, agg_b, query_b1 = algorithmic_bytes(args.docs)
        query_b = query_b1 * segs_here
        if kt[1][1] == 0:
            # fused path: ONE k_scan_query launch per query reads the three packed streams of every segment
            # of this GPU (no bitset traffic): algorithmic bytes per launch = segments x 4.25 B/row x docs
            names = ((0, "k_scan_query", query_b),)
        else:
            names = ((0, "k_leaf", filt_b * segs_here), (1, "k_colagg", agg_b * segs_here))
    for k, name, b in names:
        launches_per_query = max(kt[k][1] // reps, 1)
        per_launch_b = b / launches_per_query
        avg_ms = kt[k][0] / max(kt[k][1], 1)
        kern[name] = {"avg_ms": avg_ms, "launches": kt[k][1], "bytes_per_launch": per_launch_b,
                      "total_ms_per_query": kt[k][0] / reps, "timing": "HIP events, separate timing pass",
                      "gbs": per_launch_b / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0}
        if name == "k_scan_query" and dev_ms:
            # the one launch per step, timed inside the timed steps themselves: its in-kernel wall clock (first block
            # start to last block end, s_memrealtime) every step; the separate timing pass is kept beside it
            win = float(np.mean(dev_ms))
            kern[name].update({"avg_ms": win, "timing": "in-kernel wall clock of every timed step (mean)",
                               "timing_pass_avg_ms": avg_ms,
                               "gbs": per_launch_b / (win / 1e3) / 1e9 if win > 0 else 0.0})
    dom = max(kern, key=lambda n: kern[n]["total_ms_per_query"])
    # per GPU: this GPU's algorithmic bytes over the query time
    query_gbs = query_b / (ms_per_step / 1e3) / 1e9
    out = {
        "metric": "rows scanned/sec per query",
        "value": value,
        "unit": "rows/s",
        "n_gpus": job.n_gpus,
        "steps": steps,
        "warmup": args.warmup,
        "warmup_extra_steps": getattr(timed_steps, "extra_warmup", 0),  # untimed, to reach --warmup-seconds
        "ms_per_step": ms_per_step,
        "p50_query_ms": float(np.median(step_ms)),
        "p50_c_abi_ms": float(np.median(abi_ms)),
        "step_ms_detail": {"min": float(np.min(step_ms)), "p90": float(np.percentile(step_ms, 90)),
                           "max": float(np.max(step_ms)), "first": [round(x, 4) for x in step_ms[:4]],
                           # the device's own time per step (in-kernel wall clock / events), beside the host's
                           "device_p50": float(np.median(dev_ms)), "device_min": float(np.min(dev_ms)),
                           "device_max": float(np.max(dev_ms)),
                           "device_first": [round(x, 4) for x in dev_ms[:8]]},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 dictIds / int64 sums" + (" / u8 HLL registers" if c4 else ""),
        "data": "synthetic (seeded splitmix64 dict-encoded segments generated in HBM)",
        "config": {"workload": "%s: %d x %d-doc segments per GPU, 10 fixed-bit INT columns, %s" %
                   (workload, args.segments, args.docs, text),
                   "segments_per_gpu": args.segments, "docs_per_segment": args.docs,
                   "parallelism": "segments%d" % job.n_gpus, "path": job.path},
        "roofline": {"bound": "hbm", "achieved": kern[dom]["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": kern[dom]["gbs"] / HBM_PEAK_GBS, "traffic": measured_traffic(workload, dom),
                     "kernel": dom, "kernels": kern, "query_algorithmic_gbs": query_gbs,
                     "query_frac": query_gbs / HBM_PEAK_GBS},
    }
    if phases:
        out["merge_phases_ms"] = phases
    if gb and job.engines:
        inst = job.engines[0].stat("group.last_instance")
        out["plan"] = {"instance": inst, "name": "ring" if inst == 90000 else
                       "counted" if inst // 10000 in (3, 6) else "lds" if inst // 10000 == 1 else "other"}
    if gb:
        # the timed step returned DataTable bytes (rank 0's); the full result once for the check
        out["datatable_bytes"] = len(res)
        res, _ = job.ex.group_by_result(job.ex.prepare(text), job.segs)
        n_groups = res.num_groups()
        counts, sums = res.function_values(1 if c4 else 2)  # AVG(d8): per-group counts and sums
        chk, _ = job.ex.process_query(job.ex.prepare("SELECT COUNT(*), SUM(d8) FROM fact WHERE d2 < 800"), job.segs)
        tot = [int(counts.sum()), int(sums.sum())]
        if job.dist:  # rank 0 holds the gathered result, the other ranks none
            import torch
            t = torch.tensor([n_groups] + tot, dtype=torch.int64)
            job.dist.all_reduce(t)
            n_groups, tot = int(t[0]), [int(t[1]), int(t[2])]
        out["result"] = {"groups": n_groups, "sum_group_counts": tot[0], "sum_group_sums": tot[1]}
        out["verify"] = {"filtered_count": chk[0], "filtered_sum": int(chk[1]),
                         "match": tot == [chk[0], int(chk[1])] and n_groups == (1_000_000 if c4 else 1_600),
                         "how": "Σ per-group counts / sums == the aggregation-only COUNT(*) / SUM(d8) of the same "
                                "filter (independent kernel path) at full size; group-level parity against the oracle "
                                "at 2 x 2M docs: " + ("tests/test_gpu_configs.py::test_config4_shape, "
                                                      "tests/test_gpu_ring.py::test_ring_config4_shape" if c4 else
                                                      "tests/test_gpu_configs.py::test_lds_shape")}
    else:
        out["result"] = {"count": res[0], "sum": int(res[1]), "docs_scanned": st.num_docs_scanned}
    return out


def verify_config2(job, args, out, res_count, res_sum):
    """The full-size result against the C oracle (reference-faithful executor) over every segment of the job."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import faithful
    from concurrent.futures import ThreadPoolExecutor
    tot_c, tot_s = 0, 0.0
    names = [(i, n, c) for i, (n, c) in enumerate(COLUMNS) if n in ("d0", "d2", "d8")]
    tab = faithful.SyntheticTable(COLUMNS, args.docs, 0, BASE_SEED, needed=set())
    t0 = time.time()
    with ThreadPoolExecutor(min(args.cpu_threads, 32)) as pool:
        for s in range(args.segments * job.n_gpus):
            cols = {n: pool.submit(faithful.synth_column, BASE_SEED + s, i, c, args.docs) for i, n, c in names}
            tab.segments = [{n: f.result() for n, f in cols.items()}]
            c, v = faithful.run_and_count_sum(tab, [("d2", ("RANGE", 100, 600)), ("d0", ("IN", [1, 3, 5, 7]))],
                                              "d8", args.cpu_threads)
            tot_c += c
            tot_s += v
    return {"oracle_count": tot_c, "oracle_sum": int(tot_s), "seconds": time.time() - t0,
            "match": tot_c == res_count and int(tot_s) == res_sum}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--warmup-seconds", type=float, default=0.3,
                    help="keep warming up (untimed) until the warm-ups have run this long (clock ramp-up)")
    ap.add_argument("--workload", default="config2", choices=("config2", "config4", "lds"))
    ap.add_argument("--no-config4", action="store_true", help="config2 line without the embedded config-4 object")
    ap.add_argument("--no-lds", action="store_true", help="config2 line without the embedded LDS group-by object")
    ap.add_argument("--c4-steps", type=int, default=None, help="timed steps of the embedded config 4 (default --steps)")
    ap.add_argument("--path", default="auto", choices=("auto", "engine", "server"),
                    help="N = 1: one engine (auto) or the multi-GPU server over one GPU")
    ap.add_argument("--segments", type=int, default=8, help="segments per GPU")
    ap.add_argument("--docs", type=int, default=125_000_000, help="docs per segment")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline worker threads (default: 2 x available processors, ResourceManager.java:56-57)")
    ap.add_argument("--cpu-segments", type=int, default=None)
    ap.add_argument("--cpu-docs", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the full-size check of the GPU result against the C oracle (config 2)")
    ap.add_argument("--engine-config", default="", help='engine keys, e.g. "exec.fused=0" (unfused launches)')
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    if args.c4_steps is None:
        args.c4_steps = args.steps
    host = host_cpu_info()
    if args.cpu_threads is None:
        args.cpu_threads = min(2 * host["available_processors"], 128)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        assert world == args.gpus, "under torch.distributed.run WORLD_SIZE (%d) must equal --gpus (%d)" % (world,
                                                                                                        args.gpus)
    import torch
    torch.cuda.set_device(local_rank if world > 1 else 0)
    job = Job(args, world, rank, local_rank)

    out = measure(job, args, args.workload)
    out["segment_load_s"] = job.load_s
    head_res = dict(out["result"])
    if args.workload == "config2" and not args.no_config4:
        c4 = measure(job, args, "config4")
        keep = ("value", "unit", "ms_per_step", "p50_query_ms", "p50_c_abi_ms", "step_ms_detail", "steps", "warmup",
                "warmup_extra_steps", "dtype", "config", "roofline", "merge_phases_ms", "result", "verify", "plan")
        out["config4"] = {k: c4[k] for k in keep if k in c4}
    if args.workload == "config2" and not args.no_lds:
        lds = measure(job, args, "lds")
        keep = ("value", "unit", "ms_per_step", "p50_query_ms", "step_ms_detail", "steps", "warmup_extra_steps", "dtype",
                "config", "roofline", "result", "verify", "plan")
        out["lds_group_by"] = {k: lds[k] for k in keep if k in lds}
    cpu_ok = rank == 0 and world == 1 and job.n_gpus == 1 and not args.no_cpu_baseline
    if cpu_ok:
        host_desc = {"host": host, "threads": args.cpu_threads}
        if args.workload != "config2":
            cb = cpu_baseline_config4(args.cpu_threads, args.cpu_segments or 16, args.cpu_docs or 4_000_000,
                                      args.cpu_seconds, workload=args.workload)
        else:
            cb = cpu_baseline(args.cpu_threads, args.cpu_segments or 16, args.cpu_docs or 32_000_000,
                              args.cpu_seconds)
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "threads", "kind", "sample")}
        out["cpu_baseline"].update(host_desc)
        out["gpu_vs_cpu"] = out["value"] / cb["value"]
        if "optimized" in cb:  # SURVEY §8(d)'s second CPU line
            out["cpu_baseline_optimized"] = {k: cb["optimized"][k] for k in ("value", "unit", "cores", "threads", "kind",
                                                                             "sample")}
            out["gpu_vs_cpu_optimized"] = out["value"] / cb["optimized"]["value"]
        if "config4" in out:
            cb4 = cpu_baseline_config4(args.cpu_threads, args.cpu_segments or 16, args.cpu_docs or 4_000_000,
                                       args.cpu_seconds)
            out["config4"]["cpu_baseline"] = dict(cb4, **host_desc)
            out["config4"]["gpu_vs_cpu"] = out["config4"]["value"] / cb4["value"]
        if "lds_group_by" in out:
            cbl = cpu_baseline_config4(args.cpu_threads, args.cpu_segments or 16, args.cpu_docs or 8_000_000,
                                       args.cpu_seconds, workload="lds")
            out["lds_group_by"]["cpu_baseline"] = dict(cbl, **host_desc)
            out["lds_group_by"]["gpu_vs_cpu"] = out["lds_group_by"]["value"] / cbl["value"]
    if args.workload == "config2" and not args.no_verify and rank == 0:
        out["verify"] = verify_config2(job, args, out, head_res["count"], head_res["sum"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    job.close()


if __name__ == "__main__":
    main()
