#!/usr/bin/env python3
"""Secondary BASELINE workloads on one GPU (the headline config 2 line is bench.py's).

  --workload config4   high-cardinality group-by on the config-2 table:
                       SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM t WHERE d2 < 800 GROUP BY d6, d7
                       (1,000,000 keys; num.groups.limit = 1,000,000 so no group is dropped).
                       Algorithmic bytes = N x (10 + 10 + 10 + 20 + 16) / 8 = 8.25 B/row.
                       Self-check at full size: Σ group counts / Σ group sums == the aggregation-only
                       COUNT(*) / SUM(d8) of the same filter (an independent kernel path).
  --workload config5   config 4's group-by as per-GPU dense partials merged by an RCCL all-reduce
                       (python -m torch.distributed.run --nproc-per-node N ... --workload config5).
  --workload config3   multi-predicate AND/OR over sorted + bitmap inverted indexes (config 3):
                       s0 sorted (card 1000), b1..b4 bitmap-indexed (card 10, 100, 1000, 10000), d8, m1:
                       SELECT SUM(d8), MAX(m1) WHERE s0 IN (10..19) AND (b1 = 3 OR b2 IN (5,6,7)) AND b3 <> 0

Prints one JSON line per workload (rows/s, ms/query, kernel times, roofline fraction)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))

COLUMNS = [("d0", 16), ("d1", 100), ("d2", 1000), ("d3", 4096), ("d4", 10000), ("d5", 65536), ("d6", 1000),
           ("d7", 1000), ("d8", 1 << 20), ("d9", 1000)]
BASE_SEED = 0x5EED0000
HBM_PEAK_GBS = 8000.0
CONFIG4 = "SELECT SUM(d8), AVG(d8), DISTINCTCOUNTHLL(d5) FROM t WHERE d2 < 800 GROUP BY d6, d7 TOP 10"
CONFIG4_CHECK = "SELECT COUNT(*), SUM(d8) FROM t WHERE d2 < 800"


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    ms = []
    for _ in range(steps):
        t0 = time.perf_counter()
        r = fn()
        ms.append((time.perf_counter() - t0) * 1e3)
    return r, ms


def config4(args, eng, ex):
    segs = [eng.register_synthetic("fact_%d" % s, args.docs, COLUMNS, BASE_SEED + s) for s in range(args.segments)]
    eng.synchronize()
    ex.num_groups_limit = 1_000_000
    q = ex.prepare(CONFIG4)
    abi = []

    def run():
        r = ex.process_query(q, segs, trim=False)
        abi.append(r[1].host_ms)
        return r

    (res, st), ms = timed(run, args.steps, args.warmup)
    abi = abi[args.warmup:]
    chk, _ = ex.process_query(ex.prepare(CONFIG4_CHECK), segs)
    n_groups = len(res)
    tot_cnt = sum(v[1].count for v in res.values())
    tot_sum = sum(v[0] for v in res.values())
    eng.set_config("timing=1")
    ex.process_query(q, segs, trim=False)
    k0 = eng.last_kernel_ms(0)
    k1 = eng.last_kernel_ms(1)
    eng.set_config("timing=0")
    rows = args.segments * args.docs
    # the boundary is the C-ABI (a JNI caller reads the result arrays it returns): value = rows / C-ABI wall time;
    # the Python mirror's materialisation of 1 M {key string: [objects]} entries is reported beside it
    p50 = float(np.median(abi))
    alg = rows * 8.25
    return {"workload": "config4", "query": CONFIG4, "segments": args.segments, "docs_per_segment": args.docs,
            "value": rows / (p50 / 1e3), "unit": "rows/s", "p50_c_abi_ms": p50,
            "p50_python_map_ms": float(np.median(ms)),
            "groups": n_groups, "device_ms": st.device_ms,
            "kernels": {"filter(kind0)": {"ms": k0[0], "launches": k0[1]}, "group_by(kind1)": {"ms": k1[0], "launches": k1[1]}},
            "roofline": {"bound": "hbm", "algorithmic_bytes": alg, "achieved_query": alg / (p50 / 1e3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac_query": alg / (p50 / 1e3) / 1e9 / HBM_PEAK_GBS},
            "check": {"sum_group_counts": tot_cnt, "filtered_count": chk[0], "sum_group_sums": tot_sum,
                      "filtered_sum": chk[1], "match": tot_cnt == chk[0] and tot_sum == chk[1] and n_groups == 1_000_000}}


def config5(args, eng, ex):
    """Config 5 per rank: this rank's share of 8 segments per GPU (global segment i on rank i mod world), the
    config-4 group-by as dense partials (pinot_gpu_group_by_partial, fused sinks), all-reduced over RCCL
    (the collective runs at world size 1 too), finalised on every rank. Run under torch.distributed.run."""
    import torch
    import torch.distributed as dist
    from pinot_amd.combine import distributed_group_by
    world, rank = dist.get_world_size(), dist.get_rank()
    segs = [eng.register_synthetic("fact_%d" % (s * world + rank), args.docs, COLUMNS, BASE_SEED + s * world + rank)
            for s in range(args.segments)]
    eng.synchronize()
    ex.num_groups_limit = 1_000_000
    q = ex.prepare(CONFIG4).query

    def step():
        return distributed_group_by(ex, q, segs, group=dist.group.WORLD, world=world, force_collective=True,
                                    as_map=False)

    for _ in range(args.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        res, st = step()
        ms.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    rows = world * args.segments * args.docs
    tot_cnt = int(res.function_values(1)[0].sum())  # AVG(d8)'s per-group counts
    n_groups = res.num_groups()
    chk, _ = ex.process_query(ex.prepare(CONFIG4_CHECK), segs)
    c = torch.tensor([chk[0], int(chk[1])], dtype=torch.int64, device="cuda")
    dist.all_reduce(c)
    return {"workload": "config5", "query": CONFIG4, "n_gpus": world, "segments_per_gpu": args.segments,
            "docs_per_segment": args.docs, "value": rows * args.steps / float(el.item()), "unit": "rows/s",
            "ms_per_query": float(el.item()) * 1e3 / args.steps, "p50_query_ms": float(np.median(ms)),
            "partial_device_ms": st.device_ms, "groups": n_groups, "scaling": "weak",
            "check": {"sum_group_counts": tot_cnt, "filtered_count": int(c[0]),
                      "match": tot_cnt == int(c[0]) and n_groups == 1_000_000}}


CONFIG3_COLUMNS = [("s0", 1000, "sorted"), ("b1", 10, "inverted"), ("b2", 100, "inverted"), ("b3", 1000, "inverted"),
                   ("b4", 10000, "inverted"), ("d8", 1 << 20, "random"), ("m1", 1024, "random")]
CONFIG3 = ("SELECT SUM(d8), MAX(m1) FROM t WHERE s0 IN (10,11,12,13,14,15,16,17,18,19) "
           "AND (b1 = 3 OR b2 IN (5, 6, 7)) AND b3 <> 0")
CONFIG3_CHECK = ("SELECT COUNT(*), SUM(d8), MAX(m1) FROM t WHERE s0 IN (10,11,12,13,14,15,16,17,18,19) "
                 "AND (b1 = 3 OR b2 IN (5, 6, 7)) AND b3 <> 0")


def config3(args, eng, ex):
    t0 = time.time()
    segs = [eng.register_synthetic("idx_%d" % s, args.docs, CONFIG3_COLUMNS, BASE_SEED + 0x100 + s)
            for s in range(args.segments)]
    eng.synchronize()
    load_s = time.time() - t0
    q = ex.prepare(CONFIG3)
    (res, st), ms = timed(lambda: ex.process_query(q, segs), args.steps, args.warmup)
    eng.set_config("timing=1")
    ex.process_query(q, segs)
    k0 = eng.last_kernel_ms(0)
    k1 = eng.last_kernel_ms(1)
    eng.set_config("timing=0")
    # independent path: the unfused launch sequence on a second engine over the same host-built bytes is too
    # costly at this size; cross-check with the forced-scan plan instead (no index is used for s0/b1..b3)
    eng.set_config("filter.force=scan")
    chk, st_scan = ex.process_query(ex.prepare(CONFIG3_CHECK), segs)
    eng.set_config("filter.force=")
    rows = args.segments * args.docs
    p50 = float(np.median(ms))
    seg_bytes = [s.device_bytes() for s in segs]
    return {"workload": "config3", "query": CONFIG3, "segments": args.segments, "docs_per_segment": args.docs,
            "value": rows / (p50 / 1e3), "unit": "rows/s", "p50_query_ms": p50, "p50_c_abi_ms": st.host_ms,
            "device_ms": st.device_ms, "docs_matched": st.num_docs_scanned, "segment_build_s": load_s,
            "segment_device_bytes": sum(seg_bytes),
            "kernels": {"scan_and_index_kernels(kind0)": {"ms": k0[0], "launches": k0[1]},
                        "kind1": {"ms": k1[0], "launches": k1[1]}},
            "result": {"sum_d8": res[0], "max_m1": res[1]},
            "check_scan_plan": {"count": chk[0], "sum_d8": chk[1], "max_m1": chk[2],
                                "match": chk[1] == res[0] and chk[2] == res[1] and chk[0] == st.num_docs_scanned}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config4", choices=("config3", "config4", "config5"))
    ap.add_argument("--segments", type=int, default=8)
    ap.add_argument("--docs", type=int, default=125_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--engine-config", default="")
    args = ap.parse_args()
    import torch
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if args.workload == "config5":
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    from pinot_amd import GpuEngine, ServerQueryExecutor
    eng = GpuEngine(local_rank, args.engine_config or None)
    ex = ServerQueryExecutor(eng)
    fn = {"config3": config3, "config4": config4, "config5": config5}[args.workload]
    out = fn(args, eng, ex)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(out))
    if args.workload == "config5":
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
