"""Cross-GPU combine: `CombineOperator` / `CombineGroupByOperator` over ranks (one process per GPU).

The reference merges per-segment results on a thread pool inside one server
(pinot-core/.../operator/CombineOperator.java:75-196 with CombineService.mergeTwoBlocks :48-90;
CombineGroupByOperator.java:104-228). Here segments are dealt round-robin to the GPUs of a node
(segment i -> rank i mod world); every rank runs the whole hot path on its own
segments and the per-rank partials are merged by collectives over RCCL (backend "nccl") on the GPU
box, or gloo on CPU in the tests:

  aggregation-only   a few scalars per function: int64 SUM for COUNT and for exact integer sums,
                     float64 SUM otherwise, MIN/MAX, and MAX over the 256 HLL registers.
  group-by           dense arrays over the query's global raw-key space (identical group-by
                     dictionaries: checked within a rank by the engine, across ranks by a fingerprint in
                     agree_layout before any data collective): SUM over counts / int64 / float64 sums, MIN/MAX
                     over order-preserving encodings of doubles, MAX over HLL registers
                     (pinot_gpu_group_by_partial -> agree_layout -> all_reduce -> pinot_gpu_group_by_finalize).
The library's multi-GPU server (pinot_gpu_server_*, include/pinot_gpu.h) does the same combine with RCCL inside
the .so, for one process over several GPUs or one process per GPU.

Integer results are exact whatever the reduction order; double sums of floating-point columns
agree within 1e-9 relative (the reference's own merge order is nondeterministic,
CombineGroupByOperator.java:145-160)."""
import ctypes as C

import numpy as np

from . import _lib
from ._hll import cardinality as hll_cardinality
from ._lib import check, sv_name

INT64_MIN = -(1 << 63)
EXACT_LIMIT = 1 << 53  # below this an integral double sum is exact in both the reference and here


def shard_segments(segments, rank, world):
    """Round-robin segment placement: segment i is served by rank i mod world."""
    return [s for i, s in enumerate(segments) if i % world == rank]


def _dist():
    import torch.distributed as dist
    return dist


def combine_aggregation(query, partial, group=None, device="cpu"):
    """Merge one rank's aggregation-only intermediate results with every other rank's.

    `partial` is the list returned by ServerQueryExecutor.process_query for an aggregation-only query
    (COUNT -> int, SUM/MIN/MAX -> float, AVG -> AvgPair, DISTINCTCOUNTHLL -> HyperLogLog). Returns the
    merged list in the same shapes (what CombineOperator hands to the DataTable)."""
    import torch
    from .executor import AvgPair, HyperLogLog
    dist = _dist()
    fns = [sv_name(a["function"]) for a in query["aggregations"]]
    n = len(fns)
    isum = torch.zeros(n, dtype=torch.int64)     # COUNT, and SUM / AVG sums that are exact integers
    dsum = torch.zeros(n, dtype=torch.float64)   # SUM / AVG sums that are not
    counts = torch.zeros(n, dtype=torch.int64)   # AVG counts
    mins = torch.full((n,), float("inf"), dtype=torch.float64)
    maxs = torch.full((n,), float("-inf"), dtype=torch.float64)
    regs = torch.zeros((n, 256), dtype=torch.int32)

    def put_sum(i, s):
        s = float(s)
        if s.is_integer() and abs(s) < EXACT_LIMIT:
            isum[i] = int(s)
        else:
            dsum[i] = s

    for i, (f, v) in enumerate(zip(fns, partial)):
        if f == "COUNT":
            isum[i] = int(v)
        elif f == "SUM":
            put_sum(i, v)
        elif f == "AVG":
            put_sum(i, v.sum)
            counts[i] = int(v.count)
        elif f == "MIN":
            mins[i] = float(v)
        elif f == "MAX":
            maxs[i] = float(v)
        elif f == "DISTINCTCOUNTHLL":
            regs[i] = torch.from_numpy(np.asarray(v.registers, dtype=np.int32))
        else:
            raise ValueError(f)
    tensors = [isum, dsum, counts, mins, maxs, regs]
    if device != "cpu":
        tensors = [t.to(device) for t in tensors]
    ops = [dist.ReduceOp.SUM, dist.ReduceOp.SUM, dist.ReduceOp.SUM, dist.ReduceOp.MIN, dist.ReduceOp.MAX,
           dist.ReduceOp.MAX]
    for t, op in zip(tensors, ops):
        dist.all_reduce(t, op=op, group=group)
    isum, dsum, counts, mins, maxs, regs = [t.cpu() for t in tensors]
    out = []
    for i, f in enumerate(fns):
        if f == "COUNT":
            out.append(int(isum[i]))
        elif f in ("SUM", "AVG"):
            # exact integer partials stay exact; any non-integral partial makes it a double sum
            s = float(int(isum[i])) + float(dsum[i])
            out.append(s if f == "SUM" else AvgPair(s, int(counts[i])))
        elif f == "MIN":
            out.append(float(mins[i]))
        elif f == "MAX":
            out.append(float(maxs[i]))
        else:
            r = regs[i].numpy().astype(np.uint8)
            out.append(HyperLogLog(r, hll_cardinality(r)))
    return out


# ------------------------------------------------------------------ group-by partials
ACC_INT64_SUM, ACC_F64_SUM, ACC_MIN, ACC_MAX, ACC_HLL, ACC_NONE = range(6)


def allreduce_group_partials(acc_kinds, counts, accs, group=None):
    """In-place all-reduce of dense group-by partials (torch tensors, any device the backend serves).

    counts: int64[G]; accs[f] per acc_kinds[f]: int64[G] sums (kind 0), float64[G] sums (kind 1),
    int64[G] holding uint64 order-preserving encodings of doubles (kinds 2 = MIN, 3 = MAX; unsigned
    order is made signed by flipping the top bit around the collective), uint8[G*256] HLL registers
    (kind 4), None (kind 5: COUNT reads `counts`)."""
    dist = _dist()
    dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    for kind, t in zip(acc_kinds, accs):
        if kind in (ACC_INT64_SUM, ACC_F64_SUM):
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        elif kind in (ACC_MIN, ACC_MAX):
            t.bitwise_xor_(INT64_MIN)
            dist.all_reduce(t, op=dist.ReduceOp.MIN if kind == ACC_MIN else dist.ReduceOp.MAX, group=group)
            t.bitwise_xor_(INT64_MIN)
        elif kind == ACC_HLL:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)


def agree_layout(ok, G, kinds, fingerprint, group=None, device="cpu"):
    """Header agreement BEFORE any data collective (a rank that failed or disagrees would otherwise leave its peers
    blocked in all_reduce, or reduce arrays of different shapes): MIN and MAX all-reduce of
    [ok, G, fingerprint, kinds...]. A rank without segments passes G = None: it sends the reductions' identities
    and adopts its peers' layout. Raises on EVERY rank when any rank failed or the known fields differ.
    Returns (G, kinds) as agreed."""
    import torch
    dist = _dist()
    n = 4 + 8
    big, small = (1 << 63) - 1, -(1 << 63)
    known = ok and G is not None
    vals = [1 if ok else 0, G or 0, (fingerprint or 0) & ((1 << 63) - 1), len(kinds or [])] + list(kinds or []) + \
        [0] * (8 - len(kinds or []))
    lo = torch.tensor([vals[0]] + [v if known else big for v in vals[1:]], dtype=torch.int64, device=device)
    hi = torch.tensor([vals[0]] + [v if known else small for v in vals[1:]], dtype=torch.int64, device=device)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo, hi = lo.cpu().tolist(), hi.cpu().tolist()
    if lo[0] != 1:
        raise RuntimeError("group-by combine: a peer rank failed before the merge")
    if lo[1] == big:
        raise RuntimeError("group-by combine: no rank holds a segment")
    if lo[1:] != hi[1:]:
        raise RuntimeError("group-by combine: ranks disagree on the key space / accumulators / group-by dictionaries "
                           "(raw keys would name different groups)")
    return int(lo[1]), [int(x) for x in lo[4:4 + int(lo[3])]]


def identity_partials(G, kinds, device="cpu"):
    """Dense partials that leave a merge unchanged (a rank without segments contributes these)."""
    import torch
    counts = torch.zeros(G, dtype=torch.int64, device=device)
    accs = []
    for k in kinds:
        if k == ACC_NONE:
            accs.append(None)
        elif k == ACC_F64_SUM:
            accs.append(torch.zeros(G, dtype=torch.float64, device=device))
        elif k == ACC_HLL:
            accs.append(torch.zeros(G * 256, dtype=torch.uint8, device=device))
        elif k == ACC_MIN:
            accs.append(torch.full((G,), -1, dtype=torch.int64, device=device))  # 0xFF.. = +inf
        else:
            accs.append(torch.zeros(G, dtype=torch.int64, device=device))
    return counts, accs


def distributed_group_by(executor, query, segments, group=None, world=1, force_collective=False, as_map=True):
    """Group-by over this rank's GPU-resident `segments`, merged with the other ranks through torch.distributed.

    Runs pinot_gpu_group_by_layout / _partial into torch tensors, agrees on the layout with every rank
    (agree_layout), all-reduces, and finalizes on every rank that holds segments (a rank without segments
    contributes identity partials and returns an empty result). The library's own multi-GPU server
    (pinot_gpu_server_*) does the same merge with RCCL inside the .so; this is the path for callers that already
    run one process per GPU under a torch process group."""
    import torch
    from .executor import GroupByResult, QueryMarshal, _segment_handles
    from .pql import compile_pql
    if isinstance(query, str):
        query = compile_pql(query)
    eng = executor.engine
    lib = eng.lib
    dev = torch.device("cuda", eng.device)
    m = QueryMarshal(query, executor.num_groups_limit, executor.max_init)
    handles = _segment_handles(segments) if segments else None
    collective = world > 1 or force_collective
    stats = _lib.ExecStats()
    ok, G, kinds, fp, err = True, None, None, None, None
    counts = accs = None
    try:
        if segments:
            layout = _lib.PartialLayout()
            check(lib.pinot_gpu_group_by_layout(eng.ptr, handles, len(segments), C.byref(m.q), C.byref(layout)))
            G = int(layout.num_keys)
            kinds = [int(layout.acc_kind[i]) for i in range(layout.num_aggregations)]
            fp = int(layout.group_dictionary_fingerprint)
            counts, accs = identity_partials(G, kinds, dev)
            ptrs = (C.c_void_p * max(len(kinds), 1))(*[(a.data_ptr() if a is not None else None) for a in accs])
            torch.cuda.synchronize(dev)
            check(lib.pinot_gpu_group_by_partial(eng.ptr, handles, len(segments), C.byref(m.q),
                                                 C.c_void_p(counts.data_ptr()), ptrs, C.byref(stats)))
    except Exception as ex:  # every rank must still reach the agreement, then all fail together
        ok, err = False, ex
        if not collective:
            raise
    if collective:
        try:
            G, kinds = agree_layout(ok, G, kinds, fp, group, device=dev)
        except Exception:
            if err is not None:
                raise err
            raise
        if counts is None:
            counts, accs = identity_partials(G, kinds, dev)
        allreduce_group_partials(kinds, counts, accs, group)
        torch.cuda.synchronize(dev)
    if not segments:
        return ({} if as_map else None), stats
    ptrs = (C.c_void_p * max(len(kinds), 1))(*[(a.data_ptr() if a is not None else None) for a in accs])
    out = C.c_void_p()
    check(lib.pinot_gpu_group_by_finalize(eng.ptr, handles, len(segments), C.byref(m.q),
                                          C.c_void_p(counts.data_ptr()), ptrs, C.byref(out)))
    res = GroupByResult(lib, out, query)
    return (res.to_map() if as_map else res), stats
