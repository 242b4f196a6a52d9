"""Cross-rank combine (pinot_amd.combine) at world_size 2 over gloo on CPU.

Each rank serves the segments `shard_segments` deals it (segment i -> rank i mod world). Its per-rank
partial results stand in for what its GPU produces — they come from the CPU oracle here, since this
container has no GPU — and are merged with the product's combine functions over the collective.
The merged result must equal the oracle run over ALL segments (CombineOperator /
CombineGroupByOperator semantics): counts, integer sums, MIN/MAX, HLL registers bit-exact."""
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COLS = [("d0", 16), ("d2", 100), ("d5", 300), ("d6", 7), ("d7", 5), ("d8", 1 << 12)]
QUERIES = [
    "SELECT COUNT(*), SUM(d8), MIN(d8), MAX(d2), AVG(d8), DISTINCTCOUNTHLL(d5) FROM t "
    "WHERE d2 BETWEEN 10 AND 59 AND d0 IN (1, 3, 5, 7)",
    "SELECT COUNT(*), SUM(d8) FROM t WHERE d2 > 1000",  # empty: default aggregates
    "SELECT MAX(d8), DISTINCTCOUNTHLL(d8) FROM t",
]
GROUP_QUERY = ("SELECT COUNT(*), SUM(d8), MIN(d2), MAX(d8), AVG(d5), DISTINCTCOUNTHLL(d5) FROM t "
               "WHERE d2 < 80 GROUP BY d6, d7")
NSEG, NDOCS = 5, 3001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _segments():
    import synth
    return [synth.make_segment("s%d" % i, NDOCS, COLS, 0x5EED0000 + i) for i in range(NSEG)]


def _to_product(query, vals):
    from pinot_amd.executor import AvgPair, HyperLogLog
    out = []
    for a, v in zip(query["aggregations"], vals):
        f = a["function"].upper()
        if f == "AVG":
            out.append(AvgPair(float(v[0]), int(v[1])))
        elif f == "DISTINCTCOUNTHLL":
            out.append(HyperLogLog(np.asarray(v.reg, dtype=np.uint8), v.cardinality()))
        else:
            out.append(v)
    return out


def _ordered(d):
    """The engine's order-preserving uint64 encoding of a double (kernels.hip ordered_bits), as int64 bits."""
    u = np.array([d], dtype=np.float64).view(np.uint64)
    u = np.where(u & np.uint64(1 << 63), ~u, u | np.uint64(1 << 63))
    return u.view(np.int64)[0]


def _dense(query, result_map):
    """Oracle group map (string keys) -> dense partial arrays in the engine's layout (identity dictionaries)."""
    cards = dict(COLS)
    gcols = query["group_by"]["columns"]
    G = int(np.prod([cards[c] for c in gcols]))
    kinds, arrays = [], []
    counts = np.zeros(G, dtype=np.int64)
    for a in query["aggregations"]:
        f = a["function"].upper()
        if f == "COUNT":
            kinds.append(5)
            arrays.append(None)
        elif f in ("SUM", "AVG"):
            kinds.append(0)
            arrays.append(np.zeros(G, dtype=np.int64))
        elif f == "MIN":
            kinds.append(2)
            arrays.append(np.full(G, -1, dtype=np.int64))  # 0xFF.. = +inf identity
        elif f == "MAX":
            kinds.append(3)
            arrays.append(np.zeros(G, dtype=np.int64))
        else:
            kinds.append(4)
            arrays.append(np.zeros(G * 256, dtype=np.uint8))
    for key, vals in result_map.items():
        ids = [int(x) for x in key.split("\t")]
        k, stride = 0, 1
        for c, i in zip(gcols, ids):
            k += i * stride
            stride *= cards[c]
        for a, arr, v in zip(query["aggregations"], arrays, vals):
            f = a["function"].upper()
            if f == "COUNT":
                counts[k] = v
            elif f == "SUM":
                arr[k] = int(v)
            elif f == "AVG":
                arr[k] = int(v[0])
                counts[k] = v[1]
            elif f in ("MIN", "MAX"):
                arr[k] = _ordered(v)
            else:
                arr[k * 256:(k + 1) * 256] = v.reg
    return kinds, counts, arrays


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import torch
        import torch.distributed as dist
        import pinot_oracle as O
        from pinot_amd.combine import allreduce_group_partials, combine_aggregation, shard_segments
        from pinot_amd.pql import compile_pql
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        segs = _segments()
        mine = shard_segments(segs, rank, world)
        assert [s.name for s in mine] == ["s%d" % i for i in range(rank, NSEG, world)]
        for text in QUERIES:
            query = compile_pql(text)
            part, _ = O.execute_server(mine, query)
            got = combine_aggregation(query, _to_product(query, part))
            exp = _to_product(query, O.execute_server(segs, query)[0])
            for a, g, e in zip(query["aggregations"], got, exp):
                f = a["function"].upper()
                if f == "DISTINCTCOUNTHLL":
                    assert (g.registers == e.registers).all() and g.cardinality() == e.cardinality(), text
                elif f == "AVG":
                    assert g.sum == e.sum and g.count == e.count, text
                else:
                    assert g == e, (text, f, g, e)
        query = compile_pql(GROUP_QUERY)
        part, _ = O.execute_server(mine, query)
        kinds, counts, arrays = _dense(query, part)
        tc = torch.from_numpy(counts)
        ta = [torch.from_numpy(a) if a is not None else None for a in arrays]
        allreduce_group_partials(kinds, tc, ta)
        ekinds, ecounts, earrays = _dense(query, O.execute_server(segs, query)[0])
        assert kinds == ekinds
        assert (tc.numpy() == ecounts).all()
        for t, e in zip(ta, earrays):
            if e is not None:
                assert (t.numpy() == e).all()
        # layout agreement before any data collective: a rank without segments adopts the peers' layout and
        # contributes identity partials; a disagreeing rank makes EVERY rank fail (nobody blocks in all_reduce)
        from pinot_amd.combine import agree_layout, identity_partials
        kinds_e, counts_e, arrays_e = _dense(query, O.execute_server(segs, query)[0])
        G = counts_e.shape[0]
        if rank == 0:
            Gr, kr = agree_layout(True, G, kinds, 1234)
            _, c0, a0 = _dense(query, part)  # (counts / arrays above were merged in place)
            mc, ma = torch.from_numpy(c0), [torch.from_numpy(a) if a is not None else None for a in a0]
        else:
            Gr, kr = agree_layout(True, None, None, None)
            mc, ma = identity_partials(Gr, kr)
        assert (Gr, kr) == (G, kinds)
        allreduce_group_partials(kr, mc, ma)
        ek, ec, ea = _dense(query, O.execute_server([s for s in mine] if rank == 0 else shard_segments(segs, 0, world),
                                                    query)[0])
        assert (mc.numpy() == ec).all()
        for t, e in zip(ma, ea):
            if e is not None:
                assert (t.numpy() == e).all()
        for bad in ("fingerprint", "failed"):
            try:
                if bad == "fingerprint":
                    agree_layout(True, G, kinds, 1234 + rank)
                else:
                    agree_layout(rank == 0, G if rank == 1 else None, kinds if rank == 1 else None, 1234)
                raise AssertionError("agree_layout accepted a %s peer" % bad)
            except RuntimeError as ex:
                assert "failed" in str(ex) or "disagree" in str(ex)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as ex:  # report to the parent instead of hanging the other rank
        import traceback
        q.put((rank, "%s\n%s" % (ex, traceback.format_exc())))


@pytest.mark.timeout(300)
def test_combine_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=280) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def test_shard_segments_round_robin():
    sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
    from pinot_amd.combine import shard_segments
    segs = list(range(64))
    shards = [shard_segments(segs, r, 8) for r in range(8)]
    assert all(len(s) == 8 for s in shards)
    assert sorted(x for s in shards for x in s) == segs
    assert shards[3][:2] == [3, 11]
