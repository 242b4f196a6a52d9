"""The multi-GPU server inside the library (pinot_gpu_server_*): engines per device, RCCL communicators created
once, group-by partials merged by a reduce-scatter over the GLOBAL key space (union dictionaries, so per-segment
dictionaries may differ) and finalized per key range, aggregation partials combined; checked against the oracle's
CombineOperator / CombineGroupByOperator (CombineGroupByOperator.java:104-228, CombineOperator.java:75-196).

The GPU box has one MI355X: the servers here are one rank (ncclCommInitAll over [0]; one rank of a multi-process
communicator) and, where RCCL accepts it, two engines on the same device (two ranks, real reduce-scatter slices)."""
import numpy as np
import pytest

import pinot_oracle as O
from pinot_amd import GpuServer, PinotGpuError, ServerExecutor, build_segment, compile_pql

pytestmark = pytest.mark.gpu


def _segments(rng, n, nseg, different_dicts=True):
    segs = []
    words = ["a", "bb", "ccc", "P", "t", "zz", "Hello", "wé", "q%"]
    for i in range(nseg):
        shift = 7 * i if different_dicts else 0
        cols = {"g0": ("INT", (rng.integers(0, 300, n) + shift).tolist()),
                "g1": ("STRING", [words[k] for k in rng.integers(0, len(words) - (i % 3), n)]),
                "m": ("INT", rng.integers(-5000, 1000000, n).tolist()),
                "l": ("LONG", rng.integers(-2 ** 40, 2 ** 40, n).tolist()),
                "d": ("DOUBLE", np.round(rng.normal(0, 100, n), 3).tolist()),
                "h": ("INT", rng.integers(0, 5000, n).tolist())}
        segs.append(build_segment("seg%d" % i, cols, inverted_columns=("g1",)))
    return segs


QUERIES = [
    "SELECT COUNT(*), SUM(m), AVG(m), MIN(d), MAX(l), DISTINCTCOUNTHLL(h) FROM t WHERE m > 1000 GROUP BY g0, g1",
    "SELECT SUM(d), MAX(m), COUNT(*) FROM t WHERE g1 IN ('a', 'zz', 'q%') OR h < 100 GROUP BY g1",
    "SELECT COUNT(*), SUM(m), DISTINCTCOUNTHLL(l) FROM t GROUP BY h",
]
AGG_QUERIES = [
    "SELECT COUNT(*), SUM(m), AVG(l), MIN(m), MAX(d), SUM(d), DISTINCTCOUNTHLL(g1) FROM t WHERE h BETWEEN 10 AND 4000",
    "SELECT COUNT(*), MIN(d), MAX(l) FROM t WHERE m = 123456789",
]


def _check(server, gsegs, host, limit=100000):
    ex = ServerExecutor(server, num_groups_limit=limit)
    for text in QUERIES:
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs, trim=False)
        exp, scanned = O.execute_server(host, q, num_groups_limit=limit)
        assert st.num_docs_scanned == scanned
        assert set(got) == set(exp), text
        for k in exp:
            for a, g, e in zip(q["aggregations"], got[k], exp[k]):
                f = a["function"].upper()
                if f == "AVG":
                    assert g.count == e[1] and abs(g.sum - e[0]) <= 1e-9 * max(1.0, abs(e[0]))
                elif f == "DISTINCTCOUNTHLL":
                    assert g.cardinality() == e.cardinality()
                    assert (np.asarray(g.registers, dtype=np.int64) == e.reg).all()
                elif a["column"] == "d":
                    assert abs(g - e) <= 1e-9 * max(1.0, abs(e))
                else:
                    assert g == e, (text, k, a)
    for text in AGG_QUERIES:
        q = compile_pql(text)
        got, st = ex.process_query(q, gsegs)
        exp, scanned = O.execute_server(host, q)
        assert st.num_docs_scanned == scanned
        for a, g, e in zip(q["aggregations"], got, exp):
            f = a["function"].upper()
            if f == "AVG":
                assert g.count == e[1] and abs(g.sum - e[0]) <= 1e-9 * max(1.0, abs(e[0]))
            elif f == "DISTINCTCOUNTHLL":
                assert g.cardinality() == e.cardinality()
            elif a["column"] in ("d",):
                assert g == e or abs(g - e) <= 1e-9 * max(1.0, abs(e))
            else:
                assert g == e, (text, a)


def test_server_one_gpu_union_dictionaries():
    rng = np.random.default_rng(11)
    host = _segments(rng, 20000, 3)
    srv = GpuServer([0])
    gsegs = [srv.engines[0].register(s) for s in host]
    _check(srv, gsegs, host)
    srv.close()


def test_server_key_space_reuse_across_segment_sets():
    """Phase A's global key space is reused while its inputs match (server.cpp KeySpaceCache): the same server answers
    over one segment set, a subset of it, a set with other dictionaries (segments registered later, one of them after
    an unregister) and the first set again, each equal to the oracle's."""
    rng = np.random.default_rng(12)
    host = _segments(rng, 20000, 3)
    other = _segments(np.random.default_rng(13), 15000, 2)
    srv = GpuServer([0])
    e0 = srv.engines[0]
    gsegs = [e0.register(s) for s in host]
    _check(srv, gsegs, host)
    _check(srv, gsegs[:2], host[:2])
    gsegs[2].release()
    osegs = [e0.register(s) for s in other]
    _check(srv, osegs, other)
    _check(srv, gsegs[:2] + osegs[:1], host[:2] + other[:1])
    _check(srv, gsegs[:2], host[:2])
    srv.close()


def test_server_multi_process_form_one_rank():
    rng = np.random.default_rng(12)
    host = _segments(rng, 15000, 2)
    srv = GpuServer.rank(0, 1, 0, GpuServer.unique_id())
    gsegs = [srv.engines[0].register(s) for s in host]
    _check(srv, gsegs, host)
    srv.close()


def test_server_two_ranks_on_one_device():
    """Two engines (two RCCL ranks) on the box's one GPU: reduce-scatter into two key ranges, each finalized by
    its rank, concatenated. Skipped if RCCL refuses two ranks on one device."""
    try:
        srv = GpuServer([0, 0])
    except PinotGpuError as e:
        pytest.skip("RCCL rejects two ranks on one device here: %s" % e)
    rng = np.random.default_rng(13)
    host = _segments(rng, 12000, 4)
    gsegs = [srv.engines[i % 2].register(s) for i, s in enumerate(host)]
    _check(srv, gsegs, host)
    srv.close()


def test_server_binding_inter_segment_cap():
    """The 2 x num.groups.limit cap through the RCCL server (one rank): each segment's first-appearance holder
    (max.init.group.holder.capacity 10 makes it bind) and the inter-segment cap in segment order
    (CombineGroupByOperator.java:80,147), against the oracle's one-server combine."""
    rng = np.random.default_rng(14)
    host = _segments(rng, 8000, 3)
    srv = GpuServer([0])
    gsegs = [srv.engines[0].register(s) for s in host]
    q = compile_pql("SELECT COUNT(*) FROM t GROUP BY g0, h")
    got, st = ServerExecutor(srv, num_groups_limit=100, max_init_group_holder_capacity=10).process_query(
        q, gsegs, trim=False)
    exp, scanned = O.execute_server(host, q, num_groups_limit=100, array_threshold=10)
    assert st.num_docs_scanned == scanned and len(exp) == 200
    assert got == exp
    srv.close()


def test_torch_process_group_collective_on_engine_partials(sv_segment):
    """pinot_amd.combine over a torch process group (RCCL backend, world size 1, force_collective=True): the
    engine's dense partials go through agree_layout and the all-reduce before the finalize (the path a caller
    that already runs one process per GPU under torch.distributed uses)."""
    import socket
    import torch
    import torch.distributed as dist
    from pinot_amd import GpuEngine, ServerQueryExecutor
    from pinot_amd.combine import distributed_group_by
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        e = GpuEngine(0)
        g = e.register(sv_segment)
        q = compile_pql("SELECT COUNT(*), SUM(column1), MIN(column3), MAX(column6), AVG(column7), "
                        "DISTINCTCOUNTHLL(column1) FROM t WHERE column1 > 100000000 GROUP BY column9, column11")
        got, st = distributed_group_by(ServerQueryExecutor(e), q, [g, g], group=dist.group.WORLD, world=1,
                                       force_collective=True)
        exp, scanned = O.execute_server([sv_segment, sv_segment], q)
        assert st.num_docs_scanned == scanned and set(got) == set(exp)
        for k in exp:
            for a, gv, ev in zip(q["aggregations"], got[k], exp[k]):
                f = a["function"].upper()
                if f == "AVG":
                    assert (gv.sum, gv.count) == ev
                elif f == "DISTINCTCOUNTHLL":
                    assert gv.cardinality() == ev.cardinality()
                else:
                    assert gv == ev
        e.close()
    finally:
        dist.destroy_process_group()
