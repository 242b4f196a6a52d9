"""The C restatement (oracle/faithful.c, the CPU baseline) agrees with the numpy oracle and the HBM generator's host twin."""
import numpy as np
import pytest

import faithful
import pinot_oracle as O
import synth
from pinot_amd.pql import compile_pql

COLS = [("d0", 16), ("d1", 100), ("d2", 1000), ("d8", 1 << 12)]


@pytest.fixture(scope="module", autouse=True)
def _lib():
    faithful.load()


def test_c_synth_matches_python_synth():
    for i, (name, card) in enumerate(COLS):
        c = faithful.synth_column(0x5EED0000, i, card, 10007)
        seg = synth.make_segment("s", 10007, COLS, 0x5EED0000)
        assert bytes(c[:len(seg.columns[name].fwd)]) == seg.columns[name].fwd


def test_read_int_matches_oracle():
    rng = np.random.default_rng(3)
    lib = faithful.load()
    for b in (1, 3, 7, 13, 20, 31):
        vals = rng.integers(0, 1 << b, 500)
        from pinot_amd.segment import pack_fixed_bit
        buf = pack_fixed_bit(vals, b) + b"\0" * 8
        arr = np.frombuffer(buf, dtype=np.uint8)
        for i in (0, 1, 250, 499):
            assert lib.pinot_faithful_read_int(arr.ctypes.data, i, b) == O.read_int(buf, i, b) == vals[i]


@pytest.mark.parametrize("threads", [1, 3])
def test_faithful_query_matches_numpy_oracle(threads):
    n, nseg, seed = 50021, 3, 0x5EED0000
    table = faithful.SyntheticTable(COLS, n, nseg, seed, needed={"d0", "d2", "d8"})
    got = faithful.run_and_count_sum(table, [("d2", ("RANGE", 100, 600)), ("d0", ("IN", [1, 3, 5, 7]))], "d8", threads)
    q = compile_pql("SELECT COUNT(*), SUM(d8) FROM t WHERE d2 BETWEEN 100 AND 599 AND d0 IN (1, 3, 5, 7)")
    segs = [synth.make_segment("s%d" % s, n, COLS, seed + s) for s in range(nseg)]
    exp, _ = O.execute_server(segs, q)
    assert got[0] == exp[0]
    assert got[1] == exp[1]
