"""Host restatement of the synthetic fact-table generator (TEST INFRASTRUCTURE; see pinot_oracle.py header).

The bench builds its segments directly in HBM (`pinot_gpu_segment_register_synthetic`, kernel
k_synth_column); this module generates the same values on the host so the oracle / CPU baseline can
run the identical workload:
    column seed  s_c = seed ^ ((c + 1) * 0xD1B54A32D192ED03)
    value(d)     = d                                           if d < card
                 = splitmix64(s_c ^ (d * 0x9E3779B97F4A7C15)) % card   otherwise
Every value of [0, card) appears (docs 0..card-1), so every segment has the identity INT dictionary
[0, card) and dictId == value.
"""
import numpy as np

PHI = np.uint64(0x9E3779B97F4A7C15)
COL_MUL = 0xD1B54A32D192ED03
M64 = (1 << 64) - 1


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + PHI
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def column_values(seed, col_index, card, start, stop):
    cseed = np.uint64((seed ^ (((col_index + 1) * COL_MUL) & M64)) & M64)
    d = np.arange(start, stop, dtype=np.uint64)
    with np.errstate(over="ignore"):
        v = splitmix64(cseed ^ (d * PHI)) % np.uint64(card)
    v = v.astype(np.int64)
    small = d < np.uint64(card)
    v[small] = d[small].astype(np.int64)
    return v


def _pack(ids, bits):
    shifts = np.arange(bits - 1, -1, -1, dtype=np.uint64)
    out = []
    for s in range(0, ids.shape[0], 1 << 20):
        v = ids[s:s + (1 << 20)].astype(np.uint64)
        out.append(np.packbits(((v[:, None] >> shifts[None, :]) & np.uint64(1)).astype(np.uint8).reshape(-1),
                               bitorder="big").tobytes())
    return b"".join(out)


def make_segment(name, num_docs, columns, seed):
    """columns = [(name, cardinality)] -> a Segment object in Pinot's byte format (INT, identity dictionaries)."""
    from pinot_amd.segment import Column, Segment  # data containers only
    cols = {}
    for i, (cname, card) in enumerate(columns):
        ids = column_values(seed, i, card, 0, num_docs)
        bits = max(1, int(card - 1).bit_length())
        cols[cname] = Column(name=cname, data_type="INT", cardinality=card, bits=bits, is_sorted=False,
                             has_inverted_index=False, num_docs=num_docs,
                             dictionary=np.arange(card, dtype=">i4").tobytes(), fwd=_pack(ids, bits))
    return Segment(name=name, num_docs=num_docs, columns=cols)


def sorted_values(card, num_docs):
    """PINOT_SYNTH_SORTED: value v on docs [v*N/card, (v+1)*N/card)."""
    starts = (np.arange(card, dtype=np.int64) * num_docs) // card
    return np.searchsorted(starts, np.arange(num_docs, dtype=np.int64), side="right") - 1


def make_segment_kinds(name, num_docs, columns, seed):
    """columns = [(name, cardinality, kind)] with kind random / sorted / inverted -> Segment via the
    reference-format builder (sorted index, bitmap inverted indexes) from the same values."""
    from pinot_amd.segment import build_segment  # data containers / format writer only
    cols, inv = {}, []
    for i, (cname, card, kind) in enumerate(columns):
        if kind == "sorted":
            vals = sorted_values(card, num_docs)
        else:
            vals = column_values(seed, i, card, 0, num_docs)
        if kind == "inverted":
            inv.append(cname)
        cols[cname] = ("INT", vals.tolist())
    return build_segment(name, cols, inverted_columns=tuple(inv))
