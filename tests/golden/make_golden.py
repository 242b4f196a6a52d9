"""Regenerates the committed golden fixtures from the reference's own test data.

Run in the build container (needs /root/reference, read-only):  python tests/golden/make_golden.py

Writes (all data, no reference source text):
  test_data_sv.npz    the 11 columns BaseSingleValueQueriesTest builds its segment from
                      (pinot-core/src/test/resources/data/test_data-sv.avro, 30000 rows;
                       column list: PT/queries/BaseSingleValueQueriesTest.java:47-60,93-101)
  simple_data.npz     dim0, dim1, met of pinot-core/src/test/resources/data/simpleData200001.avro
                      (PT/query/executor/QueryExecutorTest.java:59-173)
  airline_stats.npz   Carrier, ArrDelay, DaysSinceEpoch of pinot-tools/src/main/resources/sample_data/
                      airlineStats_data.avro (9746 rows; the config-1 query shape on real data)
  padding_null.json   byte contents of the Java-written v1 segment paddingNull.tar.gz (dictionaries and
                      fixed-bit forward indexes, with metadata cardinality/bits) — a byte-level format fixture
  segments/           the three Java-written v1 segment directories paddingNull / paddingOld / paddingPercent
                      unpacked as they are (data files of LoaderTest.java:55-57,144-206)
The known answers themselves are transcribed (with file:line) in reference_kats.json.
"""
import io
import json
import os
import sys
import tarfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avro  # noqa: E402

REF = "/root/reference/pinot-core/src/test/resources/data"
SV_COLUMNS = [("column1", "INT"), ("column3", "INT"), ("column5", "STRING"), ("column6", "INT"),
              ("column7", "INT"), ("column9", "INT"), ("column11", "STRING"), ("column12", "STRING"),
              ("column17", "INT"), ("column18", "INT"), ("daysSinceEpoch", "INT")]


TOOLS_DATA = "/root/reference/pinot-tools/src/main/resources/sample_data"


def main():
    names, cols = avro.read_avro(os.path.join(REF, "test_data-sv.avro"))
    out = {}
    for n, t in SV_COLUMNS:
        v = cols[n]
        assert all(x is not None for x in v), n
        out[n] = np.array(v, dtype=np.int32) if t == "INT" else np.array(v, dtype="U")
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **out)

    names, cols = avro.read_avro(os.path.join(REF, "simpleData200001.avro"))
    np.savez_compressed(os.path.join(HERE, "simple_data.npz"),
                        **{n: np.array(cols[n], dtype=np.int32) for n in ("dim0", "dim1", "met")})

    fx = {}
    with tarfile.open(os.path.join(REF, "paddingNull.tar.gz")) as tf:
        files = {os.path.basename(m.name): tf.extractfile(m).read() for m in tf.getmembers() if m.isfile()}
    meta = {}
    for line in files["metadata.properties"].decode().splitlines():
        if "=" in line:
            k, v = line.split("=", 1)
            meta[k.strip()] = v.strip()
    for col in ("age", "name", "percent", "outgoingName1"):
        fx[col] = {
            "data_type": meta["column.%s.dataType" % col],
            "cardinality": int(meta["column.%s.cardinality" % col]),
            "bits": int(meta["column.%s.bitsPerElement" % col]),
            "string_width": int(meta["column.%s.lengthOfEachEntry" % col]),
            "num_docs": int(meta["segment.total.raw.docs"]),
            "dict_hex": files[col + ".dict"].hex(),
            "fwd_hex": files[col + ".sv.unsorted.fwd"].hex(),
        }
    with open(os.path.join(HERE, "padding_null.json"), "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    for name in ("paddingNull", "paddingOld", "paddingPercent"):
        with tarfile.open(os.path.join(REF, name + ".tar.gz")) as tf:
            for m in tf.getmembers():
                if m.isfile():
                    out = os.path.join(HERE, "segments", name, os.path.basename(m.name))
                    os.makedirs(os.path.dirname(out), exist_ok=True)
                    with open(out, "wb") as f:
                        f.write(tf.extractfile(m).read())

    # real data for the config-1 query shape: pinot-tools' airlineStats sample, the three
    # columns the query reads; ArrDelay is a nullable INT *dimension*, so nulls take Pinot's default
    # dimension null value Integer.MIN_VALUE (pinot-common/.../data/FieldSpec.java:50)
    names, cols = avro.read_avro(os.path.join(TOOLS_DATA, "airlineStats_data.avro"))
    arr = [(-2 ** 31 if x is None else x) for x in cols["ArrDelay"]]
    np.savez_compressed(os.path.join(HERE, "airline_stats.npz"), Carrier=np.array(cols["Carrier"], dtype="U"),
                        ArrDelay=np.array(arr, dtype=np.int32),
                        DaysSinceEpoch=np.array(cols["DaysSinceEpoch"], dtype=np.int32))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
