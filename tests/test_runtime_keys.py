"""Partition-key identity on both ingestion paths of the host runtime: a key value sent through
InputHandler.send (row path) and through send_columns (SoA path) must be ONE partition instance, as
PartitionStreamReceiver keys by String.valueOf(value) (C/partition/PartitionStreamReceiver.java:162-174)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))

from oracle import OracleEngine  # noqa: E402  (checker engine; CPU)
from siddhi_amd import QueryCallback, SiddhiManager  # noqa: E402


def _app(key_type):
    return (f"define stream S (k {key_type}, price float); "
            "partition with (k of S) begin @info(name='q') "
            "from every e1=S[price>20] -> e2=S[price>e1.price] "
            "select e1.price as p1, e2.price as p2 insert into M; end;")


def _run(key_type, keys_rows, keys_cols, prices_rows, prices_cols):
    rt = SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(_app(key_type))
    got = []

    class CB(QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend(tuple(e.data) for e in ins)

    rt.addCallback("q", CB())
    rt.start()
    h = rt.getInputHandler("S")
    for i, (k, p) in enumerate(zip(keys_rows, prices_rows)):
        h.send(i, [k, p])
    rt.flush()
    n0 = len(keys_rows)
    h.send_columns(np.arange(n0, n0 + len(keys_cols)), k=np.asarray(keys_cols), price=np.asarray(prices_cols, np.float32))
    rt.shutdown()
    return got


@pytest.mark.parametrize("key_type,kr,kc", [
    ("float", [1.5, 2.5], [1.5, 2.5]),
    ("double", [1.5, 2.5], [1.5, 2.5]),
    ("string", ["IBM", "WSO2"], ["IBM", "WSO2"]),
    ("bool", [True, False], [1, 0]),
    ("int", [7, 9], [7, 9]),
])
def test_same_key_both_paths(key_type, kr, kc):
    # e1 partials arrive on the row path; their e2 arrives on the column path for the same key value
    got = _run(key_type, kr, kc, [25.0, 30.0], [26.0, 31.0])
    assert sorted(got) == [(25.0, 26.0), (30.0, 31.0)], got


def test_string_ids_on_column_path_map_to_the_same_key():
    rt = SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(_app("string"))
    got = []

    class CB(QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend(tuple(e.data) for e in ins)

    rt.addCallback("q", CB())
    h = rt.getInputHandler("S")
    h.send(0, ["IBM", 25.0])
    rt.flush()
    sid = rt.strings["IBM"]
    h.send_columns(np.array([1]), k=np.array([sid], np.int32), price=np.array([26.0], np.float32))
    rt.shutdown()
    assert got == [(25.0, 26.0)]
