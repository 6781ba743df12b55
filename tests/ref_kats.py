"""Known-answer tests transcribed from the reference's Java suites (data in tests/golden/ref_kats.json, made by
tests/golden/make_ref_kats.py).  Each case is the test's action list up to its count assertion -- `send`,
`sleep` (ms), `wait_in_events` (TestUtil.waitForInEvents, T/TestUtil.java:237-247), `wait_events`
(SiddhiTestHelper.waitForEvents, C/util/SiddhiTestHelper.java:49-57) -- the rows the test asserts
(in order, T/TestUtil.java:124-143, or an inline callback's assertArrayEquals sequence) and the asserted
in-event count.  Wall-clock tests (clock "wall") run in playback with the clock advanced in 1 ms heartbeats
(SiddhiAppRuntime.advance_time -> sg_advance_time) through every sleep, starting at 1 ms: an event's timestamp
is the time it is sent at and every timer fires at its due time, as with the reference's wall-clock Scheduler.
Values: {"F": x} a Java float literal, {"D": x} a double, {"L": x} a long.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _val(v):
    if isinstance(v, dict):
        if "F" in v:
            return float(np.float32(v["F"]))
        if "D" in v:
            return float(v["D"])
        return int(v["L"])
    return v


def load():
    with open(os.path.join(HERE, "golden", "ref_kats.json")) as f:
        kats = json.load(f)
    for k in kats:
        for a in k["actions"]:
            if a[0] == "send":
                a[3] = [_val(x) for x in a[3]]
        k["expect"] = [[_val(x) for x in row] for row in k["expect"]]
    return kats


REF_KATS = load()


def check(case, rows):
    """The reference test's assertions: in-event count, and the expected rows in order (a prefix when the test
    lists fewer rows than it counts; every row when the test asserts one row inside its per-event loop)."""
    assert len(rows) == case["expect_count"], (len(rows), case["expect_count"], rows)
    exp = case["expect"]
    if case.get("expect_every"):
        assert all(r == exp[0] for r in rows), (rows, exp)
        return
    assert rows[:len(exp)] == exp, (rows, exp)


def run_ref_kat(case, engine):
    """Drive one transcribed test through the host API; returns (rows, timestamps)."""
    from siddhi_amd import QueryCallback, SiddhiManager, StreamCallback
    rt = SiddhiManager(engine=engine).createSiddhiAppRuntime(case["app"])
    rows, tss = [], []

    class QCB(QueryCallback):
        def receive(self, ts, ins, rem):
            for e in ins:
                rows.append(list(e.data))
                tss.append(e.timestamp)

    class SCB(StreamCallback):
        def receive(self, events):
            for e in events:
                rows.append(list(e.data))
                tss.append(e.timestamp)

    if case.get("stream_callback"):
        rt.addCallback(case["stream_callback"], SCB())
    else:
        rt.addCallback("query1", QCB())
    rt.start()
    handlers = {}
    wall = case["clock"] == "wall"
    clock = [1]

    def sleep(ms):
        for _ in range(ms):
            clock[0] += 1
            rt.advance_time(clock[0])

    for a in case["actions"]:
        if a[0] == "send":
            _, sid, ts, row = a
            h = handlers.setdefault(sid, rt.getInputHandler(sid))
            h.send(clock[0] if wall else ts, row)
        elif wall and a[0] == "sleep":
            sleep(a[1])
        elif wall and a[0] == "wait_in_events":
            for _ in range(a[2]):
                sleep(a[1])
                rt.flush()
                if len(rows) == 1:
                    break
        elif wall and a[0] == "wait_events":   # SiddhiTestHelper.waitForEvents(sleep, expected, count, timeout)
            _, step, expected, timeout = a
            rt.flush()
            waited = 0
            while len(rows) < expected and waited <= timeout:
                sleep(step)
                waited += step
                rt.flush()
    rt.shutdown()
    return rows, tss
