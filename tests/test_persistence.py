"""Persistence through the host API (SiddhiManager.setPersistenceStore, SiddhiAppRuntime.persist /
restoreLastRevision / restoreRevision; C/SiddhiAppRuntime.java:595-661, InMemoryPersistenceStore.java:30-90),
transcribed from the reference's PersistenceTestCase (T/managment/PersistenceTestCase.java:145-254): a count
pattern's partial match persisted, the app shut down and rebuilt, the revision restored, and the match completed
by events sent after the restore -- on the MI355X engine (general machine).  The no-store case runs on the CPU."""
import numpy as np
import pytest

from siddhi_amd import (CannotRestoreSiddhiAppStateException, InMemoryPersistenceStore, NoPersistenceStoreException,
                        QueryCallback, SiddhiManager)

APP = ("@app:name('Test') "
       "define stream Stream1 (symbol string, price float, volume int); "
       "define stream Stream2 (symbol string, price float, volume int); "
       "@info(name = 'query1') "
       "from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
       "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
       "   e1[3].price as price1_3, e2.price as price2 "
       "insert into OutputStream ;")


class _Check(QueryCallback):
    def __init__(self):
        self.count = 0
        self.rows = []

    def receive(self, ts, ins, rem):
        for e in ins:
            self.count += 1
            self.rows.append(list(e.getData()))


def _f(x):
    return float(np.float32(x))


@pytest.mark.gpu
def test_persistence_test2_count_pattern_on_gpu():
    """PersistenceTestCase.persistenceTest2 (:145-230) through the MI355X engine."""
    from siddhi_amd._native import GpuEngine
    store = InMemoryPersistenceStore()
    mgr = SiddhiManager(engine=GpuEngine)
    mgr.setPersistenceStore(store)
    cb = _Check()
    rt = mgr.createSiddhiAppRuntime(APP)
    rt.addCallback("query1", cb)
    s1 = rt.getInputHandler("Stream1")
    rt.start()
    s1.send(["WSO2", 25.6, 100])
    s1.send(["GOOG", 47.6, 100])
    s1.send(["GOOG", 13.7, 100])
    rt.flush()
    assert cb.count == 0
    rev = rt.persist().getRevision()
    assert rev.endswith("_Test")
    rt.shutdown()
    rt = mgr.createSiddhiAppRuntime(APP)
    rt.addCallback("query1", cb)
    s1 = rt.getInputHandler("Stream1")
    s2 = rt.getInputHandler("Stream2")
    rt.start()
    assert rt.restoreLastRevision() == rev
    s2.send(["IBM", 45.7, 100])
    s1.send(["GOOG", 47.8, 100])
    s2.send(["IBM", 55.7, 100])
    rt.shutdown()
    assert cb.count == 1
    assert cb.rows == [[_f(25.6), _f(47.6), None, None, _f(45.7)]]


@pytest.mark.gpu
def test_restore_revision_rejects_another_apps_state():
    from siddhi_amd._native import GpuEngine
    store = InMemoryPersistenceStore()
    mgr = SiddhiManager(engine=GpuEngine)
    mgr.setPersistenceStore(store)
    rt = mgr.createSiddhiAppRuntime(APP)
    rt.start()
    rev = rt.persist().getRevision()
    rt.shutdown()
    other = APP.replace("query1", "query9")
    rt2 = mgr.createSiddhiAppRuntime(other)
    rt2.start()
    with pytest.raises(CannotRestoreSiddhiAppStateException):
        rt2.restoreRevision(rev)
    rt2.shutdown()


def test_persistence_test3_no_store():
    """PersistenceTestCase.persistenceTest3 (:232-254): persist() without a store raises NoPersistenceStoreException
    (SnapshotService.java:530)."""
    from siddhi_amd.runtime import Batch, Outputs  # noqa: F401

    class _Null:
        def __init__(self, ctx):
            self.nsel = len(ctx.query.select)

        def push(self, b):
            pass

        def fetch(self):
            z = np.zeros(0, np.int64)
            return Outputs(z.astype(np.uint64), z, z.astype(np.int32), z.astype(np.uint32),
                           np.zeros((0, self.nsel), np.int64), np.zeros((0, self.nsel), np.uint8))

        def snapshot(self):
            return b""

        def close(self):
            pass

    rt = SiddhiManager(engine=_Null).createSiddhiAppRuntime(APP)
    rt.start()
    with pytest.raises(NoPersistenceStoreException):
        rt.persist()
    with pytest.raises(NoPersistenceStoreException):
        rt.restoreLastRevision()


def test_in_memory_store_revisions():
    s = InMemoryPersistenceStore()
    assert s.getLastRevision("a") is None
    s.save("a", "1_a", b"x")
    s.save("a", "1_a", b"y")
    s.save("a", "2_a", b"z")
    assert s.revisions["a"] == ["1_a", "2_a"] and s.load("a", "1_a") == b"y" and s.getLastRevision("a") == "2_a"
    s.clearAllRevisions("a")
    assert s.getLastRevision("a") is None and s.load("a", "2_a") is None
