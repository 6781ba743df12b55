"""Known-answer tests transcribed from the reference's own test suite.

Each case restates one reference test: the app text verbatim, the `send` sequence with explicit
timestamps (ts = cumulative Thread.sleep gaps; playback tests keep their literal timestamps), and the
expected rows the reference test asserts, flattened in delivery order.  These pin the CPU oracle
(tests/test_oracle_kats.py) and, through it, the HIP engine (tests/test_gpu_parity.py).

T/ = /root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/
"""
import numpy as np


def f(x):
    """A Java float literal as the Python float the engine returns (float32 widened)."""
    return float(np.float32(x))


S1_S2 = ("define stream Stream1 (symbol string, price float, volume int); "
         "define stream Stream2 (symbol string, price float, volume int); ")
S1 = "define stream Stream1 (symbol string, price float, volume int); "

KATS = [
    dict(  # B1  T/query/pattern/WithinPatternTestCase.java:48-98
        name="B1_within_every_two_streams",
        app=S1_S2 + "@info(name = 'query1') "
        "from every e1=Stream1[price>20] -> e2=Stream2[price>e1.price] within 1 sec "
        "select e1.symbol as symbol1, e2.symbol as symbol2 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 1500, ["GOOG", 54.0, 100]),
               ("Stream2", 2000, ["IBM", 55.7, 100])],
        expect=[["GOOG", "IBM"]]),
    dict(  # B2  WithinPatternTestCase.java:213-263 (expiry re-arm via withinEvery)
        name="B2_every_group_within_rearm",
        app=S1 + "@info(name = 'query1') "
        "from every (e1=Stream1 -> e2=Stream1[symbol == e1.symbol]) within 5 sec "
        "select e1.symbol as symbol1, e1.volume as volume1, e2.symbol as symbol2, e2.volume as volume2 "
        "insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 6000, ["WSO2", 55.7, 150]),
               ("Stream1", 6500, ["WSO2", 58.7, 200]), ("Stream1", 6500, ["WSO2", 58.7, 250])],
        expect=[["WSO2", 150, "WSO2", 200]]),
    dict(  # B3  WithinPatternTestCase.java:266-321
        name="B3_every_three_states_within",
        app=S1 + "@info(name = 'query1') "
        "from every (e1=Stream1 -> e2=Stream1[symbol == e1.symbol] -> e3=Stream1[symbol == e2.symbol]) "
        "within 5 sec select e1.symbol as symbol1, e1.volume as volume1, e2.symbol as symbol2, "
        "e2.volume as volume2, e3.symbol as symbol3, e3.volume as volume3 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 0, ["WSO2", 56.6, 150]),
               ("Stream1", 6000, ["WSO2", 57.7, 200]), ("Stream1", 6500, ["WSO2", 58.7, 250]),
               ("Stream1", 6500, ["WSO2", 57.7, 300]), ("Stream1", 6500, ["WSO2", 59.7, 350])],
        expect=[["WSO2", 200, "WSO2", 250, "WSO2", 300]]),
    dict(  # B4  WithinPatternTestCase.java:325-388
        name="B4_every_three_states_two_matches",
        app=S1 + "@info(name = 'query1') "
        "from every (e1=Stream1 -> e2=Stream1[symbol == e1.symbol] -> e3=Stream1[symbol == e2.symbol]) "
        "within 5 sec select e1.symbol as symbol1, e1.volume as volume1, e2.symbol as symbol2, "
        "e2.volume as volume2, e3.symbol as symbol3, e3.volume as volume3 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 0, ["WSO2", 55.7, 150]),
               ("Stream1", 0, ["WSO2", 58.7, 200]), ("Stream1", 0, ["WSO2", 58.7, 210]),
               ("Stream1", 500, ["WSO2", 58.7, 250]), ("Stream1", 500, ["WSO2", 58.7, 260]),
               ("Stream1", 500, ["WSO2", 58.7, 270])],
        expect=[["WSO2", 100, "WSO2", 150, "WSO2", 200], ["WSO2", 210, "WSO2", 250, "WSO2", 260]]),
    dict(  # B4b WithinPatternTestCase.java:391-446
        name="B4b_every_three_states_after_expiry",
        app=S1 + "@info(name = 'query1') "
        "from every (e1=Stream1 -> e2=Stream1[symbol == e1.symbol] -> e3=Stream1[symbol == e2.symbol]) "
        "within 5 sec select e1.symbol as symbol1, e1.volume as volume1, e2.symbol as symbol2, "
        "e2.volume as volume2, e3.symbol as symbol3, e3.volume as volume3 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 6000, ["WSO2", 56.6, 150]),
               ("Stream1", 6000, ["WSO2", 57.7, 200]), ("Stream1", 6500, ["WSO2", 58.7, 250]),
               ("Stream1", 6500, ["WSO2", 57.7, 300]), ("Stream1", 6500, ["WSO2", 59.7, 350])],
        expect=[["WSO2", 150, "WSO2", 200, "WSO2", 250]]),
    dict(  # B5  T/query/pattern/EveryPatternTestCase.java:538-601 (duplicate e1 -> first state)
        name="B5_duplicate_reference",
        app=S1 + "@info(name = 'query1') "
        "from every e1=Stream1[symbol == 'MSFT'] -> e1=Stream1[symbol == 'WSO2'] "
        "select e1.price as price1 insert into OutputStream ;",
        sends=[("Stream1", 0, ["MSFT", 55.6, 100]), ("Stream1", 100, ["MSFT", 77.6, 100]),
               ("Stream1", 200, ["WSO2", 57.6, 100])],
        expect=[[f(55.6)], [f(77.6)]]),
    dict(  # B6  T/query/pattern/CountPatternTestCase.java:47-104 (chain aliasing after min)
        name="B6_count_chain_aliasing",
        app=S1_S2 + "@info(name = 'query1') "
        "from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
        "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
        "e1[3].price as price1_3, e2.price as price2 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 25.6, 100]), ("Stream1", 100, ["GOOG", 47.6, 100]),
               ("Stream1", 200, ["GOOG", 13.7, 100]), ("Stream1", 300, ["GOOG", 47.8, 100]),
               ("Stream2", 400, ["IBM", 45.7, 100]), ("Stream2", 500, ["IBM", 55.7, 100])],
        expect=[[f(25.6), f(47.6), f(47.8), None, f(45.7)]]),
    dict(  # B7  CountPatternTestCase.java:107-164
        name="B7_count_then_next",
        app=S1_S2 + "@info(name = 'query1') "
        "from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
        "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
        "e1[3].price as price1_3, e2.price as price2 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 25.6, 100]), ("Stream1", 100, ["GOOG", 47.6, 100]),
               ("Stream1", 200, ["GOOG", 13.7, 100]), ("Stream2", 300, ["IBM", 45.7, 100]),
               ("Stream1", 400, ["GOOG", 47.8, 100]), ("Stream2", 500, ["IBM", 55.7, 100])],
        expect=[[f(25.6), f(47.6), None, None, f(45.7)]]),
    dict(  # B8  CountPatternTestCase.java:725-808 (emit at n == min)
        name="B8_every_then_count_min4",
        app="define stream EventStream (symbol string, price float, volume int); @info(name = 'query1') "
        "from every e1 = EventStream -> e2 = EventStream [e1.symbol==e2.symbol]<4:6> "
        "select e1.volume as volume1, e2[0].volume as volume2, e2[1].volume as volume3, e2[2].volume as "
        "volume4, e2[3].volume as volume5, e2[4].volume as volume6, e2[5].volume as volume7 "
        "insert into StockQuote;",
        sends=[("EventStream", 0, ["IBM", 75.6, 100]), ("EventStream", 0, ["IBM", 75.6, 200]),
               ("EventStream", 0, ["IBM", 75.6, 300]), ("EventStream", 0, ["GOOG", 21.0, 91]),
               ("EventStream", 0, ["IBM", 75.6, 400]), ("EventStream", 0, ["IBM", 75.6, 500]),
               ("EventStream", 0, ["GOOG", 21.0, 91]), ("EventStream", 0, ["IBM", 75.6, 600]),
               ("EventStream", 0, ["IBM", 75.6, 700]), ("EventStream", 0, ["IBM", 75.6, 800]),
               ("EventStream", 0, ["GOOG", 21.0, 91]), ("EventStream", 0, ["IBM", 75.6, 900])],
        expect=[[100, 200, 300, 400, 500, None, None], [200, 300, 400, 500, 600, None, None],
                [300, 400, 500, 600, 700, None, None], [400, 500, 600, 700, 800, None, None],
                [500, 600, 700, 800, 900, None, None]]),
    dict(  # B9  T/query/pattern/LogicalPatternTestCase.java:308-358
        name="B9_next_then_and",
        app=S1_S2 + "@info(name = 'query1') "
        "from e1=Stream1[price > 20] -> e2=Stream2[price > e1.price] and e3=Stream1['IBM' == symbol] "
        "select e1.symbol as symbol1, e2.price as price2, e3.price as price3 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream2", 100, ["IBM", 72.7, 100]),
               ("Stream1", 200, ["IBM", 75.7, 100])],
        expect=[["WSO2", f(72.7), f(75.7)]]),
    dict(  # B10 LogicalPatternTestCase.java:568-633
        name="B10_every_then_and_three_streams",
        app=S1_S2 + "define stream Stream3 (symbol string, price float, volume int); "
        "@info(name = 'query1') "
        "from every e1=Stream1[price >20] -> e2=Stream2['IBM' == symbol] and e3=Stream3['WSO2' == symbol]"
        "select e1.price as price1, e2.price as price2, e3.price as price3 insert into OutputStream ;",
        sends=[("Stream1", 0, ["IBM", 25.5, 100]), ("Stream1", 100, ["IBM", 59.65, 100]),
               ("Stream2", 200, ["IBM", 45.5, 100]), ("Stream3", 300, ["WSO2", 46.56, 100])],
        expect=[[f(25.5), f(45.5), f(46.56)], [f(59.65), f(45.5), f(46.56)]]),
    dict(  # B11 T/query/sequence/SequenceTestCase.java:408-471
        name="B11_sequence_every_or",
        app=S1_S2 + "@info(name = 'query1') "
        "from every e1=Stream2[price>20], e2=Stream2[price>e1.price] or e3=Stream2[symbol=='IBM'] "
        "select e1.price as price1, e2.price as price2, e3.price as price3 insert into OutputStream ;",
        sends=[("Stream2", 0, ["WSO2", 59.6, 100]), ("Stream2", 100, ["WSO2", 55.6, 100]),
               ("Stream2", 200, ["IBM", 55.7, 100]), ("Stream2", 300, ["WSO2", 57.6, 100])],
        expect=[[f(55.6), f(55.7), None], [f(55.7), f(57.6), None]]),
    dict(  # B12a SequenceTestCase.java:1078-1140
        name="B12a_sequence_plus_last",
        app=S1_S2 + "@info(name = 'query1') "
        "from every e1=Stream1[price>20], "
        "e2=Stream1[((e2[last].price is null) and price>=e1.price) or ((not (e2[last].price is null)) and "
        "price>=e2[last].price)]+, e3=Stream1[price<e2[last].price] "
        "select e1.price as price1, e2[0].price as price2, e2[1].price as price3, e3.price as price4 "
        "insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 29.6, 100]), ("Stream1", 100, ["WSO2", 25.0, 100]),
               ("Stream1", 200, ["WSO2", 35.6, 100]), ("Stream1", 300, ["WSO2", 57.6, 100]),
               ("Stream1", 400, ["IBM", 47.6, 100])],
        expect=[[f(25.0), f(35.6), f(57.6), f(47.6)]]),
    dict(  # B12b SequenceTestCase.java:1143-1208
        name="B12b_sequence_plus_last_short",
        app=S1_S2 + "@info(name = 'query1') "
        "from every e1=Stream1[price>20], "
        "e2=Stream1[((e2[last].price is null) and price>=e1.price) or ((not (e2[last].price is null)) and "
        "price>=e2[last].price)]+, e3=Stream1[price<e2[last].price] "
        "select e1.price as price1, e2[0].price as price2, e2[1].price as price3, e3.price as price4 "
        "insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 25.0, 100]), ("Stream1", 100, ["WSO2", 40.0, 100]),
               ("Stream1", 200, ["WSO2", 35.0, 100])],
        expect=[[f(25.0), f(40.0), None, f(35.0)]]),
    dict(  # B13 T/query/partition/PatternPartitionTestCase.java:171-251
        name="B13_partitioned_every",
        app="define stream Stream1 (symbol string, price float, volume int); "
        "define stream Stream2 (symbol string, price1 float, volume int); "
        "partition with (volume of Stream1,volume of Stream2) begin @info(name = 'query1') "
        "from every e1=Stream1[price>20] -> e2=Stream2[price1>e1.price] "
        "select e1.symbol as symbol1, e2.symbol as symbol2 insert into OutputStream ; end",
        stream_callback="OutputStream",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream1", 100, ["GOOG", 55.6, 100]),
               ("Stream2", 200, ["IBM", 55.7, 100]), ("Stream1", 300, ["WSO2", 55.6, 150]),
               ("Stream1", 400, ["GOOG", 55.6, 150]), ("Stream2", 500, ["IBM", 55.7, 150])],
        expect=[["WSO2", "IBM"], ["GOOG", "IBM"], ["WSO2", "IBM"], ["GOOG", "IBM"]]),
    dict(  # B14 T/query/pattern/absent/AbsentWithEveryPatternTestCase.java:277-309 (playback)
        name="B14_every_then_absent_playback",
        app="@app:playback(idle.time = '10 milliseconds', increment = '10 milliseconds') " + S1 +
        "@info(name = 'query1') "
        "from every e1=Stream1[price>20] -> not Stream1[symbol==e1.symbol and price>e1.price] for 1sec "
        "select e1.symbol as symbol insert into OutputStream ;",
        sends=[("Stream1", 1544512385000, ["WSO2", 55.6, 100]), ("Stream1", 1544512385100, ["GOOG", 55.6, 100]),
               ("Stream1", 1544512385800, ["WSO2", 55.7, 100]), ("Stream1", 1544512386200, ["GOOG", 55.6, 100])],
        expect=[["GOOG"]], expect_ts=[1544512385100 + 1000]),
    dict(  # B15 T/query/pattern/absent/EveryAbsentPatternTestCase.java:114-162 (playback)
        name="B15_every_absent_within",
        app="@app:playback " + S1_S2 + "define stream TimerStream (symbol string); @info(name = 'query1') "
        "from (e1=Stream1[price>20] -> every not Stream2[price>e1.price] for 900 milliseconds) within 2 sec "
        "select e1.symbol as symbol1 insert into OutputStream ;",
        sends=[("Stream1", 1700000000000, ["WSO2", 55.6, 100]), ("TimerStream", 1700000001000, ["UPDATE-TIME"]),
               ("TimerStream", 1700000002000, ["UPDATE-TIME"]), ("TimerStream", 1700000003000, ["UPDATE-TIME"])],
        expect=[["WSO2"], ["WSO2"]]),
    dict(  # B16 T/query/pattern/absent/AbsentPatternTestCase.java:1745-1781, re-expressed in playback
        name="B16_partitioned_absent_playback",
        app="@app:playback define stream CustomerStream (customerId string); define stream Tick (x int); "
        "partition with (customerId of CustomerStream) begin "
        "from e1=CustomerStream -> not CustomerStream[customerId == e1.customerId] for 1 sec "
        "select e1.customerId insert into OutputStream; end ",
        stream_callback="OutputStream",
        sends=[("CustomerStream", 0, ["customerA"]), ("CustomerStream", 0, ["customerB"]),
               ("CustomerStream", 500, ["customerB"]), ("Tick", 1000, [1])],
        expect=[["customerA"]]),
    # ---- absent-in-sequence (T/query/sequence/absent/AbsentSequenceTestCase.java), re-expressed in playback:
    # ts = cumulative Thread.sleep, and the trailing TestUtil.waitForInEvents(500, cb, 10) (up to 5 s of wall
    # clock for the timers) becomes a Tick event 5 s after the last send.
    dict(  # B17 AbsentSequenceTestCase.java:38-69 (testQueryAbsent1)
        name="B17_seq_then_absent_fires",
        app="@app:playback " + S1_S2 + "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>20], not Stream2[price>e1.price] for 1 sec "
        "select e1.symbol as symbol1 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Tick", 5000, [1])],
        expect=[["WSO2"]], expect_ts=[1000]),
    dict(  # B18 AbsentSequenceTestCase.java:71-106 (testQueryAbsent2): the timer fires before the late event
        name="B18_seq_absent_then_late_event",
        app="@app:playback " + S1_S2 + "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>20], not Stream2[price>e1.price] for 1 sec "
        "select e1.symbol as symbol1 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream2", 1100, ["IBM", 58.7, 100]), ("Tick", 6100, [1])],
        expect=[["WSO2"]]),
    dict(  # B19 AbsentSequenceTestCase.java:108-143 (testQueryAbsent3): a matching Stream2 event kills it
        name="B19_seq_absent_killed",
        app="@app:playback " + S1_S2 + "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>20], not Stream2[price>e1.price] for 1 sec "
        "select e1.symbol as symbol1 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream2", 100, ["IBM", 58.7, 100]), ("Tick", 5100, [1])],
        expect=[]),
    dict(  # B20 AbsentSequenceTestCase.java:145-180 (testQueryAbsent4): a non-matching Stream2 event does not
        name="B20_seq_absent_not_killed",
        app="@app:playback " + S1_S2 + "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>20], not Stream2[price>e1.price] for 1 sec "
        "select e1.symbol as symbol1 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 55.6, 100]), ("Stream2", 100, ["IBM", 50.7, 100]), ("Tick", 5100, [1])],
        expect=[["WSO2"]]),
    dict(  # B21 AbsentSequenceTestCase.java:329-368 (testQueryAbsent9): three states, killed by Stream3
        name="B21_seq_two_then_absent_killed",
        app="@app:playback " + S1_S2 + "define stream Stream3 (symbol string, price float, volume int); "
        "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>10], e2=Stream2[price>20], not Stream3[price>30] for 1 sec "
        "select e1.symbol as symbol1, e2.symbol as symbol2 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 15.6, 100]), ("Stream2", 100, ["IBM", 28.7, 100]),
               ("Stream3", 200, ["GOOGLE", 55.7, 100]), ("Tick", 5200, [1])],
        expect=[]),
    dict(  # B22 AbsentSequenceTestCase.java:370-410 (testQueryAbsent10): Stream3 below the threshold
        name="B22_seq_two_then_absent_fires",
        app="@app:playback " + S1_S2 + "define stream Stream3 (symbol string, price float, volume int); "
        "define stream Tick (x int); @info(name = 'query1') "
        "from e1=Stream1[price>10], e2=Stream2[price>20], not Stream3[price>30] for 1 sec "
        "select e1.symbol as symbol1, e2.symbol as symbol2 insert into OutputStream ;",
        sends=[("Stream1", 0, ["WSO2", 15.6, 100]), ("Stream2", 100, ["IBM", 28.7, 100]),
               ("Stream3", 200, ["GOOGLE", 25.7, 100]), ("Tick", 5200, [1])],
        expect=[["WSO2", "IBM"]]),

]


def run_kat(case, engine):
    """Drive one KAT through the host API on `engine`; returns (rows, timestamps)."""
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
    for (sid, ts, row) in case["sends"]:
        h = handlers.setdefault(sid, rt.getInputHandler(sid))
        h.send(ts, row)
    rt.shutdown()
    return rows, tss
