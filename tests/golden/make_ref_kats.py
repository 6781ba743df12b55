"""Transcribe known-answer tests from the reference's own Java test suite into data (tests/golden/ref_kats.json).

Run in the build container only (the reference tree is not on the GPU box):
    python tests/golden/make_ref_kats.py

Each reference @Test that follows the suite's common template is restated as data: the app text (string
literals concatenated as the test concatenates them), the `send` sequence with timestamps, and what the test
asserts -- the expected rows handed to TestUtil.addQueryCallback/addStreamCallback (checked in order,
TestUtil.java:124-143) and the asserted in-event count.  Tests with constructs outside that template (loops,
persistence, custom callbacks with computed checks, ...) are skipped and listed in the output.

A case is an action list up to the test's count assertion: `send` (stream, timestamp or None, row), `sleep`
(ms) and `wait_in_events` (TestUtil.waitForInEvents(ms, cb, retries), T/TestUtil.java:237-247).  Wall-clock
tests (clock "wall") are re-expressed in playback: the app gets `@app:playback` and the runner
(tests/ref_kats.py) advances the playback clock in 1 ms heartbeats through every sleep, so an event's timestamp
is the time it was sent at, every timer fires at its due time as the wall-clock Scheduler would
(Scheduler.java:89-114), and a timer re-armed from currentTime() (AbsentLogicalPreStateProcessor.java:199-209)
sees the time it fired at.  `@app:playback` tests with literal timestamps (clock "events") keep them.

Only inputs and expected outputs are written -- no reference source text is copied into the repo.
"""
import json
import os
import re
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_kats.json")

SUITES = [
    "query/pattern/absent/LogicalAbsentPatternTestCase.java",
    "query/sequence/absent/LogicalAbsentSequenceTestCase.java",
    "query/pattern/CountPatternTestCase.java",
    "query/pattern/LogicalPatternTestCase.java",
    "query/sequence/SequenceTestCase.java",
    "query/pattern/EveryPatternTestCase.java",
    "query/pattern/WithinPatternTestCase.java",
    "query/pattern/PatternTestCase.java",
    "query/partition/PatternPartitionTestCase.java",
    "query/partition/SequencePartitionTestCase.java",
    "query/pattern/absent/AbsentPatternTestCase.java",
    "query/pattern/absent/EveryAbsentPatternTestCase.java",
    "query/pattern/absent/AbsentWithEveryPatternTestCase.java",
    "query/sequence/absent/AbsentSequenceTestCase.java",
    "query/sequence/absent/EveryAbsentSequenceTestCase.java",
    "query/sequence/absent/AbsentWithEverySequenceTestCase.java",
    "query/pattern/ComplexPatternTestCase.java",
]


class Skip(Exception):
    pass


def java_strings(expr):
    """Concatenate the string literals of a Java `"a" + "b" + ...` expression."""
    out = []
    for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', expr):
        out.append(m.group(1).encode().decode("unicode_escape"))
    return "".join(out)


def java_value(tok):
    tok = tok.strip()
    if tok == "null":
        return None
    if tok in ("true", "false"):
        return tok == "true"
    m = re.fullmatch(r'"((?:[^"\\]|\\.)*)"', tok)
    if m:
        return m.group(1)
    m = re.fullmatch(r"(-?[0-9.]+(?:[eE][-+]?[0-9]+)?)([fFdDlL]?)", tok)
    if m:
        num, suf = m.groups()
        if suf in ("l", "L"):
            return {"L": int(num)}
        if suf in ("f", "F"):
            return {"F": float(num)}
        if suf in ("d", "D") or "." in num or "e" in num.lower():
            return {"D": float(num)}
        return int(num)
    m = re.fullmatch(r"\(\s*(int|long|float|double)\s*\)\s*(.+)", tok)
    if m:
        return java_value(m.group(2) + {"int": "", "long": "L", "float": "f", "double": "d"}[m.group(1)])
    raise Skip(f"value {tok!r}")


def split_args(s):
    out, depth, cur, q = [], 0, "", False
    for ch in s:
        if ch == '"':
            q = not q
        if not q and ch in "({[":
            depth += 1
        if not q and ch in ")}]":
            depth -= 1
        if not q and ch == "," and depth == 0:
            out.append(cur)
            cur = ""
            continue
        cur += ch
    if cur.strip():
        out.append(cur)
    return out


def object_arrays(s):
    rows = []
    for m in re.finditer(r"new\s+Object\[\]\s*\{((?:[^{}]|\{[^{}]*\})*)\}", s):
        rows.append([java_value(t) for t in split_args(m.group(1))])
    return rows


def statements(body):
    """Split a method body into ';'-terminated statements (string-literal aware)."""
    out, cur, q, depth = [], "", False, 0
    for ch in body:
        if ch == '"' and not cur.endswith("\\"):
            q = not q
        if not q and ch == "{":
            depth += 1
        if not q and ch == "}":
            depth -= 1
        cur += ch
        if not q and ch == ";" and depth <= 0:
            out.append(cur.strip())
            cur = ""
    return out


def take_block(text, at):
    """(block, end): the balanced {...} starting at the first '{' at or after `at`."""
    i = text.index("{", at)
    depth, q, j = 0, False, i
    while True:
        ch = text[j]
        if ch == '"' and text[j - 1] != "\\":
            q = not q
        if not q:
            depth += {"{": 1, "}": -1}.get(ch, 0)
            if depth == 0:
                return text[i:j + 1], j + 1
        j += 1


def every_event_form(block, rows):
    """One assertArrayEquals inside the callback's `for (Event e : events)` loop, not selected by an event counter:
    the test asserts that row for every event it receives."""
    return (len(rows) == 1 and re.search(r"for\s*\(\s*Event\s+\w+\s*:", block) is not None
            and re.search(r"\bcase\b|if\s*\(\s*\w*[cC]ount", block) is None)


def parse_callback(block):
    """Expected rows of an inline QueryCallback/StreamCallback: its assertArrayEquals(new Object[]{..}, ...getData())
    calls in textual order (the suites assert event k under `case k:` / `if (inEventCount == k-1)`)."""
    if re.search(r"removeEvents\s*!=\s*null\s*\)\s*\{[^}]*assert", block):
        raise Skip("remove-event assertions")
    rows = []
    for m in re.finditer(r"assertArrayEquals\((.*?)\.getData\(\)\s*\)", block, re.S):
        arr = object_arrays(m.group(1))
        if len(arr) != 1:
            raise Skip("computed expectation")
        rows.append(arr[0])
    if re.search(r"assert(?!ArrayEquals|Same|True|False|Equals\(\s*\d|Equals\(\s*\"|JUnit)\w*\(", block):
        raise Skip("other callback assertions")
    return rows


def parse_test(name, body):
    if "persist" in body or "restore" in body:
        raise Skip("persistence")
    # inline callbacks first (their `for (Event e : inEvents)` loops are not driver loops)
    expect, cb, every = None, None, False
    m = re.search(r"\w+\.addCallback\(\s*\"(\w+)\"\s*,\s*new\s+(Query|Stream)Callback\(\)", body)
    if m:
        block, e = take_block(body, m.end())
        cb = ("Query" if m.group(2) == "Query" else "Stream", m.group(1))
        expect = parse_callback(block)
        every = every_event_form(block, expect)
        body = body[:m.start()] + body[e:]
        if re.search(r"\w+\.addCallback\(", body):
            raise Skip("several callbacks")
    if re.search(r"\b(for|while)\s*\(", body):
        raise Skip("loop in the driver")
    strings, handlers, actions, count = {}, {}, [], None
    playback, app = False, None
    for st in statements(body):
        m = re.match(r"String\s+(\w+)\s*=\s*(.*);$", st, re.S)
        if m:
            strings[m.group(1)] = java_strings(m.group(2))
            continue
        m = re.search(r"createSiddhiAppRuntime\((.*)\);$", st, re.S)
        if m:
            parts = [p.strip() for p in m.group(1).split("+")]
            txt = ""
            for p in parts:
                if p in strings:
                    txt += strings[p]
                elif p.startswith('"'):
                    txt += java_strings(p)
                else:
                    raise Skip(f"app expression {p}")
            app = txt
            continue
        m = re.match(r"InputHandler\s+(\w+)\s*=\s*\w+\.getInputHandler\(\"(\w+)\"\);$", st)
        if m:
            handlers[m.group(1)] = m.group(2)
            continue
        m = re.search(r"TestUtil\.add(Query|Stream)Callback\(\w+,\s*\"(\w+)\"(.*)\);$", st, re.S)
        if m:
            if cb is not None:
                raise Skip("several callbacks")
            cb = (m.group(1), m.group(2))
            expect = object_arrays(m.group(3))
            continue
        if count is not None:
            continue   # everything after the first count assertion
        m = re.match(r"Thread\.sleep\((\d+)\);$", st)
        if m:
            actions.append(["sleep", int(m.group(1))])
            continue
        m = re.match(r"TestUtil\.waitForInEvents\((\d+),\s*\w+,\s*(\d+)\);$", st)
        if m:
            actions.append(["wait_in_events", int(m.group(1)), int(m.group(2))])
            continue
        # SiddhiTestHelper.waitForEvents(sleepTime, expectedCount, actualCount, timeout): sleep until the callback
        # has counted expectedCount events or the timeout passed (io/siddhi/core/util/SiddhiTestHelper.java:49-57)
        m = re.match(r"SiddhiTestHelper\.waitForEvents\((\d+),\s*(\d+),\s*\w+,\s*(\d+)\);$", st)
        if m:
            actions.append(["wait_events", int(m.group(1)), int(m.group(2)), int(m.group(3))])
            continue
        m = re.match(r"(\w+)\.send\((.*)\);$", st, re.S)
        if m and m.group(1) in handlers:
            args = m.group(2)
            rows = object_arrays(args)
            if len(rows) != 1:
                raise Skip("send of several events")
            head = args[:args.find("new")].strip().rstrip(",").strip()
            if head:
                if not re.fullmatch(r"\d+[lL]?", head):
                    raise Skip(f"timestamp expression {head}")
                playback = True
                actions.append(["send", handlers[m.group(1)], int(re.sub(r"[lL]$", "", head)), rows[0]])
            else:
                actions.append(["send", handlers[m.group(1)], None, rows[0]])
            continue
        m = re.search(r"assertEquals\((?:\"Number of success events\",\s*)?(\d+),\s*(?:\w+\.getInEventCount\(\)|"
                      r"inEventCount(?:\.get\(\))?)\)", st)
        if m:
            count = int(m.group(1))
            continue
        if re.search(r"SiddhiTestHelper|EventPrinter|new QueryCallback|new StreamCallback|\.send\(", st):
            raise Skip("unrecognised driver statement")
    if app is None or cb is None or count is None:
        raise Skip("template not matched")
    if re.search(r"\b(instanceOf\w*|convert|ifThenElse|coalesce|str:|math:)\s*\(", app):
        raise Skip("function executors (outside the state-engine path)")
    if re.search(r"#\w", app):
        raise Skip("inner (#) streams between partition queries: plain queries beside the pattern (outside the "
                   "state-engine path)")
    if expect and len(expect) > count and not every:
        raise Skip("more expected rows than the asserted count")
    if playback and any(a[0] == "send" and a[2] is None for a in actions):
        raise Skip("mixed explicit / implicit timestamps")
    return dict(app=app, cb=cb, actions=actions, expect=expect or [], count=count, literal_ts=playback,
                every=every)


def to_kat(name, src, p):
    app = p["app"]
    kat = dict(name=name, src=src, expect=p["expect"], expect_count=p["count"])
    if p["every"]:
        kat["expect_every"] = True
    if p["literal_ts"]:
        kat["actions"] = [a for a in p["actions"] if a[0] == "send"]
        kat["clock"] = "events"
    else:
        if "@app:playback" in app:
            raise Skip("playback app without literal timestamps")
        app = "@app:playback " + app
        kat["actions"] = p["actions"]
        kat["clock"] = "wall"
    kat["app"] = app
    if p["cb"][0] == "Stream":
        kat["stream_callback"] = p["cb"][1]
    return kat


def main():
    kats, skipped = [], []
    for rel in SUITES:
        path = REF + rel
        if not os.path.exists(path):
            continue
        src = open(path).read()
        for m in re.finditer(r"@Test[^\n]*\n\s*public void (\w+)\(\)[^{]*\{", src):
            name = m.group(1)
            i, depth = m.end(), 1
            while depth:
                depth += {"{": 1, "}": -1}.get(src[i], 0)
                i += 1
            body = src[m.end():i - 1]
            line = src[:m.start()].count("\n") + 2
            ref = f"T/{rel}:{line}"
            try:
                if "@Test(enabled = false" in src[m.start():m.start() + 40]:
                    raise Skip("disabled")
                kats.append(to_kat(f"{os.path.basename(rel)[:-5]}.{name}", ref, parse_test(name, body)))
                if len(kats) and kats[-1]["name"] in {k["name"] for k in kats[:-1]}:
                    raise Skip("duplicate name")
            except Skip as e:
                skipped.append((ref, name, str(e)))
    json.dump(kats, open(OUT, "w"), indent=0)
    print(f"{len(kats)} KATs written to {OUT}; {len(skipped)} tests skipped")
    if "-v" in sys.argv:
        for s in skipped:
            print("  skip", *s)


if __name__ == "__main__":
    main()
