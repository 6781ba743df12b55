"""CPU-side checks of the C-ABI library: it loads, exports every entry point include/siddhi_gpu.h
declares, and the ctypes mirror of the structs has the C layout.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "siddhi_gpu.h")


def header_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sg_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from siddhi_amd import _native
    lib = _native.load_library()
    syms = header_symbols()
    assert set(syms) == set(_native.SYMBOLS)
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.sg_version().decode().startswith("siddhi_gpu")


def test_struct_layout_matches_c(tmp_path):
    from siddhi_amd import _native as N
    src = tmp_path / "sz.c"
    src.write_text('#include "siddhi_gpu.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(){'
                   'printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(sg_state_desc), sizeof(sg_receiver_desc),'
                    ' sizeof(sg_nfa_desc), sizeof(sg_options), sizeof(sg_batch), sizeof(sg_matches), sizeof(sg_timing),'
                   ' offsetof(sg_nfa_desc, code), offsetof(sg_nfa_desc, shape), sizeof(sg_match_records));'
                   'printf("%zu %zu %zu\\n", sizeof(sg_match_columns), offsetof(sg_nfa_desc, n_sched),'
                   ' offsetof(sg_match_columns, nulls));return 0;}')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.dirname(HDR), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(N.sg_state_desc), ctypes.sizeof(N.sg_receiver_desc), ctypes.sizeof(N.sg_nfa_desc),
            ctypes.sizeof(N.sg_options), ctypes.sizeof(N.sg_batch), ctypes.sizeof(N.sg_matches),
            ctypes.sizeof(N.sg_timing), N.sg_nfa_desc.code.offset, N.sg_nfa_desc.shape.offset,
            ctypes.sizeof(N.sg_match_records), ctypes.sizeof(N.sg_match_columns), N.sg_nfa_desc.n_sched.offset,
            N.sg_match_columns.nulls.offset]
    assert got == want


def test_desc_builds_for_all_configs():
    from siddhi_amd import compiler as C, lowering as L, synth, _native as N
    for name, q in synth.QUERIES.items():
        app = C.parse(q)
        if app.partitions:
            p = app.partitions[0]
            ctx = L.make_context(app, p.queries[0], p, {})
        else:
            ctx = L.make_context(app, app.queries[0], None, {})
        nfa = L.lower(ctx)
        d = N.build_desc(nfa)
        assert d.n_states == len(nfa.states)
    shapes = {}
    for name in ("C1", "C2", "C4"):
        app = C.parse(synth.QUERIES[name])
        if app.partitions:
            ctx = L.make_context(app, app.partitions[0].queries[0], app.partitions[0], {})
        else:
            ctx = L.make_context(app, app.queries[0], None, {})
        shapes[name] = L.lower(ctx).shape
    assert shapes == {"C1": L.SHAPE_EVERY_NEXT_CMP, "C2": L.SHAPE_EVERY_NEXT_CMP, "C4": L.SHAPE_EVERY_ABSENT_EQ}
