"""Private-segment (scratch) and VGPR report for every gfx950 kernel in libsiddhi_gpu.so.

Scans the library for clang offload bundles (one per translation unit), extracts each gfx950 code object and reads
its kernel descriptors with llvm-readelf --notes.  Usage: python profiles/scratch_report.py [lib] [--all]
Prints the kernels whose private segment is non-zero (all kernels with --all)."""
import os
import re
import struct
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(blob):
    pos = 0
    while True:
        pos = blob.find(MAGIC, pos)
        if pos < 0:
            return
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple:
                yield blob[pos + off:pos + off + size]
        pos = q


def kernels(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        out = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    name, rows = None, []
    cur = {}
    for line in out.splitlines():
        m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_count|sgpr_count|group_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        cur[k] = v
        if k == "vgpr_count" and "name" in cur:
            rows.append((cur["name"], int(cur.get("private_segment_fixed_size", 0)), int(cur["vgpr_count"]),
                         int(cur.get("group_segment_fixed_size", 0))))
            cur = {}
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "siddhi_amd", "libsiddhi_gpu.so")
    blob = open(lib, "rb").read()
    allk = [r for co in code_objects(blob) for r in kernels(co)]
    show = allk if "--all" in sys.argv else [r for r in allk if r[1] > 0]
    for name, priv, vgpr, lds in sorted(show, key=lambda r: (-r[1], r[0])):
        print(f"{priv:6d} B private  {vgpr:4d} VGPR  {lds:6d} B LDS  {name}")
    print(f"{len(allk)} kernels, {sum(1 for r in allk if r[1] > 0)} with a private segment")


if __name__ == "__main__":
    main()
