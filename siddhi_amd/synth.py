"""Counter-based synthetic event generator for the benchmark configs.

x(col, i) = splitmix64(seed_cfg ^ (col << 56) ^ i), seed_cfg = 0x5EED0000 + cfg, so every shard can
regenerate its own slice.  Columns:
  ts_i    = T0 + floor(i / R)                      (ms, non-decreasing; @app:playback timestamps)
  price_i = float32(x(1,i) % 4001) / 100.0f        (exact IEEE division, in [0, 40])
  key_i   = x(2,i) % K                             (symbol "S%07d", dictionary-encoded to key_i)
  v_i     = int32(x(3,i) % 1000),  w_i = int32(x(5,i) % 1000)
  id_i    = i  (C1-C3, C5);  C4: id_i = x(4,i) % M,  seq_i = i
The same generator feeds the HIP engine, the CPU oracle baseline and the parity tests.
"""
from __future__ import annotations

import numpy as np

T0 = 1_700_000_000_000
GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB

CONFIGS = {
    # name: (cfg number, events, keys (or ids M for C4), rate events/ms)
    "C1": (1, 1_000_000, 1, 1),
    "C2": (2, 100_000_000, 10_000, 1_000),
    "C3": (3, 100_000_000, 10_000, 1_000),
    "C4": (4, 10_000_000, 10_000, 1),
    "C5": (5, 1_000_000_000, 1_000_000, 10_000),
    # PatternPartitionTestCase's canonical two-stream shape (T/query/partition/PatternPartitionTestCase.java:54-64)
    # at C2's scale: not a BASELINE config, the workload VERDICT r02 item 5 names for the per-key machine
    "PP": (6, 100_000_000, 10_000, 1_000),
}

QUERIES = {
    "C1": ("define stream StockStream (id long, symbol string, price float); "
           "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
           "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M;"),
    "C2": ("define stream StockStream (id long, symbol string, price float); "
           "partition with (symbol of StockStream) begin @info(name='q') "
           "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
           "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;"),
    "C3": ("define stream S (id long, symbol string, v int, w int); "
           "partition with (symbol of S) begin @info(name='q') "
           "from e1=S[v>500], e2=S[v>e1.v]<2:5>, e3=S[v<e1.v] "
           "select e1.id as i1, e2[0].id as i2a, e2[last].id as i2z, e3.id as i3 insert into M; end;"),
    "C3b": ("define stream S (id long, symbol string, v int, w int); "
            "partition with (symbol of S) begin @info(name='q') "
            "from every e1=S[v>500], e2=S[v>e1.v]<1:5>, e3=S[v<e1.v] or e4=S[w<e1.w] "
            "select e1.id as i1, e2[0].id as i2a, e2[last].id as i2z, e3.id as i3, e4.id as i4 "
            "insert into M; end;"),
    "C3c": ("define stream S (id long, symbol string, v int, w int); "
            "partition with (symbol of S) begin @info(name='q') "
            "from every e1=S[v>500] -> e2=S[v>e1.v]<2:5> -> e3=S[v<e1.v] and e4=S[w<e1.w] within 1 sec "
            "select e1.id as i1, e2[0].id as i2a, e2[last].id as i2z, e3.id as i3, e4.id as i4 "
            "insert into M; end;"),
    "C4": ("@app:playback define stream S (id long, seq long); define stream Tick (x int); "
           "@info(name='q') from every e1=S -> not S[id==e1.id] for 5 sec "
           "select e1.seq as seq1, e1.id as id1 insert into M;"),
    "PP": ("define stream Stream1 (symbol string, price float, volume int); "
           "define stream Stream2 (symbol string, price float, volume int); "
           "partition with (volume of Stream1, volume of Stream2) begin @info(name='query1') "
           "from e1=Stream1[price>20] -> e2=Stream2[price>e1.price] "
           "select e1.symbol as symbol1, e2.symbol as symbol2 insert into OutputStream; end;"),
    "PPe": ("define stream Stream1 (symbol string, price float, volume int); "
            "define stream Stream2 (symbol string, price float, volume int); "
            "partition with (volume of Stream1, volume of Stream2) begin @info(name='query1') "
            "from every e1=Stream1[price>20] -> e2=Stream2[price>e1.price] within 1 sec "
            "select e1.symbol as symbol1, e2.symbol as symbol2, e1.price as p1, e2.price as p2 "
            "insert into OutputStream; end;"),
}
QUERIES["C5"] = QUERIES["C2"]


def _base(cfg: str) -> str:
    return "C2" if cfg in ("C3b", "C3c") else ("PP" if cfg.startswith("PP") else cfg[:2])


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        return z ^ (z >> np.uint64(31))


def xcol(seed: int, col: int, idx: np.ndarray) -> np.ndarray:
    base = np.uint64((seed ^ (col << 56)) & 0xFFFFFFFFFFFFFFFF)
    return splitmix64_np(np.bitwise_xor(idx.astype(np.uint64), base))


def generate(cfg: str, start: int, count: int, keys: int = None, rate: int = None):
    """Rows [start, start+count) of config `cfg` as numpy columns (dict)."""
    num, n_total, k_default, r_default = CONFIGS[_base(cfg)]
    if cfg.startswith("C3"):
        num = 3
    seed = 0x5EED0000 + num
    K = keys if keys is not None else k_default
    R = rate if rate is not None else r_default
    i = np.arange(start, start + count, dtype=np.int64)
    out = {"ts": (T0 + i // R).astype(np.int64)}
    if cfg.startswith("PP"):   # two streams; symbol, price, volume (= the partition key)
        out["stream"] = (xcol(seed, 6, i) & np.uint64(1)).astype(np.int32)
        out["key"] = (xcol(seed, 2, i) % np.uint64(K)).astype(np.int32)
        out["price"] = ((xcol(seed, 1, i) % np.uint64(4001)).astype(np.float32) / np.float32(100.0)).astype(np.float32)
        return out
    if cfg.startswith("C4"):
        out["id"] = (xcol(seed, 4, i) % np.uint64(K)).astype(np.int64)
        out["seq"] = i.copy()
        return out
    out["key"] = (xcol(seed, 2, i) % np.uint64(K)).astype(np.int32)
    out["id"] = i.copy()
    if cfg.startswith("C3"):
        out["v"] = (xcol(seed, 3, i) % np.uint64(1000)).astype(np.int32)
        out["w"] = (xcol(seed, 5, i) % np.uint64(1000)).astype(np.int32)
    else:
        out["price"] = ((xcol(seed, 1, i) % np.uint64(4001)).astype(np.float32) / np.float32(100.0)).astype(np.float32)
    return out


def generate_torch(cfg: str, start: int, count: int, device, keys: int = None, rate: int = None):
    """Same columns generated directly in HBM with torch int64 arithmetic (wrapping multiply,
    logical shifts emulated by masking) -- used by bench.py so 1e8+ rows never cross PCIe."""
    import torch
    num, n_total, k_default, r_default = CONFIGS[_base(cfg)]
    if cfg.startswith("C3"):
        num = 3
    seed = 0x5EED0000 + num
    K = keys if keys is not None else k_default
    R = rate if rate is not None else r_default

    def s64(u):  # uint64 literal -> int64 bit pattern
        return u - (1 << 64) if u >= (1 << 63) else u

    def lsr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    def mix(z):
        z = z + s64(GOLDEN)
        z = (z ^ lsr(z, 30)) * s64(M1)
        z = (z ^ lsr(z, 27)) * s64(M2)
        return z ^ lsr(z, 31)

    def umod(z, m):
        # unsigned 64-bit modulo of an int64 bit pattern by m < 2^31
        hi = lsr(z, 32)
        lo = z & 0xFFFFFFFF
        r = (hi % m) * ((1 << 32) % m) % m
        return (r + lo % m) % m

    i = torch.arange(start, start + count, dtype=torch.int64, device=device)
    out = {"ts": T0 + torch.div(i, R, rounding_mode="floor")}

    def x(col):
        return mix(i ^ s64((seed ^ (col << 56)) & 0xFFFFFFFFFFFFFFFF))

    if cfg.startswith("C4"):
        out["id"] = umod(x(4), K)
        out["seq"] = i.clone()
        return out
    if cfg.startswith("PP"):
        out["stream"] = (x(6) & 1).to(torch.int32)
        out["key"] = umod(x(2), K).to(torch.int32)
        out["price"] = umod(x(1), 4001).to(torch.float32) / 100.0
        return out
    out["key"] = umod(x(2), K).to(torch.int32)
    out["id"] = i.clone()
    if cfg.startswith("C3"):
        out["v"] = umod(x(3), 1000).to(torch.int32)
        out["w"] = umod(x(5), 1000).to(torch.int32)
    else:
        out["price"] = umod(x(1), 4001).to(torch.float32) / 100.0
    return out


SYMBOL_SALT = 0x5359_4D42_4F4C_0000


def raw_symbols(key: np.ndarray) -> np.ndarray:
    """The partition attribute as a host sees it before dictionary encoding: one 64-bit value per symbol
    ("S%07d" % key hashed), for the native router (sg_router_route) to map to first-seen dense ids."""
    return splitmix64_np(key.astype(np.uint64) ^ np.uint64(SYMBOL_SALT)).view(np.int64)


def raw_symbols_torch(key):
    """raw_symbols computed in HBM (int64 bit patterns; same values as the numpy version)."""
    import torch

    def s64(u):
        return u - (1 << 64) if u >= (1 << 63) else u

    def lsr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)
    z = key.to(torch.int64) ^ SYMBOL_SALT
    z = z + s64(GOLDEN)
    z = (z ^ lsr(z, 30)) * s64(M1)
    z = (z ^ lsr(z, 27)) * s64(M2)
    return z ^ lsr(z, 31)
