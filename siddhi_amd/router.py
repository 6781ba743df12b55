"""Multi-GPU routing for partitioned queries.

Keys are fully isolated (one cloned runtime per key, C/partition/PartitionRuntime.java:261-308), so the
node shards by key with no data-path collective: key k belongs to rank mix64(k) % G.  Each rank runs its
own engine on its rows (global event indices preserved) and the per-rank match streams are merged by
(trigger index, timer-before-event, key) — the reference's delivery order, since timer emissions of one
clock advance follow key registration (first-seen) order and an event's own matches come from its key.
"""
from __future__ import annotations

import numpy as np

M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def mix64(k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = k.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def shard_of(keys: np.ndarray, world: int) -> np.ndarray:
    """Owning rank of each dense key id (rows with key < 0 go to rank 0, which drops them)."""
    r = (mix64(np.maximum(keys, 0)) % np.uint64(world)).astype(np.int32)
    return r


def shard_batch(batch, rank: int, world: int):
    """Rows of `batch` owned by `rank` (arrival order and global indices kept)."""
    from .runtime import Batch
    own = shard_of(batch.key, world) == rank
    idx = np.nonzero(own)[0]
    # rows keep their global index: engines see a sparse batch through an explicit index column
    gidx = (batch.index[idx] if batch.index is not None else batch.base_index + idx).astype(np.uint64)
    return idx, Batch(len(idx), int(gidx[0]) if len(idx) else batch.base_index, batch.ts[idx], batch.stream[idx],
                      batch.key[idx], [c[idx] for c in batch.cols], [None if x is None else x[idx] for x in batch.nulls],
                      gidx)


class RankShard:
    """One rank's view of the key-sharded stream.  Its keys are re-densified to local ids 0..K_r-1 in
    first-seen order (so a GPU sees a dense key space of its own size, not the node's), persistently across
    pushes so carried per-key state keeps its id; `globalize` maps match keys back before `merge`."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.g2l = np.full(0, -1, np.int32)
        self.l2g = np.zeros(0, np.int32)

    def shard(self, batch):
        idx, mine = shard_batch(batch, self.rank, self.world)
        k = mine.key
        valid = k >= 0
        if valid.any():
            top = int(k[valid].max()) + 1
            if top > len(self.g2l):
                self.g2l = np.concatenate([self.g2l, np.full(top - len(self.g2l), -1, np.int32)])
            uk, first = np.unique(k[valid], return_index=True)
            new = uk[self.g2l[uk] < 0]
            if len(new):
                order = np.argsort(first[self.g2l[uk] < 0], kind="stable")   # first-seen order
                new = new[order]
                self.g2l[new] = np.arange(len(self.l2g), len(self.l2g) + len(new), dtype=np.int32)
                self.l2g = np.concatenate([self.l2g, new.astype(np.int32)])
        local = np.where(valid, self.g2l[np.maximum(k, 0)] if len(self.g2l) else -1, -1).astype(np.int32)
        mine.key = local
        return idx, mine

    @property
    def key_bound(self) -> int:
        return len(self.l2g)

    def globalize(self, out):
        out.key = np.where(out.key >= 0, self.l2g[np.maximum(out.key, 0)] if len(self.l2g) else out.key,
                           out.key).astype(out.key.dtype)
        return out


def merge(parts, threads: int = 16):
    """Merge per-rank Outputs (each already in delivery order) into the node's delivery order: the native k-way
    merge sg_merge_order (csrc/router.cpp) by (trigger, phase, dense key), ties in rank order."""
    from ._native import merge_order
    from .runtime import Outputs
    if not parts:
        raise ValueError("nothing to merge")
    order = merge_order([p.trigger for p in parts], [p.group for p in parts], [p.key for p in parts], threads)
    cat = Outputs(*[np.concatenate([getattr(p, f) for p in parts]) for f in
                    ("trigger", "ts", "key", "group", "vals", "vnull")])
    return Outputs(*[getattr(cat, f)[order] for f in ("trigger", "ts", "key", "group", "vals", "vnull")])


# ---- on-device sharding (bench.py's C5 stream mode): the same mix64 assignment computed in HBM with torch int64
# arithmetic (wrapping multiply, logical shifts by masking), so a 1B-event stream is split without crossing PCIe.
def _lsr(z, k):
    return (z >> k) & ((1 << (64 - k)) - 1)


def _s64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def mix64_torch(k):
    z = k.to(dtype=__import__("torch").int64) + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _lsr(z, 31)


def shard_of_torch(keys, world: int):
    """shard_of on a torch tensor of dense key ids (unsigned 64-bit modulo of the int64 bit pattern)."""
    import torch
    z = mix64_torch(torch.clamp(keys.to(torch.int64), min=0))
    hi, lo = _lsr(z, 32), z & 0xFFFFFFFF
    return (((hi % world) * ((1 << 32) % world) + lo % world) % world).to(torch.int32)


def shard_tables_torch(n_keys: int, world: int, device):
    """Per key id 0..n_keys-1: owning rank and its dense id inside that rank (ascending key order), plus the number
    of keys each rank owns."""
    import torch
    k = torch.arange(n_keys, device=device)
    s = shard_of_torch(k, world)
    local = torch.empty(n_keys, dtype=torch.int32, device=device)
    counts = []
    for r in range(world):
        m = s == r
        c = int(m.sum().item())
        local[m] = torch.arange(c, dtype=torch.int32, device=device)
        counts.append(c)
    return s, local, counts


def shard_stream_torch(cfg: str, rank: int, world: int, total: int, keys: int, rate: int, device, gen=100_000_000):
    """This rank's rows of the synthetic stream `cfg` (siddhi_amd/synth.py, generated in HBM chunk by chunk): the rows
    whose key mix64-hashes to `rank`, with per-rank dense key ids (ascending key order), their global event indices,
    and the local -> global key table.  Returns (columns dict: ts, key, id, price, gidx), key_bound, l2g."""
    import torch
    from . import synth
    shard, local, counts = shard_tables_torch(keys, world, device)
    parts = {"ts": [], "key": [], "id": [], "price": [], "gidx": []}
    for start in range(0, total, gen):
        g = synth.generate_torch(cfg, start, min(gen, total - start), device, keys=keys, rate=rate)
        gk = g["key"].long()
        sel = torch.nonzero(shard[gk] == rank).squeeze(1)
        parts["ts"].append(g["ts"][sel])
        parts["key"].append(local[gk[sel]])
        parts["id"].append(g["id"][sel])
        parts["price"].append(g["price"][sel])
        parts["gidx"].append(sel + start)
        del g, gk, sel
    cols = {k: torch.cat(v) for k, v in parts.items()}
    l2g = torch.nonzero(shard == rank).squeeze(1).to(torch.int32)   # ascending key order = local id order
    return cols, counts[rank], l2g
