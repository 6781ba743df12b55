// Host partition router internals (plain C++, shared by router.cpp and the node pipeline in node.hip).
//
// Replaces the per-event key lookup of PartitionStreamReceiver.receive / PartitionRuntime.cloneIfNotExist
// (C/partition/PartitionStreamReceiver.java:80-275, C/partition/PartitionRuntime.java:255-308): raw partition-key
// values get dense ids in first-seen order (the reference's clone order), each key is owned by shard
// mix64(dense id) mod n_shards (one shard per GPU) and has a dense id of its own inside that shard.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

namespace sgr {

inline uint64_t mix64(uint64_t x) {   // splitmix64 step (same as siddhi_amd/router.py mix64)
  x += 0x9E3779B97F4A7C15ull;
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// open-addressing map int64 raw key -> int32 value (linear probing, power-of-two capacity, key and value in one
// 16-byte slot so a probe touches one cache line)
struct KeyMap {
  struct Slot {
    int64_t key;
    int32_t val;   // -1 = empty
    int32_t pad;
  };
  std::vector<Slot> slots;
  size_t mask = 0, size = 0;
  int shift = 64;
  void init(size_t cap_pow2) {
    slots.assign(cap_pow2, Slot{0, -1, 0});
    mask = cap_pow2 - 1;
    size = 0;
    shift = 64;
    for (size_t c = cap_pow2; c > 1; c >>= 1) --shift;
  }
  // Fibonacci hashing: one multiply, the top bits index the table
  size_t home(int64_t k) const { return (size_t)(((uint64_t)k * 0x9E3779B97F4A7C15ull) >> shift) & mask; }
  void prefetch(int64_t k) const { __builtin_prefetch(&slots[home(k)]); }
  int32_t find(int64_t k) const {
    size_t i = home(k);
    while (true) {
      const Slot& s = slots[i];
      if (s.val < 0) return -1;
      if (s.key == k) return s.val;
      i = (i + 1) & mask;
    }
  }
  // returns the existing value, or inserts v and returns -1
  int32_t insert(int64_t k, int32_t v) {
    if ((size + 1) * 2 > slots.size()) grow();
    size_t i = home(k);
    while (true) {
      Slot& s = slots[i];
      if (s.val < 0) {
        s.key = k;
        s.val = v;
        ++size;
        return -1;
      }
      if (s.key == k) return s.val;
      i = (i + 1) & mask;
    }
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(slots);
    init(std::max<size_t>(old.size() * 2, 1024));
    for (const Slot& s : old)
      if (s.val >= 0) insert(s.key, s.val);
  }
};

// Key lookup of one row slice.  Keys already in the dictionary resolve with one read-only probe (the common case
// once a stream's keys have all been seen); a new key gets a slice-local number encoded as -(number + 2) and is
// listed in `fresh` in first-arrival order, to be merged into the dictionary serially.
struct SliceMiss {
  std::vector<int64_t> fresh;
  KeyMap local;
  bool any = false;
};
// out[i] = dictionary id of raw[i], or -(slice-local number + 2) for a key the dictionary does not hold yet
inline void lookup_slice(const KeyMap& dict, const int64_t* raw, int64_t n, int32_t* out, SliceMiss& ms) {
  constexpr int G = 16;   // probes of the next 16 rows in flight
  for (int64_t i = 0; i < n; ++i) {
    if (i + G < n) dict.prefetch(raw[i + G]);
    const int64_t k = raw[i];
    int32_t id = dict.find(k);
    if (id < 0) {
      if (!ms.any) { ms.local.init(1 << 10); ms.any = true; }
      const int32_t nid = (int32_t)ms.fresh.size();
      const int32_t old = ms.local.insert(k, nid);
      if (old < 0) { ms.fresh.push_back(k); id = -(nid + 2); }
      else id = -(old + 2);
    }
    out[i] = id;
  }
}

// Append-only int32 array whose elements never move: a reader on another thread may index entries published to it
// earlier while the owner appends (the outer table is reserved for 2^31 entries up front, so it never reallocates).
struct BlockVec {
  static constexpr int B = 16;
  std::vector<std::unique_ptr<int32_t[]>> blocks;
  size_t n = 0;
  BlockVec() { blocks.reserve((size_t)1 << (31 - B)); }
  void push_back(int32_t v) {
    if ((n >> B) >= blocks.size()) blocks.emplace_back(new int32_t[(size_t)1 << B]);
    blocks[n >> B][n & (((size_t)1 << B) - 1)] = v;
    ++n;
  }
  int32_t operator[](size_t i) const { return blocks[i >> B][i & (((size_t)1 << B) - 1)]; }
  size_t size() const { return n; }
};

}  // namespace sgr

struct sg_router {
  int n_shards = 1, threads = 1;
  sgr::KeyMap dict;                     // raw -> dense id
  std::vector<int32_t> shard_of, local_of;
  std::vector<int32_t> shard_keys;      // keys per shard
  std::vector<sgr::BlockVec> l2d;      // per shard: local id -> dense id (readable while keys are added)
  std::string err;
  // a new key (first seen now): next dense id, its shard and per-shard id
  int32_t add_key(int64_t k) {
    const int32_t id = (int32_t)shard_of.size();
    const int32_t old = dict.insert(k, id);
    if (old >= 0) return old;
    const int32_t s = (int32_t)(sgr::mix64((uint64_t)id) % (uint64_t)n_shards);
    shard_of.push_back(s);
    local_of.push_back(shard_keys[s]++);
    l2d[s].push_back(id);
    return id;
  }
};
