// Host partition router (part of libsiddhi_gpu.so; plain C++, no device code).
//
// Replaces the per-event key lookup of PartitionStreamReceiver.receive / PartitionRuntime.cloneIfNotExist
// (C/partition/PartitionStreamReceiver.java:80-275, C/partition/PartitionRuntime.java:255-308) for SoA
// batches: raw partition-key values are dictionary-encoded into dense ids in first-seen order -- the order the
// reference clones per-key runtimes and registers their schedulers in -- and every key is assigned to one shard
// (GPU) by mix64(dense id) mod n_shards, with a dense id of its own inside the shard (first-seen order there too),
// so each GPU's key space stays dense.
//
// One call routes a batch with T threads in two parallel passes and one serial merge:
//   1. each thread numbers the keys of its contiguous slice in first-arrival order (one hash lookup per row);
//   2. the slices' keys are merged into the dictionary slice by slice (so new ids follow first arrival);
//   3. each thread maps its slice-local ids to dictionary ids (array lookups).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/siddhi_gpu.h"

namespace {

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

}  // namespace

struct sg_router {
  int n_shards = 1, threads = 1;
  KeyMap dict;                         // raw -> dense id
  std::vector<int32_t> shard_of, local_of;
  std::vector<int32_t> shard_keys;     // keys per shard
  std::string err;
};

extern "C" {

int sg_router_open(int n_shards, int threads, sg_router** out) {
  if (!out || n_shards < 1 || threads < 0) return SG_EINVAL;
  sg_router* r = new (std::nothrow) sg_router();
  if (!r) return SG_EINVAL;
  r->n_shards = n_shards;
  r->threads = threads ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  r->dict.init(1 << 12);
  r->shard_keys.assign(n_shards, 0);
  *out = r;
  return SG_OK;
}

int sg_router_route(sg_router* r, int64_t n, const int64_t* raw, int32_t* dense, int32_t* shard, int32_t* local) {
  if (!r || n < 0 || (n && !raw)) return SG_EINVAL;
  if (n == 0) return SG_OK;
  std::vector<int32_t> tmp;
  if (!dense) {
    tmp.resize((size_t)n);
    dense = tmp.data();
  }
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(r->threads, n / 65536 + 1));
  std::vector<std::vector<int64_t>> keys_of(T);   // per slice: its distinct keys in first-arrival order
  std::vector<std::vector<int32_t>> remap(T);     // per slice: slice-local id -> dictionary id
  auto slice = [&](int t, int64_t& lo, int64_t& hi) {
    lo = n * t / T;
    hi = n * (t + 1) / T;
  };
  // 1. every slice numbers its own keys in first-arrival order (one hash lookup per row; slots of the next 16
  //    rows are prefetched) and writes those slice-local ids
  auto pass1 = [&](int t) {
    int64_t lo, hi;
    slice(t, lo, hi);
    KeyMap m;
    m.init(1 << 12);
    std::vector<int64_t>& ks = keys_of[t];
    constexpr int G = 16;
    for (int64_t i = lo; i < hi; ++i) {
      if (i + G < hi) m.prefetch(raw[i + G]);
      const int64_t k = raw[i];
      const int32_t nid = (int32_t)ks.size();
      const int32_t id = m.insert(k, nid);
      if (id < 0) {
        ks.push_back(k);
        dense[i] = nid;
      } else {
        dense[i] = id;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(pass1, t);
  pass1(0);
  for (auto& th : pool) th.join();
  pool.clear();
  // 2. serial merge, slice by slice: dictionary ids in first-seen order (new keys get the next id, shard
  //    mix64(id) mod n_shards and the next dense id of that shard)
  for (int t = 0; t < T; ++t) {
    remap[t].resize(keys_of[t].size());
    for (size_t j = 0; j < keys_of[t].size(); ++j) {
      const int64_t k = keys_of[t][j];
      const int32_t id = (int32_t)r->shard_of.size();
      const int32_t old = r->dict.insert(k, id);
      if (old >= 0) {
        remap[t][j] = old;
        continue;
      }
      remap[t][j] = id;
      const int32_t s = (int32_t)(mix64((uint64_t)id) % (uint64_t)r->n_shards);
      r->shard_of.push_back(s);
      r->local_of.push_back(r->shard_keys[s]++);
    }
  }
  // 3. slice-local ids -> dictionary ids (and shard / per-shard ids): array lookups only
  auto pass3 = [&](int t) {
    int64_t lo, hi;
    slice(t, lo, hi);
    const int32_t* rm = remap[t].data();
    const int32_t* so = r->shard_of.data();
    const int32_t* lc = r->local_of.data();
    for (int64_t i = lo; i < hi; ++i) {
      const int32_t id = rm[dense[i]];
      dense[i] = id;
      if (shard) shard[i] = so[id];
      if (local) local[i] = lc[id];
    }
  };
  for (int t = 1; t < T; ++t) pool.emplace_back(pass3, t);
  pass3(0);
  for (auto& th : pool) th.join();
  return SG_OK;
}

int sg_router_keys(const sg_router* r, int64_t* n_keys, int32_t shard, int64_t* shard_keys) {
  if (!r || shard >= r->n_shards) return SG_EINVAL;
  if (n_keys) *n_keys = (int64_t)r->shard_of.size();
  if (shard_keys && shard >= 0) *shard_keys = r->shard_keys[shard];
  return SG_OK;
}

int sg_router_close(sg_router* r) {
  delete r;
  return SG_OK;
}

}  // extern "C"
