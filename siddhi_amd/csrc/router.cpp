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
//   1. each thread scans its contiguous slice and collects, in order, the keys the global dictionary lacks;
//   2. the slices' new keys are appended to the dictionary slice by slice (so the ids follow first arrival);
//   3. each thread maps its slice through the (now read-only) dictionary.
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

// open-addressing map int64 raw key -> int32 value (linear probing, power-of-two capacity)
struct KeyMap {
  std::vector<int64_t> keys;
  std::vector<int32_t> vals;   // -1 = empty
  size_t mask = 0, size = 0;
  void init(size_t cap_pow2) {
    keys.assign(cap_pow2, 0);
    vals.assign(cap_pow2, -1);
    mask = cap_pow2 - 1;
    size = 0;
  }
  int32_t find(int64_t k) const {
    size_t i = (size_t)mix64((uint64_t)k) & mask;
    while (true) {
      const int32_t v = vals[i];
      if (v < 0) return -1;
      if (keys[i] == k) return v;
      i = (i + 1) & mask;
    }
  }
  // returns the existing value, or inserts v and returns -1
  int32_t insert(int64_t k, int32_t v) {
    if ((size + 1) * 2 > keys.size()) grow();
    size_t i = (size_t)mix64((uint64_t)k) & mask;
    while (true) {
      if (vals[i] < 0) {
        keys[i] = k;
        vals[i] = v;
        ++size;
        return -1;
      }
      if (keys[i] == k) return vals[i];
      i = (i + 1) & mask;
    }
  }
  void grow() {
    std::vector<int64_t> ok;
    std::vector<int32_t> ov;
    ok.swap(keys);
    ov.swap(vals);
    init(std::max<size_t>(ok.size() * 2, 1024));
    for (size_t i = 0; i < ok.size(); ++i)
      if (ov[i] >= 0) insert(ok[i], ov[i]);
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
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(r->threads, n / 65536 + 1));
  std::vector<std::vector<int64_t>> fresh(T);
  auto slice = [&](int t, int64_t& lo, int64_t& hi) {
    lo = n * t / T;
    hi = n * (t + 1) / T;
  };
  // 1. new keys per slice, in first-arrival order (a thread-local set filters repeats inside the slice)
  auto pass1 = [&](int t) {
    int64_t lo, hi;
    slice(t, lo, hi);
    KeyMap seen;
    seen.init(1 << 10);
    std::vector<int64_t>& f = fresh[t];
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t k = raw[i];
      if (r->dict.find(k) >= 0) continue;
      if (seen.insert(k, 0) < 0) f.push_back(k);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(pass1, t);
  pass1(0);
  for (auto& th : pool) th.join();
  pool.clear();
  // 2. serial merge: dictionary ids in first-seen order, shard by mix64(id), dense id inside the shard
  for (int t = 0; t < T; ++t)
    for (int64_t k : fresh[t]) {
      const int32_t id = (int32_t)r->shard_of.size();
      if (r->dict.insert(k, id) >= 0) continue;   // first seen by an earlier slice
      const int32_t s = (int32_t)(mix64((uint64_t)id) % (uint64_t)r->n_shards);
      r->shard_of.push_back(s);
      r->local_of.push_back(r->shard_keys[s]++);
    }
  // 3. map every row
  auto pass3 = [&](int t) {
    int64_t lo, hi;
    slice(t, lo, hi);
    for (int64_t i = lo; i < hi; ++i) {
      const int32_t id = r->dict.find(raw[i]);
      if (dense) dense[i] = id;
      if (shard) shard[i] = r->shard_of[id];
      if (local) local[i] = r->local_of[id];
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
