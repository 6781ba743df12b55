// Host partition router and match-stream merge (part of libsiddhi_gpu.so; plain C++, no device code).
//
// Router: replaces the per-event key lookup of PartitionStreamReceiver.receive / PartitionRuntime.cloneIfNotExist
// (C/partition/PartitionStreamReceiver.java:80-275, C/partition/PartitionRuntime.java:255-308) for SoA batches:
// raw partition-key values are dictionary-encoded into dense ids in first-seen order -- the order the reference
// clones per-key runtimes and registers their schedulers in -- and every key is assigned to one shard (GPU) by
// mix64(dense id) mod n_shards, with a dense id of its own inside the shard (first-seen order there too), so each
// GPU's key space stays dense.
//
// One call routes a batch with T threads:
//   1. each thread looks its contiguous slice up in the dictionary (read-only, shared); keys it does not hold get
//      slice-local numbers in first-arrival order -- once a stream's keys have been seen this is the only pass;
//   2. the slices' new keys are merged into the dictionary slice by slice (so new ids follow first arrival);
//   3. rows of new keys get their dictionary ids; shard / per-shard ids are array lookups.
//
// Merge: the per-GPU match streams (each in delivery order) merged into the node's delivery order by (trigger,
// phase, key) -- the order QueryCallback.receive sees on one host (C/query/output/callback/QueryCallback.java:52-85).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/siddhi_gpu.h"
#include "router.h"

namespace {

template <class F>
void run_threads(int T, F&& f) {
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(f, t);
  f(0);
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int sg_router_open(int n_shards, int threads, sg_router** out) {
  if (!out || n_shards < 1 || threads < 0) return SG_EINVAL;
  sg_router* r = new (std::nothrow) sg_router();
  if (!r) return SG_EINVAL;
  r->n_shards = n_shards;
  r->threads = threads ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  r->dict.init(1 << 12);
  r->shard_keys.assign(n_shards, 0);
  r->l2d = std::vector<sgr::BlockVec>(n_shards);
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
  std::vector<sgr::SliceMiss> miss(T);
  auto slice = [&](int t, int64_t& lo, int64_t& hi) {
    lo = n * t / T;
    hi = n * (t + 1) / T;
  };
  // shard / per-shard ids of resolved rows (one pass when every key is known)
  auto finish = [&](int64_t lo, int64_t hi, bool only_new) {
    const int32_t* so = r->shard_of.data();
    const int32_t* lc = r->local_of.data();
    for (int64_t i = lo; i < hi; ++i) {
      const int32_t id = dense[i];
      if (only_new && id >= 0) continue;
      if (id < 0) continue;
      if (shard) shard[i] = so[id];
      if (local) local[i] = lc[id];
    }
  };
  // 1. dictionary lookups (read-only)
  run_threads(T, [&](int t) {
    int64_t lo, hi;
    slice(t, lo, hi);
    sgr::lookup_slice(r->dict, raw + lo, hi - lo, dense + lo, miss[t]);
    finish(lo, hi, false);
  });
  // 2. serial merge of new keys, slice by slice (first-seen order)
  std::vector<std::vector<int32_t>> remap(T);
  bool any = false;
  for (int t = 0; t < T; ++t) {
    if (!miss[t].any) continue;
    any = true;
    remap[t].resize(miss[t].fresh.size());
    for (size_t j = 0; j < miss[t].fresh.size(); ++j) remap[t][j] = r->add_key(miss[t].fresh[j]);
  }
  if (!any) return SG_OK;
  // 3. rows of new keys
  run_threads(T, [&](int t) {
    if (!miss[t].any) return;
    int64_t lo, hi;
    slice(t, lo, hi);
    const int32_t* rm = remap[t].data();
    const int32_t* so = r->shard_of.data();
    const int32_t* lc = r->local_of.data();
    for (int64_t i = lo; i < hi; ++i) {
      const int32_t x = dense[i];
      if (x >= 0) continue;
      const int32_t id = rm[-x - 2];
      dense[i] = id;
      if (shard) shard[i] = so[id];
      if (local) local[i] = lc[id];
    }
  });
  return SG_OK;
}

int sg_router_keys(const sg_router* r, int64_t* n_keys, int32_t shard, int64_t* shard_keys) {
  if (!r || shard >= r->n_shards) return SG_EINVAL;
  if (n_keys) *n_keys = (int64_t)r->shard_of.size();
  if (shard_keys && shard >= 0) *shard_keys = r->shard_keys[shard];
  return SG_OK;
}

int sg_router_dense_ids(const sg_router* r, int32_t shard, int32_t* dense_of_local, int64_t cap) {
  if (!r || shard < 0 || shard >= r->n_shards || cap < 0) return SG_EINVAL;
  const sgr::BlockVec& v = r->l2d[shard];
  if (cap < (int64_t)v.size()) return SG_ECAPACITY;
  for (size_t i = 0; i < v.size(); ++i) dense_of_local[i] = v[i];
  return SG_OK;
}

int sg_router_close(sg_router* r) {
  delete r;
  return SG_OK;
}

// K-way merge of match runs (each already in delivery order) into the node's delivery order: by trigger, then
// phase (group >> 24: a clock pass's timer emissions before the event's own states), then dense key (timer passes
// fire key by key in registration = first-seen order, C/util/timestamp/TimestampGeneratorImpl.java:106-125);
// ties keep run order.  out_src[i] = index of the i-th merged row in the concatenation of the runs.  Parallel
// over trigger ranges: every thread takes the rows whose trigger lies in its range from every run (boundaries by
// binary search; equal triggers never straddle two threads).
int sg_merge_order(int n_runs, const int64_t* run_len, const uint64_t* const* trigger, const uint32_t* const* group,
                   const int32_t* const* key, int threads, int64_t* out_src) {
  if (n_runs < 0 || (n_runs && (!run_len || !trigger)) || !out_src) return SG_EINVAL;
  std::vector<int64_t> base(n_runs + 1, 0);
  for (int r = 0; r < n_runs; ++r) {
    if (run_len[r] < 0 || (run_len[r] && !trigger[r])) return SG_EINVAL;
    base[r + 1] = base[r] + run_len[r];
  }
  const int64_t total = base[n_runs];
  if (total == 0) return SG_OK;
  for (int r = 0; r < n_runs; ++r)   // every run must be ordered by trigger
    for (int64_t i = 1; i < run_len[r]; ++i)
      if (trigger[r][i] < trigger[r][i - 1]) return SG_EORDER;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : 1, total / 262144 + 1));
  // splitters: triggers of the longest run at equal positions
  int big = 0;
  for (int r = 1; r < n_runs; ++r) if (run_len[r] > run_len[big]) big = r;
  std::vector<uint64_t> split(T + 1);
  split[0] = 0;
  for (int t = 1; t < T; ++t) split[t] = trigger[big][run_len[big] * t / T];
  std::vector<std::vector<int64_t>> lo(T + 1, std::vector<int64_t>(n_runs));
  for (int t = 0; t <= T; ++t)
    for (int r = 0; r < n_runs; ++r) {
      if (t == 0) { lo[t][r] = 0; continue; }
      if (t == T) { lo[t][r] = run_len[r]; continue; }
      lo[t][r] = std::lower_bound(trigger[r], trigger[r] + run_len[r], split[t]) - trigger[r];
    }
  std::vector<int64_t> out0(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    int64_t c = 0;
    for (int r = 0; r < n_runs; ++r) c += std::max<int64_t>(0, lo[t + 1][r] - lo[t][r]);
    out0[t + 1] = out0[t] + c;
  }
  auto less = [&](int ra, int64_t ia, int rb, int64_t ib) {
    const uint64_t ta = trigger[ra][ia], tb = trigger[rb][ib];
    if (ta != tb) return ta < tb;
    const uint32_t pa = group && group[ra] ? group[ra][ia] >> 24 : 0, pb = group && group[rb] ? group[rb][ib] >> 24 : 0;
    if (pa != pb) return pa < pb;
    const int32_t ka = key && key[ra] ? key[ra][ia] : 0, kb = key && key[rb] ? key[rb][ib] : 0;
    if (ka != kb) return ka < kb;
    return ra < rb;
  };
  run_threads(T, [&](int t) {
    std::vector<int64_t> cur(lo[t]), end(lo[t + 1]);
    int64_t o = out0[t];
    while (true) {
      int best = -1;
      for (int r = 0; r < n_runs; ++r)
        if (cur[r] < end[r] && (best < 0 || less(r, cur[r], best, cur[best]))) best = r;
      if (best < 0) break;
      // the whole stretch of `best` that stays ahead of every other run's head goes out in one go
      int64_t i = cur[best];
      do {
        out_src[o++] = base[best] + i;
        ++i;
        bool ahead = i < end[best];
        for (int r = 0; ahead && r < n_runs; ++r)
          if (r != best && cur[r] < end[r] && !less(best, i, r, cur[r])) ahead = false;
        if (!ahead) break;
      } while (true);
      cur[best] = i;
    }
  });
  return SG_OK;
}

}  // extern "C"
