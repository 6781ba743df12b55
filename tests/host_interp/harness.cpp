// TEST HARNESS ONLY: runs the engine's per-key NFA machine (siddhi_amd/csrc/interp.h, the exact code the
// MI355X kernel executes) on the CPU so its logic can be compared with the oracle without a GPU.
// Not linked into libsiddhi_gpu.so and not reachable from the product path.
#define SG_HOST_ONLY 1
#define SG_HD
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../siddhi_amd/csrc/sg_device.h"
#include "../../siddhi_amd/csrc/interp.h"

struct HiHandle {
  sg_nfa_desc d;
  SgGeo g;
  std::vector<std::vector<int32_t>> arenas;
  std::vector<std::vector<char>> out;
  int err = 0;
  int chunk_rows = 0;   // >0: cut each key's rows into units replaying their horizon (as interp.hip does)
};

struct HostRows {
  const sg_batch* b;
  const sg_nfa_desc* d;
  const std::vector<int64_t>* own;
  uint64_t index_of(int64_t r) { return b->index ? b->index[r] : b->base_index + (uint64_t)r; }
  int64_t first_after(int64_t pos) {
    if (!b->index) { int64_t p = pos - (int64_t)b->base_index + 1; return p < 0 ? 0 : (p > b->n ? b->n : p); }
    return std::upper_bound(b->index, b->index + b->n, (uint64_t)pos, [](uint64_t v, uint64_t x) { return v < x; }) - b->index;
  }
  int64_t n_own() { return (int64_t)own->size(); }
  int64_t own_local(int64_t i) { return (*own)[i]; }
  int64_t n_rows() { return b->n; }
  int64_t ts(int64_t r) { return b->ts[r]; }
  int64_t find_ge(int64_t from, int64_t v) {
    const int64_t* lo = b->ts + from;
    const int64_t* hi = b->ts + b->n;
    return std::lower_bound(lo, hi, v) - b->ts;
  }
  void fill(int64_t r, SgRow& row) {
    row.ts = b->ts[r];
    row.index = index_of(r);
    row.stream = b->stream ? b->stream[r] : 0;
    row.nullmask = 0;
    for (int k = 0; k < d->n_ret; ++k) {
      int c = d->ret_col[k];
      int t = d->ret_type[k];
      if (b->nulls && b->nulls[c] && b->nulls[c][r]) { row.nullmask |= 1 << k; row.vals[k] = 0; continue; }
      const void* col = b->cols[c];
      int64_t bits;
      switch (t) {
        case SG_T_LONG: bits = ((const int64_t*)col)[r]; break;
        case SG_T_DOUBLE: memcpy(&bits, (const double*)col + r, 8); break;
        case SG_T_FLOAT: { uint32_t u; memcpy(&u, (const float*)col + r, 4); bits = u; break; }
        default: bits = ((const int32_t*)col)[r]; break;
      }
      row.vals[k] = bits;
    }
  }
};

extern "C" {

HiHandle* hi_open(const sg_nfa_desc* d, int P, int E, int C, int L) {
  HiHandle* h = new HiHandle();
  h->d = *d;
  h->g = sg_make_geo(*d, P, E, C, L, L);
  return h;
}

void hi_close(HiHandle* h) { delete h; }

void hi_set_chunk(HiHandle* h, int chunk_rows) { h->chunk_rows = chunk_rows; }

int hi_chunk_rule(const sg_nfa_desc* d, int64_t* horizon) {
  SgChunkRule r = sg_chunk_rule(*d);
  *horizon = r.kind == 2 ? r.events : r.within;
  return r.kind;
}

int hi_push(HiHandle* h, const sg_batch* b) {
  const sg_nfa_desc& d = h->d;
  int64_t n = b->n;
  int32_t kmax = -1;
  for (int64_t i = 0; i < n; ++i) if (b->key && b->key[i] > kmax) kmax = b->key[i];
  if (!d.partitioned) kmax = 0;
  if ((int64_t)h->arenas.size() < kmax + 1) h->arenas.resize(kmax + 1);
  std::vector<std::vector<int64_t>> own(h->arenas.size());
  for (int64_t i = 0; i < n; ++i) {
    int s = b->stream ? b->stream[i] : 0;
    if (s < 0 || d.recv_of_stream[s] < 0) continue;
    int k = d.partitioned ? b->key[i] : 0;
    if (k < 0) continue;
    own[k].push_back(i);
  }
  unsigned long long count = 0;
  int32_t overflow = 0;
  int stride = sg_emit_stride(d.n_select);
  size_t cap = 4 * (size_t)n + 4096;
  std::vector<char> buf(cap * stride);
  int kb = 1;
  while ((1ull << kb) <= (uint64_t)h->arenas.size()) ++kb;
  for (size_t k = 0; k < h->arenas.size(); ++k) {
    if (h->arenas[k].empty()) {
      if (own[k].empty() && d.partitioned) continue;
      h->arenas[k].assign((size_t)h->g.key_words, 0);
    }
    auto run = [&](int32_t* arena, const std::vector<int64_t>* rws, int64_t emit_from) {
      KeyMachine m;
      memset(&m, 0, sizeof(m));
      m.d = &d;
      m.g = &h->g;
      m.a = arena;
      m.key = (int32_t)k;
      m.clone = d.partitioned;
      m.sink = SgEmitSink{buf.data(), (int64_t)cap, &count, &overflow, stride, kb};
      m.base_index = b->base_index;
      HostRows rows{b, &d, rws};
      sg_run_key(m, rows, !d.partitioned, emit_from);
      return m.failed;
    };
    const SgChunkRule rule = sg_chunk_rule(d);
    const int64_t nown = (int64_t)own[k].size();
    const int64_t R = h->chunk_rows;
    if (R <= 0 || rule.kind == 0 || nown <= R) {
      if (int f = run(h->arenas[k].data(), &own[k], 0)) { h->err = f; return f; }
      continue;
    }
    // chunked units: unit 0 continues the key's state; unit c > 0 replays its horizon from a fresh runtime
    // (or from the state at the push start when the horizon reaches the key's first row of this push)
    const std::vector<int32_t> snap = h->arenas[k];
    std::vector<int32_t> last;
    for (int64_t p0 = 0; p0 < nown; p0 += R) {
      const int64_t p1 = std::min(nown, p0 + R);
      if (p0 == 0) {
        std::vector<int64_t> sub(own[k].begin(), own[k].begin() + p1);
        if (int f = run(h->arenas[k].data(), &sub, 0)) { h->err = f; return f; }
        continue;
      }
      const int64_t q = sg_replay_start(rule, p0, [&](int64_t i) { return b->ts[own[k][i]]; });
      std::vector<int32_t> arena = q == 0 ? snap : std::vector<int32_t>((size_t)h->g.key_words, 0);
      std::vector<int64_t> sub(own[k].begin() + q, own[k].begin() + p1);
      if (int f = run(arena.data(), &sub, p0 - q)) { h->err = f; return f; }
      if (p1 == nown) last.swap(arena);
    }
    h->arenas[k].swap(last);
  }
  if (overflow) { h->err = SG_ECAPACITY; return SG_ECAPACITY; }
  std::vector<size_t> idx(count);
  for (size_t i = 0; i < count; ++i) idx[i] = i;
  auto sk = [&](size_t i) { uint64_t v; memcpy(&v, buf.data() + i * stride, 8); return v; };
  std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return sk(x) < sk(y); });
  for (size_t i : idx) h->out.emplace_back(buf.begin() + i * stride + 8, buf.begin() + (i + 1) * stride);
  return 0;
}

int64_t hi_count(HiHandle* h) { return (int64_t)h->out.size(); }

void hi_fetch(HiHandle* h, uint64_t* trig, int64_t* ts, int32_t* key, uint32_t* group, int64_t* vals, uint32_t* vnull) {
  int ns = h->d.n_select;
  for (size_t i = 0; i < h->out.size(); ++i) {
    const char* r = h->out[i].data();
    memcpy(trig + i, r, 8); memcpy(ts + i, r + 8, 8); memcpy(key + i, r + 16, 4); memcpy(group + i, r + 20, 4);
    memcpy(vnull + i, r + 24, 4);
    if (ns) memcpy(vals + i * ns, r + 32, 8 * (size_t)ns);
  }
  h->out.clear();
}

}
