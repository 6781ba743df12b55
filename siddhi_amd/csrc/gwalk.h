// gwalk.h -- the closed form's group walker: `every A[l] -> B[l' and B.x OP A.x] within T` when the partition has
// many keys with few rows each (C5: 1M keys, ~500 rows per key per 500M-row push, ~10 rows per `within` window).
// Included by engine_impl.h; run_group_walk is tried by run_every_next after the partition's group passes.
//
// Semantics are those of the tiled walker (engine_impl.h Walker::step, itself StreamPreStateProcessor.isExpired /
// processAndReturn, C/query/input/stream/state/StreamPreStateProcessor.java:102-113,292-337, and
// StreamPostStateProcessor.process, StreamPostStateProcessor.java:53-72): per key, e2's pending list in arrival order,
// an arriving row first drops the partials older than `within`, then completes every pending partial its compare
// accepts (delivered oldest first), then appends itself when it passes A's filter.
//
// What differs is where the work happens.  The tiled path sorts every group's rows by key into HBM (part_key),
// re-lays them out as lane-interleaved tiles (tile_transpose), walks them twice (walk_count, then walk_record with a
// random read of every emitting row's output offset) and projects.  Here one workgroup owns one group of 256 keys --
// lane t walks key 256g + t -- and streams the group's rows (pass 1b's output: the group's rows in arrival order,
// 16-byte walker records plus a 1-byte in-group key) through LDS in chunks: a stable counting sort of the chunk by
// in-group key in LDS, then every lane walks its own rows from LDS with its pending list in an LDS ring.  One walk,
// no key-sorted copy in HBM, no tiles.  Each trigger row writes one 8-byte word at its arrival position (where its
// matches start in the match area, and how many); the matches themselves go to the key's region of the match area
// in walk order: a 16-byte header per trigger (e2's time, key, compared value, payload) and 8 bytes per completed
// partial (e1's compared value, payload) -- written sequentially by the lane.  A scan over the trigger words in
// arrival order gives each trigger's first output slot, and the projection walks the triggers in arrival order,
// so the output records are written contiguously and in delivery order.
//
// The fast path declines (returns false, nothing changed) when a push needs what only the tiled path has: a key
// whose time goes back (the exact HBM-list walker), a pending list longer than the LDS ring, e1 attributes gathered
// by row, or a select reading anything but the compared values and the carried payload.
#pragma once

struct GwArgs {
  int64_t n, nc;              // batch rows; carried rows (virtual rows [0, nc))
  int64_t within;
  int64_t t0;                 // narrow records' time origin (the push's first virtual row)
  uint32_t K, ns1;            // keys; pass-1 segments per group (o1 stride)
  int32_t stack_mode;
  int32_t cap;                // LDS ring entries per lane (power of two)
  int32_t chunk;              // rows per LDS chunk (multiple of 256)
  int32_t carry_out;
  int32_t pzero;              // payload bits zero-extended (FLOAT) rather than sign-extended
  const uint32_t* o1;         // group g's rows: [o1[g * ns1], o1[(g + 1) * ns1])
  const PtU4* grec;           // pass 1b's records, grouped by group, arrival order within a group
  const uint8_t* glk;         // in-group key of each record
  const uint32_t* kbase;      // per key: its first row in the group domain (exclusive scan of per-key rows)
  uint64_t* trig;             // per batch row: match-area unit of its first header | matches << 32 (0: none)
  uint64_t* area;             // match area, 8-byte units: 3 per row of the key
  int64_t* cv_ts;             // carry: every key's final pending list as values
  int32_t* cv_key;
  int64_t* cv_val;
  int64_t* cv_pay;
  uint32_t* cv_n;
  uint32_t cv_cap;
  uint32_t* flags;            // GW_ORDER | GW_OVERFLOW | GW_INTERNAL | GW_CARRY_FULL
  uint32_t* ovf_keys;         // keys whose pending list outgrew the LDS ring (walked again by k_gw_redo)
  uint32_t* ovf_n;
  uint32_t ovf_cap;
  uint32_t* match_n;          // matches of the push (the projection's output size)
};
static const uint32_t GW_ORDER = 1, GW_OVERFLOW = 2, GW_INTERNAL = 4, GW_CARRY_FULL = 8;

// per-key rows of every group (LDS counters over the group's in-group keys)
static __global__ void __launch_bounds__(256) k_gw_count(const uint32_t* __restrict__ o1, uint32_t ns1, uint32_t K,
                                                         const uint8_t* __restrict__ glk, uint32_t* __restrict__ kcnt) {
  __shared__ uint32_t c[4][256];
  const uint32_t g = blockIdx.x, t = threadIdx.x, w = t >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q][t] = 0;
  __syncthreads();
  const uint32_t lo = o1[(size_t)g * ns1], hi = o1[(size_t)(g + 1) * ns1];
  for (uint32_t p = lo + t; p < hi; p += 256) atomicAdd(&c[w][glk[p]], 1u);
  __syncthreads();
  const uint32_t k = (g << 8) + t;
  if (k < K) kcnt[k] = c[0][t] + c[1][t] + c[2][t] + c[3][t];
}

template <int PT>
struct GwLds {
  PtU4 stage[256 * PT];
  uint32_t cw[4][256];
  uint32_t ls[256], tot[256];
  uint32_t wsum[4];
};

// Pending list of one key: an LDS ring of `cap` entries per lane (lane-strided planes: conflict-free), or -- for a key
// whose list outgrew the ring (k_gw_redo) -- unbounded HBM planes over the key's own rows.
template <class T>
struct GwLdsRing {
  T* v;
  int32_t* t;
  int32_t* p;
  uint32_t cmask, lane;
  __device__ __forceinline__ uint32_t ix(uint32_t s) const { return (s & cmask) * 256 + lane; }
  __device__ __forceinline__ bool full(uint32_t head, uint32_t top) const { return top - head == cmask + 1; }
};
template <class T>
struct GwHbmRing {
  T* v;
  int32_t* t;
  int32_t* p;
  __device__ __forceinline__ uint32_t ix(uint32_t s) const { return s; }
  __device__ __forceinline__ bool full(uint32_t, uint32_t) const { return false; }
};

// One key's walk state and step (the reference's per-event processing of e2's pending list, see the file header).
template <class T, int OP, bool STACK, class RING>
struct GwLane {
  RING R;
  uint32_t head = 0, top = 0;
  int32_t hts = 0, prev = INT32_MIN;
  T tv = T();
  bool bad = false;
  uint64_t cur = 0;   // next free unit of the key's match-area region
  uint32_t k = 0;
  uint32_t nm = 0;    // matches delivered
  // `within` compares in 32 bits: a key's times never go back on this path (such a push is redone on the tiled
  // path), so dts - hts is a non-negative difference of two 32-bit offsets and fits an unsigned 32-bit word
  uint32_t wi = 0;
  // returns false when the row would overflow the ring: the lane stops and k_gw_redo walks the whole key again
  __device__ __forceinline__ bool step(const GwArgs& a, const PtU4& q) {
    const int32_t dts = (int32_t)q.x;
    const uint32_t rowf = q.y;
    T x;
    const uint32_t xb = q.z;
    __builtin_memcpy(&x, &xb, sizeof(T));
    const int32_t pay = (int32_t)q.w;
    const uint32_t f = rowf >> 30;
    bad |= dts < prev;   // every row of the key takes part in the order check
    prev = dts;
    if (!f) return true;
    const bool live = !is_nan_val<T>(x);
    // lazy `within` expiry of the oldest partials (isExpired :102-113)
    if (head != top && (uint32_t)(dts - hts) > wi) {
      ++head;
      while (head != top) {
        hts = R.t[R.ix(head)];
        if ((uint32_t)(dts - hts) <= wi) break;
        ++head;
      }
    }
    const uint32_t r = rowf & ROW_MASK;
    uint32_t m = 0;
    if ((f & F_CONS) && live) {
      const bool emit = r >= (uint32_t)a.nc;   // a carried row completes nothing it did not complete before
      const uint64_t hdr = cur;
      if constexpr (STACK) {
        // monotone stack: the completed partials are exactly a suffix, delivered oldest first
        if (top != head && cmp_op<T>(OP, x, tv)) {
          --top;
          ++m;
          while (top != head) {
            tv = R.v[R.ix(top - 1)];
            if (!cmp_op<T>(OP, x, tv)) break;
            --top;
            ++m;
          }
        }
        if (emit && m) {
          for (uint32_t e = 0; e < m; ++e) {
            const uint32_t s = R.ix(top + e);
            a.area[hdr + 2 + e] = (uint64_t)(uint32_t)val_bits<T>(R.v[s]) | ((uint64_t)(uint32_t)R.p[s] << 32);
          }
        }
      } else {
        uint32_t wr = head;
        for (uint32_t s = head; s != top; ++s) {
          const uint32_t si = R.ix(s);
          const T e = R.v[si];
          if (cmp_op<T>(OP, x, e)) {
            if (emit) a.area[hdr + 2 + m] = (uint64_t)(uint32_t)val_bits<T>(e) | ((uint64_t)(uint32_t)R.p[si] << 32);
            ++m;
          } else {
            if (wr != s) {
              const uint32_t wx = R.ix(wr);
              R.v[wx] = e;
              R.t[wx] = R.t[si];
              R.p[wx] = R.p[si];
            }
            ++wr;
          }
        }
        top = wr;
        if (head != top) {
          hts = R.t[R.ix(head)];
          tv = R.v[R.ix(top - 1)];
        }
      }
      if (emit && m) {
        const uint64_t b = r - (uint32_t)a.nc;
        a.area[hdr] = (uint64_t)(uint32_t)dts | ((uint64_t)k << 32);
        a.area[hdr + 1] = (uint64_t)(uint32_t)val_bits<T>(x) | ((uint64_t)(uint32_t)pay << 32);
        a.trig[b] = hdr | ((uint64_t)m << 32);
        cur = hdr + 2 + m;
        nm += m;
      }
    }
    if ((f & F_CAND) && live) {
      if (R.full(head, top)) return false;
      const uint32_t s = R.ix(top);
      R.v[s] = x;
      R.t[s] = dts;
      R.p[s] = pay;
      if (top == head) hts = dts;
      tv = x;
      ++top;
    }
    return true;
  }
  // the key's final pending list as carried value rows
  __device__ __forceinline__ void carry(const GwArgs& a, uint32_t o) const {
    for (uint32_t e = 0; e < top - head; ++e) {
      const uint32_t s = R.ix(head + e);
      a.cv_ts[o + e] = a.t0 + (int64_t)R.t[s];
      a.cv_key[o + e] = (int32_t)k;
      a.cv_val[o + e] = val_bits<T>(R.v[s]);
      a.cv_pay[o + e] = a.pzero ? (int64_t)(uint32_t)R.p[s] : (int64_t)R.p[s];
    }
  }
};

template <class T, int OP, int PT, bool STACK>
__global__ void __launch_bounds__(256, 1) k_gwalk(GwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  GwLds<PT>& L = *(GwLds<PT>*)lds_raw;
  const uint32_t cap = (uint32_t)a.cap;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t g = xcd_block(blockIdx.x, gridDim.x);
  const uint32_t k = (g << 8) + t;
  const bool active = k < a.K;
  const uint32_t lo = a.o1[(size_t)g * a.ns1], hi = a.o1[(size_t)(g + 1) * a.ns1];
  GwLane<T, OP, STACK, GwLdsRing<T>> W;
  W.R.v = (T*)(lds_raw + sizeof(GwLds<PT>));            // ring planes [cap][256]: value, time, payload
  W.R.t = (int32_t*)(W.R.v + (size_t)cap * 256);
  W.R.p = W.R.t + (size_t)cap * 256;
  W.R.cmask = cap - 1;
  W.R.lane = t;
  W.k = k;
  W.wi = a.within > 0xffffffffll ? 0xffffffffu : (uint32_t)a.within;
  W.cur = active ? 3ull * a.kbase[k] : 0ull;
  bool ovf = false;
  const uint32_t ROWS = 256 * PT;
  PtU4 rc[PT], rn[PT];
  uint32_t tg[PT], tn[PT];
  // (the loads only issue here: nothing reads the registers before the next chunk's sort, so the next chunk's loads
  // stay in flight during this chunk's walk; rows past the group's end re-read its last row and are masked at use)
  auto load = [&](uint32_t base, PtU4* r, uint32_t* d) {
    const uint32_t rows = min(ROWS, hi - base);
#pragma unroll
    for (int s = 0; s < PT; ++s) {
      const uint32_t i = w * (PT * 64) + s * 64 + lane;
      const uint32_t p = base + (i < rows ? i : rows - 1);
      r[s] = __builtin_nontemporal_load(a.grec + p);
      d[s] = a.glk[p];
    }
  };
  if (lo < hi) load(lo, rc, tg);
  for (uint32_t base = lo; base < hi; base += ROWS) {
    {
      const uint32_t rows = min(ROWS, hi - base);
#pragma unroll
      for (int s = 0; s < PT; ++s)
        if (w * (PT * 64) + s * 64 + lane >= rows) tg[s] = 0xffffffffu;
    }
    // stable counting sort of the chunk by in-group key (wave ballots rank equal keys in arrival order)
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cw[q][t] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT; ++s)
      if (tg[s] != 0xffffffffu) atomicAdd(&L.cw[w][tg[s]], 1u);
    __syncthreads();
    {
      const uint32_t c0 = L.cw[0][t], c1 = L.cw[1][t], c2 = L.cw[2][t], c3 = L.cw[3][t];
      const uint32_t tt = c0 + c1 + c2 + c3;
      const uint32_t ex = block_excl_scan256(tt, L.wsum);
      L.ls[t] = ex;
      L.tot[t] = tt;
      L.cw[0][t] = ex;
      L.cw[1][t] = ex + c0;
      L.cw[2][t] = ex + c0 + c1;
      L.cw[3][t] = ex + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT; ++s) {
      const bool valid = tg[s] != 0xffffffffu;
      const uint32_t d = valid ? tg[s] : 0u;
      uint32_t rank, cnt;
      peer_rank(valid, d, 8, rank, cnt);
      if (valid) {
        const uint32_t slot = L.cw[w][d] + rank;
        if (rank == 0) L.cw[w][d] = slot + cnt;
        L.stage[slot] = rc[s];
      }
    }
    if (base + ROWS < hi) load(base + ROWS, rn, tn);   // next chunk in flight during the walk
    __syncthreads();
    // walk: lane t's rows of this chunk, in arrival order
    const uint32_t i0 = L.ls[t], i1 = i0 + L.tot[t];
    for (uint32_t i = i0; i < i1 && active && !ovf; ++i)
      if (!W.step(a, L.stage[i])) ovf = true;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT; ++s) { rc[s] = rn[s]; tg[s] = tn[s]; }
  }
  uint32_t fl = W.bad ? GW_ORDER : 0u;
  // (3 units per row bound the key's region: a header per trigger row, one unit per completed candidate row)
  if (active && W.cur > 3ull * a.kbase[k + 1]) fl |= GW_INTERNAL;
  if (ovf) {   // the key's list outgrew the ring: the whole key again on an HBM list (k_gw_redo)
    const uint32_t o = atomicAdd(a.ovf_n, 1u);
    if (o < a.ovf_cap) a.ovf_keys[o] = k;
    else fl |= GW_OVERFLOW;
  }
  if (fl) atomicOr(a.flags, fl);
  {
    uint32_t c = (active && !ovf) ? W.nm : 0u;   // (a redone key counts its matches in k_gw_redo)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if (lane == 0 && c) atomicAdd(a.match_n, c);
  }
  if (!a.carry_out) return;
  // the key's final pending list is the carry: slots reserved once per wave
  const uint32_t m = (active && !ovf) ? W.top - W.head : 0u;
  uint32_t incl = m;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
    if ((int)lane >= o) incl += y;
  }
  const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
  if (!tot) return;
  uint32_t cb = 0;
  if (lane == 63) cb = atomicAdd(a.cv_n, tot);
  cb = (uint32_t)__shfl((int)cb, 63);
  if ((uint64_t)cb + tot > (uint64_t)a.cv_cap) {
    if (lane == 63) atomicOr(a.flags, GW_CARRY_FULL);
    return;
  }
  if (m) W.carry(a, cb + incl - m);
}

// A key whose pending list outgrew the LDS ring, walked again from its first row with an unbounded list: one
// workgroup per such key gathers the key's rows from its group (arrival order kept) into the key's slice of `rows`,
// then one lane walks them (staged in LDS with the list when the key has at most GW_REDO_LDS rows, else from HBM with
// the list in HBM planes over the key's rows), rewriting the key's match-area region,
// its trigger words and its carry from the start (same walk, same rows: the same words the first walk wrote up to
// the overflow, then the rest).
static const uint32_t GW_REDO_LDS = 2048;   // rows of a redone key walked from LDS
template <class T, int OP, bool STACK>
__global__ void __launch_bounds__(256) k_gw_redo(GwArgs a, uint32_t* __restrict__ rows, T* __restrict__ hv,
                                                 int32_t* __restrict__ ht, int32_t* __restrict__ hp) {
  __shared__ uint32_t wc[4], base_s;
  __shared__ PtU4 red_stage[GW_REDO_LDS];
  __shared__ T red_v[GW_REDO_LDS];
  __shared__ int32_t red_t[GW_REDO_LDS], red_p[GW_REDO_LDS];
  const uint32_t k = a.ovf_keys[blockIdx.x];
  const uint32_t g = k >> 8, d = k & 255u, t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t lo = a.o1[(size_t)g * a.ns1], hi = a.o1[(size_t)(g + 1) * a.ns1];
  const uint32_t kb = a.kbase[k], ke = a.kbase[k + 1];
  if (t == 0) base_s = 0;
  __syncthreads();
  for (uint32_t p0 = lo; p0 < hi; p0 += 256) {
    const uint32_t p = p0 + t;
    const bool mine = p < hi && a.glk[p] == d;
    const uint64_t bm = __ballot(mine);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    if (lane == 0) wc[w] = (uint32_t)__popcll(bm);
    __syncthreads();
    uint32_t before = base_s;
    for (uint32_t q = 0; q < w; ++q) before += wc[q];
    if (mine && kb + before + below < ke) rows[kb + before + below] = p;
    __syncthreads();
    if (t == 0) base_s += wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
  const uint32_t nk = ke - kb;
  const bool in_lds = nk <= GW_REDO_LDS;   // (C5's keys: ~500 rows) records and list in LDS, else both in HBM
  if (in_lds)
    for (uint32_t i = t; i < nk; i += 256) red_stage[i] = a.grec[rows[kb + i]];
  __syncthreads();
  if (t != 0) return;
  if (kb + base_s != ke) { atomicOr(a.flags, GW_INTERNAL); return; }
  GwLane<T, OP, STACK, GwHbmRing<T>> W;
  if (in_lds) {
    W.R.v = red_v;
    W.R.t = red_t;
    W.R.p = red_p;
  } else {
    W.R.v = hv + kb;
    W.R.t = ht + kb;
    W.R.p = hp + kb;
  }
  W.k = k;
  W.wi = a.within > 0xffffffffll ? 0xffffffffu : (uint32_t)a.within;
  W.cur = 3ull * kb;
  if (in_lds) for (uint32_t i = 0; i < nk; ++i) W.step(a, red_stage[i]);
  else for (uint32_t i = kb; i < ke; ++i) W.step(a, a.grec[rows[i]]);
  uint32_t fl = W.bad ? GW_ORDER : 0u;
  if (W.cur > 3ull * ke) fl |= GW_INTERNAL;
  if (fl) atomicOr(a.flags, fl);
  if (W.nm) atomicAdd(a.match_n, W.nm);
  if (!a.carry_out) return;
  const uint32_t m = W.top - W.head;
  if (!m) return;
  const uint32_t o = atomicAdd(a.cv_n, m);
  if ((uint64_t)o + m > (uint64_t)a.cv_cap) { atomicOr(a.flags, GW_CARRY_FULL); return; }
  W.carry(a, o);
}

// Output records in delivery order: one thread per batch row (trigger order = arrival order).  A trigger's matches
// are read from its header in the match area (one 16-byte header + 8 bytes per match, contiguous) and assembled in
// LDS at their position inside the block's output range, which is then stored contiguously (whole lines, 16-byte
// stores by consecutive threads); a block whose rows deliver more than GW_PROJ_S records does it in rounds.
struct GwSel {
  int32_t n_select, stride, multi, b_slot, pzero, vfloat;
  int32_t code[SG_MAX_SELECT];   // 0 e1 payload, 1 e1 value, 2 e2 value, 3 e2 payload, 4 null
};
static const int GW_PROJ_S = 256;   // records staged per round
static const int GW_TILE = 256;     // rows per projection tile (one per thread)

// matches per 256-row tile of trigger words, eight tiles per workgroup (the projection's tile bases come from a scan
// over these)
static __global__ void __launch_bounds__(256) k_gtile_count(int64_t n, const uint64_t* __restrict__ trig,
                                                            uint32_t* __restrict__ tcount, int64_t ntile) {
  __shared__ uint32_t red[8][4];
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int64_t r = ((int64_t)blockIdx.x * 8 + s) * GW_TILE + t;
    uint32_t c = r < n ? (uint32_t)(__builtin_nontemporal_load(trig + r) >> 32) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if (lane == 0) red[s][w] = c;
  }
  __syncthreads();
  if (t < 8) {
    const int64_t tile = (int64_t)blockIdx.x * 8 + t;
    if (tile < ntile) tcount[tile] = red[t][0] + red[t][1] + red[t][2] + red[t][3];
  }
}

// Output records: one workgroup per 256-row tile (one row per thread: every trigger's header read is in flight at
// once), its first output slot from the scanned tile counts and each row's from a block scan; the tile's records are
// assembled in LDS in slot order and stored contiguously (GW_PROJ_S records per round).
static __global__ void __launch_bounds__(256) k_gscan_project(int64_t n, int64_t t0, uint64_t base_index,
                                                              const uint64_t* __restrict__ index,
                                                              const uint64_t* __restrict__ trig,
                                                              const uint64_t* __restrict__ area, GwSel sel,
                                                              int64_t out_base, char* __restrict__ out,
                                                              const uint32_t* __restrict__ tbase) {
  extern __shared__ __attribute__((aligned(16))) char stage[];
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x;
  const int64_t b = (int64_t)blockIdx.x * GW_TILE + t;
  const uint64_t tw = b < n ? __builtin_nontemporal_load(trig + b) : 0ull;
  const uint32_t m = (uint32_t)(tw >> 32);
  const uint64_t u = (uint32_t)tw;
  uint64_t h0 = 0, h1 = 0, tg = 0;
  if (m) {
    h0 = area[u];
    h1 = area[u + 1];
    tg = index ? index[b] : base_index + (uint64_t)b;
  }
  const uint32_t excl = block_excl_scan256(m, wsum);
  const uint32_t pre = tbase[blockIdx.x];
  const uint32_t o_lo = pre, o_hi = pre + (wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  const uint32_t o = pre + excl;
  auto wid = [&](uint32_t bits, bool zero) { return zero ? (int64_t)bits : (int64_t)(int32_t)bits; };
  uint32_t nmask = 0;
  for (int s = 0; s < sel.n_select; ++s) nmask |= (sel.code[s] == 4) ? 1u << s : 0u;
  const int64_t ts = t0 + (int64_t)(int32_t)(uint32_t)h0;
  const uint32_t key = (uint32_t)(h0 >> 32);
  const int64_t v2 = wid((uint32_t)h1, sel.vfloat), p2 = wid((uint32_t)(h1 >> 32), sel.pzero);
  typedef uint32_t U4 __attribute__((ext_vector_type(4)));
  for (uint32_t sub = o_lo; sub < o_hi; sub += GW_PROJ_S) {
    const uint32_t se = (o_hi - sub < (uint32_t)GW_PROJ_S) ? o_hi : sub + GW_PROJ_S;
    if (m && o < se && o + m > sub) {
      const uint32_t qa = o < sub ? sub - o : 0u, qe = (o + m > se) ? se - o : m;
      for (uint32_t q = qa; q < qe; ++q) {
        const uint64_t e = area[u + 2 + q];
        const int64_t v1 = wid((uint32_t)e, sel.vfloat), p1 = wid((uint32_t)(e >> 32), sel.pzero);
        int64_t* r = (int64_t*)(stage + (size_t)(o + q - sub) * sel.stride);
        r[0] = (int64_t)tg;
        r[1] = ts;
        r[2] = (int64_t)((uint64_t)key | ((uint64_t)((1u << 24) | (sel.multi ? (uint32_t)sel.b_slot : (0x800000u | q))) << 32));
        r[3] = (int64_t)nmask;
        for (int c = 0; c < sel.n_select; ++c) {
          const int code = sel.code[c];
          r[4 + c] = code == 0 ? p1 : code == 1 ? v1 : code == 2 ? v2 : code == 3 ? p2 : 0;
        }
      }
    }
    __syncthreads();
    const size_t bytes = (size_t)(se - sub) * sel.stride;
    char* dst = out + (size_t)(out_base + sub) * sel.stride;
    if ((((uintptr_t)dst) & 15) == 0) {
      for (size_t x = (size_t)t * 16; x < bytes; x += 256 * 16) *(U4*)(dst + x) = *(const U4*)(stage + x);
    } else {
      for (size_t x = (size_t)t * 8; x < bytes; x += 256 * 8) *(uint64_t*)(dst + x) = *(const uint64_t*)(stage + x);
    }
    __syncthreads();
  }
}

