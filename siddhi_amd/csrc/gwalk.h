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
  uint32_t* flags;            // GW_ORDER | GW_OVERFLOW | GW_INTERNAL
};
static const uint32_t GW_ORDER = 1, GW_OVERFLOW = 2, GW_INTERNAL = 4;

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

template <class T, int OP, int PT>
__global__ void __launch_bounds__(256, 1) k_gwalk(GwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  GwLds<PT>& L = *(GwLds<PT>*)lds_raw;
  const uint32_t cap = (uint32_t)a.cap, cmask = cap - 1;
  T* rv = (T*)(lds_raw + sizeof(GwLds<PT>));            // ring planes [cap][256]: value, time, payload
  int32_t* rt = (int32_t*)(rv + (size_t)cap * 256);
  int32_t* rp = rt + (size_t)cap * 256;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t g = xcd_block(blockIdx.x, gridDim.x);
  const uint32_t k = (g << 8) + t;
  const bool active = k < a.K;
  const uint32_t lo = a.o1[(size_t)g * a.ns1], hi = a.o1[(size_t)(g + 1) * a.ns1];
  auto ix = [&](uint32_t s) { return (s & cmask) * 256 + t; };
  // lane state: ring [head, top) -- oldest first; register copies of the oldest time and the newest value
  uint32_t head = 0, top = 0;
  int32_t hts = 0, prev = INT32_MIN;
  T tv = T();
  bool bad = false, ovf = false;
  uint64_t cur = active ? 3ull * a.kbase[k] : 0ull;   // next free unit of the key's match-area region
  const uint32_t ROWS = 256 * PT;
  PtU4 rc[PT], rn[PT];
  uint32_t tg[PT], tn[PT];
  auto load = [&](uint32_t base, PtU4* r, uint32_t* d) {
    const uint32_t rows = min(ROWS, hi - base);
#pragma unroll
    for (int s = 0; s < PT; ++s) {
      const uint32_t i = w * (PT * 64) + s * 64 + lane;
      const uint32_t p = base + (i < rows ? i : rows - 1);
      r[s] = __builtin_nontemporal_load(a.grec + p);
      const uint32_t kk = a.glk[p];
      d[s] = i < rows ? kk : 0xffffffffu;
    }
  };
  if (lo < hi) load(lo, rc, tg);
  for (uint32_t base = lo; base < hi; base += ROWS) {
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
    for (uint32_t i = i0; i < i1 && active && !ovf; ++i) {
      const PtU4 q = L.stage[i];
      const int32_t dts = (int32_t)q.x;
      const uint32_t rowf = q.y;
      T x;
      const uint32_t xb = q.z;
      __builtin_memcpy(&x, &xb, sizeof(T));
      const int32_t pay = (int32_t)q.w;
      const uint32_t f = rowf >> 30;
      bad |= dts < prev;   // every row of the key takes part in the order check
      prev = dts;
      if (!f) continue;
      // lazy `within` expiry of the oldest partials (isExpired :102-113)
      if (head != top && (int64_t)dts - (int64_t)hts > a.within) {
        ++head;
        while (head != top) {
          hts = rt[ix(head)];
          if ((int64_t)dts - (int64_t)hts <= a.within) break;
          ++head;
        }
      }
      const uint32_t r = rowf & ROW_MASK;
      const bool live = !is_nan_val<T>(x);
      uint32_t m = 0;
      if ((f & F_CONS) && live) {
        const bool emit = r >= (uint32_t)a.nc;   // a carried row completes nothing it did not complete before
        const uint64_t hdr = cur;
        if (a.stack_mode) {
          // monotone stack: the completed partials are exactly a suffix, delivered oldest first
          if (top != head && cmp_op<T>(OP, x, tv)) {
            --top;
            ++m;
            while (top != head) {
              tv = rv[ix(top - 1)];
              if (!cmp_op<T>(OP, x, tv)) break;
              --top;
              ++m;
            }
          }
          if (emit && m) {
            for (uint32_t e = 0; e < m; ++e) {
              const uint32_t s = ix(top + e);
              a.area[hdr + 2 + e] = (uint64_t)(uint32_t)val_bits<T>(rv[s]) | ((uint64_t)(uint32_t)rp[s] << 32);
            }
          }
        } else {
          uint32_t wr = head;
          for (uint32_t s = head; s != top; ++s) {
            const uint32_t si = ix(s);
            const T e = rv[si];
            if (cmp_op<T>(OP, x, e)) {
              if (emit) a.area[hdr + 2 + m] = (uint64_t)(uint32_t)val_bits<T>(e) | ((uint64_t)(uint32_t)rp[si] << 32);
              ++m;
            } else {
              if (wr != s) {
                const uint32_t wi = ix(wr);
                rv[wi] = e;
                rt[wi] = rt[si];
                rp[wi] = rp[si];
              }
              ++wr;
            }
          }
          top = wr;
          if (head != top) {
            hts = rt[ix(head)];
            tv = rv[ix(top - 1)];
          }
        }
        if (emit && m) {
          const uint64_t b = r - (uint32_t)a.nc;
          a.area[hdr] = (uint64_t)(uint32_t)dts | ((uint64_t)k << 32);
          a.area[hdr + 1] = (uint64_t)(uint32_t)val_bits<T>(x) | ((uint64_t)(uint32_t)pay << 32);
          a.trig[b] = hdr | ((uint64_t)m << 32);
          cur = hdr + 2 + m;
        }
      }
      if ((f & F_CAND) && live) {
        if (top - head == cap) { ovf = true; break; }
        const uint32_t s = ix(top);
        rv[s] = x;
        rt[s] = dts;
        rp[s] = pay;
        if (top == head) hts = dts;
        tv = x;
        ++top;
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT; ++s) { rc[s] = rn[s]; tg[s] = tn[s]; }
  }
  uint32_t fl = (bad ? GW_ORDER : 0u) | (ovf ? GW_OVERFLOW : 0u);
  // (3 units per row bound the key's region: a header per trigger row, one unit per completed candidate row)
  if (active && cur > 3ull * a.kbase[k + 1]) fl |= GW_INTERNAL;
  if (fl) atomicOr(a.flags, fl);
  if (!a.carry_out) return;
  // the key's final pending list is the carry: slots reserved once per wave
  const uint32_t m = (active && !ovf) ? top - head : 0u;
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
    if (lane == 63) atomicOr(a.flags, GW_INTERNAL);
    return;
  }
  const uint32_t o = cb + incl - m;
  for (uint32_t e = 0; e < m; ++e) {
    const uint32_t s = ix(head + e);
    a.cv_ts[o + e] = a.t0 + (int64_t)rt[s];
    a.cv_key[o + e] = (int32_t)k;
    a.cv_val[o + e] = val_bits<T>(rv[s]);
    a.cv_pay[o + e] = a.pzero ? (int64_t)(uint32_t)rp[s] : (int64_t)rp[s];
  }
}

// Output records in delivery order: one thread per batch row (trigger order = arrival order); a trigger's matches
// are read from its header in the match area and written at its scanned output slot, in pending order.
struct GwSel {
  int32_t n_select, stride, multi, b_slot, pzero, vfloat;
  int32_t code[SG_MAX_SELECT];   // 0 e1 payload, 1 e1 value, 2 e2 value, 3 e2 payload, 4 null
};
static __global__ void __launch_bounds__(256) k_gproject(int64_t n, int64_t t0, uint64_t base_index,
                                                         const uint64_t* __restrict__ index,
                                                         const uint64_t* __restrict__ trig, const uint32_t* __restrict__ off,
                                                         const uint64_t* __restrict__ area, GwSel sel, int64_t out_base,
                                                         char* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint64_t tw = trig[b];
  const uint32_t m = (uint32_t)(tw >> 32);
  if (!m) return;
  const uint64_t u = (uint32_t)tw;
  const uint64_t h0 = area[u], h1 = area[u + 1];
  const int64_t ts = t0 + (int64_t)(int32_t)(uint32_t)h0;
  const uint32_t key = (uint32_t)(h0 >> 32);
  auto wid = [&](uint32_t bits, bool zero) { return zero ? (int64_t)bits : (int64_t)(int32_t)bits; };
  const int64_t v2 = wid((uint32_t)h1, sel.vfloat), p2 = wid((uint32_t)(h1 >> 32), sel.pzero);
  const uint64_t tg = index ? index[b] : base_index + (uint64_t)b;
  const uint32_t o = off[b];
  uint32_t nm = 0;
  for (int s = 0; s < sel.n_select; ++s) nm |= (sel.code[s] == 4) ? 1u << s : 0u;
  for (uint32_t q = 0; q < m; ++q) {
    const uint64_t e = area[u + 2 + q];
    const int64_t v1 = wid((uint32_t)e, sel.vfloat), p1 = wid((uint32_t)(e >> 32), sel.pzero);
    int64_t* r = (int64_t*)(out + (size_t)(out_base + o + q) * sel.stride);
    r[0] = (int64_t)tg;
    r[1] = ts;
    r[2] = (int64_t)((uint64_t)key | ((uint64_t)((1u << 24) | (sel.multi ? (uint32_t)sel.b_slot : (0x800000u | q))) << 32));
    r[3] = (int64_t)nm;
    for (int s = 0; s < sel.n_select; ++s) {
      const int c = sel.code[s];
      r[4 + s] = c == 0 ? p1 : c == 1 ? v1 : c == 2 ? v2 : c == 3 ? p2 : 0;
    }
  }
}

struct GwTrigCount {
  __host__ __device__ uint32_t operator()(uint64_t x) const { return (uint32_t)(x >> 32); }
};
