#pragma once
// fgw.h -- fused group walk: the partitioned closed form `every A[l] -> B[l' and B.x OP A.x] within T` without a full
// key sort, without a count walk, without random writes or reads of per-row offsets (included by engine_impl.h).
//
// Same semantics as the walker of engine_impl.h (StreamPreStateProcessor.processAndReturn,
// C/query/input/stream/state/StreamPreStateProcessor.java:292-337: per key, e2's pending list in arrival order, lazy
// `within` expiry of the oldest, completion of every pending partial with x_j OP x_i delivered in pending order, then
// the event's own partial).  What changes is where the rows of a key meet:
//
//   part1 (k_part1)  rows -> 16-B walker records grouped by key group (the high bits of the dense key), arrival order
//                    kept inside a group ("group domain"), plus each record's in-group key.  Unchanged.
//   k_fgw            one workgroup per (group, time segment): streams the segment's group-domain rows (after a replay of
//                    the rows inside `within` before it) through LDS in 2048-row sub-tiles, sorts each sub-tile by
//                    in-group key in LDS (stable counting sort), and one lane per key walks its rows with the key's
//                    pending list resident in LDS across sub-tiles -- no key-sorted copy of the batch is ever written.
//                    A sub-tile's matches are reordered in LDS into group-domain order (its rows' arrival order) and
//                    written out contiguously: a count word per row (gm32) and 16-B compact match records (e1's value,
//                    payload and row); per projection chunk the group's first compact position (cst) and its matches.
//   k_fgw_proj       one workgroup per projection chunk (a part1 segment = 8192 consecutive rows): interleaves the
//                    groups' count words by arrival index in LDS, scans them, and writes the chunk's match records --
//                    one contiguous range of the output -- reading the compact records group by group (coalesced).
//   carry            per key, the pending partials still inside `within` of its last row, plus that row, become the next
//                    push's carried virtual rows (replaying them rebuilds exactly the pending list).
//
// Preconditions checked on the GPU (any failure reruns the push on the sorted-walker pipeline, which has none of them
// and gives the same rows): timestamps non-decreasing in arrival order within each group (the replay start is a binary
// search), every key's pending list within the LDS ring, every sub-tile's matches within the LDS staging buffer.
#include <hip/hip_runtime.h>

static const int FGW_T = 2048;            // group rows per sub-tile
static const int FGW_PT = FGW_T / 256;    // rows per thread per sub-tile
static const int FGW_EB = 1536;           // LDS match records per sub-tile
static const int FGW_CHUNK = 65536;       // largest projection chunk = part1 segment (virtual rows)
static const int FGW_SUB = 8192;          // rows of a chunk the projection orders in LDS at a time
static const uint32_t FGW_NONE = 0xffffffffu;
static const uint32_t FGW_F_ORDER = 1, FGW_F_RING = 2, FGW_F_EMIT = 4, FGW_F_INTERNAL = 8;

struct FgwSeg {
  uint32_t rs, lo, hi;   // replay start, segment [lo, hi) in the group domain
  uint32_t cb;           // compact-record base of the segment
};

struct FgwArgs {
  int64_t nc;            // carried virtual rows (never emit)
  int32_t within;        // `within` clamped to 31 bits (relative times fit 31 bits: narrow records)
  int32_t op;
  int32_t stack_mode;
  uint32_t K, lb, ng, nsw, ns1, seg1, tsw;
  uint32_t cap;          // pending-list ring entries per key (power of two, <= template CAP)
  const uint32_t* o1;    // part1 offsets: o1[g * ns1 + j] = first group-domain position of (group g, segment j)
};

template <class T, int KG, int CAP>
struct FgwLds {
  // pending lists: ring slot s of key k at (s & (CAP - 1)) * KG + k (lanes of a wave: consecutive keys, no conflicts)
  T sval[CAP * KG];
  int32_t sdts[CAP * KG];
  int32_t spay[CAP * KG];
  uint32_t srow[CAP * KG];
  PtU4 srt[FGW_T];             // the sub-tile's records sorted by in-group key
  uint16_t said[FGW_T];        // arrival-local index of each sorted slot
  uint16_t sslot[FGW_T];       // sorted slot of each arrival-local index
  uint32_t aux[FGW_T];         // before the walk: dts by arrival index (order check); after: m | emission slot << 16
                               // by sorted slot
  uint16_t eoff[FGW_T];        // exclusive scan of m over arrival order
  PtU4 ebuf[FGW_EB];           // the sub-tile's match records in walk order
  uint32_t cw[4][256];         // per-wave digit counts, then slot cursors
  uint32_t kb[256], kn[256];   // per in-group key: first sorted slot, rows
  uint32_t wsum[4];
  uint32_t etop, flags, ttot;
  uint32_t rfirst, rlast;      // arrival rows of the sub-tile's first and last segment rows
};

template <class T>
__device__ __forceinline__ T fgw_from32(uint32_t u) {
  T x;
  __builtin_memcpy(&x, &u, 4);
  return x;
}
template <class T>
__device__ __forceinline__ uint32_t fgw_to32(T x) {
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  return u;
}
template <class T>
__device__ __forceinline__ T fgw_val(const PtU4& q) { return fgw_from32<T>(q.z); }

template <class T, int OP>
__device__ __forceinline__ bool fgw_cmp(int op, T b, T a) { return cmp_sel<OP, T>(op, b, a); }

// One workgroup per (group g, walk segment jj).
template <class T, int KG, int CAP, int OP>
__global__ void __launch_bounds__(256) k_fgw(FgwArgs A, const PtU4* __restrict__ grec, const uint8_t* __restrict__ glk,
                                             const FgwSeg* __restrict__ segs, uint32_t* __restrict__ gm32,
                                             PtU4* __restrict__ comp, uint32_t* __restrict__ cst, uint32_t* __restrict__ cend,
                                             uint32_t* __restrict__ kcnt, uint32_t* __restrict__ kent,
                                             uint32_t* __restrict__ flags_out) {
  static_assert(sizeof(T) == 4, "narrow 4-byte values only");
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  FgwLds<T, KG, CAP>& L = *(FgwLds<T, KG, CAP>*)lds_raw;
  const uint32_t wgi = blockIdx.x;
  const uint32_t g = wgi / A.nsw, jj = wgi % A.nsw;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  const FgwSeg sg = segs[wgi];
  const uint32_t j0 = jj * A.tsw;
  const uint32_t j1 = min(A.ns1, j0 + A.tsw);
  const uint32_t cmask = A.cap - 1;
  if (t == 0) { L.flags = 0; }
  // the key this lane walks (KG <= 256: lanes >= KG only help with loads, sorts and write-out)
  const bool owner = t < (uint32_t)KG;
  uint32_t head = 0, top = 0;
  int32_t hts = 0;             // time of the oldest pending partial (valid while head != top)
  T tv = T();                  // value of the newest pending partial
  uint32_t lastpos = FGW_NONE; // last segment row of the key (group domain)
  int32_t prevt = INT32_MIN;   // order check across sub-tiles (thread 0 only: last row of the previous sub-tile)
  uint32_t cur = 0;            // matches emitted by this segment so far
  uint32_t nb = 0;
  while ((1u << nb) < (uint32_t)KG) ++nb;
  const uint32_t lmask = (uint32_t)KG - 1;
  auto load = [&](uint32_t base, PtU4* rc, uint32_t* tg) {
    const uint32_t rows = min((uint32_t)FGW_T, sg.hi - base);
#pragma unroll
    for (int s = 0; s < FGW_PT; ++s) {
      const uint32_t i = w * (FGW_PT * 64) + s * 64 + lane;
      const uint32_t p = base + (i < rows ? i : rows - 1);   // (clamped: branch-free loads)
      rc[s] = __builtin_nontemporal_load(grec + p);
      const uint32_t k = glk[p];
      tg[s] = i < rows ? (k & lmask) : 0xffffffffu;
    }
  };
  PtU4 rc[FGW_PT], rn[FGW_PT];
  uint32_t tg[FGW_PT], tn[FGW_PT];
  if (sg.rs < sg.hi) load(sg.rs, rc, tg);
  __syncthreads();
  for (uint32_t base = sg.rs; base < sg.hi; base += FGW_T) {
    const uint32_t rows = min((uint32_t)FGW_T, sg.hi - base);
    // ---- stable counting sort of the sub-tile by in-group key
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cw[q][t] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < FGW_PT; ++s) {
      if (tg[s] != 0xffffffffu) atomicAdd(&L.cw[w][tg[s]], 1u);
      const uint32_t i = w * (FGW_PT * 64) + s * 64 + lane;
      if (i < rows) L.aux[i] = rc[s].x;   // dts by arrival index (order check)
    }
    __syncthreads();
    {
      const uint32_t c0 = L.cw[0][t], c1 = L.cw[1][t], c2 = L.cw[2][t], c3 = L.cw[3][t];
      const uint32_t tot = c0 + c1 + c2 + c3;
      const uint32_t ex = block_excl_scan256(tot, L.wsum);
      L.kb[t] = ex;
      L.kn[t] = tot;
      L.cw[0][t] = ex;
      L.cw[1][t] = ex + c0;
      L.cw[2][t] = ex + c0 + c1;
      L.cw[3][t] = ex + c0 + c1 + c2;
    }
    // order check: timestamps non-decreasing in the group domain (the replay-start search and the walk rely on it)
    {
      bool bad = false;
      for (uint32_t i = t; i < rows; i += 256) {
        const int32_t a = (int32_t)L.aux[i];
        const int32_t b = i ? (int32_t)L.aux[i - 1] : prevt;
        bad |= a < b;
      }
      if (bad) atomicOr(&L.flags, FGW_F_ORDER);
    }
    const int32_t lastt = (int32_t)L.aux[rows - 1];   // (read before the barrier: aux is cleared after it)
    __syncthreads();
    prevt = lastt;
#pragma unroll
    for (int s = 0; s < FGW_PT; ++s) {
      const bool valid = tg[s] != 0xffffffffu;
      const uint32_t d = valid ? tg[s] : 0u;
      uint32_t rank, cnt;
      peer_rank(valid, d, nb, rank, cnt);
      if (valid) {
        const uint32_t slot = L.cw[w][d] + rank;
        if (rank == 0) L.cw[w][d] = slot + cnt;
        const uint32_t ai = w * (FGW_PT * 64) + s * 64 + lane;
        L.srt[slot] = rc[s];
        L.said[slot] = (uint16_t)ai;
        L.sslot[ai] = (uint16_t)slot;
      }
    }
    for (uint32_t i = t; i < rows; i += 256) L.aux[i] = 0;
    if (t == 0) L.etop = 0;
    // next sub-tile's loads in flight during the walk
    if (base + FGW_T < sg.hi) load(base + FGW_T, rn, tn);
    __syncthreads();
    // ---- walk: lane k steps through its key's rows of the sub-tile
    if (owner) {
      const uint32_t s0 = L.kb[t], s1 = s0 + L.kn[t];
      // segment rows (which emit) vs replay rows: only the sub-tile that straddles the segment start mixes them
      const bool seg_all = base >= sg.lo, seg_none = base + rows <= sg.lo;
      if (s1 > s0 && !seg_none) {
        const uint32_t pl = base + L.said[s1 - 1];
        if (pl >= sg.lo) lastpos = pl;
      }
      for (uint32_t s = s0; s < s1; ++s) {
        const PtU4 q = L.srt[s];
        const uint32_t f = q.y >> 30;
        const uint32_t r = q.y & ROW_MASK;
        const int32_t tt = (int32_t)q.x;
        const T x = fgw_val<T>(q);
        if (!f) continue;
        const bool in_seg = seg_all || (!seg_none && base + L.said[s] >= sg.lo);
        // lazy `within` expiry of the oldest partials (StreamPreStateProcessor.isExpired :102-113)
        if (head != top && (int64_t)tt - hts > A.within) {
          ++head;
          while (head != top) {
            hts = L.sdts[(head & cmask) * KG + t];
            if ((int64_t)tt - hts <= A.within) break;
            ++head;
          }
        }
        const bool live = !is_nan_val<T>(x);
        const bool emit = in_seg && (int64_t)r >= A.nc;
        uint32_t m = 0;
        if ((f & F_CONS) && live && head != top) {
          if (A.stack_mode) {
            // the completed partials are a suffix of the monotone stack, delivered oldest first
            if (fgw_cmp<T, OP>(A.op, x, tv)) {
              m = 1;
              while (top - m != head && fgw_cmp<T, OP>(A.op, x, L.sval[((top - m - 1) & cmask) * KG + t])) ++m;
              if (emit) {
                const uint32_t e0 = atomicAdd(&L.etop, m);
                if (e0 + m > (uint32_t)FGW_EB) {
                  atomicOr(&L.flags, FGW_F_EMIT);
                } else {
                  for (uint32_t u = 0; u < m; ++u) {
                    const uint32_t ix = ((top - m + u) & cmask) * KG + t;
                    PtU4 e;
                    e.x = fgw_to32<T>(L.sval[ix]);
                    e.y = (uint32_t)L.spay[ix];
                    e.z = L.srow[ix];
                    e.w = 0;
                    L.ebuf[e0 + u] = e;
                  }
                  L.aux[s] = m | (e0 << 16);
                }
              }
              top -= m;
              if (head != top) tv = L.sval[((top - 1) & cmask) * KG + t];
            }
          } else {
            // scanned list: complete every matching partial in list order, keep the others in order
            uint32_t wr = head, e0 = 0;
            bool room = true;
            for (uint32_t sl = head; sl != top; ++sl) {
              const uint32_t ix = (sl & cmask) * KG + t;
              const T e = L.sval[ix];
              if (fgw_cmp<T, OP>(A.op, x, e)) {
                if (emit) {
                  if (m == 0) {
                    // (reserve the worst case: every remaining partial completes)
                    e0 = atomicAdd(&L.etop, top - sl);
                    room = e0 + (top - sl) <= (uint32_t)FGW_EB;
                    if (!room) atomicOr(&L.flags, FGW_F_EMIT);
                  }
                  if (room) {
                    PtU4 q2;
                    q2.x = fgw_to32<T>(e);
                    q2.y = (uint32_t)L.spay[ix];
                    q2.z = L.srow[ix];
                    q2.w = 0;
                    L.ebuf[e0 + m] = q2;
                  }
                }
                ++m;
              } else {
                if (wr != sl) {
                  const uint32_t iw = (wr & cmask) * KG + t;
                  L.sval[iw] = e;
                  L.sdts[iw] = L.sdts[ix];
                  L.spay[iw] = L.spay[ix];
                  L.srow[iw] = L.srow[ix];
                }
                ++wr;
              }
            }
            if (emit && m && room) L.aux[s] = m | (e0 << 16);
            top = wr;
            if (head != top) {
              hts = L.sdts[(head & cmask) * KG + t];
              tv = L.sval[((top - 1) & cmask) * KG + t];
            }
          }
        }
        if ((f & F_CAND) && live) {
          if (top - head == A.cap) {
            atomicOr(&L.flags, FGW_F_RING);
          } else {
            const uint32_t ix = (top & cmask) * KG + t;
            L.sval[ix] = x;
            L.sdts[ix] = tt;
            L.spay[ix] = (int32_t)q.w;
            L.srow[ix] = r;
            if (top == head) hts = tt;
            tv = x;
            ++top;
          }
        }
      }
    }
    __syncthreads();
    // ---- the sub-tile's matches in arrival order: scan m, then contiguous writes
    {
      uint32_t sum = 0;
      uint32_t mv[FGW_PT];
#pragma unroll
      for (int q = 0; q < FGW_PT; ++q) {
        const uint32_t a = t * FGW_PT + q;
        mv[q] = a < rows ? (L.aux[L.sslot[a]] & 0xffffu) : 0u;
        sum += mv[q];
      }
      const uint32_t ex = block_excl_scan256(sum, L.wsum);
      uint32_t run = ex;
#pragma unroll
      for (int q = 0; q < FGW_PT; ++q) {
        const uint32_t a = t * FGW_PT + q;
        if (a < rows) L.eoff[a] = (uint16_t)run;
        run += mv[q];
      }
      if (t == 255) L.ttot = run;
    }
    __syncthreads();
    // per row (the lanes that loaded it): count word, match records, projection-chunk bookkeeping
#pragma unroll
    for (int s = 0; s < FGW_PT; ++s) {
      const uint32_t i = w * (FGW_PT * 64) + s * 64 + lane;
      if (i >= rows) continue;
      const uint32_t pos = base + i;
      if (pos < sg.lo) continue;
      const uint32_t av = L.aux[L.sslot[i]];
      const uint32_t m = av & 0xffffu;
      const uint32_t r = rc[s].y & ROW_MASK;
      const uint32_t j = r / A.seg1;
      gm32[pos] = (r - j * A.seg1) | (m << 16);
      const uint32_t dst = sg.cb + cur + L.eoff[i];
      if (j < j0 || j >= j1) atomicOr(&L.flags, FGW_F_INTERNAL);
      if (pos == max(base, sg.lo)) L.rfirst = r;
      if (i == rows - 1) L.rlast = r;
      if (m) {
        const uint32_t e0 = av >> 16;
        for (uint32_t u = 0; u < m; ++u) comp[dst + u] = L.ebuf[e0 + u];
      }
    }
    __syncthreads();
    // projection-chunk bookkeeping: the compact positions where each chunk's rows of this group start and end
    if (base + rows > sg.lo) {
      const uint32_t pa = max(base, sg.lo), pe = base + rows;
      const uint32_t ja = L.rfirst / A.seg1, je = L.rlast / A.seg1;
      for (uint32_t j = ja + t; j <= je; j += 256) {
        const size_t gj = (size_t)g * A.ns1 + j;
        const uint32_t p0 = A.o1[gj], p1 = A.o1[gj + 1];
        if (p0 >= pa && p0 < pe) cst[gj] = sg.cb + cur + L.eoff[p0 - base];
        if (p1 > pa && p1 <= pe)
          cend[gj] = sg.cb + cur + L.eoff[p1 - 1 - base] + (L.aux[L.sslot[p1 - 1 - base]] & 0xffffu);
      }
    }
    cur += L.ttot;
#pragma unroll
    for (int s = 0; s < FGW_PT; ++s) { rc[s] = rn[s]; tg[s] = tn[s]; }
    __syncthreads();
  }
  // ---- segment end: the keys' end states for the carry
  if (owner && kcnt && lastpos != FGW_NONE) {
    // pending partials inside `within` of the key's last row of this segment (+ that row when it is not one of them):
    // if this segment holds the key's last row of the push, these become the key's carried rows
    const size_t slot = (size_t)jj * A.K + (size_t)g * KG + t;
    const PtU4 lr = grec[lastpos];
    const int32_t tl = (int32_t)lr.x;
    const uint32_t rl = lr.y & ROW_MASK;
    uint32_t c = 0;
    uint32_t* dst = kent + slot * (A.cap + 1);
    bool last_pending = false;
    for (uint32_t sl = head; sl != top; ++sl) {
      const uint32_t ix = (sl & cmask) * KG + t;
      if ((int64_t)tl - L.sdts[ix] > A.within) continue;
      dst[c++] = L.srow[ix];
      last_pending |= L.srow[ix] == rl;
    }
    if (!last_pending) dst[c++] = rl;
    kcnt[slot] = c | ((uint32_t)jj << 24);
    (void)tl;
  }
  __syncthreads();
  if (t == 0 && L.flags) atomicOr(flags_out, L.flags);
}

// Walk-segment plan: group g's segment jj covers projection chunks [jj*tsw, (jj+1)*tsw); its replay starts at the
// group's first row inside `within` of the segment's first row.  cap = rows walked (a bound on its matches).
static __global__ void k_fgw_plan(FgwArgs A, const PtU4* __restrict__ grec, FgwSeg* __restrict__ segs, uint32_t* __restrict__ caps) {
  const uint32_t wgi = blockIdx.x * blockDim.x + threadIdx.x;
  if (wgi >= A.ng * A.nsw) return;
  const uint32_t g = wgi / A.nsw, jj = wgi % A.nsw;
  const uint32_t j0 = min(A.ns1, jj * A.tsw), j1 = min(A.ns1, j0 + A.tsw);
  const uint32_t gs = A.o1[(size_t)g * A.ns1];
  const uint32_t lo = A.o1[(size_t)g * A.ns1 + j0];
  const uint32_t hi = A.o1[(size_t)g * A.ns1 + j1];   // (j1 == ns1: the next group's first position)
  uint32_t rs = lo;
  if (lo < hi && lo > gs) {
    const int64_t tmin = (int64_t)(int32_t)grec[lo].x - (int64_t)A.within;
    uint32_t a = gs, b = lo;
    while (a < b) {
      const uint32_t mid = a + ((b - a) >> 1);
      if ((int64_t)(int32_t)grec[mid].x < tmin) a = mid + 1; else b = mid;
    }
    rs = a;
  }
  segs[wgi] = FgwSeg{rs, lo, hi, 0};
  caps[wgi] = hi - rs;
}

static __global__ void k_fgw_cb(uint32_t n, const uint32_t* __restrict__ off, FgwSeg* __restrict__ segs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) segs[i].cb = off[i];
}

// Matches per projection chunk: the sum over groups of their compact ranges (cend - cst) in the chunk.
static __global__ void __launch_bounds__(256) k_fgw_ctot(FgwArgs A, const uint32_t* __restrict__ cst,
                                                         const uint32_t* __restrict__ cend, uint32_t* __restrict__ ctot) {
  __shared__ uint32_t red[4];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  uint32_t s = 0;
  if (j < A.ns1)
    for (uint32_t g = t; g < A.ng; g += 256) {
      const size_t gj = (size_t)g * A.ns1 + j;
      if (A.o1[gj] < A.o1[gj + 1]) s += cend[gj] - cst[gj];
    }
  for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  if (t == 0) ctot[j] = red[0] + red[1] + red[2] + red[3];
}

// Projection: chunk j = virtual rows [j*seg1, (j+1)*seg1); its matches are output slots [cbase[j], cbase[j+1]).  The
// chunk is ordered FGW_SUB arrival rows at a time.  Every group's entries in the chunk are in arrival order, so a
// sub-chunk takes from each group the entries before the sub-chunk's end (found by binary search from the group's
// cursor); the groups' entry runs are concatenated and split evenly over the threads (contiguous blocks: coalesced
// count-word reads), a block scan gives every entry its compact-record position, and the counts are placed by arrival
// index in LDS, scanned, and the records written out contiguously.
struct FgwProjLds {
  uint32_t cnt[FGW_SUB];        // per arrival index in the sub-chunk: matches (0: none / a row of no group)
  uint32_t src[FGW_SUB];        // per arrival index: first compact record
  uint32_t wsum[4];
  uint32_t tot;
  // followed by gst[ng + 1], gnext[ng], gbase[ng] (dynamic)
};

template <class T>
__device__ __forceinline__ int64_t fgw_bits(uint32_t w) { return val_bits<T>(fgw_from32<T>(w)); }

template <class T>
__global__ void __launch_bounds__(256) k_fgw_proj(FgwArgs A, WalkArgs a, Virt v, ProjPlan pp, SgCols bc, SgCols cc,
                                                  const uint32_t* __restrict__ gm32, const PtU4* __restrict__ comp,
                                                  const uint32_t* __restrict__ cst, const uint32_t* __restrict__ cbase,
                                                  uint32_t* __restrict__ gcur, uint32_t* __restrict__ gsrc,
                                                  char* __restrict__ out, uint32_t* __restrict__ flags_out) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  FgwProjLds& P = *(FgwProjLds*)lds_raw;
  const uint32_t ng = A.ng;
  uint32_t* gst = (uint32_t*)(lds_raw + sizeof(FgwProjLds));
  uint32_t* gnext = gst + ng + 1;
  uint32_t* gbase = gnext + ng;
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  const int64_t r0 = (int64_t)j * A.seg1;
  const uint32_t rows = (uint32_t)min((int64_t)A.seg1, (int64_t)(v.nc + v.n) - r0);
  // per-group cursor and running compact position (global scratch [j][g]: the chunk's own slots)
  uint32_t* cur = gcur + (size_t)j * ng;
  uint32_t* srcp = gsrc + (size_t)j * ng;
  for (uint32_t g = t; g < ng; g += 256) {
    const size_t gj = (size_t)g * A.ns1 + j;
    cur[g] = A.o1[gj];
    srcp[g] = cst[gj];
  }
  uint32_t obase = cbase[j];
  const bool one = rows <= (uint32_t)FGW_SUB;
  for (uint32_t s0 = 0; s0 < rows; s0 += FGW_SUB) {
    const uint32_t sn = min((uint32_t)FGW_SUB, rows - s0);
    for (uint32_t i = t; i < sn; i += 256) P.cnt[i] = 0;
    __syncthreads();
    // 1. each group's entries of this sub-chunk: [cur, next)
    uint32_t mylen = 0;
    const uint32_t gpt = (ng + 255) / 256;        // groups per thread (contiguous)
    const uint32_t g0 = min(ng, t * gpt), g1 = min(ng, g0 + gpt);
    for (uint32_t g = g0; g < g1; ++g) {
      const size_t gj = (size_t)g * A.ns1 + j;
      const uint32_t c = cur[g], e = A.o1[gj + 1];
      uint32_t nx = e;
      if (!one) {   // first entry whose arrival index is past the sub-chunk
        uint32_t lo = c, hi = e;
        while (lo < hi) {
          const uint32_t mid = lo + ((hi - lo) >> 1);
          if ((gm32[mid] & 0xffffu) < s0 + sn) lo = mid + 1; else hi = mid;
        }
        nx = lo;
      }
      gnext[g] = nx;
      mylen += nx - c;
    }
    {
      const uint32_t ex = block_excl_scan256(mylen, P.wsum);
      uint32_t run = ex;
      for (uint32_t g = g0; g < g1; ++g) {
        gst[g] = run;
        run += gnext[g] - cur[g];
      }
      if (t == 255) gst[ng] = run;
    }
    __syncthreads();
    const uint32_t E = gst[ng];
    const uint32_t per = (E + 255) / 256;
    const uint32_t b0 = min(E, t * per), b1 = min(E, b0 + per);
    auto group_of = [&](uint32_t e) {
      uint32_t lo = 0, hi = ng;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gst[mid] <= e) lo = mid; else hi = mid;
      }
      return lo;
    };
    // 2. matches of each thread's block, block scan -> prefix of every entry over the concatenation
    uint32_t sm = 0;
    {
      uint32_t g = b0 < b1 ? group_of(b0) : 0;
      for (uint32_t e = b0; e < b1; ++e) {
        while (g + 1 < ng && gst[g + 1] <= e) ++g;
        sm += gm32[cur[g] + (e - gst[g])] >> 16;
      }
    }
    const uint32_t tx = block_excl_scan256(sm, P.wsum);
    // 3. the thread holding a group's first entry records gbase = (group's compact position) - (prefix there)
    {
      uint32_t g = b0 < b1 ? group_of(b0) : 0, run = tx;
      for (uint32_t e = b0; e < b1; ++e) {
        while (g + 1 < ng && gst[g + 1] <= e) ++g;
        if (e == gst[g]) gbase[g] = srcp[g] - run;
        run += gm32[cur[g] + (e - gst[g])] >> 16;
      }
    }
    __syncthreads();
    // 4. place counts and compact positions by arrival index; the last entry of a group advances its cursors
    {
      uint32_t g = b0 < b1 ? group_of(b0) : 0, run = tx;
      for (uint32_t e = b0; e < b1; ++e) {
        while (g + 1 < ng && gst[g + 1] <= e) ++g;
        const uint32_t wv = gm32[cur[g] + (e - gst[g])];
        const uint32_t m = wv >> 16, ai = wv & 0xffffu;
        if (ai < s0 || ai >= s0 + sn) {
          atomicOr(flags_out, FGW_F_INTERNAL);
        } else {
          P.cnt[ai - s0] = m;
          P.src[ai - s0] = gbase[g] + run;
        }
        run += m;
        if (e + 1 == gst[g + 1]) srcp[g] = gbase[g] + run;   // (the group's running position for the next sub-chunk)
      }
    }
    __syncthreads();
    for (uint32_t g = g0; g < g1; ++g) cur[g] = gnext[g];
    // 5. output offsets inside the sub-chunk (arrival order): each thread scans its block, then one lane per trigger,
    //    lanes on consecutive triggers -- every wave gathers 64 triggers' rows at once and writes their records to
    //    consecutive output slots
    const uint32_t per2 = (sn + 255) / 256;
    const uint32_t c0 = min(sn, t * per2), c1 = min(sn, c0 + per2);
    uint32_t sum = 0;
    for (uint32_t ai = c0; ai < c1; ++ai) sum += P.cnt[ai];
    uint32_t run = block_excl_scan256(sum, P.wsum);
    const uint32_t sub_tot = P.wsum[0] + P.wsum[1] + P.wsum[2] + P.wsum[3];
    for (uint32_t ai = c0; ai < c1; ++ai) {   // cnt[ai] <- output offset << 8 | matches (m < 256 checked)
      const uint32_t m = P.cnt[ai];
      if (m > 255u) atomicOr(flags_out, FGW_F_INTERNAL);
      P.cnt[ai] = (run << 8) | (m & 255u);
      run += m;
    }
    __syncthreads();
    for (uint32_t ai = t; ai < sn; ai += 256) {
      const uint32_t cw = P.cnt[ai];
      const uint32_t m = cw & 255u;
      if (!m) continue;
      const uint32_t slot0 = obase + (cw >> 8);
      const int64_t rv = r0 + s0 + ai;           // virtual row of the trigger
      const int64_t b = rv - v.nc;               // batch row
      if (b < 0) { atomicOr(flags_out, FGW_F_INTERNAL); continue; }
      const uint32_t key = a.partitioned ? (uint32_t)v.key[b] : 0u;
      const int64_t t2 = v.ts[b];
      const uint64_t trig = a.index ? a.index[b] : a.base_index + (uint64_t)b;
      const uint32_t sb = P.src[ai];
      for (uint32_t u = 0; u < m; ++u) {
        const PtU4 cr = comp[sb + u];
        int64_t* o = (int64_t*)(out + (size_t)(a.out_base + slot0 + u) * a.stride);
        uint32_t nm = 0;
        for (int s2 = 0; s2 < a.n_select; ++s2) {
          const bool src2 = pp.src[s2] != 0;
          const int kind = pp.kind[s2];
          int64_t bits = 0;
          if (kind == 0) {
            bits = v.pfloat ? (int64_t)cr.y : (int64_t)(int32_t)cr.y;
          } else if (kind == 1) {
            bits = src2 ? val_bits<T>(v_val<T>(v, (uint32_t)rv, v.val_a == v.val_b)) : fgw_bits<T>(cr.x);
          } else if (kind == 2) {
            nm |= 1u << s2;
          } else {
            const uint32_t rr = src2 ? (uint32_t)rv : cr.z;
            SgVal x = rr < v.nc ? sg_read_col(cc, pp.col[s2], pp.type[s2], rr) : sg_read_col(bc, pp.col[s2], pp.type[s2], rr - v.nc);
            if (x.null) nm |= 1u << s2;
            bits = sg_val_bits(x);
          }
          o[4 + s2] = bits;
        }
        o[0] = (int64_t)trig;
        o[1] = t2;
        o[2] = (int64_t)((uint64_t)key | ((uint64_t)((1u << 24) | (a.multi ? (uint32_t)a.b_slot : (0x800000u | u))) << 32));
        o[3] = (int64_t)nm;
      }
    }
    obase += sub_tot;
    __syncthreads();
  }
}

// Carry: per key, the end state of the segment holding its last row of the push (the largest segment with a record)
static __global__ void k_fgw_carry_count(uint32_t Kp, uint32_t nsw, const uint32_t* __restrict__ kcnt, uint32_t* __restrict__ cn,
                                  uint32_t* __restrict__ cseg) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > Kp) return;
  uint32_t c = 0, sj = FGW_NONE;
  if (k < Kp)
    for (int jj = (int)nsw - 1; jj >= 0; --jj) {
      const uint32_t x = kcnt[(size_t)jj * Kp + k];
      if (x != FGW_NONE) { c = x & 0xffffffu; sj = (uint32_t)jj; break; }
    }
  cn[k] = c;
  if (k < Kp) cseg[k] = sj;
}

template <class T>
__global__ void k_fgw_carry_copy(Virt v, uint32_t Kp, uint32_t cap1, const uint32_t* __restrict__ cseg,
                                 const uint32_t* __restrict__ coff, const uint32_t* __restrict__ kent, int n_cols,
                                 const int32_t* __restrict__ widths, SgCols bc, SgCols cc, CarryBufs dst) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Kp || cseg[k] == FGW_NONE) return;
  const uint32_t c = coff[k + 1] - coff[k];
  const uint32_t* src = kent + ((size_t)cseg[k] * Kp + k) * cap1;
  for (uint32_t e = 0; e < c; ++e) {
    const uint32_t r = src[e];
    const uint32_t d = coff[k] + e;
    dst.ts[d] = v_ts(v, r);
    dst.key[d] = (int32_t)k;
    dst.flags[d] = (uint8_t)v_flags(v, r);
    const SgCols& s = r < v.nc ? cc : bc;
    const uint32_t rr = r < v.nc ? r : (uint32_t)(r - v.nc);
    for (int q = 0; q < n_cols; ++q) {
      if (!s.col[q]) continue;
      if (widths[q] == 8) ((int64_t*)dst.col[q])[d] = ((const int64_t*)s.col[q])[rr];
      else ((int32_t*)dst.col[q])[d] = ((const int32_t*)s.col[q])[rr];
      dst.nul[q][d] = s.nul[q] ? s.nul[q][rr] : 0;
    }
  }
}

// ---- more than 256 key groups (C5's 1M keys): the group domain in two passes.  Pass 1a groups rows by supergroup
// (k_part1 with 32-bit staged keys and 16-bit in-supergroup keys); pass 1b splits each supergroup into its groups,
// arrival order kept, straight into the group-domain positions of the per-(group, segment) histogram (o1).

// per part1 segment j: rows of each group g -> h[g * ns1 + j] (up to 4096 groups, LDS counters)
static __global__ void __launch_bounds__(256) k_hist_wide(KeyOf kf, uint32_t K, uint32_t lb, uint32_t ng, uint32_t seg1,
                                                          uint32_t ns1, int64_t nt, uint32_t* __restrict__ h,
                                                          uint32_t* __restrict__ flags) {
  __shared__ uint32_t cnt[4096];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  for (uint32_t g = t; g < ng; g += 256) cnt[g] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)j * seg1, r1 = min(nt, r0 + seg1);
  uint32_t bad = 0;
  for (int64_t r = r0 + t; r < r1; r += 256) {
    const uint32_t k = kf((uint32_t)r);
    if (k < K) atomicAdd(&cnt[k >> lb], 1u);
    else if (k != 0xffffffffu) bad |= PK_KEY_RANGE;
  }
  __syncthreads();
  for (uint32_t g = t; g < ng; g += 256) h[(size_t)g * ns1 + j] = cnt[g];
  if (bad) atomicOr(flags, bad);
}

struct Part1bArgs {
  uint32_t lb;          // in-group key bits
  uint32_t lbs;         // group bits inside a supergroup
  uint32_t ns1, tsb;    // part1 segments; per pass-1b segment
  uint32_t nsb;         // pass-1b segments per supergroup
  const uint32_t* oa;   // pass-1a offsets [sg * ns1 + j]
  const uint32_t* o1;   // group-domain offsets [g * ns1 + j]
};

template <int PT>
struct Part1bLds {
  PtU4 stage[256 * PT];
  uint16_t tag[256 * PT];
  uint32_t cw[4][256];
  uint32_t ls[256], tot[256], run[256];
  uint32_t wsum[4];
};

template <int PT>
__global__ void __launch_bounds__(256) k_part1b(Part1bArgs B, const PtU4* __restrict__ grecA, const uint16_t* __restrict__ glkA,
                                                PtU4* __restrict__ grec, uint8_t* __restrict__ glk, uint32_t cap,
                                                uint32_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  Part1bLds<PT>& L = *(Part1bLds<PT>*)lds_raw;
  const uint32_t sg = blockIdx.x / B.nsb, jj = blockIdx.x % B.nsb;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t jf = min(B.ns1, jj * B.tsb), jl = min(B.ns1, jf + B.tsb);
  const uint32_t lo = B.oa[(size_t)sg * B.ns1 + jf], hi = B.oa[(size_t)sg * B.ns1 + jl];
  const uint32_t nd = 1u << B.lbs, lmask = (1u << B.lb) - 1u;
  if (t < nd) L.run[t] = B.o1[(size_t)((sg << B.lbs) | t) * B.ns1 + jf];
  const int ROWS = 256 * PT;
  auto load = [&](uint32_t base, PtU4* rc, uint32_t* tg) {
    const uint32_t rows = min((uint32_t)ROWS, hi - base);
#pragma unroll
    for (int s = 0; s < PT; ++s) {
      const uint32_t i = w * (PT * 64) + s * 64 + lane;
      const uint32_t p = base + (i < rows ? i : rows - 1);
      rc[s] = grecA[p];
      const uint32_t k = glkA[p];
      tg[s] = i < rows ? k : 0xffffffffu;
    }
  };
  PtU4 rc[PT], rn[PT];
  uint32_t tg[PT], tn[PT];
  if (lo < hi) load(lo, rc, tg);
  for (uint32_t base = lo; base < hi; base += ROWS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) L.cw[q][t] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PT; ++s)
      if (tg[s] != 0xffffffffu) atomicAdd(&L.cw[w][tg[s] >> B.lb], 1u);
    __syncthreads();
    uint32_t staged;
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
      __syncthreads();
      staged = L.ls[255] + L.tot[255];
    }
#pragma unroll
    for (int s = 0; s < PT; ++s) {
      const bool valid = tg[s] != 0xffffffffu;
      const uint32_t d = valid ? tg[s] >> B.lb : 0u;
      uint32_t rank, cnt;
      peer_rank(valid, d, B.lbs, rank, cnt);
      if (valid) {
        const uint32_t slot = L.cw[w][d] + rank;
        if (rank == 0) L.cw[w][d] = slot + cnt;
        L.stage[slot] = rc[s];
        L.tag[slot] = (uint16_t)tg[s];
      }
    }
    if (base + ROWS < hi) load(base + ROWS, rn, tn);
    __syncthreads();
    for (uint32_t q = t; q < staged; q += 256) {
      const uint32_t k = L.tag[q], d = k >> B.lb;
      const uint32_t dst = L.run[d] + q - L.ls[d];
      if (dst >= cap) { atomicOr(flags, PK_INTERNAL); continue; }
      grec[dst] = L.stage[q];
      glk[dst] = (uint8_t)(k & lmask);
    }
    __syncthreads();
    if (t < nd) L.run[t] += L.tot[t];
#pragma unroll
    for (int s = 0; s < PT; ++s) { rc[s] = rn[s]; tg[s] = tn[s]; }
  }
}
