#pragma once
// part_wide.h -- pass 1 of the closed form's LDS key partition beyond 256 key groups (engine_impl.h part1_wide).
#include <hip/hip_runtime.h>

// ---- more than 256 key groups (C5's 1M keys): the group domain in two passes.  Pass 1a groups rows by supergroup
// (k_part1 with 32-bit staged keys and 16-bit in-supergroup keys); pass 1b splits each supergroup into its groups,
// arrival order kept, straight into the group-domain positions of the per-(group, segment) histogram (o1).

// per part1 segment j: rows of each group g -> h[g * ns1 + j] (up to 4096 groups, LDS counters), and of each
// supergroup (2^lbs consecutive groups) -> ha[sg * ns1 + j] from the same counters (one pass over the keys)
static __global__ void __launch_bounds__(256) k_hist_wide(KeyOf kf, uint32_t K, uint32_t lb, uint32_t ng, uint32_t seg1,
                                                          uint32_t ns1, int64_t nt, uint32_t* __restrict__ h,
                                                          uint32_t lbs, uint32_t nsg, uint32_t* __restrict__ ha,
                                                          uint32_t* __restrict__ flags) {
  __shared__ uint32_t cnt[4096];
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  for (uint32_t g = t; g < ng; g += 256) cnt[g] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)j * seg1, r1 = min(nt, r0 + seg1);
  uint32_t bad = 0;
  for (int64_t rb = r0; rb < r1; rb += 256 * 8) {   // eight rows per thread in flight
    uint32_t k[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t r = rb + s * 256 + t;
      k[s] = r < r1 ? kf((uint32_t)r) : 0xffffffffu;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (k[s] < K) atomicAdd(&cnt[k[s] >> lb], 1u);
      else if (k[s] != 0xffffffffu) bad |= PK_KEY_RANGE;
    }
  }
  __syncthreads();
  for (uint32_t g = t; g < ng; g += 256) h[(size_t)g * ns1 + j] = cnt[g];
  for (uint32_t sg = t; sg < nsg; sg += 256) {
    uint32_t c = 0;
    for (uint32_t g = sg << lbs; g < ((sg + 1) << lbs) && g < ng; ++g) c += cnt[g];
    ha[(size_t)sg * ns1 + j] = c;
  }
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
