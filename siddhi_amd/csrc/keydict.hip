// Device key dictionary (see keydict.h).
#include "keydict.h"

#include <cstring>
#include <rocprim/rocprim.hpp>

#include <string>

#include "sg_engine.h"

#define KDCHK(x)                                                                                       \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string("keydict: " #x ": ") + hipGetErrorString(e_)); \
  } while (0)

namespace {

const int64_t KD_EMPTY = (int64_t)0x8000000000000000ull;
const int32_t KD_UNUSED = (int32_t)0x80000000u;
const int KD_BLOCK = 256;
const int KD_MAX_BLOCKS = 1024;              // at most 256K probing threads: claims overshoot the limit by <= that
const int64_t KD_MIN_CAP = (int64_t)1 << 22;  // 4M slots (48 MB): a million keys without a rebuild

struct KdView {
  int64_t* keys;
  int32_t* vals;
  uint32_t* first;
  int32_t* nslot;
  uint64_t mask;
  int32_t shift;
  int64_t cap, limit, n_keys, list_cap;
};

__device__ __forceinline__ uint64_t kd_home(int64_t k, int shift) {   // Fibonacci hashing
  return ((uint64_t)k * 0x9E3779B97F4A7C15ull) >> shift;
}

__device__ __forceinline__ void kd_claimed(const KdView& t, uint32_t* ctr, int64_t h) {
  const uint32_t q = atomicAdd(ctr, 1u);
  if ((int64_t)q < t.list_cap) t.nslot[q] = (int32_t)h;
  else atomicOr(ctr + 1, 2u);
}

__device__ __forceinline__ bool kd_room(const KdView& t, uint32_t* ctr) {
  const uint32_t c = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((int64_t)c + t.n_keys < t.limit) return true;
  atomicOr(ctr + 1, 1u);
  return false;
}

__global__ void __launch_bounds__(KD_BLOCK) k_kd_probe(KdView t, const int64_t* __restrict__ raw,
                                                       const int32_t* __restrict__ stream, int64_t n,
                                                       int32_t* __restrict__ key, uint32_t* ctr) {
  for (int64_t i = (int64_t)blockIdx.x * KD_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * KD_BLOCK) {
    if (stream && stream[i] < 0) {   // clock-only row: no key
      key[i] = -1;
      continue;
    }
    const int64_t k = raw[i];
    int32_t out = -3;
    if (k == KD_EMPTY) {   // the sentinel value itself lives in the extra slot, claimed through its value word
      const int64_t h = t.cap;
      int32_t v = __hip_atomic_load(&t.vals[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= 0) {
        out = v;
      } else {
        bool ok = true;
        if (v == KD_UNUSED) {
          if (kd_room(t, ctr)) {
            if (atomicCAS(&t.vals[h], KD_UNUSED, -1) == KD_UNUSED) kd_claimed(t, ctr, h);
          } else {
            ok = __hip_atomic_load(&t.vals[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != KD_UNUSED;
          }
        }
        if (ok) {
          atomicMin(&t.first[h], (uint32_t)i);
          out = -2;
        }
      }
    } else {
      uint64_t h = kd_home(k, t.shift);
      while (true) {
        const int64_t kk = t.keys[h];   // (a stale EMPTY is corrected by the CAS below)
        if (kk == k) {
          const int32_t v = t.vals[h];
          if (v >= 0) out = v;
          else {
            atomicMin(&t.first[h], (uint32_t)i);
            out = -2;
          }
          break;
        }
        if (kk == KD_EMPTY) {
          if (!kd_room(t, ctr)) break;   // out = -3: the table is rebuilt and the chunk probed again
          const unsigned long long old =
              atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)KD_EMPTY, (unsigned long long)k);
          if (old == (unsigned long long)KD_EMPTY) {
            atomicMin(&t.first[h], (uint32_t)i);
            kd_claimed(t, ctr, (int64_t)h);
            out = -2;
            break;
          }
          if ((int64_t)old == k) {
            atomicMin(&t.first[h], (uint32_t)i);
            out = -2;
            break;
          }
        }
        h = (h + 1) & t.mask;
      }
    }
    key[i] = out;
  }
}

__global__ void k_kd_gather(const int32_t* __restrict__ nslot, const uint32_t* __restrict__ first, int64_t m,
                            uint32_t* __restrict__ nfirst) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < m) nfirst[q] = first[nslot[q]];
}

__global__ void k_kd_assign(const int32_t* __restrict__ sslot, int64_t m, int64_t base, int32_t* __restrict__ vals) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < m) vals[sslot[r]] = (int32_t)(base + r);
}

__global__ void __launch_bounds__(KD_BLOCK) k_kd_fill(KdView t, const int64_t* __restrict__ raw, int64_t n,
                                                      int32_t* __restrict__ key) {
  for (int64_t i = (int64_t)blockIdx.x * KD_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * KD_BLOCK) {
    if (key[i] != -2) continue;
    const int64_t k = raw[i];
    if (k == KD_EMPTY) {
      key[i] = t.vals[t.cap];
      continue;
    }
    uint64_t h = kd_home(k, t.shift);
    while (t.keys[h] != k) h = (h + 1) & t.mask;
    key[i] = t.vals[h];
  }
}

__global__ void k_kd_clear(int64_t* __restrict__ keys, int32_t* __restrict__ vals, uint32_t* __restrict__ first,
                           int64_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cap; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = KD_EMPTY;
    vals[i] = i == cap ? KD_UNUSED : -1;
    first[i] = 0xffffffffu;
  }
}

// old table's assigned keys -> the new (cleared) table; pending claims are dropped
__global__ void k_kd_rehash(const int64_t* __restrict__ okeys, const int32_t* __restrict__ ovals, int64_t ocap,
                            KdView t) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= ocap; j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t v = ovals[j];
    if (v < 0) continue;
    if (j == ocap) {
      t.vals[t.cap] = v;
      continue;
    }
    const int64_t k = okeys[j];
    uint64_t h = kd_home(k, t.shift);
    while (atomicCAS((unsigned long long*)&t.keys[h], (unsigned long long)KD_EMPTY, (unsigned long long)k) !=
           (unsigned long long)KD_EMPTY)
      h = (h + 1) & t.mask;
    t.vals[h] = v;
  }
}

int log2i(int64_t x) {
  int s = 0;
  while (((int64_t)1 << s) < x) ++s;
  return s;
}

KdView view(const KeyDict& t) {
  KdView v;
  v.keys = t.keys;
  v.vals = t.vals;
  v.first = t.first;
  v.nslot = t.nslot;
  v.cap = t.cap;
  v.mask = (uint64_t)t.cap - 1;
  v.shift = 64 - log2i(t.cap);
  v.limit = t.cap / 2;
  v.n_keys = t.n_keys;
  v.list_cap = t.list_cap;
  return v;
}

unsigned grid_for(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(KD_MAX_BLOCKS, (n + KD_BLOCK - 1) / KD_BLOCK));
}

void alloc_table(KeyDict& t, int64_t cap, hipStream_t st) {
  KDCHK(hipMalloc((void**)&t.keys, sizeof(int64_t) * (cap + 1)));
  KDCHK(hipMalloc((void**)&t.vals, sizeof(int32_t) * (cap + 1)));
  KDCHK(hipMalloc((void**)&t.first, sizeof(uint32_t) * (cap + 1)));
  t.cap = cap;
  hipLaunchKernelGGL(k_kd_clear, dim3(grid_for(cap + 1)), dim3(KD_BLOCK), 0, st, t.keys, t.vals, t.first, cap);
  KDCHK(hipGetLastError());
}

void free_table(KeyDict& t, hipStream_t st) {
  KDCHK(hipStreamSynchronize(st));
  if (t.keys) KDCHK(hipFree(t.keys));
  if (t.vals) KDCHK(hipFree(t.vals));
  if (t.first) KDCHK(hipFree(t.first));
  t.keys = nullptr;
  t.vals = nullptr;
  t.first = nullptr;
}

void ensure_lists(KeyDict& t, int64_t m, hipStream_t st) {
  if (m <= t.list_cap) return;
  KDCHK(hipStreamSynchronize(st));
  for (void* p : {(void*)t.nslot, (void*)t.nfirst, (void*)t.sslot, (void*)t.sfirst})
    if (p) KDCHK(hipFree(p));
  KDCHK(hipMalloc((void**)&t.nslot, sizeof(int32_t) * m));
  KDCHK(hipMalloc((void**)&t.nfirst, sizeof(uint32_t) * m));
  KDCHK(hipMalloc((void**)&t.sslot, sizeof(int32_t) * m));
  KDCHK(hipMalloc((void**)&t.sfirst, sizeof(uint32_t) * m));
  t.list_cap = m;
}

// a 4x larger table holding the assigned keys of the current one
void rebuild(KeyDict& t, int64_t cap, hipStream_t st) {
  KeyDict nt;
  alloc_table(nt, cap, st);
  nt.n_keys = t.n_keys;
  hipLaunchKernelGGL(k_kd_rehash, dim3(grid_for(t.cap + 1)), dim3(KD_BLOCK), 0, st, t.keys, t.vals, t.cap, view(nt));
  KDCHK(hipGetLastError());
  free_table(t, st);
  t.keys = nt.keys;
  t.vals = nt.vals;
  t.first = nt.first;
  t.cap = cap;
  ensure_lists(t, cap / 2 + (int64_t)KD_MAX_BLOCKS * KD_BLOCK, st);
  ++t.rebuilds;
}

}  // namespace

int64_t kd_resolve(KeyDict& t, const int64_t* raw, const int32_t* stream, int64_t n, int32_t* key, hipStream_t st,
                   std::vector<uint32_t>* new_first) {
  if (n <= 0) return 0;
  if (n >= ((int64_t)1 << 32) - 1) throw SgError(SG_EINVAL, "keydict: chunk too large");
  if (!t.ctr) {
    KDCHK(hipMalloc((void**)&t.ctr, 2 * sizeof(uint32_t)));
    KDCHK(hipHostMalloc((void**)&t.hctr, 2 * sizeof(uint32_t), hipHostMallocDefault));
  }
  if (!t.keys || t.clear) {
    if (!t.keys) alloc_table(t, KD_MIN_CAP, st);
    else hipLaunchKernelGGL(k_kd_clear, dim3(grid_for(t.cap + 1)), dim3(KD_BLOCK), 0, st, t.keys, t.vals, t.first,
                            t.cap);
    KDCHK(hipGetLastError());
    ensure_lists(t, t.cap / 2 + (int64_t)KD_MAX_BLOCKS * KD_BLOCK, st);
    t.n_keys = 0;
    t.clear = false;
  }
  int64_t m = 0;
  while (true) {
    KDCHK(hipMemsetAsync(t.ctr, 0, 2 * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_kd_probe, dim3(grid_for(n)), dim3(KD_BLOCK), 0, st, view(t), raw, stream, n, key, t.ctr);
    KDCHK(hipGetLastError());
    KDCHK(hipMemcpyAsync(t.hctr, t.ctr, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    KDCHK(hipStreamSynchronize(st));
    ++t.probes;
    if (t.hctr[1] == 0) {
      m = t.hctr[0];
      break;
    }
    if (t.n_keys + n > ((int64_t)1 << 31) - 2) throw SgError(SG_ECAPACITY, "keydict: more than 2^31 keys");
    rebuild(t, t.cap * 4, st);
  }
  if (m == 0) return 0;
  const unsigned g = (unsigned)((m + 255) / 256);
  hipLaunchKernelGGL(k_kd_gather, dim3(g), dim3(256), 0, st, t.nslot, t.first, m, t.nfirst);
  size_t tb = 0;
  KDCHK(rocprim::radix_sort_pairs(nullptr, tb, t.nfirst, t.sfirst, t.nslot, t.sslot, (size_t)m, 0, 32, st));
  if (tb > t.tmp_bytes) {
    KDCHK(hipStreamSynchronize(st));
    if (t.tmp) KDCHK(hipFree(t.tmp));
    KDCHK(hipMalloc(&t.tmp, tb));
    t.tmp_bytes = tb;
  }
  KDCHK(rocprim::radix_sort_pairs(t.tmp, tb, t.nfirst, t.sfirst, t.nslot, t.sslot, (size_t)m, 0, 32, st));
  hipLaunchKernelGGL(k_kd_assign, dim3(g), dim3(256), 0, st, t.sslot, m, t.n_keys, t.vals);
  hipLaunchKernelGGL(k_kd_fill, dim3(grid_for(n)), dim3(KD_BLOCK), 0, st, view(t), raw, n, key);
  KDCHK(hipGetLastError());
  if (new_first) {
    new_first->resize((size_t)m);
    KDCHK(hipMemcpyAsync(new_first->data(), t.sfirst, sizeof(uint32_t) * m, hipMemcpyDeviceToHost, st));
    KDCHK(hipStreamSynchronize(st));
  }
  t.n_keys += m;
  return m;
}

void kd_reset(KeyDict& t) {
  t.clear = true;
  t.n_keys = 0;
}

void kd_free(KeyDict& t) {
  for (void* p : {(void*)t.keys, (void*)t.vals, (void*)t.first, (void*)t.nslot, (void*)t.nfirst, (void*)t.sslot,
                  (void*)t.sfirst, t.tmp, (void*)t.ctr})
    if (p) hipFree(p);
  if (t.hctr) hipHostFree(t.hctr);
  t = KeyDict();
}
