// absent.hip — MI355X closed form for  every A[l] -> not B[l' and B.x == A.x] for W   (@app:playback,
// unpartitioned; SG_SHAPE_EVERY_ABSENT_EQ, config C4).
//
// Semantics, restated from AbsentStreamPreStateProcessor (C/query/input/stream/state/
// AbsentStreamPreStateProcessor.java: addState :77-101 schedules ts_i + W, the timer pass :140-228 emits
// every pending partial with S.ts + W <= T stamped S.ts = T, processAndReturn :230-244 drops a partial
// whose `not` filter matched), AbsentStreamPostStateProcessor.process (:36-56) and Scheduler's FIFO
// (C/util/Scheduler.java:74-86,179-214) driven by TimestampGeneratorImpl.setCurrentTimestamp
// (C/util/timestamp/TimestampGeneratorImpl.java:106-125) before each row is dispatched:
//   every A row i passing A's filter opens partial i with deadline d_i = ts_i + W; the partial is
//   KILLED iff some later B row j passing B's local filter with x_j == x_i arrives with ts_j < d_i;
//   otherwise it is EMITTED in the timer pass that runs just before the first row (any stream) with
//   ts >= d_i, with output ts = d_i.  Every FIFO entry is "row ts + W" pushed in row order, so the
//   FIFO stays sorted and the timer-pass epilogue never schedules; emissions are therefore ordered by
//   deadline then arrival, i.e. by i, and the g-th emission of one timer pass is callback group g.
//
// Pipeline per sg_push (one HIP stream, inputs in HBM):
//   1. k_abs_rows     per virtual row (carried partials first): candidate / killer roles (A and B local
//                     predicates through the postfix VM), the compared value, a min/max of the values
//                     and the timestamp-order check.
//   2. sort           stable radix sort of the virtual rows by compared value (rocPRIM, only the bits
//                     the value range needs): per value, its rows in arrival order.
//   3. next killer    reverse min-scan over sorted positions -> the first killer after each position.
//   4. k_abs_decide   per candidate: killed (first later killer of the same value is before d_i),
//                     emitted (trigger = first row with ts >= d_i, binary search) or still pending.
//   5. scan           emission and carry offsets in arrival order.
//   6. k_abs_write    AoS match records (QuerySelector.processNoGroupBy projection of e1's attributes),
//                     callback group = rank within the trigger's timer pass; carried partials saved.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>

#include "sg_device.h"
#include "sg_engine.h"

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) throw SgError(SG_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace {

const uint32_t R_CAND = 1, R_KILL = 2, R_SORT = 4;   // role bits
const uint32_t NONE = 0xffffffffu;

// Pending partials carried into the next push (arrival order): deadline, compared value, projection.
struct AbsCarry {
  int64_t n = 0, cap = 0;
  int64_t* dl = nullptr;       // deadline ts_i + W
  int64_t* val = nullptr;      // compared value bits
  uint8_t* vnul = nullptr;     // compared value is null (never killed)
  int64_t* sel = nullptr;      // [cap][n_select] projected bits
  uint32_t* snul = nullptr;    // projected null mask
  void reserve(int64_t want, int nsel) {
    if (want <= cap) return;
    release();
    cap = std::max<int64_t>(want + want / 4, 1024);
    if (hipMalloc(&dl, cap * 8) != hipSuccess || hipMalloc(&val, cap * 8) != hipSuccess ||
        hipMalloc(&vnul, cap) != hipSuccess || hipMalloc(&sel, cap * 8 * std::max(nsel, 1)) != hipSuccess ||
        hipMalloc(&snul, cap * 4) != hipSuccess)
      throw SgError(SG_EHIP, "hipMalloc failed for absence carry");
  }
  void release() {
    for (void* p : {(void*)dl, (void*)val, (void*)vnul, (void*)sel, (void*)snul}) if (p) hipFree(p);
    dl = val = sel = nullptr;
    vnul = nullptr;
    snul = nullptr;
    cap = 0;
  }
};

// The Scheduler's FIFO (C/util/Scheduler.java:49, a LinkedBlockingQueue) as carried between pushes: entries not yet
// popped, in queue order.
struct AbsQueue {
  int64_t n = 0, cap = 0;
  int64_t* v = nullptr;
  void reserve(int64_t want) {
    if (want <= cap) return;
    int64_t* nv = nullptr;
    const int64_t c = std::max<int64_t>(want + want / 4, 1024);
    if (hipMalloc(&nv, c * 8) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc failed for the absence timer queue");
    if (v) hipFree(v);
    v = nv;
    cap = c;
  }
  void release() { if (v) hipFree(v); v = nullptr; n = cap = 0; }
};

struct AbsState {
  AbsCarry carry[2];
  AbsQueue q[2];               // timer FIFO (with carry[cur]: q[cur])
  int cur = 0;
  int64_t lst = 0;             // AbsentStreamPreStateProcessor.lastScheduledTime (Java default 0)
  bool seq = false;            // the state is not the closed form's: the next push runs the exact sequential pass
  int64_t* dlast = nullptr;    // device: the playback clock (largest timestamp seen; order check across pushes)
  int64_t* dminmax = nullptr;  // device: [min, max] of compared values (as order-preserving u64)
  uint32_t* dflag = nullptr;   // device: the push's first row whose time goes back (0xffffffff: none)
};

struct AbsArgs {
  int64_t n, nc, nt;
  int64_t W;
  int32_t s_a, s_b;
  int32_t col_a, col_b, type;
  int32_t prog_a_off, prog_a_len, prog_b_off, prog_b_len;
  int32_t has_stream;
  int32_t first_push;
  int32_t keep_carry;          // 0 (no_carry): partials still pending at the end of the push are dropped
  int32_t fast;                // one stream, no local filters, no stream column, no nulls: every row is
                               // candidate and killer (the C4 shape)
};

struct RowRd {
  const SgCols* c;
  const int32_t* ret_col;
  int64_t row;
  __device__ SgVal read(int, int, int slot, int type) { return sg_read_col(*c, ret_col[slot], type, row); }
};

__device__ __forceinline__ uint64_t ord64(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

// value range: wave shuffles, then LDS across the block's waves, then ONE atomic pair per block (a pair
// per wave on two global words serialises in L2: measured 0.39 ms for 10M rows)
__device__ __forceinline__ void block_minmax(uint64_t lo, uint64_t hi, unsigned long long* __restrict__ minmax) {
  __shared__ uint64_t slo[4], shi[4];
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { slo[w] = lo; shi[w] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      lo = slo[k] < lo ? slo[k] : lo;
      hi = shi[k] > hi ? shi[k] : hi;
    }
    if (lo != ~0ull) {
      atomicMin(&minmax[0], (unsigned long long)lo);
      atomicMax(&minmax[1], (unsigned long long)hi);
    }
  }
}

// 1. roles, compared values, value range, order check
__global__ void __launch_bounds__(256) k_abs_rows(AbsArgs a, SgCols cols, const DevDesc* __restrict__ dd,
                                                  const int64_t* __restrict__ ts, const int32_t* __restrict__ stream,
                                                  const int64_t* __restrict__ c_val, const uint8_t* __restrict__ c_vnul,
                                                  uint8_t* __restrict__ role, int64_t* __restrict__ vals,
                                                  unsigned long long* __restrict__ minmax, const int64_t* __restrict__ dlast,
                                                  uint32_t* __restrict__ oflag) {
  uint64_t lo = ~0ull, hi = 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.nt; v += (int64_t)gridDim.x * blockDim.x) {
    uint32_t r = 0;
    int64_t x = 0;
    if (v < a.nc) {
      r = R_CAND;
      if (!c_vnul[v]) { r |= R_SORT; x = c_val[v]; }
    } else {
      const int64_t i = v - a.nc;
      const int s = a.has_stream ? stream[i] : 0;
      RowRd rd{&cols, dd->ret_col, i};
      bool ca = s == a.s_a && sg_eval(dd->code + a.prog_a_off, a.prog_a_len, rd);
      bool ki = s == a.s_b && sg_eval(dd->code + a.prog_b_off, a.prog_b_len, rd);
      const int col = ca ? a.col_a : a.col_b;   // same column when A and B read one stream (checked on host)
      if (ca || ki) {
        SgVal sv = sg_read_col(cols, col, a.type, i);
        if (!sv.null) { x = sv.i; r |= R_SORT; }
        if (ca) r |= R_CAND;
        if (ki && !sv.null) r |= R_KILL;   // `==` with a null operand is false
      }
      if ((i > 0 && ts[i - 1] > ts[i]) || (i == 0 && !a.first_push && ts[0] < *dlast)) atomicMin(oflag, (uint32_t)i);
    }
    role[v] = (uint8_t)r;
    vals[v] = x;
    if (r & R_SORT) {
      uint64_t o = ord64(x);
      lo = o < lo ? o : lo;
      hi = o > hi ? o : hi;
    }
  }
  block_minmax(lo, hi, minmax);
}

// 1'. the C4 shape (one stream, no local filters, no nulls): every row is candidate and killer; no VM
// (the VM's operand stack would cost this streaming pass its occupancy)
template <class V>
__global__ void __launch_bounds__(256) k_abs_rows_fast(AbsArgs a, const V* __restrict__ col, const int64_t* __restrict__ ts,
                                                       const int64_t* __restrict__ c_val, const uint8_t* __restrict__ c_vnul,
                                                       uint8_t* __restrict__ role, int64_t* __restrict__ vals,
                                                       unsigned long long* __restrict__ minmax,
                                                       const int64_t* __restrict__ dlast, uint32_t* __restrict__ oflag) {
  uint64_t lo = ~0ull, hi = 0;
  uint32_t late = 0xffffffffu;   // first row whose time goes back
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.nt; v += (int64_t)gridDim.x * blockDim.x) {
    uint32_t r;
    int64_t x = 0;
    if (v < a.nc) {
      r = R_CAND;
      if (!c_vnul[v]) { r |= R_SORT; x = c_val[v]; }
    } else {
      const int64_t i = v - a.nc;
      x = (int64_t)col[i];
      r = R_CAND | R_KILL | R_SORT;
      const int64_t t = ts[i];
      if (((i > 0 && ts[i - 1] > t) || (i == 0 && !a.first_push && t < *dlast)) && (uint32_t)i < late) late = (uint32_t)i;
    }
    role[v] = (uint8_t)r;
    vals[v] = x;
    if (r & R_SORT) {
      uint64_t o = ord64(x);
      lo = o < lo ? o : lo;
      hi = o > hi ? o : hi;
    }
  }
  if (late != 0xffffffffu) atomicMin(oflag, late);
  block_minmax(lo, hi, minmax);
}

// sort keys: value - min (order preserving) for sorted rows, a sentinel above the range for the rest
template <class K>
__global__ void k_abs_keys(int64_t nt, const uint8_t* __restrict__ role, const int64_t* __restrict__ vals,
                           uint64_t omin, K sentinel, K* __restrict__ keys, uint32_t* __restrict__ ids) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nt; v += (int64_t)gridDim.x * blockDim.x) {
    keys[v] = (role[v] & R_SORT) ? (K)(ord64(vals[v]) - omin) : sentinel;
    ids[v] = (uint32_t)v;
  }
}

// 3. reversed killer positions (input of the min-scan): rk[nt-1-p] = p if sorted position p is a killer
__global__ void k_abs_rkill(int64_t nt, const uint32_t* __restrict__ sid, const uint8_t* __restrict__ role,
                            uint32_t* __restrict__ rk) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nt; p += (int64_t)gridDim.x * blockDim.x)
    rk[nt - 1 - p] = (role[sid[p]] & R_KILL) ? (uint32_t)p : NONE;
}

__device__ __forceinline__ int64_t vts(const AbsArgs& a, const int64_t* ts, const int64_t* c_dl, uint32_t v) {
  return v < a.nc ? c_dl[v] - a.W : ts[v - a.nc];
}

// 4a. kill: a candidate at sorted position p dies if the first killer after it has its value and arrives
//     before its deadline
template <class K>
__global__ void k_abs_kill(AbsArgs a, const K* __restrict__ skeys, const uint32_t* __restrict__ sid,
                           const uint8_t* __restrict__ role, const uint32_t* __restrict__ nks,
                           const int64_t* __restrict__ ts, const int64_t* __restrict__ c_dl,
                           uint8_t* __restrict__ dead, uint32_t* __restrict__ kc) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.nt; p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = sid[p];
    const uint8_t r = role[v];
    if ((r & (R_CAND | R_SORT)) != (R_CAND | R_SORT)) continue;
    uint32_t q = NONE;
    if (a.fast) {
      for (int64_t x = p + 1; x < a.nt && skeys[x] == skeys[p]; ++x)
        if (sid[x] >= a.nc) { q = (uint32_t)x; break; }
    } else if (p + 1 < a.nt) {
      q = nks[a.nt - 2 - p];   // min killer position >= p + 1
    }
    if (q == NONE || skeys[q] != skeys[p]) continue;
    const uint32_t vq = sid[q];
    if (vts(a, ts, c_dl, vq) < vts(a, ts, c_dl, v) + a.W) {
      dead[v] = 1;
      atomicAdd(&kc[vq - a.nc], 1u);   // (the killer's FIFO entries: one per partial it kills)
    }
  }
}

// 4a'. kill, fast shape (every batch row kills, every sorted row is a candidate; non-sorted rows carry the sentinel
//      key): the first killer after p is almost always p + 1, so its key, row and timestamp come from the next lane
//      instead of a second random read of the row arrays; only a carried neighbour (not a killer) makes the lane search
template <class K>
__global__ void __launch_bounds__(256) k_abs_kill_fast(AbsArgs a, const K* __restrict__ skeys,
                                                       const uint32_t* __restrict__ sid, K sentinel,
                                                       const int64_t* __restrict__ ts, const int64_t* __restrict__ c_dl,
                                                       uint8_t* __restrict__ dead, uint32_t* __restrict__ kc) {
#if defined(__AMDGCN_WAVEFRONT_SIZE)
  static_assert(__AMDGCN_WAVEFRONT_SIZE == 64, "k_abs_kill_fast reads lane + 1 by a 64-wide shuffle (CDNA wave64)");
#endif
  const int lane = threadIdx.x & 63;
  for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x; p0 < a.nt; p0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = p0 + threadIdx.x;
    const bool in = p < a.nt;
    const uint32_t v = in ? sid[p] : 0u;
    const K kp = in ? skeys[p] : sentinel;
    const bool live = kp != sentinel;
    const int64_t tv = live ? vts(a, ts, c_dl, v) : 0;
    const int64_t t1 = __shfl_down(tv, 1, 64);
    const uint32_t v1 = __shfl_down(v, 1, 64);
    const K k1 = __shfl_down(kp, 1, 64);
    if (!live) continue;
    int64_t tq = 0;
    uint32_t vk = 0;
    bool found = false;
    int64_t x = p + 1;
    if (lane < 63 && x < a.nt) {
      if (k1 != kp) continue;   // no later row with this value
      if (v1 >= (uint32_t)a.nc) { tq = t1; vk = v1; found = true; }
      else ++x;                 // a carried row: search on
    }
    if (!found)
      for (; x < a.nt && skeys[x] == kp; ++x)
        if (sid[x] >= (uint32_t)a.nc) { vk = sid[x]; tq = ts[vk - a.nc]; found = true; break; }
    if (found && tq < tv + a.W) {
      dead[v] = 1;
      atomicAdd(&kc[vk - a.nc], 1u);
    }
  }
}

// 4b. per candidate: trigger row (first row with ts >= deadline) or pending; packed counts for the scan
__global__ void k_abs_decide(AbsArgs a, const uint8_t* __restrict__ role, const uint8_t* __restrict__ dead,
                             const int64_t* __restrict__ ts, const int64_t* __restrict__ c_dl,
                             uint32_t* __restrict__ trig, uint64_t* __restrict__ cnt) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.nt; v += (int64_t)gridDim.x * blockDim.x) {
    uint64_t c = 0;
    uint32_t t = NONE;
    if ((role[v] & R_CAND) && !dead[v]) {
      const int64_t d = vts(a, ts, c_dl, (uint32_t)v) + a.W;
      int64_t lo = v < a.nc ? 0 : v - a.nc + 1, hi = a.n;   // W > 0: the trigger follows the row
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (ts[mid] < d) lo = mid + 1; else hi = mid;
      }
      if (lo < a.n) { t = (uint32_t)lo; c = 1; } else { c = 1ull << 32; }
    }
    trig[v] = t;
    cnt[v] = c;
  }
}

struct AbsOut {
  int32_t n_select, stride;
  uint64_t base_index;
  const uint64_t* index;
  int32_t sel_ok[SG_MAX_SELECT];    // 1: e1 attribute (projected), 0: null (`not` slot / chain index > 0)
  int32_t sel_col[SG_MAX_SELECT], sel_type[SG_MAX_SELECT];
};

// 6. emission records and carried partials (e1's projected attributes read straight into the record)
__device__ __forceinline__ int64_t abs_sel(const AbsOut& o, const SgCols& cols, int s, int64_t i, uint32_t& nm) {
  if (!o.sel_ok[s]) { nm |= 1u << s; return 0; }
  SgVal x = sg_read_col(cols, o.sel_col[s], o.sel_type[s], i);
  if (x.null) { nm |= 1u << s; return 0; }
  return sg_val_bits(x);
}

__global__ void __launch_bounds__(256) k_abs_write(AbsArgs a, AbsOut o, SgCols cols, const int64_t* __restrict__ ts,
                                                   const uint32_t* __restrict__ trig, const uint64_t* __restrict__ cnt,
                                                   const uint64_t* __restrict__ off, const int64_t* __restrict__ vals,
                                                   const uint8_t* __restrict__ role, AbsCarry cin, AbsCarry cout,
                                                   const uint32_t* __restrict__ first_slot, char* __restrict__ out) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.nt; v += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t c = cnt[v];
    if (!c) continue;
    const uint64_t ofs = off[v];
    const bool carried = v < a.nc;
    const int64_t i = v - a.nc;
    const int64_t d = carried ? cin.dl[v] : ts[i] + a.W;
    uint32_t nm = carried ? cin.snul[v] : 0u;
    if (c & 0xffffffffull) {   // emitted in this push
      const uint32_t sl = (uint32_t)ofs;
      const uint32_t t = trig[v];
      int64_t* r = (int64_t*)(out + (size_t)sl * o.stride);
      for (int s = 0; s < o.n_select; ++s) {
        int64_t x = carried ? cin.sel[v * o.n_select + s] : abs_sel(o, cols, s, i, nm);
        r[4 + s] = (nm >> s) & 1 ? 0 : x;
      }
      r[0] = (int64_t)(o.index ? o.index[t] : o.base_index + t);
      r[1] = d;
      // key 0 | group = rank within the trigger's timer pass (emissions are contiguous per trigger)
      r[2] = (int64_t)((uint64_t)(sl - first_slot[sl]) << 32);
      r[3] = (int64_t)nm;
    } else if (a.keep_carry) { // still pending: carried into the next push
      const uint32_t cs = (uint32_t)(ofs >> 32);
      cout.dl[cs] = d;
      cout.val[cs] = vals[v];
      cout.vnul[cs] = (role[v] & R_SORT) ? 0 : 1;
      for (int s = 0; s < o.n_select; ++s)
        cout.sel[(int64_t)cs * o.n_select + s] = carried ? cin.sel[v * o.n_select + s] : abs_sel(o, cols, s, i, nm);
      cout.snul[cs] = nm;
    }
  }
}

// first slot of each slot's trigger: segment heads, then an inclusive max-scan
__global__ void k_abs_heads(int64_t ne, const uint32_t* __restrict__ slot_trig, uint32_t* __restrict__ head) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ne; s += (int64_t)gridDim.x * blockDim.x)
    head[s] = (s == 0 || slot_trig[s] != slot_trig[s - 1]) ? (uint32_t)s : 0u;
}

__global__ void k_abs_slot_trig(int64_t nt, const uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off,
                                const uint32_t* __restrict__ trig, uint32_t* __restrict__ slot_trig) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nt; v += (int64_t)gridDim.x * blockDim.x)
    if (cnt[v] & 0xffffffffull) slot_trig[(uint32_t)off[v]] = trig[v];
}

__global__ void k_abs_init(unsigned long long* __restrict__ minmax, uint32_t* __restrict__ oflag) {
  if (threadIdx.x == 0) {
    minmax[0] = ~0ull;
    minmax[1] = 0ull;
    *oflag = 0xffffffffu;   // first row whose time goes back (none)
  }
}

__global__ void k_abs_last(int64_t n, const int64_t* __restrict__ ts, int64_t* __restrict__ dlast) {
  if (threadIdx.x == 0 && n > 0) *dlast = ts[n - 1];
}

// ---- FIFO after a closed-form push (no timestamp went back): every entry <= the clock has been popped; the rest
// are the carried entries above it, then per row of this push its kill entries and its creation entry (all
// ts + W: updateLastArrivalTime and addState, AbsentStreamPreStateProcessor.java:69-101) when above the clock
__global__ void k_abs_qcount(int64_t nq, const int64_t* __restrict__ q, int64_t n, const int64_t* __restrict__ ts,
                             const uint8_t* __restrict__ role, int64_t nc, const uint32_t* __restrict__ kc, int64_t W,
                             int64_t clock, uint32_t* __restrict__ m) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e <= nq + n; e += (int64_t)gridDim.x * blockDim.x) {
    uint32_t c = 0;
    if (e < nq) c = q[e] > clock ? 1u : 0u;
    else if (e < nq + n) {
      const int64_t i = e - nq;
      if (ts[i] + W > clock) c = kc[i] + ((role[nc + i] & R_CAND) ? 1u : 0u);
    }
    m[e] = c;
  }
}
__global__ void k_abs_qwrite(int64_t nq, const int64_t* __restrict__ q, int64_t n, const int64_t* __restrict__ ts,
                             int64_t W, const uint32_t* __restrict__ m, const uint32_t* __restrict__ off,
                             int64_t* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq + n; e += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = m[e];
    const int64_t v = e < nq ? q[e] : ts[e - nq] + W;
    for (uint32_t k = 0; k < c; ++k) out[off[e] + k] = v;
  }
}

// ---- exact sequential pass: a push in which some timestamp goes back, or a state the closed form cannot continue.
// The reference's per-row sequence for `every A -> not B[x == e1.x] for W` with the playback clock and the FIFO:
//   setCurrentTimestamp(ts): if ts >= clock, clock = ts and, while the FIFO head <= clock, a timer pass at the head
//     value T (TimestampGeneratorImpl.java:106-125, Scheduler.java:74-86,179-214): every pending partial with
//     ts_i + W <= T is emitted stamped T, in pending order; then lastScheduledTime = clock + W if clock > T + W, and a
//     pass that emitted nothing with lastScheduledTime < T schedules T + W (AbsentStreamPreStateProcessor.java:140-210);
//   a B row kills every pending partial with its value, each kill scheduling ts + W (:230-244, AbsentStreamPost-
//     StateProcessor.java:36-56); an A row opens a partial and schedules ts + W (:77-101).
// One wave walks the rows in lockstep (the FIFO makes the order of everything global): the per-row work (clock, FIFO,
// kills through a hash of the compared value, new partials) is the same on every lane; a timer pass is shared -- the
// lanes test 64 blocks' earliest deadlines at once and then one block's 64 partials at once, emitting in creation
// order by ballot.  After `min_rows` rows the pass may stop at a row boundary once the state is the closed form's
// again (FIFO sorted, above the clock, below lastScheduledTime; checked every 1024 rows): the caller runs the rest of
// the push through the closed form.
struct SeqAbs {
  int64_t n, nc, W;
  int64_t min_rows;            // stop early only after this many rows (<= 0: never; walk every row)
  const int64_t* ts;
  const uint8_t* role;
  const int64_t* vals;         // virtual rows (carried partials first)
  const int64_t* c_dl;         // carried partials' deadlines
  // FIFO in: carried entries; ring capacity qcap (power of two)
  const int64_t* q_in;
  int64_t nq_in, qcap;
  int64_t* ring;
  // partials (creation order): deadline, value, source virtual row, alive; next with the same value
  int64_t* pd;
  uint32_t* psrc;
  uint8_t* palive;
  int32_t* pnext;
  int64_t* bmin;               // per 64 partials: earliest deadline among the alive ones (or a stale lower bound)
  // hash of values of killable partials
  int64_t hcap;
  int64_t* hkey;
  int32_t* hhead;
  int32_t* htail;
  uint8_t* hused;
  // emissions in delivery order: partial, trigger row, stamp, callback group
  uint32_t* ek;
  uint32_t* erow;
  int64_t* ets;
  uint32_t* eg;
  int64_t ecap;
  // scalars: [0] clock, [1] lastScheduledTime, [2] emissions, [3] partials, [4] ring head, [5] ring tail,
  // [6] flags (1 capacity), [7] closed form can continue (1), [8] rows walked
  int64_t* sc;
};

__device__ __forceinline__ uint64_t sa_hash(int64_t x) {
  uint64_t z = (uint64_t)x * 0x9E3779B97F4A7C15ull;
  return z ^ (z >> 29);
}

__device__ __forceinline__ int64_t sa_wave_min(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_xor(v, o);
    v = y < v ? y : v;
  }
  return v;
}

__global__ void __launch_bounds__(64) k_abs_seq(SeqAbs s) {
  if (blockIdx.x != 0) return;
  const uint32_t lane = threadIdx.x;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t INF = INT64_MAX;
  int64_t clock = s.sc[0], lst = s.sc[1];
  int64_t ne = 0, np = 0, head = 0, tail = 0;
  bool cap_bad = false;
  const int64_t qmask = s.qcap - 1, hmask = s.hcap - 1;
  // (every lane runs the uniform work with the same values: the stores repeat the same word, and each lane reads
  // back only what it stored itself.  Values the wave keeps in registers instead of re-reading: the FIFO head `qh`,
  // the last partial block's earliest deadline `lbm`, the next row's inputs.)
  int64_t qh = INF;   // ring[head] while head < tail
  auto qpush = [&](int64_t v) {
    if (tail - head >= s.qcap) { cap_bad = true; return; }
    s.ring[tail & qmask] = v;
    if (tail == head) qh = v;
    ++tail;
  };
  auto hslot = [&](int64_t key, bool insert) -> int64_t {
    int64_t h = (int64_t)(sa_hash(key) & (uint64_t)hmask);
    for (int64_t probe = 0; probe < s.hcap; ++probe, h = (h + 1) & hmask) {
      if (!s.hused[h]) {
        if (!insert) return -1;
        s.hused[h] = 1;
        s.hkey[h] = key;
        s.hhead[h] = -1;
        s.htail[h] = -1;
        return h;
      }
      if (s.hkey[h] == key) return h;
    }
    cap_bad = true;
    return -1;
  };
  int64_t lbb = -1, lbm = INF;   // the last partial block and its earliest deadline (as stored in bmin)
  // h_known >= 0: the value's hash slot, found by this row's kill, whose list the kill just emptied
  auto add_partial = [&](int64_t d, uint32_t src, bool killable, int64_t key, int64_t h_known) {
    const int64_t k = np++;
    s.pd[k] = d;
    s.psrc[k] = src;
    s.palive[k] = 1;
    s.pnext[k] = -1;
    const int64_t b = k >> 6;
    if (b != lbb) { lbb = b; lbm = d; }
    else if (d < lbm) lbm = d;
    s.bmin[b] = lbm;
    if (killable) {
      if (h_known >= 0) {
        s.hhead[h_known] = (int32_t)k;
        s.htail[h_known] = (int32_t)k;
        return;
      }
      const int64_t h = hslot(key, true);
      if (h < 0) return;
      const int32_t tl = s.htail[h];
      if (tl < 0) s.hhead[h] = (int32_t)k; else s.pnext[tl] = (int32_t)k;
      s.htail[h] = (int32_t)k;
    }
  };
  int64_t lob = 0;   // first block that may hold an alive partial
  uint32_t cur_row = 0xffffffffu, grp = 0;
  auto pass = [&](int64_t T, uint32_t row) -> bool {   // one timer pass; true if it emitted
    bool any = false;
    const int64_t nb = (np + 63) >> 6;
    bool lead = true;   // still skipping leading blocks with nothing alive
    for (int64_t b0 = lob; b0 < nb; b0 += 256) {
      int64_t bm[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {   // 256 blocks' earliest deadlines per memory round trip
        const int64_t b = b0 + 64 * u + lane;
        bm[u] = b < nb ? s.bmin[b] : INF;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t bu = b0 + 64 * u;
        if (bu >= nb) break;
        if (lead) {
          const uint64_t live = __ballot(!(bu + lane < nb && bm[u] == INF));
          if (live) { lob = bu + __builtin_ctzll(live); lead = false; }
          else lob = bu + 64;
        }
        uint64_t cm = __ballot(bu + lane < nb && bm[u] <= T);
        while (cm) {
          const int64_t bb = bu + __builtin_ctzll(cm);
          cm &= cm - 1;
          const int64_t k = bb * 64 + lane;
          const bool al = k < np && s.palive[k];
          const int64_t d = al ? s.pd[k] : INF;
          const bool em = al && d <= T;
          const uint64_t emm = __ballot(em);
          const int64_t rest = sa_wave_min(em ? INF : d);
          if (emm) {
            if (row != cur_row) { cur_row = row; grp = 0; }
            const uint32_t below = (uint32_t)__popcll(emm & lt), cnt = (uint32_t)__popcll(emm);
            if (em) {
              s.palive[k] = 0;
              const int64_t slot = ne + below;
              if (slot < s.ecap) { s.ek[slot] = (uint32_t)k; s.erow[slot] = row; s.ets[slot] = T; s.eg[slot] = grp + below; }
            }
            if (ne + cnt > s.ecap) cap_bad = true;
            ne += cnt;
            grp += cnt;
            any = true;
            __threadfence_block();   // (a later kill reads these flags on every lane)
          }
          s.bmin[bb] = rest;
          if (bb == lbb) lbm = rest;
        }
      }
    }
    return any;
  };
  auto fifo_ok = [&]() -> bool {   // the closed form can continue from this state
    for (int64_t k0 = head; k0 < tail; k0 += 64) {
      const int64_t k = k0 + lane;
      bool bad = false;
      if (k < tail) {
        const int64_t x = s.ring[k & qmask];
        const int64_t prev = k > head ? s.ring[(k - 1) & qmask] : INT64_MIN;
        bad = x < prev || x <= clock || x > lst;
      }
      if (__ballot(bad)) return false;
    }
    return true;
  };
  for (int64_t k = 0; k < s.nq_in; ++k) qpush(s.q_in[k]);
  for (int64_t k = 0; k < s.nc; ++k) {
    const uint8_t r = s.role[k];
    add_partial(s.c_dl[k], (uint32_t)k, (r & R_SORT) != 0, s.vals[k], -1);
  }
  int64_t i = 0;
  bool ok = false;
  // row i's inputs, loaded one row ahead (the inputs are never written here)
  int64_t tn = 0, xn = 0;
  uint8_t rn = 0;
  if (s.n > 0) { tn = s.ts[0]; rn = s.role[s.nc]; xn = s.vals[s.nc]; }
  for (; i < s.n && !cap_bad; ++i) {
    if (s.min_rows > 0 && i >= s.min_rows && (i & 1023) == 0 && fifo_ok()) { ok = true; break; }
    const int64_t t = tn;
    const uint8_t r = rn;
    const int64_t x = xn;
    if (i + 1 < s.n) { tn = s.ts[i + 1]; rn = s.role[s.nc + i + 1]; xn = s.vals[s.nc + i + 1]; }
    if (t >= clock) {
      clock = t;
      while (head < tail && qh <= clock && !cap_bad) {
        const int64_t T = qh;
        ++head;
        qh = head < tail ? s.ring[head & qmask] : INF;
        const bool emitted = pass(T, (uint32_t)i);
        if (clock > s.W + T) lst = clock + s.W;
        if (!emitted && lst < T) {
          lst = T + s.W;
          qpush(lst);
        }
      }
    }
    const int64_t v = s.nc + i;
    int64_t h_known = -1;
    if (r & R_KILL) {
      const int64_t h = hslot(x, false);
      if (h >= 0) {
        for (int32_t k = s.hhead[h]; k >= 0; k = s.pnext[k]) {
          if (!s.palive[k]) continue;
          s.palive[k] = 0;   // (its block's earliest deadline becomes stale: a lower bound, refreshed by the next scan)
          lst = t + s.W;
          qpush(lst);
        }
        s.hhead[h] = -1;
        s.htail[h] = -1;
        h_known = h;
      }
    }
    if (r & R_CAND) {
      // (a row's kill and candidate read the same value: one compared value per row, sg_every_absent_supported)
      add_partial(t + s.W, (uint32_t)v, (r & R_SORT) != 0, x, h_known);
      lst = t + s.W;
      qpush(lst);
    }
  }
  // can the closed form continue from here?  its FIFO must be sorted and above the clock, and lastScheduledTime at
  // least its largest entry (then no later pass re-schedules while time moves forward)
  if (!ok) ok = fifo_ok();
  if (lane == 0) {
    s.sc[0] = clock;
    s.sc[1] = lst;
    s.sc[2] = ne;
    s.sc[3] = np;
    s.sc[4] = head;
    s.sc[5] = tail;
    s.sc[6] = cap_bad ? 1 : 0;
    s.sc[7] = ok ? 1 : 0;
    s.sc[8] = i;
  }
}

// FIFO ring [head, tail) -> a flat queue
__global__ void k_abs_qflat(const int64_t* __restrict__ ring, int64_t qcap, const int64_t* __restrict__ sc,
                            int64_t* __restrict__ out) {
  const int64_t head = sc[4], tail = sc[5];
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < tail - head; k += (int64_t)gridDim.x * blockDim.x)
    out[k] = ring[(head + k) & (qcap - 1)];
}

// partials still alive -> carried partials (creation order); emissions -> match records
__global__ void k_abs_seq_alive(int64_t np, const uint8_t* __restrict__ palive, uint32_t* __restrict__ flag) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= np; k += (int64_t)gridDim.x * blockDim.x)
    flag[k] = k < np ? palive[k] : 0u;
}
__global__ void k_abs_seq_carry(AbsArgs a, AbsOut o, SgCols cols, const int64_t* __restrict__ ts, int64_t np,
                                const uint32_t* __restrict__ flag, const uint32_t* __restrict__ off,
                                const uint32_t* __restrict__ psrc, const int64_t* __restrict__ pd,
                                const int64_t* __restrict__ vals, const uint8_t* __restrict__ role, AbsCarry cin,
                                AbsCarry cout) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < np; k += (int64_t)gridDim.x * blockDim.x) {
    if (!flag[k]) continue;
    const uint32_t v = psrc[k], cs = off[k];
    const bool carried = v < a.nc;
    const int64_t i = (int64_t)v - a.nc;
    uint32_t nm = carried ? cin.snul[v] : 0u;
    cout.dl[cs] = pd[k];
    cout.val[cs] = vals[v];
    cout.vnul[cs] = (role[v] & R_SORT) ? 0 : 1;
    for (int s = 0; s < o.n_select; ++s)
      cout.sel[(int64_t)cs * o.n_select + s] = carried ? cin.sel[(int64_t)v * o.n_select + s] : abs_sel(o, cols, s, i, nm);
    cout.snul[cs] = nm;
  }
}
__global__ void k_abs_seq_write(AbsArgs a, AbsOut o, SgCols cols, int64_t ne, const uint32_t* __restrict__ ek,
                                const uint32_t* __restrict__ erow, const int64_t* __restrict__ ets,
                                const uint32_t* __restrict__ eg, const uint32_t* __restrict__ psrc, AbsCarry cin,
                                char* __restrict__ out) {
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < ne; x += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = psrc[ek[x]];
    const bool carried = v < a.nc;
    const int64_t i = (int64_t)v - a.nc;
    uint32_t nm = carried ? cin.snul[v] : 0u;
    int64_t* r = (int64_t*)(out + (size_t)x * o.stride);
    for (int s = 0; s < o.n_select; ++s) {
      int64_t y = carried ? cin.sel[(int64_t)v * o.n_select + s] : abs_sel(o, cols, s, i, nm);
      r[4 + s] = (nm >> s) & 1 ? 0 : y;
    }
    const uint32_t t = erow[x];
    r[0] = (int64_t)(o.index ? o.index[t] : o.base_index + t);
    r[1] = ets[x];
    r[2] = (int64_t)((uint64_t)eg[x] << 32);
    r[3] = (int64_t)nm;
  }
}

AbsState* astate(SgHandle* h) {
  if (!h->state) {
    AbsState* s = new AbsState();
    if (hipMalloc(&s->dlast, 8) != hipSuccess || hipMalloc(&s->dminmax, 16) != hipSuccess ||
        hipMalloc(&s->dflag, 4) != hipSuccess)
      throw SgError(SG_EHIP, "hipMalloc failed for absence state");
    h->state = s;
    h->state_kind = 3;
  }
  return (AbsState*)h->state;
}

static const int64_t SEQ_MIN_ROWS = 1024;   // rows the sequential pass walks before it may hand back to the closed form
unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 16)); }
unsigned grid_red(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024)); }

template <class K>
void sort_and_kill(SgHandle* h, const AbsArgs& a, uint64_t omin, int bits, const uint8_t* role, const int64_t* vals,
                   const int64_t* ts, const int64_t* c_dl, uint8_t* dead, uint32_t* kc) {
  hipStream_t st = h->stream;
  const int64_t nt = a.nt;
  K* keys = (K*)h->ws.get("abs_keys", sizeof(K) * nt, st);
  K* skeys = (K*)h->ws.get("abs_skeys", sizeof(K) * nt, st);
  uint32_t* ids = (uint32_t*)h->ws.get("abs_ids", 4 * nt, st);
  uint32_t* sid = (uint32_t*)h->ws.get("abs_sid", 4 * nt, st);
  const K sentinel = (K)(bits >= (int)(8 * sizeof(K)) ? ~(K)0 : ((K)1 << bits) - 1);
  hipLaunchKernelGGL((k_abs_keys<K>), dim3(grid_for(nt)), dim3(256), 0, st, nt, role, vals, omin, sentinel, keys, ids);
  size_t tb = 0;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, keys, skeys, ids, sid, (size_t)nt, 0, bits, st));
  void* tmp = h->ws.get("abs_sort_tmp", tb, st);
  HIPCHK(rocprim::radix_sort_pairs(tmp, tb, keys, skeys, ids, sid, (size_t)nt, 0, bits, st));
  uint32_t* nks = nullptr;
  if (!a.fast) {
    uint32_t* rk = (uint32_t*)h->ws.get("abs_rk", 4 * nt, st);
    nks = (uint32_t*)h->ws.get("abs_nks", 4 * nt, st);
    hipLaunchKernelGGL(k_abs_rkill, dim3(grid_for(nt)), dim3(256), 0, st, nt, sid, role, rk);
    tb = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, tb, rk, nks, (size_t)nt, rocprim::minimum<uint32_t>(), st));
    tmp = h->ws.get("abs_scan_tmp", tb, st);
    HIPCHK(rocprim::inclusive_scan(tmp, tb, rk, nks, (size_t)nt, rocprim::minimum<uint32_t>(), st));
  }
  if (a.fast && bits < 64)   // below 64 bits the sentinel lies above every value key
    hipLaunchKernelGGL((k_abs_kill_fast<K>), dim3(grid_for(nt)), dim3(256), 0, st, a, skeys, sid, sentinel, ts, c_dl, dead,
                       kc);
  else
    hipLaunchKernelGGL((k_abs_kill<K>), dim3(grid_for(nt)), dim3(256), 0, st, a, skeys, sid, role, nks, ts, c_dl, dead, kc);
  HIPCHK(hipGetLastError());
}

}  // namespace

// The exact sequential pass (k_abs_seq) over rows [0, m) of a segment, from the carried state (pending partials, FIFO,
// lastScheduledTime, clock) to the next; m = every row, or (min_rows > 0) the first row boundary after min_rows rows
// where the closed form can take over again.  Returns m.
static int64_t run_seq(SgHandle* h, AbsState* as, const AbsArgs& a, const BatchView& bv, const uint8_t* role,
                       const int64_t* vals, const AbsCarry& cin, AbsCarry& cout, const int64_t* qv, int64_t nq_in,
                       AbsQueue& qout, int64_t clock0, int64_t lst0, int64_t min_rows) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  const int64_t n = a.n, nc = a.nc, P = std::max<int64_t>(nc + n, 1);
  auto pow2 = [](int64_t x) { int64_t c = 1024; while (c < x) c <<= 1; return c; };
  int64_t qcap = pow2(2 * (nq_in + 2 * P) + 1024);
  const int64_t hcap = pow2(2 * P);
  int64_t sc[9] = {};
  SeqAbs s;
  memset(&s, 0, sizeof(s));
  s.n = n;
  s.min_rows = min_rows;
  s.nc = nc;
  s.W = a.W;
  s.ts = bv.ts;
  s.role = role;
  s.vals = vals;
  s.c_dl = cin.dl;
  s.q_in = qv;
  s.nq_in = nq_in;
  s.pd = (int64_t*)h->ws.get("sa_pd", 8 * P, st);
  s.psrc = (uint32_t*)h->ws.get("sa_psrc", 4 * P, st);
  s.palive = (uint8_t*)h->ws.get("sa_palive", P, st);
  s.pnext = (int32_t*)h->ws.get("sa_pnext", 4 * P, st);
  s.bmin = (int64_t*)h->ws.get("sa_bmin", 8 * (P / 64 + 1), st);
  s.hcap = hcap;
  s.hkey = (int64_t*)h->ws.get("sa_hkey", 8 * hcap, st);
  s.hhead = (int32_t*)h->ws.get("sa_hhead", 4 * hcap, st);
  s.htail = (int32_t*)h->ws.get("sa_htail", 4 * hcap, st);
  s.hused = (uint8_t*)h->ws.get("sa_hused", hcap, st);
  s.ecap = P;
  s.ek = (uint32_t*)h->ws.get("sa_ek", 4 * P, st);
  s.erow = (uint32_t*)h->ws.get("sa_erow", 4 * P, st);
  s.ets = (int64_t*)h->ws.get("sa_ets", 8 * P, st);
  s.eg = (uint32_t*)h->ws.get("sa_eg", 4 * P, st);
  s.sc = (int64_t*)h->ws.get("sa_sc", 128, st);
  h->kbeg("abs_sequential");
  for (;;) {
    s.qcap = qcap;
    s.ring = (int64_t*)h->ws.get("sa_ring", 8 * qcap, st);
    HIPCHK(hipMemsetAsync(s.hused, 0, hcap, st));
    const int64_t init[2] = {clock0, lst0};
    HIPCHK(hipMemcpyAsync(s.sc, init, 16, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_abs_seq, dim3(1), dim3(64), 0, st, s);   // (one wave)
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(sc, s.sc, sizeof(sc), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (!(sc[6] & 1)) break;
    if (qcap >= ((int64_t)1 << 34)) throw SgError(SG_ECAPACITY, "absence timer queue beyond 2^34 entries");
    qcap <<= 1;   // the timer FIFO outgrew its ring: rerun the push with a larger one (the inputs are unchanged)
  }
  h->kend();
  h->mark(2);
  const int64_t ne = sc[2], np = sc[3];
  AbsOut o;
  memset(&o, 0, sizeof(o));
  o.n_select = d.n_select;
  o.stride = 32 + 8 * d.n_select;
  o.base_index = bv.base_index;
  o.index = bv.index;
  const int a_state = d.shape_args[0];
  for (int k = 0; k < d.n_select; ++k) {
    const int idx = d.sel_index[k];
    o.sel_ok[k] = d.sel_state[k] == a_state && (idx == 0 || idx == -1);
    o.sel_col[k] = d.ret_col[d.sel_ret[k]];
    o.sel_type[k] = d.sel_type[k];
  }
  h->mark(3);
  h->kbeg("abs_write");
  char* rec = h->out.reserve(ne, d.n_select, st);
  if (ne > 0)
    hipLaunchKernelGGL(k_abs_seq_write, dim3(grid_for(ne)), dim3(256), 0, st, a, o, bv.cols, ne, s.ek, s.erow, s.ets, s.eg,
                       s.psrc, cin, rec + (size_t)h->out.n * o.stride);
  HIPCHK(hipGetLastError());
  if (a.keep_carry) {
    uint32_t* fl = (uint32_t*)h->ws.get("sa_flag", 4 * (np + 1), st);
    uint32_t* fo = (uint32_t*)h->ws.get("sa_foff", 4 * (np + 1), st);
    hipLaunchKernelGGL(k_abs_seq_alive, dim3(grid_for(np + 1)), dim3(256), 0, st, np, s.palive, fl);
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, fl, fo, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), st));
    void* tmp = h->ws.get("sa_scan_tmp", tb, st);
    HIPCHK(rocprim::exclusive_scan(tmp, tb, fl, fo, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), st));
    uint32_t ncar = 0;
    HIPCHK(hipMemcpyAsync(&ncar, fo + np, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    cout.reserve(std::max<int64_t>(ncar, 1), d.n_select);
    if (ncar)
      hipLaunchKernelGGL(k_abs_seq_carry, dim3(grid_for(np)), dim3(256), 0, st, a, o, bv.cols, bv.ts, np, fl, fo, s.psrc,
                         s.pd, vals, role, cin, cout);
    const int64_t nq1 = sc[5] - sc[4];
    qout.reserve(std::max<int64_t>(nq1, 1));
    if (nq1) hipLaunchKernelGGL(k_abs_qflat, dim3(grid_for(nq1)), dim3(256), 0, st, s.ring, qcap, s.sc, qout.v);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(as->dlast, &sc[0], 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    cout.n = ncar;
    qout.n = nq1;
    as->lst = sc[1];
    as->seq = sc[7] == 0;
    as->cur ^= 1;
  }
  h->kend();
  h->mark(4);
  h->out.n += ne;
  h->split_out = 0;
  return sc[8];
}

bool sg_every_absent_supported(const sg_nfa_desc& d) {
  const int a = d.shape_args[0], b = d.shape_args[1];
  const int ca = d.ret_col[d.shape_args[4]], cb = d.ret_col[d.shape_args[3]];
  if (d.partitioned || d.within != -1 || !d.playback) return false;
  if (d.states[b].waiting_time <= 0) return false;
  if (d.states[a].stream == d.states[b].stream && ca != cb) return false;   // one compared value per row
  return d.col_type[ca] == d.col_type[cb];
}

// One segment of a push: rows [0, m) of bv, m returned.  The closed form takes the rows up to the first one whose time
// goes back (all of them when none does); from such a row -- or from the segment's start when the carried state is
// not the closed form's -- the exact sequential pass takes over until the state is the closed form's again.
// first: the stream's first rows (no clock, FIFO or lastScheduledTime before them); carry_in: the carried partials
// are the segment's virtual rows; keep: write the carried state for what follows.
static int64_t absent_segment(SgHandle* h, const BatchView& bv, int64_t n, bool first, bool carry_in, bool keep) {
  const sg_nfa_desc& d = h->desc;
  hipStream_t st = h->stream;
  AbsState* as = astate(h);
  AbsCarry& cin = as->carry[as->cur];
  AbsCarry& cout = as->carry[as->cur ^ 1];
  const int a_state = d.shape_args[0], b_state = d.shape_args[1];
  AbsArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.nc = carry_in ? cin.n : 0;
  a.nt = a.nc + n;
  if (a.nt >= (1ll << 31)) throw SgError(SG_EINVAL, "batch plus pending partials exceed 2^31");
  a.W = d.states[b_state].waiting_time;
  a.s_a = d.states[a_state].stream;
  a.s_b = d.states[b_state].stream;
  a.col_a = d.ret_col[d.shape_args[4]];
  a.col_b = d.ret_col[d.shape_args[3]];
  a.type = d.col_type[a.col_a];
  a.prog_a_off = d.states[a_state].prog_off;
  a.prog_a_len = d.states[a_state].prog_len;
  a.prog_b_off = d.shape_prog_off;
  a.prog_b_len = d.shape_prog_len;
  a.has_stream = bv.stream ? 1 : 0;
  a.first_push = first ? 1 : 0;
  a.keep_carry = keep ? 1 : 0;
  a.fast = (a.s_a == 0 && a.s_b == 0 && a.col_a == a.col_b && !bv.stream && a.prog_a_len == 0 && a.prog_b_len == 0 &&
            !bv.cols.nul[a.col_a] && (a.type == SG_T_LONG || a.type == SG_T_INT || a.type == SG_T_STRING)) ? 1 : 0;
  const int64_t nt = a.nt;
  h->split_out = 0;
  h->extra_marks = 0;
  h->mark(0);
  // ---- 1. roles and value range
  uint8_t* role = (uint8_t*)h->ws.get("abs_role", nt, st);
  int64_t* vals = (int64_t*)h->ws.get("abs_vals", 8 * nt, st);
  uint8_t* dead = (uint8_t*)h->ws.get("abs_dead", nt, st);
  uint32_t* kc = (uint32_t*)h->ws.get("abs_kc", 4 * (n + 1), st);
  HIPCHK(hipMemsetAsync(kc, 0, 4 * (n + 1), st));
  hipLaunchKernelGGL(k_abs_init, dim3(1), dim3(64), 0, st, (unsigned long long*)as->dminmax, as->dflag);
  HIPCHK(hipMemsetAsync(dead, 0, nt, st));
  h->kbeg("abs_roles");
  if (nt > 0 && a.fast && a.type == SG_T_LONG)
    hipLaunchKernelGGL((k_abs_rows_fast<int64_t>), dim3(grid_red(nt)), dim3(256), 0, st, a,
                       (const int64_t*)bv.cols.col[a.col_a], bv.ts, cin.val, cin.vnul, role, vals,
                       (unsigned long long*)as->dminmax, as->dlast, as->dflag);
  else if (nt > 0 && a.fast)
    hipLaunchKernelGGL((k_abs_rows_fast<int32_t>), dim3(grid_red(nt)), dim3(256), 0, st, a,
                       (const int32_t*)bv.cols.col[a.col_a], bv.ts, cin.val, cin.vnul, role, vals,
                       (unsigned long long*)as->dminmax, as->dlast, as->dflag);
  else if (nt > 0)
    hipLaunchKernelGGL(k_abs_rows, dim3(grid_red(nt)), dim3(256), 0, st, a, bv.cols, h->ddesc, bv.ts, bv.stream,
                       cin.val, cin.vnul, role, vals, (unsigned long long*)as->dminmax, as->dlast, as->dflag);
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(1);
  uint64_t mm[2] = {0, 0};
  uint32_t oflag = 0;
  int64_t clock0 = 0;
  HIPCHK(hipMemcpyAsync(mm, as->dminmax, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&oflag, as->dflag, 4, hipMemcpyDeviceToHost, st));
  if (!a.first_push) HIPCHK(hipMemcpyAsync(&clock0, as->dlast, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  AbsQueue& qin = as->q[as->cur];
  AbsQueue& qout = as->q[as->cur ^ 1];
  const int64_t nq_in = a.first_push ? 0 : qin.n;
  const int64_t lst0 = a.first_push ? 0 : as->lst;
  const bool seq_state = as->seq && !a.first_push;
  if (oflag != 0xffffffffu || seq_state) {
    const int64_t p = seq_state ? 0 : (int64_t)oflag;
    // the rows before the first late one are in order: the closed form takes them, carrying its state to the rest
    if (p > 0) return absent_segment(h, sg_slice_view(d, bv, 0, p), p, first, carry_in, true);
    // from a row whose time goes back (or a state the closed form cannot continue): the exact sequential pass, kept
    // only as long as that state lasts
    a.keep_carry = 1;
    return run_seq(h, as, a, bv, role, vals, cin, cout, qin.v, nq_in, qout, clock0, lst0, SEQ_MIN_ROWS);
  }
  // ---- 2-4. sort by value, kill
  h->kbeg("abs_sort_kill");
  if (mm[0] <= mm[1] && nt > 0) {
    const uint64_t range = mm[1] - mm[0];   // sentinel = range + 1 must fit in the key bits
    int bits = 1;
    while (bits < 64 && (range + 1) >> bits) ++bits;
    if (range + 1 == 0) bits = 64;
    if (bits <= 32)
      sort_and_kill<uint32_t>(h, a, mm[0], bits, role, vals, bv.ts, cin.dl, dead, kc);
    else
      sort_and_kill<uint64_t>(h, a, mm[0], bits, role, vals, bv.ts, cin.dl, dead, kc);
  }
  h->kend();
  h->mark(2);
  // ---- decide, scan
  uint32_t* trig = (uint32_t*)h->ws.get("abs_trig", 4 * nt, st);
  uint64_t* cnt = (uint64_t*)h->ws.get("abs_cnt", 8 * (nt + 1), st);
  uint64_t* off = (uint64_t*)h->ws.get("abs_off", 8 * (nt + 1), st);
  h->kbeg("abs_decide_scan");
  if (nt > 0)
    hipLaunchKernelGGL(k_abs_decide, dim3(grid_for(nt)), dim3(256), 0, st, a, role, dead, bv.ts, cin.dl, trig, cnt);
  HIPCHK(hipMemsetAsync(cnt + nt, 0, 8, st));
  size_t tb = 0;
  HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, (uint64_t)0, (size_t)nt + 1, rocprim::plus<uint64_t>(), st));
  void* tmp = h->ws.get("abs_oscan_tmp", tb, st);
  HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, (uint64_t)0, (size_t)nt + 1, rocprim::plus<uint64_t>(), st));
  h->kend();
  uint64_t tot = 0;
  HIPCHK(hipMemcpyAsync(&tot, off + nt, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int64_t n_emit = (int64_t)(tot & 0xffffffffull), n_carry = (int64_t)(tot >> 32);
  h->mark(3);
  // ---- 6. write
  AbsOut o;
  memset(&o, 0, sizeof(o));
  o.n_select = d.n_select;
  o.stride = 32 + 8 * d.n_select;
  o.base_index = bv.base_index;
  o.index = bv.index;
  for (int s = 0; s < d.n_select; ++s) {
    const int idx = d.sel_index[s];
    o.sel_ok[s] = d.sel_state[s] == a_state && (idx == 0 || idx == -1);
    o.sel_col[s] = d.ret_col[d.sel_ret[s]];
    o.sel_type[s] = d.sel_type[s];
  }
  char* rec = h->out.reserve(n_emit, d.n_select, st);
  char* dst = rec + (size_t)h->out.n * o.stride;
  if (a.keep_carry) cout.reserve(n_carry, d.n_select);
  uint32_t* slot_trig = (uint32_t*)h->ws.get("abs_slot_trig", 4 * (n_emit + 1), st);
  uint32_t* first_slot = (uint32_t*)h->ws.get("abs_first_slot", 4 * (n_emit + 1), st);
  h->kbeg("abs_write");
  if (n_emit > 0) {
    hipLaunchKernelGGL(k_abs_slot_trig, dim3(grid_for(nt)), dim3(256), 0, st, nt, cnt, off, trig, slot_trig);
    uint32_t* head = (uint32_t*)h->ws.get("abs_head", 4 * (n_emit + 1), st);
    hipLaunchKernelGGL(k_abs_heads, dim3(grid_for(n_emit)), dim3(256), 0, st, n_emit, slot_trig, head);
    size_t tb2 = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, tb2, head, first_slot, (size_t)n_emit, rocprim::maximum<uint32_t>(), st));
    void* tmp2 = h->ws.get("abs_head_scan_tmp", tb2, st);
    HIPCHK(rocprim::inclusive_scan(tmp2, tb2, head, first_slot, (size_t)n_emit, rocprim::maximum<uint32_t>(), st));
  }
  if (nt > 0)
    hipLaunchKernelGGL(k_abs_write, dim3(grid_for(nt)), dim3(256), 0, st, a, o, bv.cols, bv.ts, trig, cnt, off, vals,
                       role, cin, cout, first_slot, dst);
  if (n > 0) hipLaunchKernelGGL(k_abs_last, dim3(1), dim3(64), 0, st, n, bv.ts, as->dlast);
  HIPCHK(hipGetLastError());
  h->kend();
  h->mark(4);
  h->out.n += n_emit;
  if (a.keep_carry) {
    // the scheduler's FIFO above the clock (kill and creation entries of the push's last W), lastScheduledTime
    int64_t tlast = clock0;
    if (n > 0) HIPCHK(hipMemcpyAsync(&tlast, bv.ts + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int64_t clock1 = std::max(clock0, tlast);
    const int64_t ne_q = nq_in + n;
    uint32_t* qm = (uint32_t*)h->ws.get("abs_qm", 4 * (ne_q + 1), st);
    uint32_t* qo = (uint32_t*)h->ws.get("abs_qo", 4 * (ne_q + 1), st);
    hipLaunchKernelGGL(k_abs_qcount, dim3(grid_for(ne_q + 1)), dim3(256), 0, st, nq_in, qin.v, n, bv.ts, role, a.nc, kc,
                       a.W, clock1, qm);
    size_t tq = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tq, qm, qo, 0u, (size_t)ne_q + 1, rocprim::plus<uint32_t>(), st));
    void* tmpq = h->ws.get("abs_qscan_tmp", tq, st);
    HIPCHK(rocprim::exclusive_scan(tmpq, tq, qm, qo, 0u, (size_t)ne_q + 1, rocprim::plus<uint32_t>(), st));
    uint32_t nq1 = 0;
    HIPCHK(hipMemcpyAsync(&nq1, qo + ne_q, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    qout.reserve(std::max<int64_t>(nq1, 1));
    hipLaunchKernelGGL(k_abs_qwrite, dim3(grid_for(ne_q)), dim3(256), 0, st, nq_in, qin.v, n, bv.ts, a.W, qm, qo, qout.v);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    qout.n = nq1;
    // any value >= every queued entry acts alike: it is read only by a pass that emitted nothing (L < T), and new
    // entries overwrite it first
    as->lst = std::max(lst0, clock1 + a.W);
    cout.n = n_carry;
    as->seq = false;
    as->cur ^= 1;
  }
  return n;
}

void sg_run_every_absent(SgHandle* h, const BatchView& bv, int64_t n) {
  const sg_nfa_desc& d = h->desc;
  if (!sg_every_absent_supported(d)) {
    sg_run_general(h, bv, n);
    return;
  }
  const int64_t out0 = h->out.n;
  const bool fresh = h->pushes == 0 || h->opt.no_carry;
  int64_t lo = 0;
  do {   // segments: closed form, then the sequential pass from a late row until the closed form can resume, ...
    lo += absent_segment(h, sg_slice_view(d, bv, lo, n - lo), n - lo, lo == 0 && fresh,
                         lo > 0 || !h->opt.no_carry, !h->opt.no_carry);
  } while (lo < n);
  h->last_events = n;
  h->last_matches = h->out.n - out0;
  h->last_spilled = 0;
}

void sg_every_absent_reset(SgHandle* h) {
  if (h->state && h->state_kind == 3) {
    AbsState* as = (AbsState*)h->state;
    as->carry[0].n = as->carry[1].n = 0;
    as->q[0].n = as->q[1].n = 0;
    as->lst = 0;
    as->seq = false;
  }
}

void sg_every_absent_release(SgHandle* h) {
  if (!h->state || h->state_kind != 3) return;
  AbsState* as = (AbsState*)h->state;
  as->carry[0].release();
  as->carry[1].release();
  as->q[0].release();
  as->q[1].release();
  hipFree(as->dlast);
  hipFree(as->dminmax);
  hipFree(as->dflag);
  delete as;
  h->state = nullptr;
  h->state_kind = 0;
}

// Snapshot of the absence closed form: the pending partials in arrival order (deadline, compared value,
// projection) -- the Scheduler's ToNotifyQueue plus the absent pre-state's pending list
// (C/util/Scheduler.java:147-160, AbsentStreamPreStateProcessor's StreamPreStateProcessor.currentState
// C/query/input/stream/state/StreamPreStateProcessor.java:352-359) -- and the last timestamp seen.
void sg_every_absent_snapshot(SgHandle* h, SnapW& w) {
  AbsState* as = (h->state && h->state_kind == 3) ? (AbsState*)h->state : nullptr;
  const int64_t n = as ? as->carry[as->cur].n : 0;
  const int ns = std::max(h->desc.n_select, 1);
  w.pod(n);
  int64_t last = INT64_MIN;
  if (as && h->pushes > 0) {
    HIPCHK(hipMemcpyAsync(&last, as->dlast, 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  w.pod(last);
  // the scheduler's FIFO, lastScheduledTime, and whether the closed form can continue
  const int64_t nq = as ? as->q[as->cur].n : 0;
  w.pod(nq);
  w.pod(as ? as->lst : (int64_t)0);
  w.pod((int32_t)(as && as->seq ? 1 : 0));
  if (nq) w.dev(as->q[as->cur].v, nq * 8, h->stream);
  if (!n) return;
  const AbsCarry& c = as->carry[as->cur];
  w.dev(c.dl, n * 8, h->stream);
  w.dev(c.val, n * 8, h->stream);
  w.dev(c.vnul, n, h->stream);
  w.dev(c.sel, n * 8 * ns, h->stream);
  w.dev(c.snul, n * 4, h->stream);
}

void sg_every_absent_restore(SgHandle* h, SnapR& r) {
  AbsState* as = astate(h);
  const int ns = std::max(h->desc.n_select, 1);
  const int64_t n = r.pod<int64_t>();
  if (n < 0 || n >= (1ll << 31)) throw SgError(SG_EINVAL, "snapshot: bad pending-partial count");
  const int64_t last = r.pod<int64_t>();
  const int64_t nq = r.pod<int64_t>();
  if (nq < 0 || nq >= (1ll << 34)) throw SgError(SG_EINVAL, "snapshot: bad timer-queue length");
  as->lst = r.pod<int64_t>();
  as->seq = r.pod<int32_t>() != 0;
  as->carry[0].n = as->carry[1].n = 0;
  as->q[0].n = as->q[1].n = 0;
  HIPCHK(hipMemcpyAsync(as->dlast, &last, 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (nq) {
    as->q[as->cur].reserve(nq);
    r.dev(as->q[as->cur].v, nq * 8, h->stream);
    as->q[as->cur].n = nq;
  }
  if (!n) return;
  AbsCarry& c = as->carry[as->cur];
  c.reserve(n, h->desc.n_select);
  r.dev(c.dl, n * 8, h->stream);
  r.dev(c.val, n * 8, h->stream);
  r.dev(c.vnul, n, h->stream);
  r.dev(c.sel, n * 8 * ns, h->stream);
  r.dev(c.snul, n * 4, h->stream);
  c.n = n;
}
