// Host-side engine state shared by the MI355X kernels' launch code (engine.hip, interp.hip, absent.hip)
// and the C-ABI (api.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_gpu.h"
#include "sg_device.h"

typedef sg_nfa_desc DevDesc;

struct SgError {
  int code;
  std::string msg;
  SgError(int c, std::string m) : code(c), msg(std::move(m)) {}
};

// Named, grow-only device workspaces (no allocation in steady state).
struct Workspace {
  struct Buf { void* p = nullptr; size_t bytes = 0; };
  std::map<std::string, Buf> bufs;
  void* get(const std::string& name, size_t bytes, hipStream_t st) {
    Buf& b = bufs[name];
    if (bytes == 0) bytes = 16;
    if (b.bytes < bytes) {
      if (b.p) {
        hipStreamSynchronize(st);
        hipFree(b.p);
      }
      size_t want = bytes + bytes / 4;
      if (hipMalloc(&b.p, want) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc failed for workspace " + name);
      b.bytes = want;
    }
    return b.p;
  }
  void release() {
    for (auto& kv : bufs) if (kv.second.p) hipFree(kv.second.p);
    bufs.clear();
  }
};

// Pending match records in HBM, AoS, in delivery order (layout: sg_match_records).
struct OutStore {
  int64_t n = 0, cap = 0;
  int nsel = 0;
  int stride = 32;
  char* rec = nullptr;
  char* reserve(int64_t extra, int n_select, hipStream_t st) {
    nsel = n_select;
    stride = 32 + 8 * n_select;
    int64_t need = n + extra;
    if (need > cap) {
      int64_t nc = std::max<int64_t>(need + need / 4, 1024);
      void* np = nullptr;
      if (hipMalloc(&np, (size_t)nc * stride) != hipSuccess) throw SgError(SG_EHIP, "hipMalloc failed for match store");
      if (rec && n) hipMemcpyAsync(np, rec, (size_t)n * stride, hipMemcpyDeviceToDevice, st);
      hipStreamSynchronize(st);
      if (rec) hipFree(rec);
      rec = (char*)np;
      cap = nc;
    }
    return rec;
  }
  void release() {
    if (rec) hipFree(rec);
    rec = nullptr;
    n = cap = 0;
  }
  void consume(int64_t k, hipStream_t st);
};

struct BatchView {
  int64_t n;
  uint64_t base_index;
  const int64_t* ts;
  const int32_t* stream;
  const int32_t* key;
  const uint64_t* index;
  SgCols cols;
  int32_t key_bound;
};

struct SgHandle {
  int device = 0;
  sg_nfa_desc desc;
  sg_options opt;
  DevDesc* ddesc = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  Workspace ws;
  OutStore out;
  OutStore stage;             // base records of the running push when select expressions follow (desc.n_out > 0)
  std::string err;
  hipEvent_t ev[8] = {};
  hipStream_t copy_stream = nullptr;            // host-batch ingress (sg_push, on_device = 0)
  hipEvent_t ev_copied[2] = {}, ev_consumed[2] = {};
  struct Egress {                               // SoA match delivery (sg_poll_columns / sg_push_deliver)
    hipStream_t d2h = nullptr;
    char* stage[2] = {};
    int64_t cap[2] = {};
    hipEvent_t ready[2] = {}, done[2] = {};
  } eg;
  int64_t last_events = 0, last_matches = 0, last_spilled = 0;
  int pushes = 0;
  uint64_t gen = 0;           // state generation: bumped by every push / reset / restore
  std::vector<char> snap_cache;   // blob of the last size query (sg_snapshot), valid while gen == snap_gen
  uint64_t snap_gen = ~0ull;
  uint32_t key_bound_seen = 0;
  int64_t ts_max_seen = INT64_MIN;   // largest timestamp pushed so far (sg_options.bounded_lateness)
  void* state = nullptr;      // per-shape persistent state (interp / absent)
  int state_kind = 0;         // 1 every->next closed form, 2 general machine, 3 absence closed form, 4 once closed form
  int split_out = 0;          // 1: output stage timed from ev[5] (host work between ev[3] and ev[5])
  int extra_marks = 0;        // 1: ev[6]..ev[7] hold an extra match-stage interval (overflow re-pass)
  void mark(int k) { hipEventRecord(ev[k], stream); }
  // per-kernel HIP events on the launch stream (sg_timing.kernel_ms): kbeg/kend bracket one kernel or group
  hipEvent_t km[SG_MAX_KMARKS][2] = {};
  const char* km_name[SG_MAX_KMARKS] = {};
  int n_km = 0;
  void kbeg(const char* name) {
    if (n_km >= SG_MAX_KMARKS) return;
    if (!km[n_km][0]) { hipEventCreate(&km[n_km][0]); hipEventCreate(&km[n_km][1]); }
    km_name[n_km] = name;
    hipEventRecord(km[n_km][0], stream);
  }
  void kend() {
    if (n_km >= SG_MAX_KMARKS) return;
    hipEventRecord(km[n_km][1], stream);
    ++n_km;
  }
  void bump_gen() {   // any state change invalidates the serialised-state cache of sg_snapshot
    ++gen;
    if (!snap_cache.empty()) { std::vector<char>().swap(snap_cache); snap_gen = ~0ull; }
  }
};



// Snapshot blob writer / reader (sg_snapshot / sg_restore).  Device sections are copied synchronously on the
// handle's stream; the reader throws SG_EINVAL on a truncated or mismatching blob.
struct SnapW {
  std::vector<char> b;
  void put(const void* p, size_t n) {
    size_t o = b.size();
    b.resize(o + n);
    if (n) memcpy(b.data() + o, p, n);
  }
  template <class T> void pod(const T& v) { put(&v, sizeof(T)); }
  void dev(const void* dp, size_t n, hipStream_t st) {
    size_t o = b.size();
    b.resize(o + n);
    if (!n) return;
    if (hipMemcpyAsync(b.data() + o, dp, n, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      throw SgError(SG_EHIP, "snapshot: device copy failed");
  }
};
struct SnapR {
  const char* p;
  const char* e;
  const char* take(size_t n) {
    if ((size_t)(e - p) < n) throw SgError(SG_EINVAL, "snapshot blob truncated");
    const char* q = p;
    p += n;
    return q;
  }
  template <class T> T pod() {
    T v;
    memcpy(&v, take(sizeof(T)), sizeof(T));
    return v;
  }
  void dev(void* dp, size_t n, hipStream_t st) {
    const char* q = take(n);
    if (!n) return;
    if (hipMemcpyAsync(dp, q, n, hipMemcpyHostToDevice, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      throw SgError(SG_EHIP, "restore: device copy failed");
  }
};
void sg_every_next_snapshot(SgHandle* h, SnapW& w);
void sg_every_next_restore(SgHandle* h, SnapR& r);
void sg_every_absent_snapshot(SgHandle* h, SnapW& w);
void sg_every_absent_restore(SgHandle* h, SnapR& r);
void sg_general_snapshot(SgHandle* h, SnapW& w);
void sg_general_restore(SgHandle* h, SnapR& r);

// Ingress / egress building blocks of the C-ABI (api.hip), shared with the node pipeline (node.hip).
// Device buffers of one ingress slot (resolved on the calling thread: the workspace map is not thread-safe).
struct SlotPtrs {
  void* ts = nullptr;
  void* stream = nullptr;
  void* key = nullptr;
  void* index = nullptr;
  void* col[SG_MAX_COLS] = {};
  void* nul[SG_MAX_COLS] = {};
};
struct ColLayout {   // SoA staging layout of `cap` delivered matches
  int ns;
  int32_t width[SG_MAX_SELECT];
  size_t off_trig, off_ts, off_key, off_grp, off_col[SG_MAX_SELECT], off_nul[SG_MAX_SELECT], bytes;
};
int sg_col_width(int type);
SlotPtrs sg_reserve_slot(SgHandle& h, const sg_batch* b, int64_t rows, int slot);
// copy rows [lo, lo + cnt) of a host batch into a slot on stream `st` (touches no handle state: any thread)
BatchView sg_upload_to(const sg_nfa_desc& d, const SlotPtrs& p, const sg_batch* b, int64_t lo, int64_t cnt,
                       hipStream_t st);
void sg_push_view(SgHandle& h, BatchView& bv, int64_t n);   // one push of rows in HBM (engine route + select)
BatchView sg_slice_view(const sg_nfa_desc& d, const BatchView& bv, int64_t lo, int64_t cnt);   // rows [lo, lo + cnt)
ColLayout sg_col_layout(const sg_nfa_desc& d, int64_t cap);
// egress staging slot `slot` of h holds at least `bytes` (grows after the slot's last copy has read it; api.hip)
void sg_stage_reserve(SgHandle& h, int slot, int64_t bytes);
void sg_launch_to_columns(int64_t n, const char* rec, int stride, const ColLayout& L, char* stage, hipStream_t st);
void sg_egress_init(SgHandle& h);

void sg_run_every_next(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_next_f32(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_next_f64(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_next_i32(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_next_i64(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_next_reset(SgHandle* h);
void sg_every_next_release(SgHandle* h);
void sg_run_general(SgHandle* h, const BatchView& bv, int64_t n);
// SG_SHAPE_NEXT_CMP_ONCE (once.hip): state_kind 4
void sg_run_once(SgHandle* h, const BatchView& bv, int64_t n);
void sg_once_reset(SgHandle* h);
void sg_once_release(SgHandle* h);
void sg_once_snapshot(SgHandle* h, SnapW& w);
void sg_once_restore(SgHandle* h, SnapR& r);
void sg_run_every_absent(SgHandle* h, const BatchView& bv, int64_t n);
void sg_every_absent_reset(SgHandle* h);
void sg_every_absent_release(SgHandle* h);
void sg_general_reset(SgHandle* h);
void sg_general_release(SgHandle* h);
// partial-lane route of the general machine (partial.hip, chain.h)
struct PartialState;
PartialState* sg_partial_new(const sg_nfa_desc& d);   // nullptr: the query is outside the route (sg_pp_rule)
void sg_partial_free(PartialState* ps);
void sg_partial_reset(PartialState* ps);
int sg_partial_active(const PartialState* ps);
void sg_partial_deactivate(PartialState* ps);
int sg_partial_push(SgHandle* h, PartialState* ps, const BatchView& bv, int64_t n, uint32_t key_bound);
int64_t sg_partial_max_rows(SgHandle* h, PartialState* ps);
int64_t sg_partial_carried(const PartialState* ps);   // rows carried into the next push
void sg_partial_snapshot(SgHandle* h, PartialState* ps, SnapW& w);
void sg_partial_restore(SgHandle* h, PartialState* ps, SnapR& r);
