// TEST INFRASTRUCTURE ONLY: standalone drivers for AddressSanitizer / UndefinedBehaviorSanitizer builds of the
// host-side C++ -- the CPU oracle (oracle/oracle.cpp), the host build of the GPU's per-key machine
// (tests/host_interp/harness.cpp over siddhi_amd/csrc/interp.h) and the C-ABI partition router
// (siddhi_amd/csrc/router.cpp).  Executables (not libraries loaded into Python), so the sanitizer runtime is
// linked in and nothing has to be preloaded.  tests/test_sanitizers.py records engine calls from Python into a
// case file, runs the matching driver on it and compares the driver's outputs with the unsanitised build's.
//
// Case file (little-endian): "SGCASE01", then cases until EOF; each case:
//   i64 image_words, i64 image[image_words]   (oracle: lowering.oracle_image; interp: raw sg_nfa_desc bytes)
//   i64 n_sel, i64 n_cols, i64 width[n_cols], i64 n_batches, then per batch:
//   i64 n, u64 base_index, i64 has_index, i64 ts[n], i32 stream[n], i32 key[n], [u64 index[n]],
//   per column: bytes[n * width], i64 has_null, [u8 null[n]]
// Output file: per case i64 n, u64 trigger[n], i64 ts[n], i32 key[n], u32 group[n], i64 vals[n * n_sel],
//   then (oracle) u8 vnull[n * n_sel] or (interp) u32 vnull[n].
// Router mode: argv = router <n_shards> <threads> <in: i64 n, i64 raw[n] per call until EOF> <out>
//   output per call: i32 dense[n], i32 shard[n], i32 local[n]; then i64 n_keys and per shard i64 keys.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/siddhi_gpu.h"

#if defined(SAN_ORACLE)
extern "C" {
struct OrcHandle;
OrcHandle* orc_create(const int64_t* image, int64_t n, char* err, int errlen);
void orc_destroy(OrcHandle* h);
int orc_push(OrcHandle* h, int64_t n, uint64_t base_index, const int64_t* ts, const int32_t* stream, const int32_t* key,
             const uint64_t* index, const void* const* cols, const uint8_t* const* nulls, char* err, int errlen);
int64_t orc_output_count(OrcHandle* h);
int64_t orc_fetch(OrcHandle* h, int64_t cap, uint64_t* trigger, int64_t* ts, int32_t* key, uint32_t* group,
                  int64_t* vals, uint8_t* vnull);
}
#elif defined(SAN_INTERP)
extern "C" {
struct HiHandle;
HiHandle* hi_open(const sg_nfa_desc* d, int P, int E, int C, int L);
void hi_close(HiHandle* h);
void hi_set_chunk(HiHandle* h, int chunk_rows);
int hi_push(HiHandle* h, const sg_batch* b);
int64_t hi_count(HiHandle* h);
void hi_fetch(HiHandle* h, uint64_t* trig, int64_t* ts, int32_t* key, uint32_t* group, int64_t* vals, uint32_t* vnull);
}
#endif

namespace {

[[noreturn]] void die(const std::string& m) {
  fprintf(stderr, "driver: %s\n", m.c_str());
  exit(2);
}

struct Reader {
  FILE* f;
  bool eof() {
    int c = fgetc(f);
    if (c == EOF) return true;
    ungetc(c, f);
    return false;
  }
  void raw(void* p, size_t n) {
    if (n && fread(p, 1, n, f) != n) die("truncated input");
  }
  int64_t i64() {
    int64_t v;
    raw(&v, 8);
    return v;
  }
  template <class T> std::vector<T> vec(int64_t n) {
    if (n < 0 || n > (int64_t)1 << 31) die("bad length");
    std::vector<T> v((size_t)n);
    raw(v.data(), sizeof(T) * (size_t)n);
    return v;
  }
};

template <class T> void put(FILE* o, const std::vector<T>& v) {
  if (!v.empty() && fwrite(v.data(), sizeof(T), v.size(), o) != v.size()) die("write failed");
}

struct Batch {
  int64_t n;
  uint64_t base;
  std::vector<int64_t> ts;
  std::vector<int32_t> stream, key;
  std::vector<uint64_t> index;
  std::vector<std::vector<char>> cols;
  std::vector<std::vector<uint8_t>> nulls;
  std::vector<const void*> colp;
  std::vector<const uint8_t*> nulp;
};

#if defined(SAN_ORACLE) || defined(SAN_INTERP)
int run_cases(const char* in, const char* out) {
  FILE* fi = fopen(in, "rb");
  FILE* fo = fopen(out, "wb");
  if (!fi || !fo) die("cannot open files");
  Reader r{fi};
  char magic[8];
  r.raw(magic, 8);
  if (memcmp(magic, "SGCASE01", 8) != 0) die("bad magic");
  int cases = 0;
  while (!r.eof()) {
    const int64_t iw = r.i64();
    std::vector<int64_t> image = r.vec<int64_t>(iw);
    const int64_t nsel = r.i64(), ncols = r.i64();
    std::vector<int64_t> width = r.vec<int64_t>(ncols);
    const int64_t nb = r.i64();
    std::vector<Batch> bs((size_t)nb);
    for (Batch& b : bs) {
      b.n = r.i64();
      b.base = (uint64_t)r.i64();
      const int64_t has_index = r.i64();
      b.ts = r.vec<int64_t>(b.n);
      b.stream = r.vec<int32_t>(b.n);
      b.key = r.vec<int32_t>(b.n);
      if (has_index) b.index = r.vec<uint64_t>(b.n);
      for (int64_t c = 0; c < ncols; ++c) {
        b.cols.push_back(r.vec<char>(b.n * width[c]));
        if (r.i64()) b.nulls.push_back(r.vec<uint8_t>(b.n));
        else b.nulls.emplace_back();
      }
      for (int64_t c = 0; c < ncols; ++c) {
        b.colp.push_back(b.cols[c].data());
        b.nulp.push_back(b.nulls[c].empty() ? nullptr : b.nulls[c].data());
      }
    }
#if defined(SAN_ORACLE)
    char err[512] = {0};
    OrcHandle* h = orc_create(image.data(), iw, err, sizeof(err));
    if (!h) die(std::string("orc_create: ") + err);
    for (Batch& b : bs)
      if (orc_push(h, b.n, b.base, b.ts.data(), b.stream.data(), b.key.data(), b.index.empty() ? nullptr : b.index.data(),
                   b.colp.data(), b.nulp.data(), err, sizeof(err)) != 0)
        die(std::string("orc_push: ") + err);
    const int64_t n = orc_output_count(h);
    std::vector<uint64_t> tr((size_t)n);
    std::vector<int64_t> ts((size_t)n), vals((size_t)(n * nsel));
    std::vector<int32_t> ky((size_t)n);
    std::vector<uint32_t> gr((size_t)n);
    std::vector<uint8_t> vn((size_t)(n * nsel));
    if (n) orc_fetch(h, n, tr.data(), ts.data(), ky.data(), gr.data(), vals.data(), vn.data());
    orc_destroy(h);
#else
    sg_nfa_desc d;
    if ((size_t)iw * 8 < sizeof(d)) die("short descriptor");
    memcpy(&d, image.data(), sizeof(d));
    HiHandle* h = hi_open(&d, 256, 256, 256, 256);
    if (!h) die("hi_open failed");
    for (Batch& b : bs) {
      sg_batch sb;
      memset(&sb, 0, sizeof(sb));
      sb.n = b.n;
      sb.base_index = b.base;
      sb.ts = b.ts.data();
      sb.stream = b.stream.data();
      sb.key = b.key.data();
      sb.index = b.index.empty() ? nullptr : b.index.data();
      sb.cols = b.colp.data();
      sb.nulls = b.nulp.data();
      if (hi_push(h, &sb) != 0) die("hi_push failed");
    }
    const int64_t n = hi_count(h);
    std::vector<uint64_t> tr((size_t)n);
    std::vector<int64_t> ts((size_t)n), vals((size_t)(n * (nsel ? nsel : 1)));
    std::vector<int32_t> ky((size_t)n);
    std::vector<uint32_t> gr((size_t)n), vn((size_t)n);
    hi_fetch(h, tr.data(), ts.data(), ky.data(), gr.data(), vals.data(), vn.data());
    vals.resize((size_t)(n * nsel));
    hi_close(h);
#endif
    fwrite(&n, 8, 1, fo);
    put(fo, tr);
    put(fo, ts);
    put(fo, ky);
    put(fo, gr);
    put(fo, vals);
    put(fo, vn);
    ++cases;
  }
  fclose(fi);
  fclose(fo);
  fprintf(stderr, "driver: %d cases\n", cases);
  return 0;
}
#endif

#if defined(SAN_ROUTER)
int run_router(int shards, int threads, const char* in, const char* out) {
  FILE* fi = fopen(in, "rb");
  FILE* fo = fopen(out, "wb");
  if (!fi || !fo) die("cannot open files");
  Reader r{fi};
  sg_router* rt = nullptr;
  if (sg_router_open(shards, threads, &rt) != SG_OK) die("sg_router_open");
  while (!r.eof()) {
    const int64_t n = r.i64();
    std::vector<int64_t> raw = r.vec<int64_t>(n);
    std::vector<int32_t> dense((size_t)n), shard((size_t)n), local((size_t)n);
    if (sg_router_route(rt, n, raw.data(), dense.data(), shard.data(), local.data()) != SG_OK) die("sg_router_route");
    put(fo, dense);
    put(fo, shard);
    put(fo, local);
  }
  int64_t nk = 0;
  sg_router_keys(rt, &nk, -1, nullptr);
  fwrite(&nk, 8, 1, fo);
  for (int s = 0; s < shards; ++s) {
    int64_t k = 0;
    sg_router_keys(rt, nullptr, s, &k);
    fwrite(&k, 8, 1, fo);
  }
  sg_router_close(rt);
  fclose(fi);
  fclose(fo);
  return 0;
}
#endif

}  // namespace

int main(int argc, char** argv) {
#if defined(SAN_ROUTER)
  if (argc != 5) die("usage: driver <n_shards> <threads> <in> <out>");
  return run_router(atoi(argv[1]), atoi(argv[2]), argv[3], argv[4]);
#else
  if (argc != 3) die("usage: driver <case file> <out file>");
  return run_cases(argv[1], argv[2]);
#endif
}
