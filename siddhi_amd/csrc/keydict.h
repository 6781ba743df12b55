// Device key dictionary: raw 64-bit partition-key values -> dense ids in first-seen order, in HBM.
//
// The reference clones one query runtime per partition key the first time the key arrives
// (PartitionStreamReceiver.receive -> PartitionRuntime.cloneIfNotExist, C/partition/PartitionStreamReceiver.java:
// 80-275, C/partition/PartitionRuntime.java:255-308); the engine's kernels want that key as a dense id.  With a
// million keys the host dictionary is a random DRAM probe per event (the node's bottleneck); here the probe runs on
// the GPU against an open-addressing table that stays in HBM/MALL between chunks, and the host never touches a key.
//
// Per chunk (one stream of rows already in HBM):
//   probe   one thread per row: a known key resolves to its id; an unknown key claims a slot by CAS (its smallest
//           row index kept by atomicMin) and the row is marked pending;
//   order   the chunk's new keys sorted by first row (rocPRIM radix sort) get ids n_keys, n_keys + 1, ... -- the
//           first-seen order of the whole stream, chunk after chunk;
//   fill    pending rows look their key up again.
// A table that would pass half full is rebuilt 4x larger and the chunk re-probed (pending claims dropped).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

struct KeyDict {
  int64_t cap = 0;              // regular slots (power of two); slot `cap` holds the raw value KD_EMPTY itself
  int64_t n_keys = 0;
  int64_t* keys = nullptr;
  int32_t* vals = nullptr;      // dense id, -1 = claimed in the current chunk (pending); [cap]: INT32_MIN = unused
  uint32_t* first = nullptr;    // smallest row of a pending key in the current chunk
  int32_t* nslot = nullptr;     // slots claimed this chunk (list), then sorted by first row
  uint32_t* nfirst = nullptr;
  int32_t* sslot = nullptr;
  uint32_t* sfirst = nullptr;
  int64_t list_cap = 0;
  void* tmp = nullptr;          // radix sort temporary storage
  size_t tmp_bytes = 0;
  uint32_t* ctr = nullptr;      // device: [0] claims, [1] overflow bits
  uint32_t* hctr = nullptr;     // pinned host copy
  bool clear = true;            // (re)initialise before the next probe: a new stream
  int64_t probes = 0, rebuilds = 0;
};

// Resolve rows [0, n) of `raw` (device; rows whose `stream` entry is < 0 get -1) into dense ids in `key` (device),
// on stream `st` (synchronises it).  Returns the number of keys first seen in these rows; when `new_first` is given
// it receives their first rows, in id order.  Throws SgError.
int64_t kd_resolve(KeyDict& t, const int64_t* raw, const int32_t* stream, int64_t n, int32_t* key, hipStream_t st,
                   std::vector<uint32_t>* new_first);
void kd_reset(KeyDict& t);   // forget every key (the table is cleared lazily, on the next resolve)
void kd_free(KeyDict& t);
