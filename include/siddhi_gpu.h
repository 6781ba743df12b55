/*
 * siddhi_gpu.h — C-ABI of the MI355X pattern/sequence state engine.
 *
 * Drop-in boundary for Siddhi's state-engine hot path.  One handle = one HIP device = one
 * cloned-per-key state query (all partition keys of that query live in the handle).  A handle is
 * single-threaded (mirrors `synchronized receive`, C/query/input/MultiProcessStreamReceiver.java:103);
 * handles on different devices may be driven concurrently.
 *
 * What each entry point replaces in the reference (C/ = modules/siddhi-core/src/main/java/io/siddhi/core/):
 *   sg_open          StateInputStreamParser.parseInputStream (C/util/parser/StateInputStreamParser.java:76-141)
 *                    + QueryRuntime/StateStreamRuntime.setCommonProcessor/init (C/query/input/stream/state/
 *                    StateStreamRuntime.java:73-76): the lowered NFA (sg_nfa_desc) replaces the Pre/Post
 *                    processor graph; per-key runtimes are created on first sight of a key
 *                    (PartitionRuntime.cloneIfNotExist, C/partition/PartitionRuntime.java:255-308).
 *   sg_push          StreamJunction.Receiver.receive(Event[]) / receive(long, Object[])
 *                    (C/stream/StreamJunction.java:376-389) as implemented by ProcessStreamReceiver
 *                    (C/query/input/ProcessStreamReceiver.java:43-223), MultiProcessStreamReceiver
 *                    (C/query/input/MultiProcessStreamReceiver.java:98-309) and PartitionStreamReceiver
 *                    (C/partition/PartitionStreamReceiver.java:80-275); InputHandler.send's playback clock
 *                    (C/stream/input/InputHandler.java:57-65) is applied per row.
 *   sg_advance_time  TimestampGeneratorImpl.setCurrentTimestamp (C/util/timestamp/TimestampGeneratorImpl.java:106-125)
 *                    driving Scheduler.sendTimerEvents (C/util/Scheduler.java:179-214) for `not ... for T`.
 *   sg_poll          QuerySelector.process -> OutputRateLimiter.sendToCallBacks
 *                    (C/query/selector/QuerySelector.java:76-163, C/query/output/ratelimit/OutputRateLimiter.java:61-100):
 *                    projected matches in the reference's delivery order.
 *   sg_snapshot      SiddhiAppRuntime.snapshot (C/SiddhiAppRuntime.java:613-623) -> SnapshotService.fullSnapshot
 *                    (C/util/snapshot/SnapshotService.java:97-157) for this query's Snapshotables: the pending /
 *                    newAndEvery lists of every pre-state processor (StreamPreStateProcessor.currentState,
 *                    C/query/input/stream/state/StreamPreStateProcessor.java:352-359), the scheduler's
 *                    ToNotifyQueue (C/util/Scheduler.java:147-152) and every partition clone's copy of them
 *                    (C/partition/PartitionRuntime.java:342-356).
 *   sg_restore       SiddhiAppRuntime.restore (C/SiddhiAppRuntime.java:625-635) -> SnapshotService.restore
 *                    (:271-345) / restoreState of the same objects (StreamPreStateProcessor.java:361-367,
 *                    Scheduler.java:154-160).
 *   sg_close         SiddhiAppRuntime.shutdown for the query's state.
 * No exceptions cross the ABI: every call returns SG_OK or a negative status; sg_last_error() explains.
 */
#ifndef SIDDHI_GPU_H
#define SIDDHI_GPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Checked on every sg_nfa_desc and written into every snapshot.  3: sg_options.no_grow; the general route's
   snapshots carry SgGeo with off_scratch (version-2 snapshots and bindings are refused). */
#define SG_ABI_VERSION 4

#define SG_MAX_STATES 16
#define SG_MAX_STREAMS 16
#define SG_MAX_SELECT 32
#define SG_MAX_RET 16
#define SG_MAX_COLS 64
#define SG_MAX_CODE 512

/* status codes */
#define SG_OK 0
#define SG_EINVAL -1
#define SG_EHIP -2
#define SG_ECAPACITY -3     /* a per-key pool / list capacity (sg_options) was exceeded */
#define SG_EUNSUPPORTED -4
#define SG_EORDER -5        /* sg_merge_runs: a run is not ordered by trigger */

/* state kinds (Pre/Post processor pairs) */
#define SG_K_STREAM 0       /* StreamPre/PostStateProcessor */
#define SG_K_COUNT 1        /* CountPre/PostStateProcessor */
#define SG_K_LOGICAL 2      /* LogicalPre/PostStateProcessor */
#define SG_K_ABSENT 3       /* AbsentStreamPre/PostStateProcessor */
#define SG_K_ALOGICAL 4     /* AbsentLogicalPre/PostStateProcessor: the `not S [for T]` side of a logical state */

/* attribute types (Attribute.Type) */
#define SG_T_STRING 0       /* dictionary id, int32 */
#define SG_T_INT 1
#define SG_T_LONG 2
#define SG_T_FLOAT 3
#define SG_T_DOUBLE 4
#define SG_T_BOOL 5         /* int32 0/1 */

/* closed-form shapes recognised at lowering time */
#define SG_SHAPE_GENERAL 0
#define SG_SHAPE_EVERY_NEXT_CMP 1    /* every A[l] -> B[l' and B.x OP A.x] within T */
#define SG_SHAPE_EVERY_ABSENT_EQ 2   /* every A[l] -> not B[l' and B.x == A.x] for T  (playback) */
#define SG_SHAPE_NEXT_CMP_ONCE 3     /* A[l] -> B[l' and B.x OP A.x] (within T), no `every`: one match per key */

/* postfix predicate program opcodes; words are int64 */
#define SG_OP_VAR 1     /* VAR state index_in_chain retained_slot type */
#define SG_OP_CONST 2   /* CONST type bits */
#define SG_OP_CMP 3     /* CMP op(0 == 1 != 2 > 3 >= 4 < 5 <=) domain(0 i64 1 f32 2 f64 3 id) */
#define SG_OP_AND 4
#define SG_OP_OR 5
#define SG_OP_NOT 6
#define SG_OP_ISNULL 7
#define SG_OP_MATH 8    /* MATH op(0 + 1 - 2 * 3 / 4 %) result_type: Java arithmetic, null on a null operand or a
                           zero divisor (C/executor/math/{add,subtract,multiply,divide,mod}/ *.java) */

typedef struct sg_state_desc {
  int32_t kind, stream, is_start, min_count, max_count, logical_type, partner;
  int32_t next_state;     /* post.nextStatePreProcessor (-1) */
  int32_t next_every;     /* post.nextEveryStatePreProcessor (-1) */
  int32_t within_every;   /* pre.withinEveryPreStateProcessor (-1; never set for partition clones) */
  int32_t callback;       /* post.callbackPreStateProcessor (count pre) (-1) */
  int32_t has_selector;   /* post.nextProcessor != null */
  int32_t this_last;      /* pre.thisLastProcessor = post of this state id */
  int32_t prog_off, prog_len, local;
  int64_t waiting_time;   /* absent: `for T` in ms (SG_K_ALOGICAL: -1 = `not S` without `for`) */
} sg_state_desc;

typedef struct sg_receiver_desc {
  int32_t stream, multi, selector, n;
  int32_t pres[SG_MAX_STATES];   /* nextProcessors in setNext (init) order */
  int32_t stab[SG_MAX_STATES];   /* stateProcessors in addStatefulProcessor order */
} sg_receiver_desc;

typedef struct sg_nfa_desc {
  int32_t abi_version;
  int32_t type;                  /* 0 PATTERN, 1 SEQUENCE */
  int64_t within;                /* ms, -1 = none */
  int32_t playback, partitioned;
  int32_t n_states, n_streams, n_cols, n_ret, n_select;
  int32_t n_init, n_reset, n_update, n_start;
  sg_state_desc states[SG_MAX_STATES];
  int32_t recv_of_stream[SG_MAX_STREAMS];      /* receiver index or -1 */
  sg_receiver_desc receivers[SG_MAX_STREAMS];
  int32_t init_order[SG_MAX_STATES];
  int32_t reset_ops[SG_MAX_STATES];
  int32_t update_ops[SG_MAX_STATES];
  int32_t start_ids[SG_MAX_STATES];
  int32_t col_type[SG_MAX_COLS], col_stream[SG_MAX_COLS];
  int32_t ret_col[SG_MAX_RET], ret_type[SG_MAX_RET];          /* retained slot -> batch column */
  int32_t sel_state[SG_MAX_SELECT], sel_index[SG_MAX_SELECT], sel_ret[SG_MAX_SELECT], sel_type[SG_MAX_SELECT];
  int32_t shape;
  int32_t shape_args[8];
  int32_t shape_prog_off, shape_prog_len;
  int32_t code_len;
  int64_t code[SG_MAX_CODE];
  /* Select expressions (QuerySelector over math executors, C/query/selector/QuerySelector.java:125-163):
   * n_out > 0 -> output column k is the postfix program code[out_off[k] .. +out_len[k]) over the n_select
   * projected slots (VAR operands: word 3 = slot); matches then carry n_out values of type out_type[k].
   * n_out == 0 -> the n_select projected slots are the output.
   * having_len > 0 -> matches whose program code[having_off ..) over the output columns is not TRUE are
   * dropped (QuerySelector.java:138-142); requires n_out > 0. */
  int32_t n_out;
  int32_t out_type[SG_MAX_SELECT], out_off[SG_MAX_SELECT], out_len[SG_MAX_SELECT];
  int32_t having_off, having_len;
  /* Schedulers (timer FIFOs) of the SG_K_ABSENT / SG_K_ALOGICAL states in their creation order
   * (StateInputStreamParser.java:167-185,290-320 for the app runtime; *InnerStateRuntime.clone order for
   * partition clones): timers of one clock advance fire scheduler by scheduler in this order. */
  int32_t n_sched;
  int32_t sched_state[SG_MAX_STATES];
} sg_nfa_desc;

typedef struct sg_options {
  int64_t max_batch;        /* largest n per sg_push the workspaces are sized for (grown on demand) */
  int32_t pool_partials;    /* general engine: partial-match (StateEvent) pool per key */
  int32_t pool_events;      /* general engine: retained event copies per key */
  int32_t pool_chain;       /* general engine: count-chain nodes per key */
  int32_t list_cap;         /* general engine: capacity of each pending / newAndEvery list */
  int32_t force_general;    /* 1: ignore closed-form shapes (parity testing of the general kernel) */
  int32_t no_carry;         /* 1: pushes are independent streams (no state carried between them) */
  int32_t ring_cap;         /* closed form: LDS pending-list ring per walker lane (power of two 2..256;
                               0 = chosen per push from the rows per `within` window) */
  int32_t chunk_rows;       /* general engine: a key's rows are cut into units of this many rows, each unit
                               rebuilding its state by replaying the rows inside the query's horizon before
                               it (0 = chosen per push, -1 = one unit per key) */
  int32_t walker_only;      /* closed form, unpartitioned streams: 1 = always the chunked walker instead of the
                               per-candidate search (testing both paths) */
  int32_t ingress_rows;     /* host batches (on_device = 0) are copied and processed in chunks of this many rows,
                               the copy of chunk k+1 overlapping the kernels of chunk k (0: 4 chunks for batches of
                               >= 32M rows, else one copy; -1: one copy); results are identical to one push.
                               no_carry handles never split. */
  int32_t partition_sort;   /* closed form, partitioned: 0 = LDS-staged counting partition when key_bound <= 65536
                               (rocPRIM radix sort above), 1 = always the radix sort (testing both paths) */
  int32_t partial_lanes;    /* general engine, patterns whose partial matches never interact (every e1 -> ... within T
                               over stream / count / logical states of one stream): 0 = one GPU lane per partial
                               match while timestamps never decrease, -1 = always the per-key machine (testing);
                               1 / 2 = lanes, matches ordered by the trigger-row sort plus in-place tie runs / by the
                               three LSD radix sorts even where one composed key would do (testing every order path) */
  int32_t no_grow;          /* general machine: 1 = a push that runs out of a key's pool / list / timer capacity or of
                               emission space fails with SG_ECAPACITY instead of being rolled back and rerun with 4x the
                               capacity (testing) */
  int32_t bounded_lateness; /* partial lanes: 1 = the caller guarantees that no row arrives more than max_lateness_ms
                               behind the largest timestamp pushed so far; a pending partial whose e1 lies further than
                               `within` before that bound can then never emit (every state it could still reach expires
                               it or needs a row inside `within` of e1), so it is not carried into the next push.
                               0 (default) = no bound: every pending partial is carried, as the reference keeps it
                               (CountPreStateProcessor never expires a count-waiting partial, CountPreStateProcessor.java:
                               53-93), and a stream of such partials grows the carry without bound */
  int64_t max_lateness_ms;  /* the bound when bounded_lateness = 1 (>= 0) */
} sg_options;

/* One SoA batch of input rows in arrival order.  Column c holds the typed values of (stream,attr)
 * c of sg_nfa_desc (rows of other streams are ignored).  Host pointers must stay valid until
 * sg_push returns; device pointers (on_device = 1) must be HBM buffers of the handle's device. */
typedef struct sg_batch {
  int64_t n;
  uint64_t base_index;          /* global event index of row 0 (the reference's send order) */
  const int64_t* ts;            /* event timestamps (ms) */
  const int32_t* stream;        /* stream index; -1 = row that only advances the playback clock */
  const int32_t* key;           /* dense partition key id (first-seen order); -1 = null key (dropped) */
  const uint64_t* index;        /* optional global event index per row (key-sharded sub-batches); NULL =
                                   base_index + row.  Must be increasing. */
  const void* const* cols;      /* [n_cols] typed columns (width from col_type) */
  const uint8_t* const* nulls;  /* [n_cols] optional 1-byte null flags per row, or NULL */
  int32_t on_device;
  int32_t key_bound;            /* exclusive upper bound of key ids in this batch (0 = unknown) */
} sg_batch;

/* Pending matches as they sit in HBM: n AoS records of record_bytes = 32 + 8*n_select bytes (n_select = the
 * output column count: sg_nfa_desc.n_out when set, else n_select),
 * {u64 trigger; i64 ts; i32 key; u32 group; u32 vnull; u32 pad; i64 vals[n_select]} (see sg_matches). */
typedef struct sg_match_records {
  int64_t n;
  int32_t record_bytes;
  int32_t n_select;
  void* base;
} sg_match_records;

/* Match tuples in delivery order.  vals[i*n_select + k] holds the bit pattern of select column k
 * (FLOAT: f32 bits, DOUBLE: f64 bits, others sign-extended); bit k of vnull[i] marks a null. */
typedef struct sg_matches {
  int64_t n;
  uint64_t* trigger;            /* global index of the event whose arrival produced the match */
  int64_t* ts;                  /* output event timestamp (StateEvent.timestamp) */
  int32_t* key;                 /* dense partition key */
  uint32_t* group;              /* callback batch: (phase << 24) | receiver visit slot */
  int64_t* vals;
  uint32_t* vnull;
} sg_matches;

/* Typed SoA delivery of match tuples (sg_poll_columns / sg_push_deliver): each non-NULL array receives one entry
 * per delivered match, in delivery order.  cols[k] is output column k (k < n_select of sg_match_records) as its
 * Attribute.Type: 4 bytes for INT / FLOAT / STRING id / BOOL, 8 bytes for LONG / DOUBLE; nulls[k] (optional)
 * one byte per row, 1 = null.  Pinned host memory (sg_host_alloc) makes the copies asynchronous DMA. */
typedef struct sg_match_columns {
  uint64_t* trigger;
  int64_t* ts;
  int32_t* key;
  uint32_t* group;
  void* cols[SG_MAX_SELECT];
  uint8_t* nulls[SG_MAX_SELECT];
} sg_match_columns;

#define SG_MAX_KMARKS 24
typedef struct sg_timing {
  float pred_ms, partition_ms, match_ms, output_ms, total_ms;   /* HIP-event times of the last push */
  int64_t events, matches;
  int64_t spilled_units;        /* closed form: (chunk, key) units whose pending list spilled to HBM */
  int32_t n_kernels;            /* per-kernel HIP-event times of the last push, recorded on the launch stream */
  float kernel_ms[SG_MAX_KMARKS];
  char kernel_name[SG_MAX_KMARKS][32];
} sg_timing;

typedef struct sg_handle sg_handle;

int sg_open(int hip_device, const sg_nfa_desc* nfa, const sg_options* opt, sg_handle** out);
int sg_push(sg_handle* h, const sg_batch* b);
int sg_advance_time(sg_handle* h, int64_t now, uint64_t trigger_index);
int sg_pending(sg_handle* h, int64_t* n);
/* Copy up to cap pending matches into host arrays (fields may be NULL to skip) and consume them. */
int sg_poll(sg_handle* h, sg_matches* out, int64_t cap, int64_t* n);
/* Copy up to cap pending matches, transposed on the GPU into typed SoA columns, into out (NULL arrays are
 * skipped) and consume them (QuerySelector -> QueryCallback.receiveStreamEvent delivery,
 * C/query/output/callback/QueryCallback.java:52-85, as columns). */
int sg_poll_columns(sg_handle* h, const sg_match_columns* out, int64_t cap, int64_t* n);
/* One call for a batch and its matches (InputHandler.send ... QueryCallback delivery,
 * C/stream/input/InputHandler.java:57-86): a host batch is copied in chunks (sg_options.ingress_rows), each
 * chunk's kernels run while the next chunk's columns are copied in, and each chunk's matches are transposed into
 * SoA columns and copied out into `out` while the next chunk computes; *n receives the number of rows written.
 * Matches pending before the call are delivered first.  If more than cap matches are produced, the surplus
 * stays pending (sg_pending / sg_poll_columns) and SG_ECAPACITY is returned after the whole batch ran. */
int sg_push_deliver(sg_handle* h, const sg_batch* b, const sg_match_columns* out, int64_t cap, int64_t* n);
/* Zero-copy view of the pending match records in HBM (valid until the next push/poll/reset). */
int sg_device_records(sg_handle* h, sg_match_records* view);
int sg_discard(sg_handle* h);           /* drop pending matches without copying */
int sg_flush(sg_handle* h);             /* wait for all work on the handle's stream */
int sg_reset(sg_handle* h);             /* forget all per-key state (fresh runtime) */
int sg_set_stream(sg_handle* h, void* hip_stream);   /* launch on a caller-owned hipStream_t */
int sg_get_timing(sg_handle* h, sg_timing* t);
/* Serialise the per-key state (partial matches, carried rows, timer queues) into buf; *size receives the
 * blob size (buf == NULL or cap < size: size query only, nothing copied).  SG_EINVAL while matches are
 * pending (poll or discard them first: the reference has delivered them before persist() can run). */
int sg_snapshot(sg_handle* h, void* buf, size_t cap, size_t* size);
/* Replace the handle's state by a blob from sg_snapshot of a handle opened with the same query and
 * options (SG_EINVAL otherwise); pending matches are dropped.  On error call sg_reset before reuse. */
int sg_restore(sg_handle* h, const void* buf, size_t size);
int sg_close(sg_handle* h);
const char* sg_last_error(const sg_handle* h);
/* Host partition router (router.cpp): replaces the per-event key lookup of PartitionStreamReceiver.receive /
 * PartitionRuntime.cloneIfNotExist (C/partition/PartitionStreamReceiver.java:80-275,
 * C/partition/PartitionRuntime.java:255-308) for SoA batches.  Raw partition-key values (64-bit: integers, float
 * bits, or string-dictionary ids) become dense ids in first-seen order (the reference's clone order); each key is
 * assigned to shard mix64(dense) mod n_shards (one shard per GPU) and gets a dense id inside its shard.  The
 * dictionary persists across calls.  threads = 0: all hardware threads. */
typedef struct sg_router sg_router;
int sg_router_open(int n_shards, int threads, sg_router** out);
int sg_router_route(sg_router* r, int64_t n, const int64_t* raw, int32_t* dense, int32_t* shard, int32_t* local);
int sg_router_keys(const sg_router* r, int64_t* n_keys, int32_t shard, int64_t* shard_keys);
int sg_router_close(sg_router* r);
/* The router's per-shard id table: dense_of_local[l] = node-wide dense id of shard `shard`'s key l (cap entries). */
int sg_router_dense_ids(const sg_router* r, int32_t shard, int32_t* dense_of_local, int64_t cap);
/* Merge match runs (each already in delivery order) into the node's delivery order by (trigger, phase = group >> 24,
 * dense key), ties in run order: out_src[i] = index of the i-th merged row in the concatenation of the runs.
 * group / key (and their entries) may be NULL (treated as 0).  SG_EORDER if a run is not ordered by trigger.
 * Replaces the single ordered stream QueryCallback.receive sees on one host (C/query/output/callback/
 * QueryCallback.java:52-85) for key-sharded engines. */
int sg_merge_order(int n_runs, const int64_t* run_len, const uint64_t* const* trigger, const uint32_t* const* group,
                   const int32_t* const* key, int threads, int64_t* out_src);

/* ---- Node pipeline: one host process drives the node's GPUs for one partitioned query ----------------------------
 * Replaces PartitionStreamReceiver.receive(Event[]) (C/partition/PartitionStreamReceiver.java:177-221) feeding the
 * per-key cloned runtimes (C/partition/PartitionRuntime.java:255-308) and the ordered delivery to QueryCallback
 * (C/query/output/callback/QueryCallback.java:52-85).  A host batch of raw rows goes in; the node routes each row by
 * its raw partition-key value (first-seen dense ids, shard = mix64(id) mod n_gpus), streams every shard's rows to its
 * GPU in chunks (H2D, kernels and D2H of consecutive chunks overlapped; state carried between chunks and pushes),
 * and merges the shards' matches into the reference's delivery order.  Unpartitioned queries run on one GPU
 * (replicas only).  A node is single-threaded like a handle; it starts one thread per GPU internally. */
#define SG_NODE_MAX_GPUS 16
typedef struct sg_node sg_node;
typedef struct sg_node_batch {
  int64_t n;
  uint64_t base_index;          /* global event index of row 0; consecutive pushes continue the index */
  const int64_t* ts;
  const int32_t* stream;        /* optional stream index per row; -1 = clock-only row (reaches every shard) */
  const int64_t* raw_key;       /* raw 64-bit partition-key value per row (integers, float bits, dictionary ids) */
  const void* const* cols;      /* [n_cols] typed host columns (NULL entries: not read by the query) */
  const uint8_t* const* nulls;  /* optional [n_cols] null flags */
} sg_node_batch;
typedef struct sg_node_stats {  /* of the last sg_node_push */
  double total_ms;              /* wall time of the pipeline (routing .. last merged row) */
  double reserve_ms;            /* buffer sizing before the pipeline (zero once sizes are stable) */
  double route_ms, merge_ms;    /* host thread-pool time spent routing / merging */
  double gpu_ms[SG_NODE_MAX_GPUS];   /* per GPU: compute-thread busy time */
  int64_t rows, matches, chunks, chunk_rows, h2d_bytes, d2h_bytes;
  int64_t shard_rows[SG_NODE_MAX_GPUS];   /* rows each GPU has received since open/reset */
} sg_node_stats;
/* chunk_rows 0: about 16 chunks per push (4M..25M rows each); host_threads 0: all hardware threads.
 * With several GPUs and the device key dictionary, rows are sharded, exchanged and merged on the GPUs (each GPU uploads
 * a contiguous slice of the batch; peer copies between GPUs); queries with playback timers route and merge on the host.
 * One GPU, closed-form queries (`every A -> B[..]`): out->ts and B-attribute columns are filled on the host from the
 * batch's trigger rows instead of being copied back from the GPU. */
int sg_node_open(int n_gpus, const int* devices, const sg_nfa_desc* nfa, const sg_options* opt, int host_threads,
                 int64_t chunk_rows, sg_node** out);
/* Push a batch; its matches (node delivery order) go to out rows [0, *n).  out->trigger is required; other NULL
 * arrays are skipped.  SG_ECAPACITY if more than cap matches: the node must then be reset. */
int sg_node_push(sg_node* nd, const sg_node_batch* b, const sg_match_columns* out, int64_t cap, int64_t* n);
int sg_node_reset(sg_node* nd);   /* new stream: forget keys and per-key state */
/* Where partition keys are dictionary-encoded (first-seen dense ids, PartitionRuntime.cloneIfNotExist,
 * C/partition/PartitionRuntime.java:255-308): 0 auto (the device whenever the query has no playback timers, else
 * the host), 1 the host
 * router (sg_router), 2 one dictionary per GPU in HBM (raw keys are uploaded; with several GPUs rows go to shard
 * mix64(raw) mod n_gpus).  Only before the first push of a stream. */
int sg_node_set_key_dict(sg_node* nd, int mode);
int sg_node_stats_get(const sg_node* nd, sg_node_stats* st);
int sg_node_keys(const sg_node* nd, int64_t* n_keys);
int sg_node_close(sg_node* nd);
const char* sg_node_last_error(const sg_node* nd);

/* Pinned host memory for batch columns (the ingress then copies asynchronously at full PCIe rate). */
int sg_host_alloc(size_t bytes, void** p);
int sg_host_free(void* p);
const char* sg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SIDDHI_GPU_H */
