/*
 * causeweave.h -- C ABI of the MI355X-native weave for Cause (tetriscode/cause).
 *
 * One library, libcauseweave.so (gfx950 HIP kernels, cause_amd/csrc/), replaces
 * the reference's `weave-fn` plug-in point for the reconstitute-from-nodes path:
 *
 *   c.list/weave 1-arity  (list.cljc:26-28)  -> cw_weave_lists  [weave order]
 *   c.list/hide?           (list.cljc:48-55)  -> cw_weave_lists  [visible_bits]
 *   c.list/causal-list->edn count (list.cljc:57-66, 77) -> visible_bits/_count
 *   s/spin 1-arity         (shared.cljc:121-132) -> cw_weave_lists [yarn_perm]
 *   s/refresh-ts           (shared.cljc:243-249) -> cw_weave_lists [max_ts]
 *   s/refresh-caches       (shared.cljc:259-266) = all of the above in one call
 *
 * The JVM shim calls it from c.list/weave's 1-arity and from
 * s/refresh-caches; insert/append/merge reach it through a full reweave.
 *
 * Conventions
 *  - Plain pointers and sizes, no torch/HIP types.  Every buffer is owned by the
 *    caller; the library keeps nothing after a call returns except reusable
 *    device scratch inside the context.
 *  - Ids are order-preserving packed 64-bit keys (cause_amd/pack.py):
 *      key(a) < key(b)  <=>  (compare a b) < 0   (util.cljc:4-10)
 *    below 2^63 (K64); CW_NIL (all ones) is nil and is reserved (root's cause).
 *    Ids that need more bits take the K128 layout (cw_weave_lists_k128).
 *  - A document's nodes may come in any order (the ::nodes hash map,
 *    shared.cljc:62).  The root [[0 "0" 0] nil nil] (shared.cljc:22-23) is one
 *    of them, flagged CW_KIND_ROOT.
 *  - Return value: 0 ok, < 0 error (cw_last_error has the text).  Per-document
 *    problems are reported in status[] instead (CW_STATUS_*).  ROOT, ORPHAN,
 *    NON_LAMPORT and WEFT mark documents the reference's s/insert would refuse
 *    (shared.cljc:163-178) but its full reweave accepts (list.cljc:26-28): the
 *    library reweaves them by the literal fold (exact path) and their outputs
 *    are the reference's.  DUP, MAP_KEY, KEY_RANGE and INTERNAL documents
 *    cannot be a ::nodes map of the reference or a K64 key; their outputs are
 *    well-formed but unspecified.
 *  - A context is not thread-safe; use one context per host thread.  Calls are
 *    re-entrant with respect to each other's inputs (pure functions; swap!
 *    retries may repeat them).
 */
#ifndef CAUSEWEAVE_H
#define CAUSEWEAVE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CW_ABI_VERSION 1
#define CW_NIL UINT64_MAX
#define CW_MAP_ID_KEY (1ull << 63) /* map key weave keyed by an id */

/* Node value class (shared.cljc:21 special-keywords) | CW_KIND_ROOT. */
enum {
  CW_KIND_NORMAL = 0,
  CW_KIND_HIDE = 1,   /* :causal/hide   */
  CW_KIND_HHIDE = 2,  /* :causal/h.hide */
  CW_KIND_HSHOW = 3,  /* :causal/h.show */
  CW_KIND_ROOT = 4
};

/* Per-document status bits. */
enum {
  CW_STATUS_ROOT = 1u << 0,        /* no root, several roots, or root not the smallest id */
  CW_STATUS_DUP = 1u << 1,         /* two nodes share an id (shared.cljc:166-171)          */
  CW_STATUS_ORPHAN = 1u << 2,      /* a cause is not in the document (shared.cljc:175-178) */
  CW_STATUS_NON_LAMPORT = 1u << 3, /* a cause id is not older than its node                */
  CW_STATUS_MAP_KEY = 1u << 4,     /* map: a key token >= 2^token_bits                      */
  CW_STATUS_INTERNAL = 1u << 5,    /* consistency check failed inside the pipeline         */
  CW_STATUS_WEFT = 1u << 6,        /* weft: a cut id is not a node of the document         */
  CW_STATUS_KEY_RANGE = 1u << 7,   /* an id key >= 2^63: it does not fit the K64 layout
                                      (CW_NIL and its neighbours are reserved); weave the
                                      document with cw_weave_lists_k128                     */
  CW_STATUS_UNWOVEN = 1u << 8      /* reserved, never set since ABI round 4: every document
                                      the reference folds is woven (exact path); kept so
                                      client code that tests the bit still compiles         */
};

/* Where the arrays of a batch/result live. */
enum { CW_MEM_HOST = 0, CW_MEM_DEVICE = 1 };

typedef struct cw_ctx cw_ctx;

/* ABI version (CW_ABI_VERSION). */
int cw_abi_version(void);
/* Build id of this library: a hash of its sources (Makefile).  Counter tables
 * under profiles/ name the build they were measured on. */
const char *cw_build_id(void);

/* Create a context on HIP device `device` (its own stream).  0 on success. */
int cw_ctx_create(int device, cw_ctx **out);
void cw_ctx_destroy(cw_ctx *ctx);
/* Text of the last error on this context ("" if none). */
const char *cw_last_error(const cw_ctx *ctx);
/* Launch on an existing HIP stream (hipStream_t passed as void*); NULL restores
 * the context's own stream. */
int cw_ctx_set_stream(cw_ctx *ctx, void *hip_stream);
/* 0: synchronous calls (default).  1: device-memory calls return without a
 * final stream synchronisation (the caller synchronises the stream before it
 * reads the results).  They are NOT fully asynchronous: a call may wait on the
 * stream for a few bytes the host needs to pick the next kernels.
 *  - cw_weave_lists / _k32 (batches of documents < 2^16 nodes, the fused
 *    per-document kernel): one blocking 8-byte readback right after that
 *    kernel -- whether a document's ids left its rank directory (the batch is
 *    then rewoven by the separate kernels) and whether the exact path has
 *    documents to fix.  The call returns while the yarn kernel (yarn_perm) and
 *    any later kernel still run; work queued on the stream BEFORE the call
 *    is waited for too.
 *  - the other front ends wait likewise once for their 8-byte directory
 *    flag; one giant document (>= 2^22 nodes) waits for its 4-byte status.
 *  - cw_weave_maps, cw_partition_keys and the out-of-domain (exact) path read
 *    back counts they size later launches with.
 * A caller that wants to overlap host work with the weave should run it on
 * its own thread or queue the weave behind no other work. */
int cw_ctx_set_async(cw_ctx *ctx, int async);
/* Per-kernel timing with HIP events on the launch stream (event pairs are read
 * back when the stats are asked for; asynchronous calls stay asynchronous). */
int cw_ctx_set_profiling(cw_ctx *ctx, int on);
/* Restrict the per-kernel events to one kernel stat name (NULL or "" = every
 * kernel): a sub-millisecond call is then timed with two events instead of
 * two per launch. */
int cw_ctx_set_profile_only(cw_ctx *ctx, const char *kernel);

typedef struct {
  char name[48];
  uint64_t launches;
  double total_ms;     /* sum of event-measured durations                */
  double bytes_alg;    /* algorithmic HBM bytes over all launches */
} cw_kernel_stat;

/* Copies up to `cap` stats; returns how many kernels have stats. */
int cw_get_kernel_stats(const cw_ctx *ctx, cw_kernel_stat *out, int cap);
int cw_reset_kernel_stats(cw_ctx *ctx);
/* Diagnostic counter of the last call on this context (waits for the stream):
 * "continued_sublists" = sublists the last HBM walk (one-list / giant path)
 * opened because a walker's slot filled up.  0 on success, < 0 for an
 * unknown name. */
int cw_get_counter(cw_ctx *ctx, const char *name, uint64_t *value);

/* ---------------------------------------------------------------- lists ---- */
typedef struct {
  uint64_t n_docs;
  const uint64_t *doc_offsets; /* HOST memory, [n_docs+1], doc d = [off[d], off[d+1]) */
  const uint64_t *id_key;      /* [N] packed id of each node                           */
  const uint64_t *cause_key;   /* [N] packed cause id (CW_NIL for the root)            */
  const uint8_t *kind;         /* [N] CW_KIND_*                                        */
  uint32_t key_bits;           /* significant bits of id keys; 0 = find on the device   */
  uint32_t ts_shift;           /* lamport-ts = id_key >> ts_shift                       */
  uint32_t site_shift;         /* site rank = (id_key >> site_shift) & (2^site_bits-1)  */
  uint32_t site_bits;          /* 0 = no yarn output                                    */
} cw_list_batch;

typedef struct {
  uint32_t *weave_perm;    /* [N]: position doc_off[d]+p holds the doc-local input index
                              of the node at weave position p (root at p = 0)          */
  uint32_t *visible_bits;  /* [(N+31)/32]: bit g (word g/32, bit g%32) set iff global
                              weave position g renders (not hide?, list.cljc:48-55)     */
  uint32_t *visible_count; /* [n_docs] count of rendered nodes (list.cljc:77)          */
  uint64_t *max_ts;        /* [n_docs] ::lamport-ts after refresh-ts, or NULL         */
  uint32_t *status;        /* [n_docs] CW_STATUS_* bits                                */
  uint32_t *yarn_perm;     /* [N] or NULL: doc-local input indices grouped by site rank,
                              id-ascending inside a site (the ::yarns cache)            */
} cw_list_result;

/* Full reweave of a batch of independent CausalLists (N = doc_offsets[n_docs]
 * < 2^32; in a batch of several documents each is < 2^29 - 1 nodes, a batch of
 * one document may hold up to 2^31 - 2).  `memspace` says where id_key /
 * cause_key / kind and every result array live (doc_offsets is always host). */
int cw_weave_lists(cw_ctx *ctx, const cw_list_batch *batch, cw_list_result *result,
                   int memspace);

/* K32: narrow keys.  The same batch as cw_list_batch with 4-byte id and cause
 * words, for batches whose packed ids fit 32 bits (config 2 needs 20): half the
 * input bytes over PCIe and in HBM.  The keys are widened on the device and
 * woven by cw_weave_lists' pipeline, so results and limits are cw_weave_lists'.
 * Keys are below CW_K32_RESERVED; the 16 values from there up stand for the
 * top 16 K64 values (CW_NIL32 = CW_NIL is a nil cause, CW_NIL32 - 1 a cause
 * that is no id). */
#define CW_NIL32 0xFFFFFFFFu
#define CW_K32_RESERVED 0xFFFFFFF0u
typedef struct {
  uint64_t n_docs;
  const uint64_t *doc_offsets; /* HOST memory, [n_docs+1]                                */
  const uint32_t *id_key;      /* [N] packed id of each node                             */
  const uint32_t *cause_key;   /* [N] packed cause id (CW_NIL32 for the root)            */
  const uint8_t *kind;         /* [N] CW_KIND_*                                          */
  uint32_t key_bits;           /* as cw_list_batch                                        */
  uint32_t ts_shift;
  uint32_t site_shift;
  uint32_t site_bits;
  uint32_t perm16;             /* 1: result->weave_perm is uint16_t[N] (every document
                                  < 65536 nodes; device memory only): half the bytes back */
} cw_list_batch_k32;

int cw_weave_lists_k32(cw_ctx *ctx, const cw_list_batch_k32 *batch, cw_list_result *result,
                       int memspace);

/* K128: ids that need more than 63 bits (ts:64 | site_rank:32 |
 * tx:32).  Every id is two u64 words, hi then lo:
 *     hi = lamport-ts (a nat-int Long, shared.cljc:31)
 *     lo = site_rank << 32 | tx-index   (site ranks in String.compareTo order)
 * so (hi, lo) compared as an unsigned 128-bit number is (compare a b)
 * (util.cljc:4-10).  A nil cause is (CW_NIL, CW_NIL).  Same documents, same
 * results as cw_weave_lists (weave order, rendered bits and counts, status,
 * the exact path for out-of-domain documents); max_ts is the largest id's hi
 * word and yarn_perm groups by the site rank in lo's high half.  The limits on
 * document and batch sizes are cw_weave_lists'. */
typedef struct {
  uint64_t n_docs;
  const uint64_t *doc_offsets; /* HOST memory, [n_docs+1]                                */
  const uint64_t *id_key;      /* [2N]: (hi, lo) of node i at [2i], [2i+1]                */
  const uint64_t *cause_key;   /* [2N]: (hi, lo) of its cause; (CW_NIL, CW_NIL) = nil      */
  const uint8_t *kind;         /* [N] CW_KIND_*                                           */
} cw_list_batch_k128;

int cw_weave_lists_k128(cw_ctx *ctx, const cw_list_batch_k128 *batch, cw_list_result *result,
                        int memspace);

/* ----------------------------------------------------------------- maps ---- */
/* Full reweave of a batch of CausalMaps (c.map/weave 1-arity, map.cljc:26-45)
 * and last-writer-wins per key (active-node, map.cljc:47-59).
 *
 * Each node's cause is either a packed id (cause_is_id = 1: (spec/valid? ::s/id
 * cause), map.cljc:31), a key token (cause_is_id = 0: an opaque key rank,
 * < 2^token_bits) or nil (cause_is_id = 2: the nil key, cause ignored).  A
 * key-caused node is woven under the key's virtual root [[0 "0" 0] nil nil]
 * (map.cljc:35-40), whose packed id is 0 (site "0" interns to rank 0, ts 0);
 * an id-caused node lands in the weave of its cause node's key (map.cljc:32-34).
 * The reference's quirky keys are reproduced: when the cause
 * node is itself id-caused by X the key is the id X (seg_key = CW_MAP_ID_KEY |
 * packed X), and when the cause node is absent the key is nil (seg_key =
 * CW_NIL).  Every key weave is a list weave; the active node is its first
 * rendered node, blank when the root's first child is a hide.  Key weaves are
 * returned per collection in ascending seg_key order.  Ids and tokens must fit
 * 62 bits.  Collections of <= 2048 nodes are woven by one kernel per pack of
 * collections (mappack.hip), larger ones by the general path (sorts, then every
 * key weave as a list document through the list pipeline).  Both fold key
 * weaves that are not a plain F5 tree -- the nil key weave holding nodes caused
 * by the root id or by nil next to appended orphans, a cause with a larger id
 * than its node, the id key weave of a self-caused id X (cause = id; X, its
 * children and grandchildren fold there by their real causes) -- literally
 * (shared.cljc:225-241), so every collection without
 * DUP / MAP_KEY comes out as the reference's fold; CW_STATUS_NON_LAMPORT stays
 * as information. */
typedef struct {
  uint64_t n_colls;
  const uint64_t *coll_offsets; /* HOST memory, [n_colls+1]                                */
  const uint64_t *id_key;       /* [N] packed ids (< 2^63)                                 */
  const uint64_t *cause;        /* [N] packed cause id, or key token                       */
  const uint8_t *cause_is_id;   /* [N] 1 = cause is an id, 0 = a key token, 2 = nil        */
  const uint8_t *kind;          /* [N] CW_KIND_* (no root: maps have a virtual root)      */
  uint32_t key_bits;            /* significant bits of id keys (0 = find on the device)   */
  uint32_t token_bits;          /* significant bits of key tokens                         */
} cw_map_batch;

typedef struct {
  uint64_t cap_segs;      /* IN: capacity of the per-key-weave arrays (N suffices)         */
  uint64_t n_segs;        /* OUT: number of key weaves                                     */
  uint64_t *seg_offsets;  /* [cap_segs+1]: key weave s = seg_perm[seg_offsets[s] ..)        */
  uint32_t *seg_coll;     /* [cap_segs] collection of key weave s                          */
  uint64_t *seg_key;      /* [cap_segs] key token of key weave s                           */
  int64_t *seg_active;    /* [cap_segs] collection-local input index of the active node,
                             -1 = ::blank                                                   */
  uint32_t *seg_perm;     /* [N + cap_segs] weave order of every key weave: the root
                             (UINT32_MAX) then collection-local input indices               */
  uint32_t *status;       /* [n_colls] CW_STATUS_* bits                                     */
} cw_map_result;

/* memspace: where id_key / cause / cause_is_id / kind and every result array
 * live (coll_offsets is always host memory; n_segs is returned in the struct).
 * On a nonzero return every result array holds unspecified values: a
 * device-memory call that repeats the previous call's collection count takes
 * that call's pack table on trust and checks the whole layout while the kernel
 * runs, so it may have written the outputs before it finds coll_offsets
 * invalid. */
int cw_weave_maps(cw_ctx *ctx, const cw_map_batch *batch, cw_map_result *result, int memspace);

/* ---------------------------------------------------------------- merge ---- */
/* Union of two node bags per document followed by a full reweave: the result
 * of s/merge-trees (shared.cljc:300-314) and of a bulk s/insert (:151-184),
 * which equal the full reweave of the union.  Per document d the
 * nodes of a (ct1) and b (ct2) are united by id:
 *   - the same id with the same body (cause, kind, value token) is kept once
 *     (insert's idempotency, shared.cljc:164-165);
 *   - the same id with another body sets CW_STATUS_DUP ("edits-not-allowed",
 *     :166-171);
 *   - a cause missing from the union sets CW_STATUS_ORPHAN
 *     ("cause-must-exist", :175-178).
 * The reference inserts ct2's nodes one at a time in hash-map order, so it can
 * also throw :cause-must-exist when a node of ct2 precedes its own cause in
 * that order; the union is what it returns whenever it does not throw. */
typedef struct {
  cw_list_batch a;          /* ct1's nodes per document (doc_offsets: host memory)   */
  const uint64_t *a_value;  /* [Na] value token: equal tokens <=> equal values       */
  cw_list_batch b;          /* ct2's nodes, same n_docs; key layout fields unused    */
  const uint64_t *b_value;  /* [Nb]                                                  */
} cw_merge_batch;

typedef struct {
  uint64_t *merged_offsets; /* HOST memory [n_docs+1]: merged doc d is
                               [merged_offsets[d], merged_offsets[d+1])              */
  uint32_t *merged_src;     /* [Na+Nb]: merged nodes in id order, as source indices:
                               s < na_d is a's doc-local s, else b's doc-local s-na_d */
  cw_list_result weave;     /* every array sized for Na+Nb (n_docs for the per-
                               document ones), laid out by merged_offsets; weave_perm
                               holds doc-local merged indices (into merged_src)      */
} cw_merge_result;

/* Host memory only (memspace must be CW_MEM_HOST in this version). */
int cw_merge_lists(cw_ctx *ctx, const cw_merge_batch *batch, cw_merge_result *result,
                   int memspace);

/* ----------------------------------------------------------------- weft ---- */
/* s/weft (shared.cljc:268-293), time travel: per document, the root and each
 * named site's yarn up to and including its cut id, nothing of the other
 * sites, then the full reweave.  cut[(d << site_bits) | site_rank] is the
 * packed cut id of that site, or 0 for a site that is not named (its nodes are
 * dropped).  A cut id that is not a node of the document keeps the site's
 * whole yarn (take-while never stops) plus the node (new-node [id nil]) =
 * [id] -- cause nil, its value (peek) the id itself -- which kept_src marks
 * UINT32_MAX; the document gets CW_STATUS_WEFT and its weave is still the
 * reference's (exact path).  Cuts that do not preserve causality leave
 * orphans ("gibberish trees"): CW_STATUS_ORPHAN, woven like the reference.
 * ::lamport-ts of the result is the largest cut ts (max_ts is the largest kept
 * id's ts: the caller takes the cuts' max).  Kept arrays need room for
 * N + (n_docs << site_bits) nodes. */
typedef struct {
  cw_list_batch nodes;   /* site_bits must be 1..10                           */
  const uint64_t *cut;   /* HOST memory [n_docs << site_bits]                */
} cw_weft_batch;

typedef struct {
  uint64_t *kept_offsets; /* HOST memory [n_docs+1]                          */
  uint32_t *kept_src;     /* [N + (n_docs << site_bits)]: doc-local input index of
                             each kept node, in input order, then UINT32_MAX for
                             each [id] node of a cut id that is not a node        */
  cw_list_result weave;   /* laid out by kept_offsets; weave_perm holds indices
                             into kept_src                                     */
} cw_weft_result;

/* Host memory only (memspace must be CW_MEM_HOST in this version). */
int cw_weft_lists(cw_ctx *ctx, const cw_weft_batch *batch, cw_weft_result *result, int memspace);

/* ------------------------------------ the distributed giant list (config 5) ---- */
/* Building blocks for one list spread over several GPUs (cause_amd/giant.py:
 * sample sort by RCCL all-to-all, cause lookup at the owner of the cause id,
 * then the tree and the tour on one GPU).  Device memory only; the calls are
 * ordered on the context's stream. */

#define CW_NOT_FOUND 0xFFFFFFFFu
#define CW_NIL_RANK 0xFFFFFFFEu /* the rank of a nil cause (cw_lookup_keys of CW_NIL) */

/* (sort ::nodes) of one document's ids (list.cljc:28, shared.cljc:128):
 * keys_out = keys ascending, idx_out[i] = input index of keys_out[i] (stable).
 * key_bits = 0: the library finds the significant bits.  n < 2^32 - 1. */
int cw_sort_keys(cw_ctx *ctx, const uint64_t *keys, uint64_t n, uint32_t key_bits,
                 uint64_t *keys_out, uint32_t *idx_out);

/* out[i] = base + index of queries[i] among the n ascending keys `sorted`, or
 * CW_NOT_FOUND (the cause join of s/insert, shared.cljc:175-178).  status
 * (device memory, or NULL): OR'ed with CW_STATUS_DUP when `sorted` repeats a
 * key -- an id held twice (::nodes is a map, shared.cljc:62, 166-171); the
 * check runs even when m = 0. */
int cw_lookup_keys(cw_ctx *ctx, const uint64_t *sorted, uint64_t n, const uint64_t *queries,
                   uint64_t m, uint32_t base, uint32_t *out, uint32_t *status);

/* Group m keys by bucket among n_split ascending splitters (bucket of x = the
 * number of splitters <= x; n_split <= 1023): perm lists the key indices
 * bucket by bucket (stable), counts[0..n_split] (HOST memory) the bucket
 * sizes.  Synchronous (the counts are read back). */
int cw_partition_keys(cw_ctx *ctx, const uint64_t *keys, uint64_t m, const uint64_t *splitters,
                      uint32_t n_split, uint32_t *perm, uint64_t *counts);
/* cw_partition_keys with counts[n_split + 1] in DEVICE memory: no host
 * readback inside the call (the ruling set's rounds hand the counts to the
 * next collective on the device; async contexts do not wait at all). */
int cw_partition_keys_dev(cw_ctx *ctx, const uint64_t *keys, uint64_t m, const uint64_t *splitters,
                          uint32_t n_split, uint32_t *perm, uint64_t *counts);

/* dst[i] = src[idx[i]], elements of elem_size 1, 4, 8 or 16 bytes. */
int cw_gather(cw_ctx *ctx, const void *src, const uint32_t *idx, uint64_t m, uint32_t elem_size,
              void *dst);

/* dst[idx[i]] = src[i] for 4-byte elements (idx a permutation of 0..m-1). */
int cw_scatter32(cw_ctx *ctx, const uint32_t *src, const uint32_t *idx, uint64_t m, uint32_t *dst);

/* One list handed over in id order (rank r = the r-th smallest id; rank 0 the
 * root): par[r] = rank of r's cause (par[0] ignored; CW_NOT_FOUND = orphan),
 * kind[r] as in cw_list_batch.  val[r] = the value emitted for rank r (NULL:
 * r itself).  result: weave_perm[g] = val of the node at weave position g,
 * visible_bits, visible_count[0], status[0]; yarn_perm and max_ts must be NULL
 * (they need the ids: the caller has them).  n <= 2^31 - 2. */
typedef struct {
  uint64_t n;
  const uint32_t *par;
  const uint8_t *kind;
  const uint32_t *val;
} cw_ranked_list;

int cw_weave_ranked(cw_ctx *ctx, const cw_ranked_list *list, cw_list_result *result);

/* The tree step by step on the rank owning global ranks [base, base + n) of
 * the list (cause_amd/giant.py): par / kind as cw_ranked_list
 * but for those ranks only; every array is this rank's, device memory.  The
 * caller routes the queries and records between the ranks. */
#define CW_DIST_PEND 0x80000000u /* eff word: the climb goes on at the rank in the low bits */
#define CW_DIST_NONE 0xFFFFFFFFu /* eff word of the root                                   */

/* cw_sort_keys for 32-bit keys (key_bits 0 = 32). */
int cw_sort_keys32(cw_ctx *ctx, const uint32_t *keys, uint64_t n, uint32_t key_bits,
                   uint32_t *keys_out, uint32_t *idx_out);
/* status (device, one word) |= ROOT / ORPHAN / NON_LAMPORT for this run. */
int cw_dist_check(cw_ctx *ctx, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                  uint32_t *status);
/* eff[i]: effective parent of base + i, or CW_DIST_PEND | the
 * first cause outside the run the climb through special causes reached. */
int cw_dist_eff(cw_ctx *ctx, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                uint32_t *eff);
/* Answers for climbs that reached this run: out[i] = the first non-special
 * node at or above q[i] inside the run, or CW_DIST_PEND | the next rank. */
int cw_dist_climb(cw_ctx *ctx, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                  const uint64_t *q, uint64_t m, uint32_t *out);
/* keys[i] = the rank the eff word w[i] waits on, UINT64_MAX when it waits on
 * nothing (for cw_partition_keys by owner); *count (device) = how many wait. */
int cw_dist_pending(cw_ctx *ctx, const uint32_t *w, uint64_t n, uint64_t *keys, uint32_t *count);
/* key[i] = eff << 1 | (non-special), 0xFFFFFFFF for the root. */
int cw_dist_gkey(cw_ctx *ctx, const uint32_t *eff, const uint8_t *kind, uint64_t n, uint32_t *key);
/* After a stable local sort of the group keys (skey, sidx): nsc = next
 * sibling inside each run; per run a record {group, oldest, newest, kind of
 * newest} (rec: 4 words per sorted position) and okey = its e (UINT64_MAX on
 * the other positions). */
int cw_dist_runs(cw_ctx *ctx, const uint32_t *skey, const uint32_t *sidx, uint64_t n, uint32_t base,
                 const uint8_t *kind, uint32_t *nsc, uint64_t *okey, uint32_t *rec);
/* key[i] = group of received record i (a stable sort by it, the records in
 * sender order, orders each group's runs by their oldest node). */
int cw_dist_rkey(cw_ctx *ctx, const uint32_t *rec, uint64_t m, uint32_t *key);
/* At the owner of the parents, records sorted by cw_dist_rkey's key: the
 * first children fcS / fcN of its nodes (zeroed before; fcS bit 31 = that
 * child is a hide) and reply[i] = the next sibling of record i's oldest node
 * (NSC_UP-style 0x80000000 | e when it has none). */
int cw_dist_link(cw_ctx *ctx, const uint32_t *skey, const uint32_t *sidx, uint64_t m,
                 const uint32_t *rec, uint32_t base, uint64_t n, uint32_t *fcS, uint32_t *fcN,
                 uint32_t *reply);
/* nsc[oldest of rec i - base] = reply[i]. */
int cw_dist_put(cw_ctx *ctx, const uint32_t *rec, const uint32_t *reply, uint64_t m, uint32_t base,
                uint64_t n, uint32_t *nsc);
/* Thread words from nsc (the preorder successor of a childless node): the
 * successor rank, or 0x80000000 | an ancestor outside the node's 1,024-rank
 * tile whose thread it is (resolved inside each tile by pointer jumping). */
int cw_dist_thr(cw_ctx *ctx, const uint32_t *nsc, uint64_t n, uint32_t base, uint32_t *thr);
/* out[i] = first child of base + i, or CW_DIST_FROM_THR (its thread), | the
 * render bit (bit 31). */
#define CW_DIST_FROM_THR 0x7FFFFFFEu
int cw_dist_succ(cw_ctx *ctx, const uint8_t *kind, const uint32_t *fcS, const uint32_t *fcN,
                 uint64_t n, uint32_t base, uint32_t *out);

/* Ruling-set list ranking of the distributed list: the list
 * is ranked where it lies instead of on one GPU.  Rulers: global rank 0 and
 * every rank g with mix32(seed, g) * k < 2^32; each walks its sublist.
 * Replaces the rank-0 walk of cw_weave_linked for W > 1 (cause_amd/giant.py).
 *
 * cw_dist_rs_rulers: word[2i..2i+1] = {next, ruler index} of base + i (next =
 * successor, resolved thread, CW_RS_CHASE | the ancestor whose thread it is,
 * or 0x7FFFFFFF at the end; ruler index among this run's rulers, or
 * CW_RS_NONE); rlist[j] = local index of ruler j; *count (device) = rulers.
 * cw_dist_rs_walk: one exchange round.  walkers: m records {ruler, count,
 * target, 0} received from other ranks, or NULL for the run's own rulers
 * (ruler index rbase + j, j < m).  Each walker numbers the nodes it visits
 * (own[2x..2x+1] = {ruler, offset}) until its list reaches another ruler or
 * the end (a record {ruler, next ruler or CW_RS_NONE, length, 0} appended at
 * links[4 * (*nlinks)]) or leaves the run: out[4i..] = {ruler, count, target,
 * 0}, key[i] = the target's global rank (UINT64_MAX for a walker that
 * stopped), for cw_partition_keys by owner.  status |= CW_STATUS_INTERNAL on
 * a walk past its step bound.
 * cw_dist_rs_top (one GPU, all m = number of rulers links): pos[r] = weave
 * position of ruler r; status |= CW_STATUS_INTERNAL unless the links form
 * one list from ruler 0 over `total` nodes.
 * cw_dist_rs_pos: rec[2i..] = {position, val[i] | render bit << 31} of base
 * + i; key[i] = the position (key may be NULL).
 * cw_dist_rs_emit: at the owner of positions [p0, p0 + len): weave_perm,
 * visible_bits (from position p0, a multiple of 32) and *visible_count from m
 * records. */
#define CW_RS_CHASE 0x80000000u
#define CW_RS_NONE 0xFFFFFFFFu
int cw_dist_rs_rulers(cw_ctx *ctx, const uint32_t *succ, const uint32_t *thr, uint64_t n,
                      uint32_t base, uint32_t k, uint32_t seed, uint32_t *word, uint32_t *rlist,
                      uint32_t *count);
int cw_dist_rs_walk(cw_ctx *ctx, const uint32_t *walkers, uint64_t m, const uint32_t *rlist,
                    uint32_t rbase, const uint32_t *word, const uint32_t *thr, uint64_t n,
                    uint32_t base, uint32_t *own, uint32_t *links, uint32_t *nlinks, uint32_t *out,
                    uint64_t *key, uint32_t *status);
int cw_dist_rs_top(cw_ctx *ctx, const uint32_t *links, uint64_t m, uint64_t total, uint32_t *pos,
                   uint32_t *status);
int cw_dist_rs_pos(cw_ctx *ctx, const uint32_t *own, const uint32_t *pos_base, const uint32_t *succ,
                   const uint32_t *val, uint64_t n, uint32_t *rec, uint64_t *key);
int cw_dist_rs_emit(cw_ctx *ctx, const uint32_t *rec, uint64_t m, uint32_t p0, uint64_t len,
                    uint32_t *weave_perm, uint32_t *visible_bits, uint32_t *visible_count,
                    uint32_t *status);

/* One list given every node's successor word (cw_dist_succ) and thread word
 * (cw_dist_thr), in rank order; the walk chases pending threads.  val as
 * cw_ranked_list. */
typedef struct {
  uint64_t n;
  const uint32_t *succ;
  const uint32_t *thr;
  const uint32_t *val;
} cw_linked_list;

int cw_weave_linked(cw_ctx *ctx, const cw_linked_list *list, cw_list_result *result);

#ifdef __cplusplus
}
#endif
#endif /* CAUSEWEAVE_H */
