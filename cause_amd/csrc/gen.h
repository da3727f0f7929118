/* gen.h -- synthetic multi-site edit histories for the weave benchmark and tests
 * (libcauseweave_gen.so).  Not part of the weave itself: it only produces input
 * node bags in the packed layout of include/causeweave.h.
 *
 * Each document: the root plus `nodes_per_doc` nodes typed by `n_sites` sites.
 *   - op mix: hide (p_hide, caused by a random currently-visible node),
 *     h.show (p_show, caused by a random hidden node), otherwise a character
 *   - a character's cause: the current LAST weave node (p_conj, the conj- shape
 *     of list.cljc:36-40, which may be a hide -> "dirty" documents), else the
 *     site's previous character (p_chain), else a uniformly random earlier
 *     non-special node (root included)
 *   - lamport: ts = 1 + max(site clock, cause ts); all site clocks sync to the
 *     maximum every `sync_every` ops (0 = never)
 *   - node order inside the document is shuffled (hash-map order) if `shuffle`
 * Ids pack as ts << site_bits | site_rank (tx-index 0); site rank 0 is the
 * root's "0", the typing sites are ranks 1..n_sites.
 * Document d is seeded with splitmix64(seed ^ d): any shard reproduces it.
 */
#ifndef CAUSEWEAVE_GEN_H
#define CAUSEWEAVE_GEN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t nodes_per_doc; /* non-root nodes per document */
  uint32_t n_sites;
  double p_hide, p_show, p_conj, p_chain;
  uint32_t sync_every;
  uint64_t seed;
  int shuffle;
} cwg_params;

/* Packed layout: ts_bits, site_bits (tx_bits = 0). */
void cwg_layout(const cwg_params *p, uint32_t *ts_bits, uint32_t *site_bits);

/* Generate documents [doc_begin, doc_end) into flat arrays of
 * (doc_end-doc_begin)*(nodes_per_doc+1) entries.  Returns 0 on success. */
int cwg_generate(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, uint64_t *id_key,
                 uint64_t *cause_key, uint8_t *kind, int nthreads);
/* The same documents with K32 keys (cw_weave_lists_k32; nil = 0xFFFFFFFF). */
int cwg_generate32(const cwg_params *p, uint64_t doc_begin, uint64_t doc_end, uint32_t *id_key,
                   uint32_t *cause_key, uint8_t *kind, int nthreads);

/* Maps: each collection holds `nodes_per_coll` nodes
 * typed by `n_sites` sites over `n_keys` key tokens drawn Zipf(zipf_s):
 *   - key-level :causal/hide (p_hide, cause = the key token, dissoc-)
 *   - id-caused :causal/h.hide (p_hhide) / :causal/h.show (p_hshow), cause = a
 *     random earlier value write of the collection (undo/redo)
 *   - otherwise a value write (cause = the key token, assoc-)
 *   - p_bad: id-caused nodes whose cause is itself id-caused
 * cause_is_id[i] says whether cause[i] is a packed id or a key token. */
typedef struct {
  uint32_t nodes_per_coll;
  uint32_t n_sites;
  uint32_t n_keys;
  double zipf_s;
  double p_hide, p_hhide, p_hshow, p_bad;
  uint32_t sync_every;
  uint64_t seed;
  int shuffle;
} cwg_map_params;

void cwg_map_layout(const cwg_map_params *p, uint32_t *ts_bits, uint32_t *site_bits,
                    uint32_t *token_bits);
int cwg_map_generate(const cwg_map_params *p, uint64_t coll_begin, uint64_t coll_end,
                     uint64_t *id_key, uint64_t *cause, uint8_t *cause_is_id, uint8_t *kind,
                     int nthreads);

#ifdef __cplusplus
}
#endif
#endif
