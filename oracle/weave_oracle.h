/*
 * weave_oracle.h -- CPU restatement of Cause's weave (TEST INFRASTRUCTURE ONLY).
 *
 * This header declares the C oracle used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the *checker* of the HIP weave.  Nothing in the
 * product path (cause_amd/, include/, libcauseweave.so) may include, link or
 * call it.
 *
 * Parity status: the reference (tetriscode/cause) is Clojure and cannot be run in
 * this image (no JVM).  The restatement is pinned against the reference's own
 * known-answer tests (list_test.cljc, map_test.cljc) and idempotence properties
 * through tests/test_oracle.py; see DESIGN.md "Oracle".
 *
 * Domain: ids are order-preserving packed 64-bit keys (see cause_amd/pack.py):
 *   key(id) < key(id')  <=>  (compare id id') < 0      (util.cljc:4-10)
 * OR_NIL stands for Clojure nil (root's cause, (first nil), (second nil)).
 */
#ifndef CAUSE_WEAVE_ORACLE_H
#define CAUSE_WEAVE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_NIL UINT64_MAX

/* kind byte: bits 0-1 value class, bit 2 root flag.  special-keywords =
 * {:causal/hide :causal/h.hide :causal/h.show}  (shared.cljc:21) */
enum { OR_NORMAL = 0, OR_HIDE = 1, OR_HHIDE = 2, OR_HSHOW = 3, OR_ROOT = 4 };

/* Per-document status bits (same values as CW_STATUS_* in include/causeweave.h). */
enum {
  OR_ST_ROOT = 1u << 0,        /* root missing / not the smallest id / several roots */
  OR_ST_DUP = 1u << 1,         /* two nodes with the same id                        */
  OR_ST_ORPHAN = 1u << 2,      /* a cause id that is not in the document            */
  OR_ST_NON_LAMPORT = 1u << 3  /* cause id >= node id                                */
};

/* ---- lists (single document) ------------------------------------------------
 * All take the document's nodes in ARBITRARY order (the ::nodes map,
 * shared.cljc:62) and write out_perm[n] = input index of the node at each weave
 * position.  Return value: status bits (0 = in domain). */

/* Literal fold: (reduce weave [] (sort nodes)) with weave-node exactly as
 * shared.cljc:194-241 (clauses A, B, C and seen-since-asap), list.cljc:26-28. */
uint32_t or_list_fold_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm);

/* Incremental literal insertion in the given order (reduce c/insert ...):
 * weave-node of each node into the current weave, list.cljc:29-34.  order[k] is
 * an input index; order[0] must be the root. */
uint32_t or_list_insert_sequence(size_t n, const uint64_t *id, const uint64_t *cause,
                                 const uint8_t *kind, const uint32_t *order,
                                 uint32_t *out_perm);

/* linked-list fold (insert after cause; a non-special skips the
 * special run that follows).  O(n) after the sort. */
uint32_t or_list_fold_linked(size_t n, const uint64_t *id, const uint64_t *cause,
                             const uint8_t *kind, uint32_t *out_perm);

/* preorder of the effective tree (specials keep their cause as
 * parent; a non-special climbs through special causes; children: specials by
 * descending id, then non-specials by descending id). */
uint32_t or_list_eff_preorder(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm);

/* The full reweave for ANY causes (orphans, non-Lamport causes, nil causes, a
 * missing root): the rule of the product's exact path, stated on sorted nodes
 * and checked against or_list_fold_literal by the tests. */
uint32_t or_list_fold_general(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm);

/* Literal hide? over a weave (list.cljc:48-55 with partition 2 1 [nil],
 * list.cljc:57-66): vis[p] = 1 iff the node at weave position p is rendered. */
void or_list_visible_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                             const uint8_t *kind, const uint32_t *perm, uint8_t *vis);

/* Yarns (shared.cljc:112-132): nodes grouped by site ascending, id ascending
 * inside a site.  site(key) = (key >> site_shift) & site_mask. */
void or_list_yarns(size_t n, const uint64_t *id, unsigned site_shift, uint64_t site_mask,
                   uint32_t *yarn_perm);

/* ---- batches ---------------------------------------------------------------
 * method: 0 literal, 1 linked, 2 effective-tree, 3 general.  offsets[ndocs+1] index the
 * flat arrays.  out_perm is doc-local (input index inside the document);
 * out_vis[g] is per weave position (one byte each); out_status[d]. */
int or_batch_lists(size_t ndocs, const uint64_t *offsets, const uint64_t *id,
                   const uint64_t *cause, const uint8_t *kind, int method, int nthreads,
                   uint32_t *out_perm, uint8_t *out_vis, uint32_t *out_status);

/* ---- maps (single collection) ------------------------------------------------
 * cause[i] is either a packed id (cause_is_id[i] = 1: spec/valid? ::s/id,
 * map.cljc:31), an opaque key token (cause_is_id[i] = 0) or nil (cause_is_id[i]
 * = 2: the nil key, under its root).  Each key weave is a
 * list weave starting at [root-node] (map.cljc:40) whose root id is root_id.
 * Outputs, per node: node_key[i] = key token of the weave it lands in (OR_NIL
 * for a nil key), node_pos[i] = 1-based position in that weave.  Per key weave
 * (in order of first appearance in id order): seg_key[s], seg_active[s] = input
 * index of active-node (map.cljc:47-59) or -1 for ::blank.  Returns the number
 * of key weaves. */
size_t or_map_fold_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                           const uint8_t *cause_is_id, const uint8_t *kind, uint64_t root_id,
                           uint64_t *node_key, uint32_t *node_pos, uint64_t *seg_key,
                           int64_t *seg_active);

#ifdef __cplusplus
}
#endif
#endif
