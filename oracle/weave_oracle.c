/*
 * weave_oracle.c -- CPU restatement of Cause's weave.  TEST INFRASTRUCTURE ONLY:
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  Never linked into or called by the product path.
 *
 * Every function cites the reference (tetriscode/cause @ /root/reference) lines
 * it restates.  The reference cannot run here (Clojure, no JVM): this restatement
 * is pinned by the reference's own known-answer tests (tests/test_oracle.py).
 */
#include "weave_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t id;     /* packed [lamport-ts site-id tx-index]           */
  uint64_t cause;  /* packed cause id, OR_NIL for root (nil)          */
  uint32_t idx;    /* input index inside the document                 */
  uint8_t kind;    /* OR_NORMAL/HIDE/HHIDE/HSHOW | OR_ROOT            */
} lnode;

static inline int is_special(uint8_t k) { return (k & 3u) != 0; } /* shared.cljc:21 */
static inline int is_hide(uint8_t k) { return (k & 3u) == OR_HIDE || (k & 3u) == OR_HHIDE; }

static int cmp_lnode(const void *a, const void *b) {
  const lnode *x = (const lnode *)a, *y = (const lnode *)b;
  if (x->id != y->id) return x->id < y->id ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* Lists of at least this many nodes sort by LSD radix passes and find their
 * causes by one merge against the sorted ids (the same answers as qsort and
 * a binary search a node, O(n) passes instead: one list of 5e8 nodes is
 * checked in minutes, not hours). */
#define OR_RADIX_MIN 16384
#define OR_RADIX_BITS 11

static unsigned sig_bits(uint64_t x) {
  unsigned b = 0;
  while (x) { b++; x >>= 1; }
  return b;
}

/* Stable LSD radix sort of n records of `size` bytes by their u64 at offset 0
 * (the records' own order breaks ties); returns the sorted copy, frees the other. */
static void *radix_by_u64(void *a, size_t n, size_t size, unsigned bits) {
  void *t = malloc((n ? n : 1) * size);
  size_t *cnt = (size_t *)malloc(sizeof(size_t) << OR_RADIX_BITS);
  const size_t nb = (size_t)1 << OR_RADIX_BITS;
  for (unsigned sh = 0; sh < bits; sh += OR_RADIX_BITS) {
    memset(cnt, 0, sizeof(size_t) * nb);
    const char *src = (const char *)a;
    for (size_t i = 0; i < n; i++) cnt[(*(const uint64_t *)(src + i * size) >> sh) & (nb - 1)]++;
    size_t run = 0;
    for (size_t b = 0; b < nb; b++) {
      const size_t c = cnt[b];
      cnt[b] = run;
      run += c;
    }
    char *dst = (char *)t;
    for (size_t i = 0; i < n; i++) {
      const char *e = src + i * size;
      memcpy(dst + cnt[(*(const uint64_t *)e >> sh) & (nb - 1)]++ * size, e, size);
    }
    void *x = a;
    a = t;
    t = x;
  }
  free(t);
  free(cnt);
  return a;
}

/* (sort (::s/nodes ct)) -- list.cljc:28.  Map entries compare by key first and
 * ids are unique map keys, so this is an id sort (ties only for DUP docs,
 * kept in input order either way). */
static lnode *sorted_nodes(size_t n, const uint64_t *id, const uint64_t *cause,
                           const uint8_t *kind) {
  lnode *s = (lnode *)malloc((n ? n : 1) * sizeof(lnode));
  uint64_t mx = 0;
  for (size_t i = 0; i < n; i++) {
    s[i].id = id[i];
    s[i].cause = cause[i];
    s[i].idx = (uint32_t)i;
    s[i].kind = kind[i];
    if (id[i] > mx) mx = id[i];
  }
  if (n < OR_RADIX_MIN) qsort(s, n, sizeof(lnode), cmp_lnode);
  else s = (lnode *)radix_by_u64(s, n, sizeof(lnode), sig_bits(mx));
  return s;
}

/* lower_bound over the sorted ids; returns n when absent. */
static size_t find_id(const lnode *s, size_t n, uint64_t key) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t mid = lo + (hi - lo) / 2;
    if (s[mid].id < key) lo = mid + 1; else hi = mid;
  }
  return (lo < n && s[lo].id == key) ? lo : n;
}

/* Every rank's cause as a rank: find_id(s, n, s[r].cause) for each r, n when
 * absent.  Large lists: the (cause, rank) pairs radix-sorted by cause (causes
 * past the largest id clamped to one value: all absent) and merged against the
 * sorted ids. */
typedef struct {
  uint64_t c;
  uint64_t r;
} crec;
static uint32_t *cause_ranks(const lnode *s, size_t n) {
  uint32_t *cr = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
  if (n < OR_RADIX_MIN) {
    for (size_t r = 0; r < n; r++) cr[r] = (uint32_t)find_id(s, n, s[r].cause);
    return cr;
  }
  const uint64_t top = s[n - 1].id + 1 ? s[n - 1].id + 1 : s[n - 1].id;
  crec *a = (crec *)malloc(n * sizeof(crec));
  for (size_t r = 0; r < n; r++) {
    a[r].c = s[r].cause < top ? s[r].cause : top;
    a[r].r = r;
  }
  a = (crec *)radix_by_u64(a, n, sizeof(crec), sig_bits(top));
  size_t j = 0;
  for (size_t k = 0; k < n; k++) {
    const uint64_t c = a[k].c;
    while (j < n && s[j].id < c) j++;
    cr[a[k].r] = (uint32_t)(j < n && s[j].id == c && c == s[a[k].r].cause ? j : n);
  }
  free(a);
  return cr;
}

/* Domain checks shared with the HIP path (CW_STATUS_*); cr = cause_ranks. */
static uint32_t doc_status(const lnode *s, size_t n, const uint32_t *cr) {
  uint32_t st = 0;
  if (n == 0 || !(s[0].kind & OR_ROOT)) st |= OR_ST_ROOT;
  for (size_t r = 0; r < n; r++) {
    if (r > 0 && (s[r].kind & OR_ROOT)) st |= OR_ST_ROOT;
    if (r > 0 && s[r].id == s[r - 1].id) st |= OR_ST_DUP;
    if (r == 0) continue;
    if (cr[r] == n) st |= OR_ST_ORPHAN;
    else if (s[r].cause >= s[r].id) st |= OR_ST_NON_LAMPORT;
  }
  return st;
}

/* ---- seen-since-asap: a generation-stamped hash set of ids ----------------- */
typedef struct {
  uint64_t *key;
  uint32_t *gen;
  size_t mask;
  uint32_t cur;
} seenset;

static void seen_init(seenset *S, size_t n) {
  size_t cap = 16;
  while (cap < 2 * n + 2) cap <<= 1;
  S->key = (uint64_t *)calloc(cap, sizeof(uint64_t));
  S->gen = (uint32_t *)calloc(cap, sizeof(uint32_t));
  S->mask = cap - 1;
  S->cur = 0;
}
static void seen_free(seenset *S) { free(S->key); free(S->gen); }
static inline size_t seen_hash(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
  return (size_t)k;
}
static void seen_add(seenset *S, uint64_t k) {
  size_t h = seen_hash(k) & S->mask;
  while (S->gen[h] == S->cur) {
    if (S->key[h] == k) return;
    h = (h + 1) & S->mask;
  }
  S->gen[h] = S->cur;
  S->key[h] = k;
}
static int seen_has(const seenset *S, uint64_t k) {
  size_t h = seen_hash(k) & S->mask;
  while (S->gen[h] == S->cur) {
    if (S->key[h] == k) return 1;
    h = (h + 1) & S->mask;
  }
  return 0;
}

/* weave-later? -- shared.cljc:202-223, clause for clause. nl may be nil
 * (nl_id = nl_cause = OR_NIL); nr is never nil here (weave-node only calls
 * it when right is non-empty, shared.cljc:236-237). */
static int weave_later(uint64_t nl_id, uint64_t nl_cause, const lnode *nm, const lnode *nr,
                       const seenset *seen) {
  int sr = is_special(nr->kind), sm = is_special(nm->kind);
  int m_older = nm->id < nr->id; /* (<< (first nm) (first nr)) */
  /* A: shared.cljc:208-212 */
  if (sr && nm->id != nr->cause && (!sm || m_older)) return 1;
  /* B: shared.cljc:213-219 */
  if ((nl_id == nr->cause || nl_cause == nr->cause || seen_has(seen, nr->cause)) && m_older &&
      (!sm || sr))
    return 1;
  /* C: shared.cljc:220-223 */
  if (m_older && (!sm || sr)) return 1;
  return 0;
}

/* weave-node -- shared.cljc:225-241 (with weave-asap? 194-200).  W has room
 * for L + 1 + k entries; returns the new length. */
static size_t weave_node_lit(lnode *W, size_t L, const lnode *nm, const lnode *more, size_t k,
                             seenset *seen) {
  int prev_asap = 0;
  seen->cur++;
  size_t at = L;
  for (size_t i = 0;; i++) {
    uint64_t nl_id = i ? W[i - 1].id : OR_NIL;
    uint64_t nl_cause = i ? W[i - 1].cause : OR_NIL;
    if (i >= L) { at = L; break; } /* (empty? right) */
    const lnode *nr = &W[i];
    /* weave-asap?: (= (first nl) (second nm)) or (= (first nm) (second nr)) */
    int asap = prev_asap || nl_id == nm->cause || nm->id == nr->cause;
    if (asap && !weave_later(nl_id, nl_cause, nm, nr, seen)) { at = i; break; }
    if (asap) seen_add(seen, nl_id); /* (conj seen-since-asap (first nl)) */
    prev_asap = asap;
  }
  /* (into left cat [[node] more right]) */
  memmove(W + at + 1 + k, W + at, (L - at) * sizeof(lnode));
  W[at] = *nm;
  if (k) memcpy(W + at + 1, more, k * sizeof(lnode));
  return L + 1 + k;
}

uint32_t or_list_fold_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  uint32_t *cr = cause_ranks(s, n);
  uint32_t st = doc_status(s, n, cr);
  free(cr);
  lnode *W = (lnode *)malloc((n ? n : 1) * sizeof(lnode));
  seenset seen;
  seen_init(&seen, n);
  size_t L = 0;
  for (size_t r = 0; r < n; r++) L = weave_node_lit(W, L, &s[r], NULL, 0, &seen); /* list.cljc:27-28 */
  for (size_t p = 0; p < L; p++) out_perm[p] = W[p].idx;
  seen_free(&seen);
  free(W);
  free(s);
  return st;
}

uint32_t or_list_insert_sequence(size_t n, const uint64_t *id, const uint64_t *cause,
                                 const uint8_t *kind, const uint32_t *order,
                                 uint32_t *out_perm) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  uint32_t *cr = cause_ranks(s, n);
  uint32_t st = doc_status(s, n, cr);
  free(cr);
  free(s);
  lnode *W = (lnode *)malloc((n ? n : 1) * sizeof(lnode));
  seenset seen;
  seen_init(&seen, n);
  size_t L = 0;
  for (size_t k = 0; k < n; k++) {
    uint32_t i = order[k];
    lnode m = {id[i], cause[i], i, kind[i]};
    L = weave_node_lit(W, L, &m, NULL, 0, &seen); /* list.cljc:31-34 */
  }
  for (size_t p = 0; p < L; p++) out_perm[p] = W[p].idx;
  seen_free(&seen);
  free(W);
  return st;
}

/* SURVEY F4 (derived from shared.cljc:194-241 under: ascending-id fold, every
 * cause present and older).  Out-of-domain documents use the literal fold. */
uint32_t or_list_fold_linked(size_t n, const uint64_t *id, const uint64_t *cause,
                             const uint8_t *kind, uint32_t *out_perm) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  uint32_t *cr = cause_ranks(s, n);
  uint32_t st = doc_status(s, n, cr);
  if (st) {
    free(cr);
    free(s);
    or_list_fold_literal(n, id, cause, kind, out_perm);
    return st;
  }
  const uint32_t END = UINT32_MAX;
  uint32_t *next = (uint32_t *)malloc(n * sizeof(uint32_t));
  next[0] = END;
  for (size_t r = 1; r < n; r++) {
    uint32_t at = cr[r];
    if (!is_special(s[r].kind))
      while (next[at] != END && is_special(s[next[at]].kind)) at = next[at];
    next[r] = next[at];
    next[at] = (uint32_t)r;
  }
  size_t p = 0;
  for (uint32_t v = 0; v != END; v = next[v]) out_perm[p++] = s[v].idx;
  free(next);
  free(cr);
  free(s);
  return st;
}

/* The full reweave restated for ANY causes (the rule exact.hip's k_xfold
 * implements; derived from shared.cljc:194-241 with ids folded in ascending
 * order, so clauses B and C of weave-later? never hold): a node goes right
 * after its cause, or at the front when the cause is nil, or right before an
 * already woven node it causes -- whichever split comes first; a non-special
 * node then skips specials not caused by it; with no such split it is
 * appended.  Checked against the literal fold on out-of-domain histories. */
uint32_t or_list_fold_general(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  uint32_t *cr = cause_ranks(s, n);
  uint32_t st = doc_status(s, n, cr);
  const uint32_t END = UINT32_MAX, HEAD = UINT32_MAX - 1, NIL = UINT32_MAX - 2;
  uint32_t *par = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
  uint32_t *next = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
  uint8_t *early = (uint8_t *)calloc(n ? n : 1, 1);
  for (size_t r = 0; r < n; r++) {
    size_t c = cr[r];
    par[r] = s[r].cause == OR_NIL ? NIL : (c == n ? END : (uint32_t)c);
    if (c < n && c > r) early[c] = 1;
  }
  uint32_t head = END, tail = END;
  for (uint32_t m = 0; m < n; m++) {
    uint32_t c = par[m], p = END;
    if (c == NIL) p = HEAD;
    else if (early[m]) {
      uint32_t prev = HEAD;
      for (uint32_t v = head; v != END; prev = v, v = next[v]) {
        if (par[v] == m) { p = prev; break; }
        if (v == c) { p = v; break; }
      }
    } else if (c < m) p = c;
    if (p == END) p = tail == END ? HEAD : tail;
    else if (!is_special(s[m].kind))
      for (;;) {
        uint32_t q = p == HEAD ? head : next[p];
        if (q == END || !is_special(s[q].kind) || par[q] == m) break;
        p = q;
      }
    uint32_t q = p == HEAD ? head : next[p];
    next[m] = q;
    if (p == HEAD) head = m; else next[p] = m;
    if (q == END) tail = m;
  }
  size_t k = 0;
  for (uint32_t v = head; v != END; v = next[v]) out_perm[k++] = s[v].idx;
  free(par); free(next); free(early); free(cr); free(s);
  return st;
}

/* preorder of the effective tree -- a node, then its special
 * children by descending id, then its non-special children by descending id,
 * each with its subtree.  Computed in passes over the ranks instead of a walk
 * (ids ascend with rank and every cause is older, so a parent's rank is below
 * its children's): subtree sizes bottom-up, each child's offset among its
 * siblings (the sizes of the siblings before it), positions top-down.  Every
 * pass is sequential over the ranks with one independent random access a
 * node: a 2e7-node list 3x faster than walking (first child, next sibling,
 * parent) links, which the HIP Euler walk uses and this replaced (round 6). */
uint32_t or_list_eff_preorder(size_t n, const uint64_t *id, const uint64_t *cause,
                              const uint8_t *kind, uint32_t *out_perm) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  uint32_t *cr = cause_ranks(s, n);
  uint32_t st = doc_status(s, n, cr);
  if (st) {
    free(cr);
    free(s);
    or_list_fold_literal(n, id, cause, kind, out_perm);
    return st;
  }
  uint8_t *sp = (uint8_t *)malloc(n);
  uint32_t *eff = (uint32_t *)malloc(n * sizeof(uint32_t));
  uint32_t *up = (uint32_t *)malloc(n * sizeof(uint32_t));  /* nearest non-special ancestor-or-self */
  for (size_t r = 0; r < n; r++) sp[r] = (uint8_t)is_special(s[r].kind);
  up[0] = 0;
  eff[0] = 0;
  for (size_t r = 1; r < n; r++) {
    const uint32_t c = cr[r];
    /* a non-special climbs through special causes; a special keeps its cause */
    eff[r] = sp[r] ? c : up[c];
    up[r] = sp[r] ? up[c] : (uint32_t)r;
  }
  free(up);
  uint32_t *size = cr;  /* (the cause ranks are done) */
  uint32_t *spec_tot = (uint32_t *)calloc(n, sizeof(uint32_t));
  for (size_t r = 0; r < n; r++) size[r] = 1;
  for (size_t r = n - 1; r >= 1; r--) {
    size[eff[r]] += size[r];
    if (sp[r]) spec_tot[eff[r]] += size[r];
  }
  /* siblings before a child: for a special, the specials with larger ids; for a
   * non-special, every special and the non-specials with larger ids */
  uint32_t *acc_s = (uint32_t *)calloc(n, sizeof(uint32_t)), *acc_n = (uint32_t *)calloc(n, sizeof(uint32_t));
  uint32_t *pos = (uint32_t *)malloc(n * sizeof(uint32_t));  /* the offset before, then the position */
  for (size_t r = n - 1; r >= 1; r--) {
    const uint32_t c = eff[r];
    if (sp[r]) {
      pos[r] = acc_s[c];
      acc_s[c] += size[r];
    } else {
      pos[r] = spec_tot[c] + acc_n[c];
      acc_n[c] += size[r];
    }
  }
  free(acc_s);
  free(acc_n);
  free(spec_tot);
  pos[0] = 0;
  for (size_t r = 1; r < n; r++) pos[r] += pos[eff[r]] + 1;
  for (size_t r = 0; r < n; r++) out_perm[pos[r]] = s[r].idx;
  free(pos); free(eff); free(sp); free(cr); free(s);
  return st;
}

/* hide? -- list.cljc:48-55, applied over (partition 2 1 [nil] weave) as in
 * causal-list->edn, list.cljc:57-66. */
void or_list_visible_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                             const uint8_t *kind, const uint32_t *perm, uint8_t *vis) {
  for (size_t p = 0; p < n; p++) {
    uint32_t v = perm[p];
    int hidden = is_special(kind[v]) || (kind[v] & OR_ROOT);
    if (!hidden && p + 1 < n) {
      uint32_t w = perm[p + 1];
      if (is_hide(kind[w]) && cause[w] == id[v]) hidden = 1;
    }
    vis[p] = (uint8_t)!hidden;
  }
}

typedef struct { uint64_t site, id; uint32_t idx; } ynode;
static int cmp_ynode(const void *a, const void *b) {
  const ynode *x = (const ynode *)a, *y = (const ynode *)b;
  if (x->site != y->site) return x->site < y->site ? -1 : 1;
  if (x->id != y->id) return x->id < y->id ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* spin (1-arity) -- shared.cljc:121-132 via spin-sequential 112-119: each node
 * appended to its site's yarn in id order. */
void or_list_yarns(size_t n, const uint64_t *id, unsigned site_shift, uint64_t site_mask,
                   uint32_t *yarn_perm) {
  ynode *y = (ynode *)malloc((n ? n : 1) * sizeof(ynode));
  for (size_t i = 0; i < n; i++) {
    y[i].site = (id[i] >> site_shift) & site_mask;
    y[i].id = id[i];
    y[i].idx = (uint32_t)i;
  }
  qsort(y, n, sizeof(ynode), cmp_ynode);
  for (size_t i = 0; i < n; i++) yarn_perm[i] = y[i].idx;
  free(y);
}

/* ---- batch driver ----------------------------------------------------------- */
typedef struct {
  size_t ndocs;
  const uint64_t *off, *id, *cause;
  const uint8_t *kind;
  int method;
  uint32_t *perm;
  uint8_t *vis;
  uint32_t *status;
  size_t next; /* work counter (guarded by mu) */
  pthread_mutex_t mu;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *J = (batch_job *)arg;
  for (;;) {
    pthread_mutex_lock(&J->mu);
    size_t d = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (d >= J->ndocs) break;
    size_t b = J->off[d], n = J->off[d + 1] - b;
    uint32_t st;
    if (J->method == 0) st = or_list_fold_literal(n, J->id + b, J->cause + b, J->kind + b, J->perm + b);
    else if (J->method == 1) st = or_list_fold_linked(n, J->id + b, J->cause + b, J->kind + b, J->perm + b);
    else if (J->method == 2) st = or_list_eff_preorder(n, J->id + b, J->cause + b, J->kind + b, J->perm + b);
    else st = or_list_fold_general(n, J->id + b, J->cause + b, J->kind + b, J->perm + b);
    if (J->vis) or_list_visible_literal(n, J->id + b, J->cause + b, J->kind + b, J->perm + b, J->vis + b);
    if (J->status) J->status[d] = st;
  }
  return NULL;
}

int or_batch_lists(size_t ndocs, const uint64_t *offsets, const uint64_t *id,
                   const uint64_t *cause, const uint8_t *kind, int method, int nthreads,
                   uint32_t *out_perm, uint8_t *out_vis, uint32_t *out_status) {
  batch_job J;
  J.ndocs = ndocs; J.off = offsets; J.id = id; J.cause = cause; J.kind = kind;
  J.method = method; J.perm = out_perm; J.vis = out_vis; J.status = out_status; J.next = 0;
  pthread_mutex_init(&J.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &J);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&J.mu);
  return 0;
}

/* ---- maps ------------------------------------------------------------------- */
/* c.map/weave (map.cljc:26-45) for the full reweave, then active-node
 * (map.cljc:47-59) per key weave. */
typedef struct {
  uint64_t key;
  size_t len, cap;
  lnode *w;
} kweave;

size_t or_map_fold_literal(size_t n, const uint64_t *id, const uint64_t *cause,
                           const uint8_t *cause_is_id, const uint8_t *kind, uint64_t root_id,
                           uint64_t *node_key, uint32_t *node_pos, uint64_t *seg_key,
                           int64_t *seg_active) {
  lnode *s = sorted_nodes(n, id, cause, kind);
  size_t nseg = 0;
  kweave *K = (kweave *)calloc(n ? n : 1, sizeof(kweave));
  /* key -> segment: small open-addressing table */
  size_t cap = 16;
  while (cap < 2 * n + 2) cap <<= 1;
  uint64_t *hk = (uint64_t *)malloc(cap * sizeof(uint64_t));
  int64_t *hv = (int64_t *)malloc(cap * sizeof(int64_t));
  for (size_t i = 0; i < cap; i++) hv[i] = -1;
  seenset seen;
  seen_init(&seen, n + 1);
  for (size_t r = 0; r < n; r++) {
    uint32_t i = s[r].idx;
    uint64_t key, cin;
    if (cause_is_id[i] == 2) {
      /* a nil cause is not an id: key nil, woven under the root (map.cljc:31-37) */
      key = OR_NIL;
      cin = root_id;
    } else if (cause_is_id[i]) {
      /* key = (first (get-in ct [::s/nodes cause])): the cause node's cause, nil
       * when absent (map.cljc:32-34); cause-in-weave = cause (map.cljc:35-36). */
      size_t c = find_id(s, n, cause[i]);
      key = (c == n || cause_is_id[s[c].idx] == 2) ? OR_NIL : cause[s[c].idx];
      cin = cause[i];
    } else {
      key = cause[i];      /* map.cljc:34 */
      cin = root_id;       /* map.cljc:37 */
    }
    size_t h = seen_hash(key) & (cap - 1);
    while (hv[h] >= 0 && hk[h] != key) h = (h + 1) & (cap - 1);
    if (hv[h] < 0) {
      hv[h] = (int64_t)nseg;
      hk[h] = key;
      K[nseg].key = key;
      K[nseg].cap = 8;
      K[nseg].w = (lnode *)malloc(8 * sizeof(lnode));
      /* (or (get-in ct [::s/weave key]) [s/root-node]) -- map.cljc:40 */
      K[nseg].w[0].id = root_id;
      K[nseg].w[0].cause = OR_NIL;
      K[nseg].w[0].idx = UINT32_MAX;
      K[nseg].w[0].kind = OR_ROOT;
      K[nseg].len = 1;
      nseg++;
    }
    kweave *kw = &K[hv[h]];
    if (kw->len + 1 > kw->cap) {
      kw->cap *= 2;
      kw->w = (lnode *)realloc(kw->w, kw->cap * sizeof(lnode));
    }
    lnode m = {s[r].id, cin, i, s[r].kind};
    kw->len = weave_node_lit(kw->w, kw->len, &m, NULL, 0, &seen); /* map.cljc:41 */
  }
  for (size_t g = 0; g < nseg; g++) {
    kweave *kw = &K[g];
    seg_key[g] = kw->key;
    for (size_t p = 1; p < kw->len; p++) {
      node_key[kw->w[p].idx] = kw->key;
      node_pos[kw->w[p].idx] = (uint32_t)p;
    }
    /* active-node -- map.cljc:47-59 */
    int64_t act = -1;
    if (!(kw->len > 1 && is_hide(kw->w[1].kind))) {
      for (size_t p = 0; p < kw->len; p++) {
        const lnode *x = &kw->w[p];
        if (x->id == root_id) continue;
        if (is_special(x->kind)) continue;
        if (p + 1 < kw->len && is_hide(kw->w[p + 1].kind)) continue;
        act = (int64_t)x->idx;
        break;
      }
    }
    seg_active[g] = act;
    free(kw->w);
  }
  seen_free(&seen);
  free(hk);
  free(hv);
  free(K);
  free(s);
  return nseg;
}
