// exact.hip -- the exact path: the reference's full reweave for documents the
// fast path flags as outside its domain.  Included by causeweave.hip after the
// host helpers (scratch, radix_sort, ensure_tables, Launch) it uses.
//
// The fast path assumes every cause is present and older than
// its node and the root [[0 "0" 0] nil nil] is the smallest id.  The reference
// assumes none of this: c.list/weave folds s/weave-node over (sort ::nodes)
// (list.cljc:26-28, shared.cljc:225-241) whatever the causes are.  Documents
// with status ORPHAN, NON_LAMPORT or ROOT (and no DUP: ::nodes is a map, so the
// reference never sees a repeated id) are rewoven here, data-parallel, with
// the fold's result for every such document (tests/exact_model.py is the CPU
// model of this rule, checked against the literal fold on corrupted histories).
//
// The fold, restated for a full reweave.  Nodes arrive in ascending id order,
// so every node nr already in the weave has a smaller id than the incoming m:
//   * clause C of weave-later? (:220-223) needs (<< (first m) (first nr)):
//     never true; clause B (:213-219) implies C: never true;
//   * clause A (:208-212) is special(nr) & cause(nr) != id(m) & !special(m);
//   * weave-asap? (:194-200) first holds at the split right after cause(m), at
//     split 0 when cause(m) is nil ((first nil) = nil), or right before a node
//     already woven whose cause is m (a node with a smaller id than its cause:
//     a non-Lamport cause; m is then an "early" node);
//   * from that split m skips the nodes A holds for; if weave-asap? never holds
//     (an absent cause, or one that is not older, and no older child) the loop
//     runs to the (empty? right) branch (:236-237): m is APPENDED.
//
// Phase 1 -- synthetic lists (every flagged document).  A synthetic list is
// the document's ranks behind a virtual head H (rank r = synthetic r + 1, H
// = 0), woven by the fast path's tree and tour (weave_tail: parents in, no
// sort).  An appended node m is the same as a node woven under T(m), the node
// last in the weave at that moment (nothing follows it, so clause A's skip
// finds nothing, and no later step reads m's cause).  T(m) is found without
// iterating over the appended nodes (round 3 placed one per weave):
//   * everything woven after an appended node o stays in the region o opens
//     (o is last; a later node lands after o only through o's own subtree, or,
//     for a special o, through the special run o ends), so T of the next
//     appended node o' is the last node older than o' in that region, which
//     does not depend on where o itself went;
//   * o non-special: the region is o's subtree of the effective tree (F5);
//   * o special: o hides nothing (hide? compares the real cause: it renders
//     like an h.show) and ends the special run of N, the nearest non-special
//     ancestor of T(o).  The oldest non-special node y in (o, o') whose
//     effective parent is N opens the next region (y's subtree); without one,
//     the region is o's own special run;
//   * all of this is read off ONE weave of a static forest in which every
//     appended node hangs under H as a non-special root (k_xsyn_build): "the
//     last node < o' in [pos(s), end(s))" and "end(s) = the first later
//     position holding an older node" are two searches in a min-tree over the
//     synthetic index at each position (mt_first_after / mt_last_before).
//     Regions after a non-special node resolve in parallel (k_xres1); a run of
//     special appended nodes is followed in order by one wave (k_xres2).
// A second weave with every appended node under its T(m) is the fold's result
// for every document without an early node; render bits are F6's, roots
// hidden.
//
// Phase 2 -- documents with an early node.  The fold is the preorder of its
// insertion tree: each node's parent is the node right before its insertion
// point at its time, children by descending id.  From any weave W each node's
// insertion split in W restricted to the older nodes is found with min-tree
// searches (k_x2_xf, k_x2_anchor), named AFTER a node or BEFORE the older
// child woven first (which does not move from round to round); BEFORE anchors
// form chains that pointer jumping takes down to their AFTER-anchored bottom
// (k_x2_chain, k_x2_jump), and the insertion tree is woven on layout 2 (2n + 1
// slots: rank r at 2r + 2, its placeholder at 2r + 1, which holds a bottom's
// BEFORE chain; k_x2_build).  The rounds repeat until the weave reproduces
// itself -- that weave is the fold's (by induction over the nodes in id
// order) -- and chains of early nodes settle in O(log n) rounds.  A document
// of <= 4,096 nodes still moving after X_ROUND_CAP rounds takes the serial
// fold.  Render bits then come from the weave itself (hide? against the next
// node).  DESIGN.md 5f.
//
// The literal fold on one lane per document (k_xfold, ~1 us a node) is kept
// as a cross-check behind CW_XFOLD=1.

constexpr uint32_t X_NIL = 0xFFFFFFFEu;  // cause is nil (the root's, shared.cljc:22-23)
constexpr uint32_t X_END = 0xFFFFFFFFu;  // no cause in the document / end of the list
constexpr uint32_t X_HEAD = 0xFFFFFFFDu; // the split before the first node
constexpr uint32_t X_MASK = CW_STATUS_ROOT | CW_STATUS_ORPHAN | CW_STATUS_NON_LAMPORT;
// not a ::nodes map of the reference (a repeated id), not a K64 key, or a
// batch the pipeline found inconsistent (ids wider than the declared key_bits)
constexpr uint32_t X_SKIP = CW_STATUS_DUP | CW_STATUS_KEY_RANGE | CW_STATUS_INTERNAL;
constexpr uint32_t XFOLD_MAX = 1u << 22;     // CW_XFOLD: the serial fold's largest document
constexpr uint32_t X_NONE = 0xFFFFFFFFu;     // not on the synthetic path
constexpr uint32_t MT_MAX = 0xFFFFFFFFu;     // min-tree padding ("no node")

// A node weave-asap? never holds for: its cause is absent, or not older than
// it (c = its cause's rank, or X_NIL / X_END).  (An early node among these is
// appended in phase 1 and placed by phase 2.)
__device__ __forceinline__ bool x_appended(uint32_t c, uint32_t r, uint32_t n) {
  return c == X_END || (c < n && c >= r);
}

// Documents the exact path takes: non-empty, flagged by the domain checks, no
// repeated id.
__global__ __launch_bounds__(256) void k_xcount(const uint32_t *__restrict__ status,
                                                const uint32_t *__restrict__ doc_off, uint32_t D,
                                                uint32_t *__restrict__ count) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  bool take = false;
  if (d < D) {
    const uint32_t s = status[d];
    take = (s & X_MASK) && !(s & X_SKIP) && doc_off[d + 1] > doc_off[d];
  }
  const uint64_t b = __ballot(take);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (uint32_t)__popcll(b));
}

// The same count for documents known to be non-empty (the key weaves of the
// general map path: each holds its root).
__global__ __launch_bounds__(256) void k_xcount_nonempty(const uint32_t *__restrict__ status,
                                                         uint32_t D, uint32_t *__restrict__ count) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  const bool take = d < D && (status[d] & X_MASK) && !(status[d] & X_SKIP);
  const uint64_t b = __ballot(take);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (uint32_t)__popcll(b));
}

// Copy the flagged documents' nodes into one compact sub-batch (tile tables of
// the sub-batch; src_off[f] = where sub-document f starts in the caller's arrays).
__global__ __launch_bounds__(256) void k_xgather(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint64_t *__restrict__ src_off,
    const uint64_t *__restrict__ id, const uint64_t *__restrict__ cause,
    const uint8_t *__restrict__ kind, uint64_t *__restrict__ xid, uint64_t *__restrict__ xca,
    uint8_t *__restrict__ xkd) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  const uint64_t shift = src_off[f] - doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint64_t j = i + shift;
    xid[i] = id[j];
    xca[i] = cause[j];
    xkd[i] = kind[j];
  }
}

// Cause rank of every node in id order (X_NIL for a nil cause, X_END when the
// cause is not an id of the document), its kind by rank, early[c] = 1 for
// every node c that has a child with a smaller id (weave-asap?'s second test),
// per document "has an early node" and its number of appended nodes.
__global__ __launch_bounds__(256) void k_xjoin(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint64_t *__restrict__ skey,
    const uint32_t *__restrict__ sval, const uint64_t *__restrict__ xca,
    const uint8_t *__restrict__ xkd, uint32_t *__restrict__ xpar, uint8_t *__restrict__ xk,
    uint8_t *__restrict__ early, uint8_t *__restrict__ doc_early, uint32_t *__restrict__ doc_orph) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint64_t *sk = skey + base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base, v = sval[i];
    const uint64_t c = xca[base + v];
    uint32_t p = X_NIL;
    if (c != CW_NIL) {
      uint32_t lo = 0, hi = n;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sk[mid] < c) lo = mid + 1; else hi = mid;
      }
      p = (lo < n && sk[lo] == c) ? lo : X_END;
    }
    xpar[i] = p;
    xk[i] = xkd[base + v];
    if (p < n && p > r) {
      early[base + p] = 1;
      doc_early[f] = 1;
    }
    if (x_appended(p, r, n)) atomicAdd(&doc_orph[f], 1u);  // (appended nodes are few)
  }
}

// One giant list flagged by its front end (cw_ctx::xfront): the exact path's
// join from the front end's sorted ids and rank directory, no second sort --
// the cause of every rank by input index (cause | kind in one word when the
// front end packed it), its rank from one directory line (X_NIL, X_END, or a
// rank that may be younger), early children and the appended count.
__global__ __launch_bounds__(256) void k_xjoin_dir(
    const uint64_t *__restrict__ skey, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ cause_key, const uint8_t *__restrict__ kind,
    const uint64_t *__restrict__ ckk, uint32_t n, const uint4 *__restrict__ dir, uint64_t E,
    uint32_t *__restrict__ xpar, uint8_t *__restrict__ xk, uint8_t *__restrict__ early,
    uint8_t *__restrict__ doc_early, uint32_t *__restrict__ doc_orph) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool app = false;
  if (r < n) {
    constexpr uint64_t M56 = (1ull << 56) - 1;
    const uint32_t v = sval[r];
    uint64_t c;
    uint8_t kd;
    if (ckk) {
      const uint64_t w = ckk[v];
      c = w & M56;
      kd = (uint8_t)(w >> 56);
      if (c == M56) c = cause_key[v];  // nil, or a cause no id can be
    } else {
      c = cause_key[v];
      kd = kind[v];
    }
    uint32_t p = X_NIL;
    if (c != CW_NIL) {
      const uint64_t kmax = min(skey[n - 1], E * GD_KEYS - 1);
      bool present = false;
      const uint32_t rc = c <= kmax ? gd_rank(dir, c, present) : 0u;
      p = present ? rc : X_END;
    }
    xpar[r] = p;
    xk[r] = kd;
    if (p < n && p > r) {
      early[p] = 1;
      *doc_early = 1;
    }
    app = x_appended(p, r, n);
  }
  const uint64_t b = __ballot(app);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(doc_orph, (uint32_t)__popcll(b));
}

// A list handed over in rank order (cw_weave_ranked): the root's cause is nil,
// CW_NOT_FOUND stays "absent"; early children as in k_xjoin.
__global__ __launch_bounds__(256) void k_xranked_prep(const uint32_t *__restrict__ par,
                                                      const uint8_t *__restrict__ kind, uint32_t n,
                                                      uint32_t *__restrict__ xpar,
                                                      uint8_t *__restrict__ early,
                                                      uint8_t *__restrict__ doc_early,
                                                      uint32_t *__restrict__ doc_orph) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t p = par[r];
  if (r == 0 && (kind[0] & KIND_ROOT)) p = X_NIL;
  if (p == CW_NIL_RANK) p = X_NIL;
  if (p == CW_NOT_FOUND) p = X_END;
  xpar[r] = p;
  if (p < n && p > r) {
    early[p] = 1;
    *doc_early = 1;
  }
  if (x_appended(p, r, n)) atomicAdd(doc_orph, 1u);
}

// Visible bits [g0, g0 + 32) of one weave word: the bits of this document
// (mask) replace whatever the fast path left there.
__device__ __forceinline__ void x_flush(uint32_t *bits, uint64_t word, uint32_t mask, uint32_t v) {
  if (mask == 0xFFFFFFFFu) {
    bits[word] = v;
  } else {
    atomicAnd(&bits[word], ~mask);
    atomicOr(&bits[word], v & mask);
  }
}

// The fold, one lane per document (documents are sequential by nature; lanes
// walk independent documents).  xnext is the weave as a linked list over ranks.
// Outputs at the document's place in the caller's batch: weave_perm (input
// index per position: val[rank], val == nullptr: the rank), the rendered bits
// (hide?, list.cljc:48-55, on the finished weave) and the rendered count.
__global__ __launch_bounds__(64) void k_xfold(
    const uint32_t *__restrict__ doc_off, uint32_t F, const uint32_t *__restrict__ xpar,
    const uint8_t *__restrict__ xk, const uint8_t *__restrict__ early,
    uint32_t *__restrict__ xnext, const uint32_t *__restrict__ val,
    const uint64_t *__restrict__ out_off, const uint32_t *__restrict__ out_doc,
    uint32_t *__restrict__ weave_perm, uint32_t *__restrict__ visible_bits,
    uint32_t *__restrict__ visible_count, const uint8_t *__restrict__ run) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F || (run && !run[f])) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint32_t *par = xpar + base;
  const uint8_t *kd = xk + base, *er = early + base;
  uint32_t *nx = xnext + base;
  uint32_t head = X_END, tail = X_END;
  for (uint32_t m = 0; m < n; m++) {
    const uint32_t c = par[m];
    const bool sp = is_special(kd[m]);
    uint32_t p = X_END;  // the node m goes after (X_HEAD: the front); X_END: not found
    if (c == X_NIL) {
      p = X_HEAD;
    } else if (er[m]) {  // the first of: right after the cause, right before a child
      uint32_t prev = X_HEAD;
      for (uint32_t v = head; v != X_END; prev = v, v = nx[v]) {
        if (par[v] == m) {
          p = prev;
          break;
        }
        if (v == c) {
          p = v;
          break;
        }
      }
    } else if (c < m) {
      p = c;
    }
    if (p == X_END) {
      p = tail == X_END ? X_HEAD : tail;  // weave-asap? never held: the end
    } else if (!sp) {                      // clause A: skip specials not caused by m
      for (;;) {
        const uint32_t q = p == X_HEAD ? head : nx[p];
        if (q == X_END || !is_special(kd[q]) || par[q] == m) break;
        p = q;
      }
    }
    const uint32_t q = p == X_HEAD ? head : nx[p];
    nx[m] = q;
    if (p == X_HEAD) head = m;
    else nx[p] = m;
    if (q == X_END) tail = m;
  }
  // emit: weave order, hide? against the next node, rendered bits by word
  const uint64_t g0 = out_off[f];
  uint32_t cnt = 0, acc = 0, mask = 0;
  uint64_t word = g0 >> 5;
  uint64_t g = g0;
  for (uint32_t v = head; v != X_END;) {
    const uint32_t w = nx[v];
    const uint8_t k = kd[v];
    const bool hidden = is_special(k) || (k & KIND_ROOT) ||
                        (w != X_END && is_hide(kd[w]) && par[w] == v);
    weave_perm[g] = val ? val[base + v] : v;
    if (visible_bits) {
      if ((g >> 5) != word) {
        x_flush(visible_bits, word, mask, acc);
        word = g >> 5;
        acc = mask = 0;
      }
      mask |= 1u << (g & 31);
      if (!hidden) acc |= 1u << (g & 31);
    }
    cnt += hidden ? 0 : 1;
    g++;
    v = w;
  }
  if (visible_bits && mask) x_flush(visible_bits, word, mask, acc);
  visible_count[out_doc[f]] = cnt;
}

__global__ __launch_bounds__(64) void k_xmaxts(const uint32_t *__restrict__ doc_off, uint32_t F,
                                               const uint64_t *__restrict__ skey, uint32_t ts_shift,
                                               const uint32_t *__restrict__ out_doc,
                                               uint64_t *__restrict__ max_ts) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F) max_ts[out_doc[f]] = skey[doc_off[f + 1] - 1] >> ts_shift;  // the largest id
}

// dst[out_off[f] + i - doc_off[f]] = src[i] over the sub-batch's tiles.
__global__ __launch_bounds__(256) void k_xscatter(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint64_t *__restrict__ out_off,
    const uint32_t *__restrict__ src, uint32_t *__restrict__ dst) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  const uint64_t shift = out_off[f] - doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x)
    dst[i + shift] = src[i];
}

// --- min-trees over a synthetic weave -----------------------------------------
// Level 0 = an array over synthetic positions (padded with MT_MAX to a multiple
// of 16), level l + 1 = the minimum of each 16 entries of level l (padded too),
// up to a level of 16 entries.  Blocks of 16 are 64-byte aligned: a block is
// four 16-byte loads.

constexpr uint32_t MT_LEVELS = 10;
struct XMinTree {
  const uint32_t *lv[MT_LEVELS];
  uint32_t len[MT_LEVELS];
  uint32_t levels;
};

// Bit k set: entry k of the 16-entry block at b is < v.
__device__ __forceinline__ uint32_t mt_mask16(const uint32_t *b, uint32_t v) {
  const uint4 *b4 = reinterpret_cast<const uint4 *>(b);
  const uint4 x = b4[0], y = b4[1], z = b4[2], w = b4[3];
  return (x.x < v) | (x.y < v) << 1 | (x.z < v) << 2 | (x.w < v) << 3 | (y.x < v) << 4 |
         (y.y < v) << 5 | (y.z < v) << 6 | (y.w < v) << 7 | (z.x < v) << 8 | (z.y < v) << 9 |
         (z.z < v) << 10 | (z.w < v) << 11 | (w.x < v) << 12 | (w.y < v) << 13 | (w.z < v) << 14 |
         (w.w < v) << 15;
}

// The first position q > p whose entry is < v; t.len[0] if none.
__device__ uint32_t mt_first_after(const XMinTree &t, uint32_t p, uint32_t v) {
  uint32_t i = p + 1;
  for (uint32_t l = 0; l < t.levels; l++) {
    if (i >= t.len[l]) break;
    const uint32_t b0 = i & ~15u;
    const uint32_t m = mt_mask16(t.lv[l] + b0, v) & (0xFFFFu << (i & 15u));
    if (m) {
      uint32_t j = b0 + (uint32_t)__builtin_ctz(m);
      while (l > 0) {  // a block's minimum < v: one of its 16 entries is
        l--;
        j = 16 * j + (uint32_t)__builtin_ctz(mt_mask16(t.lv[l] + 16 * j, v));
      }
      return j;
    }
    i = (i >> 4) + 1;
  }
  return t.len[0];
}

// The last position q < h whose entry is < v; MT_MAX if none.
__device__ uint32_t mt_last_before(const XMinTree &t, uint32_t h, uint32_t v) {
  if (h == 0) return MT_MAX;
  uint32_t i = min(h, t.len[0]) - 1;
  for (uint32_t l = 0; l < t.levels; l++) {
    const uint32_t b0 = i & ~15u;
    const uint32_t m = mt_mask16(t.lv[l] + b0, v) & (0xFFFFu >> (15u - (i & 15u)));
    if (m) {
      uint32_t j = b0 + 31u - (uint32_t)__builtin_clz(m);
      while (l > 0) {
        l--;
        j = 16 * j + 31u - (uint32_t)__builtin_clz(mt_mask16(t.lv[l] + 16 * j, v));
      }
      return j;
    }
    if (b0 == 0) break;
    i = (i >> 4) - 1;
  }
  return MT_MAX;
}

// The minimum entry of positions [a, b) (MT_MAX when empty): the fringes of
// each level entry by entry, the whole blocks between them one level up.
__device__ uint32_t mt_range_min(const XMinTree &t, uint32_t a, uint32_t b) {
  uint32_t m = MT_MAX;
  for (uint32_t l = 0; l < t.levels && a < b; l++) {
    const uint32_t al = min(b, (a + 15u) & ~15u), br = max(al, b & ~15u);
    for (uint32_t i = a; i < al; i++) m = min(m, t.lv[l][i]);
    for (uint32_t i = br; i < b; i++) m = min(m, t.lv[l][i]);
    a = al >> 4;
    b = br >> 4;
  }
  return m;
}

__global__ __launch_bounds__(256) void k_mt_level(const uint32_t *__restrict__ in,
                                                  uint32_t in_len, uint32_t *__restrict__ out,
                                                  uint32_t out_len) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= out_len) return;
  uint32_t m = MT_MAX;
  if (16 * j < in_len) {
    const uint4 *b4 = reinterpret_cast<const uint4 *>(in + 16 * j);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 x = b4[k];
      m = min(m, min(min(x.x, x.y), min(x.z, x.w)));
    }
  }
  out[j] = m;
}

// --- phase 1: the static forest -----------------------------------------------
// Sub-batch index i = doc_off[f] + r (rank r of flagged document f); the
// synthetic list of f starts at sbase[f] (X_NONE: f is not on this path):
// sbase[f] = H, sbase[f] + 1 + r = rank r.  Synthetic parents are local
// (0 = H); "global synthetic indices" sbase[f] + s grow with f.

// Parents and kinds of the static forest: an appended node under H as a
// non-special root, a nil cause under H, every other node under its cause.
__global__ __launch_bounds__(256) void k_xsyn_build(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ xpar, const uint8_t *__restrict__ xk, uint32_t *__restrict__ spar,
    uint8_t *__restrict__ skd) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base, p = xpar[i];
    uint8_t k = xk[i] & KIND_CLASS;
    uint32_t sp;
    if (x_appended(p, r, n)) {
      sp = 0;
      k = 0;
    } else {
      sp = p == X_NIL ? 0 : p + 1;
    }
    spar[sb + 1 + r] = sp;
    skd[sb + 1 + r] = k;
    if (r == 0) {
      spar[sb] = CW_NIL_RANK;
      skd[sb] = KIND_ROOT;
    }
  }
}

// Positions of a woven synthetic list: G[x] = the global synthetic index at
// global position x, pos[g] = the position of g.  AUX[x] (mode 0, the static
// forest) = 0 where the node is structurally non-special, else G[x] -- "the
// first later position < s" then ends a special run; (mode 1, phase 2) =
// G[x] where the node is non-special, else MT_MAX.  posold != nullptr: count
// the positions that changed (phase 2's fixed point).
__global__ __launch_bounds__(256) void k_xs_pos(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint8_t *__restrict__ only, const uint32_t *__restrict__ wperm,
    const uint8_t *__restrict__ skd, const uint8_t *__restrict__ xk, uint32_t mode,
    uint32_t *__restrict__ G, uint32_t *__restrict__ AUX, uint32_t *__restrict__ pos,
    const uint32_t *__restrict__ posold, uint32_t *__restrict__ ctl) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE || (only && !only[f])) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  uint32_t changed = 0;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t q = i - base, x = sb + 1 + q, s = wperm[x];
    if (q == 0) {
      G[sb] = sb;
      pos[sb] = sb;
      AUX[sb] = mode == 0 ? 0u : sb;
    }
    if (s < 1 || s > n) {
      atomicOr(&ctl[1], 1u);  // H is always first: a later position that holds it is an error
      continue;
    }
    const uint32_t g = sb + s;
    G[x] = g;
    if (posold && posold[g] != x) changed++;
    pos[g] = x;
    const bool ns = mode == 0 ? (skd[g] & KIND_CLASS) == 0 : (xk[base + s - 1] & KIND_CLASS) == 0;
    AUX[x] = mode == 0 ? (ns ? 0u : g) : (ns ? g : MT_MAX);
  }
  if (posold) {
    for (int o = 32; o > 0; o >>= 1) changed += __shfl_xor(changed, o, 64);
    if ((threadIdx.x & 63) == 0 && changed) atomicAdd(&ctl[0], changed);
  }
}

// ctop[g] = the first of g and its static ancestors that is non-special
// (structurally: an appended node counts as non-special), or H: a special
// node's nearest non-special ancestor, and the effective parent of a
// non-special child of g.
__global__ __launch_bounds__(256) void k_xctop(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ spar, const uint8_t *__restrict__ skd, uint32_t *__restrict__ ctop) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base;
    uint32_t s = r + 1;
    while (s != 0 && (skd[sb + s] & KIND_CLASS)) s = spar[sb + s];
    ctop[sb + 1 + r] = sb + s;
    if (r == 0) ctop[sb] = sb;
  }
}

// The appended nodes of every synthetic document in id order: count per tile,
// scan over tiles, write in order.
__global__ __launch_bounds__(256) void k_xapp_count(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ xpar, uint32_t *__restrict__ tcnt) {
  __shared__ uint32_t ws[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  uint32_t c = 0;
  if (sbase[f] != X_NONE) {
    const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
    for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x)
      c += x_appended(xpar[i], i - base, n) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tcnt[t] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Exclusive scan of T tile counts in place (one workgroup of 1024).
__global__ __launch_bounds__(1024) void k_xapp_scan(uint32_t *__restrict__ tcnt, uint32_t T) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < T; c0 += 1024) {
    const uint32_t t = c0 + threadIdx.x;
    const uint32_t v = t < T ? tcnt[t] : 0;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre += wsum[w];
    if (t < T) tcnt[t] = pre + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_xapp_scatter(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ xpar, const uint32_t *__restrict__ toff,
    uint32_t *__restrict__ app_list, uint32_t *__restrict__ app_doc, uint32_t *__restrict__ app_idx) {
  __shared__ uint32_t ws[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  if (sbase[f] == X_NONE) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t k0 = toff[t];
  for (uint32_t c0 = tile_start[t]; c0 < tile_start[t + 1]; c0 += 256) {
    const uint32_t i = c0 + threadIdx.x;
    const bool a = i < tile_start[t + 1] && x_appended(xpar[i], i - base, n);
    const uint64_t b = __ballot(a);
    if (lane == 0) ws[wv] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t pre = k0;
    for (uint32_t w = 0; w < wv; w++) pre += ws[w];
    if (a) {
      const uint32_t k = pre + lanes_below(b);
      app_list[k] = i;
      app_doc[k] = f;
      if (app_idx) app_idx[i] = k;
    }
    k0 += ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
  }
}

// Regions after a non-special node (or H): T of every appended node whose
// previous appended node (in id order, same document) is non-special or H.
// Tsyn[k] = the global synthetic index of T; Nof[o] = N for a special o.
__global__ __launch_bounds__(256) void k_xres1(
    const uint32_t *__restrict__ app_list, const uint32_t *__restrict__ app_doc, uint32_t A,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint8_t *__restrict__ xk, const uint32_t *__restrict__ pos, const uint32_t *__restrict__ G,
    const uint32_t *__restrict__ ctop, XMinTree mt, uint32_t *__restrict__ Tsyn,
    uint32_t *__restrict__ Nof, uint32_t *__restrict__ ctl) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A) return;
  const uint32_t i = app_list[k], f = app_doc[k], sb = sbase[f], base = doc_off[f];
  const uint32_t o = sb + 1 + (i - base);
  uint32_t prev = sb;
  if (k > 0 && app_doc[k - 1] == f) {
    const uint32_t ip = app_list[k - 1];
    if (xk[ip] & KIND_CLASS) return;  // after a special appended node: k_xres2
    prev = sb + 1 + (ip - base);
  }
  const uint32_t e = mt_first_after(mt, pos[prev], prev);
  const uint32_t q = mt_last_before(mt, e, o);
  if (q == MT_MAX || q < pos[prev]) {  // prev itself is older than o: never
    atomicOr(&ctl[1], 2u);
    return;
  }
  const uint32_t T = G[q];
  Tsyn[k] = T;
  if (xk[i] & KIND_CLASS) Nof[o] = ctop[T];
}

// The smallest non-special child of s in the static forest with an id in
// (lo, hi), MT_MAX if none.  s's non-special children follow its special
// children's (all-special) subtrees in descending id order, and every node of
// a child's subtree is younger than the child: with the first child at or
// below lo at position qs, the wanted child is the minimum over [s0, qs).
__device__ uint32_t x_child_between(const XMinTree &mt, const XMinTree &mtx,
                                    const uint32_t *__restrict__ pos, uint32_t s, uint32_t lo,
                                    uint32_t hi) {
  const uint32_t p = pos[s];
  const uint32_t e = mt_first_after(mt, p, s);   // the end of s's subtree
  const uint32_t s0 = mt_first_after(mtx, p, s);  // its first non-special child (or e)
  if (s0 >= e) return MT_MAX;
  const uint32_t qs = min(e, mt_first_after(mt, s0 - 1, lo + 1));
  if (qs <= s0) return MT_MAX;
  const uint32_t y = mt_range_min(mt, s0, qs);
  return y < hi ? y : MT_MAX;
}

constexpr uint32_t XRUN_MAX = 64;  // special appended nodes a wave keeps (N, node) for

// Runs of special appended nodes, in order, one wave each: the wave that
// starts at entry k (its previous appended node is special and was resolved
// by k_xres1) follows the run.  The next region's y is N's oldest non-special
// child between the two appended nodes, or the oldest non-special child of a
// special appended node of the run with the same N (a node caused through it
// climbs to N): both by x_child_between, one lane per candidate parent.  With
// N = H (H also holds the appended roots) or a run longer than XRUN_MAX, the
// ranks between are scanned instead.
__global__ __launch_bounds__(64) void k_xres2(
    const uint32_t *__restrict__ app_list, const uint32_t *__restrict__ app_doc, uint32_t A,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ xpar, const uint8_t *__restrict__ xk,
    const uint32_t *__restrict__ pos, const uint32_t *__restrict__ G,
    const uint32_t *__restrict__ ctop, XMinTree mt, XMinTree mtx, uint32_t *__restrict__ Tsyn,
    uint32_t *__restrict__ Nof, uint32_t *__restrict__ ctl) {
  __shared__ uint32_t runO[XRUN_MAX], runN[XRUN_MAX];
  uint32_t k = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (k == 0 || k >= A) return;
  const uint32_t f = app_doc[k];
  if (app_doc[k - 1] != f || !(xk[app_list[k - 1]] & KIND_CLASS)) return;  // not after a special
  // the run starts here when the previous one was resolved by k_xres1
  if (k >= 2 && app_doc[k - 2] == f && (xk[app_list[k - 2]] & KIND_CLASS)) return;
  const uint32_t sb = sbase[f], base = doc_off[f], n = doc_off[f + 1] - base;
  // every lane follows the run with the same values; N stays in registers
  uint32_t N = Nof[sb + 1 + (app_list[k - 1] - base)];
  uint32_t nrun = 0;
  if (lane == 0) {
    runO[0] = sb + 1 + (app_list[k - 1] - base);
    runN[0] = N;
  }
  nrun = 1;
  __syncthreads();
  for (; k < A && app_doc[k] == f; k++) {
    const uint32_t ip = app_list[k - 1], i = app_list[k];
    const uint32_t rp = ip - base, ro = i - base;
    const uint32_t prev = sb + 1 + rp, o = sb + 1 + ro;
    // y: the oldest non-special node between them whose effective parent is N
    uint32_t y = MT_MAX;
    if (N != sb && nrun <= XRUN_MAX) {
      uint32_t c = lane == 0 ? x_child_between(mt, mtx, pos, N, prev, o) : MT_MAX;
      for (uint32_t j = lane; j < nrun; j += 64)
        if (runN[j] == N) c = min(c, x_child_between(mt, mtx, pos, runO[j], prev, o));
      for (int s2 = 32; s2 > 0; s2 >>= 1) c = min(c, (uint32_t)__shfl_xor(c, s2, 64));
      y = c;
    } else {
      for (uint32_t y0 = rp + 1; y0 < ro && y == MT_MAX; y0 += 64) {
        const uint32_t r = y0 + lane;
        bool hit = false;
        if (r < ro && !(xk[base + r] & KIND_CLASS)) {
          const uint32_t cz = xpar[base + r];
          if (!x_appended(cz, r, n)) {
            uint32_t e = cz == X_NIL ? sb : ctop[sb + 1 + cz];
            if (e != sb) {  // through a special appended node of this run: its N
              const uint32_t er = e - sb - 1;
              if ((xk[base + er] & KIND_CLASS) && x_appended(xpar[base + er], er, n))
                e = __hip_atomic_load(&Nof[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            hit = e == N;
          }
        }
        const uint64_t b = __ballot(hit);
        if (b) y = sb + 1 + y0 + (uint32_t)__builtin_ctzll(b);
      }
    }
    uint32_t q, lo;
    bool in_run;
    if (y != MT_MAX) {
      lo = pos[y];
      q = mt_last_before(mt, mt_first_after(mt, lo, y), o);
      in_run = false;
    } else {
      lo = pos[prev];
      q = mt_last_before(mt, mt_first_after(mtx, lo, prev), o);
      in_run = true;
    }
    if (q == MT_MAX || q < lo) {
      if (lane == 0) atomicOr(&ctl[1], 4u);
      return;
    }
    const uint32_t T = G[q];
    const bool sp = (xk[i] & KIND_CLASS) != 0;
    if (sp) N = in_run ? N : ctop[T];
    if (lane == 0) {
      Tsyn[k] = T;
      if (sp) {
        __hip_atomic_store(&Nof[o], N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (nrun < XRUN_MAX) {
          runO[nrun] = o;
          runN[nrun] = N;
        }
      }
    }
    if (!sp) break;  // the run ends
    nrun++;  // (past XRUN_MAX: the scan from here on)
    __syncthreads();
  }
}

// Every appended node under its T; an appended hide hides nothing (hide?
// compares the real cause), so it weaves like an h.show.
__global__ __launch_bounds__(256) void k_xsyn_final(
    const uint32_t *__restrict__ app_list, const uint32_t *__restrict__ app_doc, uint32_t A,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint8_t *__restrict__ xk, const uint32_t *__restrict__ Tsyn, uint32_t *__restrict__ spar,
    uint8_t *__restrict__ skd) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A) return;
  const uint32_t i = app_list[k], f = app_doc[k], sb = sbase[f];
  const uint32_t o = sb + 1 + (i - doc_off[f]);
  const uint8_t c = xk[i] & KIND_CLASS;
  spar[o] = Tsyn[k] - sb;
  skd[o] = c == KIND_HIDE || c == KIND_HHIDE ? 3 : c;
}

// --- phase 2: insertion-tree rounds with BEFORE anchors ----------------------
// Layout 2 (documents with an early node, round 5): the synthetic list of f
// starts at sb2[f] = H; slot 2r + 2 = rank r, slot 2r + 1 = the placeholder of
// rank r.  A round turns the weave W into one anchor per node:
//   AFTER s   right after slot s (H, or an older node: the insertion-tree
//             parent of round 4's rule), or
//   BEFORE x  right before rank x, m's older child woven first (weave-asap?'s
//             second test, shared.cljc:199-200) -- static along a chain of
//             early nodes, where "the node before x" moved one link a round
//             (a reverse chain took n - 2 rounds).
// x has at most one BEFORE child (its own cause), so BEFORE anchors form chains
// m_k -> .. -> m_1 -> b down to an AFTER-anchored bottom b, which the fold lays
// out as m_k A_k .. m_1 A_1 b A_b (A = a node's after-subtrees).  As a tree
// with children by descending slot: the placeholder 2b + 1 takes b's place
// under b's parent and holds m_k .. m_1 and b (slots descending).  Every unused
// placeholder is a leaf under slot 2r (rank r - 1, or H): the smallest slot
// there, so the last child.  Parents stay below their children, so weave_tail
// weaves layout 2 as it weaves any synthetic list (all classes normal: a plain
// preorder); positions of placeholders are transparent (MT_MAX) to the queries.

constexpr uint32_t XB_BIT = 0x80000000u;  // anchor word: BEFORE rank (low bits), else AFTER slot
constexpr uint32_t X_ROUND_CAP = 48;     // rounds before a small still-moving document is folded
                                         // (the default of cw_ctx::x_round_cap, CW_X_ROUND_CAP)
constexpr uint32_t X_CAP_FOLD_MAX = 4096;  // ... serially (k_xfold: ~n^2 steps at worst)

// Positions of a layout-2 weave.  from1: round 0's W is phase 1's weave
// (layout 1, wperm1 at sb1): rank position x' -> x = 2x', slot s' -> 2s'.
// Otherwise wperm2 (layout 2).  G[x] = the global slot at position x for a
// rank or H (MT_MAX for a placeholder), AUX[x] = G[x] where the node is
// non-special (H too), pos[slot] = x.  posold: moved[f] = 1 when a rank's
// position changed (the round did not reproduce W).
__global__ __launch_bounds__(256) void k_x2_pos(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase1,
    const uint32_t *__restrict__ sbase2, const uint8_t *__restrict__ only, uint32_t from1,
    const uint32_t *__restrict__ wperm1, const uint32_t *__restrict__ wperm2,
    const uint8_t *__restrict__ xk, uint32_t *__restrict__ G, uint32_t *__restrict__ AUX,
    uint32_t *__restrict__ pos, const uint32_t *__restrict__ posold, uint8_t *__restrict__ moved,
    uint32_t *__restrict__ ctl) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  if (sb == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  bool changed = false;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base;
    if (r == 0) {
      G[sb] = sb;
      AUX[sb] = sb;
      pos[sb] = sb;
      if (!from1 && wperm2[sb] != 0) atomicOr(&ctl[1], 16u);  // H is always first
    }
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      uint32_t x, s;
      if (from1) {
        if (h) break;
        x = 2 * r + 2;
        s = 2 * wperm1[sbase1[f] + 1 + r];
      } else {
        x = 2 * r + 1 + h;
        s = wperm2[sb + x];
      }
      if (s == 0 || s > 2 * n) {
        atomicOr(&ctl[1], 16u);
        continue;
      }
      const uint32_t g = sb + s, xg = sb + x;
      if (s & 1u) {  // a placeholder
        G[xg] = MT_MAX;
        AUX[xg] = MT_MAX;
      } else {
        G[xg] = g;
        AUX[xg] = (xk[base + (s >> 1) - 1] & KIND_CLASS) ? MT_MAX : g;
        changed |= posold && posold[g] != xg;
      }
      pos[g] = xg;
    }
  }
  if (posold && __syncthreads_or(changed) && threadIdx.x == 0) moved[f] = 1;
}

// xf[c] = the smallest position of an older child of c (weave-asap?'s second
// test), MT_MAX when none.
__global__ __launch_bounds__(256) void k_x2_xf(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint8_t *__restrict__ only, const uint32_t *__restrict__ xpar,
    const uint32_t *__restrict__ pos, uint32_t *__restrict__ xf) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  if (sb == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base, p = xpar[i];
    if (p < n && p > r) atomicMin(&xf[base + p], pos[sb + 2 * r + 2]);
  }
}

// Each node's anchor from the weave W (G, pos; mt over G, mtn over G of the
// non-special nodes): weave-node's scan on W restricted to the older nodes.
// first: W is phase 1's weave (an appended node goes after the last older node
// of the whole weave; later rounds use the region of the previous appended
// node, prevne: its sub-batch index or X_NONE).
__global__ __launch_bounds__(256) void k_x2_anchor(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint8_t *__restrict__ only, const uint32_t *__restrict__ xpar,
    const uint8_t *__restrict__ xk, const uint32_t *__restrict__ xf,
    const uint32_t *__restrict__ prevne, const uint32_t *__restrict__ pos,
    const uint32_t *__restrict__ G, XMinTree mt, XMinTree mtn, uint32_t first,
    uint32_t *__restrict__ anc, uint32_t *__restrict__ ctl) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  if (sb == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base, p = xpar[i], m = sb + 2 * r + 2;
    const bool sp = (xk[i] & KIND_CLASS) != 0;
    const uint32_t x1 = xf[i];
    const uint32_t cp = p == X_NIL ? sb : (p < r ? pos[sb + 2 * p + 2] : MT_MAX);
    uint32_t pred = MT_MAX;
    bool before = false;
    if (cp == MT_MAX && x1 == MT_MAX) {  // appended
      uint32_t e = sb + 2 * n + 1, lo = sb;
      if (!first) {  // the region of the previous appended node (not an early one)
        const uint32_t ip = prevne[i];
        const uint32_t prev = ip == X_NONE ? sb : sb + 2 * (ip - base) + 2;
        lo = pos[prev];
        e = mt_first_after(mt, lo, prev);
      }
      const uint32_t q = mt_last_before(mt, e, m);
      pred = q == MT_MAX || q < lo ? MT_MAX : G[q];
    } else if (cp != MT_MAX && cp < x1) {  // right after the cause, then clause A's skip
      if (sp) {
        pred = p == X_NIL ? sb : sb + 2 * p + 2;
      } else {
        const uint32_t stop = min(mt_first_after(mtn, cp, m), x1);
        if (stop == x1) {
          before = true;
        } else {
          const uint32_t q = mt_last_before(mt, stop, m);
          pred = q == MT_MAX || q < cp ? MT_MAX : G[q];
        }
      }
    } else {  // right before the older child woven first
      before = true;
    }
    uint32_t a;
    if (before) {
      const uint32_t gx = G[x1];
      if (gx == MT_MAX || gx < sb + 2 || gx >= m) {
        atomicOr(&ctl[1], 8u);
        a = 0;
      } else {
        a = XB_BIT | ((gx - sb - 2) >> 1);
      }
    } else if (pred == MT_MAX || pred >= m || pred < sb) {
      atomicOr(&ctl[1], 8u);
      a = 0;
    } else {
      a = pred - sb;
    }
    anc[i] = a;
  }
}

// BEFORE chains: jmp = the BEFORE target (a rank) or the node itself; hasb[x]
// = x has a BEFORE child.  k_x2_jump then doubles jmp down every chain to its
// AFTER-anchored bottom (in place: a value read mid-update is only further
// down the same chain).
__global__ __launch_bounds__(256) void k_x2_chain(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint8_t *__restrict__ only, const uint32_t *__restrict__ anc,
    uint32_t *__restrict__ jmp, uint8_t *__restrict__ hasb) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  if (sbase2[f] == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t a = anc[i];
    if (a & XB_BIT) {
      const uint32_t x = a & ~XB_BIT;
      jmp[i] = x;
      hasb[base + x] = 1;
    } else {
      jmp[i] = i - base;
    }
  }
}

constexpr uint32_t X2_JUMPS = 3;
__global__ __launch_bounds__(256) void k_x2_jump(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint8_t *__restrict__ only, uint32_t *jmp) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  if (sbase2[f] == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f];
  // X2_JUMPS jumps a launch: each one at least adds the reach every node had
  // when the launch began, so a launch multiplies it by X2_JUMPS + 1 (the
  // host launches ceil(log_{X2_JUMPS+1} n) + 1 of them)
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    uint32_t j = __hip_atomic_load(&jmp[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t q = 0; q < X2_JUMPS; q++) {
      const uint32_t k = __hip_atomic_load(&jmp[base + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == j) break;
      __hip_atomic_store(&jmp[i], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      j = k;
    }
  }
}

// The layout-2 tree of the anchors (slots local to the document, all classes
// normal): rank r under its AFTER slot, or under its placeholder when it is
// a chain bottom, or under its bottom's placeholder when BEFORE-anchored; a
// used placeholder under the bottom's AFTER slot, an unused one under 2r.
__global__ __launch_bounds__(256) void k_x2_build(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint8_t *__restrict__ only, const uint32_t *__restrict__ anc,
    const uint32_t *__restrict__ jmp, const uint8_t *__restrict__ hasb,
    uint32_t *__restrict__ spar, uint8_t *__restrict__ skd) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  if (sb == X_NONE || !only[f]) return;
  const uint32_t base = doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t r = i - base, a = anc[i];
    uint32_t pr, pp;
    if (a & XB_BIT) {
      pr = 2 * jmp[i] + 1;
      pp = 2 * r;
    } else if (hasb[i]) {
      pr = 2 * r + 1;
      pp = a;
    } else {
      pr = a;
      pp = 2 * r;
    }
    spar[sb + 2 * r + 2] = pr;
    spar[sb + 2 * r + 1] = pp;
    skd[sb + 2 * r + 2] = 0;
    skd[sb + 2 * r + 1] = 0;
    if (r == 0) {
      spar[sb] = CW_NIL_RANK;
      skd[sb] = KIND_ROOT;
    }
  }
}

// The converged layout-2 weave back to layout 1 (wperm1[sb1 + 1 + q] = rank + 1
// at output position q), for k_xsyn_emit: ranks counted per tile of positions
// (a tile of ranks [a, b) owns positions [2a + 1, 2b + 1)), a scan over tiles,
// then each rank written at its count.  Documents not on layout 2 count their
// n ranks (so a document's first tile starts at its doc_off).
__global__ __launch_bounds__(256) void k_x2_count(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase2,
    const uint32_t *__restrict__ wperm2, uint32_t *__restrict__ tcnt) {
  __shared__ uint32_t ws[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  const uint32_t base = doc_off[f], a = tile_start[t] - base, b = tile_start[t + 1] - base;
  uint32_t c = 0;
  if (sb == X_NONE) {
    c = threadIdx.x == 0 ? b - a : 0u;
  } else {
    for (uint32_t x = 2 * a + 1 + threadIdx.x; x < 2 * b + 1; x += blockDim.x) {
      const uint32_t s = wperm2[sb + x];
      c += (s != 0 && !(s & 1u)) ? 1u : 0u;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tcnt[t] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void k_x2_compact(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase1,
    const uint32_t *__restrict__ sbase2, const uint32_t *__restrict__ toff,
    const uint32_t *__restrict__ wperm2, uint32_t *__restrict__ wperm1,
    uint32_t *__restrict__ ctl) {
  __shared__ uint32_t ws[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase2[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint32_t a = tile_start[t] - base, b = tile_start[t + 1] - base;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t k0 = toff[t] - base;
  for (uint32_t x0 = 2 * a + 1; x0 < 2 * b + 1; x0 += 256) {
    const uint32_t x = x0 + threadIdx.x;
    const uint32_t s = x < 2 * b + 1 ? wperm2[sb + x] : 0u;
    const bool real = s != 0 && !(s & 1u);
    const uint64_t bb = __ballot(real);
    if (lane == 0) ws[wv] = (uint32_t)__popcll(bb);
    __syncthreads();
    uint32_t pre = k0;
    for (uint32_t w = 0; w < wv; w++) pre += ws[w];
    if (real) {
      const uint32_t q = pre + lanes_below(bb);
      if (q < n) wperm1[sbase1[f] + 1 + q] = s >> 1;
      else atomicOr(&ctl[1], 32u);
    }
    k0 += ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
  }
}

// prevne[i] for every appended node i: the previous appended node of its
// document that is not early (sub-batch index), X_NONE if none -- the region
// k_x2_anchor starts from.  A max-scan over the appended list in chunks of 256.
__device__ __forceinline__ uint32_t x_wave_maxscan_incl(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, y);
  }
  return v;
}

// (value k + 1 for a non-early entry k, 0 otherwise) -> the chunk's maximum
__global__ __launch_bounds__(256) void k_x2_ne_chunk(const uint32_t *__restrict__ app_list, uint32_t A,
                                                     const uint8_t *__restrict__ early,
                                                     uint32_t *__restrict__ cmax) {
  __shared__ uint32_t ws[4];
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  uint32_t v = (k < A && !early[app_list[k]]) ? k + 1 : 0u;
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) cmax[blockIdx.x] = max(max(ws[0], ws[1]), max(ws[2], ws[3]));
}

// exclusive max-scan of C chunk maxima in place (one workgroup of 1024)
__global__ __launch_bounds__(1024) void k_x2_ne_scan(uint32_t *__restrict__ cmax, uint32_t C) {
  __shared__ uint32_t wmax[16];
  __shared__ uint32_t carry;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < C; c0 += 1024) {
    const uint32_t c = c0 + threadIdx.x;
    const uint32_t v = c < C ? cmax[c] : 0u;
    const uint32_t inc = x_wave_maxscan_incl(v);
    if (lane == 63) wmax[wv] = inc;
    __syncthreads();
    uint32_t pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre = max(pre, wmax[w]);
    const uint32_t excl = max(pre, (uint32_t)__shfl_up(inc, 1, 64) * (lane > 0 ? 1u : 0u));
    if (c < C) cmax[c] = excl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = max(pre, inc);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_x2_ne_final(const uint32_t *__restrict__ app_list,
                                                     const uint32_t *__restrict__ app_doc, uint32_t A,
                                                     const uint8_t *__restrict__ early,
                                                     const uint32_t *__restrict__ cexcl,
                                                     uint32_t *__restrict__ prevne) {
  __shared__ uint32_t ws[4];
  const uint32_t k = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t v = (k < A && !early[app_list[k]]) ? k + 1 : 0u;
  const uint32_t inc = x_wave_maxscan_incl(v);
  if (lane == 63) ws[wv] = inc;
  __syncthreads();
  uint32_t pre = cexcl[blockIdx.x];
  for (uint32_t w = 0; w < wv; w++) pre = max(pre, ws[w]);
  const uint32_t up = __shfl_up(inc, 1, 64);
  const uint32_t prev = lane > 0 ? max(pre, up) : pre;  // the last non-early entry before k, + 1
  if (k < A)
    prevne[app_list[k]] = (prev != 0 && app_doc[prev - 1] == app_doc[k]) ? app_list[prev - 1] : X_NONE;
}

// The woven synthetic lists -> the caller's outputs: weave_perm (input index per
// position, H dropped), rendered bits and rendered counts.  adj = 0: the
// documents with only[f] == 0 (or all, only == nullptr), render bits of the
// synthetic F5 weave with roots hidden; adj = 1: the documents with only[f],
// hide? (list.cljc:48-55) against the next node of the weave itself.  The tile
// of the sub-batch stands for the same range of output positions q; one thread
// per output word.
__global__ __launch_bounds__(256) void k_xsyn_emit(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint8_t *__restrict__ only, uint32_t adj, const uint32_t *__restrict__ wperm,
    const uint32_t *__restrict__ wbits, const uint8_t *__restrict__ xk,
    const uint32_t *__restrict__ xpar, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ out_off, const uint32_t *__restrict__ out_doc,
    uint32_t *__restrict__ weave_perm, uint32_t *__restrict__ visible_bits,
    uint32_t *__restrict__ visible_count) {
  __shared__ uint32_t wsum[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE || (only ? only[f] != 0 : false) != (adj != 0)) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint32_t q0 = tile_start[t] - base, q1 = tile_start[t + 1] - base;
  const uint64_t g0 = out_off[f];
  // one position a lane, waves over 64-aligned output positions: each wave's
  // bits are two output words (x_flush merges the words a document shares)
  const uint32_t lane = threadIdx.x & 63;
  uint32_t cnt = 0;
  const uint64_t a0 = (g0 + q0) & ~63ull;
  for (uint64_t ga = a0 + (threadIdx.x & ~63u); ga < g0 + q1; ga += blockDim.x) {
    const uint64_t g = ga + lane;
    const bool in = g >= g0 + q0 && g < g0 + q1;
    bool vis = false;
    if (in) {
      const uint32_t q = (uint32_t)(g - g0), x = sb + 1 + q;  // synthetic position
      const uint32_t i = base + wperm[x] - 1;
      weave_perm[g] = sval ? sval[i] : i - base;
      const uint8_t k = xk[i];
      if (adj) {
        vis = !(k & (KIND_CLASS | KIND_ROOT));
        if (vis && q + 1 < n) {
          const uint32_t j = base + wperm[x + 1] - 1;
          vis = !(is_hide(xk[j]) && xpar[j] == i - base);
        }
      } else {
        vis = ((wbits[x >> 5] >> (x & 31)) & 1u) && !(k & KIND_ROOT);
      }
    }
    const uint64_t m = __ballot(in), v = __ballot(vis);
    cnt += vis ? 1u : 0u;
    if (visible_bits && (lane == 0 || lane == 32)) {
      const uint32_t sh = lane;
      const uint32_t mw = (uint32_t)(m >> sh);
      if (mw) x_flush(visible_bits, (ga >> 5) + (lane >> 5), mw, (uint32_t)(v >> sh));
    }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&visible_count[out_doc[f]], wsum[0] + wsum[1] + wsum[2] + wsum[3]);
}

__global__ __launch_bounds__(64) void k_xsyn_zero(const uint32_t *__restrict__ sbase, uint32_t F,
                                                  const uint32_t *__restrict__ out_doc,
                                                  uint32_t *__restrict__ visible_count) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F && sbase[f] != X_NONE) visible_count[out_doc[f]] = 0;
}

namespace {

// Upload a host array to named scratch (blocking copy: the stream is idle).
template <typename T>
T *x_upload(cw_ctx *c, const char *name, const std::vector<T> &h) {
  T *d = scratch_t<T>(c, name, h.size());
  if (!d) return nullptr;
  if (!h.empty() && hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
    return nullptr;
  return d;
}

// The upper levels of a min-tree over a (len entries, a multiple of 16,
// padded with MT_MAX) into scratch `name`.
int mt_build(cw_ctx *c, const char *name, const uint32_t *a, uint64_t len, XMinTree *t) {
  std::vector<uint64_t> lens{len};
  while (lens.back() > 16) lens.push_back(((lens.back() / 16) + 15) & ~15ull);
  if (lens.size() > MT_LEVELS || len >= 0xFFFFFFFFull) return fail(c, "exact path: min-tree of %llu", (unsigned long long)len);
  uint64_t tot = 16;
  for (size_t l = 1; l < lens.size(); l++) tot += lens[l];
  uint32_t *up = scratch_t<uint32_t>(c, name, tot);
  if (!up) return fail(c, "out of device memory (%s)", name);
  t->levels = (uint32_t)lens.size();
  t->lv[0] = a;
  t->len[0] = (uint32_t)len;
  for (size_t l = 1; l < lens.size(); l++) {
    t->lv[l] = up;
    t->len[l] = (uint32_t)lens[l];
    hipLaunchKernelGGL(k_mt_level, dim3((uint32_t)((lens[l] + 255) / 256)), dim3(256), 0, c->stream,
                       t->lv[l - 1], t->len[l - 1], up, t->len[l]);
    up += lens[l];
  }
  return check_launch(c, "mt_level");
}

// The flagged documents after the join (xpar: cause rank / X_NIL / X_END by
// rank, xk: kinds by rank, early: "has an older child" by rank, sval: input
// index by rank or nullptr; dearly / dapp: per document "has an early node"
// and its number of appended nodes): every document woven by the synthetic
// lists (phase 1, and phase 2 rounds for one with an early node), outputs
// written at out_off.
int exact_weave_flagged(cw_ctx *c, uint32_t F, const std::vector<uint64_t> &xoff,
                        const uint32_t *xpar, const uint8_t *xk, const uint8_t *early,
                        const uint32_t *sval, const uint64_t *d_oof, const uint32_t *d_odoc,
                        const uint8_t *dearly, const uint32_t *dapp, cw_list_result *out) {
  const uint32_t NX = (uint32_t)xoff.back();
  if (ensure_tables(c, F, xoff.data())) return -1;
  uint32_t *tile_start = dev_tab(c, "t_tile_start"), *tile_doc = dev_tab(c, "t_tile_doc"),
           *sub_off = dev_tab(c, "t_doc_off");
  const dim3 B256(256), GF((F + 63) / 64), B64(64);
  const uint32_t T = c->tab.T;
  if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
  std::vector<uint8_t> h_early(F), run(F, 0), x2(F, 0);
  std::vector<uint32_t> h_app(F);
  HIPCHK(c, hipMemcpyAsync(h_early.data(), dearly, F, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h_app.data(), dapp, (size_t)F * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // synthetic lists: documents without an early node, documents with one
  // (phase 2 reweaves only those), then each giant document on its own
  struct Group {
    bool giant, early;
    uint64_t base;  // first synthetic index (a multiple of 32: its bits start a word)
    std::vector<uint64_t> off;
  };
  std::vector<Group> groups;
  std::vector<uint32_t> sb(F, X_NONE);
  uint64_t NS = 0, A = 0;
  bool any_serial = false, any_x2 = false;
  {
    std::vector<uint32_t> small[2], big;
    for (uint32_t f = 0; f < F; f++) {
      const uint64_t n = xoff[f + 1] - xoff[f];
      if (c->xfold && h_early[f] && n <= XFOLD_MAX) {  // CW_XFOLD: the serial fold (cross-check)
        run[f] = 1;
        any_serial = true;
        continue;
      }
      A += h_app[f];
      x2[f] = h_early[f] ? 1 : 0;
      any_x2 |= h_early[f] != 0;
      if (n + 1 >= c->giant_min || n + 1 >= LINK_IDX) big.push_back(f);
      else small[h_early[f] ? 1 : 0].push_back(f);
    }
    for (int e = 0; e < 2; e++) {
      if (small[e].empty()) continue;
      Group g{false, e == 1, NS, {0}};
      for (uint32_t f : small[e]) {
        sb[f] = (uint32_t)(NS + g.off.back());
        g.off.push_back(g.off.back() + (xoff[f + 1] - xoff[f]) + 1);
      }
      NS = (NS + g.off.back() + 31) & ~31ull;
      groups.push_back(std::move(g));
    }
    for (uint32_t f : big) {
      const uint64_t n = xoff[f + 1] - xoff[f];
      sb[f] = (uint32_t)NS;
      groups.push_back(Group{true, h_early[f] != 0, NS, {0, n + 1}});
      NS = (NS + n + 1 + 31) & ~31ull;
    }
  }
  if (NS >= 0xFFFFFFF0ull - 16) return fail(c, "exact path: %llu synthetic nodes", (unsigned long long)NS);
  c->x_iters = 0;
  if (!groups.empty()) {
    const uint64_t NP = ((NS + 15) & ~15ull) + 16;  // min-tree level 0, padded
    uint32_t *d_sb = x_upload(c, "x_sbase", sb);
    uint8_t *d_x2 = x_upload(c, "x_x2", x2);
    uint32_t *spar = scratch_t<uint32_t>(c, "x_spar", NS), *wperm = scratch_t<uint32_t>(c, "x_wperm", NS);
    uint8_t *skd = scratch_t<uint8_t>(c, "x_skd", NS);
    uint32_t *wbits = scratch_t<uint32_t>(c, "x_wbits", NS / 32 + 1);
    uint32_t *G = scratch_t<uint32_t>(c, "x_G", NP), *AUX = scratch_t<uint32_t>(c, "x_aux", NP);
    uint32_t *posA = scratch_t<uint32_t>(c, "x_pos", NS), *ctop = scratch_t<uint32_t>(c, "x_ctop", NS);
    uint32_t *Nof = scratch_t<uint32_t>(c, "x_nof", NS), *ctl = scratch_t<uint32_t>(c, "x_ctl", 2);
    size_t gmax = 1;
    for (auto &g : groups) gmax = std::max(gmax, g.off.size() - 1);
    uint32_t *wvc = scratch_t<uint32_t>(c, "x_wvc", gmax), *wst = scratch_t<uint32_t>(c, "x_wst", gmax);
    if (!d_sb || !d_x2 || !spar || !wperm || !skd || !wbits || !G || !AUX || !posA || !ctop || !Nof ||
        !ctl || !wvc || !wst)
      return fail(c, "out of device memory (exact path, %llu synthetic nodes)", (unsigned long long)NS);
    HIPCHK(c, hipMemsetAsync(ctl, 0, 8, c->stream));
    // weave the synthetic lists of every group (or only those with an early node)
    auto weave_groups = [&](bool early_only) -> int {
      for (auto &g : groups) {
        if (early_only && !g.early) continue;
        const uint64_t Dg = g.off.size() - 1, Ng = g.off.back();
        if (ensure_tables(c, Dg, g.off.data(), g.giant)) return -1;
        HIPCHK(c, hipMemsetAsync(wst, 0, Dg * 4, c->stream));
        HIPCHK(c, hipMemsetAsync(wvc, 0, Dg * 4, c->stream));
        HIPCHK(c, hipMemsetAsync(wbits + g.base / 32, 0, (Ng + 31) / 32 * 4, c->stream));
        cw_list_result sr{};
        sr.weave_perm = wperm + g.base;
        sr.visible_bits = wbits + g.base / 32;
        sr.visible_count = wvc;
        sr.status = wst;
        if (weave_tail(c, Dg, (uint32_t)Ng, g.giant, spar + g.base, skd + g.base, nullptr, nullptr,
                       nullptr, 0, &sr))
          return -1;
        c->x_iters++;
      }
      if (ensure_tables(c, F, xoff.data())) return -1;  // the flagged documents' tiles again
      tile_start = dev_tab(c, "t_tile_start");
      tile_doc = dev_tab(c, "t_tile_doc");
      sub_off = dev_tab(c, "t_doc_off");
      return 0;
    };
    auto positions = [&](uint32_t mode, const uint8_t *only, uint32_t *pos, const uint32_t *posold) -> int {
      HIPCHK(c, hipMemsetAsync(G, 0xFF, NP * 4, c->stream));
      HIPCHK(c, hipMemsetAsync(AUX, 0xFF, NP * 4, c->stream));
      Launch L(c, "xsyn_pos", (double)NX * 13);
      hipLaunchKernelGGL(k_xs_pos, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb, only,
                         wperm, skd, xk, mode, G, AUX, pos, posold, ctl);
      return check_launch(c, "xsyn_pos");
    };
    // phase 1: the static forest, every appended node's T, the final weave
    hipLaunchKernelGGL(k_xsyn_build, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                       xpar, xk, spar, skd);
    if (check_launch(c, "xsyn_build")) return -1;
    if (weave_groups(false)) return -1;
    uint32_t *app_list = nullptr, *app_idx = nullptr;
    if (A > 0) {
      if (positions(0, nullptr, posA, nullptr)) return -1;
      XMinTree mt, mtx;
      if (mt_build(c, "x_mtG", G, NP, &mt) || mt_build(c, "x_mtA", AUX, NP, &mtx)) return -1;
      app_list = scratch_t<uint32_t>(c, "x_app", A);
      app_idx = scratch_t<uint32_t>(c, "x_appidx", NX);
      uint32_t *app_doc = scratch_t<uint32_t>(c, "x_appdoc", A), *Tsyn = scratch_t<uint32_t>(c, "x_T", A);
      uint32_t *tcnt = scratch_t<uint32_t>(c, "x_tcnt", T);
      if (!app_list || !app_idx || !app_doc || !Tsyn || !tcnt)
        return fail(c, "out of device memory (exact path, %llu appended nodes)", (unsigned long long)A);
      const uint32_t A32 = (uint32_t)A;
      {
        Launch L(c, "xsyn_resolve", (double)NX * 16 + (double)A * 256);
        hipLaunchKernelGGL(k_xctop, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb, spar,
                           skd, ctop);
        hipLaunchKernelGGL(k_xapp_count, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                           xpar, tcnt);
        hipLaunchKernelGGL(k_xapp_scan, dim3(1), dim3(1024), 0, c->stream, tcnt, T);
        hipLaunchKernelGGL(k_xapp_scatter, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off,
                           d_sb, xpar, tcnt, app_list, app_doc, app_idx);
        HIPCHK(c, hipMemsetAsync(Nof, 0xFF, NS * 4, c->stream));
        hipLaunchKernelGGL(k_xres1, dim3((A32 + 255) / 256), B256, 0, c->stream, app_list, app_doc, A32,
                           sub_off, d_sb, xk, posA, G, ctop, mt, Tsyn, Nof, ctl);
        hipLaunchKernelGGL(k_xres2, dim3(A32), B64, 0, c->stream, app_list, app_doc, A32, sub_off, d_sb,
                           xpar, xk, posA, G, ctop, mt, mtx, Tsyn, Nof, ctl);
        hipLaunchKernelGGL(k_xsyn_final, dim3((A32 + 255) / 256), B256, 0, c->stream, app_list, app_doc,
                           A32, sub_off, d_sb, xk, Tsyn, spar, skd);
      }
      if (check_launch(c, "xsyn_resolve")) return -1;
      if (weave_groups(false)) return -1;
    }
    // phase 2: documents with an early node, anchor rounds on layout 2 from
    // phase 1's weave until the weave reproduces itself (the fold's, by
    // induction over the nodes in id order); a small document still moving
    // after X_ROUND_CAP rounds is folded serially instead
    if (any_x2) {
      std::vector<uint32_t> sb2(F, X_NONE);
      std::vector<Group> groups2;
      uint64_t NS2 = 0;
      uint32_t nmax = 1;
      {
        std::vector<uint32_t> small2, big2;
        for (uint32_t f = 0; f < F; f++) {
          if (!x2[f]) continue;
          const uint64_t n = xoff[f + 1] - xoff[f];
          nmax = std::max<uint32_t>(nmax, (uint32_t)n);
          if (2 * n + 1 >= c->giant_min || 2 * n + 1 >= LINK_IDX) big2.push_back(f);
          else small2.push_back(f);
        }
        if (!small2.empty()) {
          Group g{false, true, NS2, {0}};
          for (uint32_t f : small2) {
            sb2[f] = (uint32_t)(NS2 + g.off.back());
            g.off.push_back(g.off.back() + 2 * (xoff[f + 1] - xoff[f]) + 1);
          }
          NS2 = (NS2 + g.off.back() + 31) & ~31ull;
          groups2.push_back(std::move(g));
        }
        for (uint32_t f : big2) {
          const uint64_t n = xoff[f + 1] - xoff[f];
          sb2[f] = (uint32_t)NS2;
          groups2.push_back(Group{true, true, NS2, {0, 2 * n + 1}});
          NS2 = (NS2 + 2 * n + 1 + 31) & ~31ull;
        }
      }
      if (NS2 >= 0xFFFFFFF0ull - 16) return fail(c, "exact path: %llu layout-2 nodes", (unsigned long long)NS2);
      const uint64_t NP2 = ((NS2 + 15) & ~15ull) + 16;
      uint32_t *d_sb2 = x_upload(c, "x_sbase2", sb2);
      uint8_t *d_only = x_upload(c, "x_only", x2);
      uint32_t *spar2 = scratch_t<uint32_t>(c, "x_spar2", NS2), *wperm2 = scratch_t<uint32_t>(c, "x_wperm2", NS2);
      uint8_t *skd2 = scratch_t<uint8_t>(c, "x_skd2", NS2);
      uint32_t *wbits2 = scratch_t<uint32_t>(c, "x_wbits2", NS2 / 32 + 1);
      uint32_t *G2 = scratch_t<uint32_t>(c, "x_G2", NP2), *AUX2 = scratch_t<uint32_t>(c, "x_aux2", NP2);
      uint32_t *p2A = scratch_t<uint32_t>(c, "x_pos2A", NS2), *p2B = scratch_t<uint32_t>(c, "x_pos2B", NS2);
      uint32_t *xf = scratch_t<uint32_t>(c, "x_xf", NX), *anc = scratch_t<uint32_t>(c, "x_anc", NX);
      uint32_t *jmp = scratch_t<uint32_t>(c, "x_jmp", NX), *prevne = scratch_t<uint32_t>(c, "x_prevne", NX);
      uint8_t *hasb = scratch_t<uint8_t>(c, "x_hasb", NX), *moved = scratch_t<uint8_t>(c, "x_moved", F);
      size_t gmax2 = 1;
      for (auto &g : groups2) gmax2 = std::max(gmax2, g.off.size() - 1);
      uint32_t *wvc2 = scratch_t<uint32_t>(c, "x_wvc", std::max(gmax, gmax2)),
               *wst2 = scratch_t<uint32_t>(c, "x_wst", std::max(gmax, gmax2));
      if (!d_sb2 || !d_only || !spar2 || !wperm2 || !skd2 || !wbits2 || !G2 || !AUX2 || !p2A || !p2B || !xf ||
          !anc || !jmp || !prevne || !hasb || !moved || !wvc2 || !wst2)
        return fail(c, "out of device memory (exact path rounds, %llu layout-2 nodes)", (unsigned long long)NS2);
      if (A > 0) {  // the previous non-early appended node of every appended node
        const uint32_t A32 = (uint32_t)A, C = (A32 + 255) / 256;
        uint32_t *cmax = scratch_t<uint32_t>(c, "x_necmax", C);
        uint32_t *app_doc = scratch_t<uint32_t>(c, "x_appdoc", A);
        if (!cmax || !app_doc) return fail(c, "out of device memory (exact path rounds)");
        Launch L(c, "xins_prevne", (double)A * 14);
        hipLaunchKernelGGL(k_x2_ne_chunk, dim3(C), B256, 0, c->stream, app_list, A32, early, cmax);
        hipLaunchKernelGGL(k_x2_ne_scan, dim3(1), dim3(1024), 0, c->stream, cmax, C);
        hipLaunchKernelGGL(k_x2_ne_final, dim3(C), B256, 0, c->stream, app_list, app_doc, A32, early, cmax,
                           prevne);
      }
      if (check_launch(c, "xins_prevne")) return -1;
      auto positions2 = [&](uint32_t from1, uint32_t *pos, const uint32_t *posold) -> int {
        HIPCHK(c, hipMemsetAsync(G2, 0xFF, NP2 * 4, c->stream));
        HIPCHK(c, hipMemsetAsync(AUX2, 0xFF, NP2 * 4, c->stream));
        Launch L(c, "xsyn_pos", (double)NX * 26);
        hipLaunchKernelGGL(k_x2_pos, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb, d_sb2,
                           d_only, from1, wperm, wperm2, xk, G2, AUX2, pos, posold, moved, ctl);
        return check_launch(c, "xsyn_pos");
      };
      if (positions2(1, p2A, nullptr)) return -1;
      // launches of k_x2_jump: reach (X2_JUMPS + 1)^launches >= nmax
      uint32_t jumps = 1;
      for (uint64_t reach = 1; reach < nmax; reach *= X2_JUMPS + 1) jumps++;
      std::vector<uint8_t> only(x2), h_moved(F);
      for (uint32_t round = 0;; round++) {
        XMinTree mt, mtn;
        if (mt_build(c, "x_mtG", G2, NP2, &mt) || mt_build(c, "x_mtA", AUX2, NP2, &mtn)) return -1;
        {
          Launch L(c, "xins_round", (double)NX * (40 + 8 * jumps));
          HIPCHK(c, hipMemsetAsync(xf, 0xFF, (size_t)NX * 4, c->stream));
          HIPCHK(c, hipMemsetAsync(hasb, 0, NX, c->stream));
          hipLaunchKernelGGL(k_x2_xf, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2, d_only,
                             xpar, p2A, xf);
          hipLaunchKernelGGL(k_x2_anchor, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2,
                             d_only, xpar, xk, xf, prevne, p2A, G2, mt, mtn, round == 0 ? 1u : 0u, anc, ctl);
          hipLaunchKernelGGL(k_x2_chain, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2,
                             d_only, anc, jmp, hasb);
          for (uint32_t j = 0; j < jumps; j++)
            hipLaunchKernelGGL(k_x2_jump, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2,
                               d_only, jmp);
          hipLaunchKernelGGL(k_x2_build, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2,
                             d_only, anc, jmp, hasb, spar2, skd2);
        }
        if (check_launch(c, "xins_round")) return -1;
        // weave the layout-2 groups that hold a moving document
        for (auto &g : groups2) {
          bool any = false;
          for (uint32_t f = 0; f < F && !any; f++)
            any = only[f] && sb2[f] >= g.base && sb2[f] < g.base + g.off.back();
          if (!any) continue;
          const uint64_t Dg = g.off.size() - 1, Ng = g.off.back();
          if (ensure_tables(c, Dg, g.off.data(), g.giant)) return -1;
          HIPCHK(c, hipMemsetAsync(wst2, 0, Dg * 4, c->stream));
          HIPCHK(c, hipMemsetAsync(wvc2, 0, Dg * 4, c->stream));
          cw_list_result sr{};
          sr.weave_perm = wperm2 + g.base;
          sr.visible_bits = wbits2 + g.base / 32;
          sr.visible_count = wvc2;
          sr.status = wst2;
          if (weave_tail(c, Dg, (uint32_t)Ng, g.giant, spar2 + g.base, skd2 + g.base, nullptr, nullptr,
                         nullptr, 0, &sr))
            return -1;
          c->x_iters++;
        }
        if (ensure_tables(c, F, xoff.data())) return -1;
        tile_start = dev_tab(c, "t_tile_start");
        tile_doc = dev_tab(c, "t_tile_doc");
        sub_off = dev_tab(c, "t_doc_off");
        HIPCHK(c, hipMemsetAsync(moved, 0, F, c->stream));
        if (positions2(0, p2B, p2A)) return -1;
        std::swap(p2A, p2B);
        HIPCHK(c, hipMemcpyAsync(c->pin_small, ctl, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(h_moved.data(), moved, F, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->pin_small[1]) return fail(c, "exact path: inconsistent synthetic weave (%u)", c->pin_small[1]);
        bool more = false;
        for (uint32_t f = 0; f < F; f++) {
          only[f] = only[f] && h_moved[f];  // a document that reproduced its weave is done
          if (only[f] && round + 1 >= c->x_round_cap && xoff[f + 1] - xoff[f] <= X_CAP_FOLD_MAX) {
            only[f] = 0;  // small and still moving: the serial fold (emitted after the synthetic lists)
            run[f] = 1;
            any_serial = true;
          }
          more |= only[f] != 0;
        }
        if (!more) break;
        if (round > NX + 2) return fail(c, "exact path: no fixed point after %u rounds", round);
        HIPCHK(c, hipMemcpy(d_only, only.data(), F, hipMemcpyHostToDevice));
      }
      // the converged layout-2 weaves back into layout 1 for the emission
      uint32_t *tcnt2 = scratch_t<uint32_t>(c, "x_tcnt", T);
      if (!tcnt2) return fail(c, "out of device memory (exact path)");
      {
        Launch L(c, "xsyn_compact", (double)NX * 16);
        hipLaunchKernelGGL(k_x2_count, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb2, wperm2,
                           tcnt2);
        hipLaunchKernelGGL(k_xapp_scan, dim3(1), dim3(1024), 0, c->stream, tcnt2, T);
        hipLaunchKernelGGL(k_x2_compact, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                           d_sb2, tcnt2, wperm2, wperm, ctl);
      }
      if (check_launch(c, "xsyn_compact")) return -1;
    }
    HIPCHK(c, hipMemcpyAsync(c->pin_small, ctl, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->pin_small[1]) return fail(c, "exact path: inconsistent synthetic weave (%u)", c->pin_small[1]);
    hipLaunchKernelGGL(k_xsyn_zero, GF, B64, 0, c->stream, d_sb, F, d_odoc, out->visible_count);
    for (uint32_t adj = 0; adj < (any_x2 ? 2u : 1u); adj++) {
      Launch L(c, "xsyn_emit", (double)NX * (4 + 4 + 4 + 1) + (double)NX / 8);
      hipLaunchKernelGGL(k_xsyn_emit, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb, d_x2,
                         adj, wperm, wbits, xk, xpar, sval, d_oof, d_odoc, out->weave_perm,
                         out->visible_bits, out->visible_count);
    }
    if (check_launch(c, "xsyn_emit")) return -1;
  }
  if (any_serial) {  // CW_XFOLD: the literal fold, one lane a document
    uint8_t *d_run = x_upload(c, "x_run", run);
    uint32_t *xnext = scratch_t<uint32_t>(c, "x_next", NX);
    if (!d_run || !xnext) return fail(c, "out of device memory (exact path)");
    Launch L(c, "xfold", (double)NX * 22);
    hipLaunchKernelGGL(k_xfold, GF, B64, 0, c->stream, sub_off, F, xpar, xk, early, xnext, sval,
                       d_oof, d_odoc, out->weave_perm, out->visible_bits, out->visible_count, d_run);
  }
  return check_launch(c, "xfold");
}

// exact_fixup for one giant list whose front end left its sorted ids and rank
// directory (cw_ctx::xfront): no gather, no second sort, the join through the
// directory (k_xjoin_dir), then the same path as every flagged document.
int exact_giant_front(cw_ctx *c, const cw_list_batch *bt, cw_list_result *out) {
  const auto &xf = c->xfront;
  const uint32_t N = xf.n;
  const std::vector<uint64_t> xoff = {0, N};
  if (ensure_tables(c, 1, xoff.data())) return -1;
  uint8_t *xk = scratch_t<uint8_t>(c, "x_k", N), *early = scratch_t<uint8_t>(c, "x_early", N);
  uint8_t *dearly = scratch_t<uint8_t>(c, "x_dearly", 1);
  uint32_t *dorph = scratch_t<uint32_t>(c, "x_dorph", 1), *xpar = scratch_t<uint32_t>(c, "x_par", N);
  uint32_t *odoc = scratch_t<uint32_t>(c, "x_rodoc", 1);
  uint64_t *oof = scratch_t<uint64_t>(c, "x_roof", 1);
  if (!xk || !early || !dearly || !dorph || !xpar || !odoc || !oof)
    return fail(c, "out of device memory (exact path, %u nodes)", N);
  HIPCHK(c, hipMemsetAsync(odoc, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(oof, 0, 8, c->stream));
  HIPCHK(c, hipMemsetAsync(early, 0, N, c->stream));
  HIPCHK(c, hipMemsetAsync(dearly, 0, 1, c->stream));
  HIPCHK(c, hipMemsetAsync(dorph, 0, 4, c->stream));
  {
    Launch L(c, "xjoin", (double)N * (4 + 8 + 4 + 1) + (double)N * 64);
    hipLaunchKernelGGL(k_xjoin_dir, dim3((N + 255) / 256), dim3(256), 0, c->stream, xf.skey, xf.sval,
                       bt->cause_key, bt->kind, xf.ckk, N, xf.dir, xf.E, xpar, xk, early, dearly, dorph);
  }
  if (check_launch(c, "xjoin")) return -1;
  if (out->max_ts) {
    hipLaunchKernelGGL(k_xmaxts, dim3(1), dim3(64), 0, c->stream, dev_tab(c, "t_doc_off"), 1u, xf.skey,
                       bt->ts_shift, odoc, out->max_ts);
    if (check_launch(c, "xmaxts")) return -1;
  }
  if (out->yarn_perm && bt->site_bits) {  // spin: the id order partitioned by site
    uint64_t *ykA = scratch_t<uint64_t>(c, "x_skA", N), *ykB = scratch_t<uint64_t>(c, "x_skB", N);
    uint32_t *yvA = scratch_t<uint32_t>(c, "x_svA", N), *yvB = scratch_t<uint32_t>(c, "x_yv", N);
    if (!ykA || !ykB || !yvA || !yvB) return fail(c, "out of device memory (exact path yarns)");
    uint64_t *yk;
    uint32_t *yv;
    if (radix_sort<uint64_t>(c, "xyarns", xf.skey, xf.sval, ykA, yvA, ykB, yvB, bt->site_bits,
                             bt->site_shift, N, &yk, &yv))
      return -1;
    HIPCHK(c, hipMemcpyAsync(out->yarn_perm, yv, (size_t)N * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  return exact_weave_flagged(c, 1, xoff, xpar, xk, early, xf.sval, oof, odoc, dearly, dorph, out);
}

// After the fast path has woven a batch (device arrays id/cause/kind laid out
// by bt->doc_offsets, results in `out`): reweave its flagged documents by the
// literal fold and overwrite their weave_perm, rendered bits and count, and
// (when asked for) ::lamport-ts and yarns.  Status bits stay: they say the
// document is one the reference's s/insert would have refused.  `hint` = 0
// when the front end reported no flagged document (no readback needed).
int exact_fixup(cw_ctx *c, const cw_list_batch *bt, const uint64_t *id, const uint64_t *cause,
                const uint8_t *kind, cw_list_result *out, bool hint) {
  const uint64_t D = bt->n_docs;
  const uint64_t *off = bt->doc_offsets;
  if (!hint || D == 0 || off[D] == 0) return 0;
  if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
  if (D == 1 && c->x_pending && bt->key_bits && bt->key_bits < 64) {
    // one giant list: its status was copied out after the front end (KEY_RANGE,
    // set later, needs key_bits >= 64); wait for that copy, not for the stream
    HIPCHK(c, hipEventSynchronize(c->ev_status));
    const uint32_t st = c->pin_status[0];
    if (!(st & X_MASK) || (st & X_SKIP)) return 0;
    if (c->xfront.ok && c->xfront.n == off[1]) return exact_giant_front(c, bt, out);
  } else if (D <= 16) {
    // a few documents: their status words in one readback
    HIPCHK(c, hipMemcpyAsync(c->pin_small, out->status, D * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    bool any = false;
    for (uint64_t d = 0; d < D; d++)
      any |= (c->pin_small[d] & X_MASK) && !(c->pin_small[d] & X_SKIP) && off[d + 1] > off[d];
    if (!any) return 0;
  }
  uint32_t *cnt = scratch_t<uint32_t>(c, "x_cnt", 1);
  uint32_t *doff = scratch_t<uint32_t>(c, "x_doff", D + 1);
  if (!cnt || !doff) return fail(c, "out of device memory (exact path)");
  {
    std::vector<uint32_t> h(D + 1);
    for (uint64_t d = 0; d <= D; d++) h[d] = (uint32_t)off[d];
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(doff, h.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  }
  HIPCHK(c, hipMemsetAsync(cnt, 0, 4, c->stream));
  hipLaunchKernelGGL(k_xcount, dim3((uint32_t)((D + 255) / 256)), dim3(256), 0, c->stream,
                     out->status, doff, (uint32_t)D, cnt);
  if (check_launch(c, "xcount")) return -1;
  HIPCHK(c, hipMemcpyAsync(c->pin_small, cnt, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->pin_small[0] == 0) return 0;
  // which documents
  std::vector<uint32_t> st(D);
  HIPCHK(c, hipMemcpy(st.data(), out->status, D * 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> xoff(1, 0), src;
  std::vector<uint32_t> odoc;
  for (uint64_t d = 0; d < D; d++) {
    if (!(st[d] & X_MASK) || (st[d] & X_SKIP) || off[d + 1] == off[d]) continue;
    src.push_back(off[d]);
    odoc.push_back((uint32_t)d);
    xoff.push_back(xoff.back() + (off[d + 1] - off[d]));
  }
  const uint32_t F = (uint32_t)odoc.size(), NX = (uint32_t)xoff.back();
  if (ensure_tables(c, F, xoff.data())) return -1;
  uint64_t *d_src = x_upload(c, "x_src", src);
  uint32_t *d_odoc = x_upload(c, "x_odoc", odoc);
  // (names of their own: the synthetic lists below run the list pipeline's tail)
  uint64_t *xid = scratch_t<uint64_t>(c, "x_id", NX), *xca = scratch_t<uint64_t>(c, "x_cause", NX);
  uint8_t *xkd = scratch_t<uint8_t>(c, "x_kind", NX), *xk = scratch_t<uint8_t>(c, "x_k", NX);
  uint8_t *early = scratch_t<uint8_t>(c, "x_early", NX), *dearly = scratch_t<uint8_t>(c, "x_dearly", F);
  uint32_t *dorph = scratch_t<uint32_t>(c, "x_dorph", F);
  uint64_t *skA = scratch_t<uint64_t>(c, "x_skA", NX), *skB = scratch_t<uint64_t>(c, "x_skB", NX);
  uint32_t *svA = scratch_t<uint32_t>(c, "x_svA", NX), *svB = scratch_t<uint32_t>(c, "x_svB", NX);
  uint32_t *xpar = scratch_t<uint32_t>(c, "x_par", NX);
  if (!d_src || !d_odoc || !xid || !xca || !xkd || !xk || !early || !dearly || !dorph || !skA || !skB ||
      !svA || !svB || !xpar)
    return fail(c, "out of device memory (exact path, %u nodes)", NX);
  uint32_t *tile_start = dev_tab(c, "t_tile_start"), *tile_doc = dev_tab(c, "t_tile_doc"),
           *sub_off = dev_tab(c, "t_doc_off");
  const dim3 B256(256), GF((F + 63) / 64), B64(64);
  const uint32_t T = c->tab.T;
  {
    Launch L(c, "xgather", (double)NX * 34);
    hipLaunchKernelGGL(k_xgather, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_src, id,
                       cause, kind, xid, xca, xkd);
  }
  if (check_launch(c, "xgather")) return -1;
  uint32_t key_bits = bt->key_bits;
  if (key_bits == 0 && find_key_bits(c, xid, NX, &key_bits)) return -1;
  if (key_bits > 64) key_bits = 64;
  uint64_t *skey;
  uint32_t *sval;
  if (radix_sort<uint64_t>(c, "xsort", xid, nullptr, skA, svA, skB, svB, key_bits, 0, NX, &skey,
                           &sval))
    return -1;
  HIPCHK(c, hipMemsetAsync(early, 0, NX, c->stream));
  HIPCHK(c, hipMemsetAsync(dearly, 0, F, c->stream));
  HIPCHK(c, hipMemsetAsync(dorph, 0, (size_t)F * 4, c->stream));
  {
    Launch L(c, "xjoin", (double)NX * 30);
    hipLaunchKernelGGL(k_xjoin, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, skey, sval,
                       xca, xkd, xpar, xk, early, dearly, dorph);
  }
  if (check_launch(c, "xjoin")) return -1;
  uint64_t *d_oof;
  {
    std::vector<uint64_t> oof(F);
    for (uint32_t f = 0; f < F; f++) oof[f] = src[f];
    d_oof = x_upload(c, "x_oof", oof);
    if (!d_oof) return fail(c, "out of device memory (exact path)");
  }
  // ::lamport-ts and the yarns (spin 1-arity: the id order partitioned by
  // site) do not depend on the weave
  if (out->max_ts) {
    hipLaunchKernelGGL(k_xmaxts, GF, B64, 0, c->stream, sub_off, F, skey, bt->ts_shift, d_odoc,
                       out->max_ts);
    if (check_launch(c, "xmaxts")) return -1;
  }
  if (out->yarn_perm && bt->site_bits) {
    uint64_t *ykA = skey == skA ? skB : skA;
    uint32_t *yvA = sval == svA ? svB : svA;
    uint32_t *yvB = scratch_t<uint32_t>(c, "x_yv", NX);
    if (!yvB) return fail(c, "out of device memory (exact path yarns)");
    uint64_t *yk;
    uint32_t *yv;
    if (radix_sort<uint64_t>(c, "xyarns", skey, sval, ykA, yvA, xid, yvB, bt->site_bits,
                             bt->site_shift, NX, &yk, &yv))
      return -1;
    hipLaunchKernelGGL(k_xscatter, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_oof, yv,
                       out->yarn_perm);
    if (check_launch(c, "xscatter")) return -1;
  }
  return exact_weave_flagged(c, F, xoff, xpar, xk, early, sval, d_oof, d_odoc, dearly, dorph, out);
}

// cw_weave_ranked's exact path: the one list given by (par, kind) in rank order
// (the same path as exact_fixup's documents).
int exact_ranked(cw_ctx *c, const cw_ranked_list *l, cw_list_result *out) {
  const uint32_t n = (uint32_t)l->n;
  uint32_t *xpar = scratch_t<uint32_t>(c, "x_par", n), *dorph = scratch_t<uint32_t>(c, "x_dorph", 1);
  uint8_t *early = scratch_t<uint8_t>(c, "x_early", n), *dearly = scratch_t<uint8_t>(c, "x_dearly", 1);
  uint32_t *odoc = scratch_t<uint32_t>(c, "x_rodoc", 1);
  uint64_t *oof = scratch_t<uint64_t>(c, "x_roof", 1);
  if (!xpar || !dorph || !early || !dearly || !odoc || !oof)
    return fail(c, "out of device memory (exact path, %u nodes)", n);
  HIPCHK(c, hipMemsetAsync(odoc, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(oof, 0, 8, c->stream));
  HIPCHK(c, hipMemsetAsync(early, 0, n, c->stream));
  HIPCHK(c, hipMemsetAsync(dearly, 0, 1, c->stream));
  HIPCHK(c, hipMemsetAsync(dorph, 0, 4, c->stream));
  hipLaunchKernelGGL(k_xranked_prep, dim3((n + 255) / 256), dim3(256), 0, c->stream, l->par, l->kind,
                     n, xpar, early, dearly, dorph);
  if (check_launch(c, "xranked_prep")) return -1;
  const std::vector<uint64_t> xoff = {0, n};
  return exact_weave_flagged(c, 1, xoff, xpar, l->kind, early, l->val, oof, odoc, dearly, dorph, out);
}

}  // namespace
