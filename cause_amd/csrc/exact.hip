// exact.hip -- the exact path: the reference's full reweave for documents the
// fast path flags as outside its domain.  Included by causeweave.hip after the
// host helpers (scratch, radix_sort, ensure_tables, Launch) it uses.
//
// The fast path assumes every cause is present and older than
// its node and the root [[0 "0" 0] nil nil] is the smallest id.  The reference
// assumes none of this: c.list/weave folds s/weave-node over (sort ::nodes)
// (list.cljc:26-28, shared.cljc:225-241) whatever the causes are.  Documents
// with status ORPHAN, NON_LAMPORT or ROOT (and no DUP: ::nodes is a map, so the
// reference never sees a repeated id) are rewoven here by that fold.
//
// The fold, restated for a full reweave.  Nodes arrive in ascending id order,
// so every node nr already in the weave has a smaller id than the incoming m:
//   * clause C of weave-later? (:220-223) needs (<< (first m) (first nr)):
//     never true; clause B (:213-219) implies C: never true;
//   * clause A (:208-212) is special(nr) & cause(nr) != id(m) & !special(m);
//   * weave-asap? (:194-200) first holds at the split right after cause(m), at
//     split 0 when cause(m) is nil ((first nil) = nil), or right before a node
//     already woven whose cause is m (only when that node's id is smaller than
//     its cause's: a non-Lamport cause);
//   * from that split m skips the nodes A holds for; if weave-asap? never holds
//     (an absent cause, or one with a larger id that is not woven yet) the loop
//     runs to the (empty? right) branch (:236-237) and m is appended.
// So one sequential pass per document over a linked list gives the literal
// result: O(n + skips) plus, for each node that has an earlier-id child, a walk
// from the head (O(n) each).  That serial fold (k_xfold, one lane per document,
// ~1 us a node) is kept only for documents with such a non-Lamport cause, up to
// XFOLD_MAX nodes; larger ones get CW_STATUS_UNWOVEN.
//
// Every other flagged document (absent causes, nil causes, no root or several,
// a root that is not the smallest id) is woven data-parallel.  With every cause
// present and older, or nil, or absent:
//   * a nil cause puts the node at the split before the first node: it is a
//     child of a virtual head H (rank 0 of a synthetic list, the document's
//     rank r becomes r + 1);
//   * an absent cause appends the node at the end of the weave of the nodes
//     older than it.  Appending m is the same as weaving m under the node that
//     is last at that moment, T(m) (nothing follows it, so the skip of clause A
//     finds nothing either), and no later step of the fold reads m's cause
//     (clause A compares cause(nr) with the incoming id, never equal; asap
//     reads the incoming node's own cause).  The fold only inserts, so the
//     weave at time m is the final weave restricted to the older nodes:
//     T(m) = the older node with the largest final position (H if none);
//   * with every orphan attached under its T(m) the list is in the fast path's
//     domain (effective-tree preorder), and render bits are F6's
//     with one change: an attached orphan hide does not hide its new parent
//     (hide? compares the real cause), so it weaves as an h.show (still
//     special).  Roots (KIND_ROOT, nil cause) are weaved as normal nodes under H
//     and rendered hidden.
// T(m) depends on the final weave, so the attachments are found by iteration:
// start with T(m) = the previous rank, weave the synthetic lists (weave_tail,
// the fast path's tree and tour: no sort), recompute every T(m) as a prefix
// arg-max of positions over the id order, repeat until no attachment changes.
// The fixed point is the fold's result (by induction over the orphans in id
// order: with the older orphans attached right, the weave restricted to the
// nodes older than m is the fold's, so the recomputed T(m) is right), and
// iteration k has the k oldest orphans right, so it ends within (orphans + 1)
// weaves -- in practice 2 for a document with one orphan.  Tested against
// the literal fold on corrupted histories (tests/test_gpu_exact.py).

constexpr uint32_t X_NIL = 0xFFFFFFFEu;  // cause is nil (the root's, shared.cljc:22-23)
constexpr uint32_t X_END = 0xFFFFFFFFu;  // no cause in the document / end of the list
constexpr uint32_t X_HEAD = 0xFFFFFFFDu; // the split before the first node
constexpr uint32_t X_MASK = CW_STATUS_ROOT | CW_STATUS_ORPHAN | CW_STATUS_NON_LAMPORT;
// not a ::nodes map of the reference (a repeated id) or not a K64 key
constexpr uint32_t X_SKIP = CW_STATUS_DUP | CW_STATUS_KEY_RANGE;
constexpr uint32_t XFOLD_MAX = 1u << 22;     // the serial fold's largest document (nodes)
// Routing of the documents without a non-Lamport cause: the synthetic lists
// take at most (orphans + 1) iterations, so documents with few orphans, or
// too large for the serial fold, go there; others take the serial fold.
constexpr uint32_t XSYN_FEW = 32;            // orphans: always the synthetic lists
constexpr uint32_t XSYN_MAX_ORPH = 1024;     // orphans: a document above XFOLD_MAX with more
                                             // is left CW_STATUS_UNWOVEN
constexpr uint32_t X_NONE = 0xFFFFFFFFu;     // not on the synthetic path
constexpr unsigned long long X_HEADKEY = 0xFFFFFFFFull;  // (position 0 << 32) | H

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
// cause is not an id of the document), its kind by rank, and early[c] = 1 for
// every node c that has a child with a smaller id (weave-asap?'s second test).
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
    if (p == X_END) atomicAdd(&doc_orph[f], 1u);  // (orphans are few: rarely contended)
  }
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
  if (p == X_END) atomicAdd(doc_orph, 1u);
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

// --- the synthetic lists (documents without a non-Lamport cause) ------------
// Sub-batch index i = doc_off[f] + r (rank r of flagged document f); the
// synthetic list of f starts at sbase[f] (X_NONE: f takes the serial fold):
// sbase[f] = H, sbase[f] + 1 + r = rank r.

// Build: synthetic parent rank and kind of every rank (orphans attached under
// the previous rank to start), H at rank 0.
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
    if (p < n) {
      sp = p + 1;  // a present, older cause
    } else if (p == X_NIL) {
      sp = 0;      // a nil cause: under H
    } else {       // an absent cause: under the synthetic rank r (= rank r - 1, or H)
      sp = r;
      if (k == KIND_HIDE || k == KIND_HHIDE) k = 3;  // hides nothing: renders like an h.show
    }
    spar[sb + 1 + r] = sp;
    skd[sb + 1 + r] = k;
    if (r == 0) {
      spar[sb] = CW_NIL_RANK;
      skd[sb] = KIND_ROOT;
    }
  }
}

// Positions: pos[i] = weave position (>= 1) of rank i's synthetic rank.  A tile
// of the sub-batch stands for the same range of positions (q = 0 .. n-1 is
// synthetic position q + 1).
__global__ __launch_bounds__(256) void k_xsyn_pos(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ wperm, uint32_t *__restrict__ pos, uint32_t *__restrict__ bad) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t q = i - base, s = wperm[sb + 1 + q];
    if (s >= 1 && s <= n) pos[base + s - 1] = q + 1;
    else atomicOr(bad, 1u);  // H is always first: a position 1.. that holds it is an error
  }
}

// Largest (position << 32 | rank) of each tile.
__global__ __launch_bounds__(256) void k_xsyn_tmax(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ pos, unsigned long long *__restrict__ tmax) {
  __shared__ unsigned long long wm[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  if (sbase[f] == X_NONE) return;
  const uint32_t base = doc_off[f];
  unsigned long long m = 0;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x)
    m = max(m, ((unsigned long long)pos[i] << 32) | (i - base));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) tmax[t] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
}

// Per document (one block): tcar[t] = the largest key of the ranks before tile t
// (H's key before the first).
__global__ __launch_bounds__(256) void k_xsyn_tcarry(const uint32_t *__restrict__ tile_first,
                                                     const uint32_t *__restrict__ sbase,
                                                     const unsigned long long *__restrict__ tmax,
                                                     unsigned long long *__restrict__ tcar) {
  __shared__ unsigned long long wm[4];
  const uint32_t f = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (sbase[f] == X_NONE) return;
  const uint32_t t0 = tile_first[f], t1 = tile_first[f + 1];
  unsigned long long carry = X_HEADKEY;
  for (uint32_t c0 = t0; c0 < t1; c0 += 256) {
    const uint32_t t = c0 + threadIdx.x;
    const unsigned long long v = t < t1 ? tmax[t] : 0ull;
    unsigned long long inc = v;  // inclusive max scan inside the wave
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc = max(inc, y);
    }
    if (lane == 63) wm[wv] = inc;
    __syncthreads();
    unsigned long long pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre = max(pre, wm[w]);
    const unsigned long long up = __shfl_up(inc, 1, 64);
    const unsigned long long exc = max(pre, lane ? up : 0ull);
    if (t < t1) tcar[t] = exc;
    const unsigned long long total = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
    __syncthreads();
    carry = max(carry, total);
  }
}

// At every orphan rank r: T = the rank with the largest position among ranks
// < r (H if none); its synthetic parent becomes T's synthetic rank.  Each
// thread runs over a contiguous piece of the tile with the exclusive prefix of
// the pieces before it.  Counts the attachments that change.
__global__ __launch_bounds__(256) void k_xsyn_apply(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ xpar, const uint32_t *__restrict__ pos,
    const unsigned long long *__restrict__ tcar, uint32_t *__restrict__ spar,
    uint32_t *__restrict__ changed, uint8_t *__restrict__ doc_changed) {
  __shared__ unsigned long long wm[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  const uint32_t s = tile_start[t], e = tile_start[t + 1], len = e - s;
  const uint32_t per = (len + 255) / 256;
  const uint32_t j0 = min(e, s + threadIdx.x * per), j1 = min(e, j0 + per);
  unsigned long long m = 0;
  for (uint32_t i = j0; i < j1; i++) m = max(m, ((unsigned long long)pos[i] << 32) | (i - base));
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long inc = m;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc = max(inc, y);
  }
  if (lane == 63) wm[wv] = inc;
  __syncthreads();
  unsigned long long run = tcar[t];
  for (uint32_t w = 0; w < wv; w++) run = max(run, wm[w]);
  const unsigned long long up = __shfl_up(inc, 1, 64);
  run = max(run, lane ? up : 0ull);
  uint32_t ch = 0;
  for (uint32_t i = j0; i < j1; i++) {
    const uint32_t p = xpar[i];
    if (!(p < n) && p != X_NIL) {  // an orphan: under the last node older than it
      const uint32_t T = (uint32_t)run;
      const uint32_t want = T == 0xFFFFFFFFu ? 0u : T + 1;
      uint32_t *slot = &spar[sb + 1 + (i - base)];
      if (*slot != want) {
        *slot = want;
        ch++;
      }
    }
    run = max(run, ((unsigned long long)pos[i] << 32) | (i - base));
  }
  if (ch) {
    atomicAdd(changed, ch);
    doc_changed[f] = 1;
  }
}

// The woven synthetic lists -> the caller's outputs: weave_perm (input index per
// position, H dropped), rendered bits (the synthetic render bit, roots hidden)
// and rendered counts.  The tile of the sub-batch stands for the same range of
// output positions q; one thread per output word.
__global__ __launch_bounds__(256) void k_xsyn_emit(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ wperm, const uint32_t *__restrict__ wbits,
    const uint8_t *__restrict__ xk, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ out_off, const uint32_t *__restrict__ out_doc,
    uint32_t *__restrict__ weave_perm, uint32_t *__restrict__ visible_bits,
    uint32_t *__restrict__ visible_count) {
  __shared__ uint32_t wsum[4];
  const uint32_t t = blockIdx.x, f = tile_doc[t], sb = sbase[f];
  if (sb == X_NONE) return;
  const uint32_t base = doc_off[f];
  const uint32_t q0 = tile_start[t] - base, q1 = tile_start[t + 1] - base;
  const uint64_t g0 = out_off[f];
  // output words touching [g0 + q0, g0 + q1)
  const uint64_t W0 = (g0 + q0) >> 5, W1 = (g0 + q1 - 1) >> 5;
  uint32_t cnt = 0;
  for (uint64_t W = W0 + threadIdx.x; W <= W1; W += blockDim.x) {
    const uint64_t lo = max(W << 5, g0 + q0), hi = min((W << 5) + 32, g0 + q1);
    uint32_t acc = 0, mask = 0;
    for (uint64_t g = lo; g < hi; g++) {
      const uint32_t q = (uint32_t)(g - g0), x = sb + 1 + q;  // synthetic position
      const uint32_t i = base + wperm[x] - 1;
      weave_perm[g] = sval ? sval[i] : i - base;
      const bool vis = ((wbits[x >> 5] >> (x & 31)) & 1u) && !(xk[i] & KIND_ROOT);
      mask |= 1u << (g & 31);
      if (vis) acc |= 1u << (g & 31);
      cnt += vis ? 1u : 0u;
    }
    if (visible_bits) x_flush(visible_bits, W, mask, acc);
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

__global__ __launch_bounds__(64) void k_xunwoven(const uint8_t *__restrict__ mark, uint32_t F,
                                                 const uint32_t *__restrict__ out_doc,
                                                 uint32_t *__restrict__ status) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F && mark[f]) status[out_doc[f]] |= CW_STATUS_UNWOVEN;
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

// The flagged documents after the join (xpar: cause rank / X_NIL / X_END by
// rank, xk: kinds by rank, early: "has an older child" by rank, sval: input
// index by rank or nullptr; dearly / dorph: per document "has a non-Lamport
// cause" and its number of orphans): each document to the synthetic lists,
// the serial fold or CW_STATUS_UNWOVEN, and its outputs written at out_off.
int exact_weave_flagged(cw_ctx *c, uint32_t F, const std::vector<uint64_t> &xoff,
                        const uint32_t *xpar, const uint8_t *xk, const uint8_t *early,
                        const uint32_t *sval, const uint64_t *d_oof, const uint32_t *d_odoc,
                        const uint8_t *dearly, const uint32_t *dorph, cw_list_result *out) {
  const uint32_t NX = (uint32_t)xoff.back();
  if (ensure_tables(c, F, xoff.data())) return -1;
  uint32_t *tile_start = dev_tab(c, "t_tile_start"), *tile_doc = dev_tab(c, "t_tile_doc"),
           *sub_off = dev_tab(c, "t_doc_off");
  const dim3 B256(256), GF((F + 63) / 64), B64(64);
  const uint32_t T = c->tab.T;
  if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
  // which documents take the serial fold (a non-Lamport cause), which the
  // synthetic lists
  std::vector<uint8_t> h_early(F), run(F, 0), unwoven(F, 0);
  std::vector<uint32_t> h_orph(F);
  HIPCHK(c, hipMemcpyAsync(h_early.data(), dearly, F, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h_orph.data(), dorph, (size_t)F * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint32_t orph_max = 0;
  struct Group {
    bool giant;
    uint64_t base;  // first synthetic index (a multiple of 32: its bits start a word)
    std::vector<uint64_t> off;
  };
  std::vector<Group> groups;
  std::vector<uint32_t> sb(F, X_NONE);
  uint64_t NS = 0;
  bool any_serial = false;
  {
    Group batch{false, 0, {0}};
    std::vector<uint32_t> big;
    for (uint32_t f = 0; f < F; f++) {
      const uint64_t n = xoff[f + 1] - xoff[f];
      const bool small = n <= XFOLD_MAX;
      if (h_early[f] || (small && h_orph[f] > XSYN_FEW) || (!small && h_orph[f] > XSYN_MAX_ORPH)) {
        (small ? run : unwoven)[f] = 1;
        any_serial |= small;
        continue;
      }
      orph_max = std::max(orph_max, h_orph[f]);
      if (n + 1 >= c->giant_min || n + 1 >= LINK_IDX) {
        big.push_back(f);
      } else {
        sb[f] = (uint32_t)batch.off.back();
        batch.off.push_back(batch.off.back() + n + 1);
      }
    }
    if (batch.off.size() > 1) {
      NS = (batch.off.back() + 31) & ~31ull;
      groups.push_back(std::move(batch));
    }
    for (uint32_t f : big) {
      const uint64_t n = xoff[f + 1] - xoff[f];
      sb[f] = (uint32_t)NS;
      groups.push_back(Group{true, NS, {0, n + 1}});
      NS = (NS + n + 1 + 31) & ~31ull;
    }
  }
  if (NS >= 0xFFFFFFFFull) return fail(c, "exact path: %llu synthetic nodes", (unsigned long long)NS);
  if (!groups.empty()) {
    uint32_t *d_sb = x_upload(c, "x_sbase", sb);
    uint32_t *spar = scratch_t<uint32_t>(c, "x_spar", NS), *wperm = scratch_t<uint32_t>(c, "x_wperm", NS);
    uint8_t *skd = scratch_t<uint8_t>(c, "x_skd", NS), *dch = scratch_t<uint8_t>(c, "x_dch", F);
    uint32_t *wbits = scratch_t<uint32_t>(c, "x_wbits", NS / 32 + 1);
    uint32_t *pos = scratch_t<uint32_t>(c, "x_pos", NX), *ctl = scratch_t<uint32_t>(c, "x_ctl", 2);
    unsigned long long *tmax = scratch_t<unsigned long long>(c, "x_tmax", T);
    unsigned long long *tcar = scratch_t<unsigned long long>(c, "x_tcar", T);
    size_t gmax = 1;
    for (auto &g : groups) gmax = std::max(gmax, g.off.size() - 1);
    uint32_t *wvc = scratch_t<uint32_t>(c, "x_wvc", gmax), *wst = scratch_t<uint32_t>(c, "x_wst", gmax);
    if (!d_sb || !spar || !wperm || !skd || !dch || !wbits || !pos || !ctl || !tmax || !tcar || !wvc ||
        !wst)
      return fail(c, "out of device memory (exact path, %llu synthetic nodes)", (unsigned long long)NS);
    hipLaunchKernelGGL(k_xsyn_build, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                       xpar, xk, spar, skd);
    if (check_launch(c, "xsyn_build")) return -1;
    HIPCHK(c, hipMemsetAsync(dch, 0, F, c->stream));
    uint32_t it = 0;
    for (;; it++) {
      // weave every synthetic list (the fast path's tree and tour, no sort)
      for (auto &g : groups) {
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
      }
      if (ensure_tables(c, F, xoff.data())) return -1;  // the flagged documents' tiles again
      tile_start = dev_tab(c, "t_tile_start");
      tile_doc = dev_tab(c, "t_tile_doc");
      sub_off = dev_tab(c, "t_doc_off");
      // every orphan under the last older node of that weave
      HIPCHK(c, hipMemsetAsync(ctl, 0, 8, c->stream));
      {
        Launch L(c, "xsyn_attach", (double)NX * 4 * 4);
        hipLaunchKernelGGL(k_xsyn_pos, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                           wperm, pos, ctl + 1);
        hipLaunchKernelGGL(k_xsyn_tmax, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                           pos, tmax);
        hipLaunchKernelGGL(k_xsyn_tcarry, dim3(F), B256, 0, c->stream, dev_tab(c, "t_tile_first"), d_sb,
                           tmax, tcar);
        hipLaunchKernelGGL(k_xsyn_apply, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off,
                           d_sb, xpar, pos, tcar, spar, ctl, dch);
      }
      if (check_launch(c, "xsyn_attach")) return -1;
      HIPCHK(c, hipMemcpyAsync(c->pin_small, ctl, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (c->pin_small[1]) return fail(c, "exact path: inconsistent synthetic weave");
      if (c->pin_small[0] == 0) break;
      if (it > orph_max) {  // iteration k places the k-th orphan for good: never taken
        // (not seen: one orphan is placed right per iteration) the documents
        // still moving take the serial fold, or are left unwoven
        std::vector<uint8_t> h_dch(F);
        HIPCHK(c, hipMemcpy(h_dch.data(), dch, F, hipMemcpyDeviceToHost));
        for (uint32_t f = 0; f < F; f++) {
          if (!h_dch[f] || sb[f] == X_NONE) continue;
          sb[f] = X_NONE;
          const uint64_t n = xoff[f + 1] - xoff[f];
          (n <= XFOLD_MAX ? run : unwoven)[f] = 1;
          any_serial |= n <= XFOLD_MAX;
        }
        d_sb = x_upload(c, "x_sbase", sb);
        if (!d_sb) return fail(c, "out of device memory (exact path)");
        break;
      }
      HIPCHK(c, hipMemsetAsync(dch, 0, F, c->stream));
    }
    c->x_iters = it + 1;
    hipLaunchKernelGGL(k_xsyn_zero, GF, B64, 0, c->stream, d_sb, F, d_odoc, out->visible_count);
    {
      Launch L(c, "xsyn_emit", (double)NX * (4 + 4 + 4 + 1) + (double)NX / 8);
      hipLaunchKernelGGL(k_xsyn_emit, dim3(T), B256, 0, c->stream, tile_start, tile_doc, sub_off, d_sb,
                         wperm, wbits, xk, sval, d_oof, d_odoc, out->weave_perm, out->visible_bits,
                         out->visible_count);
    }
    if (check_launch(c, "xsyn_emit")) return -1;
  }
  if (any_serial) {  // documents with a non-Lamport cause: the literal fold, one lane each
    uint8_t *d_run = x_upload(c, "x_run", run);
    uint32_t *xnext = scratch_t<uint32_t>(c, "x_next", NX);
    if (!d_run || !xnext) return fail(c, "out of device memory (exact path)");
    Launch L(c, "xfold", (double)NX * 22);
    hipLaunchKernelGGL(k_xfold, GF, B64, 0, c->stream, sub_off, F, xpar, xk, early, xnext, sval,
                       d_oof, d_odoc, out->weave_perm, out->visible_bits, out->visible_count, d_run);
  }
  if (check_launch(c, "xfold")) return -1;
  if (std::find(unwoven.begin(), unwoven.end(), 1) != unwoven.end()) {
    uint8_t *d_un = x_upload(c, "x_unwoven", unwoven);
    if (!d_un) return fail(c, "out of device memory (exact path)");
    hipLaunchKernelGGL(k_xunwoven, GF, B64, 0, c->stream, d_un, F, d_odoc, out->status);
    if (check_launch(c, "xunwoven")) return -1;
  }
    return 0;
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
// (the same routing as exact_fixup: synthetic lists, serial fold or UNWOVEN).
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
