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
// result: O(n + skips) plus a walk from the head for each node that has an
// earlier-id child.  Documents are independent: one lane per document.

constexpr uint32_t X_NIL = 0xFFFFFFFEu;  // cause is nil (the root's, shared.cljc:22-23)
constexpr uint32_t X_END = 0xFFFFFFFFu;  // no cause in the document / end of the list
constexpr uint32_t X_HEAD = 0xFFFFFFFDu; // the split before the first node
constexpr uint32_t X_MASK = CW_STATUS_ROOT | CW_STATUS_ORPHAN | CW_STATUS_NON_LAMPORT;
// not a ::nodes map of the reference (a repeated id) or not a K64 key
constexpr uint32_t X_SKIP = CW_STATUS_DUP | CW_STATUS_KEY_RANGE;

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
    uint8_t *__restrict__ early) {
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
    if (p < n && p > r) early[base + p] = 1;
  }
}

// A list handed over in rank order (cw_weave_ranked): the root's cause is nil,
// CW_NOT_FOUND stays "absent"; early children as in k_xjoin.
__global__ __launch_bounds__(256) void k_xranked_prep(const uint32_t *__restrict__ par,
                                                      const uint8_t *__restrict__ kind, uint32_t n,
                                                      uint32_t *__restrict__ xpar,
                                                      uint8_t *__restrict__ early) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t p = par[r];
  if (r == 0 && (kind[0] & KIND_ROOT)) p = X_NIL;
  if (p == CW_NOT_FOUND) p = X_END;
  xpar[r] = p;
  if (p < n && p > r) early[p] = 1;
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
    uint32_t *__restrict__ visible_count) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
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
  if (D == 1 && c->x_cached && bt->key_bits && bt->key_bits < 64) {
    // one giant list: its status came back with the walk's counter (KEY_RANGE,
    // set later, needs key_bits >= 64)
    const uint32_t st = c->x_status;
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
  auto &t = c->tab;
  uint64_t *d_src = x_upload(c, "x_src", src);
  uint32_t *d_odoc = x_upload(c, "x_odoc", odoc);
  uint64_t *xid = scratch_t<uint64_t>(c, "link", NX), *xca = scratch_t<uint64_t>(c, "x_cause", NX);
  uint8_t *xkd = scratch_t<uint8_t>(c, "x_kind", NX), *xk = scratch_t<uint8_t>(c, "skind", NX);
  uint8_t *early = scratch_t<uint8_t>(c, "x_early", NX);
  uint64_t *skA = scratch_t<uint64_t>(c, "skA", NX), *skB = scratch_t<uint64_t>(c, "skB", NX);
  uint32_t *svA = scratch_t<uint32_t>(c, "svA", NX), *svB = scratch_t<uint32_t>(c, "svB", NX);
  uint32_t *xpar = scratch_t<uint32_t>(c, "par", NX), *xnext = scratch_t<uint32_t>(c, "nsc", NX);
  if (!d_src || !d_odoc || !xid || !xca || !xkd || !xk || !early || !skA || !skB || !svA || !svB ||
      !xpar || !xnext)
    return fail(c, "out of device memory (exact path, %u nodes)", NX);
  uint32_t *tile_start = dev_tab(c, "t_tile_start"), *tile_doc = dev_tab(c, "t_tile_doc"),
           *sub_off = dev_tab(c, "t_doc_off");
  const dim3 GT(t.T), B256(256), GF((F + 63) / 64), B64(64);
  {
    Launch L(c, "xgather", (double)NX * 34);
    hipLaunchKernelGGL(k_xgather, GT, B256, 0, c->stream, tile_start, tile_doc, sub_off, d_src, id,
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
  {
    Launch L(c, "xjoin", (double)NX * 30);
    hipLaunchKernelGGL(k_xjoin, GT, B256, 0, c->stream, tile_start, tile_doc, sub_off, skey, sval,
                       xca, xkd, xpar, xk, early);
  }
  if (check_launch(c, "xjoin")) return -1;
  uint64_t *d_oof;
  {
    std::vector<uint64_t> oof(F);
    for (uint32_t f = 0; f < F; f++) oof[f] = src[f];
    d_oof = x_upload(c, "x_oof", oof);
    if (!d_oof) return fail(c, "out of device memory (exact path)");
  }
  {
    Launch L(c, "xfold", (double)NX * 22);
    hipLaunchKernelGGL(k_xfold, GF, B64, 0, c->stream, sub_off, F, xpar, xk, early, xnext, sval,
                       d_oof, d_odoc, out->weave_perm, out->visible_bits, out->visible_count);
  }
  if (check_launch(c, "xfold")) return -1;
  if (out->max_ts) {
    hipLaunchKernelGGL(k_xmaxts, GF, B64, 0, c->stream, sub_off, F, skey, bt->ts_shift, d_odoc,
                       out->max_ts);
    if (check_launch(c, "xmaxts")) return -1;
  }
  if (out->yarn_perm && bt->site_bits) {  // spin 1-arity: the id order partitioned by site
    uint64_t *ykA = skey == skA ? skB : skA;
    uint32_t *yvA = sval == svA ? svB : svA;
    uint32_t *yvB = scratch_t<uint32_t>(c, "x_yv", NX);
    if (!yvB) return fail(c, "out of device memory (exact path yarns)");
    uint64_t *yk;
    uint32_t *yv;
    if (radix_sort<uint64_t>(c, "xyarns", skey, sval, ykA, yvA, xid, yvB, bt->site_bits,
                             bt->site_shift, NX, &yk, &yv))
      return -1;
    hipLaunchKernelGGL(k_xscatter, GT, B256, 0, c->stream, tile_start, tile_doc, sub_off, d_oof, yv,
                       out->yarn_perm);
    if (check_launch(c, "xscatter")) return -1;
  }
  return 0;
}

// cw_weave_ranked's exact path: the one list given by (par, kind) in rank order.
int exact_ranked(cw_ctx *c, const cw_ranked_list *l, cw_list_result *out) {
  const uint32_t n = (uint32_t)l->n;
  uint32_t *xpar = scratch_t<uint32_t>(c, "par", n), *xnext = scratch_t<uint32_t>(c, "nsc", n);
  uint8_t *early = scratch_t<uint8_t>(c, "x_early", n);
  uint32_t *doff = scratch_t<uint32_t>(c, "x_rdoff", 2), *odoc = scratch_t<uint32_t>(c, "x_rodoc", 1);
  uint64_t *oof = scratch_t<uint64_t>(c, "x_roof", 1);
  if (!xpar || !xnext || !early || !doff || !odoc || !oof)
    return fail(c, "out of device memory (exact path, %u nodes)", n);
  const uint32_t hd[2] = {0, n};
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(doff, hd, 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemset(odoc, 0, 4));
  HIPCHK(c, hipMemset(oof, 0, 8));
  HIPCHK(c, hipMemsetAsync(early, 0, n, c->stream));
  hipLaunchKernelGGL(k_xranked_prep, dim3((n + 255) / 256), dim3(256), 0, c->stream, l->par, l->kind,
                     n, xpar, early);
  if (check_launch(c, "xranked_prep")) return -1;
  {
    Launch L(c, "xfold", (double)n * 22);
    hipLaunchKernelGGL(k_xfold, dim3(1), dim3(64), 0, c->stream, doff, 1u, xpar, l->kind, early,
                       xnext, l->val, oof, odoc, out->weave_perm, out->visible_bits,
                       out->visible_count);
  }
  return check_launch(c, "xfold");
}

}  // namespace
