// k128.hip -- cw_weave_lists_k128: ids that need more than 64 bits.  Included
// by causeweave.hip after weave_lists_dev_all.
//
// A K128 id is two words: hi = lamport-ts (a nat-int, up to 2^63 - 1 as a
// Clojure Long, shared.cljc:31), lo = site rank << 32 | tx-index.  The packed
// order is (compare a b) (util.cljc:4-10).  The weave itself only needs each
// id's place in that order, so the call
//   1. sorts every document's 128-bit ids (two stable segmented radix sorts:
//      lo, then hi) -- (sort ::nodes), list.cljc:28;
//   2. replaces each id by its rank in the document and each cause by the rank
//      of the equal id (nil stays nil; a cause that is no id of the document
//      becomes a value no id has) -- order-preserving, so the 64-bit pipeline
//      (fast path + exact path) weaves exactly the same list;
//   3. takes ::lamport-ts from the largest id's hi word (refresh-ts,
//      shared.cljc:243-249) and the yarns from a sort by (site, rank) (spin,
//      shared.cljc:121-132).

__global__ __launch_bounds__(256) void k_k128_split(const uint64_t *__restrict__ key2, uint32_t n,
                                                    uint64_t *__restrict__ hi,
                                                    uint64_t *__restrict__ lo) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ulonglong2 k = reinterpret_cast<const ulonglong2 *>(key2)[i];
  hi[i] = k.x;
  lo[i] = k.y;
}

// h1[i] = hi[doc start + v[i]] (sort values are doc-local input indices).
__global__ __launch_bounds__(256) void k_k128_gather(const uint32_t *__restrict__ tile_start,
                                                     const uint32_t *__restrict__ tile_doc,
                                                     const uint32_t *__restrict__ doc_off,
                                                     const uint64_t *__restrict__ hi,
                                                     const uint32_t *__restrict__ v,
                                                     uint64_t *__restrict__ h1) {
  const uint32_t t = blockIdx.x, base = doc_off[tile_doc[t]];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x)
    h1[i] = hi[base + v[i]];
}

// Sorted position i of its document: the id's rank (equal ids share the rank of
// the first: the pipeline then sees the repeat and flags CW_STATUS_DUP) and the
// sorted lo words for the cause search.
__global__ __launch_bounds__(256) void k_k128_rank(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint64_t *__restrict__ shi,
    const uint32_t *__restrict__ sidx, const uint64_t *__restrict__ lo,
    uint64_t *__restrict__ slo, uint64_t *__restrict__ rid) {
  const uint32_t t = blockIdx.x, f = tile_doc[t], base = doc_off[f];
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const uint32_t v = sidx[i];
    const uint64_t h = shi[i], l = lo[base + v];
    slo[i] = l;
    uint32_t r = i - base;
    if (r > 0 && shi[i - 1] == h && lo[base + sidx[i - 1]] == l) {  // a repeat: the run's first
      while (r > 0 && shi[base + r - 1] == h && lo[base + sidx[base + r - 1]] == l) r--;
    }
    rid[base + v] = r;
  }
}

// Each node's cause as a rank (binary search over the document's sorted
// 128-bit ids); nil stays CW_NIL, an absent cause becomes CW_NIL - 1.
__global__ __launch_bounds__(256) void k_k128_cause(
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ doc_off, const uint64_t *__restrict__ shi,
    const uint64_t *__restrict__ slo, const uint64_t *__restrict__ cause2,
    uint64_t *__restrict__ rcause) {
  const uint32_t t = blockIdx.x, f = tile_doc[t];
  const uint32_t base = doc_off[f], n = doc_off[f + 1] - base;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x) {
    const ulonglong2 c = reinterpret_cast<const ulonglong2 *>(cause2)[i];
    uint64_t out = CW_NIL;
    if (!(c.x == CW_NIL && c.y == CW_NIL)) {
      uint32_t a = 0, b = n;  // first sorted id >= (c.x, c.y)
      while (a < b) {
        const uint32_t m = (a + b) >> 1;
        const uint64_t h = shi[base + m], l = slo[base + m];
        if (h < c.x || (h == c.x && l < c.y)) a = m + 1; else b = m;
      }
      out = (a < n && shi[base + a] == c.x && slo[base + a] == c.y) ? (uint64_t)a : CW_NIL - 1;
    }
    rcause[i] = out;
  }
}

__global__ __launch_bounds__(256) void k_k128_yarnkey(const uint64_t *__restrict__ lo,
                                                      const uint64_t *__restrict__ rid, uint32_t n,
                                                      uint32_t rbits, uint64_t *__restrict__ yk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) yk[i] = ((lo[i] >> 32) << rbits) | rid[i];
}

__global__ __launch_bounds__(256) void k_k128_maxts(const uint32_t *__restrict__ doc_off, uint32_t D,
                                                    const uint64_t *__restrict__ shi,
                                                    uint64_t *__restrict__ max_ts) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const uint32_t a = doc_off[d], b = doc_off[d + 1];
  max_ts[d] = b > a ? shi[b - 1] : 0;
}

namespace {

int weave_lists_k128_impl(cw_ctx *c, const cw_list_batch_k128 *bt, cw_list_result *res,
                          int memspace) {
  if (!bt || !res) return fail(c, "null batch/result");
  const uint64_t D = bt->n_docs;
  const uint64_t *off = bt->doc_offsets;
  if (!off || off[0] != 0) return fail(c, "doc_offsets must start at 0");
  const uint64_t N64 = off[D];
  if (N64 >= 0xFFFFFFFFull) return fail(c, "batch too large: N=%llu", (unsigned long long)N64);
  uint64_t nmax = 0;
  for (uint64_t d = 0; d < D; d++) {
    if (off[d + 1] < off[d]) return fail(c, "doc_offsets not monotone");
    nmax = std::max(nmax, off[d + 1] - off[d]);
    if (D == 1 ? off[1] >= SUCCW_END : off[d + 1] - off[d] >= LINK_IDX)
      return fail(c, "document %llu too large", (unsigned long long)d);
  }
  if (!res->weave_perm || !res->visible_count || !res->status)
    return fail(c, "weave_perm, visible_count and status are required");
  if (memspace != CW_MEM_HOST && memspace != CW_MEM_DEVICE) return fail(c, "bad memspace");
  const uint32_t N = (uint32_t)N64;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t Ns = std::max<uint32_t>(N, 1);
  // device copies of the inputs (host memory) and of the outputs
  const uint64_t *id2 = bt->id_key, *ca2 = bt->cause_key;
  const uint8_t *kind = bt->kind;
  cw_list_result dres = *res;
  if (memspace == CW_MEM_HOST) {
    if (N && (!id2 || !ca2 || !kind)) return fail(c, "null input arrays");
    uint64_t *did = scratch_t<uint64_t>(c, "h_id", 2 * Ns), *dca = scratch_t<uint64_t>(c, "h_cause", 2 * Ns);
    uint8_t *dk = scratch_t<uint8_t>(c, "h_kind", Ns);
    dres.weave_perm = scratch_t<uint32_t>(c, "h_perm", Ns);
    dres.visible_bits = res->visible_bits ? scratch_t<uint32_t>(c, "h_bits", (Ns + 31) / 32) : nullptr;
    dres.visible_count = scratch_t<uint32_t>(c, "h_vcount", D + 1);
    dres.max_ts = res->max_ts ? scratch_t<uint64_t>(c, "h_maxts", D + 1) : nullptr;
    dres.status = scratch_t<uint32_t>(c, "h_status", D + 1);
    dres.yarn_perm = res->yarn_perm ? scratch_t<uint32_t>(c, "h_yarn", Ns) : nullptr;
    if (!did || !dca || !dk || !dres.weave_perm || !dres.visible_count || !dres.status ||
        (res->visible_bits && !dres.visible_bits) || (res->max_ts && !dres.max_ts) ||
        (res->yarn_perm && !dres.yarn_perm))
      return fail(c, "out of device memory (host-mode staging)");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (N) {
      HIPCHK(c, hipMemcpy(did, id2, (size_t)N * 16, hipMemcpyHostToDevice));
      HIPCHK(c, hipMemcpy(dca, ca2, (size_t)N * 16, hipMemcpyHostToDevice));
      HIPCHK(c, hipMemcpy(dk, kind, N, hipMemcpyHostToDevice));
    }
    id2 = did;
    ca2 = dca;
    kind = dk;
  }
  uint64_t *rid = scratch_t<uint64_t>(c, "k128_rid", Ns), *rca = scratch_t<uint64_t>(c, "k128_rca", Ns);
  if (!rid || !rca) return fail(c, "out of device memory (k128)");
  if (N) {
    if (ensure_tables(c, D, off)) return -1;
    auto &t = c->tab;
    uint64_t *hi = scratch_t<uint64_t>(c, "k128_hi", Ns), *lo = scratch_t<uint64_t>(c, "k128_lo", Ns);
    uint64_t *h1 = scratch_t<uint64_t>(c, "k128_h1", Ns), *slo = scratch_t<uint64_t>(c, "k128_slo", Ns);
    uint64_t *skA = scratch_t<uint64_t>(c, "skA", Ns), *skB = scratch_t<uint64_t>(c, "skB", Ns);
    uint32_t *svA = scratch_t<uint32_t>(c, "svA", Ns), *svB = scratch_t<uint32_t>(c, "svB", Ns);
    uint32_t *wvA = scratch_t<uint32_t>(c, "k128_vA", Ns), *wvB = scratch_t<uint32_t>(c, "k128_vB", Ns);
    if (!hi || !lo || !h1 || !slo || !skA || !skB || !svA || !svB || !wvA || !wvB)
      return fail(c, "out of device memory (k128 sort)");
    const dim3 GN((N + 255) / 256), B256(256), GT(t.T);
    hipLaunchKernelGGL(k_k128_split, GN, B256, 0, c->stream, id2, N, hi, lo);
    if (check_launch(c, "k128_split")) return -1;
    uint32_t lo_bits, hi_bits;
    if (find_key_bits(c, lo, N, &lo_bits) || find_key_bits(c, hi, N, &hi_bits)) return -1;
    // (sort ::nodes) on 128 bits: by lo, then stably by hi
    uint64_t *k1, *k2;
    uint32_t *v1, *v2;
    if (radix_sort<uint64_t>(c, "k128_sort_lo", lo, nullptr, skA, svA, skB, svB, lo_bits, 0, N, &k1, &v1))
      return -1;
    hipLaunchKernelGGL(k_k128_gather, GT, B256, 0, c->stream, dev_tab(c, "t_tile_start"),
                       dev_tab(c, "t_tile_doc"), dev_tab(c, "t_doc_off"), hi, v1, h1);
    if (check_launch(c, "k128_gather")) return -1;
    if (radix_sort<uint64_t>(c, "k128_sort_hi", h1, v1, skA == k1 ? skB : skA, wvA, k1, wvB, hi_bits,
                             0, N, &k2, &v2))
      return -1;
    // k2 = sorted hi words, v2 = doc-local input index of each sorted id
    {
      Launch L(c, "k128_rank", (double)N * 28);
      hipLaunchKernelGGL(k_k128_rank, GT, B256, 0, c->stream, dev_tab(c, "t_tile_start"),
                         dev_tab(c, "t_tile_doc"), dev_tab(c, "t_doc_off"), k2, v2, lo, slo, rid);
    }
    if (check_launch(c, "k128_rank")) return -1;
    {
      Launch L(c, "k128_cause", (double)N * 24);
      hipLaunchKernelGGL(k_k128_cause, GT, B256, 0, c->stream, dev_tab(c, "t_tile_start"),
                         dev_tab(c, "t_tile_doc"), dev_tab(c, "t_doc_off"), k2, slo, ca2, rca);
    }
    if (check_launch(c, "k128_cause")) return -1;
    // ::lamport-ts = hi word of every document's largest id; sorted hi words
    // are about to be overwritten by the weave's own sorts
    if (dres.max_ts) {
      hipLaunchKernelGGL(k_k128_maxts, dim3((uint32_t)((D + 255) / 256)), B256, 0, c->stream,
                         dev_tab(c, "t_doc_off"), (uint32_t)D, k2, dres.max_ts);
      if (check_launch(c, "k128_maxts")) return -1;
    }
  }
  // the weave on ranks (fast path + exact path), yarns from the real sites
  cw_list_batch rb{};
  rb.n_docs = D;
  rb.doc_offsets = off;
  rb.id_key = rid;
  rb.cause_key = rca;
  rb.kind = kind;
  rb.key_bits = std::max<uint32_t>(1, ceil_log2(nmax + 1));
  rb.ts_shift = 0;
  rb.site_shift = 0;
  rb.site_bits = 0;
  cw_list_result rr = dres;
  rr.max_ts = nullptr;
  rr.yarn_perm = nullptr;
  if (N) {
    HIPCHK(c, hipMemsetAsync(dres.status, 0, D * 4, c->stream));
    if (weave_lists_dev_all(c, &rb, rid, rca, kind, &rr)) return -1;
  } else if (D) {
    HIPCHK(c, hipMemsetAsync(dres.status, 0, D * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(dres.visible_count, 0, D * 4, c->stream));
    if (dres.max_ts) HIPCHK(c, hipMemsetAsync(dres.max_ts, 0, D * 8, c->stream));
  }
  if (N && dres.yarn_perm) {
    if (ensure_tables(c, D, off)) return -1;
    uint64_t *lo = scratch_t<uint64_t>(c, "k128_lo", Ns), *yk = scratch_t<uint64_t>(c, "k128_h1", Ns);
    uint64_t *skA = scratch_t<uint64_t>(c, "skA", Ns), *skB = scratch_t<uint64_t>(c, "skB", Ns);
    uint32_t *wvA = scratch_t<uint32_t>(c, "k128_vA", Ns), *wvB = scratch_t<uint32_t>(c, "k128_vB", Ns);
    const uint32_t rbits = rb.key_bits;
    uint32_t site_bits;
    if (find_key_bits(c, lo, N, &site_bits)) return -1;  // (bits of lo; the site is above 32)
    site_bits = site_bits > 32 ? site_bits - 32 : 1;
    hipLaunchKernelGGL(k_k128_yarnkey, dim3((N + 255) / 256), dim3(256), 0, c->stream, lo, rid, N,
                       rbits, yk);
    if (check_launch(c, "k128_yarnkey")) return -1;
    uint64_t *ko;
    uint32_t *vo;
    if (radix_sort<uint64_t>(c, "k128_yarns", yk, nullptr, skA, wvA, skB, wvB, rbits + site_bits, 0, N,
                             &ko, &vo))
      return -1;
    HIPCHK(c, hipMemcpyAsync(dres.yarn_perm, vo, (size_t)N * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  if (memspace == CW_MEM_HOST) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (N) {
      HIPCHK(c, hipMemcpy(res->weave_perm, dres.weave_perm, (size_t)N * 4, hipMemcpyDeviceToHost));
      if (res->visible_bits)
        HIPCHK(c, hipMemcpy(res->visible_bits, dres.visible_bits, ((size_t)N + 31) / 32 * 4,
                            hipMemcpyDeviceToHost));
      if (res->yarn_perm)
        HIPCHK(c, hipMemcpy(res->yarn_perm, dres.yarn_perm, (size_t)N * 4, hipMemcpyDeviceToHost));
    }
    HIPCHK(c, hipMemcpy(res->visible_count, dres.visible_count, D * 4, hipMemcpyDeviceToHost));
    if (res->max_ts) HIPCHK(c, hipMemcpy(res->max_ts, dres.max_ts, D * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->status, dres.status, D * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipDeviceSynchronize());
    for (uint64_t d = 0; d < D; d++)
      if (off[d + 1] == off[d]) res->status[d] |= CW_STATUS_ROOT;
  } else {
    for (uint64_t d = 0; d < D; d++)
      if (off[d + 1] == off[d])
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)(res->status + d), CW_STATUS_ROOT, 1, c->stream));
    if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (c->prof) return collect_prof(c);
  return 0;
}

}  // namespace
