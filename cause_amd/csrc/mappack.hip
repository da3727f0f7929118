// mappack.hip -- the map weave of small collections in ONE kernel (config 4).
// Included by causeweave.hip after the sort helpers (rank_subdigit, wb_elem,
// block_exscan) it uses.
//
// c.map/weave 1-arity (map.cljc:21-45) + active-node (:47-59) for a batch of
// CausalMaps whose collections have <= MPK nodes each.  One workgroup takes a
// pack of whole consecutive collections (<= MPK nodes) and does, in LDS:
//   1. (sort ::nodes) per collection: a stable LDS radix sort by (collection, id);
//      repeated ids -> CW_STATUS_DUP;
//   2. each node's key and cause-in-weave (map.cljc:31-37): a cause id is
//      looked up among the collection's sorted ids; the key is the cause node's
//      cause when that is a key token, the cause node's cause id otherwise
//      (an id key), nil when the cause node is absent; a key cause
//      weaves under the key's virtual root [[0 "0" 0] nil nil];
//   3. a stable sort by (collection, key): every key weave is a run, id order kept;
//   4. per key weave, the list weave of the root + its nodes (SURVEY F4/F5:
//      effective parents, subtree sizes, siblings specials first by descending
//      id, preorder positions) -- as k_small_weave does, for key weaves of any
//      length up to the pack;
//   5. active-node per key weave (first rendered value, ::blank behind a hide).
// Key weaves are numbered across the batch with a decoupled look-back over the
// packs (a pack publishes its count, then sums its predecessors'), so every
// output goes straight to its final place: one pass over the inputs, one over
// the outputs, instead of the eleven kernels and three host readbacks of the
// general map path (kept for collections of more than MPK nodes).
//
// In the key weave a node caused by an id whose node is itself id-caused (an id
// key) or absent (the nil key) is never next to its cause, so weave-node
// appends it (shared.cljc:236-238): it chains after the previous node of the
// key weave, as k_seg_build does -- except under a self-caused id key, whose
// key weave holds its causes (k_map_key) and is folded literally.

constexpr uint32_t MPK = 2048;                 // largest pack (nodes)
constexpr uint16_t MP_ROOT = 0xFFFFu;          // cause-in-weave = the key weave's root
constexpr uint16_t MP_CHAIN = 0xFFFEu;         // appended after the previous node
constexpr uint16_t MP_ROOT_ID = 0xFFFDu;       // caused by the root id [0 "0" 0] (not a node)
constexpr uint16_t ML_ABSENT = 0xFFFFu;        // literal fold: the cause is not in the key weave
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INC = 2ull << 62;
// look-back word: flags (2 bits) | the call's epoch (16 bits, LB_EPOCH) | count:
// a word of an earlier call reads as "not published yet", so the words need
// no clearing before each call (cw_ctx::mpack.epoch; cleared when it wraps)
constexpr uint32_t LB_EPOCH = 46;

// Stable LDS radix sort of the pack's wave-blocked items by the low `bits` of
// ck (carrying val), 6 bits per sub-pass.  On return item u holds the element
// of sorted position wb_elem(u), and ks[] the sorted keys.
template <int NT, int IT, typename KS = uint64_t>
__device__ __forceinline__ void mp_sort(uint64_t (&ck)[IT], uint32_t (&val)[IT], uint32_t len,
                                        uint32_t bits, KS *ks, uint16_t *vs,
                                        uint32_t (*wcnt)[SUB_BINS], uint32_t *run) {
  uint32_t sd[IT], pos[IT];
  for (uint32_t sh = 0; sh < bits; sh += SUB_BITS) {
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) sd[u] = (uint32_t)(ck[u] >> sh) & (SUB_BINS - 1);
    rank_subdigit<NT, IT>(sd, len, min(SUB_BITS, bits - sh), pos, wcnt, run);
#pragma unroll
    for (uint32_t u = 0; u < IT; u++)
      if (wb_elem<IT>(u) < len) {
        ks[pos[u]] = (KS)ck[u];
        vs[pos[u]] = (uint16_t)val[u];
      }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t j = wb_elem<IT>(u);
      if (j < len) {
        ck[u] = ks[j];
        val[u] = vs[j];
      }
    }
    __syncthreads();
  }
}

template <int PK, int NT>
__global__ __launch_bounds__(NT) void k_map_pack(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause,
    const uint8_t *__restrict__ cause_is_id, const uint8_t *__restrict__ kind,
    const uint64_t *__restrict__ coll_off, const uint32_t *__restrict__ pack_doc0,
    const uint64_t *__restrict__ pack_s0, uint32_t P,
    uint32_t token_bits, unsigned long long *lb, uint64_t cap_segs, uint64_t n_total,
    uint64_t *__restrict__ seg_offsets, uint32_t *__restrict__ seg_coll,
    uint64_t *__restrict__ seg_key, int64_t *__restrict__ seg_active,
    uint32_t *__restrict__ seg_perm, uint32_t *__restrict__ status, uint32_t *ctl,
    unsigned long long *__restrict__ tprof, uint32_t nd_max, uint32_t epoch) {
  // (round 3-4 A/Bs, the winners built in: sort 1 through the id directory
  // where it fits, causes found through that directory too, the element loads
  // issued before the collection starts come in, relaxed look-back atomics --
  // the 64-bit word is the whole message, flag and count, so no acquire /
  // release fences around it)
  constexpr uint32_t IT = PK / NT;
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
  auto stamp = [&](int ph) {  // diagnostic phase times (CW_TREE_PROF)
    if (tprof) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tacc[ph] += now - tlast;
      tlast = now;
    }
  };
  stamp(-1);
  // LDS by phase: A = sorted (collection, id) keys, then sorted (collection,
  // key) keys, then the key weaves' numbering (SEG, SS), siblings-before and
  // weave order (BEF, WV); B = causes by input index, then each member's parent,
  // effective parent and subtree size (PAR, EFF, SZ).  By position: I2J (id
  // order -> input), P16 (id order: cause position or MP_*), Q (id order -> key
  // order), LQ / KQ (key order: collection-local input index, kind).
  __shared__ uint64_t A[PK], B[PK];
  __shared__ __attribute__((aligned(16))) uint16_t U16[5 * PK];  // VS I2J P16 Q LQ (one block: sort 1's directory)
  uint16_t *const VS = U16, *const I2J = U16 + PK, *const P16 = U16 + 2 * PK, *const Q = U16 + 3 * PK,
                  *const LQ = U16 + 4 * PK;
  __shared__ uint8_t K8[PK], KQ[PK];
  // per collection of the pack (start, status): dynamic LDS sized by the most
  // collections a pack of this batch holds, not PK -- 4 KB less a pack at 512
  // nodes, 10 packs a CU instead of 8 (the kernel is latency-bound)
  extern __shared__ uint32_t mp_dyn[];
  uint32_t *const dstart = mp_dyn, *const dstat = mp_dyn + (nd_max + 1);
  __shared__ uint32_t wcnt[NT / 64][SUB_BINS], run[64], wtot[NT / 64];
  __shared__ uint32_t s_base;
  __shared__ unsigned long long s_or[2];
  __shared__ unsigned long long s_kor;  // sort 2's key widths (step 2)
  __shared__ uint32_t s_kcls;
  __shared__ uint8_t SLIT[PK];  // key weave woven by the literal fold (root-id / non-Lamport causes)
  uint16_t *SEG = reinterpret_cast<uint16_t *>(A), *SS = SEG + PK, *BEF = SS + PK, *WV = BEF + PK;
  uint16_t *PAR = reinterpret_cast<uint16_t *>(B), *EFF = PAR + PK;
  uint32_t *SZ = reinterpret_cast<uint32_t *>(EFF + PK);

  const uint32_t pk = blockIdx.x, tid = threadIdx.x;
  // the pack's node range from the host's pack table: the element loads go out
  // first, in flight while the collection starts come in
  const uint32_t d0 = pack_doc0[pk], nd = pack_doc0[pk + 1] - d0;
  const uint64_t s0 = pack_s0[pk];
  const uint32_t len = (uint32_t)(pack_s0[pk + 1] - s0);
  uint64_t lc[IT], lid[IT];
  uint8_t lcis[IT], lkd[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t j = wb_elem<IT>(u);
    const bool ok = j < len;
    lc[u] = ok ? cause[s0 + j] : 0ull;
    lid[u] = ok ? id_key[s0 + j] : 0ull;
    lcis[u] = ok ? cause_is_id[s0 + j] : 0;
    lkd[u] = ok ? kind[s0 + j] : 0;
  }
  for (uint32_t i = tid; i <= nd; i += NT) dstart[i] = (uint32_t)(coll_off[d0 + i] - s0);
  for (uint32_t i = tid; i < nd; i += NT) dstat[i] = 0;
  if (tid < 2) s_or[tid] = 0;
  if (tid == 0) {
    s_kor = 0;
    s_kcls = 0;
  }
  __syncthreads();
  const uint64_t tmask = (1ull << token_bits) - 1;

  // 1. load; stable sort by (collection, id) -- (sort ::nodes), map.cljc:28
  // (the pack's own key widths: ids, id causes, collections in the pack)
  uint64_t ck[IT];
  uint32_t val[IT], dl0[IT];
  unsigned long long oid = 0, oca = 0;
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t j = wb_elem<IT>(u);
    ck[u] = 0;
    val[u] = 0;
    dl0[u] = 0;
    if (j < len) {
      uint32_t lo = 0, hi = nd;  // the collection of element j
      while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (dstart[m] <= j) lo = m; else hi = m;
      }
      const uint64_t c = lc[u];
      const uint8_t cis = lcis[u];
      const bool cid = cis == 1;
      B[j] = c;
      // 0x80: the cause is an id; 0x40: the cause is nil (cause_is_id = 2)
      K8[j] = (uint8_t)((cid ? 0x80u : cis == 2 ? 0x40u : 0u) | (lkd[u] & KIND_CLASS));
      ck[u] = lid[u];
      oid |= ck[u];
      oca |= cid ? c : 0ull;
      val[u] = j;
      dl0[u] = lo;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    oid |= __shfl_xor(oid, o, 64);
    oca |= __shfl_xor(oca, o, 64);
  }
  if ((tid & 63) == 0) {
    if (oid) atomicOr(&s_or[0], oid);
    if (oca) atomicOr(&s_or[1], oca);
  }
  __syncthreads();
  const uint32_t kbits = s_or[0] ? 64 - __builtin_clzll(s_or[0]) : 1;
  const uint32_t cbits = s_or[1] ? 64 - __builtin_clzll(s_or[1]) : 1;
  const uint32_t dbits = nd > 1 ? 32 - __builtin_clz(nd - 1) : 0;
  const uint32_t W = max(max(token_bits, kbits), cbits);
  // composite sort keys must fit 63 bits: otherwise the general path (host)
  const bool fits = kbits + dbits <= 63 && W + 2 + dbits <= 63;
  if (!fits && tid == 0) atomicOr(&ctl[2], 1u);
  const uint64_t imask = (1ull << min(kbits, 63u)) - 1;
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) ck[u] = fits ? (((uint64_t)dl0[u] << kbits) | ck[u]) : 0ull;
  // Lamport ids are dense: when every collection's id range fits a slice of a
  // pack-wide bitmap (P16 | Q | LQ, 1.5 PK words), an id's sorted position is
  // the number of set bits before it -- one atomicOr and one lookup a node
  // instead of the radix passes.  A repeated id (DUP) takes the sort.
  // The directory and its word prefixes (VS) stay for step 2, which then finds
  // each id cause the same way instead of by binary search (DIRJOIN).
  constexpr uint32_t DIRW = PK;
  const uint32_t lw = kbits > 5 ? kbits - 5 : 0;  // log2 of the words per collection
  bool sorted = false;
  uint32_t *const dir = reinterpret_cast<uint32_t *>(P16);
  uint16_t *const wpre = VS;
  if (fits && ((uint64_t)nd << lw) <= DIRW) {
    const uint32_t nwd = nd << lw;
    for (uint32_t w = tid; w < nwd; w += NT) dir[w] = 0;
    __syncthreads();
    bool dup = false;
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      if (wb_elem<IT>(u) >= len) continue;
      const uint32_t x = (uint32_t)(ck[u] & imask), w = (dl0[u] << lw) + (x >> 5), m = 1u << (x & 31);
      dup |= (atomicOr(&dir[w], m) & m) != 0;
    }
    if (!__syncthreads_or(dup)) {
      // exclusive prefix of the words' popcounts: contiguous words per thread
      const uint32_t per = (nwd + NT - 1) / NT, w0 = min(nwd, tid * per), w1 = min(nwd, w0 + per);
      uint32_t c = 0;
      for (uint32_t w = w0; w < w1; w++) c += __popc(dir[w]);
      uint32_t run0 = block_exscan<NT>(c, wtot, nullptr);
      for (uint32_t w = w0; w < w1; w++) {
        wpre[w] = (uint16_t)run0;
        run0 += __popc(dir[w]);
      }
      __syncthreads();
      uint32_t pos[IT];
#pragma unroll
      for (uint32_t u = 0; u < IT; u++) {
        const uint32_t x = (uint32_t)(ck[u] & imask), w = (dl0[u] << lw) + (x >> 5);
        pos[u] = wb_elem<IT>(u) < len ? wpre[w] + __popc(dir[w] & ((1u << (x & 31)) - 1)) : 0u;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < IT; u++)
        if (wb_elem<IT>(u) < len) {
          A[pos[u]] = ck[u];
          I2J[pos[u]] = (uint16_t)val[u];
        }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < IT; u++) {
        const uint32_t j = wb_elem<IT>(u);
        if (j < len) {
          ck[u] = A[j];
          val[u] = I2J[j];
        }
      }
      __syncthreads();
      sorted = true;
    }
  }
  if (!sorted) mp_sort<NT, IT>(ck, val, len, fits ? kbits + dbits : 1, A, VS, wcnt, run);
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t i = wb_elem<IT>(u);
    if (i >= len) continue;
    I2J[i] = (uint16_t)val[u];
    // a repeated id (::nodes is a map); an id of 0 repeats the virtual root's
    if ((i > 0 && A[i - 1] == ck[u]) || (ck[u] & imask) == 0)
      atomicOr(&dstat[ck[u] >> kbits], (uint32_t)CW_STATUS_DUP);
  }
  __syncthreads();

  stamp(0);
  // 2. key and cause-in-weave of every node, in id order (map.cljc:31-37).
  // With the directory of sort 1 still in P16 | Q | LQ (DIRJOIN), an id cause
  // is a bit test and a popcount; P16 is written after a barrier then.
  const bool djoin = sorted;
  uint16_t pv[IT];
  unsigned long long kor = 0;
  uint32_t cor = 0;
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t i = wb_elem<IT>(u);
    pv[u] = 0;
    if (i >= len) continue;
    const uint32_t dl = (uint32_t)(ck[u] >> kbits), j = val[u];
    const uint64_t c = B[j];
    uint64_t key;
    uint16_t p;
    uint32_t st = 0;
    if (K8[j] & 0x80u) {  // (spec/valid? ::s/id cause): the cause node
      const uint32_t a1 = dstart[dl + 1];
      const bool inrange = (c & ~imask) == 0;
      uint32_t lo = dstart[dl];
      bool found;
      if (djoin) {
        const uint32_t x = (uint32_t)c, w = (dl << lw) + (x >> 5);
        const uint32_t dw = inrange ? dir[w] : 0u;
        found = (dw >> (x & 31)) & 1u;
        lo = found ? wpre[w] + __popc(dw & ((1u << (x & 31)) - 1)) : lo;
      } else {  // binary search among the collection's sorted ids
        const uint64_t want = ((uint64_t)dl << kbits) | c;
        uint32_t hi = a1;
        while (inrange && lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (A[m] < want) lo = m + 1; else hi = m;
        }
        found = inrange && lo < a1 && A[lo] == want;
      }
      if (found) {
        const uint32_t jc = I2J[lo];
        const uint64_t gc = B[jc];
        if (K8[jc] & 0x80u) {  // the cause node is id-caused: the key is that id (F8c)
          key = (1ull << W) | gc;
          // a chain, unless the key's node X = gc is self-caused: then X, its
          // children and grandchildren share the key weave with their causes
          // (k_map_key) -- real causes, and X's own makes it a literal key weave
          bool selfk = gc == c;
          if (!selfk && (gc & ~imask) == 0) {
            const uint64_t want = ((uint64_t)dl << kbits) | gc;
            uint32_t l2 = dstart[dl], h2 = a1;
            while (l2 < h2) {
              const uint32_t m = (l2 + h2) >> 1;
              if (A[m] < want) l2 = m + 1; else h2 = m;
            }
            if (l2 < a1 && A[l2] == want) {
              const uint32_t jx = I2J[l2];
              selfk = (K8[jx] & 0x80u) && B[jx] == gc;
            }
          }
          p = selfk ? (uint16_t)lo : MP_CHAIN;
        } else if (K8[jc] & 0x40u) {  // the cause node's cause is nil: the nil key, under it
          key = 2ull << W;
          p = (uint16_t)lo;
        } else {
          key = gc & tmask;
          if (gc > tmask) st |= CW_STATUS_MAP_KEY;
          p = (uint16_t)lo;
        }
      } else {  // the cause node is absent: the nil key
        key = 2ull << W;
        // (caused by the root id: woven right after the nil key weave's root,
        // which the literal fold below handles; other absent causes append)
        p = c == 0 ? MP_ROOT_ID : MP_CHAIN;
      }
    } else if (K8[j] & 0x40u) {  // a nil cause: the nil key, under its root (map.cljc:35-37)
      key = 2ull << W;
      p = MP_ROOT_ID;
    } else {  // a key: woven under that key's root
      key = c & tmask;
      if (c > tmask) st |= CW_STATUS_MAP_KEY;
      p = MP_ROOT;
    }
    pv[u] = p;
    if (st) atomicOr(&dstat[dl], st);
    kor |= key & ((1ull << W) - 1);
    cor |= 1u << (uint32_t)(key >> W);
    ck[u] = ((uint64_t)dl << (W + 2)) | key;
    val[u] = i;
  }
  // the widths sort 2 needs in THIS pack: the largest key value's bits, and
  // the class field only when a key weave that is not a plain key occurs (an
  // id key or the nil key; config 4's packs have none: 8 + 3 bits, two 6-bit
  // passes instead of three)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kor |= __shfl_xor(kor, o, 64);
    cor |= __shfl_xor(cor, o, 64);
  }
  if ((tid & 63) == 0) {
    if (kor) atomicOr(&s_kor, kor);
    atomicOr(&s_kcls, cor);
  }
  if (djoin) __syncthreads();  // (every directory lookup done before P16 is written)
#pragma unroll
  for (uint32_t u = 0; u < IT; u++)
    if (wb_elem<IT>(u) < len) P16[wb_elem<IT>(u)] = pv[u];
  __syncthreads();
  const uint32_t W2 = s_kor ? 64 - __builtin_clzll(s_kor) : 1;  // (<= W)
  const uint32_t CB = (s_kcls & ~1u) ? 2u : 0u, KS = W2 + CB;      // key field = class | value
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint64_t g = ck[u] & ((1ull << (W + 2)) - 1), kv = g & ((1ull << W) - 1), cl = g >> W;
    ck[u] = fits ? (((ck[u] >> (W + 2)) << KS) | (cl << W2) | kv) : 0ull;
  }

  stamp(1);
  // 3. stable sort by (collection, key): every key weave a run, id order kept
  mp_sort<NT, IT>(ck, val, len, fits ? KS + dbits : 1, A, VS, wcnt, run);
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    if (q >= len) continue;
    const uint32_t i = val[u], j = I2J[i], dl = (uint32_t)(ck[u] >> KS);
    Q[i] = (uint16_t)q;
    LQ[q] = (uint16_t)(j - dstart[dl]);
    KQ[q] = K8[j] & KIND_CLASS;
  }
  // key weave heads over contiguous runs of IT positions (A: the sorted keys)
  uint32_t heads = 0;
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t q = tid * IT + k;
    if (q < len && (q == 0 || A[q] != A[q - 1])) heads |= 1u << k;
  }
  uint32_t nseg;
  const uint32_t sfirst = block_exscan<NT>(__popc(heads), wtot, &nseg);  // (its barriers free A)
  {
    uint32_t sg = sfirst;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t q = tid * IT + k;
      if (q >= len) continue;
      if ((heads >> k) & 1u) SS[sg++] = (uint16_t)q;
      SEG[q] = (uint16_t)(sg - 1);
    }
  }
  for (uint32_t sg = tid; sg < nseg; sg += NT) SLIT[sg] = 0;
  __syncthreads();  // SEG / SS are read across threads below
  stamp(2);
  // 4. publish this pack's number of key weaves (its prefix comes after the
  // weave below, so the wait for earlier packs overlaps this pack's work)
  const unsigned long long ep = (unsigned long long)epoch << LB_EPOCH;
  if (tid == 0) {
    const unsigned long long w = (pk == 0 ? LB_INC : LB_AGG) | ep | nseg;
    __hip_atomic_store(lb + pk, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // 5. each key weave's list weave: member 0 the root, members 1..m in id order
  uint32_t mst[IT], mm[IT], mr[IT], me[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    mst[u] = mm[u] = mr[u] = me[u] = 0;
    if (q >= len) continue;
    const uint32_t sg = SEG[q], st0 = SS[sg], en = sg + 1 < nseg ? SS[sg + 1] : len;
    const uint32_t r = q - st0 + 1;
    mst[u] = st0;
    mm[u] = en - st0;
    mr[u] = r;
    const uint16_t p = P16[val[u]];
    uint32_t par = 0;
    if (p == MP_CHAIN) {
      par = r - 1;
    } else if (p == MP_ROOT_ID) {  // a child of the key weave's root, next to appended nodes
      SLIT[sg] = 1;
    } else if (p != MP_ROOT) {  // the cause node: same key, so same key weave
      const uint32_t qc = Q[p], dl = (uint32_t)(ck[u] >> KS);
      if (qc < st0 || qc >= en) {
        atomicOr(&dstat[dl], (uint32_t)CW_STATUS_INTERNAL);
      } else if (qc >= q) {  // the cause has a larger id: the literal fold
        atomicOr(&dstat[dl], (uint32_t)CW_STATUS_NON_LAMPORT);
        SLIT[sg] = 1;
        par = qc - st0 + 1;
      } else {
        par = qc - st0 + 1;
      }
    }
    PAR[q] = (uint16_t)par;
    SZ[q] = 1;
  }
  __syncthreads();
  // a key weave the literal fold takes: each member's cause-in-weave as the
  // fold sees it (0 = the root, a member, or ML_ABSENT: appended)
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    if (q >= len || !SLIT[SEG[q]]) continue;
    const uint16_t p = P16[val[u]];
    if (p == MP_CHAIN) PAR[q] = ML_ABSENT;
    else if (p == MP_ROOT_ID || p == MP_ROOT) PAR[q] = 0;
    me[u] = 0;
  }
  __syncthreads();
  // effective parent: a non-special climbs through special causes
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    if (q >= len) continue;
    if (SLIT[SEG[q]]) continue;  // (the literal fold below)
    uint32_t e = PAR[q];
    if (!is_special(KQ[q]))
      for (uint32_t it = 0; e != 0 && is_special(KQ[mst[u] + e - 1]) && it < mm[u]; it++)
        e = PAR[mst[u] + e - 1];
    EFF[q] = (uint16_t)e;
    me[u] = e;
  }
  __syncthreads();
  // subtree sizes: every member counts itself into each effective ancestor
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    uint32_t a = me[u];
    for (uint32_t it = 0; a != 0 && it < mm[u]; it++) {
      atomicAdd(&SZ[mst[u] + a - 1], 1u);
      a = EFF[mst[u] + a - 1];
    }
  }
  __syncthreads();
  stamp(6);
  // siblings before me (weave order inside a parent: specials by descending
  // id, then non-specials by descending id): the members, fed in descending
  // id order, sorted stably by (parent, class) -- each parent's children are
  // then one run in weave order -- and a segmented exclusive prefix sum of
  // their subtree sizes over each run (VS, P16, dstart are free by now)
  {
    // keys (parent index << 1 | class), parent index < PK + key weaves <= 2 PK:
    // SB bits (two 6-bit passes at PK = 512, three at 2048); members of literal
    // key weaves sort last
    constexpr uint32_t SB = 33 - __builtin_clz(2u * PK);
    constexpr uint64_t NOKEY = (1ull << SB) - 1;
    uint64_t gk[IT];
    uint32_t gv[IT];
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t j = wb_elem<IT>(u);
      gk[u] = NOKEY;
      gv[u] = 0;
      if (j >= len) continue;
      const uint32_t q = len - 1 - j, sg = SEG[q];
      gv[u] = q;
      if (SLIT[sg]) continue;
      const uint32_t e = EFF[q], pidx = e ? SS[sg] + e - 1 : PK + sg;  // (PK + sg: the root)
      gk[u] = ((uint64_t)pidx << 1) | (is_special(KQ[q]) ? 0u : 1u);
    }
    mp_sort<NT, IT, uint16_t>(gk, gv, len, SB, VS, P16, wcnt, run);
    // segmented inclusive prefix sums in registers: lanes by shuffles, the
    // wave's IT chunks of 64 in order, then the carry from earlier waves
    const uint32_t lane = tid & 63, wv = tid >> 6;
    uint32_t x[IT], sz[IT], gs[IT], carry = 0, cseg = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t j = wb_elem<IT>(u);
      gs[u] = (uint32_t)(gk[u] >> 1);
      sz[u] = j < len ? SZ[gv[u]] : 0u;
      uint32_t v = sz[u];
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64), sy = __shfl_up(gs[u], o, 64);
        if (lane >= o && sy == gs[u]) v += y;
      }
      if (gs[u] == cseg) v += carry;
      carry = __shfl(v, 63, 64);
      cseg = __shfl(gs[u], 63, 64);
      x[u] = v;
    }
    uint32_t *wl = wtot, *wsl = run, *wsf = run + NT / 64;  // (free after the sort)
    const uint32_t first = __shfl(gs[0], 0, 64);
    if (lane == 0) {
      wl[wv] = carry;
      wsl[wv] = cseg;
      wsf[wv] = first;
    }
    __syncthreads();
    uint32_t cin = 0;
    for (int w2 = (int)wv - 1; w2 >= 0; w2--) {  // earlier waves ending in my first run
      if (wsl[w2] != first) break;
      cin += wl[w2];
      if (wsf[w2] != first) break;  // the run starts inside that wave
    }
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t j = wb_elem<IT>(u);
      if (gs[u] == first) x[u] += cin;
      if (j < len && gk[u] != NOKEY) BEF[gv[u]] = (uint16_t)(x[u] - sz[u]);
    }
  }
  __syncthreads();
  stamp(7);
  // preorder position = sum over the effective ancestors of (1 + siblings before)
  uint32_t mpos[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    mpos[u] = 0;
    if (q >= len || SLIT[SEG[q]]) continue;
    uint32_t pos = 0, x = mr[u];
    for (uint32_t it = 0; x != 0 && it < mm[u]; it++) {
      pos += 1 + BEF[mst[u] + x - 1];
      x = EFF[mst[u] + x - 1];
    }
    if (pos < 1 || pos > mm[u]) {
      atomicOr(&dstat[(uint32_t)(ck[u] >> KS)], (uint32_t)CW_STATUS_INTERNAL);
      continue;
    }
    WV[mst[u] + pos - 1] = (uint16_t)q;
    mpos[u] = pos;
  }
  __syncthreads();
  // the literal fold (shared.cljc:225-241, as exact.hip's k_xfold) for key
  // weaves whose nodes are not all children of their causes in id order: one
  // thread per such key weave, a linked list over its members (EFF = next,
  // SZ = "a member with a smaller id is caused by me"); then each member's
  // weave position into BEF
  for (uint32_t sg = tid; sg < nseg; sg += NT) {
    if (!SLIT[sg]) continue;
    const uint32_t st0 = SS[sg], m = (sg + 1 < nseg ? SS[sg + 1] : len) - st0;
    constexpr uint32_t END = 0xFFFFu, HEAD = 0xFFFEu;
    for (uint32_t x = 1; x <= m; x++) SZ[st0 + x - 1] = 0;
    for (uint32_t x = 1; x <= m; x++) {
      const uint32_t c = PAR[st0 + x - 1];
      if (c != ML_ABSENT && c > x && c <= m) SZ[st0 + c - 1] = 1;
    }
    uint32_t head = END, tail = END;
    auto nxt = [&](uint32_t v) -> uint32_t { return v == HEAD ? head : EFF[st0 + v - 1]; };
    for (uint32_t x = 1; x <= m; x++) {
      const uint32_t c = PAR[st0 + x - 1];
      const bool sp = is_special(KQ[st0 + x - 1]);
      uint32_t at = END;  // the node x goes after (HEAD: right after the root)
      if (c == 0) {
        at = HEAD;
      } else if (SZ[st0 + x - 1]) {  // first of: after the cause, before a child
        uint32_t prev = HEAD;
        for (uint32_t v = head; v != END; prev = v, v = EFF[st0 + v - 1]) {
          if (PAR[st0 + v - 1] == x) {
            at = prev;
            break;
          }
          if (v == c) {
            at = v;
            break;
          }
        }
      } else if (c != ML_ABSENT && c < x) {
        at = c;
      }
      if (at == END) {
        at = tail == END ? HEAD : tail;  // weave-asap? never held: the end
      } else if (!sp) {                   // clause A: skip specials not caused by x
        for (;;) {
          const uint32_t q2 = nxt(at);
          if (q2 == END || !is_special(KQ[st0 + q2 - 1]) || PAR[st0 + q2 - 1] == x) break;
          at = q2;
        }
      }
      const uint32_t q2 = nxt(at);
      EFF[st0 + x - 1] = (uint16_t)q2;
      if (at == HEAD) head = x;
      else EFF[st0 + at - 1] = (uint16_t)x;
      if (q2 == END) tail = x;
    }
    uint32_t pos = 1;
    for (uint32_t v = head; v != END && pos <= m; v = EFF[st0 + v - 1], pos++) {
      WV[st0 + pos - 1] = (uint16_t)(st0 + v - 1);
      BEF[st0 + v - 1] = (uint16_t)pos;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t q = wb_elem<IT>(u);
    if (q < len && SLIT[SEG[q]]) mpos[u] = BEF[q];
  }
  // 6. active-node per key weave (map.cljc:47-59): blank when the first node
  // after the root is a hide; else the first non-special not followed by a hide
  int32_t *ACT = reinterpret_cast<int32_t *>(SZ);  // (sizes are done)
  for (uint32_t sg = tid; sg < nseg; sg += NT) {
    const uint32_t st0 = SS[sg], m = (sg + 1 < nseg ? SS[sg + 1] : len) - st0;
    int32_t act = -1;
    uint32_t k = KQ[WV[st0]];
    if (!is_hide((uint8_t)k)) {
      for (uint32_t p = 1; p <= m; p++) {
        const uint32_t nk = p < m ? KQ[WV[st0 + p]] : 0u;
        if (!is_special((uint8_t)k) && !(p < m && is_hide((uint8_t)nk))) {
          act = (int32_t)LQ[WV[st0 + p - 1]];
          break;
        }
        k = nk;
      }
    }
    ACT[sg] = act;
  }
  stamp(4);
  // 7. this pack's first key weave number: decoupled look-back over the packs,
  // one wave reading LBW windows of 64 predecessors per round trip (earlier
  // packs are dispatched first and publish their counts before weaving, so the
  // wait always ends).  The resident packs reach their look-backs together, so
  // the nearest inclusive prefix is typically a whole residency (~500 packs)
  // back: one window per round trip cost ~8 L2 round trips (20k clocks).
  if (tid < 64) {
    constexpr uint32_t LBW = 1, lbw = 1;  // (four windows a round trip lost in round 3)
    const uint32_t lane = tid;
    uint32_t base = 0;
    if (pk > 0) {
      for (int64_t q0 = (int64_t)pk - 1;;) {
        unsigned long long v[LBW];
#pragma unroll
        for (uint32_t k = 0; k < LBW; k++) {
          const int64_t q = q0 - 64 * (int64_t)k - lane;  // lane 0 of window 0 = the nearest
          v[k] = !(q >= 0 && k < lbw) ? (k < lbw ? LB_INC | ep : 0ull)
                 : __hip_atomic_load(lb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (((v[k] >> LB_EPOCH) & 0xFFFFull) != epoch) v[k] = 0;  // an earlier call's word
        }
        bool done = false, retry = false;  // (wave-uniform: ballots)
#pragma unroll
        for (uint32_t k = 0; k < LBW; k++) {
          if (done || retry || k >= lbw) continue;
          const uint64_t inc = __ballot((v[k] >> 62) == 2), none = __ballot((v[k] >> 62) == 0);
          const uint32_t first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;  // nearest inclusive
          const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
          if (none & need) {  // a pack in this window has not counted its key weaves yet
            retry = true;
            continue;
          }
          uint32_t x = lane <= first ? (uint32_t)v[k] : 0u;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
          base += x;
          if (first < 64) done = true;
          else q0 -= 64;
        }
        if (done) break;
        if (retry) __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0)
      {
        __hip_atomic_store(lb + pk, LB_INC | ep | (base + nseg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (lane == 0) {
      s_base = base;
      if ((uint64_t)base + nseg > cap_segs) atomicOr(&ctl[1], 1u);
      if (pk == P - 1) {  // the batch's number of key weaves, and the end offset
        ctl[0] = base + nseg;
        if ((uint64_t)base + nseg <= cap_segs) seg_offsets[base + nseg] = n_total + base + nseg;
      }
    }
  }
  __syncthreads();
  stamp(3);
  const uint32_t sbase = s_base;
  // 8. outputs: key weave sg = its root, then its members in weave order
  if ((uint64_t)sbase + nseg <= cap_segs) {
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t q = wb_elem<IT>(u);
      if (q >= len || mpos[u] == 0) continue;
      const uint32_t sg = SEG[q];
      const uint64_t goff = s0 + mst[u] + sbase + sg;
      seg_perm[goff + mpos[u]] = LQ[q];
      if (mr[u] == 1) {
        const uint64_t g = ck[u] & ((1ull << KS) - 1), cls = g >> W2, kv = g & ((1ull << W2) - 1);
        seg_perm[goff] = 0xFFFFFFFFu;
        seg_offsets[sbase + sg] = goff;
        seg_coll[sbase + sg] = d0 + (uint32_t)(ck[u] >> KS);
        seg_key[sbase + sg] = cls == 0 ? kv : cls == 1 ? (CW_MAP_ID_KEY | kv) : CW_NIL;
      }
    }
    for (uint32_t sg = tid; sg < nseg; sg += NT) seg_active[sbase + sg] = ACT[sg];
  }
  for (uint32_t dl = tid; dl < nd; dl += NT) status[d0 + dl] = dstat[dl];
  stamp(5);
  if (tprof && tid == 0)
    for (int ph = 0; ph < 8; ph++) tprof[(size_t)pk * 8 + ph] = tacc[ph];
}

namespace {

// cw_weave_maps through k_map_pack: every collection <= MPK nodes and every
// pack's sort keys fit 63 bits (each pack finds its own key widths: no
// reduction over the batch and no readback before the kernel).  Returns 1 when it does not apply (the caller takes
// the general path), 2 when the layout taken on trust (pc.verify) differs from
// the cached one (the caller checks it and calls again), 0 on success, -1 on
// error.
int weave_maps_packed(cw_ctx *c, const cw_map_batch *bt, cw_map_result *res, bool dev,
                      const uint64_t *id, const uint64_t *cause, const uint8_t *cis,
                      const uint8_t *kind) {
  const uint64_t D = bt->n_colls, *off = bt->coll_offsets;
  const uint32_t N = (uint32_t)off[D];
  // pack table, cached while the collection layout repeats
  auto &pc = c->mpack;
  // pack size: the smallest of 512 / 1024 / 2048
  // nodes that holds the largest collection -- smaller packs are more
  // workgroups a CU with cheaper barriers (config 4: 2048 nodes 3.77 ms,
  // 1024 3.26, 512 3.15; 256 nodes / one wave: 3.95)
  const uint64_t mc = pc.maxcoll;
  const uint32_t PKN = mc <= 512 ? 512u : mc <= 1024 ? 1024u : MPK;
  if (!(pc.pk == PKN && pc.same)) {
    pc.off.assign(off, off + D + 1);
    pc.pk = PKN;
    pc.doc0.clear();
    pc.ok = true;
    uint32_t dmax = 1;
    pc.dmax = 1;
    for (uint64_t d = 0; d < D;) {
      const uint64_t a = d;
      while (d < D && off[d + 1] - off[a] <= PKN) d++;
      if (d == a) {  // a collection of more than MPK nodes
        pc.ok = false;
        break;
      }
      pc.doc0.push_back((uint32_t)a);
      dmax = std::max<uint32_t>(dmax, (uint32_t)(d - a));
    }
    pc.doc0.push_back((uint32_t)D);
    pc.dbits = ceil_log2(dmax);
    pc.dmax = dmax;
    if (pc.ok) {
      uint32_t *dp = scratch_t<uint32_t>(c, "mp_doc0", pc.doc0.size());
      uint64_t *dof = scratch_t<uint64_t>(c, "mp_off", D + 1);
      uint64_t *ds0 = scratch_t<uint64_t>(c, "mp_s0", pc.doc0.size());  // each pack's first node
      if (!dp || !dof) return fail(c, "out of device memory (map packs)");
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipMemcpy(dp, pc.doc0.data(), pc.doc0.size() * 4, hipMemcpyHostToDevice));
      std::vector<uint64_t> s0(pc.doc0.size());
      for (size_t k = 0; k < s0.size(); k++) s0[k] = off[pc.doc0[k]];
      if (!ds0) return fail(c, "out of device memory (map packs)");
      HIPCHK(c, hipMemcpy(ds0, s0.data(), s0.size() * 8, hipMemcpyHostToDevice));
      HIPCHK(c, hipMemcpy(dof, off, (D + 1) * 8, hipMemcpyHostToDevice));
    }
  }
  if (!pc.ok) return 1;
  const uint32_t P = (uint32_t)pc.doc0.size() - 1;
  const uint64_t cap = res->cap_segs;
  unsigned long long *lb = scratch_t<unsigned long long>(c, "mp_lb", P);
  uint32_t *ctl = scratch_t<uint32_t>(c, "mp_ctl", 4);
  if (!lb || !ctl) return fail(c, "out of device memory (map packs)");
  // outputs: the caller's arrays (device memory) or staging (host memory)
  uint64_t *so = res->seg_offsets, *sk = res->seg_key;
  uint32_t *sc = res->seg_coll, *sp = res->seg_perm, *st = res->status;
  int64_t *sa = res->seg_active;
  if (!dev) {
    so = scratch_t<uint64_t>(c, "mp_so", cap + 1);
    sk = scratch_t<uint64_t>(c, "mp_sk", cap);
    sc = scratch_t<uint32_t>(c, "mp_sc", cap);
    sp = scratch_t<uint32_t>(c, "mp_sp", N + cap);
    st = scratch_t<uint32_t>(c, "mp_st", D);
    sa = scratch_t<int64_t>(c, "mp_sa", cap);
    if (!so || !sk || !sc || !sp || !st || !sa) return fail(c, "out of device memory (map outputs)");
  }
  unsigned long long *tprof = nullptr;
  if (c->tree_prof) {
    tprof = scratch_t<unsigned long long>(c, "mp_tprof", (size_t)P * 8);
    if (!tprof) return fail(c, "out of device memory (tprof)");
    HIPCHK(c, hipMemsetAsync(tprof, 0, (size_t)P * 64, c->stream));
  }
  // a new epoch per call; the words are cleared only when the epoch wraps or
  // the buffer was (re)allocated for more packs than it held
  if (++pc.epoch >= 0xFFFF || lb != pc.lb || P > pc.lb_packs) {
    HIPCHK(c, hipMemsetAsync(lb, 0, (size_t)P * 8, c->stream));
    pc.epoch = 1;
    pc.lb = lb;
    pc.lb_packs = P;
  }
  HIPCHK(c, hipMemsetAsync(ctl, 0, 16, c->stream));
  {
    // ids, causes, flags and kinds in; per node seg_perm, per key weave
    // offsets, collection, key, active node out
    Launch L(c, "m_pack", (double)N * (8 + 8 + 1 + 1 + 4) + (double)N * 0.42 * (4 + 8 + 4 + 8 + 8));
#define CW_MAP_PACK_LAUNCH(PK_, NT_)                                                              \
  hipLaunchKernelGGL((k_map_pack<PK_, NT_>), dim3(P), dim3(NT_), (size_t)(2 * pc.dmax + 1) * 4,       \
                     c->stream, id, cause, cis, kind,                                                  \
                     (const uint64_t *)c->bufs["mp_off"].p, (const uint32_t *)c->bufs["mp_doc0"].p, \
                     (const uint64_t *)c->bufs["mp_s0"].p,                                             \
                     P, bt->token_bits, lb, cap, (uint64_t)N, so, sc, sk, sa,                          \
                     sp, st, ctl, tprof, pc.dmax, pc.epoch)
    if (pc.pk == 512) CW_MAP_PACK_LAUNCH(512, 128);
    else if (pc.pk == 1024) CW_MAP_PACK_LAUNCH(1024, 256);
    else CW_MAP_PACK_LAUNCH(2048, 512);
#undef CW_MAP_PACK_LAUNCH
  }
  if (check_launch(c, "map_pack")) return -1;
  if (pc.verify &&
      memcmp(pc.off.data(), off, (D + 1) * 8) != 0)  // (the kernel runs meanwhile)
    return 2;  // another layout after all: the caller checks it and weaves again
  if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
  HIPCHK(c, hipMemcpyAsync(c->pin_small, ctl, 12, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->pin_small[2]) return 1;  // a pack's keys need more than 63 bits: the general path
  const uint64_t S = c->pin_small[0];
  if (c->pin_small[1]) return fail(c, "cap_segs too small: %llu key weaves", (unsigned long long)S);
  if (tprof) {
    std::vector<unsigned long long> h((size_t)P * 8);
    HIPCHK(c, hipMemcpy(h.data(), tprof, (size_t)P * 64, hipMemcpyDeviceToHost));
    double a[8] = {0};
    for (uint32_t q = 0; q < P; q++)
      for (int ph = 0; ph < 8; ph++) a[ph] += (double)h[(size_t)q * 8 + ph];
    fprintf(stderr, "map pack phases (memtime ticks per pack): sort1 %.0f keys %.0f sort2 %.0f "
            "weave+active %.0f (of which eff+sizes %.0f, siblings-before %.0f) lookback %.0f "
            "outputs %.0f\n", a[0] / P, a[1] / P, a[2] / P, (a[4] + a[6] + a[7]) / P, a[6] / P, a[7] / P,
            a[3] / P, a[5] / P);
  }
  if (!dev) {
    HIPCHK(c, hipMemcpy(res->seg_perm, sp, ((size_t)N + S) * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->seg_offsets, so, (S + 1) * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->seg_coll, sc, S * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->seg_key, sk, S * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->seg_active, sa, S * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->status, st, D * 4, hipMemcpyDeviceToHost));
  }
  res->n_segs = S;
  if (c->prof) return collect_prof(c);
  return 0;
}

}  // namespace
