// dist.hip -- the tree of ONE list spread over several GPUs (BASELINE config
// 5), rank by rank.  Included by causeweave.hip after weave_tail.
//
// After the sample sort and the cause join (cause_amd/giant.py) rank r holds
// the nodes of global ranks [base, base + n) -- a contiguous run of the id
// order -- with par (global rank of the cause) and kind.  The single-GPU tree
// (k_geff / k_gsib / k_gthr: SURVEY F5 effective parents, sibling order, F6
// visibility, preorder successors) needs nodes of other ranks in three places,
// each resolved by all-to-all rounds between kernels of this file:
//
//   effective parent: a non-special node climbs through special causes
//     (weave-later? clause A, shared.cljc:208-212).  cw_dist_eff climbs while
//     the cause is local; a climb that leaves the run asks the owner of the
//     next cause (cw_dist_climb answers with its own local climb).
//   siblings: children of e, specials first, each class newest first
//     (shared.cljc:194-223).  Every rank sorts its (e, class) group keys and
//     links its local runs (cw_dist_runs); one record per run (its oldest and
//     newest node) goes to the owner of e, which orders the runs of every
//     group (cw_dist_link): the newest run's newest node is e's first child
//     of that class, each older run's newest node the next sibling of the
//     next run's oldest, and the oldest special's next sibling is e's newest
//     non-special.  The answers go back (cw_dist_put).
//   threads: thr(x) = next sibling of x, else thr(e(x)) -- the preorder
//     successor of a node without children.  cw_dist_thr resolves the chains
//     inside each 1,024-rank tile by pointer jumping in LDS (as k_gthr); a
//     chain that leaves the tile keeps THRW_PEND | the ancestor, and the walk
//     on the gathering GPU chases it through the gathered thread words (as
//     the single-GPU giant path does) -- no exchange rounds.
//
// cw_dist_succ then gives every node its successor (first child, or
// DIST_FROM_THR: its thread) and render bit, and the list ranking runs on one
// GPU (cw_weave_linked).

constexpr uint32_t DIST_PEND = 0x80000000u;  // eff: climb goes on at the rank in the low bits
constexpr uint32_t DIST_NONE = 0xFFFFFFFFu;  // eff of the root
constexpr uint32_t DIST_FROM_THR = 0x7FFFFFFEu;  // successor word: the node's thread
constexpr uint32_t FCS_HIDE = 0x80000000u;   // fcS word: the newest special child is a hide
constexpr uint32_t DIST_ROOT_KEY = 0xFFFFFFFFu;  // group key of the root: sorts last

__global__ __launch_bounds__(256) void k_dist_check(const uint32_t *__restrict__ par,
                                                    const uint8_t *__restrict__ kind, uint32_t n,
                                                    uint32_t base, uint32_t *__restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st = 0;
  if (i < n) {
    const uint32_t g = base + i;
    const bool root = (kind[i] & KIND_ROOT) != 0;
    if ((g == 0) != root) st |= CW_STATUS_ROOT;
    if (g > 0 && par[i] >= g) st |= par[i] >= CW_NIL_RANK ? CW_STATUS_ORPHAN : CW_STATUS_NON_LAMPORT;
  }
  if (__syncthreads_or(st != 0)) {
    if (st) atomicOr(status, st);
  }
}

// Climb from global rank c (local or not) through local special nodes: the
// first local non-special, or DIST_PEND | the first rank outside the run.
__device__ __forceinline__ uint32_t dist_climb(uint32_t c, const uint32_t *__restrict__ par,
                                               const uint8_t *__restrict__ kind, uint32_t n,
                                               uint32_t base) {
  for (uint32_t hop = 0; hop <= n; hop++) {
    if (c < base || c - base >= n) return DIST_PEND | c;
    if (!is_special(kind[c - base])) return c;
    const uint32_t p = par[c - base];
    if (p >= c) return 0;  // (out of domain: checked before; keeps the climb bounded)
    c = p;
  }
  return 0;
}

__global__ __launch_bounds__(256) void k_dist_eff(const uint32_t *__restrict__ par,
                                                  const uint8_t *__restrict__ kind, uint32_t n,
                                                  uint32_t base, uint32_t *__restrict__ eff) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (base + i == 0) {
    eff[i] = DIST_NONE;
    return;
  }
  eff[i] = is_special(kind[i]) ? par[i] : dist_climb(par[i], par, kind, n, base);
}

__global__ __launch_bounds__(256) void k_dist_climb(const uint32_t *__restrict__ par,
                                                    const uint8_t *__restrict__ kind, uint32_t n,
                                                    uint32_t base, const uint64_t *__restrict__ q,
                                                    uint32_t m, uint32_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = dist_climb((uint32_t)q[i], par, kind, n, base);
}

// Partition keys of the eff words still waiting on another rank (UINT64_MAX:
// none), and their number.
__global__ __launch_bounds__(256) void k_dist_pending(const uint32_t *__restrict__ w, uint32_t n,
                                                      uint64_t *__restrict__ keys,
                                                      uint32_t *__restrict__ count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool pend = false;
  if (i < n) {
    const uint32_t x = w[i];
    pend = (x & DIST_PEND) && x != DIST_NONE;
    keys[i] = pend ? (uint64_t)(x & ~DIST_PEND) : ~0ull;
  }
  const uint64_t b = __ballot(pend);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (uint32_t)__popcll(b));
}

// Group keys (e << 1 | class; special = 0; e < 2^31 - 1) for the local sort;
// the root last.
__global__ __launch_bounds__(256) void k_dist_gkey(const uint32_t *__restrict__ eff,
                                                   const uint8_t *__restrict__ kind, uint32_t n,
                                                   uint32_t *__restrict__ key) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = eff[i];
  key[i] = e == DIST_NONE ? DIST_ROOT_KEY : ((e << 1) | (is_special(kind[i]) ? 0u : 1u));
}

// Runs of equal group keys in the locally sorted order: inside a run each node's
// next sibling is the next older node; a run's oldest node waits for the owner
// of e (record: group, oldest, newest, kind of the newest; key = e for the
// partition by owner, UINT64_MAX on the other positions).
__global__ __launch_bounds__(256) void k_dist_runs(const uint32_t *__restrict__ skey,
                                                   const uint32_t *__restrict__ sidx, uint32_t n,
                                                   uint32_t base, const uint8_t *__restrict__ kind,
                                                   uint32_t *__restrict__ nsc,
                                                   uint64_t *__restrict__ okey,
                                                   uint4 *__restrict__ rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = skey[i];
  okey[i] = ~0ull;
  const uint32_t x = sidx[i];
  if (k == DIST_ROOT_KEY) {  // the root: no siblings
    nsc[x] = 0;
    return;
  }
  if (i > 0 && skey[i - 1] == k) {
    nsc[x] = base + sidx[i - 1];
    return;
  }
  // the run's end (first position with a larger key): runs are short, so
  // gallop from here, then bisect
  uint32_t lo = i + 1, step = 1;
  while (lo < n && skey[lo] == k) {
    lo = i + 1 + step;
    step <<= 1;
  }
  uint32_t hi = min(lo, n);
  lo = i + 1 + (step >> 2);
  if (lo > hi) lo = hi;
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if (skey[mid] <= k) lo = mid + 1; else hi = mid;
  }
  const uint32_t newest = sidx[lo - 1];
  nsc[x] = NSC_UP | (k >> 1);  // placeholder until the owner answers
  okey[i] = k >> 1;
  rec[i] = make_uint4(k, base + x, base + newest, kind[newest]);
}

// At the owner of e: a stable sort by group of the records as received (in
// sender order, i.e. by rank run) orders every group's runs by their oldest.
__global__ __launch_bounds__(256) void k_dist_rkey(const uint4 *__restrict__ rec, uint32_t m,
                                                   uint32_t *__restrict__ key) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key[i] = rec[i].x;
}

__global__ __launch_bounds__(256) void k_dist_link(const uint32_t *__restrict__ skey,
                                                   const uint32_t *__restrict__ sidx, uint32_t m,
                                                   const uint4 *__restrict__ rec, uint32_t base,
                                                   uint32_t n, uint32_t *__restrict__ fcS,
                                                   uint32_t *__restrict__ fcN,
                                                   uint32_t *__restrict__ reply) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t g = skey[j], e = g >> 1;
  const uint4 r = rec[sidx[j]];
  const bool first = j == 0 || skey[j - 1] != g;
  const bool last = j + 1 == m || skey[j + 1] != g;
  uint32_t ns = NSC_UP | e;
  if (!first) {
    ns = rec[sidx[j - 1]].z;
  } else if (!(g & 1)) {  // the oldest special: e's newest non-special follows the specials
    const uint64_t want = (uint64_t)(g | 1u) + 1;  // first key of the next group
    uint32_t lo = j, hi = m;
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      if (skey[mid] < want) lo = mid + 1; else hi = mid;
    }
    if (lo > 0 && skey[lo - 1] == (g | 1u)) ns = rec[sidx[lo - 1]].z;
  }
  reply[sidx[j]] = ns;
  if (last && e >= base && e - base < n) {
    if (g & 1) fcN[e - base] = r.z;
    else fcS[e - base] = r.z | (is_hide((uint8_t)r.w) ? FCS_HIDE : 0u);
  }
}

__global__ __launch_bounds__(256) void k_dist_put(const uint4 *__restrict__ rec,
                                                  const uint32_t *__restrict__ reply, uint32_t m,
                                                  uint32_t base, uint32_t n,
                                                  uint32_t *__restrict__ nsc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t x = rec[i].y - base;
  if (x < n) nsc[x] = reply[i];
}

// Thread words of one 1,024-rank tile of the run: resolved successor, or
// THRW_PEND | an ancestor outside the tile (chased by the walk); pointer
// jumping in LDS as k_gthr (pointers go to lower ranks).
template <int NT, int TT>
__global__ __launch_bounds__(NT) void k_dist_thr(const uint32_t *__restrict__ nsc, uint32_t n,
                                                 uint32_t base, uint32_t *__restrict__ thr) {
  constexpr uint32_t IT = TT / NT;
  constexpr uint64_t RES = 1ull << 63, OUT = 1ull << 62;
  __shared__ uint64_t T[TT];
  const uint32_t r0 = blockIdx.x * TT, tid = threadIdx.x, len = min((uint32_t)TT, n - r0);
  const uint32_t g0 = base + r0;
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = k * NT + tid;
    if (j >= len) continue;
    const uint32_t s = nsc[r0 + j], g = g0 + j;
    uint64_t tv;
    if (g == 0) tv = RES | SUCCW_END;
    else if (!(s & NSC_UP)) tv = RES | s;
    else {
      const uint32_t e = s & ~NSC_UP;
      tv = e >= g0 ? (e < g ? (uint64_t)(e - g0) : (RES | SUCCW_END)) : (OUT | e);
    }
    T[j] = tv;
  }
  __syncthreads();
  for (;;) {
    bool open = false;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid;
      if (j < len) {
        const uint64_t a = T[j];
        if (!(a & (RES | OUT))) {
          const uint64_t b = T[(uint32_t)a];
          T[j] = b;
          open |= !(b & (RES | OUT));
        }
      }
    }
    if (!__syncthreads_or(open)) break;
  }
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = k * NT + tid;
    if (j >= len) continue;
    const uint64_t a = T[j];
    thr[r0 + j] = (a & RES) ? (uint32_t)a : (THRW_PEND | (uint32_t)a);
  }
}

// Successor (first child -- the newest special, else the newest non-special --
// else the thread) and render bit of every node of the run.
__global__ __launch_bounds__(256) void k_dist_succ(const uint8_t *__restrict__ kind,
                                                   const uint32_t *__restrict__ fcS,
                                                   const uint32_t *__restrict__ fcN, uint32_t n,
                                                   uint32_t base, uint32_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t fs = fcS[i], fn = fcN[i];
  const uint32_t succ = (fs & ~FCS_HIDE) ? (fs & ~FCS_HIDE) : fn ? fn : DIST_FROM_THR;
  const bool vis = !is_special(kind[i]) && base + i != 0 && !(fs && (fs & FCS_HIDE));
  out[i] = succ | (vis ? LINK_VIS : 0u);
}

// cw_weave_linked: link words for the giant walk from successor | render bit
// and the thread words (a successor that is a pending thread: LINK_PEND, the
// walk chases it through thr).
__global__ __launch_bounds__(256) void k_linked_words(const uint32_t *__restrict__ sv,
                                                      const uint32_t *__restrict__ th,
                                                      const uint32_t *__restrict__ val, uint32_t n,
                                                      uint64_t *__restrict__ link,
                                                      uint32_t *__restrict__ thr) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t w = sv[r], t = th[r];
  uint32_t succ = w & ~LINK_VIS;
  bool pend = false;
  if (succ == DIST_FROM_THR) {
    succ = t & ~THRW_PEND;
    pend = (t & THRW_PEND) != 0;
  }
  link[r] = wide_link(succ < n ? succ : SUCCW_END, pend, val ? val[r] : r, (w & LINK_VIS) != 0);
  thr[r] = (t & THRW_PEND) ? t : (t < n ? t : SUCCW_END);
}

// ---- Ruling-set list ranking over the ranks ------------------
// The preorder list crosses ranks at ~42% of its steps (W = 8), so it is
// ranked where it lies: rulers (global rank 0, and every node whose hash falls
// under 2^32 / K) start one walker each; a walker numbers the nodes it visits
// (own = {ruler, offset}) until it reaches the next ruler or the list's end
// (a link {ruler, next ruler, length}), and hops to another rank as a message
// {ruler, count, target} whenever the list does.  The links -- one per ruler
// -- are ranked on one GPU (k_rs_jump), and every node's weave position is
// its ruler's position + its offset.
constexpr uint32_t RS_CHASE = 0x80000000u;  // next word / target: follow this node's thread
constexpr uint32_t RS_NONE = 0xFFFFFFFFu;   // word.y of a non-ruler; link: the list ends

__device__ __forceinline__ bool rs_is_ruler(uint32_t g, uint32_t k, uint32_t seed) {
  return g == 0 || (uint64_t)mix32(seed, g) * k < (1ull << 32);
}

// Pass 1 of the ruler numbering: in-block exclusive count (parked in word.y)
// and the block's total.
__global__ __launch_bounds__(1024) void k_rs_flag(uint32_t n, uint32_t base, uint32_t k,
                                                  uint32_t seed, uint2 *__restrict__ word,
                                                  uint32_t *__restrict__ sums) {
  __shared__ uint32_t wtot[16];
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t f = i < n && rs_is_ruler(base + i, k, seed) ? 1u : 0u;
  uint32_t tot;
  const uint32_t ex = block_exscan<1024>(f, wtot, &tot);
  if (i < n) word[i].y = ex;
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Pass 2: word = {next, ruler index or RS_NONE}; next = the successor, the
// resolved thread, RS_CHASE | the ancestor whose thread it is, or SUCCW_END.
__global__ __launch_bounds__(1024) void k_rs_index(const uint32_t *__restrict__ succ,
                                                   const uint32_t *__restrict__ thr, uint32_t n,
                                                   uint32_t base, uint32_t k, uint32_t seed,
                                                   const uint32_t *__restrict__ sums,
                                                   uint2 *__restrict__ word,
                                                   uint32_t *__restrict__ rlist) {
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  if (i >= n) return;
  uint32_t nx = succ[i] & ~LINK_VIS;
  if (nx == DIST_FROM_THR) {
    const uint32_t t = thr[i];
    nx = (t & THRW_PEND) ? (RS_CHASE | (t & ~THRW_PEND)) : t;
  }
  uint32_t r = RS_NONE;
  if (rs_is_ruler(base + i, k, seed)) {
    r = word[i].y + sums[blockIdx.x];
    rlist[r] = i;
  }
  word[i] = make_uint2(nx, r);
}

// One launch per exchange round: walker i (walkers == NULL: the run's ruler
// i, starting) walks while its list stays on this rank.  Messages: out[i] =
// {ruler, count, target, 0} with key[i] = the target's global rank (for the
// partition by owner), UINT64_MAX when walker i stopped here.
__global__ __launch_bounds__(256) void k_rs_walk(const uint4 *__restrict__ wk, uint32_t m,
                                                 const uint32_t *__restrict__ rlist, uint32_t rbase,
                                                 const uint2 *__restrict__ word,
                                                 const uint32_t *__restrict__ thr, uint32_t n,
                                                 uint32_t base, uint2 *__restrict__ own,
                                                 uint4 *__restrict__ links,
                                                 uint32_t *__restrict__ nlinks,
                                                 uint4 *__restrict__ out,
                                                 uint64_t *__restrict__ key,
                                                 uint32_t *__restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  uint32_t R, cnt, tgt;
  if (wk) {
    const uint4 w = wk[i];
    R = w.x;
    cnt = w.y;
    tgt = w.z;
  } else {
    R = rbase + i;
    cnt = 0;
    tgt = base + rlist[i];
  }
  uint64_t kk = ~0ull;
  bool link = false, bad = false;
  uint32_t lnext = RS_NONE;
  // every step numbers a node of the run or climbs to an older ancestor
  // (threads point to lower ranks): 2n + 2 steps bound a valid walk
  for (uint32_t hop = 0;; hop++) {
    if (hop > 2 * n + 2) {
      bad = true;
      break;
    }
    const uint32_t a = tgt & ~RS_CHASE;
    if (a - base >= n) {  // another rank's node (a < base wraps)
      kk = a;
      break;
    }
    uint32_t nx;
    if (tgt & RS_CHASE) {
      const uint32_t t = thr[a - base];
      nx = (t & THRW_PEND) ? (RS_CHASE | (t & ~THRW_PEND)) : t;
    } else {
      const uint2 wd = word[a - base];
      if (wd.y != RS_NONE && cnt > 0) {  // the next ruler: this sublist ends
        link = true;
        lnext = rbase + wd.y;
        break;
      }
      own[a - base] = make_uint2(R, cnt);
      cnt++;
      nx = wd.x;
    }
    if (nx == SUCCW_END) {
      link = true;
      break;
    }
    tgt = nx;
  }
  key[i] = kk;
  out[i] = make_uint4(R, cnt, tgt, 0u);
  if (bad) atomicOr(status, CW_STATUS_INTERNAL);
  // links appended with one atomic per wave
  const uint64_t b = __ballot(link);
  if (b) {
    const uint32_t lane = threadIdx.x & 63, lead = (uint32_t)__ffsll((long long)b) - 1;
    uint32_t s0 = 0;
    if (lane == lead) s0 = atomicAdd(nlinks, (uint32_t)__popcll(b));
    s0 = __shfl(s0, lead, 64);
    if (link) links[s0 + lanes_below(b)] = make_uint4(R, lnext, cnt, 0u);
  }
}

// The ruler list on one GPU: A[r] = {next ruler, length} from the links.
__global__ __launch_bounds__(256) void k_rs_links(const uint4 *__restrict__ links, uint32_t m,
                                                  uint2 *__restrict__ A) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint4 l = links[j];
  if (l.x < m) A[l.x] = make_uint2(l.y, l.z);
}

// One pointer-jumping round: {next, nodes from here to the end}.
__global__ __launch_bounds__(256) void k_rs_jump(const uint2 *__restrict__ A, uint32_t m,
                                                 uint2 *__restrict__ B) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint2 v = A[j];
  if (v.x < m) {
    const uint2 w = A[v.x];
    B[j] = make_uint2(w.x, v.y + w.y);
  } else {
    B[j] = make_uint2(RS_NONE, v.y);
  }
}

// Large ruler lists rank in two levels: sub-rulers (ruler 0 and ~1/16 of the
// rest, by hash) walk their stretch of the ruler list summing lengths, the
// sub-ruler list is pointer-jumped, and each ruler's position is its
// sub-ruler's plus its offset.  R4[r] = {next, length, sub-ruler index or
// RS_NONE, 0}.
constexpr uint32_t RS_TOP_DIRECT = 1u << 21;  // rulers ranked by pointer jumping alone
constexpr uint32_t RS_SUB_K = 16;
constexpr uint32_t RS_SUB_SEED = 0x68E31DA4u;

__global__ __launch_bounds__(256) void k_rs_links4(const uint4 *__restrict__ links, uint32_t m,
                                                   uint4 *__restrict__ R4) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint4 l = links[j];
  if (l.x < m) R4[l.x] = make_uint4(l.y, l.z, 0u, 0u);
}

__global__ __launch_bounds__(1024) void k_rs_tflag(uint32_t m, uint4 *__restrict__ R4,
                                                   uint32_t *__restrict__ sums) {
  __shared__ uint32_t wtot[16];
  const uint32_t r = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t f = r < m && rs_is_ruler(r, RS_SUB_K, RS_SUB_SEED) ? 1u : 0u;
  uint32_t tot;
  const uint32_t ex = block_exscan<1024>(f, wtot, &tot);
  if (r < m) R4[r].z = ex;
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_rs_tindex(uint32_t m, const uint32_t *__restrict__ sums,
                                                    uint4 *__restrict__ R4,
                                                    uint32_t *__restrict__ slist) {
  const uint32_t r = blockIdx.x * 1024 + threadIdx.x;
  if (r >= m) return;
  uint32_t s = RS_NONE;
  if (rs_is_ruler(r, RS_SUB_K, RS_SUB_SEED)) {
    s = R4[r].z + sums[blockIdx.x];
    slist[s] = r;
  }
  R4[r].z = s;
}

// Sub-ruler j walks the ruler list to the next sub-ruler: own2[r] = {j,
// nodes before r in the stretch}; A2[j] = {next sub-ruler, nodes}.
__global__ __launch_bounds__(256) void k_rs_twalk(const uint32_t *__restrict__ slist, uint32_t m2,
                                                  const uint4 *__restrict__ R4, uint32_t m,
                                                  uint2 *__restrict__ own2,
                                                  uint2 *__restrict__ A2,
                                                  uint32_t *__restrict__ status) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m2) return;
  uint32_t r = slist[j], sum = 0, nx2 = RS_NONE;
  for (uint32_t hop = 0;; hop++) {
    const uint4 v = R4[r];
    if (hop > 0 && v.z != RS_NONE) {
      nx2 = v.z;
      break;
    }
    if (hop > m) {
      atomicOr(status, CW_STATUS_INTERNAL);
      break;
    }
    own2[r] = make_uint2(j, sum);
    sum += v.y;
    if (v.x >= m) break;
    r = v.x;
  }
  A2[j] = make_uint2(nx2, sum);
}

__global__ __launch_bounds__(256) void k_rs_tpos(const uint2 *__restrict__ own2, uint32_t m,
                                                 const uint2 *__restrict__ A2, uint32_t m2,
                                                 uint32_t total, uint32_t *__restrict__ pos,
                                                 uint32_t *__restrict__ status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  const uint2 o = own2[r];
  if (o.x >= m2) {  // a ruler no sub-ruler reached (a broken list)
    pos[r] = 0;
    atomicOr(status, CW_STATUS_INTERNAL);
    return;
  }
  pos[r] = total - A2[o.x].y + o.y;
  if (r == 0 && (A2[0].y != total || A2[0].x != RS_NONE)) atomicOr(status, CW_STATUS_INTERNAL);
}

__global__ __launch_bounds__(256) void k_rs_base(const uint2 *__restrict__ A, uint32_t m,
                                                 uint32_t total, uint32_t *__restrict__ pos,
                                                 uint32_t *__restrict__ status) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint2 v = A[j];
  pos[j] = total - v.y;
  // one list from ruler 0 over every node, and every walk ran to the end
  if (j == 0 && (v.y != total || v.x != RS_NONE)) atomicOr(status, CW_STATUS_INTERNAL);
}

// Weave position of each node of the run and its emit record {position,
// val | render << 31}; key = the position (for an emit spread by position).
__global__ __launch_bounds__(256) void k_rs_pos(const uint2 *__restrict__ own,
                                                const uint32_t *__restrict__ pbase,
                                                const uint32_t *__restrict__ succ,
                                                const uint32_t *__restrict__ val, uint32_t n,
                                                uint2 *__restrict__ rec,
                                                uint64_t *__restrict__ key) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint2 o = own[i];
  const uint32_t p = pbase[o.x] + o.y;
  rec[i] = make_uint2(p, (val[i] & 0x7FFFFFFFu) | (succ[i] & LINK_VIS));
  if (key) key[i] = p;
}

// At the owner of positions [p0, p0 + len): weave_perm and the render bytes;
// one count atomic per block (grid-stride over a fixed grid).
__global__ __launch_bounds__(256) void k_rs_emit(const uint2 *__restrict__ rec, uint32_t m,
                                                 uint32_t p0, uint32_t len,
                                                 uint32_t *__restrict__ perm,
                                                 uint8_t *__restrict__ vis8,
                                                 uint32_t *__restrict__ count,
                                                 uint32_t *__restrict__ status) {
  __shared__ uint32_t wsum[4];
  uint32_t c = 0;
  bool bad = false;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
    const uint2 r = rec[j];
    const uint32_t p = r.x - p0;
    if (p >= len) {
      bad = true;
      continue;
    }
    perm[p] = r.y & 0x7FFFFFFFu;
    vis8[p] = (uint8_t)(r.y >> 31);
    c += r.y >> 31;
  }
  if (bad) atomicOr(status, CW_STATUS_INTERNAL);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t) atomicAdd(count, t);
  }
}

int dist_launch_ok(cw_ctx *c, const char *nm) { return check_launch(c, nm); }

#define DIST_GRID(m) dim3((uint32_t)(((m) + 255) / 256)), dim3(256), 0, c->stream

int dist_check_impl(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                    uint32_t *status) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_dist_check, DIST_GRID(n), par, kind, (uint32_t)n, base, status);
  return dist_launch_ok(c, "dist_check");
}

int dist_eff_impl(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                  uint32_t *eff) {
  if (!n) return 0;
  Launch L(c, "dist_eff", (double)n * (4 + 1 + 4));
  hipLaunchKernelGGL(k_dist_eff, DIST_GRID(n), par, kind, (uint32_t)n, base, eff);
  return dist_launch_ok(c, "dist_eff");
}

int dist_climb_impl(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                    const uint64_t *q, uint64_t m, uint32_t *out) {
  if (!m) return 0;
  hipLaunchKernelGGL(k_dist_climb, DIST_GRID(m), par, kind, (uint32_t)n, base, q, (uint32_t)m, out);
  return dist_launch_ok(c, "dist_climb");
}

int dist_pending_impl(cw_ctx *c, const uint32_t *w, uint64_t n, uint64_t *keys, uint32_t *count) {
  HIPCHK(c, hipMemsetAsync(count, 0, 4, c->stream));
  if (!n) return 0;
  hipLaunchKernelGGL(k_dist_pending, DIST_GRID(n), w, (uint32_t)n, keys, count);
  return dist_launch_ok(c, "dist_pending");
}

int dist_gkey_impl(cw_ctx *c, const uint32_t *eff, const uint8_t *kind, uint64_t n, uint32_t *key) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_dist_gkey, DIST_GRID(n), eff, kind, (uint32_t)n, key);
  return dist_launch_ok(c, "dist_gkey");
}

int dist_runs_impl(cw_ctx *c, const uint32_t *skey, const uint32_t *sidx, uint64_t n, uint32_t base,
                   const uint8_t *kind, uint32_t *nsc, uint64_t *okey, uint32_t *rec) {
  if (!n) return 0;
  Launch L(c, "dist_runs", (double)n * (8 + 4 + 4 + 8) + (double)n * 0.4 * 16);
  hipLaunchKernelGGL(k_dist_runs, DIST_GRID(n), skey, sidx, (uint32_t)n, base, kind, nsc, okey,
                     reinterpret_cast<uint4 *>(rec));
  return dist_launch_ok(c, "dist_runs");
}

int dist_rkey_impl(cw_ctx *c, const uint32_t *rec, uint64_t m, uint32_t *key) {
  if (!m) return 0;
  hipLaunchKernelGGL(k_dist_rkey, DIST_GRID(m), reinterpret_cast<const uint4 *>(rec), (uint32_t)m, key);
  return dist_launch_ok(c, "dist_rkey");
}

int dist_link_impl(cw_ctx *c, const uint32_t *skey, const uint32_t *sidx, uint64_t m,
                   const uint32_t *rec, uint32_t base, uint64_t n, uint32_t *fcS, uint32_t *fcN,
                   uint32_t *reply) {
  if (!m) return 0;
  Launch L(c, "dist_link", (double)m * (8 + 4 + 16 + 4 + 4));
  hipLaunchKernelGGL(k_dist_link, DIST_GRID(m), skey, sidx, (uint32_t)m,
                     reinterpret_cast<const uint4 *>(rec), base, (uint32_t)n, fcS, fcN, reply);
  return dist_launch_ok(c, "dist_link");
}

int dist_put_impl(cw_ctx *c, const uint32_t *rec, const uint32_t *reply, uint64_t m, uint32_t base,
                  uint64_t n, uint32_t *nsc) {
  if (!m) return 0;
  hipLaunchKernelGGL(k_dist_put, DIST_GRID(m), reinterpret_cast<const uint4 *>(rec), reply,
                     (uint32_t)m, base, (uint32_t)n, nsc);
  return dist_launch_ok(c, "dist_put");
}

int dist_thr_impl(cw_ctx *c, const uint32_t *nsc, uint64_t n, uint32_t base, uint32_t *thr) {
  if (!n) return 0;
  Launch L(c, "dist_thr", (double)n * (4 + 4));
  hipLaunchKernelGGL((k_dist_thr<256, 1024>), dim3((uint32_t)((n + 1023) / 1024)), dim3(256), 0,
                     c->stream, nsc, (uint32_t)n, base, thr);
  return dist_launch_ok(c, "dist_thr");
}

int dist_succ_impl(cw_ctx *c, const uint8_t *kind, const uint32_t *fcS, const uint32_t *fcN,
                   uint64_t n, uint32_t base, uint32_t *out) {
  if (!n) return 0;
  Launch L(c, "dist_succ", (double)n * (1 + 4 + 4 + 4));
  hipLaunchKernelGGL(k_dist_succ, DIST_GRID(n), kind, fcS, fcN, (uint32_t)n, base, out);
  return dist_launch_ok(c, "dist_succ");
}

int dist_rs_rulers_impl(cw_ctx *c, const uint32_t *succ, const uint32_t *thr, uint64_t n,
                        uint32_t base, uint32_t k, uint32_t seed, uint32_t *word, uint32_t *rlist,
                        uint32_t *count) {
  if (k == 0) return fail(c, "rs_rulers: k >= 1");
  if (!n) {
    HIPCHK(c, hipMemsetAsync(count, 0, 4, c->stream));
    return 0;
  }
  const uint32_t nb = (uint32_t)((n + 1023) / 1024);
  uint32_t *sums = scratch_t<uint32_t>(c, "rs_sums", (size_t)nb + 1);
  if (!sums) return fail(c, "out of device memory (rs_rulers)");
  uint2 *w2 = reinterpret_cast<uint2 *>(word);
  Launch L(c, "rs_rulers", (double)n * (4 + 4 + 8 + 8 + 4.0 / k));
  hipLaunchKernelGGL(k_rs_flag, dim3(nb), dim3(1024), 0, c->stream, (uint32_t)n, base, k, seed, w2,
                     sums);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, c->stream, sums, nb, sums + nb);
  hipLaunchKernelGGL(k_rs_index, dim3(nb), dim3(1024), 0, c->stream, succ, thr, (uint32_t)n, base,
                     k, seed, sums, w2, rlist);
  HIPCHK(c, hipMemcpyAsync(count, sums + nb, 4, hipMemcpyDeviceToDevice, c->stream));
  return dist_launch_ok(c, "rs_rulers");
}

int dist_rs_walk_impl(cw_ctx *c, const uint32_t *walkers, uint64_t m, const uint32_t *rlist,
                      uint32_t rbase, const uint32_t *word, const uint32_t *thr, uint64_t n,
                      uint32_t base, uint32_t *own, uint32_t *links, uint32_t *nlinks,
                      uint32_t *out, uint64_t *key, uint32_t *status) {
  if (!m) return 0;
  if (!walkers && !rlist) return fail(c, "rs_walk: walkers or rlist");
  Launch L(c, "rs_walk", (double)m * (16 + 16 + 8) + (double)n * (8 + 8));
  hipLaunchKernelGGL(k_rs_walk, DIST_GRID(m), reinterpret_cast<const uint4 *>(walkers), (uint32_t)m,
                     rlist, rbase, reinterpret_cast<const uint2 *>(word), thr, (uint32_t)n, base,
                     reinterpret_cast<uint2 *>(own), reinterpret_cast<uint4 *>(links), nlinks,
                     reinterpret_cast<uint4 *>(out), key, status);
  return dist_launch_ok(c, "rs_walk");
}

int dist_rs_top_impl(cw_ctx *c, const uint32_t *links, uint64_t m, uint64_t total, uint32_t *pos,
                     uint32_t *status) {
  if (!m) return 0;
  if (m >= RS_NONE || total >= SUCCW_END) return fail(c, "rs_top: sizes");
  if (m <= RS_TOP_DIRECT) {
    uint2 *A = scratch_t<uint2>(c, "rs_a", m), *B = scratch_t<uint2>(c, "rs_b", m);
    if (!A || !B) return fail(c, "out of device memory (rs_top, m=%llu)", (unsigned long long)m);
    // a ruler without a link (a broken walk) points past the end with no length
    HIPCHK(c, hipMemsetAsync(A, 0xFF, m * sizeof(uint2), c->stream));
    uint32_t rounds = 0;
    while ((1ull << rounds) < m) rounds++;
    Launch L(c, "rs_top", (double)m * (16 + 8) + (double)rounds * m * (8 + 8 + 8) + (double)m * 12);
    hipLaunchKernelGGL(k_rs_links, DIST_GRID(m), reinterpret_cast<const uint4 *>(links),
                       (uint32_t)m, A);
    for (uint32_t r = 0; r < rounds; r++) {
      hipLaunchKernelGGL(k_rs_jump, DIST_GRID(m), A, (uint32_t)m, B);
      std::swap(A, B);
    }
    hipLaunchKernelGGL(k_rs_base, DIST_GRID(m), A, (uint32_t)m, (uint32_t)total, pos, status);
    return dist_launch_ok(c, "rs_top");
  }
  // two levels: sub-rulers walk the ruler list, the sub-ruler list is jumped
  const uint32_t nb = (uint32_t)((m + 1023) / 1024);
  uint4 *R4 = scratch_t<uint4>(c, "rs_r4", m);
  uint2 *own2 = scratch_t<uint2>(c, "rs_own2", m);
  uint32_t *sums = scratch_t<uint32_t>(c, "rs_sums", (size_t)nb + 1);
  uint32_t *slist = scratch_t<uint32_t>(c, "rs_slist", m);
  if (!R4 || !own2 || !sums || !slist)
    return fail(c, "out of device memory (rs_top, m=%llu)", (unsigned long long)m);
  HIPCHK(c, hipMemsetAsync(R4, 0xFF, m * sizeof(uint4), c->stream));
  HIPCHK(c, hipMemsetAsync(own2, 0xFF, m * sizeof(uint2), c->stream));
  hipLaunchKernelGGL(k_rs_links4, DIST_GRID(m), reinterpret_cast<const uint4 *>(links),
                     (uint32_t)m, R4);
  hipLaunchKernelGGL(k_rs_tflag, dim3(nb), dim3(1024), 0, c->stream, (uint32_t)m, R4, sums);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, c->stream, sums, nb, sums + nb);
  hipLaunchKernelGGL(k_rs_tindex, dim3(nb), dim3(1024), 0, c->stream, (uint32_t)m, sums, R4, slist);
  uint32_t m2 = 0;
  HIPCHK(c, hipMemcpyAsync(&m2, sums + nb, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (m2 == 0 || m2 > m) return fail(c, "rs_top: %u sub-rulers", m2);
  uint2 *A = scratch_t<uint2>(c, "rs_a", m2), *B = scratch_t<uint2>(c, "rs_b", m2);
  if (!A || !B) return fail(c, "out of device memory (rs_top, m2=%u)", m2);
  uint32_t rounds = 0;
  while ((1ull << rounds) < m2) rounds++;
  Launch L(c, "rs_top", (double)m * (16 + 16 + 16 + 8 + 8 + 12) + (double)rounds * m2 * 24);
  hipLaunchKernelGGL(k_rs_twalk, DIST_GRID(m2), slist, m2, R4, (uint32_t)m, own2, A, status);
  for (uint32_t r = 0; r < rounds; r++) {
    hipLaunchKernelGGL(k_rs_jump, DIST_GRID(m2), A, m2, B);
    std::swap(A, B);
  }
  hipLaunchKernelGGL(k_rs_tpos, DIST_GRID(m), own2, (uint32_t)m, A, m2, (uint32_t)total, pos,
                     status);
  return dist_launch_ok(c, "rs_top");
}

int dist_rs_pos_impl(cw_ctx *c, const uint32_t *own, const uint32_t *pbase, const uint32_t *succ,
                     const uint32_t *val, uint64_t n, uint32_t *rec, uint64_t *key) {
  if (!n) return 0;
  Launch L(c, "rs_pos", (double)n * (8 + 4 + 4 + 4 + 8 + (key ? 8 : 0)));
  hipLaunchKernelGGL(k_rs_pos, DIST_GRID(n), reinterpret_cast<const uint2 *>(own), pbase, succ, val,
                     (uint32_t)n, reinterpret_cast<uint2 *>(rec), key);
  return dist_launch_ok(c, "rs_pos");
}

int dist_rs_emit_impl(cw_ctx *c, const uint32_t *rec, uint64_t m, uint32_t p0, uint64_t len,
                      uint32_t *perm, uint32_t *bits, uint32_t *count, uint32_t *status) {
  HIPCHK(c, hipMemsetAsync(count, 0, 4, c->stream));
  if (!len) return 0;
  uint8_t *vis8 = scratch_t<uint8_t>(c, "rs_vis", (size_t)len + 32);
  if (!vis8) return fail(c, "out of device memory (rs_emit)");
  Launch L(c, "rs_emit", (double)m * (8 + 4 + 1) + (double)len * (1 + 0.125));
  if (m) {
    const uint32_t nb = (uint32_t)std::min<uint64_t>((m + 255) / 256, 2048);
    hipLaunchKernelGGL(k_rs_emit, dim3(nb), dim3(256), 0, c->stream,
                       reinterpret_cast<const uint2 *>(rec), (uint32_t)m, p0, (uint32_t)len, perm,
                       vis8, count, status);
  }
  hipLaunchKernelGGL(k_pack_bits, dim3((uint32_t)((len + 31) / 32 + 255) / 256), dim3(256), 0,
                     c->stream, vis8, (uint32_t)len, bits);
  return dist_launch_ok(c, "rs_emit");
}

// The walk, ranking and emit of one list given every node's successor.
int weave_linked_impl(cw_ctx *c, const cw_linked_list *in, cw_list_result *out) {
  if (!in || !out) return fail(c, "null list/result");
  if (!out->weave_perm || !out->visible_count || !out->status)
    return fail(c, "weave_perm, visible_count and status are required");
  if (out->yarn_perm || out->max_ts) return fail(c, "yarn_perm / max_ts: not produced from links");
  const uint64_t n64 = in->n;
  if (n64 == 0 || n64 >= SUCCW_END) return fail(c, "list size %llu (1 .. 2^31-2)", (unsigned long long)n64);
  if (!in->succ || !in->thr) return fail(c, "null input arrays");
  const uint32_t n = (uint32_t)n64;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t off[2] = {0, n64};
  if (ensure_tables(c, 1, off, true)) return -1;
  HIPCHK(c, hipMemsetAsync(out->status, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(out->visible_count, 0, 4, c->stream));
  if (out->visible_bits)
    HIPCHK(c, hipMemsetAsync(out->visible_bits, 0, ((size_t)n + 31) / 32 * 4, c->stream));
  uint64_t *link = scratch_t<uint64_t>(c, "link", n);
  uint32_t *thr = scratch_t<uint32_t>(c, "thr", n);
  if (!link || !thr) return fail(c, "out of device memory (linked, n=%u)", n);
  {
    Launch L(c, "linked", (double)n * (4 + 4 + 8 + 4));
    hipLaunchKernelGGL(k_linked_words, DIST_GRID(n), in->succ, in->thr, in->val, n, link, thr);
  }
  if (dist_launch_ok(c, "linked")) return -1;
  if (weave_tail(c, 1, n, true, nullptr, nullptr, in->val, nullptr, nullptr, 0, out, nullptr, nullptr,
                 true))
    return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->prof) return collect_prof(c);
  return 0;
}

#undef DIST_GRID
