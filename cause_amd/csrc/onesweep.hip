// onesweep.hip -- one-pass-per-digit LSD radix sort of ONE array (included by
// causeweave.hip; the id sort of one giant list, list.cljc:28 / shared.cljc:128,
// and the giant tree's sort of cross-tile children).
//
// The histogram-scan-scatter sort (k_radix_hist / k_gscan_* / k_radix_scatter)
// reads the keys twice a pass and runs a chain of small scan launches between
// (config 5's 2e9 ids: hist 11.7 + scan 3.1 + scatter 80.8 ms).  Here a pass is
// k_os_hist (the pass input's digit counts), k_os_scan (bucket bases, one
// block) and k_os_pass: a tile of 8,192 keys is ranked by its digit inside LDS
// (one wave-ballot match of the whole digit, per-wave bucket counters),
// publishes its digit counts, learns the counts of the tiles before it by a
// decoupled look-back, and writes its digit runs out from LDS.
//
// Measured (round 6, 2e8 random 35-bit keys, 4 passes, timing switches
// CW_OS_EXP): the passes take 4.7 ms without the look-back and 7.7 ms with one
// chain over the whole array -- one chain's inclusive prefix advances OS_LBW
// tiles per agent-scope round trip (~1 us), and that rate, not the bytes,
// bounds the pass.  So the pass input is cut into OS_RANGES ranges of whole
// tiles, each its own look-back chain, with bucket bases per range (the keys of
// buckets < b, plus the keys of bucket b in ranges < x): 6.5 ms.  Per-range
// bases need each range's digit counts of the pass INPUT, which for every pass
// after the first is the previous pass's output, so every pass has its own
// histogram launch (a range's counts depend on where the previous pass put the
// keys).  Block b takes the next tile of range b % 8 from the range's ticket
// counter: a tile waits only on tiles of its range with smaller tickets, taken
// by workgroups already running, so the smallest unfinished tile of a range
// always finishes, wherever the blocks land.  (Lost on the way, round 6: one
// histogram launch for all passes with one chain -- exact, slower; per-XCD
// chains with bases from the first pass's histogram -- wrong after the first
// pass; persistent workgroups counting the next pass's digits while they write
// -- 8.2 ms, the LDS atomic a key and one workgroup a CU; 4,096-key tiles at two
// workgroups a CU -- 9.0 ms; the first look-back words loaded before the LDS
// scatter -- 7.0 ms, more second trips.)
//
// Look-back words (u64, one per tile and bucket): bit 63 = inclusive prefix,
// bit 62 = aggregate (this tile's count only), bits 32-47 = the pass's epoch
// (a word of an earlier pass reads as "not published": no clearing between
// passes), bits 0-31 = the count.  Relaxed agent-scope atomics: the word is the
// whole message, and the L2s of the XCDs are not coherent.

constexpr uint32_t OS_MAX_BITS = 9;                 // digit bits a pass (<= 512 buckets)
constexpr uint32_t OS_MAX_BINS = 1u << OS_MAX_BITS;
constexpr uint32_t OS_MAX_PASSES = 8;
constexpr unsigned long long OS_INC = 1ull << 63, OS_AGG = 1ull << 62;
constexpr uint32_t OS_LBW = 16;                     // look-back words read a round trip

struct OsDigits {  // the digits of every pass
  uint32_t passes;
  uint32_t shift[OS_MAX_PASSES], bits[OS_MAX_PASSES];
};

// Every pass's digit counts per range of the input: hist[(p * OS_RANGES + x) *
// OS_MAX_BINS + b] for the keys of range x = [x * rlen, (x + 1) * rlen) (one
// range, nr = 1, for the single-chain geometries CW_ONESWEEP = 1-3, which
// count every pass at once).  Block b counts range b % nr
// in spans of OS_HIST_ITEMS * 256 keys, grid-strided (rlen is a multiple of a
// span), and flushes once: a block per span flushed 512 atomics a span onto
// the same 512 words -- 9.3 ms at 2e9 keys, contention, not the LDS counting.
// Each wave counts into its own copy (dynamic LDS: 4 x passes x OS_MAX_BINS).
constexpr uint32_t OS_HIST_ITEMS = 16;
constexpr uint32_t OS_RANGES = 8;
template <typename K>
__global__ __launch_bounds__(256) void k_os_hist(const K *__restrict__ keys, uint32_t n, OsDigits dg,
                                                 uint32_t rlen, uint32_t nr, uint32_t *__restrict__ hist) {
  extern __shared__ uint32_t lds_osh[];
  constexpr uint32_t SPAN = 256 * OS_HIST_ITEMS;
  const uint32_t tid = threadIdx.x, w = tid >> 6, words = dg.passes * OS_MAX_BINS;
  for (uint32_t i = tid; i < 4 * words; i += 256) lds_osh[i] = 0;
  __syncthreads();
  uint32_t *const h = lds_osh + w * words;
  const uint32_t x = blockIdx.x % nr, per = gridDim.x / nr;
  const uint64_t r0 = (uint64_t)x * rlen, r1 = min<uint64_t>(n, r0 + rlen);
  for (uint64_t i0 = r0 + (uint64_t)(blockIdx.x / nr) * SPAN; i0 < r1; i0 += (uint64_t)per * SPAN) {
    K kk[OS_HIST_ITEMS];
#pragma unroll
    for (uint32_t k = 0; k < OS_HIST_ITEMS; k++) {
      const uint64_t i = i0 + k * 256 + tid;
      kk[k] = i < r1 ? keys[i] : (K)0;
    }
    for (uint32_t p = 0; p < dg.passes; p++) {
      const uint32_t sh = dg.shift[p], m = (1u << dg.bits[p]) - 1;
      uint32_t *const hp = h + p * OS_MAX_BINS;
#pragma unroll
      for (uint32_t k = 0; k < OS_HIST_ITEMS; k++)
        if (i0 + k * 256 + tid < r1) atomicAdd(&hp[(uint32_t)(kk[k] >> sh) & m], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < words; i += 256) {
    const uint32_t c = lds_osh[i] + lds_osh[words + i] + lds_osh[2 * words + i] + lds_osh[3 * words + i];
    const uint32_t p = i / OS_MAX_BINS, b = i % OS_MAX_BINS;
    if (c) atomicAdd(&hist[((size_t)p * OS_RANGES + x) * OS_MAX_BINS + b], c);
  }
}

// Bucket bases: base[(p * OS_RANGES + x) * OS_MAX_BINS + b] = the keys of every
// bucket < b (all ranges) + the keys of bucket b in ranges < x.  One block per
// pass, one thread per bucket.
__global__ __launch_bounds__(OS_MAX_BINS) void k_os_scan(const uint32_t *__restrict__ hist, OsDigits dg,
                                                         uint32_t *__restrict__ base) {
  __shared__ uint32_t wtot[OS_MAX_BINS / 64];
  const uint32_t p = blockIdx.x, b = threadIdx.x, nb = 1u << dg.bits[p];
  uint32_t c_in[OS_RANGES], tot = 0;
#pragma unroll
  for (uint32_t x = 0; x < OS_RANGES; x++) {
    c_in[x] = b < nb ? hist[((size_t)p * OS_RANGES + x) * OS_MAX_BINS + b] : 0u;
    tot += c_in[x];
  }
  uint32_t run = block_exscan<OS_MAX_BINS>(tot, wtot, nullptr);
#pragma unroll
  for (uint32_t x = 0; x < OS_RANGES; x++) {
    base[((size_t)p * OS_RANGES + x) * OS_MAX_BINS + b] = run;
    run += c_in[x];
  }
}

// A second value carried through the passes (PL): config 5's cause and kind.
// With kb = the sort's key bits (<= OS_PL_MAX_BITS) the cause is clamped to
// c' = min(cause, 2^kb) (2^kb: no id -- above every id of the sort), and
//   lo = c' & 0xFFFFFFFF           a u32 array beside the values,
//   hi = c' >> 32 | kind << CH     in the key's unused bits above kb,
// CH = max(kb, 32) - 31; the last pass writes the bare ids and hi into its own
// u32 array.  The first pass packs it from the inputs (cause, kind by element
// index); the id sort then leaves every rank's cause and kind in rank order,
// and the join reads them sequentially instead of gathering them by input
// index (round 6).  (A u64 payload a key cost 16 B a key and pass instead of
// 8: +6.9 ms over the passes of 2^29 keys.)  OS_PL_MAX_BITS, os_pl_ch:
// cw_internal.h.
struct OsPayload {
  const uint64_t *cause;  // the first pass's source (by element index)
  const uint8_t *kind;
  const uint32_t *lo_in;  // later passes' source
  uint32_t *lo_out;
  uint32_t *hi_out;       // the last pass: hi of every key, the keys written bare
  uint32_t *status;       // the first pass: CW_STATUS_INTERNAL for an id past kb bits
  uint32_t kb;
};

// One LSD pass.  NT threads, IT keys a thread (wave-blocked: wave w holds the
// tile's elements [w * IT * 64, (w + 1) * IT * 64)), digit = (key >> shift) &
// (2^dbits - 1), dbits <= OS_MAX_BITS, NT >= 2^dbits.  vals_in == nullptr: the
// value is the element's index.  keys_out == nullptr: values only.  inv: also
// inv[value] = the element's sorted position (the last pass of a sort whose
// values are input indices).  PL: the payload above, staged through the key
// buffer after the keys are out.  PLM (the payload's role in this pass, each a
// kernel of its own so no pass carries another's code): 0 none, bit 1 carried
// (lo in and out), bit 2 the first pass (packed from cause / kind), bit 4 the
// last pass (bare ids, hi apart).
template <typename K, int NT, int IT, int PLM = 0>
__global__ __launch_bounds__(NT) void k_os_pass(
    const K *__restrict__ keys_in, const uint32_t *__restrict__ vals_in, K *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, uint32_t *__restrict__ inv, uint32_t n, uint32_t shift,
    uint32_t dbits, const uint32_t *__restrict__ base, unsigned long long *lb, uint32_t epoch,
    uint32_t exp, uint32_t tiles_per_range, uint32_t *__restrict__ ticket, OsPayload pl) {
  constexpr uint32_t TS = NT * IT, NW = NT / 64;
  constexpr bool PL = PLM != 0, PL_FIRST = (PLM & 2) != 0, PL_LAST = (PLM & 4) != 0;
  static_assert(!PL || sizeof(K) == 8, "hi rides in a u64 key");
  static_assert(NT >= OS_MAX_BINS, "one thread per bucket");
  const uint32_t EXPS = exp;
  __shared__ K skey[TS];
  __shared__ uint32_t sval[TS];
  __shared__ uint32_t cw[NW][OS_MAX_BINS];  // per wave: its count, then its offset inside the bucket
  __shared__ uint32_t bstart[OS_MAX_BINS];  // bucket start inside the tile
  __shared__ uint32_t goff[OS_MAX_BINS];    // output position of the tile's bucket start, minus bstart
  __shared__ uint32_t wtot[NW];
  __shared__ uint32_t s_li;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = 1u << dbits, dmask = nb - 1;
  // ranged (ticket != nullptr): block b takes the next tile of range b % 8 from
  // its ticket counter; otherwise tile = block, one range
  const uint32_t x = ticket ? blockIdx.x % OS_RANGES : 0u, Tr = tiles_per_range;
  if (ticket && tid == 0) s_li = atomicAdd(&ticket[x], 1u);
  for (uint32_t b = lane; b < OS_MAX_BINS; b += 64) cw[w][b] = 0;
  __syncthreads();
  const uint32_t li = ticket ? s_li : blockIdx.x;  // tile index inside the range
  const uint32_t g = x * Tr + li;                  // its look-back words
  const uint64_t s64 = (uint64_t)x * Tr * TS + (uint64_t)li * TS;
  const uint32_t s = (uint32_t)min<uint64_t>(s64, n), len = (uint32_t)min<uint64_t>(TS, n - s);
  const uint32_t *const bx = base + (size_t)x * OS_MAX_BINS;
  K key[IT];
  uint32_t val[IT], dig[IT], pin[IT];
  uint32_t pv[PL ? IT : 1];
  bool wide = false;  // (an id past kb bits: the caller's key_bits are wrong)
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = (w * IT + k) * 64 + lane;
    const bool v = j < len;
    key[k] = v ? keys_in[s + j] : (K)0;
    val[k] = v ? (vals_in ? vals_in[s + j] : s + j) : 0u;
    if (PL_FIRST) {
      const uint64_t c = v ? min(pl.cause[s + j], 1ull << pl.kb) : 0ull;
      const uint64_t kd = v ? pl.kind[s + j] : 0u;
      pv[k] = (uint32_t)c;
      wide |= (key[k] >> pl.kb) != 0;
      key[k] = (key[k] & ((1ull << pl.kb) - 1)) | ((c >> 32) | kd << os_pl_ch(pl.kb)) << pl.kb;
    } else if (PL) {
      pv[k] = v ? pl.lo_in[s + j] : 0u;
    }
  }
  if (PL_FIRST && __ballot(wide) && lane == 0) atomicOr(pl.status, (uint32_t)CW_STATUS_INTERNAL);
  // rank of every key among the keys of its digit in its wave (stable: item
  // order, then lane order); the wave's LDS operations run in order, so the
  // counter row needs no barrier inside the wave
  uint32_t *const cr = cw[w];
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = (w * IT + k) * 64 + lane;
    const bool v = j < len;
    const uint32_t d = (uint32_t)(key[k] >> shift) & dmask;
    dig[k] = d;
    uint64_t m = __ballot(v);
    for (uint32_t bit = 0; bit < (EXPS & 1u ? 0u : dbits); bit++) {
      const bool on = (d >> bit) & 1u;
      const uint64_t bb = __ballot(on);
      m &= on ? bb : ~bb;
    }
    const uint32_t lr = lanes_below(m);
    const uint32_t before = cr[d];
    pin[k] = before + lr;
    __builtin_amdgcn_wave_barrier();
    if (v && lr == 0) cr[d] = before + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per bucket (thread b): the waves' offsets and the tile's count, published
  // at once as this tile's aggregate
  uint32_t cnt = 0;
  if (tid < OS_MAX_BINS) {
#pragma unroll
    for (uint32_t ww = 0; ww < NW; ww++) {
      const uint32_t c = cw[ww][tid];
      cw[ww][tid] = cnt;
      cnt += c;
    }
    if (tid < nb && li > 0)
      __hip_atomic_store(lb + (size_t)g * OS_MAX_BINS + tid,
                         OS_AGG | ((unsigned long long)epoch << 32) | cnt, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t bs = block_exscan<NT>(tid < nb ? cnt : 0u, wtot, nullptr);
  if (tid < OS_MAX_BINS) bstart[tid] = bs;
  __syncthreads();
  // the tile sorted by digit in LDS
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = (w * IT + k) * 64 + lane;
    if (j < len) {
      const uint32_t pos = bstart[dig[k]] + cw[w][dig[k]] + pin[k];
      pin[k] = pos;  // (kept for the payload)
      skey[pos] = key[k];
      sval[pos] = val[k];
    }
  }
  // (exp: timing experiments only, wrong results -- 1: no digit match in the
  // ranking, 2: no look-back, 4: no write-out, 8: one look-back window, no wait)
  // look-back over the earlier tiles of the range, one thread per bucket,
  // OS_LBW tiles a round trip (a look-back word is an agent-scope load past the
  // XCD's L2, ~1 us: walking one tile a trip back to the nearest inclusive
  // prefix cost more than the tile's own work).  Issued only now: the nearest
  // words loaded before the scan and the LDS scatter were more often not
  // published yet and cost a second trip (7.0 vs 6.5 ms of passes at 2e8 keys).
  if (tid < nb) {
    uint32_t pre = 0;
    for (int64_t q0 = (EXPS & 2u) ? -1 : (int64_t)li - 1; q0 >= 0;) {
      unsigned long long v[OS_LBW];
#pragma unroll
      for (uint32_t i = 0; i < OS_LBW; i++)
        v[i] = q0 - (int64_t)i >= 0
                   ? __hip_atomic_load(lb + ((size_t)x * Tr + (size_t)(q0 - i)) * OS_MAX_BINS + tid,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : (OS_INC | ((unsigned long long)epoch << 32));  // before tile 0: prefix 0
      // sum from the nearest tile back to the first inclusive prefix; a tile
      // not published yet before it means another trip for this window
      uint32_t sum = 0, used = 0;
      bool inc = false, wait = false;
#pragma unroll
      for (uint32_t i = 0; i < OS_LBW; i++) {
        if (inc || wait) continue;
        const bool ok = ((v[i] >> 32) & 0xFFFFull) == epoch && (v[i] & (OS_INC | OS_AGG));
        if (!ok) {
          wait = true;
          continue;
        }
        sum += (uint32_t)v[i];
        used = i + 1;
        inc = (v[i] & OS_INC) != 0;
      }
      pre += sum;
      if (inc || (EXPS & 8u)) break;
      q0 -= used;  // (the published aggregates are kept; the rest is read again)
      if (wait) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(lb + (size_t)g * OS_MAX_BINS + tid,
                       OS_INC | ((unsigned long long)epoch << 32) | (pre + cnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    goff[tid] = bx[tid] + pre - bs;
  }
  __syncthreads();
  // digit runs out, coalesced
  uint32_t dk[PL ? IT : 1];
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = tid + k * NT;
    if (PL) dk[k] = 0xFFFFFFFFu;
    if (j >= (EXPS & 4u ? 0u : len)) continue;
    const K kk = skey[j];
    uint32_t dst = goff[(uint32_t)(kk >> shift) & dmask] + j;
    if (EXPS) dst %= n;  // (an experiment's positions are garbage: keep them in the buffer)
    if (PL) dk[k] = dst;
    if (PL_LAST) {  // (bare ids, hi apart)
      keys_out[dst] = kk & ((1ull << pl.kb) - 1);
      pl.hi_out[dst] = (uint32_t)(kk >> pl.kb);
    } else if (keys_out) {
      keys_out[dst] = kk;
    }
    const uint32_t vv = sval[j];
    vals_out[dst] = vv;
    if (inv) inv[vv] = dst;
  }
  if (PL) {
    // lo through the value buffer: the same positions, the same runs
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
      if ((w * IT + k) * 64 + lane < len) sval[pin[k]] = pv[k];
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
      if (dk[k] != 0xFFFFFFFFu) pl.lo_out[dk[k]] = sval[tid + k * NT];
  }
}
