// onesweep.hip -- one-pass-per-digit LSD radix sort of ONE array (included by
// causeweave.hip; the id sort of one giant list, list.cljc:28 / shared.cljc:128,
// and the giant tree's sort of cross-tile children).
//
// The histogram-scan-scatter sort (k_radix_hist / k_gscan_* / k_radix_scatter)
// reads the keys twice a pass and runs a chain of small scan launches between.
// Here one kernel, k_os_hist, reads the keys ONCE for every pass's digit counts,
// k_os_scan turns them into bucket bases, and each pass is one kernel,
// k_os_pass: a tile of keys is ranked by its digit inside LDS (one
// wave-ballot match of the whole digit, per-wave bucket counters), publishes its
// digit counts, learns the counts of the tiles before it by a decoupled
// look-back, and writes its digit runs out from LDS.
//
// Tiles are processed in block order: tile g's look-back waits only on tiles
// g - 1, g - 2, ..., whose blocks were dispatched before it (the in-order
// dispatch k_map_pack's look-back relies on too), so the smallest unfinished
// tile always finishes.  (Round 6 first cut the array into one look-back chain
// per XCD with per-chunk bucket bases from the histogram; that is exact for the
// first pass only -- a later pass reads the previous pass's output, whose chunks
// hold other keys than the input's.)
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

// Every pass's digit counts: hist[p * OS_MAX_BINS + b] (the counts of a pass
// do not depend on the order its input arrives in).  A block takes
// OS_HIST_ITEMS * 256 consecutive keys; each wave counts into its own copy of
// the counters (dynamic LDS: 4 waves x passes x OS_MAX_BINS words), so the
// LDS atomics of different waves never meet.
constexpr uint32_t OS_HIST_ITEMS = 16;
template <typename K>
__global__ __launch_bounds__(256) void k_os_hist(const K *__restrict__ keys, uint32_t n, OsDigits dg,
                                                 uint32_t *__restrict__ hist) {
  extern __shared__ uint32_t lds_osh[];
  const uint32_t tid = threadIdx.x, w = tid >> 6, words = dg.passes * OS_MAX_BINS;
  for (uint32_t i = tid; i < 4 * words; i += 256) lds_osh[i] = 0;
  __syncthreads();
  uint32_t *const h = lds_osh + w * words;
  const uint64_t i0 = (uint64_t)blockIdx.x * (256 * OS_HIST_ITEMS);
  K kk[OS_HIST_ITEMS];
#pragma unroll
  for (uint32_t k = 0; k < OS_HIST_ITEMS; k++) {
    const uint64_t i = i0 + k * 256 + tid;
    kk[k] = i < n ? keys[i] : (K)0;
  }
  for (uint32_t p = 0; p < dg.passes; p++) {
    const uint32_t sh = dg.shift[p], m = (1u << dg.bits[p]) - 1;
    uint32_t *const hp = h + p * OS_MAX_BINS;
#pragma unroll
    for (uint32_t k = 0; k < OS_HIST_ITEMS; k++)
      if (i0 + k * 256 + tid < n) atomicAdd(&hp[(uint32_t)(kk[k] >> sh) & m], 1u);
  }
  __syncthreads();
  for (uint32_t i = tid; i < words; i += 256) {
    const uint32_t c = lds_osh[i] + lds_osh[words + i] + lds_osh[2 * words + i] + lds_osh[3 * words + i];
    if (c) atomicAdd(&hist[i], c);
  }
}

// Bucket bases: base[p * OS_MAX_BINS + b] = the keys of every bucket < b.
// One block per pass, one thread per bucket.
__global__ __launch_bounds__(OS_MAX_BINS) void k_os_scan(const uint32_t *__restrict__ hist, OsDigits dg,
                                                         uint32_t *__restrict__ base) {
  __shared__ uint32_t wtot[OS_MAX_BINS / 64];
  const uint32_t p = blockIdx.x, b = threadIdx.x, nb = 1u << dg.bits[p];
  const uint32_t c = b < nb ? hist[(size_t)p * OS_MAX_BINS + b] : 0u;
  base[(size_t)p * OS_MAX_BINS + b] = block_exscan<OS_MAX_BINS>(c, wtot, nullptr);
}

// One LSD pass.  NT threads, IT keys a thread (wave-blocked: wave w holds the
// tile's elements [w * IT * 64, (w + 1) * IT * 64)), digit = (key >> shift) &
// (2^dbits - 1), dbits <= OS_MAX_BITS, NT >= 2^dbits.  vals_in == nullptr: the
// value is the element's index.  keys_out == nullptr: values only.  inv: also
// inv[value] = the element's sorted position (the last pass of a sort whose
// values are input indices).
template <typename K, int NT, int IT>
__global__ __launch_bounds__(NT) void k_os_pass(
    const K *__restrict__ keys_in, const uint32_t *__restrict__ vals_in, K *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, uint32_t *__restrict__ inv, uint32_t n, uint32_t shift,
    uint32_t dbits, const uint32_t *__restrict__ base, unsigned long long *lb, uint32_t epoch) {
  constexpr uint32_t TS = NT * IT, NW = NT / 64;
  static_assert(NT >= OS_MAX_BINS, "one thread per bucket");
  __shared__ K skey[TS];
  __shared__ uint32_t sval[TS];
  __shared__ uint32_t cw[NW][OS_MAX_BINS];  // per wave: its count, then its offset inside the bucket
  __shared__ uint32_t bstart[OS_MAX_BINS];  // bucket start inside the tile
  __shared__ uint32_t goff[OS_MAX_BINS];    // output position of the tile's bucket start, minus bstart
  __shared__ uint32_t wtot[NW];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = 1u << dbits, dmask = nb - 1;
  for (uint32_t b = lane; b < OS_MAX_BINS; b += 64) cw[w][b] = 0;
  __syncthreads();
  const uint32_t g = blockIdx.x;  // tile index (dispatch order)
  const uint64_t s64 = (uint64_t)g * TS;
  const uint32_t s = (uint32_t)min<uint64_t>(s64, n), len = (uint32_t)min<uint64_t>(TS, n - s);
  K key[IT];
  uint32_t val[IT], dig[IT], pin[IT];
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = (w * IT + k) * 64 + lane;
    const bool v = j < len;
    key[k] = v ? keys_in[s + j] : (K)0;
    val[k] = v ? (vals_in ? vals_in[s + j] : s + j) : 0u;
  }
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
    for (uint32_t bit = 0; bit < dbits; bit++) {
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
    if (tid < nb && g > 0)
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
      skey[pos] = key[k];
      sval[pos] = val[k];
    }
  }
  // look-back over the earlier tiles, one thread per bucket, OS_LBW tiles a
  // round trip (a look-back word is an agent-scope load past the XCD's L2,
  // ~1 us: walking one tile a trip back to the nearest inclusive prefix cost
  // more than the tile's own work)
  if (tid < nb) {
    uint32_t pre = 0;
    for (int64_t q0 = (int64_t)g - 1; q0 >= 0;) {
      unsigned long long v[OS_LBW];
#pragma unroll
      for (uint32_t i = 0; i < OS_LBW; i++)
        v[i] = q0 - (int64_t)i >= 0
                   ? __hip_atomic_load(lb + (size_t)(q0 - i) * OS_MAX_BINS + tid, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT)
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
      if (inc) break;
      q0 -= used;  // (the published aggregates are kept; the rest is read again)
      if (wait) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(lb + (size_t)g * OS_MAX_BINS + tid,
                       OS_INC | ((unsigned long long)epoch << 32) | (pre + cnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    goff[tid] = base[tid] + pre - bs;
  }
  __syncthreads();
  // digit runs out, coalesced
  for (uint32_t j = tid; j < len; j += NT) {
    const K kk = skey[j];
    const uint32_t dst = goff[(uint32_t)(kk >> shift) & dmask] + j;
    if (keys_out) keys_out[dst] = kk;
    const uint32_t vv = sval[j];
    vals_out[dst] = vv;
    if (inv) inv[vv] = dst;
  }
}
