// causeweave.hip -- MI355X (gfx950) weave for Cause: kernels + the C ABI of
// include/causeweave.h.
//
// Pipeline for a batch of independent CausalLists (DESIGN.md has the byte
// accounting and the reference lines each stage replaces):
//
//   1-2. front end  (dense ids) k_fdir / k_frank / k_fplace: per-document rank
//                   directory (id bitmap + popcounts) -> id order, cause ranks
//                   and the domain checks of shared.cljc:163-178, written in
//                   rank order through window records; (sparse ids) segmented
//                   LSD radix sort + bucket index + join -- (sort (::s/nodes ct)),
//                   list.cljc:28, and the cause scan of weave-node
//   3-5. tree       k_tree, one workgroup per document: effective parents
//                   (SURVEY F5), sibling order (weave-later?, shared.cljc:202-223),
//                   first children, threads -> each node's preorder successor,
//                   visibility (hide?, list.cljc:48-55 via SURVEY F6), splitters
//   6.   walk       each splitter's walker follows successors to the next splitter
//   7.   rank       per-document list ranking of the sublists in LDS
//   8.   emit       weave position -> weave_perm, visibility, counts
//   9.   pack       visibility bytes -> bitmap
//  (10.  yarns      stable radix partition of the id order by site, spin 1-arity)
//
// Maps (cw_weave_maps), merge (cw_merge_lists) and weft (cw_weft_lists) reuse
// the pipeline after their own selection / grouping kernels; tiny documents
// (map key weaves) have their own in-LDS sort and weave kernels.
//
// Everything is integer work bounded by HBM/L2 traffic and latency; MFMA is
// not used.  Tile grids map documents contiguously onto one XCD so the blocks
// that touch one document run close together in time and share its L2.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <chrono>
#include <string>
#include <vector>

#include "causeweave.h"
#include "cw_internal.h"

using namespace cw;

// ============================================================================
// Device kernels
// ============================================================================

// Block-wide exclusive scan of one value per thread (blockDim.x = 64*W,
// wtot has blockDim.x/64 entries).  NT = 0: block size taken at run time.
template <int NT>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wtot, uint32_t *total) {
  const int nw = NT ? NT / 64 : (int)(blockDim.x >> 6);
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (int i = 0; i < nw; i++) {
    uint32_t t = wtot[i];
    before += (i < (int)w) ? t : 0u;
    all += t;
  }
  if (total) *total = all;
  __syncthreads();
  return before + x - v;
}

// --- segmented LSD radix sort ------------------------------------------------
// A pass sorts by one digit of <= MAX_DIGIT bits (<= 2048 bins).  Each tile is
// first sorted by the digit inside LDS (two stable sub-passes of <= 6 bits:
// wave ballots + per-wave counters), then written out as digit runs.
template <typename K>
__global__ __launch_bounds__(256) void k_radix_hist(const K *__restrict__ keys,
                                                    const uint32_t *__restrict__ tile_start,
                                                    uint32_t shift, uint32_t dbits,
                                                    uint32_t *__restrict__ hist) {
  __shared__ uint32_t h[4][MAX_BINS];
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), tid = threadIdx.x, w = tid >> 6;
  const uint32_t nb = 1u << dbits, dmask = nb - 1;
  for (uint32_t i = tid; i < 4 * nb; i += 256) h[i / nb][i % nb] = 0;
  __syncthreads();
  const uint32_t s = tile_start[t], e = tile_start[t + 1];
  // a tile is <= TILE keys: all of a thread's loads issue before its first
  // LDS atomic (16 in flight, not one per loop trip)
  constexpr uint32_t HI = TILE / 256;
  K kk[HI];
#pragma unroll
  for (uint32_t k = 0; k < HI; k++) {
    const uint32_t i = s + tid + k * 256;
    kk[k] = i < e ? keys[i] : (K)0;
  }
#pragma unroll
  for (uint32_t k = 0; k < HI; k++)
    if (s + tid + k * 256 < e) atomicAdd(&h[w][(uint32_t)(kk[k] >> shift) & dmask], 1u);
  __syncthreads();
  for (uint32_t b = tid; b < nb; b += 256)
    hist[(size_t)t * nb + b] = h[0][b] + h[1][b] + h[2][b] + h[3][b];
}

// Per document: turn the (tile, digit) counts into global output offsets,
// digit-major then tile order (stable).  1024 threads, <= 2 bins each.
__global__ __launch_bounds__(1024) void k_radix_scan(uint32_t *__restrict__ hist,
                                                     const uint32_t *__restrict__ tile_first,
                                                     const uint32_t *__restrict__ doc_off,
                                                     uint32_t dbits) {
  __shared__ uint32_t wtot[16];
  const uint32_t d = blockIdx.x, nb = 1u << dbits;
  const uint32_t bpt = (nb + blockDim.x - 1) / blockDim.x;  // 1 or 2
  const uint32_t b0 = threadIdx.x * bpt;
  const uint32_t t0 = tile_first[d], t1 = tile_first[d + 1];
  if (t0 == t1) return;  // empty document (uniform per block)
  uint32_t tot[2] = {0, 0};
  for (uint32_t t = t0; t < t1; t++)
    for (uint32_t k = 0; k < bpt; k++)
      if (b0 + k < nb) tot[k] += hist[(size_t)t * nb + b0 + k];
  uint32_t run[2];
  run[0] = doc_off[d] + block_exscan<0>(tot[0] + tot[1], wtot, nullptr);
  run[1] = run[0] + tot[0];
  for (uint32_t t = t0; t < t1; t++)
    for (uint32_t k = 0; k < bpt; k++)
      if (b0 + k < nb) {
        const uint32_t c = hist[(size_t)t * nb + b0 + k];
        hist[(size_t)t * nb + b0 + k] = run[k];
        run[k] += c;
      }
}

// One document of many tiles (the giant-document path): the per-document scan
// above would walk every tile in one workgroup.  Chunked scan instead, in
// digit-major then tile order: per-chunk column sums, a scan over chunks per
// digit, a scan over digits, and each chunk applies its bases.
constexpr uint32_t GSCAN_CHUNK = 128;  // tiles per chunk
// Loads issued together before the dependent stores / sums: a loop that
// stores between loads waits one memory round trip a trip (the serial scan
// over 3,815 chunks at 2e9 nodes)
constexpr uint32_t GSCAN_BATCH = 16;

__global__ __launch_bounds__(1024) void k_gscan_colsum(const uint32_t *__restrict__ hist, uint32_t T,
                                                       uint32_t nb, uint32_t *__restrict__ cs) {
  const uint32_t c = blockIdx.x, t0 = c * GSCAN_CHUNK, t1 = min(T, t0 + GSCAN_CHUNK);
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    uint32_t sum = 0;
    for (uint32_t t = t0; t < t1; t += GSCAN_BATCH) {
      uint32_t v[GSCAN_BATCH];
#pragma unroll
      for (uint32_t k = 0; k < GSCAN_BATCH; k++) v[k] = t + k < t1 ? hist[(size_t)(t + k) * nb + b] : 0u;
#pragma unroll
      for (uint32_t k = 0; k < GSCAN_BATCH; k++) sum += v[k];
    }
    cs[(size_t)c * nb + b] = sum;
  }
}

__global__ __launch_bounds__(1024) void k_gscan_chunks(uint32_t *__restrict__ cs, uint32_t nc,
                                                       uint32_t nb, uint32_t *__restrict__ tot) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  uint32_t run = 0;
  for (uint32_t c0 = 0; c0 < nc; c0 += GSCAN_BATCH) {
    uint32_t v[GSCAN_BATCH];
#pragma unroll
    for (uint32_t k = 0; k < GSCAN_BATCH; k++) v[k] = c0 + k < nc ? cs[(size_t)(c0 + k) * nb + b] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < GSCAN_BATCH; k++)
      if (c0 + k < nc) {
        cs[(size_t)(c0 + k) * nb + b] = run;
        run += v[k];
      }
  }
  tot[b] = run;
}

__global__ __launch_bounds__(1024) void k_gscan_bins(uint32_t *__restrict__ tot, uint32_t nb,
                                                     uint32_t base) {
  __shared__ uint32_t wtot[16];
  const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
  uint32_t v[2] = {0, 0}, sum = 0;
  for (uint32_t k = 0; k < per && k < 2; k++) {
    v[k] = b0 + k < nb ? tot[b0 + k] : 0u;
    sum += v[k];
  }
  uint32_t run = base + block_exscan<1024>(sum, wtot, nullptr);
  for (uint32_t k = 0; k < per && k < 2; k++)
    if (b0 + k < nb) {
      tot[b0 + k] = run;
      run += v[k];
    }
}

__global__ __launch_bounds__(1024) void k_gscan_apply(uint32_t *__restrict__ hist, uint32_t T,
                                                      uint32_t nb, const uint32_t *__restrict__ cs,
                                                      const uint32_t *__restrict__ tot) {
  const uint32_t c = blockIdx.x, t0 = c * GSCAN_CHUNK, t1 = min(T, t0 + GSCAN_CHUNK);
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    uint32_t run = tot[b] + cs[(size_t)c * nb + b];
    constexpr uint32_t AB = GSCAN_BATCH / 2;  // (16: SGPR spills of the 16 offsets)
    for (uint32_t t = t0; t < t1; t += AB) {
      uint32_t *h = hist + (size_t)t * nb + b;
      const uint32_t m = min(AB, t1 - t);
      uint32_t v[AB];
#pragma unroll
      for (uint32_t k = 0; k < AB; k++) v[k] = k < m ? h[k * nb] : 0u;
#pragma unroll
      for (uint32_t k = 0; k < AB; k++)
        if (k < m) {
          h[k * nb] = run;
          run += v[k];
        }
    }
  }
}

// Element index of item k of the calling lane when ITEMS items per lane are
// wave-blocked: wave w owns elements [w*ITEMS*64, (w+1)*ITEMS*64), item k of
// lane l is element (w*ITEMS + k)*64 + l.
template <int ITEMS>
__device__ __forceinline__ uint32_t wb_elem(uint32_t k) {
  return (((threadIdx.x >> 6) * ITEMS + k) << 6) + (threadIdx.x & 63);
}

// Stable rank of wave-blocked items (wb_elem) by a sub-digit of sbits (<= 6)
// bits: returns each item's position inside the tile of `len` elements.  Each
// wave counts its own items in a private LDS row (LDS ops of one wave execute
// in order, so no barrier is needed inside the wave); two barriers combine the
// waves.  wcnt is [NT/64][SUB_BINS], run is [64].
template <int NT, int ITEMS>
__device__ __forceinline__ void rank_subdigit(const uint32_t (&sd)[ITEMS], uint32_t len,
                                              uint32_t sbits, uint32_t (&pos)[ITEMS],
                                              uint32_t (*wcnt)[SUB_BINS], uint32_t *run) {
  constexpr int NW = NT / 64;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *cw = wcnt[w];
  cw[lane] = 0;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (uint32_t k = 0; k < ITEMS; k++) {
    const bool valid = wb_elem<ITEMS>(k) < len;
    const uint32_t dd = sd[k];
    uint64_t m = __ballot(valid);
    for (uint32_t bit = 0; bit < sbits; bit++) {
      const bool on = (dd >> bit) & 1u;
      const uint64_t bb = __ballot(on);
      m &= on ? bb : ~bb;
    }
    const uint32_t lr = lanes_below(m);
    const uint32_t before = cw[dd];
    pos[k] = before + lr;
    __builtin_amdgcn_wave_barrier();
    if (valid && lr == 0) cw[dd] = before + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // per bin: wave offsets, then bin starts
    const uint32_t bn = threadIdx.x;
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < NW; ww++) {
      const uint32_t c = wcnt[ww][bn];
      wcnt[ww][bn] = tot;
      tot += c;
    }
    const uint32_t v = bn < (1u << sbits) ? tot : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (bn >= (uint32_t)o) x += y;
    }
    run[bn] = x - v;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < ITEMS; k++) pos[k] += run[sd[k]] + cw[sd[k]];
  __syncthreads();
}

// rank_subdigit for many waves (k_tree_l: 16): the per-bin prefix over the
// waves is a segmented shuffle scan over all threads (NW lanes per bin) rather
// than one lane walking NW rows, and every wave scans the 64 bin totals itself
// (its digits pick their bin start by a lane shuffle), so there is no serial
// chain of NW dependent LDS round trips.  btot is [64].
template <int NT, int ITEMS>
__device__ __forceinline__ void rank_subdigit_par(const uint32_t (&sd)[ITEMS], uint32_t len,
                                                  uint32_t sbits, uint32_t (&pos)[ITEMS],
                                                  uint32_t (*wcnt)[SUB_BINS], uint32_t *btot) {
  constexpr int NW = NT / 64;
  static_assert(NW >= 2 && (NW & (NW - 1)) == 0 && NW <= 64, "power-of-two wave count");
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *cw = wcnt[w];
  cw[lane] = 0;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (uint32_t k = 0; k < ITEMS; k++) {
    const bool valid = wb_elem<ITEMS>(k) < len;
    const uint32_t dd = sd[k];
    uint64_t m = __ballot(valid);
    for (uint32_t bit = 0; bit < sbits; bit++) {
      const bool on = (dd >> bit) & 1u;
      const uint64_t bb = __ballot(on);
      m &= on ? bb : ~bb;
    }
    const uint32_t lr = lanes_below(m);
    const uint32_t before = cw[dd];
    pos[k] = before + lr;
    __builtin_amdgcn_wave_barrier();
    if (valid && lr == 0) cw[dd] = before + (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  {
    const uint32_t ww = threadIdx.x & (NW - 1), bn = threadIdx.x / NW;
    const uint32_t c = wcnt[ww][bn];
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < NW; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, NW);
      if (ww >= (uint32_t)o) x += y;
    }
    wcnt[ww][bn] = x - c;
    if (ww == NW - 1) btot[bn] = x;
  }
  __syncthreads();
  const uint32_t v = lane < (1u << sbits) ? btot[lane] : 0u;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  const uint32_t ex = x - v;
#pragma unroll
  for (uint32_t k = 0; k < ITEMS; k++) pos[k] += __shfl(ex, (int)sd[k], 64) + cw[sd[k]];
  __syncthreads();
}

// Stable scatter of one tile by digit (key >> shift) & (2^dbits - 1).
// vals_in == nullptr means "value = doc-local index of the element".
// inv != nullptr (last pass only) also records each input node's rank.
template <typename K>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_scatter(
    const K *__restrict__ keys_in, const uint32_t *__restrict__ vals_in, K *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, const uint32_t *__restrict__ tile_start,
    const uint32_t *__restrict__ tile_doc, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ offs, uint32_t shift, uint32_t dbits, uint32_t sub0,
    uint32_t *__restrict__ inv) {
  __shared__ K skey[TILE];
  __shared__ uint32_t sval[TILE];
  __shared__ uint32_t soff[MAX_BINS], bstart[MAX_BINS];
  __shared__ uint32_t wcnt[SORT_WAVES][SUB_BINS];
  __shared__ uint32_t run[64];
  __shared__ uint32_t wtot[SORT_WAVES];

  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), tid = threadIdx.x;
  const uint32_t s = tile_start[t], e = tile_start[t + 1];
  const uint32_t len = e - s;
  const uint32_t lbase = s - doc_off[tile_doc[t]];
  const uint32_t nb = 1u << dbits, dmask = nb - 1;

  for (uint32_t b = tid; b < nb; b += SORT_THREADS) {
    soff[b] = offs[(size_t)t * nb + b];
    bstart[b] = 0;
  }
  __syncthreads();
  K key[SORT_ITEMS];
  uint32_t val[SORT_ITEMS], sd[SORT_ITEMS], pos[SORT_ITEMS];
#pragma unroll
  for (uint32_t k = 0; k < SORT_ITEMS; k++) {
    const uint32_t j = wb_elem<SORT_ITEMS>(k);
    const bool valid = j < len;
    key[k] = valid ? keys_in[s + j] : (K)0;
    val[k] = valid ? (vals_in ? vals_in[s + j] : lbase + j) : 0u;
    const uint32_t dg = (uint32_t)(key[k] >> shift) & dmask;
    if (valid) atomicAdd(&bstart[dg], 1u);
    sd[k] = dg & ((1u << sub0) - 1);
  }
  // sub-pass A: low sub-digit
  rank_subdigit<SORT_THREADS, SORT_ITEMS>(sd, len, sub0, pos, wcnt, run);
  const uint32_t sub1 = dbits - sub0;
  if (sub1 > 0) {
#pragma unroll
    for (uint32_t k = 0; k < SORT_ITEMS; k++)
      if (wb_elem<SORT_ITEMS>(k) < len) {
        skey[pos[k]] = key[k];
        sval[pos[k]] = val[k];
      }
    __syncthreads();
    // sub-pass B: high sub-digit, over the tile in sub-pass A order
#pragma unroll
    for (uint32_t k = 0; k < SORT_ITEMS; k++) {
      const uint32_t j = wb_elem<SORT_ITEMS>(k);
      if (j < len) {
        key[k] = skey[j];
        val[k] = sval[j];
      }
      sd[k] = ((uint32_t)(key[k] >> shift) & dmask) >> sub0;
    }
    rank_subdigit<SORT_THREADS, SORT_ITEMS>(sd, len, sub1, pos, wcnt, run);
  }
#pragma unroll
  for (uint32_t k = 0; k < SORT_ITEMS; k++)
    if (wb_elem<SORT_ITEMS>(k) < len) {
      skey[pos[k]] = key[k];
      sval[pos[k]] = val[k];
    }
  // digit starts inside the tile
  {
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;  // <= 4 bins per lane (2048 / 512)
    const uint32_t b0 = tid * 4;
    if (b0 < nb) { c0 = bstart[b0]; c1 = bstart[b0 + 1]; c2 = bstart[b0 + 2]; c3 = bstart[b0 + 3]; }
    if (nb < 4 && b0 < nb) { c1 = nb > 1 ? c1 : 0; c2 = nb > 2 ? c2 : 0; c3 = 0; }
    const uint32_t ex = block_exscan<SORT_THREADS>(c0 + c1 + c2 + c3, wtot, nullptr);
    if (b0 < nb) {
      bstart[b0] = ex;
      if (b0 + 1 < nb) bstart[b0 + 1] = ex + c0;
      if (b0 + 2 < nb) bstart[b0 + 2] = ex + c0 + c1;
      if (b0 + 3 < nb) bstart[b0 + 3] = ex + c0 + c1 + c2;
    }
  }
  __syncthreads();
  for (uint32_t j = tid; j < len; j += SORT_THREADS) {
    const K kk = skey[j];
    const uint32_t d = (uint32_t)(kk >> shift) & dmask;
    const uint32_t dst = soff[d] + j - bstart[d];
    if (keys_out) keys_out[dst] = kk;  // (null: the caller wants the values only)
    vals_out[dst] = sval[j];
    if (inv) inv[s - lbase + sval[j]] = dst - (s - lbase);  // rank of each input node
  }
}

// Small documents (every one <= TILE): packs of whole consecutive documents
// (<= TILE elements) are sorted entirely in LDS by (document in pack, digit
// bits of the key) -- stable LSD sub-passes -- and written back in place, one
// kernel instead of the global hist/scan/scatter passes (maps: 10^6
// collections of ~100 nodes, and their key weaves).
template <typename K>
__global__ __launch_bounds__(SORT_THREADS) void k_pack_sort(
    const K *__restrict__ keys_in, const uint32_t *__restrict__ vals_in, K *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, const uint32_t *__restrict__ pack_doc0,
    const uint32_t *__restrict__ doc_off, uint32_t shift, uint32_t kbits, uint32_t dbits) {
  constexpr uint32_t IT = SORT_ITEMS;
  __shared__ K skey[TILE];
  __shared__ uint32_t sval[TILE];
  __shared__ uint32_t dstart[TILE + 1];
  __shared__ uint32_t wcnt[SORT_WAVES][SUB_BINS];
  __shared__ uint32_t run[64];
  const uint32_t pk = blockIdx.x, tid = threadIdx.x;
  const uint32_t d0 = pack_doc0[pk], d1 = pack_doc0[pk + 1], nd = d1 - d0;
  const uint32_t s = doc_off[d0], len = doc_off[d1] - s;
  for (uint32_t i = tid; i <= nd; i += SORT_THREADS) dstart[i] = doc_off[d0 + i] - s;
  __syncthreads();
  const K kmask = kbits >= 8 * sizeof(K) ? ~(K)0 : (((K)1 << kbits) - 1);
  K ck[IT];  // composite key: document in pack above the key bits
  K key[IT];
  uint32_t val[IT], sd[IT], pos[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t j = wb_elem<IT>(u);
    key[u] = 0;
    val[u] = 0;
    ck[u] = 0;
    if (j < len) {
      uint32_t lo = 0, hi = nd;  // document of element j
      while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (dstart[m] <= j) lo = m; else hi = m;
      }
      key[u] = keys_in[s + j];
      val[u] = vals_in ? vals_in[s + j] : j - dstart[lo];
      ck[u] = ((K)lo << kbits) | ((key[u] >> shift) & kmask);
    }
  }
  const uint32_t bits = kbits + dbits;
  for (uint32_t sh = 0; sh < bits; sh += SUB_BITS) {
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) sd[u] = (uint32_t)(ck[u] >> sh) & (SUB_BINS - 1);
    rank_subdigit<SORT_THREADS, IT>(sd, len, min(SUB_BITS, bits - sh), pos, wcnt, run);
#pragma unroll
    for (uint32_t u = 0; u < IT; u++)
      if (wb_elem<IT>(u) < len) {
        skey[pos[u]] = key[u];
        sval[pos[u]] = val[u];
        dstart[pos[u]] = (uint32_t)(ck[u] >> kbits);  // the document, to rebuild ck
      }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
      const uint32_t j = wb_elem<IT>(u);
      if (j < len) {
        key[u] = skey[j];
        val[u] = sval[j];
        ck[u] = ((K)dstart[j] << kbits) | ((key[u] >> shift) & kmask);
      }
    }
    __syncthreads();
  }
  for (uint32_t j = tid; j < len; j += SORT_THREADS) {
    keys_out[s + j] = skey[j];
    vals_out[s + j] = sval[j];
  }
}

// --- join: cause -> parent rank ---------------------------------------------
__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t *__restrict__ a, uint32_t n,
                                                    uint64_t x) {
  uint32_t lo = 0, len = n;
  while (len > 0) {
    const uint32_t half = len >> 1;
    if (a[lo + half] < x) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

// Per document: a bucket index over the sorted ids and the duplicate-id check
// (shared.cljc:166-171).  With kmin/kmax the smallest/largest id and a shift
// s chosen so that at most max(n/4, 1) buckets cover [kmin, kmax], entry h of
// the index is the first rank whose id has (id - kmin) >> s >= h (entry NB =
// n).  Lamport ids are close to uniform over their range, so a bucket holds a
// handful of ids: the join finds a cause with two index reads and one short
// search inside a line of sorted ids.  Coalesced reads; neighbours compared
// across lanes with a shuffle.
__device__ __forceinline__ uint32_t bucket_shift(uint64_t range, uint32_t n) {
  const uint64_t nbmax = max(n >> 2, 1u);
  uint32_t s = 0;
  while ((range >> s) > nbmax) s++;
  return s;
}

__global__ __launch_bounds__(256) void k_index(const uint64_t *__restrict__ skey,
                                               const uint32_t *__restrict__ doc_off,
                                               const uint32_t *__restrict__ bkt_off,
                                               uint32_t *__restrict__ bkt,
                                               uint32_t *__restrict__ status) {
  const uint32_t d = blockIdx.x, base = doc_off[d], n = doc_off[d + 1] - base;
  if (n == 0) return;
  const uint64_t kmin = skey[base], kmax = skey[base + n - 1];
  const uint32_t sh = bucket_shift(kmax - kmin, n);
  const uint32_t nb = (uint32_t)((kmax - kmin) >> sh) + 1;
  uint32_t *B = bkt + bkt_off[d];
  const uint32_t lane = threadIdx.x & 63;
  bool dup = false;
  for (uint32_t i0 = threadIdx.x & ~63u; i0 < n; i0 += blockDim.x) {
    const uint32_t i = i0 + lane;
    const uint64_t x = i < n ? skey[base + i] : kmax;
    uint64_t prev = __shfl_up(x, 1, 64);
    if (lane == 0 && i > 0 && i < n) prev = skey[base + i - 1];
    if (i < n) {
      const uint32_t h = (uint32_t)((x - kmin) >> sh);
      uint32_t h0 = 0;
      if (i > 0) {
        dup |= prev == x;
        h0 = (uint32_t)((prev - kmin) >> sh) + 1;
      }
      for (uint32_t hh = h0; hh <= h; hh++) B[hh] = i;
    }
  }
  if (threadIdx.x == 0) B[nb] = n;
  if (__syncthreads_or(dup) && threadIdx.x == 0) atomicOr(&status[d], (uint32_t)CW_STATUS_DUP);
}

// k_index for a batch that is one (large) document: one thread per sorted id.
__global__ __launch_bounds__(256) void k_index_flat(const uint64_t *__restrict__ skey, uint32_t n,
                                                    uint32_t *__restrict__ bkt,
                                                    uint32_t *__restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t kmin = skey[0], kmax = skey[n - 1];
  const uint32_t sh = bucket_shift(kmax - kmin, n);
  const uint64_t x = skey[i];
  const uint32_t h = (uint32_t)((x - kmin) >> sh);
  uint32_t h0 = 0;
  if (i > 0) {
    const uint64_t prev = skey[i - 1];
    if (prev == x) atomicOr(&status[0], (uint32_t)CW_STATUS_DUP);
    h0 = (uint32_t)((prev - kmin) >> sh) + 1;
  }
  for (uint32_t hh = h0; hh <= h; hh++) bkt[hh] = i;
  if (i == n - 1) bkt[(uint32_t)((kmax - kmin) >> sh) + 1] = n;
}

// Join in sorted order: gather each node's cause id and kind, find the cause
// among the document's sorted ids through the bucket index (k_index).  Each
// lane handles JOIN_ITEMS nodes with their loads and searches interleaved.
__global__ __launch_bounds__(1024) void k_join(
    const uint64_t *__restrict__ skey, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ cause_key, const uint8_t *__restrict__ kind,
    const uint32_t *__restrict__ bkt, const uint32_t *__restrict__ bkt_off,
    const uint32_t *__restrict__ tile_start,
    const uint32_t *__restrict__ tile_doc, const uint32_t *__restrict__ doc_off,
    uint32_t *__restrict__ par, uint8_t *__restrict__ skind, uint32_t *__restrict__ status) {
  constexpr int IT = JOIN_ITEMS;
  __shared__ uint32_t bst;
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), d = tile_doc[t];
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base;
  const uint64_t kmin = skey[base], kmax = skey[base + n - 1];
  const uint32_t sh = bucket_shift(kmax - kmin, n);
  const uint32_t *B = bkt + bkt_off[d];
  if (threadIdx.x == 0) bst = 0;
  __syncthreads();
  const uint32_t ts = tile_start[t], te = tile_start[t + 1];
  uint32_t st = 0;
  for (uint32_t i0 = ts + threadIdx.x; i0 < te; i0 += IT * blockDim.x) {
    uint32_t gi[IT], lo[IT], hi[IT];
    uint8_t kd[IT];
    uint64_t ck[IT];
    bool v[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const uint32_t i = i0 + k * blockDim.x;
      v[k] = i < te;
      gi[k] = v[k] ? base + sval[i] : base;
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {
      kd[k] = v[k] ? kind[gi[k]] : 0;
      ck[k] = v[k] ? cause_key[gi[k]] : 0;
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {
      lo[k] = hi[k] = 0;
      if (v[k] && ck[k] >= kmin && ck[k] <= kmax) {
        const uint32_t h = (uint32_t)((ck[k] - kmin) >> sh);
        lo[k] = B[h];
        hi[k] = B[h + 1];
      }
    }
    // search inside the bucket (a few ids, usually one line)
    for (bool more = true; more;) {
      more = false;
#pragma unroll
      for (int k = 0; k < IT; k++) {
        if (lo[k] < hi[k]) {
          const uint32_t m = (lo[k] + hi[k]) >> 1;
          if (skey[base + m] < ck[k]) lo[k] = m + 1; else hi[k] = m;
          more |= lo[k] < hi[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {
      if (!v[k]) continue;
      const uint32_t i = i0 + k * blockDim.x;
      const uint32_t r = i - base;
      uint32_t p = 0;
      if (r == 0) {
        if (!(kd[k] & KIND_ROOT)) st |= CW_STATUS_ROOT;
      } else {
        if (kd[k] & KIND_ROOT) st |= CW_STATUS_ROOT;
        const uint32_t c = lo[k];
        if (ck[k] < kmin || ck[k] > kmax || c >= n || skey[base + c] != ck[k])
          st |= CW_STATUS_ORPHAN;
        else if (c >= r) st |= CW_STATUS_NON_LAMPORT;
        else p = c;
      }
      par[i] = p;
      skind[i] = kd[k];
    }
  }
  if (st) atomicOr(&bst, st);
  __syncthreads();
  if (threadIdx.x == 0 && bst) atomicOr(&status[d], bst);
}

// --- one giant document: the id order and the join by a global rank directory ----
// (config 5)  Lamport ids are dense over [0, 2^key_bits): a bitmap
// over that range with a running popcount ranks every id and every cause
// directly, so the giant path's radix sort of the ids, its bucket index and
// its searching join (a random 8-byte gather of each cause by input index)
// become one pass that sets bits (atomicOr: a bit already set is a repeated
// id), a scan, and one pass in INPUT order: two directory lines read per node
// (its id's, its cause's) and par / kind / input index scattered by rank.
// Entry e covers keys [480 e, 480 e + 480): word 0 = ones before the entry,
// words 1..15 = the bits -- one 64-byte line answers "present?" and "rank".
constexpr uint32_t GD_KEYS = 480, GD_WORDS = 16;
constexpr uint32_t GD_MAX_BITS = 35;  // key range of the directory (<= 4.6 GB)

__device__ __forceinline__ void gd_split(uint64_t x, uint64_t &e, uint32_t &b) {
  e = x / GD_KEYS;
  b = (uint32_t)(x - e * GD_KEYS);
}

// rank of key x (the number of set keys below it) and whether x is set
__device__ __forceinline__ uint32_t gd_rank(const uint4 *__restrict__ dir, uint64_t x, bool &present) {
  uint64_t e;
  uint32_t b;
  gd_split(x, e, b);
  const uint4 *q = dir + e * (GD_WORDS / 4);
  const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const uint32_t w[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                          q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
  const uint32_t wi = b >> 5, bit = b & 31;
  uint32_t r = w[0], hit = 0;
#pragma unroll
  for (uint32_t k = 0; k < 15; k++) {  // (masks, no run-time index: stays in VGPRs)
    const uint32_t word = w[k + 1];
    const uint32_t m = k < wi ? 0xFFFFFFFFu : (k == wi ? (1u << bit) - 1u : 0u);
    r += __popc(word & m);
    hit |= k == wi ? (word >> bit) & 1u : 0u;
  }
  present = hit != 0;
  return r;
}

__global__ __launch_bounds__(256) void k_gd_set(const uint64_t *__restrict__ id, uint32_t n,
                                                uint64_t E, uint32_t *__restrict__ dir,
                                                unsigned long long *__restrict__ maxid,
                                                uint32_t *__restrict__ status) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t x = 0;
  bool dup = false, out = false;
  if (j < n) {
    x = id[j];
    uint64_t e;
    uint32_t b;
    gd_split(x, e, b);
    const uint32_t bit = 1u << (b & 31);
    if (e < E) dup = (atomicOr(&dir[e * GD_WORDS + 1 + (b >> 5)], bit) & bit) != 0;
    else out = true;  // an id beyond key_bits: the caller's layout is wrong
  }
  if (__ballot(out) && (threadIdx.x & 63) == 0) atomicOr(status, (uint32_t)CW_STATUS_INTERNAL);
  unsigned long long m = out ? 0ull : x;
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
  const uint64_t anydup = __ballot(dup);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(maxid, m);
    if (anydup) atomicOr(status, (uint32_t)CW_STATUS_DUP);
  }
}

// per 1024 entries: ones of each entry -> exclusive prefix inside the block
// (word 0) and the block's total
__global__ __launch_bounds__(1024) void k_gd_count(uint32_t *__restrict__ dir, uint64_t E,
                                                   uint32_t *__restrict__ sums) {
  __shared__ uint32_t wtot[16];
  const uint64_t e = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t v = 0;
  uint4 *q = reinterpret_cast<uint4 *>(dir) + e * (GD_WORDS / 4);
  if (e < E) {
    const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
    v = __popc(q0.y) + __popc(q0.z) + __popc(q0.w) + __popc(q1.x) + __popc(q1.y) + __popc(q1.z) +
        __popc(q1.w) + __popc(q2.x) + __popc(q2.y) + __popc(q2.z) + __popc(q2.w) + __popc(q3.x) +
        __popc(q3.y) + __popc(q3.z) + __popc(q3.w);
  }
  uint32_t tot;
  const uint32_t ex = block_exscan<1024>(v, wtot, &tot);
  if (e < E) dir[e * GD_WORDS] = ex;
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_gd_add(uint32_t *__restrict__ dir, uint64_t E,
                                                 const uint32_t *__restrict__ sums) {
  const uint64_t e = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  if (e < E) dir[e * GD_WORDS] += sums[blockIdx.x];
}

// The directory in ONE pass over the sorted ids (round 3's two kernels read
// them twice and wrote every entry twice, the second time as scattered 4-byte
// words: 28 ms at 2e9 nodes).  A block takes GDB_KEYS
// consecutive sorted ids and builds the entries they fall in in LDS -- one
// slot per distinct entry, bits by LDS atomics, word 0 = the index of the
// entry's first id -- then writes each as a whole 64-byte line.  Every entry
// has one writer, the block holding its first id ("lead"): ids at the start
// of a block that continue the previous block's entry are left to that block,
// which reads ahead for them (<= GD_KEYS ids).  Entries between two ids get
// word 0 = the next id's index from that id's thread.  The slots go through LDS
// GDB_SLOTS at a time (round 6: 512 ids and a slot for each, 36 KB a block,
// cleared whole -- four blocks a CU, 16 KB of ids in flight, 15.4 ms at config
// 5's 2e9 ids; config 5's ids fill ~18 entries a 512-id block).
constexpr uint32_t GDB_KEYS = 1024, GDB_SLOTS = 128;
__global__ __launch_bounds__(256) void k_gd_build(const uint64_t *__restrict__ skey, uint32_t n,
                                                  uint64_t E, uint32_t *__restrict__ dir,
                                                  uint32_t *__restrict__ status) {
  constexpr uint32_t KT = GDB_KEYS / 256;  // consecutive ids a thread
  __shared__ uint32_t sbits[GDB_SLOTS][GD_WORDS];
  __shared__ uint64_t sent[GDB_SLOTS];
  __shared__ uint32_t wtot[4];
  const uint32_t tid = threadIdx.x, i0 = blockIdx.x * GDB_KEYS;
  const uint32_t i1 = min(i0 + GDB_KEYS, n);
  auto ent = [&](uint64_t x) { return min(x / GD_KEYS, E - 1); };  // (ids past E: flagged)
  uint64_t key[KT];
  bool lead[KT];
  uint32_t nl = 0, st = 0;
  uint64_t prev = 0;  // the id before this thread's first
  {
    const uint32_t i = i0 + tid * KT;
    if (i > 0 && i < i1) prev = skey[i - 1];
  }
#pragma unroll
  for (uint32_t k = 0; k < KT; k++) {
    const uint32_t i = i0 + tid * KT + k;
    key[k] = i < i1 ? skey[i] : 0ull;
  }
#pragma unroll
  for (uint32_t k = 0; k < KT; k++) {
    const uint32_t i = i0 + tid * KT + k;
    lead[k] = false;
    if (i >= i1) continue;
    const uint64_t xp = k > 0 ? key[k - 1] : prev;
    if (i > 0 && xp == key[k]) st |= CW_STATUS_DUP;
    if (key[k] / GD_KEYS >= E) st |= CW_STATUS_INTERNAL;  // an id beyond key_bits
    const uint64_t e = ent(key[k]);
    lead[k] = i == 0 || ent(xp) != e;
    if (lead[k]) {
      nl++;
      for (uint64_t x = i == 0 ? 0 : ent(xp) + 1; x < e; x++) {  // the gap before it
        uint4 *q = reinterpret_cast<uint4 *>(dir + x * GD_WORDS);
        q[0] = make_uint4(i, 0, 0, 0);
        q[1] = q[2] = q[3] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  uint32_t nslot;
  const uint32_t s0 = block_exscan<256>(nl, wtot, &nslot);
  // an id's slot: the leads at or before it, less one; none: the previous
  // block's entry (skipped)
  uint32_t slot[KT], seen = s0;
#pragma unroll
  for (uint32_t k = 0; k < KT; k++) {
    const uint32_t i = i0 + tid * KT + k;
    if (lead[k]) seen++;
    slot[k] = seen > 0 && i < i1 ? seen - 1 : 0xFFFFFFFFu;
  }
  for (uint32_t r0 = 0; r0 < nslot; r0 += GDB_SLOTS) {
    const uint32_t ns = min(GDB_SLOTS, nslot - r0);
    for (uint32_t w = tid; w < ns * GD_WORDS; w += 256) (&sbits[0][0])[w] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < KT; k++) {
      const uint32_t q = slot[k] - r0;
      if (lead[k] && q < ns) {
        sent[q] = ent(key[k]);
        sbits[q][0] = i0 + tid * KT + k;
      }
    }
    __syncthreads();  // (word 0 before the bits' atomics of the same line)
#pragma unroll
    for (uint32_t k = 0; k < KT; k++) {
      const uint32_t q = slot[k] - r0;
      if (q < ns && key[k] / GD_KEYS < E) {
        const uint32_t b = (uint32_t)(key[k] % GD_KEYS);
        atomicOr(&sbits[q][1 + (b >> 5)], 1u << (b & 31));
      }
    }
    if (r0 + ns == nslot) {  // the next block's ids in this block's last entry
      const uint64_t elast = sent[ns - 1];
      for (uint32_t j = i1 + tid; j < n && j < i1 + GD_KEYS; j += 256) {
        const uint64_t x = skey[j];
        if (ent(x) == elast && x / GD_KEYS < E) {
          const uint32_t b = (uint32_t)(x % GD_KEYS);
          atomicOr(&sbits[ns - 1][1 + (b >> 5)], 1u << (b & 31));
        }
      }
    }
    __syncthreads();
    for (uint32_t w = tid; w < ns * GD_WORDS; w += 256) {
      const uint32_t q = w / GD_WORDS, wd = w % GD_WORDS;
      dir[sent[q] * GD_WORDS + wd] = sbits[q][wd];
    }
    __syncthreads();
  }
  const uint64_t any = __ballot(st != 0);
  if (any) {
    for (int o = 32; o > 0; o >>= 1) st |= __shfl_xor(st, o, 64);
    if ((threadIdx.x & 63) == 0) atomicOr(status, st);
  }
}

// k_join for one giant document with the directory: each rank's cause and kind
// gathered by input index (as k_join), the cause's rank from one directory
// line instead of the bucket index and a search.
constexpr int GJOIN_ITEMS = 4;
// ckk: cause | kind << 56 in one word per input node (k_gpack), so
// the gather by input index is one random line a node instead of two
__global__ __launch_bounds__(256) void k_gpack(const uint64_t *__restrict__ cause_key,
                                               const uint8_t *__restrict__ kind, uint32_t n,
                                               uint64_t *__restrict__ ckk) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  // (a cause of 2^56 or more can be no id -- the ids fit 55 bits here -- so it
  // packs as 2^56 - 1, which is above every id as well)
  constexpr uint64_t M56 = (1ull << 56) - 1;
  if (i < n) {
    const uint64_t c = cause_key[i];
    ckk[i] = (c < M56 ? c : M56) | ((uint64_t)kind[i] << 56);
  }
}

// the rank of every cause through the directory, par and kind by rank, the
// domain checks (k_gjoin, k_gjoin_r)
__device__ __forceinline__ void gjoin_items(const uint64_t (&ck)[GJOIN_ITEMS], const uint8_t (&kd)[GJOIN_ITEMS],
                                            uint32_t i0, uint32_t n, uint64_t kmax,
                                            const uint4 *__restrict__ dir, uint32_t *__restrict__ par,
                                            uint8_t *__restrict__ skind, uint32_t *__restrict__ status);

__global__ __launch_bounds__(256) void k_gjoin(const uint64_t *__restrict__ skey,
                                               const uint32_t *__restrict__ sval,
                                               const uint64_t *__restrict__ cause_key,
                                               const uint8_t *__restrict__ kind, uint32_t n,
                                               const uint64_t *__restrict__ ckk,
                                               const uint4 *__restrict__ dir, uint64_t E,
                                               uint32_t *__restrict__ par, uint8_t *__restrict__ skind,
                                               uint32_t *__restrict__ status) {
  const uint32_t i0 = blockIdx.x * (256 * GJOIN_ITEMS) + threadIdx.x;
  // causes are looked up only up to the largest id the directory holds: ids
  // past its E entries (a key_bits too small for the batch) were flagged
  // INTERNAL by the directory build and must not be read
  const uint64_t kmax = min(skey[n - 1], E * GD_KEYS - 1);
  uint32_t gi[GJOIN_ITEMS];
  uint64_t ck[GJOIN_ITEMS];
  uint8_t kd[GJOIN_ITEMS];
#pragma unroll
  for (int k = 0; k < GJOIN_ITEMS; k++) {
    const uint32_t i = i0 + k * 256;
    gi[k] = i < n ? sval[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < GJOIN_ITEMS; k++) {
    const uint32_t i = i0 + k * 256;
    if (ckk) {
      const uint64_t w = i < n ? ckk[gi[k]] : 0ull;
      ck[k] = w & ((1ull << 56) - 1);
      kd[k] = (uint8_t)(w >> 56);
    } else {
      ck[k] = i < n ? cause_key[gi[k]] : 0ull;
      kd[k] = i < n ? kind[gi[k]] : 0;
    }
  }
  gjoin_items(ck, kd, i0, n, kmax, dir, par, skind, status);
}

// k_gjoin after an id sort that carried cause and kind (OsPayload, kb key
// bits): both read in rank order, lo and hi, instead of gathered by input index
// -- a random line a node (round 5: 58 ms of config 5's 2e9 nodes)
__global__ __launch_bounds__(256) void k_gjoin_r(const uint64_t *__restrict__ skey,
                                                 const uint32_t *__restrict__ plo,
                                                 const uint32_t *__restrict__ phi, uint32_t kb,
                                                 uint32_t n, const uint4 *__restrict__ dir, uint64_t E,
                                                 uint32_t *__restrict__ par, uint8_t *__restrict__ skind,
                                                 uint32_t *__restrict__ status) {
  const uint32_t i0 = blockIdx.x * (256 * GJOIN_ITEMS) + threadIdx.x;
  const uint64_t kmax = min(skey[n - 1], E * GD_KEYS - 1);
  const uint32_t ch = os_pl_ch(kb);
  uint64_t ck[GJOIN_ITEMS];
  uint8_t kd[GJOIN_ITEMS];
#pragma unroll
  for (int k = 0; k < GJOIN_ITEMS; k++) {
    const uint32_t i = i0 + k * 256;
    const uint32_t lo = i < n ? plo[i] : 0u, hi = i < n ? phi[i] : 0u;
    ck[k] = (uint64_t)(hi & ((1u << ch) - 1)) << 32 | lo;  // (2^kb: no id, above kmax)
    kd[k] = (uint8_t)(hi >> ch);
  }
  gjoin_items(ck, kd, i0, n, kmax, dir, par, skind, status);
}

__device__ __forceinline__ void gjoin_items(const uint64_t (&ck)[GJOIN_ITEMS], const uint8_t (&kd)[GJOIN_ITEMS],
                                            uint32_t i0, uint32_t n, uint64_t kmax,
                                            const uint4 *__restrict__ dir, uint32_t *__restrict__ par,
                                            uint8_t *__restrict__ skind, uint32_t *__restrict__ status) {
  uint32_t st = 0;
#pragma unroll
  for (int k = 0; k < GJOIN_ITEMS; k++) {
    const uint32_t r = i0 + k * 256;
    if (r >= n) continue;
    uint32_t p = 0;
    if (r == 0) {
      if (!(kd[k] & KIND_ROOT)) st |= CW_STATUS_ROOT;
    } else {
      if (kd[k] & KIND_ROOT) st |= CW_STATUS_ROOT;
      bool cp = false;
      const uint32_t rc = ck[k] <= kmax ? gd_rank(dir, ck[k], cp) : 0u;
      if (!cp) st |= CW_STATUS_ORPHAN;
      else if (rc >= r) st |= CW_STATUS_NON_LAMPORT;
      else p = rc;
    }
    par[r] = p;
    skind[r] = kd[k];
  }
  const uint64_t any = __ballot(st != 0);
  if (any) {
    for (int o = 32; o > 0; o >>= 1) st |= __shfl_xor(st, o, 64);
    if ((threadIdx.x & 63) == 0) atomicOr(status, st);
  }
}

// In input order: rank of the id and of the cause, the domain checks of
// k_join, and par / kind / input index (/ the id for the yarns) by rank.
__global__ __launch_bounds__(256) void k_gd_place(
    const uint64_t *__restrict__ id, const uint64_t *__restrict__ cause,
    const uint8_t *__restrict__ kind, uint32_t n, const uint4 *__restrict__ dir,
    const unsigned long long *__restrict__ maxid, uint32_t ts_shift, uint64_t *__restrict__ max_ts,
    uint32_t *__restrict__ par, uint8_t *__restrict__ skind, uint32_t *__restrict__ sval,
    uint64_t *__restrict__ skey, uint32_t *__restrict__ status) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st = 0;
  if (j < n) {
    const uint64_t kmax = *maxid;
    const uint64_t x = min((unsigned long long)id[j], kmax), c = cause[j];  // (min: see k_gd_set)
    const uint8_t kd = kind[j];
    bool pres;
    const uint32_t r = gd_rank(dir, x, pres);
    uint32_t p = 0;
    if (r == 0) {
      if (!(kd & KIND_ROOT)) st |= CW_STATUS_ROOT;
    } else {
      if (kd & KIND_ROOT) st |= CW_STATUS_ROOT;
      bool cp = false;
      const uint32_t rc = c <= kmax ? gd_rank(dir, c, cp) : 0u;
      if (!cp) st |= CW_STATUS_ORPHAN;
      else if (rc >= r) st |= CW_STATUS_NON_LAMPORT;
      else p = rc;
    }
    if (r < n) {  // (a repeated id ranks two nodes alike: the document is flagged DUP)
      par[r] = p;
      skind[r] = kd;
      sval[r] = j;
      if (skey) skey[r] = x;
    }
    if (j == 0 && max_ts) *max_ts = kmax >> ts_shift;
  }
  const uint64_t any = __ballot(st != 0);
  if (any) {
    for (int o = 32; o > 0; o >>= 1) st |= __shfl_xor(st, o, 64);
    if ((threadIdx.x & 63) == 0) atomicOr(status, st);
  }
}

// --- front end by rank directory: id order and cause join without a sort ---------
// Lamport ids are dense: a document of n nodes from s sites has ids inside a
// range of about (max ts) * 2^site_bits keys.  A bitmap over [kmin, kmax]
// with a running popcount gives each id its rank in (sort ::nodes) directly
// (list.cljc:28) and each cause its parent rank (the join), so the two radix
// passes, the bucket index and the search disappear.  Directory layout, per
// group of 96 key values: uint4 {ones before the group, bits 0-31, 32-63,
// 64-95}; one 16-byte LDS read answers "present?" and "rank".
constexpr uint32_t FR_GROUP_BITS = 96;
constexpr uint32_t FR_BIG = 0xFFFFFFFFu;  // dgroups[d]: range too wide for a slot

__device__ __forceinline__ uint32_t fr_word(const uint4 &q, uint32_t w) {
  return w == 0 ? q.y : (w == 1 ? q.z : q.w);
}

// x = key - kmin < groups * 96.  present: bit x is set; returns the rank.
// (masks instead of picking a word by index: an indexed uint4 lands in scratch)
__device__ __forceinline__ uint32_t fr_rank(const uint4 *__restrict__ dir, uint32_t x,
                                            bool *present) {
  const uint32_t g = x / FR_GROUP_BITS, b = x - g * FR_GROUP_BITS;
  const uint4 q = dir[g];
  const uint32_t sh = b & 31, below = (1u << sh) - 1, bit = 1u << sh;
  const uint32_t m0 = b >= 32 ? 0xFFFFFFFFu : below;
  const uint32_t m1 = b >= 64 ? 0xFFFFFFFFu : (b >= 32 ? below : 0u);
  const uint32_t m2 = b >= 64 ? below : 0u;
  const uint32_t hit = b < 32 ? (q.y & bit) : (b < 64 ? (q.z & bit) : (q.w & bit));
  *present = hit != 0;
  return q.x + __popc(q.y & m0) + __popc(q.z & m1) + __popc(q.w & m2);
}

// One workgroup per document, one pass over its ids: bitmap in LDS over the
// key range [0, slot) (a bit set twice is a duplicate id, shared.cljc:166-171;
// the root [0 "0" 0] is the smallest id, so the range starts at 0 in every
// well-formed document), the largest id (::lamport-ts = max ts, refresh-ts,
// shared.cljc:243-249), group prefix counts, copy to the document's directory
// slot.  An id past the slot marks the document FR_BIG and counts it in
// big[0]; big[1] = the largest group count.
template <int NT, uint32_t U = 4>
__global__ __launch_bounds__(NT) void k_fdir(const uint64_t *__restrict__ id_key,
                                             const uint32_t *__restrict__ doc_off,
                                             uint32_t slot_groups, uint4 *__restrict__ dir,
                                             uint64_t *__restrict__ dkmin,
                                             uint32_t *__restrict__ dgroups,
                                             uint64_t *__restrict__ max_ts, uint32_t ts_shift,
                                             uint32_t *__restrict__ status,
                                             uint32_t *__restrict__ big) {
  extern __shared__ __attribute__((aligned(16))) uint4 sdir[];
  __shared__ uint64_t rmax[NT / 64];
  __shared__ uint32_t wtot[NT / 64];
  const uint32_t d = blockIdx.x, tid = threadIdx.x, base = doc_off[d];
  const uint32_t n = doc_off[d + 1] - base;
  if (n == 0) {
    if (tid == 0) dgroups[d] = 0;
    return;
  }
  for (uint32_t g = tid; g < slot_groups; g += NT) sdir[g] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  uint32_t *sw = reinterpret_cast<uint32_t *>(sdir);
  const uint64_t lim = (uint64_t)slot_groups * FR_GROUP_BITS;
  uint64_t mx = 0;
  bool dup = false, far = false;
  for (uint32_t i0 = tid; i0 < n; i0 += U * NT) {
    uint64_t x[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t i = i0 + u * NT;
      x[u] = i < n ? id_key[base + i] : 0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      if (i0 + u * NT >= n) continue;
      mx = max(mx, x[u]);
      if (x[u] >= lim) {
        far = true;
        continue;
      }
      const uint32_t xi = (uint32_t)x[u];
      const uint32_t g = xi / FR_GROUP_BITS, b = xi - g * FR_GROUP_BITS, m = 1u << (b & 31);
      const uint32_t old = atomicOr(&sw[g * 4 + 1 + (b >> 5)], m);
      dup |= (old & m) != 0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) rmax[tid >> 6] = mx;
  const bool any_far = __syncthreads_or(far);
  mx = rmax[0];
#pragma unroll
  for (int w = 1; w < NT / 64; w++) mx = max(mx, rmax[w]);
  if (tid == 0 && max_ts) max_ts[d] = mx >> ts_shift;
  if (any_far) {
    if (tid == 0) {
      dgroups[d] = FR_BIG;
      atomicAdd(&big[0], 1u);
    }
    return;
  }
  const uint32_t G = (uint32_t)(mx / FR_GROUP_BITS) + 1;
  if (tid == 0) {
    dkmin[d] = 0;
    dgroups[d] = G;
    atomicMax(&big[1], G);
  }
  // group prefix counts: each thread owns a contiguous run of groups
  const uint32_t per = (G + NT - 1) / NT, g0 = min(G, tid * per), g1 = min(G, g0 + per);
  uint32_t cnt = 0;
  for (uint32_t g = g0; g < g1; g++) {
    const uint4 q = sdir[g];
    cnt += __popc(q.y) + __popc(q.z) + __popc(q.w);
  }
  uint32_t run = block_exscan<NT>(cnt, wtot, nullptr);
  for (uint32_t g = g0; g < g1; g++) {
    const uint4 q = sdir[g];
    sw[g * 4] = run;
    run += __popc(q.y) + __popc(q.z) + __popc(q.w);
  }
  __syncthreads();
  uint4 *out = dir + (size_t)d * slot_groups;
  for (uint32_t g = tid; g < G; g += NT) out[g] = sdir[g];
  if (__syncthreads_or(dup) && tid == 0) atomicOr(&status[d], (uint32_t)CW_STATUS_DUP);
}

// Pass 1, per tile (XCD-contiguous like the sort tiles): stage the document's
// directory in LDS, rank every node and its cause, and do the domain checks
// of s/insert (shared.cljc:163-178): root at rank 0 only, cause present
// (orphan), cause older than the node (lamport).  A random 4-byte store per
// node into the rank-ordered arrays would cost a partial line each, so the
// tile is sorted in LDS by rank window (rank >> 12, a window = the ranks of
// one tile) and written out coalesced as records: meta = rank & 4095 |
// (tile-local index) << 12 | class << 24, and the cause rank.  woff[t][w] =
// start of window w's records inside tile t.
template <int NT>
__global__ __launch_bounds__(NT) void k_frank(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause_key,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ tile_start,
    const uint32_t *__restrict__ tile_doc, const uint32_t *__restrict__ tile_first,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ woff_base,
    const uint4 *__restrict__ dir, uint32_t slot_groups, const uint64_t *__restrict__ dkmin,
    const uint32_t *__restrict__ dgroups, uint32_t *__restrict__ rec_meta,
    uint32_t *__restrict__ rec_par, uint32_t *__restrict__ woff, uint32_t *__restrict__ status) {
  constexpr uint32_t IT = TILE / NT;
  // the directory, then (once every node is ranked) the tile's records: the
  // dynamic LDS is max(directory, 2 * TILE words) so 4 blocks fit on a CU
  extern __shared__ __attribute__((aligned(16))) uint4 sdir[];
  uint32_t *st_meta = reinterpret_cast<uint32_t *>(sdir), *st_par = st_meta + TILE;
  __shared__ uint32_t wcnt[NT / 64][SUB_BINS];
  __shared__ uint32_t run[64];
  __shared__ uint32_t bst;
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), d = tile_doc[t], tid = threadIdx.x;
  const uint32_t nwin = tile_first[d + 1] - tile_first[d];
  const uint32_t wbits = nwin <= 1 ? 0u : 32u - __clz(nwin - 1);  // <= 6
  const uint32_t G = dgroups[d];
  const uint64_t kmin = dkmin[d], xend = (uint64_t)G * FR_GROUP_BITS;
  const uint4 *src = dir + (size_t)d * slot_groups;
  // the tile's nodes are loaded while the directory is staged
  const uint32_t s = tile_start[t], len = tile_start[t + 1] - s;
  uint64_t k[IT], c[IT];
  uint8_t kd[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t j = wb_elem<IT>(u);
    k[u] = j < len ? id_key[s + j] : kmin;
    c[u] = j < len ? cause_key[s + j] : 0;
    kd[u] = j < len ? kind[s + j] : 0;
  }
  for (uint32_t g = tid; g < G; g += NT) sdir[g] = src[g];
  if (tid == 0) bst = 0;
  __syncthreads();
  uint32_t st = 0, meta[IT], pr[IT], sd[IT], pos[IT];
#pragma unroll
  for (uint32_t u = 0; u < IT; u++) {
    const uint32_t j = wb_elem<IT>(u);
    bool pres;
    const uint32_t r = fr_rank(sdir, (uint32_t)(k[u] - kmin), &pres);
    uint32_t p = 0;
    if (j < len) {
      if (r == 0) {
        if (!(kd[u] & KIND_ROOT)) st |= CW_STATUS_ROOT;
      } else {
        if (kd[u] & KIND_ROOT) st |= CW_STATUS_ROOT;
        const uint64_t cx = c[u] - kmin;
        bool cp = false;
        uint32_t cr = 0;
        if (c[u] >= kmin && cx < xend) cr = fr_rank(sdir, (uint32_t)cx, &cp);
        if (!cp) st |= CW_STATUS_ORPHAN;
        else if (c[u] >= k[u]) st |= CW_STATUS_NON_LAMPORT;
        else p = cr;
      }
    }
    meta[u] = (r & (TILE - 1)) | (j << 12) | ((uint32_t)(kd[u] & KIND_CLASS) << 24);
    pr[u] = p;
    sd[u] = min(r >> 12, nwin - 1);  // duplicates can push ranks past the end
  }
  if (wbits) {
    rank_subdigit<NT, IT>(sd, len, wbits, pos, wcnt, run);  // barriers: the directory is free
  } else {
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) pos[u] = wb_elem<IT>(u);
    if (tid == 0) run[0] = 0;
    __syncthreads();
  }
#pragma unroll
  for (uint32_t u = 0; u < IT; u++)
    if (wb_elem<IT>(u) < len) {
      st_meta[pos[u]] = meta[u];
      st_par[pos[u]] = pr[u];
    }
  if (st) atomicOr(&bst, st);
  __syncthreads();
  uint32_t *wo = woff + woff_base[t];
  for (uint32_t w = tid; w <= nwin; w += NT) wo[w] = w < nwin ? (wbits ? run[w] : 0u) : len;
  for (uint32_t j = tid; j < len; j += NT) {
    rec_meta[s + j] = st_meta[j];
    rec_par[s + j] = st_par[j];
  }
  if (tid == 0 && bst) atomicOr(&status[d], bst);
}

constexpr uint32_t KBM_WORDS = 2 * TILE / 32;  // per tile: special bits, then hide bits
constexpr uint32_t FRONT_FUSED_SG = 2560;       // k_front's directory: 40 KiB, 245,760 keys

// Pass 2, one block per window (window w of document d covers ranks
// [4096 w, 4096 (w+1)), the ranks of tile w): gather the window's records from
// every tile of the document (one contiguous run each), place them by rank in
// LDS and write sval (input index), par (cause rank), skind and, for the yarn
// sort, skey in rank order, coalesced.
template <int NT>
__global__ __launch_bounds__(NT) void k_fplace(
    const uint32_t *__restrict__ rec_meta, const uint32_t *__restrict__ rec_par,
    const uint32_t *__restrict__ woff, const uint32_t *__restrict__ woff_base,
    const uint32_t *__restrict__ tile_start, const uint32_t *__restrict__ tile_doc,
    const uint32_t *__restrict__ tile_first, const uint32_t *__restrict__ doc_off,
    const uint64_t *__restrict__ id_key, uint32_t *__restrict__ sval, uint32_t *__restrict__ par,
    uint8_t *__restrict__ skind, uint64_t *__restrict__ skey, uint32_t *__restrict__ kbm) {
  __shared__ uint32_t s_val[TILE], s_par[TILE];
  __shared__ uint8_t s_kind[TILE];
  __shared__ uint32_t s_run[65], s_src[64];
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), d = tile_doc[t], tid = threadIdx.x;
  const uint32_t t0 = tile_first[d], ntile = tile_first[d + 1] - t0, w = t - t0;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base;
  const uint32_t r0 = w << 12, wlen = min(TILE, n - r0);
  if (tid < 64) {  // run lengths of this window in every tile, prefix in LDS
    uint32_t a = 0, l = 0;
    if (tid < ntile) {
      const uint32_t *wo = woff + woff_base[t0 + tid];
      a = wo[w];
      l = wo[w + 1] - a;
      s_src[tid] = tile_start[t0 + tid] + a;
    }
    uint32_t x = l;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (tid >= (uint32_t)o) x += y;
    }
    s_run[tid + 1] = x;
    if (tid == 0) s_run[0] = 0;
  }
  for (uint32_t j = tid; j < wlen; j += NT) {
    s_val[j] = 0;
    s_par[j] = 0;
    s_kind[j] = 0;
  }
  __syncthreads();
  const uint32_t total = min(s_run[ntile], wlen);
  for (uint32_t j = tid; j < total; j += NT) {
    uint32_t lo = 0, hi = ntile;  // last tile whose run starts at or before j
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if (s_run[m] <= j) lo = m; else hi = m;
    }
    const uint32_t g = s_src[lo] + (j - s_run[lo]);
    const uint32_t meta = rec_meta[g], rr = meta & (TILE - 1);
    s_val[rr] = (lo << 12) | ((meta >> 12) & (TILE - 1));
    s_par[rr] = rec_par[g];
    s_kind[rr] = (uint8_t)(meta >> 24);
  }
  __syncthreads();
  for (uint32_t j = tid; j < wlen; j += NT) {
    const uint32_t v = s_val[j];
    sval[base + r0 + j] = v;
    par[base + r0 + j] = s_par[j];
    skind[base + r0 + j] = s_kind[j];
    if (skey) skey[base + r0 + j] = id_key[base + (v < n ? v : 0u)];
  }
  // special and hide bits of the window's ranks (KBM_WORDS per tile) for k_tree
  for (uint32_t j0 = (tid >> 6) << 6; j0 < TILE; j0 += NT) {
    const uint32_t j = j0 + (tid & 63);
    const uint8_t k = j < wlen ? s_kind[j] : 0;
    const uint64_t sm = __ballot(is_special(k)), hm = __ballot(is_hide(k));
    if ((tid & 63) == 0) {
      uint32_t *o = kbm + (size_t)t * KBM_WORDS + (j0 >> 5);
      o[0] = (uint32_t)sm;
      o[1] = (uint32_t)(sm >> 32);
      o[TILE / 32] = (uint32_t)hm;
      o[TILE / 32 + 1] = (uint32_t)(hm >> 32);
    }
  }
}

// --- fused front end for documents of < 2^16 nodes (one workgroup per document) --
// k_fdir + k_frank + k_fplace in one pass over LDS: the rank directory of the
// document, then every node's rank and cause rank (s/insert's checks,
// shared.cljc:163-178) with par (u16) and the class bits placed by rank in LDS;
// par, skind and the per-tile special/hide bitmaps are written out coalesced;
// then the input index of every rank (sval, u16 in LDS) from the ranks kept in
// a u16 scratch.  No window records, no second kernel.  A document whose ids
// leave the directory slot counts in big[0] and the host reruns the batch on
// the three-kernel front end.  LDS: front_lds_bytes().
__host__ __device__ inline uint32_t front_lds_bytes(uint32_t nmax, uint32_t sg) {
  return sg * 16 + 4 * ((nmax + 1) / 2) + 8 * ((nmax + 31) / 32);
}

// one document d (the whole workgroup); lds: the dynamic LDS.  Returns false
// when the document's ids leave the directory (big[0] counts it).  PT / VT:
// the width of par / sval (u16 inside k_weave_doc: n < 2^16); skind may be
// null (the tree reads the class bitmaps).
// U1 / U2 / U3: items a thread keeps in flight in the directory, rank and
// input-index passes (the fused kernel's front end is latency-bound: CW_FRONT_U)
// Where the fused front end writes the yarns' site bytes (round 6 A/B).
#ifndef CW_SITE8_RANKPASS
#define CW_SITE8_RANKPASS 0
#endif
constexpr bool SITE8_PASS1 = CW_SITE8_RANKPASS == 0;

template <int NT, typename PT = uint32_t, typename VT = uint32_t, uint32_t U1 = 4, uint32_t U2 = 4,
          uint32_t U3 = 4>
__device__ __forceinline__ bool front_doc(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause_key,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ tile_first, uint32_t sg, PT *__restrict__ par,
    uint8_t *__restrict__ skind, VT *__restrict__ sval, uint32_t *__restrict__ kbm,
    uint64_t *__restrict__ skey, uint16_t *rank16, uint64_t *__restrict__ max_ts, uint32_t ts_shift,
    uint32_t *__restrict__ status, uint32_t *__restrict__ big,
    unsigned long long *__restrict__ tprof, uint32_t d, uint4 *sdir,
    uint8_t *__restrict__ site8 = nullptr, uint32_t site_shift = 0, uint32_t site_mask = 0) {
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = 0;
  auto stamp = [&](int ph) {  // diagnostic phase times (CW_TREE_PROF)
    if (tprof) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tacc[ph] += now - tlast;
      tlast = now;
    }
  };
  stamp(-1);
  __shared__ uint64_t rmax[NT / 64];
  __shared__ uint32_t wtot[NT / 64];
  __shared__ uint32_t bst;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, nw = (n + 31) / 32;
  const uint64_t *const idD = id_key + base, *const causeD = cause_key + base;
  const uint8_t *const kindD = kind + base;
  uint16_t *const rankD = rank16 + base;
  PT *const parD = par + base;
  VT *const svalD = sval + base;
  uint8_t *const skindD = skind ? skind + base : nullptr;
  if (n == 0) return true;
  uint32_t *sw = reinterpret_cast<uint32_t *>(sdir);
  uint16_t *p16 = reinterpret_cast<uint16_t *>(sdir + sg);  // par, then sval, by rank
  uint32_t *clsA = reinterpret_cast<uint32_t *>(p16) + (n + 1) / 2, *clsB = clsA + nw;
  for (uint32_t g = tid; g < sg; g += NT) sdir[g] = make_uint4(0u, 0u, 0u, 0u);
  for (uint32_t w = tid; w < nw; w += NT) clsA[w] = clsB[w] = 0;
  if (tid == 0) bst = 0;
  __syncthreads();
  // 1. directory bits over [0, slot) (the root, ts 0, is the smallest id)
  const uint64_t lim = (uint64_t)sg * FR_GROUP_BITS;
  uint64_t mx = 0;
  bool dup = false, far = false;
  for (uint32_t i0 = tid; i0 < n; i0 += U1 * NT) {
    uint64_t x[U1];
#pragma unroll
    for (uint32_t u = 0; u < U1; u++) {
      const uint32_t i = i0 + u * NT;
      x[u] = i < n ? lane_at(idD, i) : 0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < U1; u++) {
      if (i0 + u * NT >= n) continue;
      mx = max(mx, x[u]);
      // the site of every input for the yarns (k_yarn_doc): one coalesced byte,
      // written in this pass, whose loads are few and early (CW_SITE8_RANKPASS = 1
      // at build time: in the rank pass, as round 5 had it)
      if (SITE8_PASS1 && site8) lane_at(site8 + base, i0 + u * NT) = (uint8_t)((x[u] >> site_shift) & site_mask);
      if (x[u] >= lim) {
        far = true;
        continue;
      }
      const uint32_t xi = (uint32_t)x[u];
      const uint32_t g = xi / FR_GROUP_BITS, b = xi - g * FR_GROUP_BITS, m = 1u << (b & 31);
      // no returned value (a non-returning LDS atomic): a repeated id shows as
      // fewer directory bits than ids, counted below
      atomicOr(&sw[g * 4 + 1 + (b >> 5)], m);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, o, 64));
  if (lane == 0) rmax[tid >> 6] = mx;
  const bool any_far = __syncthreads_or(far);
  mx = rmax[0];
#pragma unroll
  for (int w = 1; w < NT / 64; w++) mx = max(mx, rmax[w]);
  if (tid == 0 && max_ts) max_ts[d] = mx >> ts_shift;
  if (any_far) {
    if (tid == 0) atomicAdd(&big[0], 1u);
    return false;
  }
  stamp(0);
  const uint32_t G = (uint32_t)(mx / FR_GROUP_BITS) + 1;
  {  // group prefix counts
    const uint32_t per = (G + NT - 1) / NT, g0 = min(G, tid * per), g1 = min(G, g0 + per);
    uint32_t cnt = 0;
    for (uint32_t g = g0; g < g1; g++) {
      const uint4 q = sdir[g];
      cnt += __popc(q.y) + __popc(q.z) + __popc(q.w);
    }
    uint32_t distinct;
    uint32_t run = block_exscan<NT>(cnt, wtot, &distinct);
    dup = distinct != n;  // every id is < lim here: one bit per distinct id
    for (uint32_t g = g0; g < g1; g++) {
      const uint4 q = sdir[g];
      sw[g * 4] = run;
      run += __popc(q.y) + __popc(q.z) + __popc(q.w);
    }
  }
  __syncthreads();
  // 2. ranks, checks, par and class bits by rank
  const uint64_t xend = (uint64_t)G * FR_GROUP_BITS;
  uint32_t st = 0;
  // the next group's loads are issued before this group is ranked
  uint64_t qk[U2], qc[U2];
  uint8_t qd[U2];
  auto load_group = [&](uint32_t i0) {
#pragma unroll
    for (uint32_t u = 0; u < U2; u++) {
      const uint32_t i = i0 + u * NT;
      qk[u] = i < n ? lane_at(idD, i) : 0ull;
      qc[u] = i < n ? lane_at(causeD, i) : 0ull;
      qd[u] = i < n ? lane_at(kindD, i) : 0;
    }
  };
  // (U2 <= 4: the next group's loads go out before this group is ranked;
  // wider groups load and rank in turn -- double-buffered they spill)
  constexpr bool PF = U2 <= 4;
  if (PF) load_group(tid);
  for (uint32_t i0 = tid; i0 < n; i0 += U2 * NT) {
    uint64_t k[U2], c[U2];
    uint8_t kd[U2];
    if (!PF) load_group(i0);
#pragma unroll
    for (uint32_t u = 0; u < U2; u++) {
      k[u] = qk[u];
      c[u] = qc[u];
      kd[u] = qd[u];
    }
    if (PF && i0 + U2 * NT < n) load_group(i0 + U2 * NT);
#pragma unroll
    for (uint32_t u = 0; u < U2; u++) {
      const uint32_t i = i0 + u * NT;
      if (i >= n) continue;
      bool pres;
      const uint32_t r = fr_rank(sdir, (uint32_t)k[u], &pres);
      uint32_t p = 0;
      if (r == 0) {
        if (!(kd[u] & KIND_ROOT)) st |= CW_STATUS_ROOT;
      } else {
        if (kd[u] & KIND_ROOT) st |= CW_STATUS_ROOT;
        bool cp = false;
        uint32_t cr = 0;
        if (c[u] < xend) cr = fr_rank(sdir, (uint32_t)c[u], &cp);
        if (!cp) st |= CW_STATUS_ORPHAN;
        else if (c[u] >= k[u]) st |= CW_STATUS_NON_LAMPORT;
        else p = cr;
      }
      if (r < n) {  // (duplicates can push ranks past the end; flagged above)
        p16[r] = (uint16_t)p;
        const uint32_t cls = kd[u] & KIND_CLASS;
        if (cls & 1) atomicOr(&clsA[r >> 5], 1u << (r & 31));
        if (cls & 2) atomicOr(&clsB[r >> 5], 1u << (r & 31));
      }
      lane_at(rankD, i) = (uint16_t)min(r, 0xFFFFu);
      // the site of every input for the yarns (k_yarn_doc): one coalesced byte
      if (!SITE8_PASS1 && site8) lane_at(site8 + base, i) = (uint8_t)((k[u] >> site_shift) & site_mask);
    }
  }
  if (st) atomicOr(&bst, st);
  __syncthreads();
  stamp(1);
  // par, skind, special/hide bitmaps per 4096-rank tile, coalesced
  for (uint32_t r = tid; r < n; r += NT) {
    const uint32_t p = p16[r];
    lane_at(parD, r) = (PT)p;
    const uint32_t a = (clsA[r >> 5] >> (r & 31)) & 1u, b = (clsB[r >> 5] >> (r & 31)) & 1u;
    if (skindD) lane_at(skindD, r) = (uint8_t)(a | (b << 1));  // the class, as k_fplace writes it
  }
  uint32_t *kb = kbm + (size_t)tile_first[d] * KBM_WORDS;
  for (uint32_t w = tid; w < nw; w += NT) {  // word w of the document = word w & 127 of tile w >> 7
    const uint32_t a = clsA[w], b = clsB[w];
    uint32_t *o = kb + (size_t)(w >> 7) * KBM_WORDS + (w & 127);
    o[0] = a | b;            // special
    o[TILE / 32] = a ^ b;    // hide / h.hide
  }
  if (tid == 0 && bst) atomicOr(&status[d], bst);
  // documents for the exact path (exact.hip): counted here, read back with big[0]
  if (tid == 0 && (bst & (CW_STATUS_ROOT | CW_STATUS_ORPHAN | CW_STATUS_NON_LAMPORT)))
    atomicAdd(&big[1], 1u);
  if (__syncthreads_or(dup) && tid == 0) atomicOr(&status[d], (uint32_t)CW_STATUS_DUP);
  stamp(2);
  // 3. the input index of every rank (the rank scratch was written by this
  // workgroup: one CU, one L1, lines not cached before; the barrier orders it)
  for (uint32_t i0 = tid; i0 < n; i0 += U3 * NT) {
    uint32_t r[U3];
#pragma unroll
    for (uint32_t u = 0; u < U3; u++) {
      const uint32_t i = i0 + u * NT;
      r[u] = i < n ? lane_at(rankD, i) : 0xFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < U3; u++)
      if (r[u] < n) p16[r[u]] = (uint16_t)(i0 + u * NT);
  }
  __syncthreads();
  stamp(3);
  for (uint32_t r = tid; r < n; r += NT) lane_at(svalD, r) = (VT)p16[r];
  if (skey) {
    // the ids in rank order (the yarns sort by them) straight from the
    // directory: group g's set bits are ids g * FR_GROUP_BITS + b, ranked from
    // its word 0 on -- no gather of idD by input index (a random 8-byte read
    // a node: the front end of a yarns call took 2.9x as long)
    const uint32_t per = (G + NT - 1) / NT, g0 = min(G, tid * per), g1 = min(G, g0 + per);
    for (uint32_t g = g0; g < g1; g++) {
      const uint4 q = sdir[g];
      uint32_t r = q.x;
      const uint32_t wv[3] = {q.y, q.z, q.w};
#pragma unroll
      for (uint32_t k = 0; k < 3; k++)
        for (uint32_t m = wv[k]; m != 0 && r < n; m &= m - 1)
          skey[base + r++] = (uint64_t)g * FR_GROUP_BITS + 32 * k + (uint32_t)(__ffs(m) - 1);
    }
  }
  stamp(4);
  if (tprof && tid == 0)
    for (int ph = 0; ph < 6; ph++) tprof[(size_t)d * 8 + ph] = tacc[ph];
  return true;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_front(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause_key,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ tile_first, uint32_t sg, uint32_t *__restrict__ par,
    uint8_t *__restrict__ skind, uint32_t *__restrict__ sval, uint32_t *__restrict__ kbm,
    uint64_t *__restrict__ skey, uint16_t *rank16, uint64_t *__restrict__ max_ts, uint32_t ts_shift,
    uint32_t *__restrict__ status, uint32_t *__restrict__ big,
    unsigned long long *__restrict__ tprof, uint32_t doc0 = 0) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_fr[];
  front_doc<NT>(id_key, cause_key, kind, doc_off, tile_first, sg, par, skind, sval, kbm, skey, rank16,
                max_ts, ts_shift, status, big, tprof, doc0 + blockIdx.x, lds_fr);
}

// dst bits [off, off + nbits) |= src bits [0, nbits) (dst zeroed beforehand).
__global__ __launch_bounds__(256) void k_or_bits_at(const uint32_t *__restrict__ src, uint32_t nbits,
                                                    uint32_t *__restrict__ dst, uint32_t off) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i * 32 >= nbits) return;
  uint32_t x = src[i];
  const uint32_t len = min(32u, nbits - i * 32);
  if (len < 32) x &= (1u << len) - 1;
  if (!x) return;
  const uint32_t p = off + i * 32, w = p >> 5, sh = p & 31;
  atomicOr(&dst[w], x << sh);
  if (sh) {
    const uint32_t hi = x >> (32 - sh);
    if (hi) atomicOr(&dst[w + 1], hi);
  }
}

// --- tree: effective parents, sibling order, links (one workgroup per document) --
// Effective parent: a special keeps its cause, a non-special climbs
// through special causes.  Siblings are ordered specials by descending id, then
// non-specials by descending id (weave-later?, shared.cljc:202-223): with the
// group key (eff parent, class) the next sibling of r is the previous node of
// the same group in rank order, and the first child is the group's last node.
// Ranks are swept in tiles of TILE_T ranks: each tile is sorted by group key in
// LDS (stable), neighbours inside the tile link directly, and a per-group
// "last node so far" table (fcS/fcN, which ends as the first-child table)
// links across tiles.  A second sweep assembles the link word the walk uses.
template <int NT, int TILE_T>
__global__ __launch_bounds__(NT) void k_tree(
    const uint32_t *__restrict__ par, const uint8_t *__restrict__ skind,
    const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ doc_log2k, uint32_t kbits, uint32_t bm_words,
    uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
    uint32_t *__restrict__ fcN, uint32_t *__restrict__ thr, uint32_t *__restrict__ link,
    uint32_t *__restrict__ status, unsigned long long *__restrict__ tprof,
    const uint32_t *__restrict__ kbm, const uint32_t *__restrict__ tile_first) {
  constexpr uint32_t IT = TILE_T / NT;
  // diagnostic phase stamps (tprof != nullptr only under CW_TREE_PROF)
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
  auto stamp = [&](int ph) {
    if (tprof) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tacc[ph] += now - tlast;
      tlast = now;
    }
  };
  stamp(-1);
  __shared__ uint32_t tkey[TILE_T], trank[TILE_T], tns[TILE_T];
  // ptab[x] (the group's last node of earlier tiles, by original position) is
  // read by the thread that then writes tns[x]: the two share one array
  uint32_t *const ptab = tns;
  __shared__ uint32_t wcnt[NT / 64][SUB_BINS];
  __shared__ uint32_t run[64];
  // special / hide bit per rank (LDS when the document fits bm_words words)
  extern __shared__ __attribute__((aligned(16))) uint32_t bm[];
  const uint32_t d = blockIdx.x, tid = threadIdx.x;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, log2k = doc_log2k[d];
  const bool in_lds = ((n + 31) >> 5) <= bm_words;
  uint32_t *spec_bm = bm, *hide_bm = bm + bm_words;
  if (in_lds && kbm) {
    // the front end wrote both bitmaps per 4096-rank tile: coalesced word loads
    const uint32_t *src = kbm + (size_t)tile_first[d] * KBM_WORDS;
    for (uint32_t wi = tid; wi < ((n + 31) >> 5); wi += NT) {
      const uint32_t *tw = src + (size_t)(wi >> 7) * KBM_WORDS + (wi & 127);
      spec_bm[wi] = tw[0];
      hide_bm[wi] = tw[TILE / 32];
    }
    __syncthreads();
  } else if (in_lds) {
    // one ballot per wave per 64 ranks: bit r of the bitmap = special(rank r);
    // eight loads in flight per lane
    constexpr uint32_t BU = 8;
    for (uint32_t rb = (tid >> 6) << 6; rb < n; rb += NT * BU) {
      uint8_t kd[BU];
#pragma unroll
      for (uint32_t u = 0; u < BU; u++) {
        const uint32_t r = rb + u * NT + (tid & 63);
        kd[u] = r < n ? skind[base + r] : 0;
      }
#pragma unroll
      for (uint32_t u = 0; u < BU; u++) {
        const uint32_t r0 = rb + u * NT, r = r0 + (tid & 63);
        const uint64_t sm = __ballot(r < n && is_special(kd[u]));
        const uint64_t hm = __ballot(r < n && is_hide(kd[u]));
        if ((tid & 63) == 0 && r0 < n) {
          spec_bm[r0 >> 5] = (uint32_t)sm;
          hide_bm[r0 >> 5] = (uint32_t)hm;
          if ((r0 >> 5) + 1 < bm_words) {
            spec_bm[(r0 >> 5) + 1] = (uint32_t)(sm >> 32);
            hide_bm[(r0 >> 5) + 1] = (uint32_t)(hm >> 32);
          }
        }
      }
    }
    __syncthreads();
  }
  stamp(0);
  auto special_at = [&](uint32_t r) -> bool {
    return in_lds ? ((spec_bm[r >> 5] >> (r & 31)) & 1u) : is_special(skind[base + r]);
  };
  auto hide_at = [&](uint32_t r) -> bool {
    return in_lds ? ((hide_bm[r >> 5] >> (r & 31)) & 1u) : is_hide(skind[base + r]);
  };
  // parents of the next tile are loaded while this tile is sorted
  uint32_t qpar[IT];
  auto load_par = [&](uint32_t r0) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t r = r0 + wb_elem<IT>(k);
      qpar[k] = r < n ? par[base + r] : 0u;
    }
  };
  load_par(0);
  for (uint32_t r0 = 0; r0 < n; r0 += TILE_T) {
    const uint32_t len = min((uint32_t)TILE_T, n - r0);
    uint32_t key[IT], rk[IT], sd[IT], pos[IT], cpar[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) cpar[k] = qpar[k];
    if (r0 + TILE_T < n) load_par(r0 + TILE_T);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k), r = r0 + j;
      key[k] = 0;
      rk[k] = j;
      if (j < len) {
        // this node's own "last child" entries start empty (its children come
        // later in rank order; the sort's barriers order this before their use)
        fcS[base + r] = 0;
        fcN[base + r] = 0;
      }
      if (j < len && r > 0) {
        const bool sp = special_at(r);
        // causes are older (c < r); the clamps only keep out-of-domain
        // documents (duplicate ids leave ranks unwritten) in bounds
        uint32_t c = cpar[k];
        c = c < r ? c : 0u;
        if (!sp)
          while (c != 0 && special_at(c)) {
            const uint32_t pc = par[base + c];
            c = pc < c ? pc : 0u;
          }
        key[k] = ((c + 1) << 1) | (sp ? 0u : 1u);
      }
    }
    // the group's last node of earlier tiles, loaded now so the load overlaps
    // the sort (earlier tiles' updates are complete: barrier at tile end); a
    // parent inside this tile has no children in earlier tiles (and its
    // entries were only just cleared above)
    uint32_t ptv[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t kk = key[k], e = (kk >> 1) - 1;
      ptv[k] = (kk && e < r0) ? ((kk & 1) ? fcN : fcS)[base + e] : 0u;
    }
    stamp(1);
    // stable LDS sort of the tile by group key, 6 bits per sub-pass
    for (uint32_t shift = 0; shift < kbits; shift += SUB_BITS) {
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) sd[k] = (key[k] >> shift) & (SUB_BINS - 1);
      rank_subdigit<NT, IT>(sd, len, min(SUB_BITS, kbits - shift), pos, wcnt, run);
#pragma unroll
      for (uint32_t k = 0; k < IT; k++)
        if (wb_elem<IT>(k) < len) {
          tkey[pos[k]] = key[k];
          trank[pos[k]] = rk[k];
        }
      if (shift + SUB_BITS >= kbits) {
#pragma unroll
        for (uint32_t k = 0; k < IT; k++) ptab[wb_elem<IT>(k)] = ptv[k];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = wb_elem<IT>(k);
        if (j < len) {
          key[k] = tkey[j];
          rk[k] = trank[j];
        }
      }
      __syncthreads();
    }
    stamp(2);
    // next sibling inside the class: previous node of the group; a group's
    // first node in the tile takes the group's last node of earlier tiles
    uint32_t prv[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k);
      const uint32_t kk = key[k];
      prv[k] = 0;
      if (j < len && kk != 0) {
        if (j > 0 && tkey[j - 1] == kk) {
          prv[k] = r0 + trank[j - 1];
        } else {
          prv[k] = ptab[rk[k]];
        }
      }
    }
    // nsc = next sibling, or NSC_UP | effective parent for a group's oldest
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
      if (wb_elem<IT>(k) < len) tns[rk[k]] = prv[k] ? prv[k] : (NSC_UP | ((key[k] >> 1) - 1));
    __syncthreads();  // every group's old "last" is read before it is replaced
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k);
      if (j >= len) continue;
      const uint32_t kk = key[k];
      if (kk != 0 && !(j + 1 < len && tkey[j + 1] == kk)) {
        uint32_t *tab = (kk & 1) ? fcN : fcS;
        tab[base + (kk >> 1) - 1] = r0 + rk[k];
      }
    }
    for (uint32_t j = tid; j < len; j += NT) nsc[base + r0 + j] = tns[j];
    __syncthreads();
    stamp(3);
  }
  // the sweep below reads what this workgroup wrote above: all waves of a
  // workgroup share one CU and its L1, so the barrier's workgroup-scope
  // ordering is enough (agent-scope accesses would push every line to L2)
  __syncthreads();
  // Preorder successor of every node: its first child, else its thread = the
  // next sibling of the nearest ancestor-or-self that has one (SUCC_END for
  // the last node).  thr(r) = ns(r) ?: thr(e(r)), and e(r) < r, so a
  // sweep in rank order resolves each tile from earlier tiles' threads (thr,
  // global) plus pointer jumping over the tile's own parents in LDS.
  constexpr uint32_t RES = 0x80000000u;
  // T: this tile's threads (pointer jumping); P: the previous tile's resolved
  // threads, so a parent in the previous tile needs no global read.  The next
  // tile's fcS/fcN/nsc are loaded while this tile is resolved.
  uint32_t *T = tkey, *P = trank;
  uint32_t qfs[IT], qfn[IT], qns[IT];
  auto load_tile = [&](uint32_t r0) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t r = r0 + k * NT + tid;
      const bool ok = r < n;
      qfs[k] = ok ? fcS[base + r] : 0u;
      qfn[k] = ok ? fcN[base + r] : 0u;
      qns[k] = ok ? nsc[base + r] : 0u;
    }
  };
  // loads that depend on a node's nsc, issued one tile ahead: the newest
  // non-special of a last special's parent, and the thread of a parent two or
  // more tiles back (both final by then)
  uint32_t dfn[IT], dth[IT];
  auto load_dep = [&](uint32_t r0) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t r = r0 + k * NT + tid, ns = qns[k], e = ns & ~NSC_UP;
      const bool up = r < n && r > 0 && (ns & NSC_UP);
      dfn[k] = up && special_at(r) ? fcN[base + e] : 0u;
      dth[k] = up && e + TILE_T < r0 ? thr[base + e] : 0u;
    }
  };
  load_tile(0);
  load_dep(0);
  for (uint32_t r0 = 0; r0 < n; r0 += TILE_T) {
    const uint32_t len = min((uint32_t)TILE_T, n - r0);
    uint32_t fs4[IT], ns4[IT], fcr[IT], flg[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      fs4[k] = qfs[k];
      fcr[k] = qfs[k] ? qfs[k] : qfn[k];
      ns4[k] = qns[k];
    }
    if (r0 + TILE_T < n) load_tile(r0 + TILE_T);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid, r = r0 + j;
      flg[k] = 0;
      if (j >= len) continue;
      const bool sp = special_at(r);
      uint32_t tv;
      if (r == 0) {
        tv = RES | SUCC_END;
      } else {
        uint32_t ns = ns4[k], e = 0;
        if (ns & NSC_UP) {
          e = ns & ~NSC_UP;
          ns = sp ? dfn[k] : 0u;  // last special -> newest non-special
        }
        if (ns) tv = RES | ns;
        else if (e >= r0) tv = e - r0;
        else if (e + TILE_T >= r0) tv = P[e + TILE_T - r0];
        else tv = RES | dth[k];
      }
      T[j] = tv;
      // after a non-special comes its first child, which is its
      // newest special child when it has one.
      const uint32_t fs = fs4[k];
      const bool vis = !sp && r != 0 && !(fs && hide_at(fs));
      const bool split = r == split_node(d, r >> log2k, log2k, n);
      flg[k] = (vis ? LINK_VIS : 0u) | (split ? LINK_SPLIT : 0u);
    }
    __syncthreads();
    stamp(4);
    for (;;) {  // pointer jumping: every value stays an ancestor's thread or pointer
      bool open = false;
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = k * NT + tid;
        if (j < len) {
          const uint32_t t0 = T[j];
          if (!(t0 & RES)) {
            const uint32_t t1 = T[t0];
            T[j] = t1;
            open |= !(t1 & RES);
          }
        }
      }
      if (!__syncthreads_or(open)) break;
    }
    stamp(5);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid, r = r0 + j;
      if (j >= len) continue;
      const uint32_t th = T[j] & ~RES;
      thr[base + r] = th;
      link[base + r] = (fcr[k] ? fcr[k] : th) | flg[k];
    }
    __syncthreads();
    stamp(6);
    uint32_t *x = T;  // this tile's resolved threads become the previous tile's
    T = P;
    P = x;
    if (r0 + TILE_T < n) load_dep(r0 + TILE_T);
  }
  if (tprof && tid == 0)
    for (int ph = 0; ph < 8; ph++) tprof[(size_t)d * 16 + ph] = tacc[ph];
}

// --- tree with its random-access tables in LDS (documents of <= tree_l_max nodes) --
// The same two sweeps as k_tree, one document per workgroup and one workgroup
// per CU: the last-child table of the non-special class (sweep 1) and the
// thread table (sweep 2) are u16 arrays over the whole document in LDS, so the
// accesses to far parents -- k_tree's random HBM line traffic, 1.3 requests a
// node -- become LDS accesses.  The table ends sweep 1 as each
// node's newest non-special child, which sweep 2 reads for a tile before it
// overwrites the tile's entries with their threads.  What stays in HBM: the
// special class's table fcS (specials are a minority), nsc, and the list of
// oldest special children, whose next sibling (their parent's newest
// non-special) is patched into nsc once the table is final.  The thread
// table's u16 sentinel for SUCC_END is TL_END.
constexpr uint32_t TL_END = 0xFFFFu;


// LDS of k_tree_l: the tile tables (hash / sort buffer, member lists, digit
// counters: tree_l_tile_bytes, at the front of the dynamic buffer) and the
// document tables (two bitmaps + the u16 table: tree_l_lds_bytes).  (A
// static array would add to the other phases' LDS in the fused kernel.)
__host__ __device__ constexpr uint32_t tree_l_tile_bytes(uint32_t nt, uint32_t tile) {
  return 4 * tile * 4 + (nt / 64) * SUB_BINS * 4 + tile * 2;
}
__host__ __device__ constexpr uint32_t tree_l_static_bytes(uint32_t nt, uint32_t tile) {
  return tree_l_tile_bytes(nt, tile) + 64 * 4 + 4;
}
__host__ __device__ inline uint32_t tree_l_lds_bytes(uint32_t nmax) {
  return ((nmax + 31) / 32) * 8 + ((nmax + 1) / 2) * 4;  // two bitmaps + u16 table
}

// Sweep 2 of the tree without the barrier between pointer jumping and the
// write-out (round 6; CW_S2_JUMP_BARRIER=1 at build time restores it for A/Bs).
#ifndef CW_S2_JUMP_BARRIER
#define CW_S2_JUMP_BARRIER 0
#endif
constexpr bool S2_JUMP_NOBAR = CW_S2_JUMP_BARRIER == 0;

// MODE 4 (the one built; round 3's A/B variants 0-3 lost and are gone): a
// group whose parent lies in the tile (69% of config-2 nodes) keeps its list
// head in a direct table indexed by (class, parent - tile start): one exchange
// instead of a claiming CAS + exchange; other groups go through the hash
// one document d (the whole workgroup); lds: the dynamic LDS (16-byte aligned)
template <int NT, int TILE_T, bool PROF, int MODE, typename PT = uint32_t>
__device__ __forceinline__ void tree_l_doc(
    const PT *__restrict__ par, const uint8_t *__restrict__ skind,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ doc_log2k, uint32_t kbits,
    uint32_t bm_words, uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
    uint32_t *__restrict__ link, uint32_t *__restrict__ osp,
    unsigned long long *__restrict__ tprof,
    const uint32_t *__restrict__ kbm, const uint32_t *__restrict__ tile_first, uint32_t d,
    uint32_t *lds) {
  constexpr uint32_t IT = TILE_T / NT;
  unsigned long long tacc[16] = {}, tlast = 0;
  auto stamp = [&](int ph) {  // diagnostic phase times (CW_TREE_PROF)
    if (PROF) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tacc[ph] += now - tlast;
      tlast = now;
    }
  };
  stamp(-1);
  // one tile's group-key hash: hk[slot] = group key (0 = empty), hh[slot] =
  // the head of the slot's member list (a tile index); nxt: next member,
  // TL_END ends.  The fallback sort's tkey/trank/tns and sweep 2's T live in
  // the same buffer.
  static_assert(MODE == 4, "k_tree_l is built with direct list heads only");
  constexpr bool DH = true;
  constexpr uint32_t HS = DH ? TILE_T : 2 * TILE_T, GMAX = 16, HB = TILE_T <= 2048 ? 11 : 12;
  static_assert(TILE_T <= (1u << HB) && 17 + HB <= 32, "slot word layout");
  static_assert(2 * HS + (DH ? 2 * TILE_T : 0) == 4 * TILE_T, "hash (+ direct heads) = 4 TILE_T words");
  uint32_t *const hbuf = lds;  // 4 TILE_T words: hash keys, hash heads (, direct heads)
  uint32_t(*const wcnt)[SUB_BINS] = reinterpret_cast<uint32_t(*)[SUB_BINS]>(lds + 4 * TILE_T);
  uint16_t *const nxt = reinterpret_cast<uint16_t *>(lds + 4 * TILE_T + (NT / 64) * SUB_BINS);
  uint32_t *const bm = lds + tree_l_tile_bytes(NT, TILE_T) / 4;
  uint32_t *const hw = hbuf, *const hk = hbuf, *const hh = hbuf + HS;
  uint32_t *const tkey = hbuf, *const trank = hbuf + TILE_T, *const tns = hbuf + 2 * TILE_T;
  uint32_t *const ptab = tns;
  __shared__ uint32_t run[64];
  __shared__ uint32_t n_osp;
  const uint32_t tid = threadIdx.x;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, log2k = doc_log2k[d];
  // this document's slices (wave-uniform bases, lane offsets: lane_at)
  const PT *const parD = par + base;
  uint32_t *const fcSD = fcS + base, *const nscD = nsc + base;
  uint32_t *const linkD = link + base, *const ospD = osp + base;
  uint32_t *const spec_bm = bm, *const hide_bm = bm + bm_words;
  uint16_t *const tab = reinterpret_cast<uint16_t *>(bm + 2 * bm_words);
  const uint32_t nw = (n + 31) >> 5;
  if (kbm) {
    const uint32_t *src = kbm + (size_t)tile_first[d] * KBM_WORDS;
    for (uint32_t wi = tid; wi < nw; wi += NT) {
      const uint32_t *tw = src + (size_t)(wi >> 7) * KBM_WORDS + (wi & 127);
      spec_bm[wi] = tw[0];
      hide_bm[wi] = tw[TILE / 32];
    }
  } else {
    for (uint32_t rb = (tid >> 6) << 6; rb < n; rb += NT) {
      const uint32_t r = rb + (tid & 63);
      const uint8_t kd = r < n ? skind[base + r] : 0;
      const uint64_t sm = __ballot(r < n && is_special(kd));
      const uint64_t hm = __ballot(r < n && is_hide(kd));
      if ((tid & 63) == 0) {
        spec_bm[rb >> 5] = (uint32_t)sm;
        hide_bm[rb >> 5] = (uint32_t)hm;
        if ((rb >> 5) + 1 < nw) {
          spec_bm[(rb >> 5) + 1] = (uint32_t)(sm >> 32);
          hide_bm[(rb >> 5) + 1] = (uint32_t)(hm >> 32);
        }
      }
    }
  }
  __syncthreads();
  stamp(0);
  auto special_at = [&](uint32_t r) -> bool { return (spec_bm[r >> 5] >> (r & 31)) & 1u; };
  auto hide_at = [&](uint32_t r) -> bool { return (hide_bm[r >> 5] >> (r & 31)) & 1u; };
  uint32_t qpar[IT];
  auto load_par = [&](uint32_t r0) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t r = r0 + wb_elem<IT>(k);
      qpar[k] = r < n ? lane_at(parD, r) : 0u;
    }
  };
  // sweep 1: group keys, next siblings, last-child tables.  A group (effective
  // parent, class) rarely has more than one member in a tile: members are
  // hashed by key into per-slot lists; a member's next sibling is the largest
  // smaller member of its list, or the group's last node of earlier tiles
  // (tab / fcS); the list's largest member updates the table.  A tile with a
  // group of more than GMAX members (e.g. many children of the root) is
  // sorted by group key instead, as in k_tree.
  auto clear_hash = [&]() {
    for (uint32_t i = tid; i < HS; i += NT) {
      hw[i] = 0;
      hh[i] = TL_END;
    }
    if (DH)
      for (uint32_t i = tid; i < 2 * TILE_T; i += NT) hbuf[2 * HS + i] = TL_END;
  };
  clear_hash();
  if (tid == 0) n_osp = 0;
  load_par(0);
  __syncthreads();
  // full tiles and the document's last, partial tile compile separately (the
  // guards of a full tile fold away)
  auto tile1 = [&](uint32_t r0, auto fullc) {
    constexpr bool F = decltype(fullc)::value;
    const uint32_t len = F ? TILE_T : min((uint32_t)TILE_T, n - r0);
    uint32_t key[IT], cpar[IT], ptv[IT], ptvS[IT], slot[IT];
    bool rdS[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) cpar[k] = qpar[k];
    stamp(8);
    // specials keep their cause: their table reads are unconditional (a node
    // without one reads entry 0), so no later wait has to be conservative
    auto load_ptvS = [&]() {
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = wb_elem<IT>(k), r = r0 + j, c = cpar[k] < r ? cpar[k] : 0u;
        rdS[k] = j < len && r > 0 && c < r0 && special_at(r);
        ptvS[k] = lane_at(fcSD, rdS[k] ? c : 0u);
      }
      if (r0 + TILE_T < n) load_par(r0 + TILE_T);
    };
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) ptv[k] = 0;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k), r = r0 + j;
      key[k] = 0;
      if (j < len) {
        tab[r] = 0;
        lane_at(fcSD, r) = 0;
      }
      if (j < len && r > 0) {
        const bool sp = special_at(r);
        uint32_t c = cpar[k];
        c = c < r ? c : 0u;
        if (!sp)
          while (c != 0 && special_at(c)) {
            const uint32_t pc = lane_at(parD, c);
            c = pc < c ? pc : 0u;
          }
        key[k] = ((c + 1) << 1) | (sp ? 0u : 1u);
        if (!sp) ptv[k] = c < r0 ? (uint32_t)tab[c] : 0u;
      }
    }
    stamp(9);
    load_ptvS();
    stamp(10);
    // insert: claim the key's slot (linear probing), push onto its list
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k), kk = key[k];
      slot[k] = 0;
      if (j < len && kk) {
        uint32_t h = (kk * 0x9E3779B1u) >> (32 - __builtin_ctz(HS));
        const uint32_t e = (kk >> 1) - 1;
        if (DH && e >= r0) {  // slot = the head's word in hbuf
          const uint32_t s = 2 * HS + (kk & 1) * TILE_T + (e - r0);
          nxt[j] = (uint16_t)atomicExch(&hbuf[s], j);
          slot[k] = s;
          continue;
        }
        for (;;) {  // claim the key (hk), then push (exchange on hh)
          const uint32_t old = atomicCAS(&hk[h], 0u, kk);
          if (old == 0u || old == kk) break;
          h = (h + 1) & (HS - 1);
        }
        nxt[j] = (uint16_t)atomicExch(&hh[h], j);
        slot[k] = DH ? HS + h : h;
      }
    }
    stamp(11);
    __syncthreads();
    stamp(1);
    // walk the slot's list: prv1 = 1 + the largest smaller member (0: none)
    uint32_t prv1[IT];
    bool last[IT], big = false;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k);
      uint32_t x = !(j < len && key[k]) ? TL_END
                   : DH ? hbuf[slot[k]] : hh[slot[k]];
      uint32_t p1 = 0, steps = 0;
      bool ls = true;
#pragma unroll 1
      for (; x != TL_END && steps <= GMAX; steps++) {
        p1 = x < j ? max(p1, x + 1) : p1;
        ls = ls && x <= j;
        x = nxt[x];
      }
      big |= x != TL_END;
      prv1[k] = p1;
      last[k] = ls;
    }
    stamp(12);
    const bool any_big = __syncthreads_or(big);
    stamp(13);
    if (any_big) {
      // fallback: stable LDS sort of the tile by group key (k_tree's sweep 1)
      uint32_t rk[IT], sd[IT], pos[IT];
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) rk[k] = wb_elem<IT>(k);
      for (uint32_t shift = 0; shift < kbits; shift += SUB_BITS) {
#pragma unroll
        for (uint32_t k = 0; k < IT; k++) sd[k] = (key[k] >> shift) & (SUB_BINS - 1);
        rank_subdigit<NT, IT>(sd, len, min(SUB_BITS, kbits - shift), pos, wcnt, run);
#pragma unroll
        for (uint32_t k = 0; k < IT; k++)
          if (wb_elem<IT>(k) < len) {
            tkey[pos[k]] = key[k];
            trank[pos[k]] = rk[k];
          }
        if (shift + SUB_BITS >= kbits) {
#pragma unroll
          for (uint32_t k = 0; k < IT; k++) ptab[wb_elem<IT>(k)] = rdS[k] ? ptvS[k] : ptv[k];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < IT; k++) {
          const uint32_t j = wb_elem<IT>(k);
          if (j < len) {
            key[k] = tkey[j];
            rk[k] = trank[j];
          }
        }
        __syncthreads();
      }
      uint32_t pv[IT];
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = wb_elem<IT>(k);
        const uint32_t kk = key[k];
        pv[k] = 0;
        if (j < len && kk != 0) pv[k] = (j > 0 && tkey[j - 1] == kk) ? r0 + trank[j - 1] : ptab[rk[k]];
      }
#pragma unroll
      for (uint32_t k = 0; k < IT; k++)
        if (wb_elem<IT>(k) < len) {
          const uint32_t kk = key[k], e = (kk >> 1) - 1;
          tns[rk[k]] = pv[k] ? pv[k] : (NSC_UP | e);
          if (kk && !(kk & 1) && !pv[k]) lane_at(ospD, atomicAdd(&n_osp, 1u)) = ((r0 + rk[k]) << 16) | e;
        }
      __syncthreads();
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = wb_elem<IT>(k);
        if (j >= len) continue;
        const uint32_t kk = key[k];
        if (kk != 0 && !(j + 1 < len && tkey[j + 1] == kk)) {
          const uint32_t e = (kk >> 1) - 1, v = r0 + rk[k];
          if (kk & 1) tab[e] = (uint16_t)v;
          else lane_at(fcSD, e) = v;
        }
      }
      for (uint32_t j = tid; j < len; j += NT) lane_at(nscD, r0 + j) = tns[j];
      __syncthreads();
      clear_hash();
      __syncthreads();
    } else {
#pragma unroll
      for (uint32_t k = 0; k < IT; k++) {
        const uint32_t j = wb_elem<IT>(k), r = r0 + j, kk = key[k];
        if (j >= len) continue;
        const uint32_t e = (kk >> 1) - 1;
        const uint32_t pv = prv1[k] ? r0 + prv1[k] - 1 : (rdS[k] ? ptvS[k] : ptv[k]);
        lane_at(nscD, r) = kk == 0 ? 0u : (pv ? pv : (NSC_UP | e));
        if (kk && !(kk & 1) && !pv) lane_at(ospD, atomicAdd(&n_osp, 1u)) = (r << 16) | e;
        if (kk && last[k]) {
          if (kk & 1) tab[e] = (uint16_t)r;
          else lane_at(fcSD, e) = r;
        }
        if (kk && DH) {
          if (slot[k] < 2 * HS) hk[slot[k] - HS] = 0;
          hbuf[slot[k]] = TL_END;
        } else if (kk) {
          hw[slot[k]] = 0;
          hh[slot[k]] = TL_END;
        }
      }
      __syncthreads();
    }
    stamp(3);
  };
  uint32_t r0t = 0;
  for (; r0t + TILE_T <= n; r0t += TILE_T) tile1(r0t, std::true_type());
  if (r0t < n) tile1(r0t, std::false_type());
  // the oldest special child's next sibling is its parent's newest
  // non-special (weave-later?): patched into nsc now that tab is final.  The
  // newest non-special children stay in tab: sweep 2 reads tile t's entries
  // before it overwrites them with tile t's threads.
  for (uint32_t i = tid; i < n_osp; i += NT) {
    const uint32_t v = lane_at(ospD, i), f = tab[v & 0xFFFFu];
    if (f) lane_at(nscD, (v >> 16)) = f;
  }
  __syncthreads();
  // sweep 2: preorder successors; thr(r) = ns(r) ?: thr(e(r)) with the earlier
  // tiles' threads in tab (u16) and this tile's resolved by pointer jumping.
  // Tile loads run two tiles ahead.
  constexpr uint32_t RES = 0x80000000u;
  uint32_t *const T = hbuf;
  struct Q {
    uint32_t fs[IT], ns[IT];
  };
  auto load_tile = [&](Q &q, uint32_t r0) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t r = r0 + k * NT + tid;
      const bool ok = r < n;
      q.fs[k] = ok ? lane_at(fcSD, r) : 0u;
      q.ns[k] = ok ? lane_at(nscD, r) : 0u;
    }
  };
  // one tile: X holds its loads (and is refilled with tile r0 + 2 TILE_T)
  auto tile2f = [&](uint32_t r0, Q &X, auto fullc) {
    constexpr bool F = decltype(fullc)::value;
    const uint32_t len = F ? TILE_T : min((uint32_t)TILE_T, n - r0);
    uint32_t flg[IT], fcr[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid, r = r0 + j;
      flg[k] = 0;
      fcr[k] = 0;
      if (j >= len) continue;
      fcr[k] = X.fs[k] ? X.fs[k] : (uint32_t)tab[r];
      const bool sp = special_at(r);
      uint32_t tv;
      if (r == 0) {
        tv = RES | SUCC_END;
      } else {
        uint32_t ns = X.ns[k], e = 0;
        if (ns & NSC_UP) {
          e = ns & ~NSC_UP;
          ns = 0;
        }
        if (ns) {
          tv = RES | ns;
        } else if (e >= r0) {
          tv = e - r0;
        } else {
          const uint32_t t = tab[e];
          tv = RES | (t == TL_END ? SUCC_END : t);
        }
      }
      T[j] = tv;
      const uint32_t fs = X.fs[k];
      const bool vis = !sp && r != 0 && !(fs && hide_at(fs));
      const bool split = r == split_node(d, r >> log2k, log2k, n);
      flg[k] = (vis ? LINK_VIS : 0u) | (split ? LINK_SPLIT : 0u);
    }
    if (r0 + 2 * TILE_T < n) load_tile(X, r0 + 2 * TILE_T);
    __syncthreads();
    stamp(5);
    // pointer jumping without barriers: every value in T is an ancestor's
    // pointer or a resolved thread at any time, so a lane may read its
    // target's entry whenever it likes; each lane stops when its own entries
    // are resolved (targets are smaller indices of the same tile)
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid;
      if (j < len) {
        uint32_t t = T[j];
        while (!(t & RES)) {
          t = T[t];
          T[j] = t;
        }
      }
    }
    // (no barrier here: a lane writes out only the entries it resolved itself,
    // into tab and the links, which no jumping lane reads; the barrier after
    // the writes keeps the next tile's T and its reads of tab apart -- round 6)
    if (!S2_JUMP_NOBAR) __syncthreads();
    stamp(6);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = k * NT + tid, r = r0 + j;
      if (j >= len) continue;
      const uint32_t th = T[j] & ~RES;
      tab[r] = (uint16_t)(th == SUCC_END ? TL_END : th);
      lane_at(linkD, r) = (fcr[k] ? fcr[k] : th) | flg[k];
    }
    __syncthreads();
    stamp(7);
  };
  auto tile2 = [&](uint32_t r0, Q &X) {
    if (r0 + TILE_T <= n) tile2f(r0, X, std::true_type());
    else tile2f(r0, X, std::false_type());
  };
  Q qa, qb;
  load_tile(qa, 0);
  if (TILE_T < n) load_tile(qb, TILE_T);
  stamp(4);
  for (uint32_t r0 = 0; r0 < n; r0 += 2 * TILE_T) {
    tile2(r0, qa);
    if (r0 + TILE_T < n) tile2(r0 + TILE_T, qb);
  }
  if (PROF && tid == 0)
    for (int ph = 0; ph < 16; ph++) tprof[(size_t)d * 16 + ph] = tacc[ph];
}

template <int NT, int TILE_T, bool PROF, int MODE>
__global__ __launch_bounds__(NT) void k_tree_l(
    const uint32_t *__restrict__ par, const uint8_t *__restrict__ skind,
    const uint32_t *__restrict__ doc_off, const uint32_t *__restrict__ doc_log2k, uint32_t kbits,
    uint32_t bm_words, uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
    uint32_t *__restrict__ link, uint32_t *__restrict__ osp,
    unsigned long long *__restrict__ tprof,
    const uint32_t *__restrict__ kbm, const uint32_t *__restrict__ tile_first, uint32_t doc0 = 0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_tl[];
  tree_l_doc<NT, TILE_T, PROF, MODE>(par, skind, doc_off, doc_log2k, kbits, bm_words, nsc, fcS, link,
                                     osp, tprof, kbm, tile_first, doc0 + blockIdx.x, lds_tl);
}

// --- tree for one giant document (all tiles in parallel) -------------------------
// k_tree sweeps a document in order in one workgroup, which is hopeless for a
// single list of 10^8+ nodes (BASELINE config 5).  Same tree, three passes
// over all ranks at once:
//   k_geff   effective parent and class per rank -> group key (e << 1 | class);
//   (the keys are radix sorted, stable in rank: siblings become adjacent)
//   k_gsib   next sibling of every node from its sorted neighbour, last child of
//            every group (-> first children), the oldest special's next sibling
//            = its parent's newest non-special (binary search in the keys);
//   k_gthr   per tile: threads by pointer jumping inside the tile; a chain that
//            leaves the tile is left to the walk (LINK_PEND: thr[x] is chased).
// (also clears k_gsib's last-child tables and zeroes two counters at r == 0:
// fewer launches on the one-list path, where each costs a visible share)
// tcnt != nullptr (the tile-local sibling links, k_glocal): per GL_TILE-rank
// tile, the children whose effective parent lies in an earlier tile ("cross"
// children, counted into tcnt), and no clearing of fcS / fcN (k_glocal writes
// every entry).
constexpr uint32_t GL_TILE = 2048;
__global__ __launch_bounds__(256) void k_geff(const uint32_t *__restrict__ par,
                                              const uint8_t *__restrict__ skind, uint32_t n,
                                              uint32_t root_key, uint32_t *__restrict__ gk,
                                              uint32_t *__restrict__ fcS, uint32_t *__restrict__ fcN,
                                              uint32_t *__restrict__ zero_a,
                                              uint32_t *__restrict__ zero_b,
                                              uint32_t *__restrict__ tcnt) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool cross = false;
  if (r < n) {
    if (!tcnt) {
      fcS[r] = 0;
      fcN[r] = 0;
    }
    if (r == 0) {
      gk[0] = root_key;  // the root has no group: it sorts last
      if (zero_a) *zero_a = 0;
      if (zero_b) *zero_b = 0;
    } else {
      const bool sp = is_special(skind[r]);
      uint32_t c = par[r];
      c = c < r ? c : 0u;  // clamps keep out-of-domain documents in bounds
      if (!sp)
        while (c != 0 && is_special(skind[c])) {
          const uint32_t pc = par[c];
          c = pc < c ? pc : 0u;
        }
      gk[r] = (c << 1) | (sp ? 0u : 1u);
      cross = c < (r & ~(GL_TILE - 1));
    }
  }
  if (tcnt) {  // (a block lies inside one tile: 256 | GL_TILE)
    const uint64_t m = __ballot(cross);
    __shared__ uint32_t bc;
    if (threadIdx.x == 0) bc = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&bc, (uint32_t)__popcll(m));
    __syncthreads();
    if (threadIdx.x == 0 && bc) atomicAdd(&tcnt[blockIdx.x * blockDim.x / GL_TILE], bc);
  }
}

// --- the tree's sibling links without sorting every node (round 4) ----------------
// Two thirds of config-2/5 nodes have their effective parent inside their own
// GL_TILE-rank tile.  A group (parent e, class) lists its members in rank
// order: first the ones in e's own tile ("local", all in that one tile), then
// the ones in later tiles ("cross").  So:
//   k_glocal   per tile, in LDS: the local children sorted by (e - r0, class)
//              (a 13-bit stable sort, cross children and the root last): each
//              local child's next sibling = the previous local member (final:
//              local members come first), each local group's last member into
//              fcS / fcN (every entry of the tile written); the cross children
//              compacted, in rank order, at the tile's offset (k_geff counted
//              them, a scan placed them);
//   sort       the cross children only, by group key (stable in rank);
//   k_gcross_ns  a cross child's next sibling: the previous cross member of its
//              group, or for the first one the group's last local member
//              (fcS / fcN as k_glocal left them);
//   k_gcross_fc  the last cross member of a group becomes its last child.
// The oldest special's next sibling (the newest non-special of its parent,
// weave-later?) is read by k_gthr from the final fcN.  Replaces the sort of all
// group keys and k_gsib.
template <int NT>
__global__ __launch_bounds__(NT) void k_glocal(const uint32_t *__restrict__ gk, uint32_t n,
                                               const uint32_t *__restrict__ toff,
                                               uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
                                               uint32_t *__restrict__ fcN, uint32_t *__restrict__ ckey,
                                               uint32_t *__restrict__ cval, uint32_t *__restrict__ mtot) {
  constexpr uint32_t IT = GL_TILE / NT, SENT = 2 * GL_TILE;  // key 13 bits: SENT = not local
  __shared__ uint16_t tkey[GL_TILE], tj[GL_TILE];
  __shared__ uint32_t nsv[GL_TILE], fcl[2][GL_TILE];
  __shared__ uint32_t wcnt[NT / 64][SUB_BINS], run[64];
  const uint32_t t = blockIdx.x, r0 = t * GL_TILE, tid = threadIdx.x;
  const uint32_t len = min(GL_TILE, n - r0);
  for (uint32_t j = tid; j < GL_TILE; j += NT) fcl[0][j] = fcl[1][j] = 0;
  uint32_t key[IT], val[IT], sd[IT], pos[IT], g[IT];
  uint32_t ncross = 0;
  bool crs[IT];
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = wb_elem<IT>(k), r = r0 + j;
    g[k] = j < len ? gk[r] : 0xFFFFFFFFu;
    const uint32_t e = g[k] >> 1;
    const bool node = j < len && r > 0 && (uint64_t)g[k] < 2ull * n;
    const bool loc = node && e >= r0;
    crs[k] = node && !loc;
    ncross += crs[k] ? 1u : 0u;
    key[k] = loc ? (((e - r0) << 1) | (g[k] & 1u)) : SENT;
    val[k] = j;
  }
  // the cross children, compacted in rank order: element j of the tile is
  // item k of lane l of wave w with j = (w IT + k) 64 + l (wb_elem), so the
  // 64-lane slots w IT + k are in element order -- a ballot a slot, a scan over
  // the (GL_TILE / 64) slots
  {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      // cross items before this one: all items of earlier (wave, k') slots plus
      // the lanes below in this slot
      const uint64_t m = __ballot(crs[k]);
      const uint32_t lane = tid & 63, w = tid >> 6;
      if (lane == 0) run[(w * IT + k) & 63] = (uint32_t)__popcll(m);  // (NT / 64 * IT <= 64)
      pos[k] = lanes_below(m);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan over the slots in element order
      const uint32_t v = tid < (NT / 64) * IT ? run[tid] : 0u;
      uint32_t x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (tid >= (uint32_t)o) x += y;
      }
      run[tid] = x - v;
      if (tid == 63 && t == gridDim.x - 1 && mtot) *mtot = toff[t] + x;
    }
    __syncthreads();
    const uint32_t base = toff[t], w = tid >> 6;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
      if (crs[k]) {
        const uint32_t o = base + run[w * IT + k] + pos[k];
        ckey[o] = g[k];
        cval[o] = r0 + wb_elem<IT>(k);
      }
    __syncthreads();
  }
  // stable sort of the tile by key (13 bits: 6 + 6 + 1)
  for (uint32_t sh = 0; sh < 13; sh += SUB_BITS) {
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) sd[k] = (key[k] >> sh) & (SUB_BINS - 1);
    rank_subdigit<NT, IT>(sd, len, min(SUB_BITS, 13u - sh), pos, wcnt, run);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
      if (wb_elem<IT>(k) < len) {
        tkey[pos[k]] = (uint16_t)key[k];
        tj[pos[k]] = (uint16_t)val[k];
      }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
      const uint32_t j = wb_elem<IT>(k);
      if (j < len) {
        key[k] = tkey[j];
        val[k] = tj[j];
      }
    }
    __syncthreads();
  }
  // sorted: tkey / tj hold the tile in (key, rank) order
  for (uint32_t p = tid; p < len; p += NT) {
    const uint32_t kk = tkey[p];
    if (kk >= SENT) continue;
    const uint32_t j = tj[p], e = r0 + (kk >> 1);
    const bool first = p == 0 || tkey[p - 1] != kk, last = p + 1 == len || tkey[p + 1] != kk;
    nsv[j] = first ? (NSC_UP | e) : r0 + tj[p - 1];
    if (last) fcl[kk & 1][kk >> 1] = r0 + j;
  }
  __syncthreads();
  for (uint32_t j = tid; j < len; j += NT) {
    const uint32_t r = r0 + j, gg = gk[r];  // (cached: this block read it)
    const bool node = r > 0 && (uint64_t)gg < 2ull * n;
    if (node && (gg >> 1) >= r0) nsc[r] = nsv[j];  // (cross children: k_gcross_ns)
    fcS[r] = fcl[0][j];
    fcN[r] = fcl[1][j];
  }
}

// next sibling of each cross child (sorted by group key, stable in rank)
__global__ __launch_bounds__(256) void k_gcross_ns(const uint32_t *__restrict__ key,
                                                   const uint32_t *__restrict__ val,
                                                   const uint32_t *__restrict__ mtot,
                                                   uint32_t *__restrict__ nsc,
                                                   const uint32_t *__restrict__ fcS,
                                                   const uint32_t *__restrict__ fcN) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, m = *mtot;
  if (i >= m) return;
  const uint32_t g = key[i], r = val[i], e = g >> 1;
  uint32_t ns;
  if (i > 0 && key[i - 1] == g) ns = val[i - 1];
  else ns = ((g & 1) ? fcN : fcS)[e];  // the group's last local member (or none)
  nsc[r] = ns ? ns : (NSC_UP | e);
}

// ... and the last cross member of each group: its parent's last child
__global__ __launch_bounds__(256) void k_gcross_fc(const uint32_t *__restrict__ key,
                                                   const uint32_t *__restrict__ val,
                                                   const uint32_t *__restrict__ mtot,
                                                   uint32_t *__restrict__ fcS, uint32_t *__restrict__ fcN) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, m = *mtot;
  if (i >= m) return;
  const uint32_t g = key[i];
  if (i + 1 == m || key[i + 1] != g) ((g & 1) ? fcN : fcS)[g >> 1] = val[i];
}

__global__ __launch_bounds__(256) void k_gsib(const uint32_t *__restrict__ key,
                                              const uint32_t *__restrict__ val, uint32_t n,
                                              uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
                                              uint32_t *__restrict__ fcN) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = key[i];
  if ((uint64_t)g >= 2ull * n) return;  // the root
  const uint32_t r = val[i], e = g >> 1;
  const bool first = i == 0 || key[i - 1] != g, last = i + 1 == n || key[i + 1] != g;
  if (last) ((g & 1) ? fcN : fcS)[e] = r;
  uint32_t ns = first ? 0u : val[i - 1];
  if (first && !(g & 1)) {  // oldest special: the newest non-special of e follows its group
    // The two groups of e are adjacent (keys g, g | 1), so the end of the
    // second is near: gallop forward from i, then bisect the last step.  (A
    // bisection over [i, n) was ~log2 n dependent cache misses for every
    // special group head -- the kernel's whole time at 2e9 nodes.)
    const uint32_t want = g | 1u;
    uint32_t lo = i + 1, hi = n, step = 1;  // invariant: key[< lo] <= want
    while (lo < n) {
      const uint32_t p = n - lo > step - 1 ? lo + step - 1 : n - 1;
      if (key[p] <= want) {
        lo = p + 1;
        step <<= 1;
      } else {
        hi = p;
        break;
      }
    }
    while (lo < hi) {
      const uint32_t m = lo + ((hi - lo) >> 1);
      if (key[m] <= want) lo = m + 1; else hi = m;
    }
    if (lo > 0 && key[lo - 1] == want) ns = val[lo - 1];
  }
  nsc[r] = ns ? ns : (NSC_UP | e);
}

template <int NT, int TT>
__global__ __launch_bounds__(NT) void k_gthr(const uint32_t *__restrict__ nsc,
                                             const uint32_t *__restrict__ fcS,
                                             const uint32_t *__restrict__ fcN,
                                             const uint8_t *__restrict__ skind, uint32_t n,
                                             const uint32_t *__restrict__ sval,
                                             uint32_t *__restrict__ thr,
                                             uint64_t *__restrict__ link) {
  // T: a pointer to a lower rank of the tile, RES | resolved thread, or OUT | an
  // ancestor outside the tile (its thread is left to the walk)
  constexpr uint32_t IT = TT / NT;
  constexpr uint64_t RES = 1ull << 63, OUT = 1ull << 62;
  __shared__ uint64_t T[TT];
  const uint32_t r0 = blockIdx.x * TT, tid = threadIdx.x, len = min((uint32_t)TT, n - r0);
  uint32_t fcr[IT], flg[IT];
#pragma unroll
  for (uint32_t k = 0; k < IT; k++) {
    const uint32_t j = k * NT + tid, r = r0 + j;
    fcr[k] = flg[k] = 0;
    if (j >= len) continue;
    const uint32_t fs = fcS[r], fn = fcN[r];
    uint32_t ns = nsc[r];
    const bool sp = is_special(skind[r]);
    // the oldest special child (no earlier special sibling) is followed by its
    // parent's newest non-special (weave-later?); k_gsib patched it already,
    // the tile-local links (k_glocal) leave it to this final fcN
    if (sp && r != 0 && (ns & NSC_UP)) {
      const uint32_t f = fcN[ns & ~NSC_UP];
      if (f) ns = f;
    }
    fcr[k] = fs ? fs : fn;
    uint64_t tv;
    if (r == 0) tv = RES | SUCCW_END;
    else if (!(ns & NSC_UP)) tv = RES | ns;
    else {
      const uint32_t e = ns & ~NSC_UP;
      tv = e >= r0 ? (e < r ? (uint64_t)(e - r0) : (RES | SUCCW_END)) : (OUT | e);
    }
    T[j] = tv;
    const bool vis = !sp && r != 0 && !(fs && is_hide(skind[fs]));
    flg[k] = vis ? LINK_VIS : 0u;
  }
  __syncthreads();
  for (;;) {  // pointer jumping inside the tile (pointers go to lower ranks)
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
    const uint32_t j = k * NT + tid, r = r0 + j;
    if (j >= len) continue;
    const uint64_t a = T[j];
    const bool res = (a & RES) != 0;
    const uint32_t v = (uint32_t)a;  // resolved thread, or the ancestor to chase
    thr[r] = res ? v : (THRW_PEND | v);
    const uint32_t succ = fcr[k] ? fcr[k] : v;
    link[r] = wide_link(succ, !fcr[k] && !res, sval ? sval[r] : r, flg[k] != 0);
  }
}

// Walker w of document d starts at the splitter node of rank block w and
// follows preorder successors up to the next splitter (or the end).  The nodes
// it passes (rank | renders << 31) are appended to its sublist's slot of `cap`
// entries; a full slot continues as a new sublist (id >= W, from a per-document
// counter), so slots are written sequentially by one lane, no per-node scatter.
template <bool WIDE>
__global__ __launch_bounds__(1024) void k_walk(
    const void *__restrict__ linkp, const uint32_t *__restrict__ thr,
    const uint32_t *__restrict__ wblk_doc,
    const uint32_t *__restrict__ wblk_w0, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ doc_log2k, const uint32_t *__restrict__ doc_log2cap,
    const uint32_t *__restrict__ doc_W, const uint32_t *__restrict__ doc_Wcap,
    const uint32_t *__restrict__ walk_first, const uint64_t *__restrict__ slot_first,
    uint32_t *__restrict__ slots, uint32_t *__restrict__ wcnt, uint32_t *__restrict__ wnext,
    uint32_t *__restrict__ dyn_ctr, uint32_t *__restrict__ status, uint32_t walk_span,
    unsigned long long *__restrict__ wprof) {
  __shared__ uint32_t next_walker;
  uint32_t n_steps = 0, n_pend = 0, n_hops = 0;  // (wprof: CW_TREE_PROF diagnostics)
  const uint32_t b = xcd_tile(blockIdx.x, gridDim.x), d = wblk_doc[b];
  const uint32_t W = doc_W[d], Wcap = doc_Wcap[d];
  const uint32_t w0 = wblk_w0[b], w1 = min(w0 + walk_span, W);
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, log2k = doc_log2k[d];
  const uint32_t log2cap = doc_log2cap[d], cap = 1u << log2cap;
  const uint32_t f = walk_first[d];
  uint32_t *const sl = slots + slot_first[d];
  // link word of node x: successor index and LINK_* flags (narrow: one u32;
  // wide: u64 = successor | flags << 32)
  constexpr uint32_t END = WIDE ? SUCCW_END : SUCC_END;
  // (wide: the LINK_* flags rebuilt -- the splitter bit from the rank -- and
  // the node's slot entry = the value it emits, so the emit gathers nothing;
  // narrow: the entry is the rank)
  auto load = [&](uint32_t x, uint32_t &succ, uint32_t &ent) -> uint32_t {
    if (WIDE) {
      const uint64_t L = static_cast<const uint64_t *>(linkp)[base + x];
      succ = (uint32_t)L & SUCCW_END;
      const bool vis = (L >> 63) != 0;
      ent = (uint32_t)(L >> 32) & SLOT_IDX;
      ent |= vis ? 0x80000000u : 0u;
      return (vis ? LINK_VIS : 0u) | (((uint32_t)L >> 31) ? LINK_PEND : 0u) |
             (x == split_node(d, x >> log2k, log2k, n) ? LINK_SPLIT : 0u);
    }
    const uint32_t L = static_cast<const uint32_t *>(linkp)[base + x];
    succ = L & LINK_IDX;
    ent = x | (L & LINK_VIS);
    return L & ~LINK_IDX;
  };
  // a finished sublist's {node count, next sublist}: wide (the one-list path,
  // ranked by k_lvl_walk's random reads) one u64 word in wcnt's room, so a
  // ranking step reads one line; narrow two arrays
  auto put_sub = [&](uint32_t x, uint32_t cnt, uint32_t next) {
    if (WIDE) {
      reinterpret_cast<uint64_t *>(wcnt)[f + x] = cnt | (uint64_t)next << 32;
    } else {
      wcnt[f + x] = cnt;
      wnext[f + x] = next;
    }
  };
  if (threadIdx.x == 0) next_walker = w0 + blockDim.x;
  __syncthreads();
  // (one walker a thread by default, walk_span == blockDim.x: a refilling
  // loop -- a lane takes the next walker as soon as its own ends, in this
  // block or from a grid-wide pool -- was measured slower, 1.8 -> 5.4 ms at
  // 6.7e7 nodes for spans of 4,096: the walkers in flight spread over a wider
  // range of the list, and the line reuse between neighbouring walkers drops)
  for (uint32_t lw = w0 + threadIdx.x; lw < w1; lw = atomicAdd(&next_walker, 1u)) {
    const uint32_t v = split_node(d, lw, log2k, n);
    uint32_t sv, ev;
    uint32_t L = load(v, sv, ev);
    uint32_t x = lw, cnt = 1, nextsub = NX_END;
    // entries are buffered four at a time and written as one 16-byte store
    // (slots are 16-byte aligned: cap >= 4 and every slot start is a multiple)
    uint4 q = make_uint4(ev, 0u, 0u, 0u);
    for (uint32_t steps = 0;; steps++) {
      uint32_t u = sv;
      n_steps++;
      n_pend += (L & LINK_PEND) ? 1u : 0u;
      if (L & LINK_PEND)  // the successor is the thread of an ancestor: chase it
        for (uint32_t hop = 0; hop <= n; hop++) {
          n_hops++;
          const uint32_t tv = thr[base + (u < n ? u : 0u)];
          bool pend;
          if (WIDE) {
            u = tv & ~THRW_PEND;
            pend = (tv & THRW_PEND) != 0;
          } else {
            u = tv & LINK_IDX;
            pend = (tv & LINK_PEND) != 0;
          }
          if (!pend || u >= n) break;
        }
      if (u >= n) {  // the end marker: the tour is over
        if (u != END) atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
        break;
      }
      uint32_t su, eu;
      const uint32_t Lu = load(u, su, eu);
      if (Lu & LINK_SPLIT) {
        nextsub = u >> log2k;
        break;
      }
      // slot full (and flushed): continue as a new sublist; the lanes of a
      // wave that overflow together take their ids with one atomic (a giant
      // document has one counter for all its walkers)
      const bool full = cnt == cap;
      const uint64_t fm = __ballot(full);
      if (full) {
        const uint32_t lead = (uint32_t)__ffsll((unsigned long long)fm) - 1;
        const uint32_t lane = threadIdx.x & 63;
        uint32_t y0 = 0;
        if (lane == lead) y0 = atomicAdd(&dyn_ctr[d], (uint32_t)__popcll(fm));
        y0 = __shfl(y0, lead, 64);
        const uint32_t y = W + y0 + lanes_below(fm);
        if (y >= Wcap) {
          atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
          break;
        }
        put_sub(x, cap, y);
        x = y;
        cnt = 0;
      }
      const uint32_t e = eu;
      switch (cnt & 3) {
        case 0: q.x = e; break;
        case 1: q.y = e; break;
        case 2: q.z = e; break;
        default: q.w = e; break;
      }
      cnt++;
      if ((cnt & 3) == 0)
        *reinterpret_cast<uint4 *>(sl + ((size_t)x << log2cap) + cnt - 4) = q;
      L = Lu;
      sv = su;
      if (steps > n) {
        atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
        break;
      }
    }
    if (cnt & 3) {  // flush the partial group
      uint32_t *dst = sl + ((size_t)x << log2cap) + (cnt & ~3u);
      dst[0] = q.x;
      if ((cnt & 3) > 1) dst[1] = q.y;
      if ((cnt & 3) > 2) dst[2] = q.z;
    }
    put_sub(x, cnt, nextsub);
  }
  if (wprof) {
    atomicAdd(&wprof[0], (unsigned long long)n_steps);
    atomicAdd(&wprof[1], (unsigned long long)n_pend);
    atomicAdd(&wprof[2], (unsigned long long)n_hops);
  }
}

// --- sublist ranking: one workgroup per document, all in LDS -------------------
// The W sublists of a document form one linked list (the preorder).  Every
// CHAIN-th sublist id heads an LDS chain; one lane per head walks its chain
// (prefix sums in place), lane 0 ranks the <= W/CHAIN chains, then every
// sublist gets chain base + local prefix = number of nodes before it, and
// its index in tour order (order[] lists sublists in tour order for the emit).
__global__ __launch_bounds__(256) void k_rank(const uint32_t *__restrict__ wcnt,
                                              const uint32_t *__restrict__ wnext,
                                              const uint32_t *__restrict__ walk_first,
                                              const uint32_t *__restrict__ doc_W,
                                              const uint32_t *__restrict__ dyn_ctr,
                                              const uint32_t *__restrict__ doc_off,
                                              const uint64_t *__restrict__ skey, uint32_t ts_shift,
                                              uint32_t *__restrict__ sbase,
                                              uint32_t *__restrict__ order,
                                              uint64_t *__restrict__ max_ts,
                                              uint32_t *__restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];  // nx[W], val[W]
  constexpr uint32_t NCH = MAX_SUBLISTS / CHAIN;
  __shared__ uint32_t ch_next[NCH], ch_sum[NCH], ch_len[NCH], ch_base[NCH], ch_tbase[NCH];
  __shared__ uint32_t bad_s;
  const uint32_t d = blockIdx.x, f = walk_first[d];
  const uint32_t W = min(doc_W[d] + dyn_ctr[d], walk_first[d + 1] - f);  // static + continued
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base;
  if (threadIdx.x == 0 && max_ts) max_ts[d] = n ? (skey[base + n - 1] >> ts_shift) : 0ull;
  if (W == 0) return;
  uint32_t *nx = sm, *val = sm + W;
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) {
    nx[i] = wnext[f + i];
    val[i] = wcnt[f + i];
  }
  if (threadIdx.x == 0) bad_s = 0;
  __syncthreads();
  const uint32_t C = (W + CHAIN - 1) / CHAIN;
  for (uint32_t h = threadIdx.x; h < C; h += blockDim.x) {
    uint32_t j = h * CHAIN, acc = 0, len = 0;
    for (;;) {
      const uint32_t x = nx[j], cval = val[j];
      val[j] = acc;            // nodes before j inside the chain
      nx[j] = (h << 24) | len;  // chain of j, index of j inside the chain
      acc += cval;
      len++;
      if (x == NX_END || x % CHAIN == 0 || x >= W || len > W) {
        ch_next[h] = (x == NX_END || x >= W) ? NX_END : x / CHAIN;
        ch_sum[h] = acc;
        ch_len[h] = len;
        if (x != NX_END && x % CHAIN != 0) bad_s = 1;
        break;
      }
      j = x;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0, trun = 0, c = 0, steps = 0;
    while (c != NX_END && steps++ <= C) {
      ch_base[c] = run;
      ch_tbase[c] = trun;
      run += ch_sum[c];
      trun += ch_len[c];
      c = ch_next[c];
    }
    if (run != n || trun != W || bad_s) atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) {
    const uint32_t h = min(nx[i] >> 24, C - 1), li = nx[i] & 0xFFFFFFu;
    sbase[f + i] = ch_base[h] + val[i];
    const uint32_t ti = ch_tbase[h] + li;
    if (ti < W) order[f + ti] = i;
  }
}

// --- multi-level sublist ranking (one giant document) ----------------------------
// The sublists form one linked list.  A level: every K-th element below
// Wsplit starts a walker that follows the links to the next such element,
// recording for each element it passes {its walker, the nodes and sublists
// before it inside the walk}; per walker {nodes, sublists, next walker}.
// Levels repeat until <= SUP_MAX walkers remain, which one workgroup ranks in
// LDS (k_sup_rank); k_lvl_apply hands the bases back down.  Each record is one
// word (the sublists: k_walk's u64 {nodes, next}; a level's walkers: uint4),
// so a walker's step reads one random line and writes one: the 2e9-node list
// has 1.25e8 sublists, and three separate arrays each way cost six.
template <bool SUBL>
__global__ __launch_bounds__(256) void k_lvl_walk(const void *__restrict__ in, uint32_t Wsplit,
                                                  uint32_t Wall, uint32_t K, uint32_t S,
                                                  uint4 *__restrict__ pos, uint4 *__restrict__ wout,
                                                  uint32_t *__restrict__ status,
                                                  const uint32_t *__restrict__ dyn, uint32_t Wstat) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= S) return;
  // Wall is the capacity; with dyn the walkers in use are the static ones plus
  // those the walk added, so a link into the unused range is caught
  if (dyn) Wall = min(Wstat + dyn[0], Wall);
  uint32_t x = q * K, acc = 0, cnt = 0, nq = NX_END;
  for (uint32_t steps = 0; steps <= Wall; steps++) {
    uint32_t a, b, nx;
    if (SUBL) {
      const uint64_t v = static_cast<const uint64_t *>(in)[x];
      a = (uint32_t)v;
      b = 1;
      nx = (uint32_t)(v >> 32);
    } else {
      const uint4 v = static_cast<const uint4 *>(in)[x];
      a = v.x;
      b = v.y;
      nx = v.z;
    }
    if (pos) pos[x] = make_uint4(q, acc, cnt, 0u);  // (none on the sublist level: k_lvl_emit)
    acc += a;
    cnt += b;
    if (nx == NX_END) break;
    if (nx >= Wall) {
      atomicOr(&status[0], (uint32_t)CW_STATUS_INTERNAL);
      break;
    }
    if (nx < Wsplit && nx % K == 0) {
      nq = nx / K;
      break;
    }
    x = nx;
  }
  wout[q] = make_uint4(acc, cnt, nq, 0u);
}

// Bases of a level's elements from their walker's: walker q's {node base, tour
// index} from `base` (uint2) or, for the top level, k_sup_rank's nb / tb.
// pos == nullptr: the elements are the top level's walkers themselves.
// erec != nullptr (the sublist level): erec[tour index] = {sublist, node base,
// node count} -- what the emit reads, in tour order; otherwise out[x].
__global__ __launch_bounds__(256) void k_lvl_apply(const uint4 *__restrict__ pos,
                                                   const uint32_t *__restrict__ nb,
                                                   const uint32_t *__restrict__ tb,
                                                   const uint2 *__restrict__ base,
                                                   const uint64_t *__restrict__ wl, uint32_t Wall,
                                                   uint2 *__restrict__ out, uint4 *__restrict__ erec,
                                                   const uint32_t *__restrict__ dyn, uint32_t Wstat) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (dyn) Wall = min(Wstat + dyn[0], Wall);  // walkers in use (Wall: the capacity)
  if (x >= Wall) return;
  uint32_t q = x, pa = 0, pb = 0;
  if (pos) {
    const uint4 P = pos[x];
    q = P.x;
    pa = P.y;
    pb = P.z;
  }
  uint32_t va, vb;
  if (base) {
    const uint2 B = base[q];
    va = B.x + pa;
    vb = B.y + pb;
  } else {
    va = nb[q] + pa;
    vb = tb[q] + pb;
  }
  if (erec) {
    if (vb < Wall) erec[vb] = make_uint4(x, va, (uint32_t)wl[x], 0u);
  } else {
    out[x] = make_uint2(va, vb);
  }
}

// The sublist level's emit records: each walker of the first level walks its
// sublists a second time, now with its node base and tour index known (from
// the level above, base, or the top level's nb / tb), and writes the record
// of each sublist it passes -- {sublist, node base, node count} at tour index
// base + k, consecutive for a walker.  A second pass of random 8-byte reads
// instead of writing every sublist's {walker, offsets} to pos[x] and the
// records from there: two scattered 16-byte stores a sublist, the slowest
// access there is (k_lvl_walk's walkers pass a geometric number of sublists,
// so per-walker slots overflow too often to be the alternative).
__global__ __launch_bounds__(256) void k_lvl_emit(const uint64_t *__restrict__ wl, uint32_t Wsplit,
                                                  uint32_t Wall, uint32_t K, uint32_t S,
                                                  const uint32_t *__restrict__ nb,
                                                  const uint32_t *__restrict__ tb,
                                                  const uint2 *__restrict__ base,
                                                  uint4 *__restrict__ erec,
                                                  const uint32_t *__restrict__ dyn, uint32_t Wstat) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= S) return;
  if (dyn) Wall = min(Wstat + dyn[0], Wall);
  uint32_t va, vb;
  if (base) {
    const uint2 B = base[q];
    va = B.x;
    vb = B.y;
  } else {
    va = nb[q];
    vb = tb[q];
  }
  uint32_t x = q * K;
  for (uint32_t steps = 0; steps <= Wall; steps++) {
    const uint64_t v = wl[x];
    const uint32_t a = (uint32_t)v, nx = (uint32_t)(v >> 32);
    if (vb < Wall) erec[vb] = make_uint4(x, va, a, 0u);
    va += a;
    vb++;
    // (the first walk flagged a bad link; stop where it stopped)
    if (nx == NX_END || nx >= Wall || (nx < Wsplit && nx % K == 0)) break;
    x = nx;
  }
}

constexpr uint32_t SUP_MAX = 8192;  // elements k_sup_rank ranks in LDS (12 B each)

__global__ __launch_bounds__(1024) void k_sup_rank(const uint32_t *__restrict__ scnt,
                                                   const uint32_t *__restrict__ ssub,
                                                   const uint32_t *__restrict__ snext, uint32_t stride,
                                                   uint32_t S2,
                                                   uint32_t n, uint32_t Weff, uint32_t *__restrict__ nb,
                                                   uint32_t *__restrict__ tb,
                                                   uint32_t *__restrict__ status,
                                                   uint32_t *__restrict__ order = nullptr,
                                                   const uint32_t *__restrict__ dyn = nullptr,
                                                   uint32_t Wstat = 0, uint32_t Wcap = 0) {
  // the top level (<= 8192 elements) ranked by pointer jumping in LDS: suffix
  // sums of nodes and sublists along the list, element 0 (the root's) first.
  // ssub == nullptr: the elements are the sublists themselves (one each), and
  // order[tour index] = element replaces tb (a giant document of few sublists
  // ranks them here directly, without the walk levels)
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];  // next, count, sublists
  constexpr uint32_t PT = 8;  // elements per thread: S2 <= 8192
  // dyn: the walkers in use are Wstat + dyn[0] (<= Wcap), known on the device only;
  // the elements are those walkers themselves when ssub == nullptr
  if (dyn) {
    Weff = min(Wstat + dyn[0], Wcap);
    if (!ssub) S2 = Weff;
  }
  uint32_t *nx = sm, *cn = sm + S2, *sb = sm + 2 * S2;
  for (uint32_t i = threadIdx.x; i < S2; i += blockDim.x) {
    nx[i] = snext[(size_t)i * stride];  // (stride: the fields of packed records)
    cn[i] = scnt[(size_t)i * stride];
    sb[i] = ssub ? ssub[(size_t)i * stride] : 1u;
  }
  __syncthreads();
  for (uint32_t round = 0; (1u << round) < 2 * S2; round++) {
    uint32_t a[PT], b[PT], q2[PT];
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) {
      const uint32_t i = threadIdx.x + k * blockDim.x;
      if (i < S2) {
        const uint32_t q = nx[i];
        const bool on = q < S2;
        a[k] = cn[i] + (on ? cn[q] : 0u);
        b[k] = sb[i] + (on ? sb[q] : 0u);
        q2[k] = on ? nx[q] : NX_END;
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) {
      const uint32_t i = threadIdx.x + k * blockDim.x;
      if (i < S2) {
        cn[i] = a[k];
        sb[i] = b[k];
        nx[i] = q2[k];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && (S2 == 0 || cn[0] != n || sb[0] != Weff))
    atomicOr(&status[0], (uint32_t)CW_STATUS_INTERNAL);
  for (uint32_t i = threadIdx.x; i < S2; i += blockDim.x) {
    nb[i] = n - min(cn[i], n);
    const uint32_t t = Weff - min(sb[i], Weff);
    if (!order) tb[i] = t;
    else if (t < Weff) order[t] = i;
  }
}

// --- emit: sublist slots -> weave order ------------------------------------------
// Entry k of sublist x is the node at weave position sbase[x] + k.  One lane
// per sublist (its slot is contiguous); a block covers 256 consecutive
// sublists of one document.
__global__ __launch_bounds__(256) void k_emit(
    const uint32_t *__restrict__ slots, const uint64_t *__restrict__ slot_first,
    const uint32_t *__restrict__ wcnt, const uint32_t *__restrict__ sbase,
    const uint32_t *__restrict__ order, const uint32_t *__restrict__ sval,
    const uint4 *__restrict__ erec, const uint32_t *__restrict__ eblk_doc,
    const uint32_t *__restrict__ eblk_x0, const uint32_t *__restrict__ walk_first,
    const uint32_t *__restrict__ doc_W, const uint32_t *__restrict__ dyn_ctr,
    const uint32_t *__restrict__ doc_log2cap, const uint32_t *__restrict__ doc_off,
    uint32_t *__restrict__ perm, uint8_t *__restrict__ vis8, uint32_t *__restrict__ vcount,
    uint32_t *__restrict__ status) {
  // The block's sublists are consecutive in tour order, so their entries fill
  // one contiguous range of weave positions: stage it in LDS, then write it
  // out coalesced (full lines instead of one 4-byte store per lane and line).
  __shared__ uint32_t wtot[4];
  __shared__ uint32_t stage_p[EMIT_STAGE];
  __shared__ uint8_t stage_v[EMIT_STAGE];
  __shared__ uint32_t P0s;
  const uint32_t b = xcd_tile(blockIdx.x, gridDim.x), d = eblk_doc[b];
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, f = walk_first[d];
  const uint32_t Weff = min(doc_W[d] + dyn_ctr[d], walk_first[d + 1] - f);
  const uint32_t log2cap = doc_log2cap[d], cap = 1u << log2cap;
  const uint32_t ti = eblk_x0[b] + threadIdx.x;  // tour index
  uint32_t nvis = 0, cnt = 0, p0 = 0;
  bool bad = false;
  // erec (one giant document): {sublist, node base, count} in tour order, read
  // coalesced; otherwise the sublist from order and its tables
  uint4 rec = make_uint4(0u, 0u, 0u, 0u);
  if (erec && ti < Weff) rec = erec[f + ti];
  const uint32_t x = ti < Weff ? (erec ? rec.x : order[f + ti]) : 0u;
  const uint4 *sl4 = nullptr;
  if (ti < Weff) {
    if (x < Weff) {
      cnt = erec ? rec.z : wcnt[f + x];
      p0 = erec ? rec.y : sbase[f + x];
      sl4 = reinterpret_cast<const uint4 *>(slots + slot_first[d] + ((size_t)x << log2cap));
      if (p0 + cnt > n || cnt > cap) bad = true;
    } else {
      bad = true;
    }
  }
  if (bad) cnt = 0;
  uint32_t total;
  const uint32_t off = block_exscan<0>(cnt, wtot, &total);
  if (threadIdx.x == 0) P0s = p0;  // lane 0 holds the block's first sublist
  __syncthreads();
  const uint32_t P0 = P0s;
  if (cnt && p0 != P0 + off) {  // tour order and sublist bases disagree
    bad = true;
    cnt = 0;
  }
  const bool staged = total <= EMIT_STAGE && P0 + total <= n;
  for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
    const uint4 q = sl4[k0 >> 2];
    const uint32_t e4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t k = k0 + u;
      if (k >= cnt) break;
      const uint32_t r = e4[u] & SLOT_IDX;
      if (r >= n) {
        bad = true;
        continue;
      }
      const uint32_t v = e4[u] >> 31;
      const uint32_t pv = sval ? sval[base + r] : r;
      if (staged) {
        stage_p[off + k] = pv;
        stage_v[off + k] = (uint8_t)v;
      } else {
        perm[base + p0 + k] = pv;
        vis8[base + p0 + k] = (uint8_t)v;
      }
      nvis += v;
    }
  }
  if (staged) {
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < total; j += 256) {
      perm[base + P0 + j] = stage_p[j];
      vis8[base + P0 + j] = stage_v[j];
    }
  }
  if (bad) atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
  uint32_t vtotal;
  block_exscan<0>(nvis, wtot, &vtotal);
  if (threadIdx.x == 0 && vtotal) atomicAdd(&vcount[d], vtotal);
}

// --- fused tour for documents of < 2^16 nodes: walk, rank and emit in LDS --------
// The whole successor list of one document (u16 per node), its render and
// splitter bits and the sublist tables (u16) stay in LDS, one workgroup per
// document:
//   walk   every sublist (splitter to splitter) for its length and successor
//          sublist; each lane runs its own walker state machine and takes the
//          next sublist from an LDS counter as soon as one ends (a wave never
//          waits for its longest walk); each node's (sublist, index) goes to
//          HBM scratch with fire-and-forget stores;
//   jump   suffix sums over the sublists by pointer jumping -> sublist bases;
//   place  coalesced over nodes: position = base + index, sval (u16) into an
//          LDS weave where the successors were, render bits by position;
//   write  weave_perm and render bytes, coalesced.
// Replaces k_walk + k_rank + k_emit and their slot buffer in HBM.
constexpr uint32_t TOUR_END = 0xFFFFu;
constexpr uint32_t TOUR_LDS_MAX = 159 * 1024;  // dynamic LDS of k_tour (static: < 1 KiB)

__host__ __device__ inline uint32_t tour_lds_bytes(uint32_t nmax, uint32_t log2k) {
  const uint32_t S = (nmax + (1u << log2k) - 1) >> log2k;
  // succ u16 (later sval u16), render + splitter bits, acc/nx u16
  return 4 * ((nmax + 1) / 2 + 2 * ((nmax + 31) / 32) + S);
}

template <int NT, typename VT = uint32_t>
__device__ __forceinline__ void tour_doc(const uint32_t *__restrict__ link,
                                             const VT *__restrict__ sval,
                                             const uint32_t *__restrict__ doc_off,
                                             const uint32_t *__restrict__ doc_log2k,
                                             const uint64_t *__restrict__ skey, uint32_t ts_shift,
                                             uint64_t *__restrict__ max_ts,
                                             uint32_t *__restrict__ perm, uint32_t *__restrict__ vbits,
                                             uint32_t *__restrict__ vcount,
                                             uint32_t *__restrict__ status, uint32_t *loc,
                                             unsigned long long *__restrict__ tprof,
                                             uint32_t d, uint32_t *sm) {
  constexpr uint32_t SPT = 8;  // sublists per thread in the jumping rounds: S <= SPT * NT
  __shared__ uint32_t wtot[NT / 64];
  __shared__ uint32_t bad_s, next_j;
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = 0;
  auto stamp = [&](int ph) {  // diagnostic phase times (CW_TREE_PROF)
    if (tprof) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tacc[ph] += now - tlast;
      tlast = now;
    }
  };
  stamp(-1);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base, log2k = doc_log2k[d];
  const uint32_t *const linkD = link + base;
  uint32_t *const locD = loc + base, *const permD = perm + base;
  if (tid == 0 && max_ts) max_ts[d] = n ? (skey[base + n - 1] >> ts_shift) : 0ull;
  if (n == 0) return;
  const uint32_t S = (n + (1u << log2k) - 1) >> log2k, nw = (n + 31) / 32;
  uint16_t *succ = reinterpret_cast<uint16_t *>(sm);
  uint32_t *vbm = sm + (n + 1) / 2, *sbm = vbm + nw;
  // per sublist: acc (nodes, later the suffix sum) | next sublist << 16, one word
  uint32_t *const sub = sbm + nw;
  if (tid == 0) {
    bad_s = 0;
    next_j = NT;  // the first NT walkers are handed out by thread index
  }
  // load: successor (SUCC_END -> TOUR_END), render and splitter bits (ballots),
  // 8 loads in flight per lane
  constexpr uint32_t LU = 8;
  for (uint32_t r0 = wv * 64; r0 < n; r0 += NT * LU) {
    uint32_t L[LU];
#pragma unroll
    for (uint32_t k = 0; k < LU; k++) {
      const uint32_t r = r0 + k * NT + lane;
      L[k] = r < n ? lane_at(linkD, r) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < LU; k++) {
      const uint32_t rb = r0 + k * NT, r = rb + lane, u = L[k] & LINK_IDX;
      if (r < n) succ[r] = (uint16_t)(u < n ? u : TOUR_END);
      const uint64_t vm = __ballot(r < n && (L[k] & LINK_VIS));
      const uint64_t sp = __ballot(r < n && (L[k] & LINK_SPLIT));
      if (lane == 0 && rb < n) {
        vbm[rb >> 5] = (uint32_t)vm;
        sbm[rb >> 5] = (uint32_t)sp;
        if ((rb >> 5) + 1 < nw) {
          vbm[(rb >> 5) + 1] = (uint32_t)(vm >> 32);
          sbm[(rb >> 5) + 1] = (uint32_t)(sp >> 32);
        }
      }
    }
  }
  __syncthreads();
  stamp(0);
  bool bad = false;
  // pass 1: per-lane walker state machines over the sublists; every node's
  // (sublist, index inside it) goes to HBM scratch (fire-and-forget stores).
  // A step reads the node's successor and its splitter bit together (one LDS
  // round trip a node; round 5: 12.28 -> 12.22 ms a config-2 step.  Two
  // walkers a lane stepped together lost, 12.54 ms, and so did the tree's two
  // chains a lane in its list walk and pointer jumping, 13.04 ms:
  // profiles/r05_tour_chains_ab.txt)
  {
    uint32_t j = tid, u = 0, cnt = 0;
    bool live = j < S;
    if (live) {
      const uint32_t v = split_node(d, j, log2k, n);
      lane_at(locD, v) = j << 16;
      u = succ[v];
      cnt = 1;
    }
    while (live) {
      const uint32_t us = u < n ? u : 0u;
      const uint32_t nx = succ[us], sw = sbm[us >> 5];  // both reads in flight
      const bool end = u >= n || ((sw >> (us & 31)) & 1u) || cnt > n;
      if (end) {
        bad |= (u != TOUR_END && u >= n) || cnt > n;
        sub[j] = min(cnt, 0xFFFFu) | (u < n ? (u >> log2k) : TOUR_END) << 16;
        j = atomicAdd(&next_j, 1u);
        live = j < S;
        if (live) {
          const uint32_t v = split_node(d, j, log2k, n);
          lane_at(locD, v) = j << 16;
          u = succ[v];
          cnt = 1;
        }
      } else {
        lane_at(locD, u) = (j << 16) | cnt;
        cnt++;
        u = nx;
      }
    }
  }
  __syncthreads();
  if (tid == 0) next_j = NT;
  stamp(1);
  // suffix sums along the sublist list by pointer jumping: sub[j] & 0xFFFF = nodes from
  // sublist j to the end of the tour (<= n < 2^16)
  for (uint32_t round = 0; (1u << round) < 2 * S; round++) {
    uint32_t na[SPT], nn[SPT];
#pragma unroll
    for (uint32_t k = 0; k < SPT; k++) {
      const uint32_t j = tid + k * NT;
      if (j < S) {
        const uint32_t sj = sub[j], q = sj >> 16;
        const uint32_t sq = q < S ? sub[q] : TOUR_END << 16;
        na[k] = (sj & 0xFFFFu) + (sq & 0xFFFFu);
        nn[k] = sq >> 16;
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < SPT; k++) {
      const uint32_t j = tid + k * NT;
      if (j < S) {
        sub[j] = min(na[k], 0xFFFFu) | nn[k] << 16;
      }
    }
    __syncthreads();
  }
  stamp(2);
  if (tid == 0 && (sub[0] & 0xFFFFu) != n) bad_s = 1;  // the root's sublist starts the tour
  // place: coalesced over nodes, position = sublist base + index; the weave
  // (sval as u16) and its render bits are assembled in LDS where the
  // successors and splitter bits were, then written out coalesced.  (The
  // scratch stores above are read by other waves of this workgroup: one CU,
  // one L1, lines not cached before; the barriers order them.)
  uint16_t *out = succ;
  uint32_t *pvis = sbm;
  for (uint32_t w = tid; w < nw; w += NT) pvis[w] = 0;
  __syncthreads();
  for (uint32_t r0 = tid; r0 < n; r0 += NT * LU) {
    uint32_t lc[LU], x[LU];
#pragma unroll
    for (uint32_t k = 0; k < LU; k++) {
      const uint32_t r = r0 + k * NT;
      lc[k] = r < n ? lane_at(locD, r) : 0u;
      x[k] = r < n ? (sval ? lane_at(sval + base, r) : r) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < LU; k++) {
      const uint32_t r = r0 + k * NT;
      if (r >= n) continue;
      const uint32_t j = lc[k] >> 16;
      const uint32_t pos = (j < S ? n - min(sub[j] & 0xFFFFu, n) : n) + (lc[k] & 0xFFFFu);
      if (pos >= n) {
        bad = true;
        continue;
      }
      out[pos] = (uint16_t)x[k];
      if ((vbm[r >> 5] >> (r & 31)) & 1u) atomicOr(&pvis[pos >> 5], 1u << (pos & 31));
    }
  }
  __syncthreads();
  stamp(3);
  uint32_t nvis = 0;
  for (uint32_t g = tid; g < n; g += NT) lane_at(permD, g) = out[g];
  for (uint32_t w = tid; w < nw; w += NT) nvis += __popc(pvis[w]);
  if (vbits) {
    // the render bits straight into the batch's bitmap: global word W holds
    // positions [32 W, 32 W + 32); the two end words are shared with the
    // neighbouring documents (atomicOr on a zeroed bitmap)
    const uint32_t W0 = base >> 5, W1 = (base + n - 1) >> 5;
    for (uint32_t W = W0 + tid; W <= W1; W += NT) {
      const uint32_t lo = max(W << 5, base), hi = min((W << 5) + 32, base + n);
      const uint32_t g = lo - base, len = hi - lo, w0 = g >> 5, off = g & 31;
      uint32_t x = pvis[w0] >> off;
      if (off && w0 + 1 < nw) x |= pvis[w0 + 1] << (32 - off);
      if (len < 32) x &= (1u << len) - 1;
      x <<= lo - (W << 5);
      if (W == W0 || W == W1) {
        if (x) atomicOr(&vbits[W], x);
      } else {
        vbits[W] = x;
      }
    }
  }
  uint32_t total;
  block_exscan<NT>(nvis, wtot, &total);
  if (__syncthreads_or(bad) || bad_s) {
    if (tid == 0) atomicOr(&status[d], (uint32_t)CW_STATUS_INTERNAL);
  }
  if (tid == 0) vcount[d] = total;
  stamp(4);
  if (tprof && tid == 0)
    for (int ph = 0; ph < 6; ph++) tprof[(size_t)d * 8 + ph] = tacc[ph];
}

template <int NT>
__global__ __launch_bounds__(NT) void k_tour(const uint32_t *__restrict__ link,
                                             const uint32_t *__restrict__ sval,
                                             const uint32_t *__restrict__ doc_off,
                                             const uint32_t *__restrict__ doc_log2k,
                                             const uint64_t *__restrict__ skey, uint32_t ts_shift,
                                             uint64_t *__restrict__ max_ts,
                                             uint32_t *__restrict__ perm, uint32_t *__restrict__ vbits,
                                             uint32_t *__restrict__ vcount,
                                             uint32_t *__restrict__ status, uint32_t *loc,
                                             unsigned long long *__restrict__ tprof,
                                             uint32_t doc0 = 0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_t[];
  tour_doc<NT>(link, sval, doc_off, doc_log2k, skey, ts_shift, max_ts, perm, vbits, vcount, status, loc, tprof, doc0 + blockIdx.x, lds_t);
}

// --- the whole weave of one document in ONE workgroup (CW_FUSED, round 3) -------
// front end, tree and tour of document blockIdx.x back to back: the three
// phases reuse the same LDS, the handoffs (par, class bitmaps, sval; nsc, fcS;
// link) go through memory written by this workgroup a moment earlier (its
// L2 slice has them), the CUs of the chip are at different phases at any time
// (the front end streams HBM while the tree and the tour wait on LDS), and
// there is one tail instead of three.  A document whose ids leave the front
// end's directory counts itself in big[0] and stops: the host then weaves the
// batch with the separate kernels.
template <int NT, int TILE_T, typename VT, bool PROF, int TLM = 0, int FV = 0>
__global__ __launch_bounds__(NT) void k_weave_doc(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause_key,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ tile_first, uint32_t sg, uint16_t *__restrict__ par,
    uint8_t *__restrict__ skind, VT *__restrict__ sval, uint32_t *__restrict__ kbm,
    uint64_t *__restrict__ skey, uint16_t *rank16, uint64_t *__restrict__ max_ts, uint32_t ts_shift,
    uint32_t *__restrict__ status, uint32_t *__restrict__ big, const uint32_t *__restrict__ doc_log2k,
    uint32_t kbits, uint32_t bm_words, uint32_t *__restrict__ nsc, uint32_t *__restrict__ fcS,
    uint32_t *__restrict__ link, uint32_t *__restrict__ osp, uint32_t *__restrict__ perm,
    uint32_t *__restrict__ vbits, uint32_t *__restrict__ vcount, uint32_t *loc,
    unsigned long long *__restrict__ tprof, uint8_t *__restrict__ site8, uint32_t site_shift,
    uint32_t site_mask) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_w[];
  const uint32_t d = blockIdx.x;
  // (tprof, CW_TREE_PROF: the three phases' clocks per document)
  const unsigned long long t0 = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  // FV (CW_FRONT_U): items in flight per thread in the front end's directory
  // and input-index passes (1: 16, 0: 4 as in k_front); the rank pass loads
  // and ranks 6 items a thread in turn (round 5: 4 double-buffered, 12.17 ->
  // 12.11 ms a config-2 step; 8 spill)
  constexpr uint32_t U1 = FV == 0 ? 4 : 16, U2 = 6, U3 = U1;
  if (!front_doc<NT, uint16_t, VT, U1, U2, U3>(id_key, cause_key, kind, doc_off, tile_first, sg, par, skind, sval, kbm, skey,
                     rank16, max_ts, ts_shift, status, big, nullptr, d,
                     reinterpret_cast<uint4 *>(lds_w), site8, site_shift, site_mask))
    return;
  __syncthreads();  // (workgroup-scope release/acquire: this CU's writes are visible to it)
  const unsigned long long t1 = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  tree_l_doc<NT, TILE_T, false, TLM, uint16_t>(par, skind, doc_off, doc_log2k, kbits, bm_words, nsc, fcS, link,
                                   osp, nullptr, kbm, tile_first, d, lds_w);
  __syncthreads();
  const unsigned long long t2 = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  tour_doc<NT, VT>(link, sval, doc_off, doc_log2k, nullptr, 0u, nullptr, perm, vbits, vcount, status,
                   loc, nullptr, d, lds_w);
  if (PROF && threadIdx.x == 0) {
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    tprof[(size_t)d * 4] = t1 - t0;
    tprof[(size_t)d * 4 + 1] = t2 - t1;
    tprof[(size_t)d * 4 + 2] = t3 - t2;
  }
}

// The yarns of the documents k_weave_doc took (spin 1-arity, shared.cljc:121-132:
// the id order partitioned by site, id-ascending inside a site), one workgroup
// per document after it, from what it leaves in HBM: every input's rank
// (rank16) and site byte (site8, written by the fused kernel's front end) and
// every rank's input index (sval16).  In LDS: the site of every rank (a byte,
// 50 KB at 50,001 nodes: two workgroups a CU); the yarn is written straight
// from a wave-level multisplit, each wave's ranks going to 16 runs that grow a
// chunk at a time; each wave's per-site counts are LDS atomics made while the
// sites are scattered (round 6: a pass of ballots over the site bytes before,
// yarns 1.46-1.49 -> 1.36-1.40 ms).  9 B a node: site 1 + rank 2 + sval 2 in,
// yarn_perm 4 out (+1 B in the fused kernel for the site byte).  Round 4 placed the yarns
// inside the fused kernel's front end: +3.9 ms on a config-2 step; round 5:
// an LDS-staged version there, +3.8 ms; this kernel with per-thread rank
// ranges and the yarn staged in LDS, 2.60 ms; the multisplit with no staging,
// 2.37 ms; site bytes instead of ids, 1.76 ms; the input indices loaded eight
// chunks at a time, 1.47 ms (profiles/r05_yarn_ab.txt).
__host__ __device__ inline uint32_t yarn_lds_bytes(uint32_t nmax) {
  return (nmax + 3) & ~3u;  // the site of every rank (a byte)
}

template <int NT>
__global__ __launch_bounds__(NT) void k_yarn_doc(const uint8_t *__restrict__ site8,
                                                 const uint16_t *__restrict__ rank16,
                                                 const uint16_t *__restrict__ sval16,
                                                 const uint32_t *__restrict__ doc_off,
                                                 uint32_t *__restrict__ yarn) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_y[];
  __shared__ uint32_t wrow[NT / 64][16];
  const uint32_t tid = threadIdx.x;
  const uint32_t d = blockIdx.x;
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base;
  uint8_t *const sr = reinterpret_cast<uint8_t *>(lds_y);
  for (uint32_t w = tid; w < (n + 3) / 4; w += NT) lds_y[w] = 0xFFFFFFFFu;  // (no site: a DUP doc)
  constexpr uint32_t NW = NT / 64;
  const uint32_t perw = ((n + NW - 1) / NW + 63) & ~63u;  // ranks a wave places (pass B)
  for (uint32_t w = tid; w < NW * 16; w += NT) (&wrow[0][0])[w] = 0;
  __syncthreads();
  // 1. the site of every rank (the fused kernel's front end wrote each input's
  // site byte beside its rank)
  constexpr uint32_t U = 16;
  for (uint32_t i0 = tid; i0 < n; i0 += U * NT) {
    uint32_t x[U], r[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t i = i0 + u * NT;
      x[u] = i < n ? lane_at(site8 + base, i) : 0u;
      r[u] = i < n ? lane_at(rank16 + base, i) : 0xFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (r[u] < n) {
        sr[r[u]] = (uint8_t)x[u];
        // each wave's per-site counts over the ranks it places, counted here
        // rather than in a pass over the site bytes (round 6)
        atomicAdd(&wrow[r[u] / perw][x[u] & 15u], 1u);
      }
  }
  __syncthreads();
  // 2-3. a wave-level multisplit: wave wv owns a contiguous range of ranks and
  // takes them 64 at a time, lane = rank; four ballots of the site bits give
  // every lane the mask of its site's lanes, so a site's count is a popcount
  // and a rank's place among its site's ranks of the chunk is the popcount of
  // that mask below the lane.  Pass A counts per site and wave (wave-uniform
  // registers), the 16 x 16 totals go through LDS, pass B places every rank's
  // input index at its site's running offset (lane s of the wave holds site
  // s's).  (Round 5 v3 gave each thread a contiguous range and sixteen 16-bit
  // counters: 2.55 ms a config-2 step, its counting and placement ALU-bound.)
  {
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t w0 = min(n, wv * perw), w1 = min(n, w0 + perw);
    // the lanes of site `st` among this chunk's ballots (st = 0xFF: none)
    auto site_mask = [&](uint32_t st, uint64_t valid, uint64_t b0, uint64_t b1, uint64_t b2,
                         uint64_t b3) -> uint64_t {
      return valid & ((st & 1u) ? b0 : ~b0) & ((st & 2u) ? b1 : ~b1) & ((st & 4u) ? b2 : ~b2) &
             ((st & 8u) ? b3 : ~b3);
    };
    // (pass A, the per-site counts of the wave's ranks, came with the scatter)
    // lane s: the ranks of sites < s (all waves) + of site s in earlier waves
    uint32_t before = 0, tot = 0;
    if (lane < 16) {
#pragma unroll 1
      for (uint32_t i = 0; i < NW; i++) {
        const uint32_t t = wrow[i][lane];
        before += i < wv ? t : 0u;
        tot += t;
      }
    }
    uint32_t ex = tot;  // exclusive scan of the site totals over lanes 0..15
#pragma unroll
    for (uint32_t o = 1; o < 16; o <<= 1) {
      const uint32_t y = __shfl_up(ex, o, 64);
      if (lane >= o) ex += y;
    }
    uint32_t off = ex - tot + before;  // lane s: where this wave's next site-s rank goes
    // pass B: the input indices of PB chunks loaded together (one HBM latency
    // per PB chunks, not per chunk)
    const uint16_t *const svD = sval16 + base;
    uint32_t *const yD = yarn + base;
    constexpr uint32_t PB = 8;
    for (uint32_t c0 = w0; c0 < w1; c0 += PB * 64) {
      uint32_t v[PB];
#pragma unroll
      for (uint32_t k = 0; k < PB; k++) {
        const uint32_t r = c0 + k * 64 + lane;
        v[k] = r < w1 ? svD[r] : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < PB; k++) {
        const uint32_t c = c0 + k * 64;
        if (c >= w1) break;  // (wave-uniform)
        const uint32_t r = c + lane;
        const uint32_t st = r < w1 ? sr[r] : 0xFFu;
        const uint64_t valid = __ballot(st < 16u), b0 = __ballot(st & 1u), b1 = __ballot(st & 2u),
                       b2 = __ballot(st & 4u), b3 = __ballot(st & 8u);
        const uint32_t base_s = __shfl(off, st & 15u, 64);
        if (st < 16u) yD[base_s + lanes_below(site_mask(st, valid, b0, b1, b2, b3))] = v[k];
        off += (uint32_t)__popcll(site_mask(lane, valid, b0, b1, b2, b3));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_pack_bits(const uint8_t *__restrict__ vis8, uint32_t N,
                                                   uint32_t *__restrict__ bits) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g0 = w * 32;
  if (g0 >= N) return;
  uint32_t m = 0;
  if (g0 + 32 <= N) {
    const uint4 a = *reinterpret_cast<const uint4 *>(vis8 + g0);
    const uint4 b = *reinterpret_cast<const uint4 *>(vis8 + g0 + 16);
    const uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 8; q++)
#pragma unroll
      for (int y = 0; y < 4; y++) m |= ((x[q] >> (8 * y)) & 1u) << (4 * q + y);
  } else {
    for (uint32_t g = g0; g < N; g++) m |= (uint32_t)(vis8[g] & 1u) << (g - g0);
  }
  bits[w] = m;
}

__global__ void k_max_ts1(const uint64_t *__restrict__ skey, uint32_t n, uint32_t ts_shift,
                          uint64_t *__restrict__ max_ts) {
  if (threadIdx.x == 0) max_ts[0] = n ? skey[n - 1] >> ts_shift : 0ull;
}

// OR of two key arrays at once (map ids and causes: one readback)
__global__ void k_or_reduce2(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
                             uint32_t N, unsigned long long *__restrict__ out) {
  uint64_t x = 0, y = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    x |= a[i];
    y |= b[i];
  }
  for (int o = 32; o > 0; o >>= 1) {
    x |= __shfl_xor(x, o, 64);
    y |= __shfl_xor(y, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (x) atomicOr(&out[0], (unsigned long long)x);
    if (y) atomicOr(&out[1], (unsigned long long)y);
  }
}

__global__ void k_or_reduce(const uint64_t *__restrict__ keys, uint32_t N,
                            unsigned long long *__restrict__ out) {
  uint64_t acc = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    acc |= keys[i];
  for (int o = 32; o > 0; o >>= 1) acc |= __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicOr(out, (unsigned long long)acc);
}

// K64 keys are < 2^63 (include/causeweave.h): flag the documents of a batch
// whose ids use the top bit (run only when the batch's keys reach 64 bits).
__global__ __launch_bounds__(256) void k_key_range(const uint64_t *__restrict__ id,
                                                   const uint32_t *__restrict__ tile_start,
                                                   const uint32_t *__restrict__ tile_doc,
                                                   uint32_t *__restrict__ status) {
  const uint32_t t = blockIdx.x;
  bool hi = false;
  for (uint32_t i = tile_start[t] + threadIdx.x; i < tile_start[t + 1]; i += blockDim.x)
    hi |= (id[i] >> 63) != 0;
  if (__syncthreads_or(hi) && threadIdx.x == 0)
    atomicOr(&status[tile_doc[t]], (uint32_t)CW_STATUS_KEY_RANGE);
}

// ============================================================================
// Maps (c.map/weave 1-arity, map.cljc:26-45): every (collection, key) pair is
// an independent list weave rooted at a virtual [[0 "0" 0] nil nil].  The map
// kernels resolve each node's key, group nodes by key and lay every key weave
// out as a list document (root first), which the list pipeline then weaves.
// ============================================================================
constexpr uint32_t MAP_NO_PARENT = 0xFFFFFFFFu;  // cause-in-weave = the virtual root
constexpr uint32_t MAP_CHAIN = 0xFFFFFFFEu;      // orphan: appended after its predecessor
constexpr uint32_t MAP_ORPHAN = 0xFFFFFFFDu;     // nil key: the absent cause id itself (the
                                                 // list pipeline flags ORPHAN, the literal fold
                                                 // appends the node)

// Per id-sorted node: the key (map.cljc:31-34) as a grouping value and the
// rank of its cause-in-weave (map.cljc:35-37).  Grouping values, with
// W = max(token_bits, key_bits):
//   token t                         t              (cause is a key)
//   id X               1 << W | X     (the cause node is id-caused by X)
//   nil                             2 << W         (the cause node is absent, or
//                                                   the cause or the cause node's
//                                                   cause is nil: cause_is_id = 2)
// In an id key weave X no node's cause is in the weave (each is an orphan
// there), so weave-node appends every node at the end: the weave is the root
// then the nodes in id order (shared.cljc:226-241, asap never holds) -- a chain.
// The one exception is a self-caused X (cause = id: the spec of new-node
// forbids it, shared.cljc:98, but a ::nodes map can hold it): node n lands in
// the key weave cause(cause(n)) and its cause c in cause(cause(c)), equal for
// every n exactly when cause(X) = X, so X, its children and its grandchildren
// all share the key weave X with their causes in it.  Those nodes keep their
// real cause-in-weave; X's own cause is X, so the list pipeline flags the key
// weave NON_LAMPORT and the literal fold (exact.hip) weaves it.
// The nil key weave also holds nodes caused by the root id [0 "0" 0] or by nil
// (cause-in-weave = the root, map.cljc:35-37) and their children, next to the
// appended orphans: its nodes keep their real cause-in-weave, the list pipeline
// flags the orphans and the literal fold (exact.hip) weaves that key weave.
// Is the id key X of a node caused by c self-caused (see above)?  c is the
// node's cause, found in the collection; X is that cause node's cause id.
__device__ __forceinline__ bool map_self_key(const uint64_t *__restrict__ skey,
                                             const uint32_t *__restrict__ sval,
                                             const uint64_t *__restrict__ cause,
                                             const uint8_t *__restrict__ cause_is_id, uint32_t n,
                                             uint64_t c, uint64_t X) {
  if (X == c) return true;  // the cause node is X itself
  const uint32_t rx = lower_bound_u64(skey, n, X);
  if (rx >= n || skey[rx] != X) return false;
  const uint32_t gx = sval[rx];
  return cause_is_id[gx] == 1 && cause[gx] == X;
}

__global__ __launch_bounds__(256) void k_map_key(
    const uint64_t *__restrict__ skey, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ cause, const uint8_t *__restrict__ cause_is_id,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ tile_start,
    const uint32_t *__restrict__ tile_doc, const uint32_t *__restrict__ doc_off,
    uint32_t token_bits, uint32_t W, uint64_t *__restrict__ segk, uint32_t *__restrict__ mpar,
    uint8_t *__restrict__ mkind, uint32_t *__restrict__ status) {
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x), d = tile_doc[t];
  const uint32_t base = doc_off[d], n = doc_off[d + 1] - base;
  const uint32_t s = tile_start[t], e = tile_start[t + 1];
  const uint64_t tmask = (1ull << token_bits) - 1;
  uint32_t bad = 0;
  for (uint32_t i = s + threadIdx.x; i < e; i += blockDim.x) {
    const uint32_t gi = base + sval[i];
    const uint64_t c = cause[gi];
    uint64_t key;
    uint32_t p;
    if (i > base && skey[i - 1] == skey[i]) bad |= CW_STATUS_DUP;
    const uint8_t ci = cause_is_id[gi];
    if (ci == 1) {
      const uint32_t r = lower_bound_u64(skey + base, n, c);
      if (r < n && skey[base + r] == c) {
        const uint32_t gc = base + sval[base + r];
        const uint8_t cci = cause_is_id[gc];
        if (cci == 1) {
          const uint64_t X = cause[gc];
          key = (1ull << W) | X;
          p = map_self_key(skey + base, sval + base, cause + base, cause_is_id + base, n, c, X)
                  ? r : MAP_CHAIN;
        } else if (cci == 2) {  // the cause node's cause is nil: the nil key, under it
          key = 2ull << W;
          p = r;
        } else {
          key = cause[gc] & tmask;
          if (cause[gc] > tmask) bad |= CW_STATUS_MAP_KEY;
          p = r;
        }
      } else {  // the cause node is absent: the nil key; the root id is its root
        key = 2ull << W;
        p = c == 0 ? MAP_NO_PARENT : MAP_ORPHAN;
      }
    } else if (ci == 2) {  // a nil cause: the nil key, woven under its root
      key = 2ull << W;
      p = MAP_NO_PARENT;
    } else {
      key = c & tmask;
      if (c > tmask) bad |= CW_STATUS_MAP_KEY;
      p = MAP_NO_PARENT;
    }
    segk[i] = key;
    mpar[i] = p;
    mkind[i] = kind[gi];
  }
  if (bad) atomicOr(&status[d], bad);
}

// Key-weave heads in the key-sorted order: element j starts a key weave when
// it is the first of its collection or its key differs from j-1's.
__device__ __forceinline__ bool seg_head(const uint64_t *__restrict__ segk, uint32_t j,
                                         uint32_t cbase) {
  return j == cbase || segk[j] != segk[j - 1];
}

__global__ __launch_bounds__(256) void k_seg_count(const uint64_t *__restrict__ segk,
                                                   const uint32_t *__restrict__ tile_start,
                                                   const uint32_t *__restrict__ tile_doc,
                                                   const uint32_t *__restrict__ doc_off,
                                                   uint32_t *__restrict__ tile_cnt) {
  __shared__ uint32_t wtot[4];
  const uint32_t t = blockIdx.x, cbase = doc_off[tile_doc[t]];
  const uint32_t s = tile_start[t], e = tile_start[t + 1];
  uint32_t cnt = 0;
  for (uint32_t j = s + threadIdx.x; j < e; j += 256) cnt += seg_head(segk, j, cbase) ? 1u : 0u;
  uint32_t total;
  block_exscan<256>(cnt, wtot, &total);
  if (threadIdx.x == 0) tile_cnt[t] = total;
}

// Numbers the key weaves (tile_sbase = exclusive prefix of k_seg_count) and
// records, per key weave, its first sorted element, collection and key; per
// element, its key weave.  Each lane owns a contiguous run of the tile.
__global__ __launch_bounds__(256) void k_seg_mark(
    const uint64_t *__restrict__ segk, const uint32_t *__restrict__ tile_start,
    const uint32_t *__restrict__ tile_doc, const uint32_t *__restrict__ doc_off,
    const uint32_t *__restrict__ tile_sbase, uint32_t W, uint32_t *__restrict__ seg_of,
    uint32_t *__restrict__ seg_start, uint32_t *__restrict__ seg_coll,
    uint64_t *__restrict__ seg_key) {
  __shared__ uint32_t wtot[4];
  const uint32_t t = blockIdx.x, d = tile_doc[t], cbase = doc_off[d];
  const uint32_t s = tile_start[t], e = tile_start[t + 1];
  const uint32_t per = (e - s + 255) / 256;
  const uint32_t j0 = min(e, s + threadIdx.x * per), j1 = min(e, j0 + per);
  uint32_t cnt = 0;
  for (uint32_t j = j0; j < j1; j++) cnt += seg_head(segk, j, cbase) ? 1u : 0u;
  uint32_t sid = tile_sbase[t] + block_exscan<256>(cnt, wtot, nullptr) - 1;
  for (uint32_t j = j0; j < j1; j++) {
    if (seg_head(segk, j, cbase)) {
      sid++;
      seg_start[sid] = j;
      seg_coll[sid] = d;
      const uint64_t g = segk[j], cls = g >> W;
      seg_key[sid] = cls == 0 ? g : cls == 1 ? (CW_MAP_ID_KEY | (g & ((1ull << W) - 1))) : CW_NIL;
    }
    seg_of[j] = sid;
  }
}

// Lays the key weaves out as list documents: key weave s occupies
// [seg_start[s] + s, seg_start[s+1] + s + 1) with its root first.  Ids keep
// their packing (real ids are > 0, the virtual root is id 0).
__global__ __launch_bounds__(256) void k_seg_build(
    const uint64_t *__restrict__ skey, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ cause,
    const uint32_t *__restrict__ mpar, const uint8_t *__restrict__ mkind,
    const uint32_t *__restrict__ rank_s, const uint32_t *__restrict__ seg_of,
    const uint32_t *__restrict__ seg_coll, const uint32_t *__restrict__ coll_off, uint32_t N,
    uint64_t *__restrict__ lid, uint64_t *__restrict__ lcause, uint8_t *__restrict__ lkind,
    uint32_t *__restrict__ lmap) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const uint32_t sg = seg_of[j], cbase = coll_off[seg_coll[sg]];
  const uint32_t i = cbase + rank_s[j];
  const uint32_t out = j + sg + 1;
  const uint32_t p = mpar[i];
  uint64_t lc;
  if (p == MAP_NO_PARENT) {
    lc = 0ull;
  } else if (p == MAP_CHAIN) {  // the previous node of the key weave (or its root)
    lc = (j > 0 && seg_of[j - 1] == sg) ? skey[cbase + rank_s[j - 1]] : 0ull;
  } else if (p == MAP_ORPHAN) {  // the absent cause id: an orphan of the key weave
    lc = cause[cbase + sval[i]];
  } else {
    lc = skey[cbase + p];
  }
  lid[out] = skey[i];
  lcause[out] = lc;
  lkind[out] = mkind[i] & 3u;  // a map has no root node of its own
  lmap[out] = sval[i];
}

__global__ __launch_bounds__(256) void k_seg_roots(const uint32_t *__restrict__ seg_start,
                                                   uint32_t S, uint64_t *__restrict__ lid,
                                                   uint64_t *__restrict__ lcause,
                                                   uint8_t *__restrict__ lkind,
                                                   uint32_t *__restrict__ lmap) {
  const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
  if (sg >= S) return;
  const uint32_t out = seg_start[sg] + sg;
  lid[out] = 0;
  lcause[out] = CW_NIL;
  lkind[out] = CW_KIND_ROOT;
  lmap[out] = 0xFFFFFFFFu;
}

// Weave positions -> collection-local input indices (root -> UINT32_MAX).
__global__ __launch_bounds__(256) void k_seg_perm(const uint32_t *__restrict__ lperm,
                                                  const uint32_t *__restrict__ lmap,
                                                  const uint64_t *__restrict__ seg_off,
                                                  const uint32_t *__restrict__ seg_of,
                                                  const uint32_t *__restrict__ seg_start,
                                                  uint32_t N, uint32_t S,
                                                  uint32_t *__restrict__ seg_perm) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t g, sg;
  if (x < N) {
    sg = seg_of[x];
    g = x + sg + 1;
  } else if (x < N + S) {
    sg = x - N;
    g = seg_start[sg] + sg;
  } else {
    return;
  }
  const uint64_t o = seg_off[sg];
  seg_perm[g] = lmap[o + lperm[g]];
}

// active-node (map.cljc:47-59) per key weave, and the collection status.
// Scans the key weave from its first node; in practice it stops within a few.
__global__ __launch_bounds__(256) void k_seg_active(
    const uint32_t *__restrict__ lperm, const uint8_t *__restrict__ lkind,
    const uint32_t *__restrict__ seg_perm, const uint64_t *__restrict__ seg_off,
    const uint32_t *__restrict__ seg_coll, const uint32_t *__restrict__ lstatus, uint32_t S,
    int64_t *__restrict__ seg_active, uint32_t *__restrict__ status) {
  const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
  if (sg >= S) return;
  const uint64_t o = seg_off[sg];
  const uint32_t len = (uint32_t)(seg_off[sg + 1] - o);
  auto kd = [&](uint32_t p) { return (uint32_t)lkind[o + lperm[o + p]]; };
  int64_t act = -1;
  // [_ [_ _ first-v]]: a hide right after the root blanks the key
  if (!(len > 1 && is_hide(kd(1)))) {
    uint32_t k = len > 1 ? kd(1) : 0u;
    for (uint32_t p = 1; p < len; p++) {
      const uint32_t nk = p + 1 < len ? kd(p + 1) : 0u;
      if (!is_special(k) && !(p + 1 < len && is_hide(nk))) {
        act = (int64_t)seg_perm[o + p];
        break;
      }
      k = nk;
    }
  }
  seg_active[sg] = act;
  // an orphan is how the nil key weave appends (its literal fold ran): not a
  // status of the map; NON_LAMPORT stays as information
  const uint32_t ls = lstatus[sg] & ~(uint32_t)CW_STATUS_ORPHAN;
  if (ls) atomicOr(&status[seg_coll[sg]], ls);
}

// ============================================================================
// Merge (s/merge-trees, shared.cljc:300-314; bulk s/insert, :151-184): union
// of two node bags per document, deduplicated by id, then the list pipeline.
// ============================================================================
// Document d's a-nodes then b-nodes into one capacity slot [coff[d], coff[d+1]).
__global__ __launch_bounds__(256) void k_merge_concat(
    const uint64_t *__restrict__ aid, const uint64_t *__restrict__ acause,
    const uint8_t *__restrict__ akind, const uint64_t *__restrict__ aval,
    const uint64_t *__restrict__ bid, const uint64_t *__restrict__ bcause,
    const uint8_t *__restrict__ bkind, const uint64_t *__restrict__ bval,
    const uint32_t *__restrict__ aoff, const uint32_t *__restrict__ boff,
    const uint32_t *__restrict__ coff, uint64_t *__restrict__ cid,
    uint64_t *__restrict__ ccause, uint8_t *__restrict__ ckind, uint64_t *__restrict__ cval) {
  const uint32_t d = blockIdx.x;
  const uint32_t a0 = aoff[d], na = aoff[d + 1] - a0, b0 = boff[d], nb = boff[d + 1] - b0;
  const uint32_t c0 = coff[d];
  for (uint32_t i = threadIdx.x; i < na + nb; i += blockDim.x) {
    const bool fa = i < na;
    const uint32_t g = fa ? a0 + i : b0 + (i - na);
    cid[c0 + i] = fa ? aid[g] : bid[g];
    ccause[c0 + i] = fa ? acause[g] : bcause[g];
    ckind[c0 + i] = fa ? akind[g] : bkind[g];
    cval[c0 + i] = fa ? aval[g] : bval[g];
  }
}

// Walks document d's id-sorted capacity slot: a node is kept when its id
// differs from its predecessor's; a repeated id must repeat the body (cause,
// kind, value token) or the document gets CW_STATUS_DUP.  pass 0 counts the
// kept nodes (mcount[d]); pass 1 writes them at moff[d] (ids in order, causes,
// kinds and source indices).
template <int NT>
__global__ __launch_bounds__(NT) void k_merge_dedup(
    const uint64_t *__restrict__ skey, const uint32_t *__restrict__ sval,
    const uint64_t *__restrict__ ccause, const uint8_t *__restrict__ ckind,
    const uint64_t *__restrict__ cval, const uint32_t *__restrict__ coff, int pass,
    uint32_t *__restrict__ mcount, const uint32_t *__restrict__ moff,
    uint64_t *__restrict__ mid, uint64_t *__restrict__ mcause, uint8_t *__restrict__ mkind,
    uint32_t *__restrict__ msrc, uint32_t *__restrict__ mstatus) {
  __shared__ uint32_t wtot[NT / 64];
  const uint32_t d = blockIdx.x, c0 = coff[d], n = coff[d + 1] - c0;
  uint32_t run = 0;
  bool conflict = false;
  for (uint32_t i0 = 0; i0 < n; i0 += NT) {
    const uint32_t i = i0 + threadIdx.x;
    bool keep = false;
    uint64_t k = 0;
    uint32_t v = 0;
    if (i < n) {
      k = skey[c0 + i];
      v = sval[c0 + i];
      keep = i == 0 || skey[c0 + i - 1] != k;
      if (!keep && pass == 0) {
        const uint32_t u = sval[c0 + i - 1];
        conflict |= ccause[c0 + u] != ccause[c0 + v] || ckind[c0 + u] != ckind[c0 + v] ||
                    cval[c0 + u] != cval[c0 + v];
      }
    }
    uint32_t tot;
    const uint32_t pos = run + block_exscan<NT>(keep ? 1u : 0u, wtot, &tot);
    if (pass == 1 && keep) {
      const uint32_t o = moff[d] + pos;
      mid[o] = k;
      mcause[o] = ccause[c0 + v];
      mkind[o] = ckind[c0 + v];
      msrc[o] = v;
    }
    run += tot;
  }
  if (pass == 0) {
    if (__syncthreads_or(conflict) && threadIdx.x == 0) mstatus[d] = CW_STATUS_DUP;
    else if (threadIdx.x == 0) mstatus[d] = 0;
    if (threadIdx.x == 0) mcount[d] = run;
  }
}

// merged weave positions -> doc-local merged index is what the list pipeline
// returns already; status of the union (conflicts) joins the weave's.
__global__ void k_or_status(const uint32_t *__restrict__ a, uint32_t *__restrict__ b, uint32_t D) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < D) b[d] |= a[d];
}

// Weft (s/weft, shared.cljc:268-293): keep the root and, per named site, the
// site's yarn up to its cut id: (take-while #(not= id (first %)) yarn) then
// (conj (new-node [id (get ::nodes id)])).  When the cut id is a node that is
// the yarn's ids <= cut (yarns are id-sorted).  When it is not, take-while
// keeps the WHOLE yarn and (new-node [id nil]) = (into [id] nil) = [id] is a
// one-element node: cause nil, (peek node) = the id itself.  Such a node goes
// after the kept nodes (id = cut, cause nil, kind normal, ksrc = UINT32_MAX)
// and the document gets CW_STATUS_WEFT.  Count pass, then write pass at koff.
template <int NT>
__global__ __launch_bounds__(NT) void k_weft_select(
    const uint64_t *__restrict__ id_key, const uint64_t *__restrict__ cause_key,
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ doc_off,
    const uint64_t *__restrict__ cut, uint32_t site_shift, uint32_t site_bits, int pass,
    uint32_t *__restrict__ kcount, const uint32_t *__restrict__ koff, uint64_t *__restrict__ kid,
    uint64_t *__restrict__ kcause, uint8_t *__restrict__ kkind, uint32_t *__restrict__ ksrc,
    uint32_t *__restrict__ kstatus) {
  __shared__ uint32_t wtot[NT / 64];
  __shared__ uint32_t found[1024 / 32];
  const uint32_t d = blockIdx.x, base = doc_off[d], n = doc_off[d + 1] - base;
  const uint32_t S = 1u << site_bits, smask = S - 1;
  const uint64_t *dc = cut + ((size_t)d << site_bits);
  for (uint32_t i = threadIdx.x; i < 32; i += NT) found[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += NT) {  // which cut ids are nodes
    const uint64_t k = id_key[base + i];
    const uint32_t site = (uint32_t)(k >> site_shift) & smask;
    if (dc[site] != 0 && k == dc[site]) atomicOr(&found[site >> 5], 1u << (site & 31));
  }
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += NT) {
    const uint32_t i = i0 + threadIdx.x;
    bool keep = false;
    uint64_t k = 0;
    if (i < n) {
      k = id_key[base + i];
      const uint32_t site = (uint32_t)(k >> site_shift) & smask;
      const uint64_t c = dc[site];
      const bool hit = (found[site >> 5] >> (site & 31)) & 1u;
      keep = (kind[base + i] & KIND_ROOT) || (c != 0 && (!hit || k <= c));
    }
    uint32_t tot;
    const uint32_t pos = run + block_exscan<NT>(keep ? 1u : 0u, wtot, &tot);
    if (pass == 1 && keep) {
      const uint32_t o = koff[d] + pos;
      kid[o] = k;
      kcause[o] = cause_key[base + i];
      kkind[o] = kind[base + i];
      ksrc[o] = i;
    }
    run += tot;
  }
  // the [id] nodes of cut ids that are not nodes, in site order
  uint32_t miss = 0;
  for (uint32_t s0 = 0; s0 < S; s0 += NT) {
    const uint32_t s = s0 + threadIdx.x;
    const bool m = s < S && dc[s] != 0 && !((found[s >> 5] >> (s & 31)) & 1u);
    uint32_t tot;
    const uint32_t pos = run + miss + block_exscan<NT>(m ? 1u : 0u, wtot, &tot);
    if (pass == 1 && m) {
      const uint32_t o = koff[d] + pos;
      kid[o] = dc[s];
      kcause[o] = CW_NIL;
      kkind[o] = 0;
      ksrc[o] = 0xFFFFFFFFu;
    }
    miss += tot;
  }
  if (pass == 0 && threadIdx.x == 0) {
    kcount[d] = run + miss;
    kstatus[d] = miss ? (uint32_t)CW_STATUS_WEFT : 0u;
  }
}

// --- tiny documents: one block weaves every document that starts in its chunk ----
// The same exact weave (F5 preorder) as the list pipeline, for the
// key weaves of maps (config 4: ~3 nodes per key) where the per-document
// kernels of the pipeline would dominate.  A block takes the documents (of <=
// SMALL_MAX nodes) that start in its 192-node chunk -- at most 255 nodes, one
// per thread -- and works in LDS: ranks by counting inside the document, cause
// ranks by binary search, effective parents, subtree sizes and preorder
// positions by walking each node's ancestor chain (no per-step barriers).
constexpr uint32_t SMALL_MAX = 64, SMALL_CHUNK = 192, SMALL_SLOTS = 256;

__global__ __launch_bounds__(SMALL_SLOTS) void k_small_weave(
    const uint64_t *__restrict__ doc_off, uint32_t D, const uint64_t *__restrict__ id_key,
    const uint64_t *__restrict__ cause_key, const uint8_t *__restrict__ kind,
    uint32_t *__restrict__ weave_perm, uint32_t *__restrict__ status) {
  __shared__ uint64_t sid[SMALL_SLOTS];
  __shared__ uint32_t ds[SMALL_CHUNK + 2], at[SMALL_SLOTS], par[SMALL_SLOTS], eff[SMALL_SLOTS];
  __shared__ uint32_t size[SMALL_SLOTS], before[SMALL_SLOTS], dst[SMALL_CHUNK + 1];
  __shared__ uint8_t spk[SMALL_SLOTS];
  __shared__ uint32_t s_df, s_nd;
  __shared__ uint64_t s_base;
  const uint32_t tid = threadIdx.x;
  const uint64_t NL = doc_off[D], c0 = (uint64_t)blockIdx.x * SMALL_CHUNK;
  const uint64_t c1 = min(c0 + SMALL_CHUNK, NL);
  if (tid < 2) {  // documents [df, dl) start in [c0, c1)
    const uint64_t x = tid == 0 ? c0 : c1;
    uint32_t lo = 0, hi = D + 1;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (doc_off[m] < x) lo = m + 1; else hi = m;
    }
    if (tid == 0) s_df = lo; else s_nd = lo;
  }
  __syncthreads();
  const uint32_t df = s_df, nd = (c1 > c0 ? s_nd : s_df) - df;
  if (nd == 0) return;  // uniform
  if (tid <= nd) ds[tid] = (uint32_t)(doc_off[df + tid] - doc_off[df]);
  if (tid < nd) dst[tid] = 0;
  if (tid == 0) s_base = doc_off[df];
  __syncthreads();
  const uint64_t base = s_base;
  const uint32_t span = ds[nd];
  const bool v = tid < span;
  uint32_t di = 0;  // my document (in the chunk)
  if (v) {
    uint32_t lo = 0, hi = nd;
    while (hi - lo > 1) {
      const uint32_t m = (lo + hi) >> 1;
      if (ds[m] <= tid) lo = m; else hi = m;
    }
    di = lo;
  }
  const uint32_t g0 = v ? ds[di] : 0u, m = v ? ds[di + 1] - g0 : 0u, li = tid - g0;
  const uint64_t id = v ? id_key[base + tid] : 0, ca = v ? cause_key[base + tid] : 0;
  const uint32_t kd = v ? kind[base + tid] : 0u;
  if (v) sid[tid] = id;
  __syncthreads();
  // 1. rank in the document (count of smaller ids); duplicates flag the document
  uint32_t r = 0, st = 0;
  for (uint32_t j = 0; j < m; j++) {
    const uint64_t o = sid[g0 + j];
    r += o < id ? 1u : 0u;
    if (o == id && j != li) st |= CW_STATUS_DUP;
  }
  if (v && m > SMALL_MAX) st |= CW_STATUS_INTERNAL;
  if (st) atomicOr(&dst[di], st);
  __syncthreads();
  const bool dirty = v && (dst[di] & CW_STATUS_DUP);
  if (dirty) r = li;  // any permutation (the document is flagged)
  if (v) at[g0 + r] = tid;
  __syncthreads();
  // 2. domain checks; cause rank by binary search over the ranked ids
  uint32_t p = 0;
  if (v) {
    if (r == 0) {
      if (!(kd & KIND_ROOT)) st |= CW_STATUS_ROOT;
    } else {
      if (kd & KIND_ROOT) st |= CW_STATUS_ROOT;
      uint32_t lo = 0, hi = m;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sid[at[g0 + mid]] < ca) lo = mid + 1; else hi = mid;
      }
      if (lo >= m || sid[at[g0 + lo]] != ca) st |= CW_STATUS_ORPHAN;
      else if (lo >= r) st |= CW_STATUS_NON_LAMPORT;
      else p = lo;
    }
    par[g0 + r] = p;
    spk[g0 + r] = (uint8_t)(is_special((uint8_t)kd) ? 1 : 0);
    size[g0 + r] = 1;
  }
  if (st) atomicOr(&dst[di], st);
  __syncthreads();
  // 3. effective parent: a non-special climbs through special causes
  const bool sp = v && is_special((uint8_t)kd);
  uint32_t e = p;
  if (v && r > 0 && !sp)
    for (uint32_t it = 0; e != 0 && spk[g0 + e] && it < m; it++) e = par[g0 + e];
  if (v) eff[g0 + r] = e;
  __syncthreads();
  // 4. subtree sizes: every node counts itself into each ancestor
  if (v && r > 0) {
    uint32_t a = e;
    for (uint32_t it = 0; it < m; it++) {
      atomicAdd(&size[g0 + a], 1u);
      if (a == 0) break;
      a = eff[g0 + a];
    }
  }
  __syncthreads();
  // 5. siblings before me: specials first, each class by descending id
  if (v && r > 0) {
    uint32_t bf = 0;
    for (uint32_t q = 1; q < m; q++) {
      if (q == r || eff[g0 + q] != e) continue;
      const bool sq = spk[g0 + q];
      if ((sq && !sp) || (sq == sp && q > r)) bf += size[g0 + q];
    }
    before[g0 + r] = bf;
  }
  __syncthreads();
  // 6. preorder position = sum over the ancestor chain of (1 + siblings before)
  if (v) {
    uint32_t pos = 0, x = r;
    for (uint32_t it = 0; x != 0 && it < m; it++) {
      pos += 1 + before[g0 + x];
      x = eff[g0 + x];
    }
    if (pos < m) weave_perm[base + g0 + pos] = li;
  }
  if (tid < nd) status[df + tid] = dst[tid];
}

// --- device exclusive scan of u32 counts (map key-weave numbering) ---------------
// chunk sums (1024 per block) -> one block scans the sums -> chunks add their base
__global__ __launch_bounds__(1024) void k_scan_chunks(const uint32_t *__restrict__ in, uint32_t n,
                                                      uint32_t *__restrict__ out,
                                                      uint32_t *__restrict__ sums) {
  __shared__ uint32_t wtot[16];
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t v = i < n ? in[i] : 0u;
  uint32_t tot;
  const uint32_t ex = block_exscan<1024>(v, wtot, &tot);
  if (i < n) out[i] = ex;
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint32_t *__restrict__ sums, uint32_t nb,
                                                    uint32_t *__restrict__ total) {
  __shared__ uint32_t wtot[16];
  uint32_t run = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_exscan<1024>(v, wtot, &tot);
    if (i < nb) sums[i] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) *total = run;
}

__global__ __launch_bounds__(1024) void k_scan_add(uint32_t *__restrict__ out, uint32_t n,
                                                   const uint32_t *__restrict__ sums) {
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  if (i < n) out[i] += sums[blockIdx.x];
}

// Key weave s is list document [seg_start[s] + s, seg_start[s+1] + s + 1): its
// offset, and the longest key weave (atomicMax into *maxlen).
__global__ __launch_bounds__(256) void k_seg_off(const uint32_t *__restrict__ seg_start, uint32_t S,
                                                 uint32_t N, uint64_t *__restrict__ seg_off,
                                                 uint32_t *__restrict__ maxlen) {
  // grid-stride over a fixed grid, one atomic per block: atomics on one word
  // serialise (a per-segment atomic took 7.5 ms for config 4's 4.2e7 key weaves)
  __shared__ uint32_t wmax[4];
  uint32_t len = 0;
  for (uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x; sg <= S; sg += gridDim.x * blockDim.x) {
    const uint64_t o = sg < S ? (uint64_t)seg_start[sg] + sg : (uint64_t)N + S;
    seg_off[sg] = o;
    if (sg < S) {
      const uint32_t e = sg + 1 < S ? seg_start[sg + 1] + sg + 1 : N + S;
      len = max(len, (uint32_t)(e - o));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) len = max(len, (uint32_t)__shfl_xor(len, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (m) atomicMax(maxlen, m);
  }
}

// ============================================================================
// Host side
// ============================================================================

namespace {

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
};

struct KStat {
  uint64_t launches = 0;
  double ms = 0, bytes = 0;
};

struct PendingEvt {
  std::string name;
  hipEvent_t a, b;
  double bytes;
};

}  // namespace

struct cw_ctx {
  int device = 0;
  uint32_t lds_max = 160 * 1024;  // LDS a workgroup may use on this device (queried at create)
  size_t hbm_total = 0;             // device memory (queried at create)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  bool async = false;
  bool prof = false;
  std::string prof_only;           // cw_ctx_set_profile_only: time this kernel stat only
  std::string err;
  std::map<std::string, DevBuf> bufs;
  void *pinned = nullptr;
  size_t pinned_bytes = 0;
  std::map<std::string, KStat> stats;
  std::vector<PendingEvt> pending;
  std::vector<hipEvent_t> evt_pool;
  // cached host tables (reused when the document layout repeats)
  std::vector<uint64_t> last_off;
  struct Tables {
    std::vector<uint32_t> doc_off, tile_start, tile_doc, tile_first, doc_log2k, doc_W, walk_first,
        wblk_doc, wblk_w0, bkt_off, doc_log2cap, doc_Wcap, eblk_doc, eblk_x0, woff_base,
        pack_doc0;
    std::vector<uint64_t> slot_first;
    uint32_t T = 0, Wtot = 0, Bw = 0, Be = 0, nmax = 0, Btot = 0, Wmax = 0, Wofftot = 0;
    uint32_t pack_dmax = 0;  // most documents in one sort pack (k_pack_sort)
    uint64_t slots = 0;
    bool tour = false;       // every document goes through k_tour (LDS walk + rank + emit)
    uint32_t tour_log2k = 3;  // its splitter blocks
  } tab;
  bool tab_on_device = false;
  bool last_giant = false;
  // launch geometry (fixed at cw_ctx_create)
  uint32_t tb = 1024, walk_threads = 1024, walk_span = 1024, giant_log2cap = 5, glocal = 1, glocal_min = 1u << 20, min_log2k = 5,
           max_digit = MAX_DIGIT, min_log2cap = 4;
  // rank-directory front end (CW_FRONT, CW_FRONT_SLOT bytes per document)
  uint32_t front = 1, front_slot_groups = 4096, front_min_avg = 1024;
  uint32_t *pin_small = nullptr;  // pinned 16-byte readback
  uint32_t tree_prof = 0;          // CW_TREE_PROF: diagnostic phase stamps
  uint32_t tree_l = 2048;          // CW_TREE_L: k_tree_l (tables in LDS) when the largest document fits: its tile (2048 or 1024; 0 = k_tree)
  uint32_t gdir = 32;              // CW_GDIR: MiB of global rank directory a giant document may use
  uint32_t gjoin = 1;              // CW_GJOIN: the giant path joins through a directory of its sorted ids
  uint32_t id_payload = 1;         // CW_ID_PAYLOAD: the id sort carries cause | kind to rank order (round 6)
  uint32_t map_small = 1;          // CW_MAP_SMALL: one wave per key weave of <= 64 nodes
  uint32_t pack_sort = 1;          // CW_PACK_SORT: in-LDS sort of packs of small documents
  uint32_t giant_min = 1u << 16;   // CW_GIANT_MIN: a one-document batch this large uses the giant tree
  uint32_t tour = 1;               // CW_TOUR: fused LDS tour for documents of < 2^16 nodes
  uint32_t giant_docs_max = 32;    // CW_GIANT_DOCS: batches of up to this many large documents
                                   // go through the giant path document by document
  uint32_t front_fused = 1;        // CW_FRONT_FUSED: one-kernel front end (k_front)
  uint32_t tour_log2k = 3;         // CW_TOUR_LOG2K: nodes per splitter block on that path
  uint32_t giant_log2k = 4;        // CW_GIANT_LOG2K: least splitter block of a giant document
  uint32_t fused = 1;              // CW_FUSED: front end + tree + tour in one kernel (k_weave_doc)
  bool x_hint = true;              // the last list weave may have flagged documents (exact.hip)
  uint32_t onesweep = 4;           // CW_ONESWEEP: one-array sorts by the one-sweep passes
                                   // (tiles of 4,096 keys x 512 threads, 8,192 x 1,024,
                                   // 8,192 x 512: 1-3 in one look-back chain, 4-6 in
                                   // OS_RANGES chains; 0: histogram-scan-scatter)
  uint32_t n_cu = 256;             // compute units of the device (histogram grid)
  uint32_t os_exp = 0;             // CW_OS_EXP: onesweep timing experiments (wrong results)
  uint32_t onesweep_min = 1u << 16;  // CW_ONESWEEP_MIN: ... for arrays of at least this many keys
  const void *os_lb = nullptr;     // onesweep.hip's look-back words: buffer, size, last epoch
  size_t os_lb_words = 0;
  uint32_t os_epoch = 0;
  const uint32_t *last_dyn = nullptr;  // the last HBM walk's continued-sublist counters
  uint32_t last_dyn_n = 0;             // ... (one per document of that walk)
  uint32_t x_iters = 0;            // synthetic-list weaves of the last exact path (exact.hip)
  uint32_t xfold = 0;              // CW_XFOLD: documents with an early node take the serial fold
  uint32_t x_round_cap = 48;       // CW_X_ROUND_CAP: anchor rounds before a small still-moving
                                   // document takes the serial fold (exact.hip X_ROUND_CAP)
  uint32_t *pin_status = nullptr;  // pinned: a giant document's status, copied after the front end
  hipEvent_t ev_status = nullptr;  // ... and recorded there (exact.hip waits on it, not the stream)
  bool x_pending = false;          // pin_status / ev_status hold this call's giant document
  struct XFront {                  // a flagged giant list's front end, handed to the exact path
    const uint64_t *skey = nullptr;  // sorted ids
    const uint32_t *sval = nullptr;  // input index by rank
    const uint4 *dir = nullptr;      // rank directory of the sorted ids (E entries)
    uint64_t E = 0;
    const uint64_t *ckk = nullptr;   // cause | kind << 56 by input index, or nullptr
    uint32_t n = 0;
    bool ok = false;
  } xfront;
  uint32_t map_fused = 1;          // CW_MAP_FUSED: one-kernel map weave of small collections
  struct MapPacks {                // k_map_pack's pack table, cached by collection layout
    std::vector<uint64_t> off;
    std::vector<uint32_t> doc0;
    uint32_t dbits = 0, pk = 0, dmax = 1;  // (dmax: most collections in one pack)
    uint32_t epoch = 0, lb_packs = 0;      // look-back words' epoch (mappack.hip)
    const void *lb = nullptr;
    uint64_t maxcoll = 0;          // the largest collection of the cached layout
    bool ok = false;
    bool same = false;             // this call's coll_offsets equal off (set by cw_weave_maps)
    bool verify = false;           // ... taken on trust: compared while the kernel runs
  } mpack;
};

namespace {

int fail(cw_ctx *c, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return -1;
}

#define HIPCHK(c, x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail((c), "%s: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                \
  } while (0)

void *scratch(cw_ctx *c, const char *name, size_t bytes) {
  DevBuf &b = c->bufs[name];
  if (bytes == 0) bytes = 16;
  if (b.bytes < bytes) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    // headroom for slightly larger batches, at most 256 MiB (a 2e9-node list
    // would otherwise hold 12% of its scratch idle)
    size_t want = bytes + std::min(bytes / 8, (size_t)256 << 20);
    if (hipMalloc(&b.p, want) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    b.bytes = want;
  }
  return b.p;
}

template <typename T>
T *scratch_t(cw_ctx *c, const char *name, size_t count) {
  return reinterpret_cast<T *>(scratch(c, name, count * sizeof(T)));
}

hipEvent_t get_event(cw_ctx *c) {
  if (!c->evt_pool.empty()) {
    hipEvent_t e = c->evt_pool.back();
    c->evt_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Launch helper: optional per-kernel event timing on the launch stream.
struct Launch {
  cw_ctx *c;
  const char *name;
  double bytes;
  hipStream_t s;
  hipEvent_t a = nullptr;
  Launch(cw_ctx *c_, const char *n, double by, hipStream_t st = nullptr)
      : c(c_), name(n), bytes(by), s(st ? st : c_->stream) {
    if (c->prof && (c->prof_only.empty() || c->prof_only == n)) {
      a = get_event(c);
      (void)hipEventRecord(a, s);
    }
  }
  ~Launch() {
    if (c->prof && a) {
      hipEvent_t b = get_event(c);
      (void)hipEventRecord(b, s);
      c->pending.push_back({name, a, b, bytes});
    }
  }
};

// HSA dispatch packets carry the grid size in work-items as 32 bits.
bool grid_ok(uint64_t blocks, uint64_t threads) { return blocks * threads < (1ull << 32); }

int check_launch(cw_ctx *c, const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(c, "launch %s: %s", what, hipGetErrorString(e));
  return 0;
}

// Event pairs are read back when the stats are asked for (or a call is
// synchronous, or many are pending): an asynchronous call under profiling
// does not wait for its kernels.
int collect_prof(cw_ctx *c, bool now = false) {
  if (c->pending.empty()) return 0;
  if (!now && c->async && c->pending.size() < 8192) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (auto &p : c->pending) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    KStat &s = c->stats[p.name];
    s.launches++;
    s.ms += ms;
    s.bytes += p.bytes;
    c->evt_pool.push_back(p.a);
    c->evt_pool.push_back(p.b);
  }
  c->pending.clear();
  return 0;
}

uint32_t ceil_log2(uint64_t x) {
  uint32_t r = 0;
  while ((1ull << r) < x) r++;
  return r;
}

// Host tables: tiles (sort/pass grids), splitter blocks and walker blocks.
void build_tables(cw_ctx *c, uint64_t D, const uint64_t *off, bool giant) {
  auto &t = c->tab;
  t.doc_off.resize(D + 1);
  t.tile_start.clear();
  t.tile_doc.clear();
  t.tile_first.resize(D + 1);
  t.doc_log2k.resize(D);
  t.doc_W.resize(D);
  t.walk_first.resize(D + 1);
  t.wblk_doc.clear();
  t.wblk_w0.clear();
  t.eblk_doc.clear();
  t.eblk_x0.clear();
  t.woff_base.clear();
  uint32_t wofft = 0;
  t.doc_log2cap.resize(D);
  t.doc_Wcap.resize(D);
  t.slot_first.resize(D + 1);
  uint64_t slots = 0;
  t.bkt_off.resize(D + 1);
  uint32_t wtot = 0, stot = 0;
  t.nmax = 0;
  t.Wmax = 0;
  uint64_t nmax = 0;
  for (uint64_t d = 0; d < D; d++) nmax = std::max<uint64_t>(nmax, off[d + 1] - off[d]);
  // the fused LDS tour: documents of < 2^16 nodes whose list fits the LDS
  // (the splitter blocks grow until the tables fit next to the successors)
  t.tour = false;
  t.tour_log2k = c->tour_log2k;
  if (c->tour && !giant && nmax <= TOUR_END) {
    auto lds = [&](uint32_t l2k) { return tour_lds_bytes((uint32_t)nmax, l2k); };
    while (t.tour_log2k < 8 && (lds(t.tour_log2k) > std::min(TOUR_LDS_MAX, c->lds_max - 1024) ||
                                ((nmax + (1u << t.tour_log2k) - 1) >> t.tour_log2k) > 8 * 1024))
      t.tour_log2k++;
    t.tour = lds(t.tour_log2k) <= std::min(TOUR_LDS_MAX, c->lds_max - 1024);
  }
  for (uint64_t d = 0; d < D; d++) {
    const uint32_t b = (uint32_t)off[d], n = (uint32_t)(off[d + 1] - off[d]);
    t.doc_off[d] = b;
    t.nmax = std::max(t.nmax, n);
    t.tile_first[d] = (uint32_t)t.tile_start.size();
    const uint32_t ntile = (n + TILE - 1) / TILE;
    for (uint32_t s = 0; s < n; s += TILE) {
      t.tile_start.push_back(b + s);
      t.tile_doc.push_back((uint32_t)d);
      // rank-window table of this tile: ntile + 1 entries (front end only,
      // which takes documents of <= 64 tiles)
      t.woff_base.push_back(wofft);
      if (ntile <= 64) wofft += ntile + 1;
    }
    // splitter block size K = 2^log2k and slot capacity 2^log2cap: static
    // sublists 2*ceil(n/K) plus continued ones (<= ceil(n/cap)) fit the LDS rank
    uint32_t log2k = t.tour ? t.tour_log2k : c->min_log2k, log2cap = c->min_log2cap;
    // one giant document: every slot overflow takes a sublist id from one
    // counter; 32-entry slots overflow ~8x less often (walk 2.8 -> 1.5 ms at
    // 6.7e7 nodes) for 4 more bytes a node (16-node blocks), so whenever the
    // list fits the device with them (round 5: the rule was n < 2^30, and the
    // 2e9-node walk ran 1.8x slower a node than at 5.4e8 -- the same loads,
    // L2 misses and HBM bytes a node, twice the continuation sublists;
    // DESIGN 5e).  (CW_GIANT_LOG2CAP: the tests shrink it to send walks
    // through many continuation sublists)
    // (the knob sets the giant slot size itself, also below min_log2cap)
    // The test is against the device memory free at this call plus the
    // scratch this context already holds (it is reused), not the device's
    // total: a shared device or large caller buffers keep 16-entry slots.
    bool cap32 = giant && n < (1u << 30);
    if (giant && !cap32) {
      size_t fr = 0, tot = 0;
      uint64_t held = 0;
      for (auto &kv : c->bufs) held += kv.second.bytes;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess) cap32 = (uint64_t)n * GIANT_CAP32_BYTES <= fr + held;
    }
    if (cap32) log2cap = c->giant_log2cap;
    // and 16-node splitter blocks: half the sublists to rank for a slightly
    // longer walk (15.68 -> 15.17 ms a step at 6.7e7 nodes; 32 nodes: 16.8),
    // once there are walkers enough to fill the chip (config 1's 10^5 nodes:
    // walk 0.044 -> 0.085 ms with 16)
    if (giant && n >= (1u << 22)) log2k = std::max(log2k, c->giant_log2k);
    auto subl = [&]() {
      return (uint64_t)((n + (1u << log2k) - 1) >> log2k) +
             (uint64_t)((n + (1u << log2cap) - 1) >> log2cap) + 1;
    };
    // (a giant document ranks its sublists in two levels: no LDS limit here)
    while (!giant && subl() > MAX_SUBLISTS) {
      if (log2k < log2cap) log2k++;
      else log2cap++;
    }
    const uint32_t W = n ? ((n + (1u << log2k) - 1) >> log2k) : 0;  // one walker per splitter
    const uint32_t Wcap = n ? (uint32_t)subl() : 0;
    t.doc_log2k[d] = log2k;
    t.doc_log2cap[d] = log2cap;
    t.doc_W[d] = W;
    t.doc_Wcap[d] = Wcap;
    t.Wmax = std::max(t.Wmax, Wcap);
    t.walk_first[d] = wtot;
    t.slot_first[d] = slots;
    slots += (uint64_t)Wcap << log2cap;
    for (uint32_t w0 = 0; w0 < W; w0 += c->walk_span) {
      t.wblk_doc.push_back((uint32_t)d);
      t.wblk_w0.push_back(w0);
    }
    for (uint32_t x0 = 0; x0 < Wcap; x0 += 256) {
      t.eblk_doc.push_back((uint32_t)d);
      t.eblk_x0.push_back(x0);
    }
    wtot += Wcap;
    // join bucket index: <= max(n/4, 1) buckets + 1 end entry (k_index)
    t.bkt_off[d] = stot;
    stot += n ? std::max(n >> 2, 1u) + 2 : 0;
  }
  t.doc_off[D] = (uint32_t)off[D];
  t.tile_first[D] = (uint32_t)t.tile_start.size();
  t.walk_first[D] = wtot;
  t.slot_first[D] = slots;
  t.slots = slots;
  t.Be = (uint32_t)t.eblk_doc.size();
  t.Wofftot = wofft;
  // sort packs: runs of whole consecutive documents of <= TILE nodes in all
  // (only used when every document fits one tile)
  t.pack_doc0.clear();
  t.pack_dmax = 0;
  if (t.nmax <= TILE) {
    uint64_t d = 0;
    while (d < D) {
      const uint64_t d0 = d;
      while (d < D && off[d + 1] - off[d0] <= TILE) d++;
      if (d == d0) d++;  // (cannot happen: every document <= TILE)
      t.pack_doc0.push_back((uint32_t)d0);
      t.pack_dmax = std::max(t.pack_dmax, (uint32_t)(d - d0));
    }
    t.pack_doc0.push_back((uint32_t)D);
  }
  t.bkt_off[D] = stot;
  t.Btot = stot;
  t.T = (uint32_t)t.tile_doc.size();
  t.tile_start.push_back((uint32_t)off[D]);
  t.Wtot = wtot;
  t.Bw = (uint32_t)t.wblk_doc.size();
}

int upload_tables(cw_ctx *c) {
  auto &t = c->tab;
  std::vector<std::pair<const char *, const std::vector<uint32_t> *>> items = {
      {"t_doc_off", &t.doc_off},   {"t_tile_start", &t.tile_start}, {"t_tile_doc", &t.tile_doc},
      {"t_tile_first", &t.tile_first}, {"t_doc_log2k", &t.doc_log2k}, {"t_doc_W", &t.doc_W},
      {"t_walk_first", &t.walk_first}, {"t_wblk_doc", &t.wblk_doc},  {"t_wblk_w0", &t.wblk_w0},
      {"t_bkt_off", &t.bkt_off}, {"t_doc_log2cap", &t.doc_log2cap},
      {"t_doc_Wcap", &t.doc_Wcap}, {"t_eblk_doc", &t.eblk_doc}, {"t_eblk_x0", &t.eblk_x0},
      {"t_woff_base", &t.woff_base}, {"t_pack_doc0", &t.pack_doc0}};
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the pinned staging may still be read
  size_t total = (t.slot_first.size() + 64) * 8;
  for (auto &it : items) total += (it.second->size() + 64) * 4;
  if (c->pinned_bytes < total) {
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    HIPCHK(c, hipHostMalloc(&c->pinned, total, hipHostMallocDefault));
    c->pinned_bytes = total;
  }
  char *p = (char *)c->pinned;
  for (auto &it : items) {
    size_t bytes = it.second->size() * 4;
    void *dst = scratch(c, it.first, bytes);
    if (!dst) return fail(c, "out of device memory (%s)", it.first);
    if (bytes) {
      memcpy(p, it.second->data(), bytes);
      HIPCHK(c, hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, c->stream));
    }
    p += (it.second->size() + 64) * 4;
  }
  {
    size_t bytes = t.slot_first.size() * 8;
    void *dst = scratch(c, "t_slot_first", bytes);
    if (!dst) return fail(c, "out of device memory (t_slot_first)");
    memcpy(p, t.slot_first.data(), bytes);
    HIPCHK(c, hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, c->stream));
  }
  return 0;
}

uint32_t *dev_tab(cw_ctx *c, const char *name) { return (uint32_t *)c->bufs[name].p; }

// One segmented radix sort over key bits [shift0, shift0+bits): LSD passes of
// <= MAX_DIGIT bits (at least one pass).  Pass 0 reads (kin, vin) -- vin ==
// nullptr means identity values -- and the passes ping-pong between (kA,vA)
// and (kB,vB).
#include "onesweep.hip"

// The cause / kind payload of an id sort (OsPayload): its source, two u32
// buffers for lo in turn, one for the last pass's hi, and where the last pass
// left lo (lo_out == nullptr: the sort did not carry it -- not the one-sweep
// path, or more than OS_PL_MAX_BITS key bits).  An id past the key bits sets
// CW_STATUS_INTERNAL in *status (the keys are cut to the key bits: nothing
// downstream reads past the directory).
struct OsPayloadBufs {
  const uint64_t *cause;
  const uint8_t *kind;
  uint32_t *lo[2], *hi;
  uint32_t *lo_out;
  uint32_t *status;
};

// One array (one document, or rt's one list): the one-sweep passes
// (onesweep.hip) -- one histogram launch for every pass, one scan launch, one
// launch a pass.  Same contract as radix_sort.
template <typename K>
int onesweep_sort(cw_ctx *c, const char *tag, const K *kin, const uint32_t *vin, K *kA, uint32_t *vA,
                  K *kB, uint32_t *vB, uint32_t bits, uint32_t shift0, uint32_t N, K **kout,
                  uint32_t **vout, uint32_t *inv, uint32_t *vfinal, OsPayloadBufs *plb = nullptr) {
  const uint32_t geom = c->onesweep;
  // 1-3 one chain: 512 x 8, 1024 x 8, 512 x 16 keys a tile; 4-6 the same in
  // OS_RANGES chains (4 = 1024 x 8, 5 = 512 x 8, 6 = 512 x 16)
  const uint32_t shape = geom == 4 ? 2 : geom == 5 ? 1 : geom == 6 ? 3 : geom;
  const uint32_t TS = shape == 1 ? 4096 : 8192;
  const bool ranged = geom > 3;
  OsDigits dg{};
  dg.passes = (bits + OS_MAX_BITS - 1) / OS_MAX_BITS;
  if (dg.passes > OS_MAX_PASSES) return fail(c, "onesweep: %u key bits", bits);
  for (uint32_t p = 0, sh = shift0; p < dg.passes; p++) {
    // the wider digits last, as radix_sort
    dg.bits[p] = bits / dg.passes + (p >= dg.passes - bits % dg.passes ? 1u : 0u);
    dg.shift[p] = sh;
    sh += dg.bits[p];
  }
  const uint32_t T = (N + TS - 1) / TS;
  const uint32_t nr = ranged ? OS_RANGES : 1u;
  const uint32_t Tr = (T + nr - 1) / nr;  // tiles a range
  const uint32_t rlen = ranged ? Tr * TS : 0xFFFFFFFFu;
  const size_t hist_words = (size_t)OS_MAX_PASSES * OS_RANGES * OS_MAX_BINS;
  uint32_t *hist = scratch_t<uint32_t>(c, "os_hist", 2 * hist_words + OS_MAX_PASSES * OS_RANGES);
  const size_t lb_words = (size_t)Tr * nr * OS_MAX_BINS;
  unsigned long long *lb = scratch_t<unsigned long long>(c, "os_lb", lb_words);
  if (!hist || !lb) return fail(c, "out of device memory (onesweep)");
  uint32_t *base = hist + hist_words, *ticket = base + hist_words;
  // look-back words: cleared when the buffer is new or the 16-bit epoch wraps
  if (lb != c->os_lb || lb_words > c->os_lb_words || c->os_epoch + dg.passes > 0xFFFFu) {
    HIPCHK(c, hipMemsetAsync(lb, 0, c->bufs["os_lb"].bytes, c->stream));
    c->os_lb = lb;
    c->os_lb_words = c->bufs["os_lb"].bytes / 8;
    c->os_epoch = 0;
  }
  HIPCHK(c, hipMemsetAsync(hist, 0, hist_words * 4, c->stream));
  if (ranged) HIPCHK(c, hipMemsetAsync(ticket, 0, OS_MAX_PASSES * OS_RANGES * 4, c->stream));
  char nm[48], nm_scan[48], nm_hist[48];
  snprintf(nm, sizeof nm, "%s_scatter", tag);
  snprintf(nm_scan, sizeof nm_scan, "%s_scan", tag);
  snprintf(nm_hist, sizeof nm_hist, "%s_hist", tag);
  // the digit counts of a pass's input (every pass at once when there is one
  // range: the counts do not depend on the order), then the bucket bases
  auto count = [&](const K *keys, uint32_t p0, uint32_t np) -> int {
    OsDigits d = dg;
    d.passes = np;
    for (uint32_t q = 0; q < np; q++) {
      d.shift[q] = dg.shift[p0 + q];
      d.bits[q] = dg.bits[p0 + q];
    }
    uint32_t *hp = hist + (size_t)p0 * OS_RANGES * OS_MAX_BINS;
    {
      Launch L(c, nm_hist, (double)N * sizeof(K));
      const uint32_t span = 256 * OS_HIST_ITEMS;
      const uint32_t G = std::max(nr, std::min(c->n_cu * 4, (N + span - 1) / span) / nr * nr);
      hipLaunchKernelGGL(k_os_hist<K>, dim3(G), dim3(256), (size_t)4 * np * OS_MAX_BINS * 4, c->stream,
                         keys, N, d, rlen, nr, hp);
    }
    if (check_launch(c, nm_hist)) return -1;
    {
      Launch L(c, nm_scan, (double)np * OS_RANGES * OS_MAX_BINS * 8);
      hipLaunchKernelGGL(k_os_scan, dim3(np), dim3(OS_MAX_BINS), 0, c->stream, hp, d,
                         base + (size_t)p0 * OS_RANGES * OS_MAX_BINS);
    }
    return check_launch(c, nm_scan);
  };
  if (!ranged && count(kin, 0, dg.passes)) return -1;
  const K *ki = kin;
  const uint32_t *vi = vin;
  K *ko = kA;
  uint32_t *vo = vA;
  for (uint32_t p = 0; p < dg.passes; p++) {
    const bool last = p + 1 == dg.passes;
    if (last && vfinal) {
      ko = nullptr;
      vo = vfinal;
    }
    // ranged: each pass counts its own input by range (a range's counts depend
    // on which keys the previous pass put there)
    if (ranged && count(ki, p, 1)) return -1;
    const uint32_t ep = ++c->os_epoch;
    const size_t pw = (size_t)p * OS_RANGES * OS_MAX_BINS;
    // the payload: packed from its source in pass 0, then the half buffers in turn
    OsPayload pl{};
    const bool carry = plb && sizeof(K) == 8 && shape == 2 && shift0 == 0 && bits <= OS_PL_MAX_BITS && ko;
    if (carry) {
      pl.cause = p == 0 ? plb->cause : nullptr;
      pl.kind = p == 0 ? plb->kind : nullptr;
      pl.lo_in = p == 0 ? nullptr : plb->lo[(p + 1) & 1];
      pl.lo_out = plb->lo[p & 1];
      pl.hi_out = last ? plb->hi : nullptr;
      pl.status = plb->status;
      pl.kb = bits;
    }
    {
      Launch L(c, nm, (double)N * ((ko ? 2 : 1) * sizeof(K) + (vi ? 8 : 4) + (last && inv ? 4 : 0) +
                                   (carry ? (p == 0 ? 9 : 4) + 4 + (last ? 4 : 0) : 0)));
      auto launch = [&](auto kern, uint32_t nt) {
        hipLaunchKernelGGL(kern, dim3(Tr * nr), dim3(nt), 0, c->stream, ki, vi, ko, vo,
                           last ? inv : nullptr, N, dg.shift[p], dg.bits[p], base + pw, lb, ep, c->os_exp,
                           Tr, ranged ? ticket + p * OS_RANGES : nullptr, pl);
      };
      if (shape == 1) {
        launch(k_os_pass<K, 512, 8>, 512);
      } else if (shape == 3) {
        launch(k_os_pass<K, 512, 16>, 512);
      } else if (!carry) {
        launch(k_os_pass<K, 1024, 8>, 1024);
      } else if constexpr (sizeof(K) == 8) {  // (the payload's role: a kernel each)
        const int m = 1 | (p == 0 ? 2 : 0) | (last ? 4 : 0);
        if (m == 1) launch(k_os_pass<K, 1024, 8, 1>, 1024);
        else if (m == 3) launch(k_os_pass<K, 1024, 8, 3>, 1024);
        else if (m == 5) launch(k_os_pass<K, 1024, 8, 5>, 1024);
        else launch(k_os_pass<K, 1024, 8, 7>, 1024);
      }
    }
    if (check_launch(c, nm)) return -1;
    ki = ko;
    vi = vo;
    ko = (ko == kA) ? kB : kA;
    vo = (vo == vA) ? vB : vA;
  }
  *kout = const_cast<K *>(ki);
  *vout = const_cast<uint32_t *>(vi);
  if (plb) {
    const bool carried = sizeof(K) == 8 && shape == 2 && shift0 == 0 && bits <= OS_PL_MAX_BITS && !vfinal;
    plb->lo_out = carried ? plb->lo[(dg.passes + 1) & 1] : nullptr;
  }
  return 0;
}

// rt: the tiles of another array than the batch's (one device-sized list, the
// giant tree's cross-tile children), instead of c->tab's
struct RSTab {
  uint32_t T, D;
  const uint32_t *tile_start, *tile_doc, *doc_off, *tile_first;
};

template <typename K>
int radix_sort(cw_ctx *c, const char *tag, const K *kin, const uint32_t *vin, K *kA,
               uint32_t *vA, K *kB, uint32_t *vB, uint32_t bits, uint32_t shift0, uint32_t N,
               K **kout, uint32_t **vout, uint32_t *inv = nullptr, uint32_t *vfinal = nullptr,
               const RSTab *rt = nullptr, OsPayloadBufs *plb = nullptr) {
  if (plb) plb->lo_out = nullptr;  // (carried only by the one-sweep passes)
  auto &t = c->tab;
  const RSTab tt = rt ? *rt
                      : RSTab{t.T, (uint32_t)(t.doc_off.size() - 1), dev_tab(c, "t_tile_start"),
                              dev_tab(c, "t_tile_doc"), dev_tab(c, "t_doc_off"),
                              dev_tab(c, "t_tile_first")};
  if (bits == 0) bits = 1;
  const uint32_t dbits_pack = ceil_log2(std::max(t.pack_dmax, 1u));
  if (c->pack_sort && !inv && !vfinal && !rt && !t.pack_doc0.empty() && bits + dbits_pack <= 8 * sizeof(K)) {
    // every document fits one tile: one in-LDS sort per pack of documents
    const uint32_t P = (uint32_t)t.pack_doc0.size() - 1;
    char nm[48];
    snprintf(nm, sizeof nm, "%s_pack", tag);
    {
      Launch L(c, nm, (double)N * (2 * sizeof(K) + (vin ? 8 : 4)));
      hipLaunchKernelGGL(k_pack_sort<K>, dim3(P), dim3(SORT_THREADS), 0, c->stream, kin, vin, kA,
                         vA, dev_tab(c, "t_pack_doc0"), dev_tab(c, "t_doc_off"), shift0, bits,
                         dbits_pack);
    }
    if (check_launch(c, nm)) return -1;
    *kout = kA;
    *vout = vA;
    return 0;
  }
  // one array (config 5's ids, the giant tree's cross-tile children): the
  // one-sweep passes (CW_ONESWEEP; 0 = the histogram-scan-scatter passes below)
  if (c->onesweep && tt.D == 1 && N >= c->onesweep_min)
    return onesweep_sort<K>(c, tag, kin, vin, kA, vA, kB, vB, bits, shift0, N, kout, vout, inv, vfinal, plb);
  const uint32_t maxd = std::min<uint32_t>(c->max_digit, MAX_DIGIT);
  const int passes = (int)((bits + maxd - 1) / maxd);
  uint32_t *hist = scratch_t<uint32_t>(c, "hist", (size_t)tt.T * (1u << ((bits + passes - 1) / passes)));
  if (!hist) return fail(c, "out of device memory (hist)");
  const K *ki = kin;
  const uint32_t *vi = vin;
  K *ko = kA;
  uint32_t *vo = vA;
  char nm[48];
  const uint32_t D = tt.D;
  uint32_t shift = shift0;
  for (int p = 0; p < passes; p++) {
    // the wider digits last: keys that arrive nearly sorted (the giant path's
    // group keys, parent ~ rank) spread over every bin only in the low pass,
    // whose tile runs are then longer (2 keys a bin and tile at 11 bits)
    const uint32_t dbits = bits / passes + ((uint32_t)p >= passes - bits % passes ? 1u : 0u);
    const uint32_t nb = 1u << dbits;
    const uint32_t sub0 = dbits <= SUB_BITS ? dbits : (dbits + 1) / 2;
    snprintf(nm, sizeof nm, "%s_hist", tag);
    {
      Launch L(c, nm, (double)N * sizeof(K) + (double)tt.T * nb * 4);
      hipLaunchKernelGGL(k_radix_hist<K>, dim3(tt.T), dim3(256), 0, c->stream, ki,
                         tt.tile_start, shift, dbits, hist);
    }
    if (check_launch(c, nm)) return -1;
    snprintf(nm, sizeof nm, "%s_scan", tag);
    if (D == 1 && tt.T > GSCAN_CHUNK) {
      // one document of many tiles: chunked scan over all workgroups (up to
      // one chunk of tiles, the one-workgroup scan is a single launch instead
      // of four)
      const uint32_t nc = (tt.T + GSCAN_CHUNK - 1) / GSCAN_CHUNK;
      uint32_t *cs = scratch_t<uint32_t>(c, "gscan_cs", (size_t)nc * nb);
      uint32_t *tot = scratch_t<uint32_t>(c, "gscan_tot", nb);
      if (!cs || !tot) return fail(c, "out of device memory (scan)");
      Launch L(c, nm, (double)tt.T * nb * 12);
      hipLaunchKernelGGL(k_gscan_colsum, dim3(nc), dim3(1024), 0, c->stream, hist, tt.T, nb, cs);
      hipLaunchKernelGGL(k_gscan_chunks, dim3((nb + 1023) / 1024), dim3(1024), 0, c->stream, cs, nc,
                         nb, tot);
      hipLaunchKernelGGL(k_gscan_bins, dim3(1), dim3(1024), 0, c->stream, tot, nb, 0u);
      hipLaunchKernelGGL(k_gscan_apply, dim3(nc), dim3(1024), 0, c->stream, hist, tt.T, nb, cs, tot);
    } else {
      Launch L(c, nm, (double)tt.T * nb * 8);
      hipLaunchKernelGGL(k_radix_scan, dim3(D), dim3(1024), 0, c->stream, hist,
                         tt.tile_first, tt.doc_off, dbits);
    }
    if (check_launch(c, nm)) return -1;
    snprintf(nm, sizeof nm, "%s_scatter", tag);
    {
      const bool last = p + 1 == passes;
      // vfinal: the last pass writes the values there and no keys
      if (last && vfinal) {
        ko = nullptr;
        vo = vfinal;
      }
      Launch L(c, nm, (double)N * ((ko ? 2 : 1) * sizeof(K) + (vi ? 8 : 4) + (last && inv ? 4 : 0)) +
                          (double)tt.T * nb * 4);
      hipLaunchKernelGGL(k_radix_scatter<K>, dim3(tt.T), dim3(SORT_THREADS), 0, c->stream, ki, vi,
                         ko, vo, tt.tile_start, tt.tile_doc,
                         tt.doc_off, hist, shift, dbits, sub0,
                         last ? inv : nullptr);
    }
    if (check_launch(c, nm)) return -1;
    shift += dbits;
    ki = ko;
    vi = vo;
    ko = (ko == kA) ? kB : kA;
    vo = (vo == vA) ? vB : vA;
  }
  *kout = const_cast<K *>(ki);
  *vout = const_cast<uint32_t *>(vi);
  return 0;
}

// Significant bits of a device array of keys (one OR reduction + 8-byte D2H).
int find_key_bits(cw_ctx *c, const uint64_t *keys, uint32_t N, uint32_t *bits) {
  unsigned long long *red = scratch_t<unsigned long long>(c, "red", 1);
  if (!red) return fail(c, "out of device memory (red)");
  HIPCHK(c, hipMemsetAsync(red, 0, 8, c->stream));
  hipLaunchKernelGGL(k_or_reduce, dim3(1024), dim3(256), 0, c->stream, keys, N, red);
  if (check_launch(c, "or_reduce")) return -1;
  unsigned long long v = 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(&v, red, 8, hipMemcpyDeviceToHost));
  *bits = v ? 64 - __builtin_clzll(v) : 1;
  return 0;
}

// Host tables for a document layout, rebuilt only when the layout changes.
// A one-document batch this large takes the giant-document path.
bool is_giant(const cw_ctx *c, uint64_t D, const uint64_t *off) {
  return D == 1 && (off[1] >= c->giant_min || off[1] >= LINK_IDX);
}

int ensure_tables(cw_ctx *c, uint64_t D, const uint64_t *off, bool force_giant = false) {
  const bool giant = force_giant || is_giant(c, D, off);
  const bool same = c->tab_on_device && c->last_off.size() == D + 1 && c->last_giant == giant &&
                    memcmp(c->last_off.data(), off, (D + 1) * 8) == 0;
  if (same) return 0;
  c->tab_on_device = false;
  build_tables(c, D, off, giant);
  if (upload_tables(c)) return -1;
  c->last_off.assign(off, off + D + 1);
  c->last_giant = giant;
  c->tab_on_device = true;
  return 0;
}

// Steps 3-9 of the list weave from the rank-ordered arrays: par (cause rank),
// skind, sval (the value emitted for each rank; nullptr = the rank itself).
// skey != nullptr: ::lamport-ts from the largest sorted id (otherwise the
// front end wrote it).  kbm: the front end's special/hide bitmaps or nullptr.
// spare: nullptr or two free buffers of >= 8 N bytes each (the id sort's
// ping-pong pair), which the giant tree's group-key sort then reuses.
int weave_tail(cw_ctx *c, uint64_t D, uint32_t N, bool giant, const uint32_t *par,
               const uint8_t *skind, const uint32_t *sval, const uint32_t *kbm,
               const uint64_t *skey, uint32_t ts_shift, cw_list_result *out,
               void *spareA = nullptr, void *spareB = nullptr, bool linked = false) {
  auto &t = c->tab;
  const dim3 B256(256);
  if (giant && out->max_ts && skey) {  // ::lamport-ts = largest id (k_fdir wrote it otherwise)
    hipLaunchKernelGGL(k_max_ts1, dim3(1), dim3(64), 0, c->stream, skey, N, ts_shift, out->max_ts);
    if (check_launch(c, "max_ts")) return -1;
  }
  uint32_t *nsc = scratch_t<uint32_t>(c, "nsc", N);
  uint32_t *fcS = scratch_t<uint32_t>(c, "fcS", N), *fcN = scratch_t<uint32_t>(c, "fcN", N);
  uint64_t *link = scratch_t<uint64_t>(c, "link", N);  // u32 or u64 links; room for the yarn sort
  uint32_t *thr = scratch_t<uint32_t>(c, "thr", N);
  uint8_t *vis8 = scratch_t<uint8_t>(c, "vis8", (size_t)N + 64);
  if (!nsc || !fcS || !fcN || !link || !thr || !vis8)
    return fail(c, "out of device memory (N=%u)", N);
  // the HBM walk's sublist buffers (the fused tour keeps its sublists in LDS)
  const bool hbm_walk = !(t.tour && !giant);
  uint32_t *slots = nullptr, *dyn_ctr = nullptr, *wcnt = nullptr, *wnext = nullptr,
           *sbase = nullptr, *order = nullptr;
  if (hbm_walk) {
    slots = scratch_t<uint32_t>(c, "slots", t.slots);
    dyn_ctr = scratch_t<uint32_t>(c, "dyn_ctr", D);
    // (one giant document: u64 {count, next} words, see k_walk)
    wcnt = scratch_t<uint32_t>(c, "wcnt", (giant ? 2 : 1) * (size_t)t.Wtot);
    wnext = scratch_t<uint32_t>(c, "wnext", t.Wtot);
    sbase = scratch_t<uint32_t>(c, "sbase", t.Wtot);
    order = scratch_t<uint32_t>(c, "order", t.Wtot);
    if (!slots || !dyn_ctr || !wcnt || !wnext || !sbase || !order)
      return fail(c, "out of device memory (walk, N=%u)", N);
  }
  uint32_t *doc_off = dev_tab(c, "t_doc_off"), *doc_log2k = dev_tab(c, "t_doc_log2k");
  uint32_t *doc_W = dev_tab(c, "t_doc_W"), *walk_first = dev_tab(c, "t_walk_first");
  // 3-5. effective parents, sibling order, links (linked: the caller wrote
  // link and thr, cw_weave_linked)
  if (giant && !linked) {
    const uint32_t gbits = ceil_log2(2ull * N + 2);
    const uint32_t root_key = gbits >= 32 ? 0xFFFFFFFFu : (1u << gbits) - 1;
    // group keys: sort input in thr (written only after the sort), ping-pong
    // pairs in the spare buffers when the caller has them
    uint32_t *gk = thr, *gkA, *gvA, *gkB, *gvB;
    if (spareA && spareB) {
      gkA = (uint32_t *)spareA;
      gvA = gkA + N;
      gkB = (uint32_t *)spareB;
      gvB = gkB + N;
    } else {
      gkA = scratch_t<uint32_t>(c, "g_keyA", N), gkB = scratch_t<uint32_t>(c, "g_keyB", N);
      gvA = scratch_t<uint32_t>(c, "g_valA", N), gvB = scratch_t<uint32_t>(c, "g_valB", N);
    }
    if (!gkA || !gkB || !gvA || !gvB || !gk) return fail(c, "out of device memory (giant tree)");
    const dim3 GN((N + 255) / 256);
    const bool glocal = c->glocal && N >= c->glocal_min;
    const uint32_t TL = (N + GL_TILE - 1) / GL_TILE;
    uint32_t *tcnt = nullptr;
    if (glocal) {
      tcnt = scratch_t<uint32_t>(c, "gl_tcnt", (size_t)TL + 1);
      if (!tcnt) return fail(c, "out of device memory (giant tree)");
      HIPCHK(c, hipMemsetAsync(tcnt, 0, ((size_t)TL + 1) * 4, c->stream));
    }
    {
      Launch L(c, "geff", (double)N * (4 + 1 + 4) + (glocal ? 0.0 : (double)N * 8));
      // (the walk's counter and the emit's rendered count zeroed here)
      hipLaunchKernelGGL(k_geff, GN, B256, 0, c->stream, par, skind, N, root_key, gk, fcS, fcN,
                         hbm_walk ? dyn_ctr : nullptr, out->visible_count, tcnt);
    }
    if (check_launch(c, "geff")) return -1;
    if (glocal) {
      // cross children's offsets: an exclusive scan of the tile counts in place
      // (the sort's chunked scan with one bin)
      const uint32_t nc = (TL + GSCAN_CHUNK - 1) / GSCAN_CHUNK;
      uint32_t *cs = scratch_t<uint32_t>(c, "gl_cs", (size_t)nc + 1);
      uint32_t *aux = scratch_t<uint32_t>(c, "gl_aux", 4);
      if (!cs || !aux) return fail(c, "out of device memory (giant tree)");
      uint32_t *mtot = aux + 1;
      {
        Launch L(c, "glocal", (double)N * (4 + 4 + 8 + 4 + 8 * 0.34));
        hipLaunchKernelGGL(k_gscan_colsum, dim3(nc), dim3(1024), 0, c->stream, tcnt, TL, 1u, cs);
        hipLaunchKernelGGL(k_gscan_chunks, dim3(1), dim3(1024), 0, c->stream, cs, nc, 1u, aux);
        hipLaunchKernelGGL(k_gscan_bins, dim3(1), dim3(1024), 0, c->stream, aux, 1u, 0u);
        hipLaunchKernelGGL(k_gscan_apply, dim3(nc), dim3(1024), 0, c->stream, tcnt, TL, 1u, cs, aux);
        hipLaunchKernelGGL(k_glocal<512>, dim3(TL), dim3(512), 0, c->stream, gk, N, tcnt, nsc, fcS, fcN,
                           gkA, gvA, mtot);
      }
      if (check_launch(c, "glocal")) return -1;
      // the cross children's count sizes their sort (one readback)
      if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
      HIPCHK(c, hipMemcpyAsync(c->pin_small, mtot, 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      const uint32_t M = c->pin_small[0];
      if (M > N) return fail(c, "cross children %u > %u", M, N);
      if (M) {
        const uint32_t TR = (M + TILE - 1) / TILE;
        std::vector<uint32_t> h((size_t)TR + 1 + TR + 2 + 2);
        for (uint32_t i = 0; i <= TR; i++) h[i] = std::min(i * TILE, M);  // tile_start
        for (uint32_t i = 0; i < TR; i++) h[TR + 1 + i] = 0;                // tile_doc
        h[2 * TR + 1] = 0, h[2 * TR + 2] = M;                               // doc_off
        h[2 * TR + 3] = 0, h[2 * TR + 4] = TR;                              // tile_first
        uint32_t *dt = scratch_t<uint32_t>(c, "gl_rtab", h.size());
        if (!dt) return fail(c, "out of device memory (giant tree)");
        HIPCHK(c, hipMemcpy(dt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        const RSTab rt{TR, 1u, dt, dt + TR + 1, dt + 2 * TR + 1, dt + 2 * TR + 3};
        uint32_t *gks, *gvs;  // (ping-pong through the input pair itself)
        if (radix_sort<uint32_t>(c, "gsort", gkA, gvA, gkB, gvB, gkA, gvA, gbits, 0, M, &gks, &gvs,
                                 nullptr, nullptr, &rt))
          return -1;
        {
          Launch L(c, "gcross", (double)M * (8 + 4 + 4 + 8));
          const dim3 GM((M + 255) / 256);
          hipLaunchKernelGGL(k_gcross_ns, GM, B256, 0, c->stream, gks, gvs, mtot, nsc, fcS, fcN);
          hipLaunchKernelGGL(k_gcross_fc, GM, B256, 0, c->stream, gks, gvs, mtot, fcS, fcN);
        }
        if (check_launch(c, "gcross")) return -1;
      }
    } else {
      uint32_t *gks, *gvs;
      if (radix_sort<uint32_t>(c, "gsort", gk, nullptr, gkA, gvA, gkB, gvB, gbits, 0, N, &gks, &gvs))
        return -1;
      {
        Launch L(c, "gsib", (double)N * (4 + 4 + 4 + 4));
        hipLaunchKernelGGL(k_gsib, GN, B256, 0, c->stream, gks, gvs, N, nsc, fcS, fcN);
      }
      if (check_launch(c, "gsib")) return -1;
    }
    {
      Launch L(c, "gthr", (double)N * (4 + 4 + 4 + 1 + 4 + 4));
      hipLaunchKernelGGL((k_gthr<256, 1024>), dim3((N + 1023) / 1024), B256, 0, c->stream, nsc,
                         fcS, fcN, skind, N, sval, thr, link);
    }
    if (check_launch(c, "gthr")) return -1;
  }
  if (!giant) {
    const uint32_t kbits = ceil_log2((uint64_t)t.nmax + 1) + 1;
    // special/hide bitmaps in LDS for documents up to 2^18 nodes
    const uint32_t bm_words = std::min<uint32_t>((t.nmax + 31) / 32, (1u << 18) / 32);
    // par, skind in; nsc, last-node tables, thr, link out; sweep 2 reads nsc
    // and the tables back
    unsigned long long *tprof = nullptr;
    if (c->tree_prof) {
      tprof = scratch_t<unsigned long long>(c, "tprof", (size_t)D * 16);
      HIPCHK(c, hipMemsetAsync(tprof, 0, (size_t)D * 128, c->stream));
    }
    constexpr uint32_t TL_NT = 1024;
    const uint32_t tl_dyn = tree_l_lds_bytes(t.nmax);
    // k_tree_l with 2,048-rank tiles, or 1,024 when the document needs the room
    const uint32_t tree_l = !c->tree_l ? 0
                            : c->tree_l == 2048 && tl_dyn + tree_l_static_bytes(TL_NT, 2048) <= c->lds_max ? 2048
                            : tl_dyn + tree_l_static_bytes(TL_NT, 1024) <= c->lds_max ? 1024 : 0;
    // k_tree_l: par 4 + kind bits in; fcS clear 4, nsc 4 out; sweep 2 reads
    // fcS, nsc (8) and writes link 4
    Launch L(c, "tree", tree_l ? (double)N * (4 + 1 + 4 + 4 + 8 + 4)
                               : (double)N * (4 + 1 + 4 + 8 + 4 + 8 + 4 + 4));
    auto tree_l_kernel = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((uint32_t)D), dim3(TL_NT),
                         (size_t)tl_dyn + tree_l_tile_bytes(TL_NT, tree_l), c->stream, par, skind,
                         doc_off, doc_log2k, kbits, (t.nmax + 31) / 32, nsc, fcS,
                         (uint32_t *)link, thr, tprof, kbm, dev_tab(c, "t_tile_first"), 0u);
    };
    auto tree_l_mode = [&](auto prof, auto mode) {
      constexpr bool P = decltype(prof)::value;
      constexpr int M = decltype(mode)::value;
      if (tree_l == 2048) tree_l_kernel(k_tree_l<TL_NT, 2048, P, M>);
      else tree_l_kernel(k_tree_l<TL_NT, 1024, P, M>);
    };
    auto tree_l_prof = [&](auto prof) { tree_l_mode(prof, std::integral_constant<int, 4>()); };
    if (tree_l) {
      if (tprof) tree_l_prof(std::true_type());
      else tree_l_prof(std::false_type());
    }
    else
      hipLaunchKernelGGL((k_tree<256, 1024>), dim3((uint32_t)D), dim3(256), (size_t)bm_words * 8,
                         c->stream, par, skind, doc_off, doc_log2k, kbits, bm_words, nsc, fcS, fcN, thr,
                         (uint32_t *)link, out->status, tprof, kbm, dev_tab(c, "t_tile_first"));
  }
  if (check_launch(c, "tree")) return -1;
  if (c->tree_prof && !giant) {
    std::vector<unsigned long long> h((size_t)D * 16);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h.data(), c->bufs["tprof"].p, (size_t)D * 128, hipMemcpyDeviceToHost));
    double acc[16] = {0};
    for (uint64_t d = 0; d < D; d++)
      for (int ph = 0; ph < 16; ph++) acc[ph] += (double)h[d * 16 + ph];
    // k_tree: bitmap climb sort prv s2load jump s2write; k_tree_l: bitmap barA . end
    // s2init s2calc jump s2write head keys issue insert walk barB
    fprintf(stderr, "tree phases (memtime ticks per doc):");
    for (int ph = 0; ph < 16; ph++) fprintf(stderr, " %d:%.0f", ph, acc[ph] / D);
    fprintf(stderr, "\n");
  }

  if (t.tour && !giant) {
    // 6-8. walk, rank and emit of every document in LDS
    unsigned long long *tprof = nullptr;
    if (c->tree_prof) {
      tprof = scratch_t<unsigned long long>(c, "tprof2", (size_t)D * 8);
      HIPCHK(c, hipMemsetAsync(tprof, 0, (size_t)D * 64, c->stream));
    }
    uint32_t *loc = scratch_t<uint32_t>(c, "tour_loc", N);
    if (!loc) return fail(c, "out of device memory (tour)");
    {
      Launch L(c, "tour", (double)N * (4 + 4 + 4 + 1 + 4 + 4));
      hipLaunchKernelGGL(k_tour<1024>, dim3((uint32_t)D), dim3(1024),
                         (size_t)tour_lds_bytes(t.nmax, t.tour_log2k), c->stream,
                         (const uint32_t *)link, sval, doc_off, doc_log2k, skey, ts_shift,
                         skey ? out->max_ts : nullptr, out->weave_perm, out->visible_bits,
                         out->visible_count, out->status, loc, tprof);
    }
    if (check_launch(c, "tour")) return -1;
    if (tprof) {
      std::vector<unsigned long long> h((size_t)D * 8);
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipMemcpy(h.data(), tprof, (size_t)D * 64, hipMemcpyDeviceToHost));
      double a[6] = {0};
      for (uint64_t d = 0; d < D; d++)
        for (int ph = 0; ph < 6; ph++) a[ph] += (double)h[d * 8 + ph];
      fprintf(stderr, "tour phases (memtime ticks per doc): load %.0f walk %.0f jump %.0f place %.0f "
              "write %.0f\n", a[0] / D, a[1] / D, a[2] / D, a[3] / D, a[4] / D);
    }
  } else {
    // 6. walk: sublists of the preorder successor list
    if (!(giant && !linked)) HIPCHK(c, hipMemsetAsync(dyn_ctr, 0, D * 4, c->stream));  // (k_geff did)
    c->last_dyn = dyn_ctr;  // (cw_get_counter "continued_sublists")
    c->last_dyn_n = (uint32_t)D;
    unsigned long long *wprof = nullptr;
    if (c->tree_prof && giant) {
      wprof = scratch_t<unsigned long long>(c, "wprof", 4);
      HIPCHK(c, hipMemsetAsync(wprof, 0, 32, c->stream));
    }
    {
      Launch L(c, "walk", (double)N * (4 + 4));
      hipLaunchKernelGGL(giant ? k_walk<true> : k_walk<false>, dim3(t.Bw), dim3(c->walk_threads),
                         0, c->stream, (const void *)link, thr,
                         dev_tab(c, "t_wblk_doc"), dev_tab(c, "t_wblk_w0"), doc_off, doc_log2k,
                         dev_tab(c, "t_doc_log2cap"), doc_W, dev_tab(c, "t_doc_Wcap"), walk_first,
                         (const uint64_t *)c->bufs["t_slot_first"].p, slots, wcnt, wnext, dyn_ctr,
                         out->status, c->walk_span, wprof);
    }
    if (check_launch(c, "walk")) return -1;
    if (wprof) {
      unsigned long long h[4];
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipMemcpy(h, wprof, 32, hipMemcpyDeviceToHost));
      fprintf(stderr, "walk profile: nodes %u steps %llu pending %llu thread hops %llu\n", N, h[0], h[1],
              h[2]);
    }

    // 7. rank sublists (+ max lamport-ts per document)
    uint4 *erec = nullptr;
    if (giant) {
      // the walkers the walk added (pending threads) stay on the device: the
      // ranking kernels read W + dyn_ctr[0] themselves, no readback (sync) here
      const uint32_t W = t.doc_W[0], Wcap = t.Wtot;
      const uint64_t *wl = reinterpret_cast<const uint64_t *>(wcnt);  // k_walk<true>'s words
      erec = scratch_t<uint4>(c, "g_erec", Wcap);
      if (!erec) return fail(c, "out of device memory (rank)");
      if (Wcap <= SUP_MAX) {  // few sublists: one LDS ranking, no walk levels
        uint32_t *nbt = scratch_t<uint32_t>(c, "g_nbt", 2 * (size_t)Wcap);
        if (!nbt) return fail(c, "out of device memory (rank)");
        Launch L(c, "rank", (double)Wcap * 36);
        hipLaunchKernelGGL(k_sup_rank, dim3(1), dim3(1024), (size_t)Wcap * 12, c->stream, wcnt, nullptr,
                           wcnt + 1, 2u, Wcap, N, Wcap, nbt, nbt + Wcap, out->status, nullptr, dyn_ctr, W,
                           Wcap);
        hipLaunchKernelGGL(k_lvl_apply, dim3((Wcap + 255) / 256), B256, 0, c->stream, nullptr, nbt,
                           nbt + Wcap, nullptr, wl, Wcap, nullptr, erec, dyn_ctr, W);
      } else {
        // levels: K = 16, until the walkers fit one LDS ranking; the last level
        // takes a longer stride (<= 64) instead of one more level of launches
        struct Lv { uint32_t E, Ws, K, S; size_t pos, wout, base; };
        std::vector<Lv> lv;
        size_t words = 0;  // (uint32 words of one scratch buffer, 16-byte units)
        uint32_t E = Wcap, Ws = W;
        while (lv.empty() || lv.back().S > SUP_MAX) {
          const uint32_t need = (Ws + SUP_MAX - 1) / SUP_MAX;
          uint32_t K = 16;
          if (need <= 64) {
            K = 1;
            while (K < need) K <<= 1;
          }
          Lv v{E, Ws, K, (Ws + K - 1) / K, 0, 0, 0};
          v.pos = words, words += lv.empty() ? 0 : 4 * (size_t)v.E;  // (sublist level: none)
          v.wout = words, words += 4 * (size_t)v.S;
          v.base = words, words += lv.empty() ? 0 : 4 * (((size_t)v.E + 1) / 2);
          lv.push_back(v);
          E = Ws = v.S;
        }
        const size_t nbt_off = words;
        words += 2 * (size_t)lv.back().S + 4;
        uint32_t *lb = scratch_t<uint32_t>(c, "g_levels", words);
        if (!lb) return fail(c, "out of device memory (multi-level rank)");
        auto u4 = [&](size_t o) { return reinterpret_cast<uint4 *>(lb + o); };
        auto u2 = [&](size_t o) { return reinterpret_cast<uint2 *>(lb + o); };
        Launch L(c, "rank", (double)Wcap * 40 + (double)lv[0].S * 40);
        for (size_t i = 0; i < lv.size(); i++) {
          const Lv &v = lv[i];
          if (i == 0)  // (no per-sublist records: k_lvl_emit walks again)
            hipLaunchKernelGGL(k_lvl_walk<true>, dim3((v.S + 255) / 256), B256, 0, c->stream,
                               (const void *)wl, v.Ws, v.E, v.K, v.S, nullptr, u4(v.wout), out->status,
                               dyn_ctr, W);
          else
            hipLaunchKernelGGL(k_lvl_walk<false>, dim3((v.S + 255) / 256), B256, 0, c->stream,
                               (const void *)u4(lv[i - 1].wout), v.Ws, v.E, v.K, v.S, u4(v.pos),
                               u4(v.wout), out->status, nullptr, 0u);
        }
        const Lv &top = lv.back();
        uint32_t *nb = lb + nbt_off, *tb = nb + top.S;
        const uint32_t *tw = lb + top.wout;
        hipLaunchKernelGGL(k_sup_rank, dim3(1), dim3(1024), (size_t)top.S * 12, c->stream, tw, tw + 1,
                           tw + 2, 4u, top.S, N, Wcap, nb, tb, out->status, nullptr, dyn_ctr, W, Wcap);
        for (size_t i = lv.size(); i-- > 0;) {
          const Lv &v = lv[i];
          const bool is_top = i + 1 == lv.size();
          const uint2 *bq = is_top ? nullptr : u2(lv[i + 1].base);
          if (i == 0) {
            hipLaunchKernelGGL(k_lvl_emit, dim3((v.S + 255) / 256), B256, 0, c->stream, wl, v.Ws, v.E, v.K,
                               v.S, nb, tb, bq, erec, dyn_ctr, W);
          } else
            hipLaunchKernelGGL(k_lvl_apply, dim3((v.E + 255) / 256), B256, 0, c->stream, u4(v.pos), nb,
                               tb, bq, nullptr, v.E, u2(v.base), nullptr, nullptr, 0u);
        }
      }
      if (check_launch(c, "rank")) return -1;
    } else {
      Launch L(c, "rank", (double)t.Wtot * 12);
      hipLaunchKernelGGL(k_rank, dim3((uint32_t)D), B256, (size_t)t.Wmax * 8, c->stream, wcnt,
                         wnext, walk_first, doc_W, dyn_ctr, doc_off, skey, ts_shift, sbase,
                         order, skey ? out->max_ts : nullptr, out->status);
    }
    if (check_launch(c, "rank")) return -1;

    // 8. emit
    {
      Launch L(c, "emit", (double)N * (4 + 4 + 4 + 1) + (double)t.Wtot * 8);
      // (giant: the slot entries hold the emitted values already, see k_walk)
      hipLaunchKernelGGL(k_emit, dim3(t.Be), B256, 0, c->stream, slots,
                         (const uint64_t *)c->bufs["t_slot_first"].p, wcnt, sbase, order,
                         giant ? nullptr : sval, erec,
                         dev_tab(c, "t_eblk_doc"), dev_tab(c, "t_eblk_x0"), walk_first, doc_W,
                         dyn_ctr, dev_tab(c, "t_doc_log2cap"), doc_off, out->weave_perm, vis8,
                         out->visible_count, out->status);
    }
    if (check_launch(c, "emit")) return -1;
  }

  // 9. visibility bitmap (the fused tour wrote it)
  if (out->visible_bits && !(t.tour && !giant)) {
    const uint32_t words = (N + 31) / 32;
    Launch L(c, "packbits", (double)N + (double)words * 4);
    hipLaunchKernelGGL(k_pack_bits, dim3((words + 255) / 256), B256, 0, c->stream, vis8, N,
                       out->visible_bits);
  }
  if (check_launch(c, "packbits")) return -1;

  return 0;
}

int weave_lists_device(cw_ctx *c, const cw_list_batch *bt, const uint64_t *id_key,
                       const uint64_t *cause_key, const uint8_t *kind, cw_list_result *out) {
  const uint64_t D = bt->n_docs;
  const uint32_t N = (uint32_t)bt->doc_offsets[D];
  auto &t = c->tab;
  const dim3 B256(256);

  HIPCHK(c, hipMemsetAsync(out->status, 0, D * 4, c->stream));
  c->xfront = cw_ctx::XFront{};
  // one giant document: k_geff zeroes the count, k_pack_bits writes every word
  const bool giant1 = is_giant(c, D, bt->doc_offsets);
  if (!giant1) HIPCHK(c, hipMemsetAsync(out->visible_count, 0, D * 4, c->stream));
  if (out->visible_bits && N && !giant1)
    HIPCHK(c, hipMemsetAsync(out->visible_bits, 0, ((size_t)N + 31) / 32 * 4, c->stream));
  c->x_hint = true;  // unknown unless the fused front end counts the flagged documents

  uint32_t key_bits = bt->key_bits;
  if (key_bits == 0 && N && find_key_bits(c, id_key, N, &key_bits)) return -1;
  if (key_bits > 64) key_bits = 64;

  uint64_t *skA = scratch_t<uint64_t>(c, "skA", N), *skB = scratch_t<uint64_t>(c, "skB", N);
  uint32_t *svA = scratch_t<uint32_t>(c, "svA", N), *svB = scratch_t<uint32_t>(c, "svB", N);
  uint32_t *par = scratch_t<uint32_t>(c, "par", N);
  uint8_t *skind = scratch_t<uint8_t>(c, "skind", N);
  // (the tail's node arrays; the yarn sort below reuses two of them)
  uint32_t *nsc = scratch_t<uint32_t>(c, "nsc", N);
  uint64_t *link = scratch_t<uint64_t>(c, "link", N);
  if (!skA || !skB || !svA || !svB || !par || !skind || !nsc || !link)
    return fail(c, "out of device memory (N=%u)", N);

  uint32_t *tile_start = dev_tab(c, "t_tile_start"), *tile_doc = dev_tab(c, "t_tile_doc");
  uint32_t *doc_off = dev_tab(c, "t_doc_off");
  const dim3 GT(t.T);
  const dim3 TB(c->tb);
  if (!grid_ok(t.T, std::max(c->tb, SORT_THREADS)) || !grid_ok(t.Bw, c->walk_threads) ||
      !grid_ok(t.Be, 256) || !grid_ok(D, 1024))
    return fail(c, "batch too large for one dispatch (split the batch)");

  if (N) {
    uint64_t *skey = nullptr;
    uint32_t *sval = nullptr;
    const bool want_yarns = out->yarn_perm && bt->site_bits;
    // 1-2 (dense ids). id order and join through per-document rank directories
    bool front_done = false, fused_done = false, yarns_fused = false;
    uint32_t *kbm = nullptr;  // special / hide bitmaps per tile (front end -> tree)
    // fused front end: documents of < 2^16 nodes whose ids fit a 40 KiB directory
    if (c->front && c->front_fused && N >= (uint64_t)c->front_min_avg * D &&
        t.nmax <= 0xFFFFu && front_lds_bytes(t.nmax, FRONT_FUSED_SG) <= c->lds_max - 1024) {
      uint32_t *big = scratch_t<uint32_t>(c, "fr_big", 4);
      uint16_t *rank16 = scratch_t<uint16_t>(c, "fr_rank16", N);
      kbm = scratch_t<uint32_t>(c, "fr_kbm", (size_t)t.T * KBM_WORDS);
      if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
      if (!big || !rank16 || !kbm) return fail(c, "out of device memory (front)");
      HIPCHK(c, hipMemsetAsync(big, 0, 16, c->stream));
      sval = svA;
      // the yarns by k_yarn_doc after the fused kernel (site fields of <= 4
      // bits, the document's sites and yarn in LDS): no ids in rank order
      // written, no sort by site afterwards
      yarns_fused = want_yarns && bt->site_bits <= 4 && yarn_lds_bytes(t.nmax) + 64 <= c->lds_max;
      unsigned long long *tprof_f = nullptr;
      if (c->tree_prof) {
        tprof_f = scratch_t<unsigned long long>(c, "tprof3", (size_t)D * 8);
        HIPCHK(c, hipMemsetAsync(tprof_f, 0, (size_t)D * 64, c->stream));
      }
      // the whole weave in one kernel when every phase fits: k_tree_l's
      // 2,048-rank tiles and the fused tour (CW_FUSED)
      const uint32_t fr_lds = front_lds_bytes(t.nmax, FRONT_FUSED_SG);
      const uint32_t tl_lds = tree_l_lds_bytes(t.nmax) + tree_l_tile_bytes(1024, 2048);
      const uint32_t to_lds = tour_lds_bytes(t.nmax, t.tour_log2k);
      const uint32_t wd_lds = std::max(fr_lds, std::max(tl_lds, to_lds));
      // (the fused kernel needs k_tree_l's 2,048-rank tiles: CW_TREE_L = 0 or
      // 1024 run the separate kernels)
      fused_done = c->fused && t.tour && !giant1 && c->tree_l == 2048 &&
                   tl_lds + 64 * 4 + 4 <= c->lds_max &&
                   wd_lds + 1024 <= c->lds_max && to_lds <= TOUR_LDS_MAX;
      // (k_front writes the ids for the yarn sort)
      yarns_fused = yarns_fused && fused_done;
      skey = want_yarns && !yarns_fused ? skA : nullptr;
      if (fused_done) {
        uint32_t *fcS = scratch_t<uint32_t>(c, "fcS", N), *thr = scratch_t<uint32_t>(c, "thr", N);
        uint32_t *loc = scratch_t<uint32_t>(c, "tour_loc", N);
        if (!fcS || !thr || !loc)
          return fail(c, "out of device memory (fused weave)");
        const uint32_t kbits_t = ceil_log2((uint64_t)t.nmax + 1) + 1;
        // par and (without yarns, which sort by it) sval as u16, no skind
        uint16_t *par16 = scratch_t<uint16_t>(c, "par16", N);
        // the site of every input, for k_yarn_doc (one byte a node)
        uint8_t *site8 = yarns_fused ? scratch_t<uint8_t>(c, "site8", N) : nullptr;
        if (yarns_fused && !site8) return fail(c, "out of device memory (fused weave)");
        uint16_t *sval16 = want_yarns && !yarns_fused ? nullptr : scratch_t<uint16_t>(c, "sval16", N);
        if (!par16 || (!(want_yarns && !yarns_fused) && !sval16))
          return fail(c, "out of device memory (fused weave)");
        // algorithmic bytes: front end (ids twice, causes, kinds, the rank scratch
        // out and back, par 2, sval 2 or 4, class bitmaps), tree (par 2, kind bits;
        // fcS clear 4, nsc 4; fcS + nsc back 8, link 4), tour (link 4, sval, the
        // (sublist, index) records out and back 8, weave_perm 4, bits)
        const double sv = want_yarns ? 4 : 2;
        Launch L(c, "weave", (double)N * (8 + 8 + 8 + 1 + 2 + 2 + 2 + sv + (skey ? 16 : 0) + (site8 ? 1 : 0) + 0.25) +
                                 (double)N * (2 + 0.25 + 4 + 4 + 8 + 4) +
                                 (double)N * (4 + sv + 8 + 4 + 0.125));
        auto launch = [&](auto kern, auto *sv_ptr) {
          hipLaunchKernelGGL(kern, dim3((uint32_t)D), dim3(1024), (size_t)wd_lds, c->stream, id_key,
                             cause_key, kind, doc_off, dev_tab(c, "t_tile_first"), FRONT_FUSED_SG, par16,
                             nullptr, sv_ptr, kbm, skey, rank16, out->max_ts, bt->ts_shift, out->status,
                             big, dev_tab(c, "t_doc_log2k"), kbits_t, (t.nmax + 31) / 32, nsc, fcS,
                             (uint32_t *)link, thr, out->weave_perm, out->visible_bits,
                             out->visible_count, loc, tprof_f, site8, bt->site_shift,
                             (1u << bt->site_bits) - 1u);
        };
        const bool wy = want_yarns && !yarns_fused;  // (u32 sval: the yarn sort's values)
        if (tprof_f) {  // (the default front-end depth, so the clocks are the product's)
          if (wy) launch(k_weave_doc<1024, 2048, uint32_t, true, 4, 1>, sval);
          else launch(k_weave_doc<1024, 2048, uint16_t, true, 4, 1>, sval16);
        } else {
          if (wy) launch(k_weave_doc<1024, 2048, uint32_t, false, 4, 1>, sval);
          else launch(k_weave_doc<1024, 2048, uint16_t, false, 4, 1>, sval16);
        }
      } else {
        Launch L(c, "front", (double)N * (8 + 8 + 1 + 2 + 4 + 1 + 2 + 4 + (skey ? 16 : 0)) + (double)N * 8);
        hipLaunchKernelGGL(k_front<1024>, dim3((uint32_t)D), dim3(1024),
                           (size_t)fr_lds, c->stream, id_key,
                           cause_key, kind, doc_off, dev_tab(c, "t_tile_first"), FRONT_FUSED_SG, par,
                           skind, sval, kbm, skey, rank16, out->max_ts, bt->ts_shift, out->status, big,
                           tprof_f);
      }
      if (check_launch(c, fused_done ? "weave" : "front")) return -1;
      if (tprof_f && fused_done) {
        std::vector<unsigned long long> h((size_t)D * 8);
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(h.data(), tprof_f, (size_t)D * 64, hipMemcpyDeviceToHost));
        double a[3] = {0};
        for (uint64_t dd = 0; dd < D; dd++)
          for (int ph = 0; ph < 3; ph++) a[ph] += (double)h[dd * 4 + ph];
        fprintf(stderr, "weave phases (memtime ticks per doc): front %.0f tree %.0f tour %.0f\n", a[0] / D,
                a[1] / D, a[2] / D);
      } else if (tprof_f) {
        std::vector<unsigned long long> h((size_t)D * 8);
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(h.data(), tprof_f, (size_t)D * 64, hipMemcpyDeviceToHost));
        double a[6] = {0};
        for (uint64_t dd = 0; dd < D; dd++)
          for (int ph = 0; ph < 6; ph++) a[ph] += (double)h[dd * 8 + ph];
        fprintf(stderr, "front phases (memtime ticks per doc): dir %.0f rank %.0f write %.0f sval %.0f "
                "svwrite %.0f\n", a[0] / D, a[1] / D, a[2] / D, a[3] / D, a[4] / D);
      }
      HIPCHK(c, hipMemcpyAsync(c->pin_small, big, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (c->pin_small[0] == 0) {
        front_done = true;
        c->x_hint = c->pin_small[1] != 0;  // flagged documents, for the exact path
        if (fused_done && yarns_fused) {
          Launch L(c, "yarns", (double)N * (1 + 2 + 2 + 4));
          hipLaunchKernelGGL(k_yarn_doc<1024>, dim3((uint32_t)D), dim3(1024), (size_t)yarn_lds_bytes(t.nmax),
                             c->stream, (const uint8_t *)c->bufs["site8"].p, rank16,
                             (const uint16_t *)c->bufs["sval16"].p, doc_off, out->yarn_perm);
        }
        if (check_launch(c, "yarns")) return -1;
      } else {  // a document's ids leave the small directory: the three-kernel front end
        HIPCHK(c, hipMemsetAsync(out->status, 0, D * 4, c->stream));
        if (fused_done) {  // (and the separate tree and tour: the fused kernel stopped early)
          fused_done = false;
          HIPCHK(c, hipMemsetAsync(out->visible_count, 0, D * 4, c->stream));
          if (out->visible_bits)
            HIPCHK(c, hipMemsetAsync(out->visible_bits, 0, ((size_t)N + 31) / 32 * 4, c->stream));
        }
        sval = nullptr;
        skey = nullptr;
        kbm = nullptr;
      }
    }
    // one giant document whose ids fit a global rank directory:
    // no id sort, no bucket index, no searching join
    // (a directory larger than the caches makes k_gd_set's atomics HBM round
    // trips: 6.7e7 nodes over 2^31 keys took 12.8 ms against 8.3 for sort +
    // join, so the directory is taken only while it stays small)
    if (!front_done && c->gdir && is_giant(c, D, bt->doc_offsets) && key_bits <= GD_MAX_BITS &&
        (1ull << key_bits) / GD_KEYS * GD_WORDS * 4 <= (uint64_t)c->gdir * (1ull << 20)) {
      const uint64_t E = ((1ull << key_bits) + GD_KEYS - 1) / GD_KEYS;
      const uint32_t nb = (uint32_t)((E + 1023) / 1024);
      uint32_t *dir = scratch_t<uint32_t>(c, "gd_dir", E * GD_WORDS);
      uint32_t *sums = scratch_t<uint32_t>(c, "gd_sums", nb + 1);
      unsigned long long *maxid = scratch_t<unsigned long long>(c, "gd_max", 1);
      if (dir && sums && maxid) {
        HIPCHK(c, hipMemsetAsync(dir, 0, E * GD_WORDS * 4, c->stream));
        HIPCHK(c, hipMemsetAsync(maxid, 0, 8, c->stream));
        const dim3 GN((N + 255) / 256);
        {
          Launch L(c, "gdir", (double)N * 8 + (double)E * GD_WORDS * 4 * 2);
          hipLaunchKernelGGL(k_gd_set, GN, dim3(256), 0, c->stream, id_key, N, E, dir, maxid,
                             out->status);
          hipLaunchKernelGGL(k_gd_count, dim3(nb), dim3(1024), 0, c->stream, dir, E, sums);
          hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, c->stream, sums, nb, sums + nb);
          hipLaunchKernelGGL(k_gd_add, dim3(nb), dim3(1024), 0, c->stream, dir, E, sums);
        }
        if (check_launch(c, "gdir")) return -1;
        skey = want_yarns ? skA : nullptr;
        sval = svA;
        {
          // (SURVEY 8d's bytes: ids, causes and kinds in, par, kind, sval (and keys)
          // out -- not the directory lines each lookup touches: those are traffic)
          Launch L(c, "gplace", (double)N * (8 + 8 + 1 + 4 + 1 + 4 + (skey ? 8 : 0)));
          hipLaunchKernelGGL(k_gd_place, GN, dim3(256), 0, c->stream, id_key, cause_key, kind, N,
                             reinterpret_cast<const uint4 *>(dir), maxid, bt->ts_shift, out->max_ts,
                             par, skind, sval, skey, out->status);
        }
        if (check_launch(c, "gplace")) return -1;
        front_done = true;
      }
    }
    if (!front_done && c->front && N >= (uint64_t)c->front_min_avg * D && t.nmax <= 64 * TILE) {
      const uint32_t SG = c->front_slot_groups;
      uint4 *dir = scratch_t<uint4>(c, "fr_dir", (size_t)D * SG);
      uint64_t *dkmin = scratch_t<uint64_t>(c, "fr_kmin", D);
      uint32_t *dgroups = scratch_t<uint32_t>(c, "fr_groups", D);
      uint32_t *big = scratch_t<uint32_t>(c, "fr_big", 4);
      if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
      if (!dir || !dkmin || !dgroups || !big) return fail(c, "out of device memory (rank directory)");
      HIPCHK(c, hipMemsetAsync(big, 0, 16, c->stream));
      {
        Launch L(c, "fdir", (double)N * 8 + (double)N / 6.0 * 1.0);  // ids once + directory
        // few documents: one workgroup reads a whole large document, so keep
        // 16 loads in flight per lane instead of 4
        auto *fdir = D <= 64 ? k_fdir<1024, 16> : k_fdir<1024, 4>;
        hipLaunchKernelGGL(fdir, dim3((uint32_t)D), dim3(1024),
                           (size_t)SG * 16, c->stream, id_key, doc_off, SG, dir, dkmin, dgroups,
                           out->max_ts, bt->ts_shift, out->status, big);
      }
      if (check_launch(c, "fdir")) return -1;
      HIPCHK(c, hipMemcpyAsync(c->pin_small, big, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      const uint32_t nbig = c->pin_small[0], gmax = c->pin_small[1];
      if (nbig == 0) {
        skey = want_yarns ? skA : nullptr;
        sval = svA;
        uint32_t *rec_meta = svB, *rec_par = (uint32_t *)skB;  // free until the yarn sort
        uint32_t *woff = scratch_t<uint32_t>(c, "fr_woff", t.Wofftot);
        kbm = scratch_t<uint32_t>(c, "fr_kbm", (size_t)t.T * KBM_WORDS);
        if (!woff || !kbm) return fail(c, "out of device memory (window table)");
        {
          Launch L(c, "frank", (double)N * (8 + 8 + 1 + 4 + 4));
          hipLaunchKernelGGL((k_frank<512>), GT, dim3(512),
                             std::max<size_t>((size_t)gmax * 16, 2 * TILE * 4),
                             c->stream, id_key, cause_key, kind, tile_start, tile_doc,
                             dev_tab(c, "t_tile_first"), doc_off, dev_tab(c, "t_woff_base"), dir,
                             SG, dkmin, dgroups, rec_meta, rec_par, woff, out->status);
        }
        if (check_launch(c, "frank")) return -1;
        {
          Launch L(c, "fplace", (double)N * (4 + 4 + 4 + 4 + 1 + (skey ? 16 : 0)));
          hipLaunchKernelGGL((k_fplace<512>), GT, dim3(512), 0, c->stream, rec_meta, rec_par,
                             woff, dev_tab(c, "t_woff_base"), tile_start, tile_doc,
                             dev_tab(c, "t_tile_first"), doc_off, id_key, sval, par, skind, skey,
                             kbm);
        }
        if (check_launch(c, "fplace")) return -1;
        front_done = true;
      } else {
        // some document's ids are too sparse for a slot: general path for the batch
        HIPCHK(c, hipMemsetAsync(out->status, 0, D * 4, c->stream));
      }
    }
    if (!front_done) {
    // 1. id sort (one giant document: carrying every node's cause and kind to
    // rank order, in the giant tree's four u32 buffers, free until the tree)
    const bool gd_join = is_giant(c, D, bt->doc_offsets) && c->gjoin && key_bits <= GD_MAX_BITS;
    OsPayloadBufs plb{};
    OsPayloadBufs *plp = nullptr;
    if (gd_join && key_bits <= OS_PL_MAX_BITS && c->id_payload) {
      plb.cause = cause_key;
      plb.kind = kind;
      plb.status = out->status;
      plb.lo[0] = scratch_t<uint32_t>(c, "g_keyA", N);
      plb.lo[1] = scratch_t<uint32_t>(c, "g_keyB", N);
      plb.hi = scratch_t<uint32_t>(c, "g_valA", N);
      if (!plb.lo[0] || !plb.lo[1] || !plb.hi) return fail(c, "out of device memory (id sort)");
      plp = &plb;
    }
    if (radix_sort<uint64_t>(c, "idsort", id_key, nullptr, skA, svA, skB, svB, key_bits, 0, N,
                             &skey, &sval, nullptr, nullptr, nullptr, plp))
      return -1;

    // 2. join
    // one giant document: a rank directory built from the sorted ids answers
    // each cause with one line (no bucket index, no search)
    const uint64_t E = ((1ull << std::min(key_bits, 63u)) + GD_KEYS - 1) / GD_KEYS;
    uint32_t *gdir = nullptr;
    if (gd_join) gdir = scratch_t<uint32_t>(c, "gd_dir", E * GD_WORDS);
    if (gdir) {
      {
        Launch L(c, "index", (double)N * 8 + (double)N / 15 * 64);
        hipLaunchKernelGGL(k_gd_build, dim3((N + GDB_KEYS - 1) / GDB_KEYS), B256, 0, c->stream, skey, N,
                           E, gdir, out->status);
      }
      if (check_launch(c, "index")) return -1;
      if (plp && plb.lo_out) {
        {
          // SURVEY 8d's join bytes: the cause (with the kind) read, the parent
          // rank and kind written -- all in rank order now
          Launch L(c, "join", (double)N * (8 + 4 + 1));
          hipLaunchKernelGGL(k_gjoin_r, dim3((N + 256 * GJOIN_ITEMS - 1) / (256 * GJOIN_ITEMS)), B256, 0,
                             c->stream, skey, plb.lo_out, plb.hi, key_bits, N,
                             reinterpret_cast<const uint4 *>(gdir), E, par, skind, out->status);
        }
        if (check_launch(c, "join")) return -1;
        // (the exact path gathers causes by input index: the carried ones go
        // with the giant tree's buffers)
        c->xfront = {skey, sval, reinterpret_cast<const uint4 *>(gdir), E, nullptr, N, false};
      } else {
      // cause and kind packed in one word per input node when the ids leave
      // 9 bits (the id sort's other key buffer is free by now)
      uint64_t *ckk = key_bits <= 55 ? (skey == skA ? skB : skA) : nullptr;
      if (ckk) {
        Launch L(c, "gpack", (double)N * (8 + 1 + 8));
        hipLaunchKernelGGL(k_gpack, dim3((N + 255) / 256), B256, 0, c->stream, cause_key, kind, N, ckk);
      }
      {
        // SURVEY 8d's join bytes (the cause read, the parent rank written) plus
        // the sorted position's input index and kind: not the directory line a
        // lookup touches (round 5 counted N x 64 of those as algorithmic)
        Launch L(c, "join", (double)N * (4 + 8 + 8 + 1 + 4 + 1));
        hipLaunchKernelGGL(k_gjoin, dim3((N + 256 * GJOIN_ITEMS - 1) / (256 * GJOIN_ITEMS)), B256, 0,
                           c->stream, skey, sval, cause_key, kind, N, ckk,
                           reinterpret_cast<const uint4 *>(gdir), E, par, skind, out->status);
      }
      if (check_launch(c, "join")) return -1;
      c->xfront = {skey, sval, reinterpret_cast<const uint4 *>(gdir), E, ckk, N, false};
      }
    } else {
    uint32_t *bkt = scratch_t<uint32_t>(c, "bkt", t.Btot);
    if (!bkt) return fail(c, "out of device memory (bucket index)");
    {
      Launch L(c, "index", (double)N * 8 + (double)t.Btot * 4);
      if (D == 1 && N > (1u << 16))  // one large document: a thread per id
        hipLaunchKernelGGL(k_index_flat, dim3((N + 255) / 256), B256, 0, c->stream, skey, N, bkt,
                           out->status);
      else
        hipLaunchKernelGGL(k_index, dim3((uint32_t)D), B256, 0, c->stream, skey, doc_off,
                           dev_tab(c, "t_bkt_off"), bkt, out->status);
    }
    if (check_launch(c, "index")) return -1;
    {
      Launch L(c, "join", (double)N * (4 + 8 + 8 + 1 + 4 + 1));
      hipLaunchKernelGGL(k_join, GT, TB, 0, c->stream, skey, sval, cause_key, kind, bkt,
                         dev_tab(c, "t_bkt_off"), tile_start, tile_doc, doc_off, par, skind,
                         out->status);
    }
    if (check_launch(c, "join")) return -1;
    }  // bucket index
    }  // general front end

    // 3-9. tree, walk, rank, emit, visibility
    // one giant document: its status (domain bits final now) goes to pinned
    // memory behind an event, so the exact path's check waits for this point
    // of the stream only, not for the whole weave (no sync between launches)
    if (is_giant(c, D, bt->doc_offsets)) {
      if (!c->pin_status) HIPCHK(c, hipHostMalloc((void **)&c->pin_status, 64, hipHostMallocDefault));
      if (!c->ev_status) HIPCHK(c, hipEventCreateWithFlags(&c->ev_status, hipEventDisableTiming));
      HIPCHK(c, hipMemcpyAsync(c->pin_status, out->status, 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipEventRecord(c->ev_status, c->stream));
      c->x_pending = true;
    }
    // A large list the front end flagged for the exact path (exact.hip, which
    // rewrites every output of it) skips the fast path's tree, tour and yarns:
    // one wait for the status copy, worth it above 2^22 nodes (the tail of
    // 6.7e7 nodes is ~9 ms; config 1's 1e5 nodes keep the call sync-free).
    bool flagged = false;
    if (c->x_pending && N >= (1u << 22) && bt->key_bits && bt->key_bits < 64) {
      HIPCHK(c, hipEventSynchronize(c->ev_status));
      const uint32_t st = c->pin_status[0];
      flagged = (st & (CW_STATUS_ROOT | CW_STATUS_ORPHAN | CW_STATUS_NON_LAMPORT)) &&
                !(st & (CW_STATUS_DUP | CW_STATUS_KEY_RANGE | CW_STATUS_INTERNAL));
      // the sorted ids and the directory stay intact (no tail): the exact path
      // joins from them instead of sorting again
      c->xfront.ok = flagged && c->xfront.skey && c->xfront.n == N;
    }
    // without yarns the id-sort buffers are free once the ids are joined
    const bool spare = !want_yarns;
    if (!fused_done && !flagged &&
        weave_tail(c, D, N, is_giant(c, D, bt->doc_offsets), par, skind, sval, kbm,
                   front_done ? nullptr : skey, bt->ts_shift, out, spare ? skA : nullptr,
                   spare ? skB : nullptr))
      return -1;

    // 10. yarns: stable partition of the id order by site rank (unless the
    // fused kernel wrote them)
    if (want_yarns && !flagged && !(fused_done && yarns_fused)) {
      uint64_t *yk;
      uint32_t *yv;
      uint64_t *ykA = skey == skA ? skB : skA;
      uint32_t *yvA = sval == svA ? svB : svA;
      // (skey, sval) stay intact: ping-pong through the free id buffers + link/loc
      // (the last pass writes yarn_perm itself, without the keys)
      if (radix_sort<uint64_t>(c, "yarns", skey, sval, ykA, yvA, link, nsc, bt->site_bits,
                               bt->site_shift, N, &yk, &yv, nullptr, out->yarn_perm))
        return -1;
    }
    // ids of 64 significant bits: the documents with an id >= 2^63 (KEY_RANGE)
    if (key_bits >= 64) {
      hipLaunchKernelGGL(k_key_range, GT, B256, 0, c->stream, id_key, tile_start, tile_doc,
                         out->status);
      if (check_launch(c, "key_range")) return -1;
    }
  }
  // empty documents (no root) are flagged by the host wrapper
  return 0;
}

}  // namespace

#include "exact.hip"
#include "mappack.hip"
#include "dist.hip"

namespace {

// The list weave of a batch already in device memory (dres: device arrays):
// the fast path, then the exact path for its flagged documents.
int weave_lists_dev_all(cw_ctx *c, const cw_list_batch *bt, const uint64_t *id,
                        const uint64_t *cause, const uint8_t *kind, cw_list_result *dres_p) {
  cw_list_result &dres = *dres_p;
  const uint64_t D = bt->n_docs;
  const uint32_t N = (uint32_t)bt->doc_offsets[D];
  // A few large documents would leave the per-document tree with a handful of
  // workgroups on a 256-CU GPU: weave them one by one on the all-parallel
  // giant-document path instead (render bits merged at each document's offset).
  // (estimated times: the per-document tree sweeps ~22 ns a node in one
  // workgroup, all documents at once; the giant path costs ~0.4 ms a call plus
  // ~0.3 ns a node, documents one after another)
  // A document below giant_min goes through its one-document sub-call on the
  // per-document tree (one workgroup), so it counts at that rate.
  double t_tree = 0, t_giant = 0;
  uint64_t nd_max = 0;
  for (uint64_t d = 0; d < D; d++) {
    const uint64_t n = bt->doc_offsets[d + 1] - bt->doc_offsets[d];
    const double nd = (double)n;
    nd_max = std::max(nd_max, n);
    t_tree = std::max(t_tree, nd * 22e-9);
    t_giant += n >= c->giant_min ? 0.4e-3 + nd * 0.3e-9 : 0.1e-3 + nd * 22e-9;
  }
  bool x_hint = false;
  c->x_pending = false;
  if (D > 1 && D <= c->giant_docs_max && nd_max >= c->giant_min && t_giant < t_tree) {
    if (dres.visible_bits)
      HIPCHK(c, hipMemsetAsync(dres.visible_bits, 0, ((size_t)N + 31) / 32 * 4, c->stream));
    for (uint64_t d = 0; d < D; d++) {
      const uint64_t b = bt->doc_offsets[d], nd = bt->doc_offsets[d + 1] - b;
      if (nd == 0) {
        HIPCHK(c, hipMemsetAsync(dres.status + d, 0, 4, c->stream));
        HIPCHK(c, hipMemsetAsync(dres.visible_count + d, 0, 4, c->stream));
        if (dres.max_ts) HIPCHK(c, hipMemsetAsync(dres.max_ts + d, 0, 8, c->stream));
        continue;
      }
      const uint64_t off1[2] = {0, nd};
      if (ensure_tables(c, 1, off1)) return -1;
      cw_list_batch sb = *bt;
      sb.n_docs = 1;
      sb.doc_offsets = off1;
      cw_list_result sr{};
      sr.weave_perm = dres.weave_perm + b;
      sr.visible_count = dres.visible_count + d;
      sr.max_ts = dres.max_ts ? dres.max_ts + d : nullptr;
      sr.status = dres.status + d;
      sr.yarn_perm = dres.yarn_perm ? dres.yarn_perm + b : nullptr;
      uint32_t *vb = nullptr;
      if (dres.visible_bits) {
        vb = scratch_t<uint32_t>(c, "gd_bits", (nd + 31) / 32 + 1);
        if (!vb) return fail(c, "out of device memory (bits)");
      }
      sr.visible_bits = vb;
      if (weave_lists_device(c, &sb, id + b, cause + b, kind + b, &sr)) return -1;
      x_hint |= c->x_hint;
      if (vb) {
        const uint32_t words = (uint32_t)((nd + 31) / 32);
        hipLaunchKernelGGL(k_or_bits_at, dim3((words + 255) / 256), dim3(256), 0, c->stream, vb,
                           (uint32_t)nd, dres.visible_bits, (uint32_t)b);
        if (check_launch(c, "or_bits")) return -1;
      }
    }
  } else {
    if (weave_lists_device(c, bt, id, cause, kind, &dres)) return -1;
    x_hint = c->x_hint;
  }
  // documents outside the fast path's domain: the literal fold (exact.hip)
  if (exact_fixup(c, bt, id, cause, kind, &dres, x_hint)) return -1;
  return 0;

}

// dev_inputs: id_key / cause_key / kind are device arrays even when the results
// are host memory (cw_weave_lists_k32 widens its keys on the device first).
int weave_lists_impl(cw_ctx *c, const cw_list_batch *bt, cw_list_result *res, int memspace,
                     bool dev_inputs = false) {
  if (!bt || !res) return fail(c, "null batch/result");
  const uint64_t D = bt->n_docs;
  if (!bt->doc_offsets) return fail(c, "doc_offsets is required (host memory)");
  const uint64_t N64 = bt->doc_offsets[D];
  if (bt->doc_offsets[0] != 0) return fail(c, "doc_offsets[0] must be 0");
  if (N64 >= 0xFFFFFFFFull) return fail(c, "batch too large: N=%llu (limit 2^32-1)",
                                        (unsigned long long)N64);
  // a one-document batch takes the giant path (wide links) up to 2^31 - 2
  // nodes; in a batch of several documents each stays below 2^29 - 1
  for (uint64_t d = 0; d < D; d++) {
    if (bt->doc_offsets[d + 1] < bt->doc_offsets[d]) return fail(c, "doc_offsets not monotone");
    const uint64_t nd = bt->doc_offsets[d + 1] - bt->doc_offsets[d];
    if (D == 1 ? nd >= SUCCW_END : nd >= LINK_IDX)
      return fail(c, "document %llu too large (limit %s nodes)", (unsigned long long)d,
                  D == 1 ? "2^31-2" : "2^29-2 in a batch of several documents");
  }
  if (!res->weave_perm || !res->visible_count || !res->status)
    return fail(c, "weave_perm, visible_count and status are required");
  const uint32_t N = (uint32_t)N64;
  HIPCHK(c, hipSetDevice(c->device));

  // host tables (cached while the document layout repeats)
  if (ensure_tables(c, D, bt->doc_offsets)) return -1;

  const uint64_t *id = bt->id_key, *cause = bt->cause_key;
  const uint8_t *kind = bt->kind;
  cw_list_result dres = *res;
  if (memspace == CW_MEM_HOST) {
    if (N && (!id || !cause || !kind)) return fail(c, "null input arrays");
    uint64_t *did = dev_inputs ? nullptr : scratch_t<uint64_t>(c, "h_id", N);
    uint64_t *dca = dev_inputs ? nullptr : scratch_t<uint64_t>(c, "h_cause", N);
    uint8_t *dk = dev_inputs ? nullptr : scratch_t<uint8_t>(c, "h_kind", N);
    dres.weave_perm = scratch_t<uint32_t>(c, "h_perm", N);
    dres.visible_bits = res->visible_bits ? scratch_t<uint32_t>(c, "h_bits", ((size_t)N + 31) / 32) : nullptr;
    dres.visible_count = scratch_t<uint32_t>(c, "h_vcount", D);
    dres.max_ts = res->max_ts ? scratch_t<uint64_t>(c, "h_maxts", D) : nullptr;
    dres.status = scratch_t<uint32_t>(c, "h_status", D);
    dres.yarn_perm = res->yarn_perm ? scratch_t<uint32_t>(c, "h_yarn", N) : nullptr;
    if ((!dev_inputs && (!did || !dca || !dk)) || !dres.weave_perm || !dres.visible_count ||
        !dres.status || (res->visible_bits && !dres.visible_bits) || (res->max_ts && !dres.max_ts) ||
        (res->yarn_perm && !dres.yarn_perm))
      return fail(c, "out of device memory (host-mode staging)");
    if (!dev_inputs) {
      // Pageable host memory: blocking copies (hipMemcpyAsync from/to pageable
      // memory is not reliably ordered by a later stream synchronize).
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (N) {
        HIPCHK(c, hipMemcpy(did, id, (size_t)N * 8, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(dca, cause, (size_t)N * 8, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(dk, kind, N, hipMemcpyHostToDevice));
      }
      id = did;
      cause = dca;
      kind = dk;
    }
  }
  if (weave_lists_dev_all(c, bt, id, cause, kind, &dres)) return -1;

  if (memspace == CW_MEM_HOST) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(res->weave_perm, dres.weave_perm, (size_t)N * 4, hipMemcpyDeviceToHost));
    if (res->visible_bits)
      HIPCHK(c, hipMemcpy(res->visible_bits, dres.visible_bits, ((size_t)N + 31) / 32 * 4,
                          hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->visible_count, dres.visible_count, D * 4, hipMemcpyDeviceToHost));
    if (res->max_ts)
      HIPCHK(c, hipMemcpy(res->max_ts, dres.max_ts, D * 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(res->status, dres.status, D * 4, hipMemcpyDeviceToHost));
    if (res->yarn_perm)
      HIPCHK(c, hipMemcpy(res->yarn_perm, dres.yarn_perm, (size_t)N * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipDeviceSynchronize());
    // documents with no nodes have no root
    for (uint64_t d = 0; d < D; d++)
      if (bt->doc_offsets[d + 1] == bt->doc_offsets[d]) res->status[d] |= CW_STATUS_ROOT;
  } else {
    // empty documents: set the ROOT bit on the device
    for (uint64_t d = 0; d < D; d++)
      if (bt->doc_offsets[d + 1] == bt->doc_offsets[d])
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)(res->status + d), CW_STATUS_ROOT, 1,
                                    c->stream));
    if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (c->prof) return collect_prof(c);
  return 0;
}

// --- K32: narrow keys (cw_weave_lists_k32) ---------------------------------------
// Ids and causes arrive as u32 (half the bytes over PCIe and in HBM for a batch
// whose packed ids fit 32 bits: config 2 needs 20) and are widened on the device
// into the K64 pipeline's scratch.  The top 16 K32 values are the reserved top
// of the K64 range (CW_NIL32 -> CW_NIL, CW_NIL32 - 1 -> the non-id cause, ...):
// they widen by sign extension, everything else by zero extension.
__global__ __launch_bounds__(256) void k_widen32(const uint32_t *__restrict__ id32,
                                                 const uint32_t *__restrict__ ca32, uint32_t n,
                                                 uint64_t *__restrict__ id,
                                                 uint64_t *__restrict__ ca) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t x = id32[i], c = ca32[i];
  id[i] = x >= CW_K32_RESERVED ? (uint64_t)(int64_t)(int32_t)x : (uint64_t)x;
  ca[i] = c >= CW_K32_RESERVED ? (uint64_t)(int64_t)(int32_t)c : (uint64_t)c;
}

__global__ __launch_bounds__(256) void k_narrow16(const uint32_t *__restrict__ src, uint32_t n,
                                                  uint16_t *__restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (uint16_t)src[i];
}

int weave_lists_k32_impl(cw_ctx *c, const cw_list_batch_k32 *b, cw_list_result *res, int memspace) {
  if (!b || !res) return fail(c, "null batch/result");
  if (!b->doc_offsets) return fail(c, "doc_offsets is required (host memory)");
  if (memspace != CW_MEM_HOST && memspace != CW_MEM_DEVICE) return fail(c, "bad memspace");
  const uint64_t D = b->n_docs, N64 = b->doc_offsets[D];
  if (N64 >= 0xFFFFFFFFull) return fail(c, "batch too large: N=%llu (limit 2^32-1)",
                                        (unsigned long long)N64);
  const uint32_t N = (uint32_t)N64;
  const size_t Ns = std::max<uint32_t>(N, 1);
  const uint32_t *id32 = b->id_key, *ca32 = b->cause_key;
  const uint8_t *kind = b->kind;
  if (N && (!id32 || !ca32 || !kind)) return fail(c, "null input arrays");
  HIPCHK(c, hipSetDevice(c->device));
  uint64_t *wid = scratch_t<uint64_t>(c, "k32_id", Ns), *wca = scratch_t<uint64_t>(c, "k32_cause", Ns);
  if (!wid || !wca) return fail(c, "out of device memory (k32)");
  if (memspace == CW_MEM_HOST && N) {
    uint32_t *d32 = scratch_t<uint32_t>(c, "k32_h", 2 * Ns);
    uint8_t *dk = scratch_t<uint8_t>(c, "h_kind", Ns);
    if (!d32 || !dk) return fail(c, "out of device memory (k32 staging)");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(d32, id32, (size_t)N * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d32 + Ns, ca32, (size_t)N * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(dk, kind, N, hipMemcpyHostToDevice));
    id32 = d32;
    ca32 = d32 + Ns;
    kind = dk;
  }
  if (N) {
    Launch L(c, "widen32", (double)N * (4 + 4 + 8 + 8));
    hipLaunchKernelGGL(k_widen32, dim3((N + 255) / 256), dim3(256), 0, c->stream, id32, ca32, N, wid,
                       wca);
  }
  if (check_launch(c, "widen32")) return -1;
  cw_list_batch wb{};
  wb.n_docs = D;
  wb.doc_offsets = b->doc_offsets;
  wb.id_key = wid;
  wb.cause_key = wca;
  wb.kind = kind;
  wb.key_bits = b->key_bits;
  wb.ts_shift = b->ts_shift;
  wb.site_shift = b->site_shift;
  wb.site_bits = b->site_bits;
  if (!b->perm16) return weave_lists_impl(c, &wb, res, memspace, true);
  // 16-bit weave_perm: documents below 2^16 nodes, the weave into scratch, narrowed
  if (memspace != CW_MEM_DEVICE) return fail(c, "perm16 needs device memory");
  for (uint64_t d = 0; d < D; d++)
    if (b->doc_offsets[d + 1] - b->doc_offsets[d] > 0xFFFFull)
      return fail(c, "perm16: document %llu has more than 65535 nodes", (unsigned long long)d);
  cw_list_result r32 = *res;
  r32.weave_perm = scratch_t<uint32_t>(c, "k32_perm", Ns);
  if (!r32.weave_perm || !res->weave_perm) return fail(c, "out of device memory (perm16)");
  if (weave_lists_impl(c, &wb, &r32, memspace, true)) return -1;
  if (N) {
    Launch L(c, "narrow16", (double)N * 6);
    hipLaunchKernelGGL(k_narrow16, dim3((N + 255) / 256), dim3(256), 0, c->stream, r32.weave_perm, N,
                       reinterpret_cast<uint16_t *>(res->weave_perm));
  }
  if (check_launch(c, "narrow16")) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

// --- building blocks of the distributed giant list (cause_amd/giant.py) ---------
// Gather dst[i] = src[idx[i]].
template <typename E>
__global__ __launch_bounds__(256) void k_gather(const E *__restrict__ src,
                                                const uint32_t *__restrict__ idx, uint64_t m,
                                                E *__restrict__ dst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) dst[i] = src[idx[i]];
}

// A stable partition by bucket for few buckets (<= PB_MAX: the exchange of
// a distributed round has W + 1), with no sort and no host tables: count per
// block and bucket, one scan (bucket-major), scatter in order.  The sizes of
// the buckets land in device memory, so the caller need not wait.
constexpr uint32_t PB_MAX = 16, PB_ITEMS = 8, PB_NT = 256, PB_CHUNK = PB_ITEMS * PB_NT;

__device__ __forceinline__ uint32_t pb_bucket(const uint64_t *__restrict__ split, uint32_t ns,
                                              uint64_t x) {
  uint32_t lo = 0, hi = ns;  // first splitter > x
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (split[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(PB_NT) void k_pb_count(const uint64_t *__restrict__ keys, uint32_t m,
                                                    const uint64_t *__restrict__ split, uint32_t ns,
                                                    uint32_t *__restrict__ bcnt, uint32_t nblk) {
  __shared__ uint32_t c[PB_MAX];
  if (threadIdx.x < PB_MAX) c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i0 = blockIdx.x * PB_CHUNK + threadIdx.x * PB_ITEMS;
#pragma unroll
  for (uint32_t u = 0; u < PB_ITEMS; u++)
    if (i0 + u < m) atomicAdd(&c[pb_bucket(split, ns, keys[i0 + u])], 1u);
  __syncthreads();
  if (threadIdx.x <= ns) bcnt[threadIdx.x * nblk + blockIdx.x] = c[threadIdx.x];
}

// exclusive scan of the (ns + 1) x nblk counts, bucket-major, in place; the
// bucket sizes into counts[0..ns]
__global__ __launch_bounds__(1024) void k_pb_scan(uint32_t *__restrict__ bcnt, uint32_t nblk,
                                                  uint32_t ns, unsigned long long *__restrict__ counts) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, T = (ns + 1) * nblk;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < T; c0 += 1024) {
    const uint32_t t = c0 + threadIdx.x;
    const uint32_t v = t < T ? bcnt[t] : 0;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre += wsum[w];
    if (t < T) bcnt[t] = pre + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + inc;
    __syncthreads();
  }
  // bucket b spans [bcnt[b * nblk], bcnt[(b + 1) * nblk]) (the last ends at the total)
  if (threadIdx.x <= ns) {
    const uint32_t b = threadIdx.x;
    const uint32_t lo = bcnt[b * nblk], hi = b < ns ? bcnt[(b + 1) * nblk] : carry;
    counts[b] = hi - lo;
  }
}

__global__ __launch_bounds__(PB_NT) void k_pb_scatter(const uint64_t *__restrict__ keys, uint32_t m,
                                                      const uint64_t *__restrict__ split, uint32_t ns,
                                                      const uint32_t *__restrict__ boff,
                                                      uint32_t nblk, uint32_t *__restrict__ perm) {
  __shared__ uint32_t wtot[PB_NT / 64];
  const uint32_t i0 = blockIdx.x * PB_CHUNK + threadIdx.x * PB_ITEMS;
  uint32_t bk[PB_ITEMS];
#pragma unroll
  for (uint32_t u = 0; u < PB_ITEMS; u++)
    bk[u] = i0 + u < m ? pb_bucket(split, ns, keys[i0 + u]) : 0xFFFFFFFFu;
  for (uint32_t b = 0; b <= ns; b++) {
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t u = 0; u < PB_ITEMS; u++) mine += bk[u] == b ? 1u : 0u;
    uint32_t at = boff[b * nblk + blockIdx.x] + block_exscan<PB_NT>(mine, wtot, nullptr);
#pragma unroll
    for (uint32_t u = 0; u < PB_ITEMS; u++)
      if (bk[u] == b) perm[at++] = i0 + u;
  }
}

// Bucket of each key among ns ascending splitters (number of splitters <= key)
// as a sort key, and the bucket sizes.
__global__ __launch_bounds__(256) void k_bucket(const uint64_t *__restrict__ keys, uint64_t m,
                                                const uint64_t *__restrict__ split, uint32_t ns,
                                                uint64_t *__restrict__ bucket,
                                                unsigned long long *__restrict__ counts) {
  // grid-stride over a few thousand blocks: one global atomic per block and
  // bucket (a block per 256 keys would serialise on the count words)
  __shared__ unsigned long long cnt[1024];
  for (uint32_t j = threadIdx.x; j <= ns; j += blockDim.x) cnt[j] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < m; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    uint32_t my = 0xFFFFFFFFu;
    if (i < m) {
      const uint64_t x = keys[i];
      uint32_t lo = 0, hi = ns;  // first splitter > x
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (split[mid] <= x) lo = mid + 1; else hi = mid;
      }
      bucket[i] = lo;
      my = lo;
    }
    // few buckets: a ballot per bucket (one LDS atomic per wave and bucket)
    if (ns < 64) {
      for (uint32_t b = 0; b <= ns; b++) {
        const uint64_t bal = __ballot(my == b);
        if ((threadIdx.x & 63) == 0 && bal) atomicAdd(&cnt[b], (unsigned long long)__popcll(bal));
      }
    } else if (i < m) {
      atomicAdd(&cnt[my], 1ull);
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j <= ns; j += blockDim.x)
    if (cnt[j]) atomicAdd(&counts[j], cnt[j]);
}

// Scatter dst[idx[i]] = src[i] (idx a permutation).
__global__ __launch_bounds__(256) void k_scatter32(const uint32_t *__restrict__ src,
                                                   const uint32_t *__restrict__ idx, uint64_t m,
                                                   uint32_t *__restrict__ dst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) dst[idx[i]] = src[i];
}

// Index of each query among n sorted unique keys (bucket index from
// k_index_flat), or CW_NOT_FOUND.
__global__ __launch_bounds__(256) void k_lookup(const uint64_t *__restrict__ skey, uint32_t n,
                                                const uint32_t *__restrict__ bkt,
                                                const uint64_t *__restrict__ q, uint64_t m,
                                                uint32_t base, uint32_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t kmin = skey[0], kmax = skey[n - 1], x = q[i];
  uint32_t r = x == CW_NIL ? CW_NIL_RANK : CW_NOT_FOUND;
  if (x >= kmin && x <= kmax && x != CW_NIL) {
    const uint32_t sh = bucket_shift(kmax - kmin, n), h = (uint32_t)((x - kmin) >> sh);
    uint32_t lo = bkt[h], hi = bkt[h + 1];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (skey[mid] < x) lo = mid + 1; else hi = mid;
    }
    if (lo < n && skey[lo] == x) r = base + lo;
  }
  out[i] = r;
}

// Root at rank 0 only, causes older than their node (s/insert's checks,
// shared.cljc:163-178) for a list handed over in rank order.
__global__ __launch_bounds__(256) void k_ranked_check(const uint32_t *__restrict__ par,
                                                      const uint8_t *__restrict__ kind, uint32_t n,
                                                      uint32_t *__restrict__ status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st = 0;
  if (r < n) {
    const bool root = (kind[r] & KIND_ROOT) != 0;
    if ((r == 0) != root) st |= CW_STATUS_ROOT;
    if (r > 0 && par[r] >= r)
      st |= par[r] >= CW_NIL_RANK ? CW_STATUS_ORPHAN : CW_STATUS_NON_LAMPORT;
  }
  if (__syncthreads_or(st != 0)) {
    if (st) atomicOr(status, st);
  }
}

int sort_keys_impl(cw_ctx *c, const uint64_t *keys, uint64_t n64, uint32_t key_bits,
                   uint64_t *keys_out, uint32_t *idx_out) {
  if (n64 == 0) return 0;
  if (!keys || !keys_out || !idx_out) return fail(c, "null array");
  if (n64 >= 0xFFFFFFFFull) return fail(c, "too many keys: %llu", (unsigned long long)n64);
  const uint32_t n = (uint32_t)n64;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t off[2] = {0, n64};
  if (ensure_tables(c, 1, off)) return -1;
  if (key_bits == 0 && find_key_bits(c, keys, n, &key_bits)) return -1;
  if (key_bits > 64) key_bits = 64;
  uint64_t *kB = scratch_t<uint64_t>(c, "skB", n);
  uint32_t *vB = scratch_t<uint32_t>(c, "svB", n);
  if (!kB || !vB) return fail(c, "out of device memory (sort)");
  uint64_t *ko;
  uint32_t *vo;
  if (radix_sort<uint64_t>(c, "ksort", keys, nullptr, keys_out, idx_out, kB, vB, key_bits, 0, n,
                           &ko, &vo))
    return -1;
  if (ko != keys_out) {
    HIPCHK(c, hipMemcpyAsync(keys_out, ko, (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(idx_out, vo, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  return 0;
}

// The same for 32-bit keys (the distributed tree's group keys).
int sort_keys32_impl(cw_ctx *c, const uint32_t *keys, uint64_t n64, uint32_t key_bits,
                     uint32_t *keys_out, uint32_t *idx_out) {
  if (n64 == 0) return 0;
  if (!keys || !keys_out || !idx_out) return fail(c, "null array");
  if (n64 >= 0xFFFFFFFFull) return fail(c, "too many keys: %llu", (unsigned long long)n64);
  const uint32_t n = (uint32_t)n64;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t off[2] = {0, n64};
  if (ensure_tables(c, 1, off)) return -1;
  if (key_bits == 0 || key_bits > 32) key_bits = 32;
  uint32_t *kB = scratch_t<uint32_t>(c, "k32_kB", n), *vB = scratch_t<uint32_t>(c, "k32_vB", n);
  if (!kB || !vB) return fail(c, "out of device memory (sort)");
  uint32_t *ko, *vo;
  if (radix_sort<uint32_t>(c, "ksort32", keys, nullptr, keys_out, idx_out, kB, vB, key_bits, 0, n,
                           &ko, &vo))
    return -1;
  if (ko != keys_out) {
    HIPCHK(c, hipMemcpyAsync(keys_out, ko, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(idx_out, vo, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  return 0;
}

int lookup_keys_impl(cw_ctx *c, const uint64_t *sorted, uint64_t n64, const uint64_t *q,
                     uint64_t m, uint32_t base, uint32_t *out, uint32_t *status) {
  if (m == 0 && (!status || n64 == 0)) return 0;
  if ((m && (!q || !out)) || (n64 && !sorted)) return fail(c, "null array");
  if (n64 >= 0xFFFFFFFFull) return fail(c, "too many keys: %llu", (unsigned long long)n64);
  HIPCHK(c, hipSetDevice(c->device));
  if (n64 == 0) {
    HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)out, CW_NOT_FOUND, m, c->stream));
    return 0;
  }
  const uint32_t n = (uint32_t)n64;
  uint32_t *bkt = scratch_t<uint32_t>(c, "lk_bkt", (size_t)std::max(n >> 2, 1u) + 2);
  // repeated ids (the same id held by two ranks meets at its owner) go to the
  // caller's status word, or to a scratch word nobody reads
  uint32_t *st = status ? status : scratch_t<uint32_t>(c, "lk_status", 1);
  if (!bkt || !st) return fail(c, "out of device memory (lookup)");
  if (!status) HIPCHK(c, hipMemsetAsync(st, 0, 4, c->stream));
  {
    Launch L(c, "lk_index", (double)n * 8);
    hipLaunchKernelGGL(k_index_flat, dim3((n + 255) / 256), dim3(256), 0, c->stream, sorted, n, bkt, st);
  }
  if (check_launch(c, "lk_index")) return -1;
  if (m == 0) return 0;
  {
    Launch L(c, "lookup", (double)m * (8 + 4 + 8 + 8));
    hipLaunchKernelGGL(k_lookup, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, c->stream, sorted,
                       n, bkt, q, m, base, out);
  }
  return check_launch(c, "lookup");
}

int gather_impl(cw_ctx *c, const void *src, const uint32_t *idx, uint64_t m, uint32_t es,
                void *dst) {
  if (m == 0) return 0;
  if (!src || !idx || !dst) return fail(c, "null array");
  HIPCHK(c, hipSetDevice(c->device));
  const dim3 G((uint32_t)((m + 255) / 256)), B(256);
  Launch L(c, "gather", (double)m * (4 + 2 * es));
  if (es == 8)
    hipLaunchKernelGGL(k_gather<uint64_t>, G, B, 0, c->stream, (const uint64_t *)src, idx, m, (uint64_t *)dst);
  else if (es == 4)
    hipLaunchKernelGGL(k_gather<uint32_t>, G, B, 0, c->stream, (const uint32_t *)src, idx, m, (uint32_t *)dst);
  else if (es == 1)
    hipLaunchKernelGGL(k_gather<uint8_t>, G, B, 0, c->stream, (const uint8_t *)src, idx, m, (uint8_t *)dst);
  else if (es == 16)
    hipLaunchKernelGGL(k_gather<uint4>, G, B, 0, c->stream, (const uint4 *)src, idx, m, (uint4 *)dst);
  else
    return fail(c, "gather: element size %u (1, 4, 8 or 16)", es);
  return check_launch(c, "gather");
}

// counts: host memory (the call waits for it), or device memory when
// dev_counts (nothing waits: the caller's next collective reads it in order)
int partition_keys_impl(cw_ctx *c, const uint64_t *keys, uint64_t m64, const uint64_t *split,
                        uint32_t ns, uint32_t *perm, uint64_t *counts, bool dev_counts = false) {
  if (ns > 1023) return fail(c, "partition: at most 1023 splitters");
  if (!counts) return fail(c, "null counts");
  if (m64 == 0) {
    if (dev_counts) HIPCHK(c, hipMemsetAsync(counts, 0, (size_t)(ns + 1) * 8, c->stream));
    else memset(counts, 0, (size_t)(ns + 1) * 8);
    return 0;
  }
  if (!keys || !perm || (ns && !split)) return fail(c, "null array");
  if (m64 >= 0xFFFFFFFFull) return fail(c, "too many keys: %llu", (unsigned long long)m64);
  const uint32_t m = (uint32_t)m64;
  HIPCHK(c, hipSetDevice(c->device));
  if (ns + 1 <= PB_MAX) {  // few buckets: counts, one scan, an ordered scatter
    const uint32_t nblk = (m + PB_CHUNK - 1) / PB_CHUNK;
    uint32_t *bcnt = scratch_t<uint32_t>(c, "pb_cnt", (size_t)(ns + 1) * nblk);
    unsigned long long *dc = dev_counts ? reinterpret_cast<unsigned long long *>(counts)
                                        : scratch_t<unsigned long long>(c, "pt_counts", ns + 1);
    if (!bcnt || !dc) return fail(c, "out of device memory (partition)");
    {
      Launch L(c, "bucket", (double)m * 8 * 2 + (double)m * 4);
      hipLaunchKernelGGL(k_pb_count, dim3(nblk), dim3(PB_NT), 0, c->stream, keys, m, split, ns, bcnt,
                         nblk);
      hipLaunchKernelGGL(k_pb_scan, dim3(1), dim3(1024), 0, c->stream, bcnt, nblk, ns, dc);
      hipLaunchKernelGGL(k_pb_scatter, dim3(nblk), dim3(PB_NT), 0, c->stream, keys, m, split, ns, bcnt,
                         nblk, perm);
    }
    if (check_launch(c, "bucket")) return -1;
    if (dev_counts) return 0;
    HIPCHK(c, hipMemcpyAsync(counts, dc, (size_t)(ns + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
  }
  const uint64_t off[2] = {0, m64};
  if (ensure_tables(c, 1, off)) return -1;
  uint64_t *bk = scratch_t<uint64_t>(c, "pt_bucket", m), *kA = scratch_t<uint64_t>(c, "skA", m);
  uint64_t *kB = scratch_t<uint64_t>(c, "skB", m);
  uint32_t *vB = scratch_t<uint32_t>(c, "svB", m);
  unsigned long long *dc = scratch_t<unsigned long long>(c, "pt_counts", ns + 1);
  if (!bk || !kA || !kB || !vB || !dc) return fail(c, "out of device memory (partition)");
  HIPCHK(c, hipMemsetAsync(dc, 0, (size_t)(ns + 1) * 8, c->stream));
  {
    Launch L(c, "bucket", (double)m * 16);
    hipLaunchKernelGGL(k_bucket, dim3(std::min<uint32_t>((m + 255) / 256, 4096)), dim3(256), 0,
                       c->stream, keys, m, split, ns, bk, dc);
  }
  if (check_launch(c, "bucket")) return -1;
  uint64_t *ko;
  uint32_t *vo;
  if (radix_sort<uint64_t>(c, "psort", bk, nullptr, kA, perm, kB, vB, std::max(1u, ceil_log2(ns + 1)),
                           0, m, &ko, &vo))
    return -1;
  if (vo != perm) HIPCHK(c, hipMemcpyAsync(perm, vo, (size_t)m * 4, hipMemcpyDeviceToDevice, c->stream));
  if (dev_counts) {
    HIPCHK(c, hipMemcpyAsync(counts, dc, (size_t)(ns + 1) * 8, hipMemcpyDeviceToDevice, c->stream));
    return 0;
  }
  HIPCHK(c, hipMemcpyAsync(counts, dc, (size_t)(ns + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

int scatter_impl(cw_ctx *c, const uint32_t *src, const uint32_t *idx, uint64_t m, uint32_t *dst) {
  if (m == 0) return 0;
  if (!src || !idx || !dst) return fail(c, "null array");
  HIPCHK(c, hipSetDevice(c->device));
  Launch L(c, "scatter", (double)m * 12);
  hipLaunchKernelGGL(k_scatter32, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, c->stream, src, idx,
                     m, dst);
  return check_launch(c, "scatter");
}

int weave_ranked_impl(cw_ctx *c, const cw_ranked_list *in, cw_list_result *out) {
  if (!in || !out) return fail(c, "null list/result");
  if (!out->weave_perm || !out->visible_count || !out->status)
    return fail(c, "weave_perm, visible_count and status are required");
  if (out->yarn_perm || out->max_ts) return fail(c, "yarn_perm / max_ts: not produced from ranks");
  const uint64_t n64 = in->n;
  if (n64 == 0 || n64 >= SUCCW_END) return fail(c, "list size %llu (1 .. 2^31-2)", (unsigned long long)n64);
  if (!in->par || !in->kind) return fail(c, "null input arrays");
  const uint32_t n = (uint32_t)n64;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t off[2] = {0, n64};
  if (ensure_tables(c, 1, off, true)) return -1;
  HIPCHK(c, hipMemsetAsync(out->status, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(out->visible_count, 0, 4, c->stream));
  if (out->visible_bits)
    HIPCHK(c, hipMemsetAsync(out->visible_bits, 0, ((size_t)n + 31) / 32 * 4, c->stream));
  hipLaunchKernelGGL(k_ranked_check, dim3((n + 255) / 256), dim3(256), 0, c->stream, in->par,
                     in->kind, n, out->status);
  if (check_launch(c, "ranked_check")) return -1;
  if (weave_tail(c, 1, n, true, in->par, in->kind, in->val, nullptr, nullptr, 0, out)) return -1;
  {  // flagged (orphan / non-Lamport / root): the literal fold (exact.hip)
    if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
    HIPCHK(c, hipMemcpyAsync(c->pin_small, out->status, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((c->pin_small[0] & X_MASK) && !(c->pin_small[0] & CW_STATUS_DUP) && exact_ranked(c, in, out))
      return -1;
  }
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->prof) return collect_prof(c);
  return 0;
}

// Key weaves of at most this many documents / nodes go through one list call
// (keeps every launch grid of the list pipeline inside the dispatch limits).
constexpr uint64_t MAP_CHUNK_DOCS = 1ull << 20, MAP_CHUNK_NODES = 1ull << 30;

int weave_maps_impl(cw_ctx *c, const cw_map_batch *bt, cw_map_result *res, int memspace) {
  if (!bt || !res) return fail(c, "null batch/result");
  if (memspace != CW_MEM_HOST && memspace != CW_MEM_DEVICE) return fail(c, "bad memspace");
  const bool dev = memspace == CW_MEM_DEVICE;
  const uint64_t D = bt->n_colls;
  if (!bt->coll_offsets) return fail(c, "coll_offsets is required (host memory)");
  if (bt->coll_offsets[0] != 0) return fail(c, "coll_offsets[0] must be 0");
  const uint64_t N64 = bt->coll_offsets[D];
  // key weaves add one root each: N + S <= 2N must stay below 2^32
  if (N64 >= 0x7FFFFFFFull) return fail(c, "batch too large: N=%llu (limit 2^31-1)",
                                        (unsigned long long)N64);
  // the layout of the previous call (validated then, its pack table cached):
  // one compare instead of the checks (10^6 collections: ~1 ms of host time
  // a call otherwise).  For device memory that compare runs while the map
  // kernel does (c->mpack.verify, mappack.hip): the cached table is taken when
  // the size and a few offsets agree, and a layout that then differs is woven
  // again from a fresh table (every output rewritten).
  c->mpack.verify = false;
  if (dev && c->map_fused && c->mpack.ok && c->mpack.off.size() == D + 1 && D > 4096 &&
      c->mpack.off[D] == bt->coll_offsets[D] && c->mpack.off[D / 2] == bt->coll_offsets[D / 2] &&
      c->mpack.off[D / 3] == bt->coll_offsets[D / 3]) {
    c->mpack.same = true;
    c->mpack.verify = true;
  } else {
    c->mpack.same = c->mpack.off.size() == D + 1 &&
                    memcmp(c->mpack.off.data(), bt->coll_offsets, (D + 1) * 8) == 0;
  }
  auto check_layout = [&]() -> int {
    const uint64_t *o = bt->coll_offsets;
    uint64_t back = 0, big = 0, mx = 0;
    for (uint64_t d = 0; d < D; d++) {  // branch-free: vectorizes
      back |= (uint64_t)(o[d + 1] < o[d]);
      big |= (uint64_t)(o[d + 1] - o[d] >= LINK_IDX - 1);
      mx = std::max<uint64_t>(mx, o[d + 1] - o[d]);
    }
    c->mpack.maxcoll = mx;
    if (back) return fail(c, "coll_offsets not monotone");
    if (big)
      for (uint64_t d = 0; d < D; d++)
        if (o[d + 1] - o[d] >= LINK_IDX - 1) return fail(c, "collection %llu too large", (unsigned long long)d);
    return 0;
  };
  if (!c->mpack.same && check_layout()) return -1;
  if (!res->seg_offsets || !res->seg_coll || !res->seg_key || !res->seg_active ||
      !res->seg_perm || !res->status)
    return fail(c, "every cw_map_result array is required");
  if (bt->token_bits == 0 || bt->token_bits > 62) return fail(c, "token_bits must be 1..62");
  const uint32_t N = (uint32_t)N64;
  HIPCHK(c, hipSetDevice(c->device));
  res->n_segs = 0;
  if (N == 0) {
    if (dev) {
      HIPCHK(c, hipMemsetAsync(res->status, 0, D * 4, c->stream));
      HIPCHK(c, hipMemsetAsync(res->seg_offsets, 0, 8, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    } else {
      memset(res->status, 0, D * 4);
      res->seg_offsets[0] = 0;
    }
    return 0;
  }
  if (!bt->id_key || !bt->cause || !bt->cause_is_id || !bt->kind)
    return fail(c, "null input arrays");

  const uint64_t *id = dev ? bt->id_key : scratch_t<uint64_t>(c, "m_id", N);
  const uint64_t *cause = dev ? bt->cause : scratch_t<uint64_t>(c, "m_cause", N);
  const uint8_t *cis = dev ? bt->cause_is_id : scratch_t<uint8_t>(c, "m_cis", N);
  const uint8_t *kind = dev ? bt->kind : scratch_t<uint8_t>(c, "m_kind", N);
  if (!id || !cause || !cis || !kind) return fail(c, "out of device memory (maps, N=%u)", N);
  if (!dev) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy((void *)id, bt->id_key, (size_t)N * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy((void *)cause, bt->cause, (size_t)N * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy((void *)cis, bt->cause_is_id, N, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy((void *)kind, bt->kind, N, hipMemcpyHostToDevice));
  }
  if (c->map_fused) {  // small collections: one kernel (mappack.hip)
    int rc = weave_maps_packed(c, bt, res, dev, id, cause, cis, kind);
    if (rc == 2) {  // the speculated layout was not the cached one: check it, weave again
      c->mpack.same = false;
      c->mpack.verify = false;
      if (check_layout()) return -1;
      rc = weave_maps_packed(c, bt, res, dev, id, cause, cis, kind);
    }
    if (rc <= 0) return rc;
  }
  // significant bits of the ids and of the causes (id keys, SURVEY F8c, are
  // cause ids, which may lie outside the collection): one reduction, one readback
  uint32_t key_bits = bt->key_bits, cause_bits = 0;
  {
    unsigned long long *red = scratch_t<unsigned long long>(c, "red2", 2);
    if (!red) return fail(c, "out of device memory (red)");
    HIPCHK(c, hipMemsetAsync(red, 0, 16, c->stream));
    hipLaunchKernelGGL(k_or_reduce2, dim3(1024), dim3(256), 0, c->stream, id, cause, N, red);
    if (check_launch(c, "or_reduce2")) return -1;
    if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
    HIPCHK(c, hipMemcpyAsync(c->pin_small, red, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t *v = reinterpret_cast<const uint64_t *>(c->pin_small);
    const uint32_t ib = v[0] ? 64 - __builtin_clzll(v[0]) : 1, cb = v[1] ? 64 - __builtin_clzll(v[1]) : 1;
    if (key_bits == 0) key_bits = ib;
    cause_bits = cb;
  }
  if (key_bits > 62 || cause_bits > 62)
    return fail(c, "map ids need %u bits (limit 62)", std::max(key_bits, cause_bits));

  // the general path: collection tables (id sort, key resolution and key
  // grouping run per collection), then every key weave through a list weave
  if (ensure_tables(c, D, bt->coll_offsets)) return -1;
  auto &t = c->tab;
  const uint32_t T = t.T;
  uint32_t *status = scratch_t<uint32_t>(c, "m_status", D);
  uint64_t *skA = scratch_t<uint64_t>(c, "skA", N), *skB = scratch_t<uint64_t>(c, "skB", N);
  uint32_t *svA = scratch_t<uint32_t>(c, "svA", N), *svB = scratch_t<uint32_t>(c, "svB", N);
  uint64_t *segk = scratch_t<uint64_t>(c, "m_segk", N);
  uint32_t *mpar = scratch_t<uint32_t>(c, "m_mpar", N);
  uint8_t *mkind = scratch_t<uint8_t>(c, "m_mkind", N);
  uint64_t *kA = scratch_t<uint64_t>(c, "m_kA", N), *kB = scratch_t<uint64_t>(c, "m_kB", N);
  uint32_t *vA = scratch_t<uint32_t>(c, "m_vA", N), *vB = scratch_t<uint32_t>(c, "m_vB", N);
  uint32_t *tcnt = scratch_t<uint32_t>(c, "m_tcnt", T), *tsb = scratch_t<uint32_t>(c, "m_tsb", T);
  uint32_t *seg_of = scratch_t<uint32_t>(c, "m_segof", N);
  if (!status || !skA || !skB || !svA || !svB || !segk ||
      !mpar || !mkind || !kA || !kB || !vA || !vB || !tcnt || !tsb || !seg_of)
    return fail(c, "out of device memory (maps, N=%u)", N);
  if (!grid_ok(T, SORT_THREADS) || !grid_ok(D, 1024)) return fail(c, "batch too large for one dispatch");
  HIPCHK(c, hipMemsetAsync(status, 0, D * 4, c->stream));
  const uint32_t W = std::max(std::max(bt->token_bits, key_bits), cause_bits);

  // 1. (sort (::s/nodes ct)) per collection -- map.cljc:28
  uint64_t *skey;
  uint32_t *sval;
  if (radix_sort<uint64_t>(c, "m_idsort", id, nullptr, skA, svA, skB, svB, key_bits, 0, N, &skey,
                           &sval))
    return -1;
  // 2. key and cause-in-weave per node -- map.cljc:31-37
  {
    Launch L(c, "m_key", (double)N * (8 + 4 + 8 + 1 + 1 + 8 + 4 + 1) + (double)N * 2 * 8);
    hipLaunchKernelGGL(k_map_key, dim3(T), dim3(256), 0, c->stream, skey, sval, cause, cis, kind,
                       dev_tab(c, "t_tile_start"), dev_tab(c, "t_tile_doc"),
                       dev_tab(c, "t_doc_off"), bt->token_bits, W, segk, mpar, mkind, status);
  }
  if (check_launch(c, "m_key")) return -1;
  // 3. stable grouping by key (id order kept inside a key)
  uint64_t *ks;
  uint32_t *rank_s;
  if (radix_sort<uint64_t>(c, "m_keysort", segk, nullptr, kA, vA, kB, vB, W + 2, 0, N, &ks,
                           &rank_s))
    return -1;
  {
    Launch L(c, "m_segcount", (double)N * 8);
    hipLaunchKernelGGL(k_seg_count, dim3(T), dim3(256), 0, c->stream, ks,
                       dev_tab(c, "t_tile_start"), dev_tab(c, "t_tile_doc"),
                       dev_tab(c, "t_doc_off"), tcnt);
  }
  if (check_launch(c, "m_segcount")) return -1;
  // key weaves before each tile (device scan) and their number S (one readback)
  uint32_t *chunk = scratch_t<uint32_t>(c, "m_chunk", (T + 1023) / 1024 + 1);
  uint32_t *small = scratch_t<uint32_t>(c, "m_small", 4);
  if (!chunk || !small) return fail(c, "out of device memory (maps scan)");
  if (!c->pin_small) HIPCHK(c, hipHostMalloc((void **)&c->pin_small, 64, hipHostMallocDefault));
  HIPCHK(c, hipMemsetAsync(small, 0, 16, c->stream));
  {
    const uint32_t nb = (T + 1023) / 1024;
    hipLaunchKernelGGL(k_scan_chunks, dim3(nb), dim3(1024), 0, c->stream, tcnt, T, tsb, chunk);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, c->stream, chunk, nb, small);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(1024), 0, c->stream, tsb, T, chunk);
  }
  if (check_launch(c, "m_scan")) return -1;
  HIPCHK(c, hipMemcpyAsync(c->pin_small, small, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t S = c->pin_small[0];
  if (S > res->cap_segs)
    return fail(c, "cap_segs too small: %llu key weaves", (unsigned long long)S);
  uint32_t *seg_start = scratch_t<uint32_t>(c, "m_segstart", S + 1);
  uint32_t *seg_coll = scratch_t<uint32_t>(c, "m_segcoll", S);
  uint64_t *seg_key = scratch_t<uint64_t>(c, "m_segkey", S);
  const size_t NL = (size_t)N + S;
  uint64_t *lid = scratch_t<uint64_t>(c, "m_lid", NL), *lcause = scratch_t<uint64_t>(c, "m_lcause", NL);
  uint8_t *lkind = scratch_t<uint8_t>(c, "m_lkind", NL);
  uint32_t *lmap = scratch_t<uint32_t>(c, "m_lmap", NL), *lperm = scratch_t<uint32_t>(c, "m_lperm", NL);
  uint32_t *lvc = scratch_t<uint32_t>(c, "m_lvc", S), *lst = scratch_t<uint32_t>(c, "m_lst", S);
  uint64_t *seg_off = scratch_t<uint64_t>(c, "m_segoff", S + 1);
  uint32_t *seg_perm = scratch_t<uint32_t>(c, "m_segperm", NL);
  int64_t *seg_act = scratch_t<int64_t>(c, "m_segact", S);
  if (!seg_start || !seg_coll || !seg_key || !lid || !lcause || !lkind || !lmap || !lperm || !lvc ||
      !lst || !seg_off || !seg_perm || !seg_act)
    return fail(c, "out of device memory (maps, S=%llu)", (unsigned long long)S);
  {
    Launch L(c, "m_segmark", (double)N * (8 + 4) + (double)S * (4 + 4 + 8));
    hipLaunchKernelGGL(k_seg_mark, dim3(T), dim3(256), 0, c->stream, ks,
                       dev_tab(c, "t_tile_start"), dev_tab(c, "t_tile_doc"),
                       dev_tab(c, "t_doc_off"), tsb, W, seg_of, seg_start, seg_coll, seg_key);
  }
  if (check_launch(c, "m_segmark")) return -1;
  {
    Launch L(c, "m_segbuild", (double)N * (4 + 4 + 4 + 8 + 4 + 8 + 1 + 8 + 8 + 1 + 4));
    hipLaunchKernelGGL(k_seg_build, dim3((N + 255) / 256), dim3(256), 0, c->stream, skey, sval,
                       cause, mpar, mkind, rank_s, seg_of, seg_coll, dev_tab(c, "t_doc_off"), N, lid,
                       lcause, lkind, lmap);
  }
  if (check_launch(c, "m_segbuild")) return -1;
  {
    Launch L(c, "m_segroots", (double)S * 25);
    hipLaunchKernelGGL(k_seg_roots, dim3((uint32_t)((S + 255) / 256)), dim3(256), 0, c->stream,
                       seg_start, (uint32_t)S, lid, lcause, lkind, lmap);
  }
  if (check_launch(c, "m_segroots")) return -1;

  // key weave s = list document [seg_start[s] + s, seg_start[s+1] + s + 1)
  {
    Launch L(c, "m_segoff", (double)S * 12);
    hipLaunchKernelGGL(k_seg_off, dim3((uint32_t)std::min<uint64_t>((S + 256) / 256, 2048)), dim3(256),
                       0, c->stream, seg_start, (uint32_t)S, N, seg_off, small + 1);
  }
  if (check_launch(c, "m_segoff")) return -1;
  HIPCHK(c, hipMemcpyAsync(c->pin_small, small + 1, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t max_len = c->pin_small[0];
  std::vector<uint64_t> loff;  // host copy, only for the list pipeline's chunks
  if (!(c->map_small && max_len <= SMALL_MAX)) {
    loff.resize(S + 1);
    HIPCHK(c, hipMemcpy(loff.data(), seg_off, (S + 1) * 8, hipMemcpyDeviceToHost));
  }

  // 4. every key weave is a list weave -- (s/weave-node key-weave ...), map.cljc:40-41
  if (c->map_small && max_len <= SMALL_MAX) {
    // key weaves are tiny (config 4: a few nodes per key): one wave each
    Launch L(c, "m_small", (double)NL * (8 + 8 + 1 + 4) + (double)S * 12);
    hipLaunchKernelGGL(k_small_weave, dim3((uint32_t)((NL + SMALL_CHUNK - 1) / SMALL_CHUNK)),
                       dim3(SMALL_SLOTS), 0, c->stream, seg_off, (uint32_t)S, lid, lcause, lkind,
                       lperm, lst);
  }
  if (check_launch(c, "m_small")) return -1;
  std::vector<uint64_t> rel;
  for (uint64_t s0 = (c->map_small && max_len <= SMALL_MAX) ? S : 0; s0 < S;) {
    uint64_t s1 = s0 + 1;
    while (s1 < S && s1 - s0 < MAP_CHUNK_DOCS && loff[s1 + 1] - loff[s0] <= MAP_CHUNK_NODES) s1++;
    rel.resize(s1 - s0 + 1);
    for (uint64_t sg = s0; sg <= s1; sg++) rel[sg - s0] = loff[sg] - loff[s0];
    if (ensure_tables(c, s1 - s0, rel.data())) return -1;
    cw_list_batch lb{};
    lb.n_docs = s1 - s0;
    lb.doc_offsets = rel.data();
    lb.key_bits = key_bits;
    cw_list_result lr{};
    lr.weave_perm = lperm + loff[s0];
    lr.visible_count = lvc + s0;
    lr.status = lst + s0;
    if (weave_lists_device(c, &lb, lid + loff[s0], lcause + loff[s0], lkind + loff[s0], &lr))
      return -1;
    s0 = s1;
  }
  // key weaves outside the fast weave's domain -- the nil key weave with its
  // appended orphans next to children of the root, a cause with a larger id
  // than its node (map.cljc:40-41 folds them whatever their causes) -- by the
  // literal fold (exact.hip), as the fused path's literal key weaves
  {
    HIPCHK(c, hipMemsetAsync(small, 0, 4, c->stream));
    hipLaunchKernelGGL(k_xcount_nonempty, dim3((uint32_t)((S + 255) / 256)), dim3(256), 0, c->stream,
                       lst, (uint32_t)S, small);
    if (check_launch(c, "m_xcount")) return -1;
    HIPCHK(c, hipMemcpyAsync(c->pin_small, small, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->pin_small[0]) {
      if (loff.empty()) {
        loff.resize(S + 1);
        HIPCHK(c, hipMemcpy(loff.data(), seg_off, (S + 1) * 8, hipMemcpyDeviceToHost));
      }
      cw_list_batch lb{};
      lb.n_docs = S;
      lb.doc_offsets = loff.data();
      lb.key_bits = key_bits;
      cw_list_result lr{};
      lr.weave_perm = lperm;
      lr.visible_count = lvc;
      lr.status = lst;
      c->x_pending = false;  // (a chunk's giant key weave left its own status there)
      if (exact_fixup(c, &lb, lid, lcause, lkind, &lr, true)) return -1;
    }
  }

  // 5. key weaves in collection-local input indices, active-node per key
  {
    Launch L(c, "m_segperm", (double)N * (4 + 4 + 8 + 4 + 4) + (double)S * 4);
    hipLaunchKernelGGL(k_seg_perm, dim3((uint32_t)((NL + 255) / 256)), dim3(256), 0, c->stream,
                       lperm, lmap, seg_off, seg_of, seg_start, N, (uint32_t)S, seg_perm);
  }
  if (check_launch(c, "m_segperm")) return -1;
  {
    Launch L(c, "m_active", (double)S * (16 + 4 + 4 + 8 + 3 * 9));
    hipLaunchKernelGGL(k_seg_active, dim3((uint32_t)((S + 255) / 256)), dim3(256), 0, c->stream,
                       lperm, lkind, seg_perm, seg_off, seg_coll, lst, (uint32_t)S, seg_act,
                       status);
  }
  if (check_launch(c, "m_active")) return -1;

  const hipMemcpyKind out_kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  HIPCHK(c, hipMemcpyAsync(res->seg_perm, seg_perm, NL * 4, out_kind, c->stream));
  HIPCHK(c, hipMemcpyAsync(res->seg_offsets, seg_off, (S + 1) * 8, out_kind, c->stream));
  HIPCHK(c, hipMemcpyAsync(res->seg_coll, seg_coll, S * 4, out_kind, c->stream));
  HIPCHK(c, hipMemcpyAsync(res->seg_key, seg_key, S * 8, out_kind, c->stream));
  HIPCHK(c, hipMemcpyAsync(res->seg_active, seg_act, S * 8, out_kind, c->stream));
  HIPCHK(c, hipMemcpyAsync(res->status, status, D * 4, out_kind, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  res->n_segs = S;
  if (c->prof) return collect_prof(c);
  return 0;
}

int merge_lists_impl(cw_ctx *c, const cw_merge_batch *bt, cw_merge_result *res, int memspace) {
  if (!bt || !res) return fail(c, "null batch/result");
  if (memspace != CW_MEM_HOST) return fail(c, "cw_merge_lists: only CW_MEM_HOST is supported");
  const uint64_t D = bt->a.n_docs;
  if (bt->b.n_docs != D) return fail(c, "a and b must have the same number of documents");
  const uint64_t *ao = bt->a.doc_offsets, *bo = bt->b.doc_offsets;
  if (!ao || !bo || ao[0] != 0 || bo[0] != 0) return fail(c, "doc_offsets must start at 0");
  const uint64_t Na = ao[D], Nb = bo[D], NC = Na + Nb;
  if (NC >= 0x7FFFFFFFull) return fail(c, "merge too large: %llu nodes", (unsigned long long)NC);
  std::vector<uint32_t> h_ao(D + 1), h_bo(D + 1), h_co(D + 1);
  std::vector<uint64_t> cap(D + 1);
  for (uint64_t d = 0; d <= D; d++) {
    if (d < D && (ao[d + 1] < ao[d] || bo[d + 1] < bo[d])) return fail(c, "doc_offsets not monotone");
    h_ao[d] = (uint32_t)ao[d];
    h_bo[d] = (uint32_t)bo[d];
    cap[d] = ao[d] + bo[d];
    h_co[d] = (uint32_t)cap[d];
  }
  for (uint64_t d = 0; d < D; d++)
    if (cap[d + 1] - cap[d] >= LINK_IDX) return fail(c, "document %llu too large", (unsigned long long)d);
  cw_list_result &W = res->weave;
  if (!res->merged_offsets || !res->merged_src || !W.weave_perm || !W.visible_count || !W.status)
    return fail(c, "merged_offsets, merged_src, weave_perm, visible_count and status are required");
  if ((Na && (!bt->a.id_key || !bt->a.cause_key || !bt->a.kind || !bt->a_value)) ||
      (Nb && (!bt->b.id_key || !bt->b.cause_key || !bt->b.kind || !bt->b_value)))
    return fail(c, "null input arrays");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t NCs = std::max<uint64_t>(NC, 1);
  uint64_t *aid = scratch_t<uint64_t>(c, "g_aid", std::max<uint64_t>(Na, 1)),
           *aca = scratch_t<uint64_t>(c, "g_aca", std::max<uint64_t>(Na, 1)),
           *ava = scratch_t<uint64_t>(c, "g_ava", std::max<uint64_t>(Na, 1));
  uint64_t *bid = scratch_t<uint64_t>(c, "g_bid", std::max<uint64_t>(Nb, 1)),
           *bca = scratch_t<uint64_t>(c, "g_bca", std::max<uint64_t>(Nb, 1)),
           *bva = scratch_t<uint64_t>(c, "g_bva", std::max<uint64_t>(Nb, 1));
  uint8_t *akd = scratch_t<uint8_t>(c, "g_akd", std::max<uint64_t>(Na, 1)),
          *bkd = scratch_t<uint8_t>(c, "g_bkd", std::max<uint64_t>(Nb, 1));
  uint32_t *dao = scratch_t<uint32_t>(c, "g_aoff", D + 1), *dbo = scratch_t<uint32_t>(c, "g_boff", D + 1),
           *dco = scratch_t<uint32_t>(c, "g_coff", D + 1), *dmo = scratch_t<uint32_t>(c, "g_moff", D + 1);
  uint64_t *cid = scratch_t<uint64_t>(c, "g_cid", NCs), *cca = scratch_t<uint64_t>(c, "g_cca", NCs),
           *cva = scratch_t<uint64_t>(c, "g_cva", NCs);
  uint8_t *ckd = scratch_t<uint8_t>(c, "g_ckd", NCs);
  uint64_t *mid = scratch_t<uint64_t>(c, "g_mid", NCs), *mca = scratch_t<uint64_t>(c, "g_mca", NCs);
  uint8_t *mkd = scratch_t<uint8_t>(c, "g_mkd", NCs);
  uint32_t *msrc = scratch_t<uint32_t>(c, "g_msrc", NCs), *mcnt = scratch_t<uint32_t>(c, "g_mcnt", D + 1),
           *mst = scratch_t<uint32_t>(c, "g_mst", D + 1);
  uint64_t *uskA = scratch_t<uint64_t>(c, "g_skA", NCs), *uskB = scratch_t<uint64_t>(c, "g_skB", NCs);
  uint32_t *usvA = scratch_t<uint32_t>(c, "g_svA", NCs), *usvB = scratch_t<uint32_t>(c, "g_svB", NCs);
  if (!aid || !aca || !ava || !bid || !bca || !bva || !akd || !bkd || !dao || !dbo || !dco || !dmo ||
      !cid || !cca || !cva || !ckd || !mid || !mca || !mkd || !msrc || !mcnt || !mst || !uskA ||
      !uskB || !usvA || !usvB)
    return fail(c, "out of device memory (merge, N=%llu)", (unsigned long long)NC);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (Na) {
    HIPCHK(c, hipMemcpy(aid, bt->a.id_key, Na * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(aca, bt->a.cause_key, Na * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(ava, bt->a_value, Na * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(akd, bt->a.kind, Na, hipMemcpyHostToDevice));
  }
  if (Nb) {
    HIPCHK(c, hipMemcpy(bid, bt->b.id_key, Nb * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(bca, bt->b.cause_key, Nb * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(bva, bt->b_value, Nb * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(bkd, bt->b.kind, Nb, hipMemcpyHostToDevice));
  }
  HIPCHK(c, hipMemcpy(dao, h_ao.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(dbo, h_bo.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(dco, h_co.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  if (!grid_ok(D, 1024)) return fail(c, "batch too large for one dispatch");
  uint64_t *mo = res->merged_offsets;
  mo[0] = 0;
  if (NC == 0) {
    for (uint64_t d = 0; d < D; d++) {
      mo[d + 1] = 0;
      W.status[d] = CW_STATUS_ROOT;
      W.visible_count[d] = 0;
      if (W.max_ts) W.max_ts[d] = 0;
    }
    return 0;
  }
  // 1. union: a then b per document, in capacity slots
  hipLaunchKernelGGL(k_merge_concat, dim3((uint32_t)D), dim3(256), 0, c->stream, aid, aca, akd,
                     ava, bid, bca, bkd, bva, dao, dbo, dco, cid, cca, ckd, cva);
  if (check_launch(c, "merge_concat")) return -1;
  // 2. id order per capacity slot (the general segmented radix sort)
  if (ensure_tables(c, D, cap.data())) return -1;
  uint32_t key_bits = bt->a.key_bits;
  if (key_bits == 0 && find_key_bits(c, cid, (uint32_t)NC, &key_bits)) return -1;
  uint64_t *skey;
  uint32_t *sval;
  if (radix_sort<uint64_t>(c, "m_idsort", cid, nullptr, uskA, usvA, uskB, usvB, key_bits, 0,
                           (uint32_t)NC, &skey, &sval))
    return -1;
  // 3. dedup: count, offsets, write
  hipLaunchKernelGGL((k_merge_dedup<1024>), dim3((uint32_t)D), dim3(1024), 0, c->stream, skey, sval,
                     cca, ckd, cva, dco, 0, mcnt, dmo, mid, mca, mkd, msrc, mst);
  if (check_launch(c, "merge_count")) return -1;
  std::vector<uint32_t> h_cnt(D);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(h_cnt.data(), mcnt, D * 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> h_mo(D + 1);
  for (uint64_t d = 0; d < D; d++) {
    mo[d + 1] = mo[d] + h_cnt[d];
    h_mo[d] = (uint32_t)mo[d];
  }
  h_mo[D] = (uint32_t)mo[D];
  HIPCHK(c, hipMemcpy(dmo, h_mo.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((k_merge_dedup<1024>), dim3((uint32_t)D), dim3(1024), 0, c->stream, skey, sval,
                     cca, ckd, cva, dco, 1, mcnt, dmo, mid, mca, mkd, msrc, mst);
  if (check_launch(c, "merge_write")) return -1;
  // 4. the merged documents through the list pipeline
  const uint64_t NM = mo[D];
  if (ensure_tables(c, D, mo)) return -1;
  cw_list_batch lb = bt->a;
  lb.doc_offsets = mo;
  lb.key_bits = key_bits;
  cw_list_result lr{};
  lr.weave_perm = scratch_t<uint32_t>(c, "g_perm", NCs);
  lr.visible_bits = W.visible_bits ? scratch_t<uint32_t>(c, "g_bits", (NCs + 31) / 32) : nullptr;
  lr.visible_count = scratch_t<uint32_t>(c, "g_vc", D + 1);
  lr.max_ts = W.max_ts ? scratch_t<uint64_t>(c, "g_mts", D + 1) : nullptr;
  lr.status = scratch_t<uint32_t>(c, "g_st", D + 1);
  lr.yarn_perm = W.yarn_perm ? scratch_t<uint32_t>(c, "g_yarn", NCs) : nullptr;
  if (!lr.weave_perm || !lr.visible_count || !lr.status || (W.visible_bits && !lr.visible_bits) ||
      (W.max_ts && !lr.max_ts) || (W.yarn_perm && !lr.yarn_perm))
    return fail(c, "out of device memory (merge outputs)");
  if (weave_lists_device(c, &lb, mid, mca, mkd, &lr)) return -1;
  if (exact_fixup(c, &lb, mid, mca, mkd, &lr, c->x_hint)) return -1;
  hipLaunchKernelGGL(k_or_status, dim3((uint32_t)((D + 255) / 256)), dim3(256), 0, c->stream, mst,
                     lr.status, (uint32_t)D);
  if (check_launch(c, "or_status")) return -1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(res->merged_src, msrc, NM * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(W.weave_perm, lr.weave_perm, NM * 4, hipMemcpyDeviceToHost));
  if (W.visible_bits)
    HIPCHK(c, hipMemcpy(W.visible_bits, lr.visible_bits, (NM + 31) / 32 * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(W.visible_count, lr.visible_count, D * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(W.status, lr.status, D * 4, hipMemcpyDeviceToHost));
  if (W.max_ts) HIPCHK(c, hipMemcpy(W.max_ts, lr.max_ts, D * 8, hipMemcpyDeviceToHost));
  if (W.yarn_perm) HIPCHK(c, hipMemcpy(W.yarn_perm, lr.yarn_perm, NM * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipDeviceSynchronize());
  for (uint64_t d = 0; d < D; d++)
    if (mo[d + 1] == mo[d]) W.status[d] |= CW_STATUS_ROOT;
  if (c->prof) return collect_prof(c);
  return 0;
}

int weft_lists_impl(cw_ctx *c, const cw_weft_batch *bt, cw_weft_result *res, int memspace) {
  if (!bt || !res) return fail(c, "null batch/result");
  if (memspace != CW_MEM_HOST) return fail(c, "cw_weft_lists: only CW_MEM_HOST is supported");
  const cw_list_batch &L = bt->nodes;
  const uint64_t D = L.n_docs;
  const uint64_t *off = L.doc_offsets;
  if (!off || off[0] != 0) return fail(c, "doc_offsets must start at 0");
  if (L.site_bits == 0 || L.site_bits > 10) return fail(c, "weft needs site_bits in 1..10");
  if (!bt->cut) return fail(c, "cut is required");
  const uint64_t N = off[D];
  if (N >= 0xFFFFFFFFull) return fail(c, "batch too large");
  cw_list_result &W = res->weave;
  if (!res->kept_offsets || !res->kept_src || !W.weave_perm || !W.visible_count || !W.status)
    return fail(c, "kept_offsets, kept_src, weave_perm, visible_count and status are required");
  std::vector<uint32_t> h_off(D + 1);
  for (uint64_t d = 0; d <= D; d++) {
    if (d < D && off[d + 1] < off[d]) return fail(c, "doc_offsets not monotone");
    h_off[d] = (uint32_t)off[d];
  }
  HIPCHK(c, hipSetDevice(c->device));
  const size_t Ns = std::max<uint64_t>(N, 1), NC = (size_t)D << L.site_bits;
  uint64_t *id = scratch_t<uint64_t>(c, "w_id", Ns), *ca = scratch_t<uint64_t>(c, "w_ca", Ns);
  uint8_t *kd = scratch_t<uint8_t>(c, "w_kd", Ns);
  uint64_t *cut = scratch_t<uint64_t>(c, "w_cut", std::max<size_t>(NC, 1));
  uint32_t *doff = scratch_t<uint32_t>(c, "w_off", D + 1), *koff = scratch_t<uint32_t>(c, "w_koff", D + 1);
  uint32_t *kcnt = scratch_t<uint32_t>(c, "w_kcnt", D + 1), *kst = scratch_t<uint32_t>(c, "w_kst", D + 1);
  // kept nodes: at most the document's nodes plus one [id] node per named site
  const size_t NKcap = Ns + NC;
  if (N + NC >= 0xFFFFFFFFull) return fail(c, "batch too large");
  uint64_t *kid = scratch_t<uint64_t>(c, "w_kid", NKcap), *kca = scratch_t<uint64_t>(c, "w_kca", NKcap);
  uint8_t *kkd = scratch_t<uint8_t>(c, "w_kkd", NKcap);
  uint32_t *ksrc = scratch_t<uint32_t>(c, "w_ksrc", NKcap);
  if (!id || !ca || !kd || !cut || !doff || !koff || !kcnt || !kst || !kid || !kca || !kkd || !ksrc)
    return fail(c, "out of device memory (weft)");
  if (!grid_ok(D, 1024)) return fail(c, "batch too large for one dispatch");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (N) {
    if (!L.id_key || !L.cause_key || !L.kind) return fail(c, "null input arrays");
    HIPCHK(c, hipMemcpy(id, L.id_key, N * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(ca, L.cause_key, N * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(kd, L.kind, N, hipMemcpyHostToDevice));
  }
  if (NC) HIPCHK(c, hipMemcpy(cut, bt->cut, NC * 8, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(doff, h_off.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  uint64_t *ko = res->kept_offsets;
  ko[0] = 0;
  if (D == 0) return 0;
  hipLaunchKernelGGL((k_weft_select<1024>), dim3((uint32_t)D), dim3(1024), 0, c->stream, id, ca, kd,
                     doff, cut, L.site_shift, L.site_bits, 0, kcnt, koff, kid, kca, kkd, ksrc, kst);
  if (check_launch(c, "weft_count")) return -1;
  std::vector<uint32_t> h_cnt(D), h_ko(D + 1);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(h_cnt.data(), kcnt, D * 4, hipMemcpyDeviceToHost));
  for (uint64_t d = 0; d < D; d++) {
    ko[d + 1] = ko[d] + h_cnt[d];
    h_ko[d] = (uint32_t)ko[d];
  }
  h_ko[D] = (uint32_t)ko[D];
  HIPCHK(c, hipMemcpy(koff, h_ko.data(), (D + 1) * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((k_weft_select<1024>), dim3((uint32_t)D), dim3(1024), 0, c->stream, id, ca, kd,
                     doff, cut, L.site_shift, L.site_bits, 1, kcnt, koff, kid, kca, kkd, ksrc, kst);
  if (check_launch(c, "weft_write")) return -1;
  const uint64_t NK = ko[D];
  if (ensure_tables(c, D, ko)) return -1;
  cw_list_batch lb = L;
  lb.doc_offsets = ko;
  const size_t NKs = std::max<uint64_t>(NK, 1);
  cw_list_result lr{};
  lr.weave_perm = scratch_t<uint32_t>(c, "w_perm", NKs);
  lr.visible_bits = W.visible_bits ? scratch_t<uint32_t>(c, "w_bits", (NKs + 31) / 32) : nullptr;
  lr.visible_count = scratch_t<uint32_t>(c, "w_vc", D + 1);
  lr.max_ts = W.max_ts ? scratch_t<uint64_t>(c, "w_mts", D + 1) : nullptr;
  lr.status = scratch_t<uint32_t>(c, "w_st", D + 1);
  lr.yarn_perm = W.yarn_perm ? scratch_t<uint32_t>(c, "w_yarn", NKs) : nullptr;
  if (!lr.weave_perm || !lr.visible_count || !lr.status || (W.visible_bits && !lr.visible_bits) ||
      (W.max_ts && !lr.max_ts) || (W.yarn_perm && !lr.yarn_perm))
    return fail(c, "out of device memory (weft outputs)");
  if (weave_lists_device(c, &lb, kid, kca, kkd, &lr)) return -1;
  if (exact_fixup(c, &lb, kid, kca, kkd, &lr, c->x_hint)) return -1;
  hipLaunchKernelGGL(k_or_status, dim3((uint32_t)((D + 255) / 256)), dim3(256), 0, c->stream, kst,
                     lr.status, (uint32_t)D);
  if (check_launch(c, "or_status")) return -1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (NK) {
    HIPCHK(c, hipMemcpy(res->kept_src, ksrc, NK * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(W.weave_perm, lr.weave_perm, NK * 4, hipMemcpyDeviceToHost));
    if (W.visible_bits)
      HIPCHK(c, hipMemcpy(W.visible_bits, lr.visible_bits, (NK + 31) / 32 * 4, hipMemcpyDeviceToHost));
    if (W.yarn_perm) HIPCHK(c, hipMemcpy(W.yarn_perm, lr.yarn_perm, NK * 4, hipMemcpyDeviceToHost));
  }
  HIPCHK(c, hipMemcpy(W.visible_count, lr.visible_count, D * 4, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(W.status, lr.status, D * 4, hipMemcpyDeviceToHost));
  if (W.max_ts) HIPCHK(c, hipMemcpy(W.max_ts, lr.max_ts, D * 8, hipMemcpyDeviceToHost));
  HIPCHK(c, hipDeviceSynchronize());
  for (uint64_t d = 0; d < D; d++)
    if (ko[d + 1] == ko[d]) W.status[d] |= CW_STATUS_ROOT;
  if (c->prof) return collect_prof(c);
  return 0;
}

}  // namespace

#include "k128.hip"

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int cw_abi_version(void) { return CW_ABI_VERSION; }

#ifndef CW_BUILD_ID
#define CW_BUILD_ID "unknown"
#endif
const char *cw_build_id(void) { return CW_BUILD_ID; }

int cw_ctx_create(int device, cw_ctx **out) {
  if (!out) return -1;
  *out = nullptr;
  cw_ctx *c = new cw_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return -1;
  }
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return -1;
  }
  c->stream = c->own_stream;
  {
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess &&
        lds > 0)
      c->lds_max = (uint32_t)lds;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) c->hbm_total = tot;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      c->n_cu = (uint32_t)ncu;
  }
  auto knob = [](const char *name, uint32_t dflt) {
    const char *v = getenv(name);
    return v ? (uint32_t)strtoul(v, nullptr, 0) : dflt;
  };
  // launch geometry (round 5: the A/B knobs CW_TB, CW_WALK_THREADS, CW_WALK_SPAN,
  // CW_LOG2K, CW_LOG2CAP and CW_MAX_DIGIT are gone, their measured values stay):
  // one walker per thread (span == threads: a dynamic walker queue per block was slower)
  c->tb = 1024;
  c->walk_threads = 512;
  c->walk_span = 512;
  c->min_log2k = MIN_LOG2K;
  c->min_log2cap = 4;
  c->max_digit = MAX_DIGIT;
  c->front = knob("CW_FRONT", 1);
  c->tree_prof = knob("CW_TREE_PROF", 0);
  c->tree_l = knob("CW_TREE_L", 2048);
  c->gdir = knob("CW_GDIR", 32);
  c->gjoin = knob("CW_GJOIN", 1);
  c->id_payload = knob("CW_ID_PAYLOAD", 1);
  c->glocal = knob("CW_GLOCAL", 1);
  c->glocal_min = knob("CW_GLOCAL_MIN", 1u << 20);
  c->map_small = knob("CW_MAP_SMALL", 1);
  c->map_fused = knob("CW_MAP_FUSED", 1);
  c->pack_sort = knob("CW_PACK_SORT", 1);
  c->giant_min = knob("CW_GIANT_MIN", 1u << 16);
  c->tour = knob("CW_TOUR", 1);
  c->giant_docs_max = knob("CW_GIANT_DOCS", 32);
  c->front_fused = knob("CW_FRONT_FUSED", 1);
  c->tour_log2k = std::max(MIN_LOG2K, std::min(knob("CW_TOUR_LOG2K", 3), 12u));
  c->giant_log2k = std::max(MIN_LOG2K, std::min(knob("CW_GIANT_LOG2K", 4), 12u));
  c->giant_log2cap = std::max(2u, std::min(knob("CW_GIANT_LOG2CAP", 5), 12u));
  c->fused = knob("CW_FUSED", 1);
  c->xfold = knob("CW_XFOLD", 0);
  c->x_round_cap = std::max(1u, knob("CW_X_ROUND_CAP", 48));
  c->onesweep = std::min(knob("CW_ONESWEEP", 4), 6u);
  c->onesweep_min = knob("CW_ONESWEEP_MIN", 1u << 16);
  c->os_exp = knob("CW_OS_EXP", 0);
  c->front_slot_groups = std::max(1u, std::min(knob("CW_FRONT_SLOT", 65536), 131072u) / 16);
  c->front_min_avg = knob("CW_FRONT_MIN_AVG", 1024);
  *out = c;
  return 0;
}

void cw_ctx_destroy(cw_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto &kv : c->bufs)
    if (kv.second.p) (void)hipFree(kv.second.p);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->pin_small) (void)hipHostFree(c->pin_small);
  if (c->pin_status) (void)hipHostFree(c->pin_status);
  if (c->ev_status) (void)hipEventDestroy(c->ev_status);
  for (auto &p : c->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : c->evt_pool) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char *cw_last_error(const cw_ctx *c) { return c ? c->err.c_str() : "null context"; }

int cw_ctx_set_stream(cw_ctx *c, void *s) {
  if (!c) return -1;
  if (collect_prof(c, true)) return -1;
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return 0;
}

int cw_ctx_set_async(cw_ctx *c, int a) {
  if (!c) return -1;
  if (collect_prof(c, true)) return -1;
  c->async = a != 0;
  return 0;
}

int cw_ctx_set_profiling(cw_ctx *c, int on) {
  if (!c) return -1;
  if (collect_prof(c, true)) return -1;
  c->prof = on != 0;
  return 0;
}

int cw_ctx_set_profile_only(cw_ctx *c, const char *kernel) {
  if (!c) return -1;
  c->prof_only = kernel ? kernel : "";
  return 0;
}

int cw_get_kernel_stats(const cw_ctx *c, cw_kernel_stat *out, int cap) {
  if (!c) return -1;
  if (collect_prof(const_cast<cw_ctx *>(c), true)) return -1;
  int i = 0;
  for (auto &kv : c->stats) {
    if (i < cap && out) {
      memset(&out[i], 0, sizeof(cw_kernel_stat));
      snprintf(out[i].name, sizeof out[i].name, "%s", kv.first.c_str());
      out[i].launches = kv.second.launches;
      out[i].total_ms = kv.second.ms;
      out[i].bytes_alg = kv.second.bytes;
    }
    i++;
  }
  return i;
}

int cw_weave_lists(cw_ctx *c, const cw_list_batch *b, cw_list_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  if (memspace != CW_MEM_HOST && memspace != CW_MEM_DEVICE) return fail(c, "bad memspace");
  return weave_lists_impl(c, b, r, memspace);
}

int cw_weave_lists_k32(cw_ctx *c, const cw_list_batch_k32 *b, cw_list_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  return weave_lists_k32_impl(c, b, r, memspace);
}

int cw_weave_lists_k128(cw_ctx *c, const cw_list_batch_k128 *b, cw_list_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  return weave_lists_k128_impl(c, b, r, memspace);
}

int cw_weave_maps(cw_ctx *c, const cw_map_batch *b, cw_map_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  return weave_maps_impl(c, b, r, memspace);
}

int cw_merge_lists(cw_ctx *c, const cw_merge_batch *b, cw_merge_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  return merge_lists_impl(c, b, r, memspace);
}

int cw_weft_lists(cw_ctx *c, const cw_weft_batch *b, cw_weft_result *r, int memspace) {
  if (!c) return -1;
  c->err.clear();
  return weft_lists_impl(c, b, r, memspace);
}

int cw_sort_keys(cw_ctx *c, const uint64_t *keys, uint64_t n, uint32_t key_bits, uint64_t *keys_out,
                 uint32_t *idx_out) {
  if (!c) return -1;
  c->err.clear();
  if (sort_keys_impl(c, keys, n, key_bits, keys_out, idx_out)) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

int cw_lookup_keys(cw_ctx *c, const uint64_t *sorted, uint64_t n, const uint64_t *queries,
                   uint64_t m, uint32_t base, uint32_t *out, uint32_t *status) {
  if (!c) return -1;
  c->err.clear();
  if (lookup_keys_impl(c, sorted, n, queries, m, base, out, status)) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

int cw_gather(cw_ctx *c, const void *src, const uint32_t *idx, uint64_t m, uint32_t elem_size,
              void *dst) {
  if (!c) return -1;
  c->err.clear();
  if (gather_impl(c, src, idx, m, elem_size, dst)) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

int cw_partition_keys(cw_ctx *c, const uint64_t *keys, uint64_t m, const uint64_t *splitters,
                      uint32_t n_split, uint32_t *perm, uint64_t *counts) {
  if (!c) return -1;
  c->err.clear();
  if (partition_keys_impl(c, keys, m, splitters, n_split, perm, counts)) return -1;
  return c->prof ? collect_prof(c) : 0;
}

int cw_partition_keys_dev(cw_ctx *c, const uint64_t *keys, uint64_t m, const uint64_t *splitters,
                          uint32_t n_split, uint32_t *perm, uint64_t *counts) {
  if (!c) return -1;
  c->err.clear();
  HIPCHK(c, hipSetDevice(c->device));
  if (partition_keys_impl(c, keys, m, splitters, n_split, perm, counts, true)) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

int cw_scatter32(cw_ctx *c, const uint32_t *src, const uint32_t *idx, uint64_t m, uint32_t *dst) {
  if (!c) return -1;
  c->err.clear();
  if (scatter_impl(c, src, idx, m, dst)) return -1;
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream));
  return c->prof ? collect_prof(c) : 0;
}

int cw_weave_ranked(cw_ctx *c, const cw_ranked_list *l, cw_list_result *r) {
  if (!c) return -1;
  c->err.clear();
  return weave_ranked_impl(c, l, r);
}

// distributed tree (dist.hip): device memory, ordered on the context's stream
#define CW_DIST_ENTRY(call)                                \
  if (!c) return -1;                                       \
  c->err.clear();                                          \
  HIPCHK(c, hipSetDevice(c->device));                      \
  if (call) return -1;                                     \
  if (!c->async) HIPCHK(c, hipStreamSynchronize(c->stream)); \
  return c->prof ? collect_prof(c) : 0;

int cw_sort_keys32(cw_ctx *c, const uint32_t *keys, uint64_t n, uint32_t key_bits,
                   uint32_t *keys_out, uint32_t *idx_out) {
  CW_DIST_ENTRY(sort_keys32_impl(c, keys, n, key_bits, keys_out, idx_out))
}
int cw_dist_check(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                  uint32_t *status) {
  CW_DIST_ENTRY(dist_check_impl(c, n, base, par, kind, status))
}
int cw_dist_eff(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                uint32_t *eff) {
  CW_DIST_ENTRY(dist_eff_impl(c, n, base, par, kind, eff))
}
int cw_dist_climb(cw_ctx *c, uint64_t n, uint32_t base, const uint32_t *par, const uint8_t *kind,
                  const uint64_t *q, uint64_t m, uint32_t *out) {
  CW_DIST_ENTRY(dist_climb_impl(c, n, base, par, kind, q, m, out))
}
int cw_dist_pending(cw_ctx *c, const uint32_t *w, uint64_t n, uint64_t *keys, uint32_t *count) {
  CW_DIST_ENTRY(dist_pending_impl(c, w, n, keys, count))
}
int cw_dist_gkey(cw_ctx *c, const uint32_t *eff, const uint8_t *kind, uint64_t n, uint32_t *key) {
  CW_DIST_ENTRY(dist_gkey_impl(c, eff, kind, n, key))
}
int cw_dist_runs(cw_ctx *c, const uint32_t *skey, const uint32_t *sidx, uint64_t n, uint32_t base,
                 const uint8_t *kind, uint32_t *nsc, uint64_t *okey, uint32_t *rec) {
  CW_DIST_ENTRY(dist_runs_impl(c, skey, sidx, n, base, kind, nsc, okey, rec))
}
int cw_dist_rkey(cw_ctx *c, const uint32_t *rec, uint64_t m, uint32_t *key) {
  CW_DIST_ENTRY(dist_rkey_impl(c, rec, m, key))
}
int cw_dist_link(cw_ctx *c, const uint32_t *skey, const uint32_t *sidx, uint64_t m,
                 const uint32_t *rec, uint32_t base, uint64_t n, uint32_t *fcS, uint32_t *fcN,
                 uint32_t *reply) {
  CW_DIST_ENTRY(dist_link_impl(c, skey, sidx, m, rec, base, n, fcS, fcN, reply))
}
int cw_dist_put(cw_ctx *c, const uint32_t *rec, const uint32_t *reply, uint64_t m, uint32_t base,
                uint64_t n, uint32_t *nsc) {
  CW_DIST_ENTRY(dist_put_impl(c, rec, reply, m, base, n, nsc))
}
int cw_dist_thr(cw_ctx *c, const uint32_t *nsc, uint64_t n, uint32_t base, uint32_t *T) {
  CW_DIST_ENTRY(dist_thr_impl(c, nsc, n, base, T))
}
int cw_dist_succ(cw_ctx *c, const uint8_t *kind, const uint32_t *fcS, const uint32_t *fcN,
                 uint64_t n, uint32_t base, uint32_t *out) {
  CW_DIST_ENTRY(dist_succ_impl(c, kind, fcS, fcN, n, base, out))
}
int cw_dist_rs_rulers(cw_ctx *c, const uint32_t *succ, const uint32_t *thr, uint64_t n,
                      uint32_t base, uint32_t k, uint32_t seed, uint32_t *word, uint32_t *rlist,
                      uint32_t *count) {
  CW_DIST_ENTRY(dist_rs_rulers_impl(c, succ, thr, n, base, k, seed, word, rlist, count))
}
int cw_dist_rs_walk(cw_ctx *c, const uint32_t *walkers, uint64_t m, const uint32_t *rlist,
                    uint32_t rbase, const uint32_t *word, const uint32_t *thr, uint64_t n,
                    uint32_t base, uint32_t *own, uint32_t *links, uint32_t *nlinks, uint32_t *out,
                    uint64_t *key, uint32_t *status) {
  CW_DIST_ENTRY(dist_rs_walk_impl(c, walkers, m, rlist, rbase, word, thr, n, base, own, links,
                                  nlinks, out, key, status))
}
int cw_dist_rs_top(cw_ctx *c, const uint32_t *links, uint64_t m, uint64_t total, uint32_t *pos,
                   uint32_t *status) {
  CW_DIST_ENTRY(dist_rs_top_impl(c, links, m, total, pos, status))
}
int cw_dist_rs_pos(cw_ctx *c, const uint32_t *own, const uint32_t *pos_base, const uint32_t *succ,
                   const uint32_t *val, uint64_t n, uint32_t *rec, uint64_t *key) {
  CW_DIST_ENTRY(dist_rs_pos_impl(c, own, pos_base, succ, val, n, rec, key))
}
int cw_dist_rs_emit(cw_ctx *c, const uint32_t *rec, uint64_t m, uint32_t p0, uint64_t len,
                    uint32_t *weave_perm, uint32_t *visible_bits, uint32_t *visible_count,
                    uint32_t *status) {
  CW_DIST_ENTRY(dist_rs_emit_impl(c, rec, m, p0, len, weave_perm, visible_bits, visible_count,
                                  status))
}
#undef CW_DIST_ENTRY

int cw_weave_linked(cw_ctx *c, const cw_linked_list *l, cw_list_result *r) {
  if (!c) return -1;
  c->err.clear();
  return weave_linked_impl(c, l, r);
}

int cw_get_counter(cw_ctx *c, const char *name, uint64_t *value) {
  if (!c || !name || !value) return -1;
  if (strcmp(name, "continued_sublists") != 0) return fail(c, "unknown counter %s", name);
  *value = 0;
  if (!c->last_dyn || !c->last_dyn_n) return 0;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<uint32_t> h(c->last_dyn_n);
  HIPCHK(c, hipMemcpy(h.data(), c->last_dyn, h.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t v : h) *value += v;
  return 0;
}

int cw_reset_kernel_stats(cw_ctx *c) {
  if (!c) return -1;
  if (collect_prof(c, true)) return -1;
  c->stats.clear();
  return 0;
}

}  // extern "C"
