// cw_internal.h -- constants and small device helpers shared by the weave kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace cw {

// Sort tiles: a tile is a run of <= TILE consecutive nodes of ONE document.
constexpr uint32_t TILE = 4096;
constexpr uint32_t SORT_THREADS = 512;            // 8 waves
constexpr uint32_t SORT_ITEMS = TILE / SORT_THREADS;
constexpr uint32_t SORT_WAVES = SORT_THREADS / 64;
constexpr uint32_t MAX_DIGIT = 11;                // bits per LSD pass
constexpr uint32_t MAX_BINS = 1u << MAX_DIGIT;
constexpr uint32_t SUB_BITS = 6;                  // in-tile sub-pass digit
constexpr uint32_t SUB_BINS = 1u << SUB_BITS;


// Join (general front end): nodes per lane, their loads and bucket searches interleaved.
constexpr int JOIN_ITEMS = 4;

// Walk: one walker per splitter node; <= MAX_SUBLISTS sublists per document
// so the sublist ranking of a document fits one workgroup's LDS.
constexpr uint32_t MAX_SUBLISTS = 16384;          // rank: 128 KiB of LDS
constexpr uint32_t CHAIN = 64;                     // rank: sublists per LDS chain head
constexpr uint32_t MIN_LOG2K = 3;                 // >= 8 nodes per splitter block
// One giant document takes 32-entry walk slots when n * this many bytes of
// device memory are free (plus the context's own reusable scratch) at the
// call: the library's scratch with them is ~92 B a node (2e9 nodes: 218 GiB
// in use with the caller's 21 B a node of inputs and outputs).
constexpr uint64_t GIANT_CAP32_BYTES = 100;

// An id sort's carried cause and kind (onesweep.hip OsPayload): the cause's
// bits above 32 and the kind ride in the key's bits above kb, CH + 8 of them.
constexpr uint32_t OS_PL_MAX_BITS = 43;  // CH + 8 <= 64 - kb
__host__ __device__ constexpr uint32_t os_pl_ch(uint32_t kb) { return (kb > 32 ? kb : 32) - 31; }

// link word (u32): low 29 bits = the node's preorder successor (SUCC_END for the
// last node), bit 31 = the node renders, bit 30 = the node is a splitter, bit
// 29 = the successor is thr[low bits] (a thread the giant-document tree left
// to the walk: thr entries are a successor or again LINK_PEND | node).
constexpr uint32_t LINK_VIS = 0x80000000u;
constexpr uint32_t LINK_SPLIT = 0x40000000u;
constexpr uint32_t LINK_PEND = 0x20000000u;
constexpr uint32_t LINK_IDX = 0x1FFFFFFFu;        // documents < 2^29 nodes
constexpr uint32_t EMIT_STAGE = 4096;          // weave positions staged per emit block
constexpr uint32_t NSC_UP = 0x80000000u;         // nsc: no next sibling, low bits = eff parent
constexpr uint32_t SUCC_END = LINK_IDX;           // the last node in preorder
constexpr uint32_t NX_END = 0xFFFFFFFFu;          // last sublist of a document
// Wide links (the giant-document path, documents < 2^31 - 1 nodes): a u64 link
// word = successor (bits 0-30; SUCCW_END for the last node) | pending thread
// (bit 31) | the value the emit writes for this node (bits 32-62: its input
// index, so the emit gathers nothing) | renders (bit 63).  Splitters are
// recomputed from the rank (split_node).  thr entries = node | THRW_PEND when
// still pending.
constexpr uint32_t SUCCW_END = 0x7FFFFFFFu;
constexpr uint32_t THRW_PEND = 0x80000000u;
__host__ __device__ constexpr uint64_t wide_link(uint32_t succ, bool pend, uint32_t val, bool vis) {
  return (uint64_t)(succ & SUCCW_END) | (pend ? 0x80000000ull : 0ull) |
         ((uint64_t)(val & 0x7FFFFFFFu) << 32) | (vis ? (1ull << 63) : 0ull);
}
constexpr uint32_t SLOT_IDX = 0x7FFFFFFFu;        // walk slot entry: rank | renders << 31

constexpr uint8_t KIND_CLASS = 3, KIND_ROOT = 4, KIND_HIDE = 1, KIND_HHIDE = 2;

__device__ __forceinline__ bool is_special(uint8_t k) { return (k & KIND_CLASS) != 0; }
__device__ __forceinline__ bool is_hide(uint8_t k) {
  return (k & KIND_CLASS) == KIND_HIDE || (k & KIND_CLASS) == KIND_HHIDE;
}

// Number of lanes below this one whose bit is set in m (wave64).
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Element i of a wave-uniform base pointer, addressed as base + zext(i * size):
// the global access takes the scalar base and a 32-bit lane offset (saddr
// form), no 64-bit address arithmetic per lane.  i * sizeof(T) < 2^32.
template <typename T>
__device__ __forceinline__ T &lane_at(T *b, uint32_t i) {
  using C = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return *reinterpret_cast<T *>(reinterpret_cast<C *>(b) + (size_t)(i * (uint32_t)sizeof(T)));
}

// Blocks b, b+8, b+16, ... are dealt to the same XCD (MI355X_MICROARCH.md,
// "Workgroup dispatch").  Give each XCD a contiguous range of tiles so one
// document's tiles share one L2; bijective for any grid size.  Speed only.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
  const uint32_t q = nb >> 3, r = nb & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

// 32-bit mix of (a, b): murmur3's finalizer over a * golden + b (three
// 32-bit multiplies; split_node runs for every node of the tree's sweep 2).
__device__ __forceinline__ uint32_t mix32(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u + b;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// The splitter node of block j (nodes [j*K, (j+1)*K) of a document of n nodes):
// the root for block 0, else a hashed position inside the block (a multiply-
// high reduction of the hash onto the block's length, no division).  Hashing
// avoids the periodicity of interleaved site chains.
__device__ __forceinline__ uint32_t split_node(uint32_t doc, uint32_t j, uint32_t log2k, uint32_t n) {
  if (j == 0) return 0;
  const uint32_t lo = j << log2k, m = min(1u << log2k, n - lo);
  return lo + __umulhi(mix32(doc, j), m);
}

}  // namespace cw
