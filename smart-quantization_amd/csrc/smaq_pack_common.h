// smaq_pack_common.h — the packed SmaQ container's format constants and element-coding helpers
// (include/smq.h "Packed SmaQ container", format version 2), shared by the packer kernels
// (smaq_pack.hip) and the single launch that also packs (smaq_fused.hip, PACK variant). Internal.
#pragma once

#include <hip/hip_runtime.h>

#include "smq.h"
#include "smq_common.h"

namespace smq {

constexpr int kPB = SMQ_PACK_BLOCK;          // 4096 elements per block
constexpr int kMaskWords = kPB / 32;         // 128
constexpr int kMaxWidth = 24;                // widest code (num_bits - 1)
constexpr int kGroup = 64;                   // blocks per group sum (one per lane of a wave)
constexpr int kVarCap = 768;                 // scratch words per block for its variable section
constexpr int kSegs = 16;                    // rank segments of a block: 4 slots x 4 waves

static_assert(sizeof(SmqPackedHeader) == 128, "packed header layout");

// directory entries incl. the padding that keeps the fixed region 16-B aligned
__host__ __device__ inline int64_t dir_entries(int64_t nb) { return (nb + 1) & ~(int64_t)1; }
__host__ __device__ inline uint32_t fixed_words(int wm) { return kMaskWords + 128u * (uint32_t)wm; }
__host__ __device__ inline uint32_t ext_words(int we, uint32_t n_out) {
  return ((uint32_t)we * n_out + 31u) / 32u;
}

// Code of one element (smq.h format rules), branch-free integer form: v = q + 2^(wm-1) for a main
// (fits: v < 2^wm; the code is v ^ 2^(wm-1) = q's wm-bit two's complement), |q| on the element's
// side for an outlier (fits: v < 2^(wo-1); the code is side << (wo-1) | v). |q| > 2^24, inf and NaN
// always escape; an escaped main codes 0, an escaped outlier its side bit alone.
// hm = 2^(wm-1), side = 2^(wo-1), lim_m = 2^wm
__device__ __forceinline__ uint32_t code_sel(float q, bool o, bool lo, uint32_t hm, uint32_t side,
                                             uint32_t lim_m, bool& esc) {
  const int qi = (int)q;
  const bool big = !(__builtin_fabsf(q) <= 0x1p24f);     // also NaN
  const uint32_t hsel = o ? 0u : hm;
  const uint32_t vv = lo ? (uint32_t)(-qi) : (uint32_t)qi + hsel;
  const uint32_t lim = o ? side : lim_m;
  esc = big | !(vv < lim);
  const uint32_t sb = lo ? side : 0u;
  return esc ? sb : ((vv ^ hsel) | sb);
}

// OR a chunk of up to 64 bits at bit pos of an LDS bit stream (two or three words; the third only
// when bits land there).
__device__ __forceinline__ void or_bits64(uint32_t* base, uint32_t pos, uint64_t chunk) {
  const uint32_t sft = pos & 31u, w0 = pos >> 5;
  const uint64_t lo = chunk << sft;
  const uint32_t hi = sft ? (uint32_t)(chunk >> (64u - sft)) : 0u;
  if ((uint32_t)lo) atomicOr(base + w0, (uint32_t)lo);
  if ((uint32_t)(lo >> 32)) atomicOr(base + w0 + 1, (uint32_t)(lo >> 32));
  if (hi) atomicOr(base + w0 + 2, hi);
}

// OR a chunk of up to 32 bits at bit pos of an LDS bit stream (one or two words).
__device__ __forceinline__ void or_bits32(uint32_t* base, uint32_t pos, uint32_t chunk) {
  const uint32_t sft = pos & 31u, w0 = pos >> 5;
  atomicOr(base + w0, chunk << sft);
  const uint32_t hi = sft ? (chunk >> (32u - sft)) : 0u;
  if (hi) atomicOr(base + w0 + 1, hi);
}

// Escapes of one rank segment (256 elements) a block keeps in LDS before the segment bases are
// known; a segment with more (an escape-heavy block) makes the var kernel re-code the block.
constexpr int kSegEsc = 32;

// The stream's total_bytes for a caller that learns it without an event or a copy
// (smq_smaq_roundtrip_compress_notify): a system-scope store of the saturated 32-bit value, so
// host-mapped coherent memory holds it as soon as the header is written. NULL: no notification.
__device__ __forceinline__ void notify_total(uint32_t* p, uint64_t total) {
  if (p)
    __hip_atomic_store(p, total < SMQ_NOTIFY_SATURATED ? (uint32_t)total : SMQ_NOTIFY_SATURATED,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace smq
