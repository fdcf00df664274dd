// smq_common.h — shared device/host helpers of libsmq (gfx950 only).
//
// Numerics contract: every fp32 operation of the reference's ATen op
// chain is issued as its own IEEE-754 round-to-nearest operation in the same order. The library is
// compiled with -ffp-contract=off so `a * b + c` never fuses into an FMA, and `/` lowers to the
// correctly rounded v_div_scale / v_div_fmas / v_div_fixup sequence.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "smq.h"

#include <stdlib.h>

namespace smq {

// Measurement knobs: environment overrides of tuning constants, read ONLY by experiment builds
// (tools/build_variant.py <name> -DSMQ_KNOBS=1). The shipped library never consults the
// environment for them, so no stray variable can change a launch shape or a reduction order (and
// with it the bits a caller gets).
#ifndef SMQ_KNOBS
#define SMQ_KNOBS 0
#endif
static inline const char* knob_env(const char* name) {
#if SMQ_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

constexpr int kBlock = 256;  // 4 wave64 per workgroup
constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// Counter-based RNG. Element i of a call draws from counter c = offset + i, so the value of an
// element never depends on the launch geometry and the CPU oracle reproduces it bit for bit
// (oracle/rng.py). One "lowbias32" finaliser (C. Wellons) = 2 v_mul_lo_u32 per hash: per element
// for the float quantiser (rng_u32), per four elements for SmaQ's rounding draws (smaq_u24).
// The 64-bit seed is folded into a 32-bit key once per launch on the host.
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t rng_key(uint64_t seed) {
  return mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) ^ 0x9e3779b9U));
}

__host__ __device__ __forceinline__ uint32_t rng_u32(uint32_t key, uint64_t ctr) {
  const uint32_t lo = (uint32_t)ctr;
  const uint32_t hi = (uint32_t)(ctr >> 32);
  return mix32(lo ^ ((hi << 16) | (hi >> 16)) ^ key);
}

// SmaQ's stochastic-rounding draws (smart.py:93-98's rand_like): 24-bit uniforms as integers
// < 2^24, ONE counter hash per four consecutive counters. Counter c reads the quad word
// h = quad_word(key, c >> 2); lane r = c & 3 takes the top 24 bits of h * draw_mul(r), an odd
// multiplier (a bijection of the 32-bit word: every lane is uniform; lane 0's is 1). An aligned
// float4 of elements costs one hash, 3 multiplies, 4 shifts and 4 conversions instead of four
// hashes (the packer and the half-input apply are VALU-bound: DESIGN.md §3). The quad hash is
// "triple32" (C. Wellons; 3 multiplies): lowbias32 over 2^22 consecutive counters leaves the top
// 12 bits 8-11 sigma off uniform (chi-square), triple32 within 4 (tests/test_rng_quality.py).
// The float quantiser (qtorch) keeps rng_u32 per element: it reads the low bits of its words too.
__host__ __device__ __forceinline__ uint32_t mix32x3(uint32_t x) {
  x ^= x >> 17;
  x *= 0xed5ad4bbU;
  x ^= x >> 11;
  x *= 0xac4c1b51U;
  x ^= x >> 15;
  x *= 0x31848babU;
  x ^= x >> 14;
  return x;
}

__host__ __device__ __forceinline__ uint32_t quad_word(uint32_t key, uint64_t q) {
  const uint32_t lo = (uint32_t)q;
  const uint32_t hi = (uint32_t)(q >> 32);
  return mix32x3(lo ^ ((hi << 16) | (hi >> 16)) ^ key);
}

__host__ __device__ __forceinline__ uint32_t draw_mul(uint32_t r) {
  return r == 0u ? 1u : r == 1u ? 0x9e3779b1u : r == 2u ? 0x85ebca77u : 0xc2b2ae3du;
}

__host__ __device__ __forceinline__ uint32_t smaq_u24(uint32_t key, uint64_t c) {
  return (quad_word(key, c >> 2) * draw_mul((uint32_t)c & 3u)) >> 8;
}

// U[0,1) with 24 random bits, the resolution of torch.rand_like for fp32.
__host__ __device__ __forceinline__ float u32_to_unit(uint32_t h) {
  return (float)(h >> 8) * 5.9604644775390625e-08f;  // 2^-24
}

// ---------------------------------------------------------------------------------------------
// 16-byte streaming accesses (global_load/store_dwordx4, optionally with the nt hint)
// ---------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 load_nt(const float4* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void store_nt(float4* p, const float4& v) {
  f32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
}

// Streaming output store of the element kernels: write-through + non-temporal (`sc0 sc1 nt`).
// Measured on the 256M round trip (interleaved A/B, 3 pairs): 0.515 ms/step against 0.520 with
// `nt` alone, 0.545-0.55 with plain or `sc1` stores — the next call's statistics sweep runs
// faster behind it. SMQ_STORE_SC=0 builds the plain `nt` store.
#ifndef SMQ_STORE_SC
#define SMQ_STORE_SC 1
#endif
//
// The store is inline asm, which the compiler's hazard recognizer cannot see as a VMEM store of
// 16 bytes: a VALU write of the data VGPRs right behind it would race the store's read of them
// (a wave64 store reads its data 16 lanes per cycle; measured on gfx950: the first element of 16
// lanes of some tiles came out as the next value written to that register). The trailing
// `s_nop 1` gives the two wait states the hazard needs, inside the asm statement.
__device__ __forceinline__ void store_stream(float4* p, const float4& v) {
#if SMQ_STORE_SC
  const f32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
#else
  store_nt(p, v);
#endif
}

// ---------------------------------------------------------------------------------------------
// Wave64 / workgroup reductions
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// DPP lane permutations (GFX9 encodings): quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror,
// row_mirror.
constexpr int kDppXor1 = 0xb1, kDppXor2 = 0x4e, kDppHalfMirror = 0x141, kDppMirror = 0x140;

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xf, 0xf, false));
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Wave64 sum in the ASCENDING xor-butterfly order (partners at distance 1, 2, 4, 8, 16, 32), the
// same value in every lane (a wave-uniform result). After the step at distance o the value is
// uniform over each aligned group of 2o lanes, so any lane of the partner group serves as lane
// l ^ o: quad permutes for 1 and 2, the half-row / row mirrors for 4 and 8 (VALU DPP moves, no
// LDS round trip), and the four row totals by readlane: (r0 + r1) + (r2 + r3), which is what the
// last two butterfly steps compute in every lane (fp add is commutative). All 64 lanes active.
__device__ __forceinline__ double wave_sum_asc(double v) {
  v += dpp_f64<kDppXor1>(v);
  v += dpp_f64<kDppXor2>(v);
  v += dpp_f64<kDppHalfMirror>(v);
  v += dpp_f64<kDppMirror>(v);
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// The same butterfly for a NaN-propagating max (torch.max): max is order-free up to NaN payloads.
__device__ __forceinline__ float nan_max2(float a, float b) { return (b > a || b != b) ? b : a; }
__device__ __forceinline__ float wave_nanmax_asc(float v) {
  v = nan_max2(v, dpp_f32<kDppXor1>(v));
  v = nan_max2(v, dpp_f32<kDppXor2>(v));
  v = nan_max2(v, dpp_f32<kDppHalfMirror>(v));
  v = nan_max2(v, dpp_f32<kDppMirror>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return nan_max2(nan_max2(r0, r1), nan_max2(r2, r3));
}

// fminf / fmaxf over the wave by DPP moves and readlanes (no LDS round trips; order-free up to the
// sign of a zero result); every lane gets the result.
__device__ __forceinline__ float wave_min_dpp(float v) {
  v = fminf(v, dpp_f32<kDppXor1>(v));
  v = fminf(v, dpp_f32<kDppXor2>(v));
  v = fminf(v, dpp_f32<kDppHalfMirror>(v));
  v = fminf(v, dpp_f32<kDppMirror>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return fminf(fminf(r0, r1), fminf(r2, r3));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f32<kDppXor1>(v));
  v = fmaxf(v, dpp_f32<kDppXor2>(v));
  v = fmaxf(v, dpp_f32<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f32<kDppMirror>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Cross-workgroup hand-off of per-workgroup partials WITHOUT release/acquire fences
// (MI355X_MICROARCH.md §inter-workgroup visibility, "Valid forms", table row 1): the partial is
// stored write-through (sc1, relaxed agent-scope atomic stores), the storing wave drains vmcnt,
// then ONE lane adds to ONE counter; the workgroup whose add returned count-1 is last and reads
// every partial with sc1 loads (bypassing its L1). A per-workgroup release fence (buffer_wbl2)
// instead measured ~30 % slower on a 1 GiB statistics sweep (2048 fences piling up at the tail).
__device__ __forceinline__ void st_sc1_u64(void* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1_u64(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f64(void* p, double v) {
  st_sc1_u64(p, __builtin_bit_cast(uint64_t, v));
}
__device__ __forceinline__ double ld_sc1_f64(const void* p) {
  return __builtin_bit_cast(double, ld_sc1_u64(p));
}
__device__ __forceinline__ void st_sc1_f32x2(void* p, float a, float b) {
  st_sc1_u64(p, (uint64_t)__builtin_bit_cast(uint32_t, a) |
                    ((uint64_t)__builtin_bit_cast(uint32_t, b) << 32));
}
__device__ __forceinline__ void ld_sc1_f32x2(const void* p, float& a, float& b) {
  const uint64_t v = ld_sc1_u64(p);
  a = __builtin_bit_cast(float, (uint32_t)v);
  b = __builtin_bit_cast(float, (uint32_t)(v >> 32));
}

__device__ __forceinline__ void st_sc1_u32(void* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Fill of n words on the stream: the library's replacement of hipMemsetAsync. A captured small
// memset node (4 bytes: the packer's group sums) was seen to leave its bytes unzeroed on hipGraph
// replays interleaved with other device work (tests/test_gpu_packed.py, captured-graph test); a
// kernel node has no such problem and costs the same dispatch.
template <typename T>
__global__ __launch_bounds__(256) void smq_fill_kernel(T* p, T v, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) p[i] = v;
}
template <typename T>
static inline void fill_async(T* p, T v, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(smq_fill_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, v,
                     (uint32_t)n);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads, stores and atomics (__syncthreads' workgroup fence also drains those).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Thread 0 has stored this workgroup's partial with st_sc1_*; count the arrival. Returns the
// pre-increment value in every thread (== expected - 1 in the last workgroup).
__device__ __forceinline__ uint32_t block_arrive(uint32_t* counter, uint32_t* lds_slot) {
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sc1 partial stores have landed
    *lds_slot = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return *lds_slot;
}

// Tagged arrival counter (one lane): one 64-bit word, call tag in the high half, arrivals in the low half.
// The finalising workgroup leaves (next_tag, 0) behind, so the next call on the workspace (whose
// tag the host predicted, arrive_tag() in smaq.hip) finds its own tag and takes the single atomic
// add. A word with another tag (an unzeroed workspace, a call that never finished, another
// workspace sharing the host's tag slot) is stale: the arrival that meets it installs
// (tag, 1) — or joins a tag another stale arrival installed first — by compare-and-swap. The add
// that met the stale word only changed the stale word, which the install overwrites. Returns the
// number of earlier arrivals of this call in every thread (== expected - 1 in the last one).
__device__ __forceinline__ uint32_t arrive_tagged_finish(unsigned long long* ctr, uint32_t tag,
                                                         unsigned long long old) {
  if ((uint32_t)(old >> 32) == tag) return (uint32_t)old;
  // The add met a stale word. One arrival installs (tag, 1); the others then add to the installed
  // word (a bounded number of atomics each: a CAS loop per arrival would cost O(arrivals^2) when
  // every add of a call met the stale word, e.g. adds issued long before they are looked at).
  for (;;) {
    unsigned long long cur = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(cur >> 32) != tag) {
      if (__hip_atomic_compare_exchange_strong(ctr, &cur, ((unsigned long long)tag << 32) | 1ull,
                                               __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        return 0u;
      if ((uint32_t)(cur >> 32) != tag) continue;  // another stale value: look again
    }
    old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(old >> 32) == tag) return (uint32_t)old;
  }
}

// arrive_tagged in two halves: the add (issue it early) and, where the count is needed, the check
// of the word it returned (arrive_tagged_finish).
// An atomic INC (with the bound 2^64 - 1: a plain +1), not an add: the atomic optimizer rewrites a
// lane-divergent add into one wave-level add whose return value it broadcasts to the lanes right
// away — an s_waitcnt vmcnt(0) at the issue, which would stall the issuing wave for the whole
// contended round trip. It leaves inc alone, so the value is waited for only where it is used.
__device__ __forceinline__ unsigned long long arrive_tagged_issue(unsigned long long* ctr) {
  typedef __attribute__((address_space(1))) volatile unsigned long gu64v;
  return __builtin_amdgcn_atomic_inc64((gu64v*)(ctr), ~0ul,
                                       __ATOMIC_RELAXED, "agent");
}

__device__ __forceinline__ uint32_t arrive_tagged(unsigned long long* ctr, uint32_t tag) {
  return arrive_tagged_finish(ctr, tag, arrive_tagged_issue(ctr));
}

// Arrivals of G workgroups sharded by residue: workgroup b adds to sub[(b & 7) * stride] (issued
// with arrive_tagged_issue, `old` its return), the last of each residue adds to `top`. Same-address
// atomics serialise at ~12 ns each (MI355X_MICROARCH.md, fanin): eight words of <= 32 arrivals and
// one of <= 8 instead of one word of 256. True for the call's last arrival.
__device__ __forceinline__ bool arrive_sharded_finish(unsigned long long* top,
                                                      unsigned long long* sub, int stride, int b,
                                                      int G, uint32_t tag, unsigned long long old) {
  const uint32_t s = (uint32_t)b & 7u;
  const uint32_t n_s = ((uint32_t)G - 1u - s) / 8u + 1u;  // workgroups of residue s
  return arrive_tagged_finish(sub + s * stride, tag, old) == n_s - 1u &&
         arrive_tagged(top, tag) == (G < 8 ? (uint32_t)G : 8u) - 1u;
}
__device__ __forceinline__ void rearm_sharded(unsigned long long* top, unsigned long long* sub,
                                              int stride, uint32_t next_tag) {
  const unsigned long long armed = (unsigned long long)next_tag << 32;
  st_sc1_u64(top, armed);
#pragma unroll
  for (int r = 0; r < 8; ++r) st_sc1_u64(sub + r * stride, armed);
}

// The same for a workgroup whose thread 0 stored a partial with st_sc1_*: drain, arrive, and hand
// the count to every thread.
__device__ __forceinline__ uint32_t block_arrive_tagged(unsigned long long* ctr, uint32_t tag,
                                                        uint32_t* lds_slot) {
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sc1 partial stores have landed
    *lds_slot = arrive_tagged(ctr, tag);
  }
  __syncthreads();
  return *lds_slot;
}

// What the finalising workgroup leaves in a tagged counter for the next call.
__device__ __forceinline__ void arrive_reset(unsigned long long* ctr, uint32_t next_tag) {
  *ctr = (unsigned long long)next_tag << 32;
}

// Stats partial of one workgroup: shifted fp64 sums plus fp32 extrema.
struct alignas(32) StatPartial {
  double s1;  // sum (x - shift)
  double s2;  // sum (x - shift)^2
  float mn, mx;
  int64_t cnt;
};

// Workspace layout of a single-tensor SmaQ call.
struct SmaqWsLayout {
  static constexpr size_t kHeader = 64;     // SmqSmaqStats
  static constexpr size_t kDeferRec = kHeader;  // {shift, stream position} (deferred statistics)
  static constexpr size_t kSlots = SMQ_WS_OUTLIER_SLOTS_OFFSET;  // uint64[SMQ_WS_OUTLIER_SLOTS]
  static constexpr size_t kPartials = kSlots + 8 * SMQ_WS_OUTLIER_SLOTS;  // StatPartial[grid]
  // tagged arrival counters, one per tag residue: a call with tag t arrives on word t % kTagWords
  // and leaves (next, 0) in word next % kTagWords. Eager calls take consecutive tags (next = t + 1);
  // a call captured into a graph keeps its tag (next = t), so up to kTagWords calls on one
  // workspace captured into one graph each find their own word on every replay.
  static constexpr size_t kTagCounters = SMQ_WS_SAMPLES_OFFSET + 8 * SMQ_MAX_DEVICE_SAMPLES;
  static constexpr int kTagWords = 64;
  // single-launch round trip (smaq_fused.hip): generation word, the arrival words (one top word,
  // eight per-residue words of workgroups b % 8 == s, each on a 128-B line of its own), then the
  // granules [kFusedRep][256][kFusedWords] of the partials
  static constexpr size_t kFused = SMQ_WS_FUSED_OFFSET;
  static constexpr size_t kFusedGen = kFused;
  static constexpr size_t kFusedLeft = kFused + 128;
  static constexpr size_t kFusedSub = kFused + 256;
  static constexpr size_t kFusedSubStride = 128;
  static constexpr size_t kFusedGran = kFusedSub + 8 * kFusedSubStride;
  static constexpr int kFusedRep = 8;
  static constexpr int kFusedWords = 6;  // s1 low / high, s2 low / high, min, max
  static constexpr size_t kFusedEnd = kFusedGran + 8 * (size_t)kFusedRep * kFusedWords * 256;
  // the PACK variant's per-workgroup aggregates (granule index in replica 0, behind the 4-word
  // partials of 256 workgroups; the range form's 6-word partials, which it never runs with, reach
  // here but carry other calls' epochs)
  static constexpr size_t kFusedPackLook = 1024;
  // a counted call's per-workgroup outlier counts (granule index: replica 1's spare words)
  static constexpr size_t kFusedRecGran = 256 * kFusedWords + 1024;
  static constexpr size_t kTotal = kFusedEnd;
};
static_assert(SmaqWsLayout::kTagCounters + 8 * SmaqWsLayout::kTagWords <= SMQ_WS_FUSED_OFFSET,
              "smq.h SMQ_WS_FUSED_OFFSET overlaps the tag counters");
static_assert(SmaqWsLayout::kFusedEnd <= SMQ_WS_LARGE_SAMPLES_OFFSET,
              "smq.h SMQ_WS_LARGE_SAMPLES_OFFSET overlaps the fused region");

// Inclusive wave64 prefix sum by DPP row shifts and row broadcasts (GFX9 rows of 16 lanes; the
// classic AMDGPU scan: row_shr 1, 2, 4, 8, then row_bcast:15 into rows 1 and 3 and row_bcast:31
// into rows 2 and 3). Six VALU ops; lanes without a source read 0.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}

// OR of each aligned group of 8 lanes, complete in the group's last lane (lane & 7 == 7): three
// DPP row shifts (a group never crosses a 16-lane row).
__device__ __forceinline__ uint32_t group8_or_to_last(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  return v;
}

// Wave64 sum in every lane: the DPP scan, then lane 63's total.
__device__ __forceinline__ uint32_t wave_total_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(v), 63);
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

}  // namespace smq

// Thread-local error reporting shared by all translation units.
namespace smq {
void set_error(const char* fmt, ...);
int check_launch(const char* what);

// Host: the tag a call uses for the tagged arrival counters of workspace `ws` and the tag it leaves
// behind for the next call (block_arrive_tagged). Tags come from a small per-workspace-slot table;
// a wrong prediction costs one compare-and-swap, never a miscount. While `st` is being captured
// into a graph, next == tag, so every replay finds its own tag.
struct ArriveTag {
  uint32_t tag, next;
};
ArriveTag arrive_tag(const void* ws, hipStream_t st);
}  // namespace smq
