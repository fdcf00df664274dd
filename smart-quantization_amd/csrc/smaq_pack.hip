// Packed SmaQ container (include/smq.h "Packed SmaQ container") on gfx950.
//
// compress = statistics (smaq.hip, full or sampled) + the streaming packer (default, code widths
// <= 14 bits; see "streaming packer" below): smaq_code_kernel (one 16-bit record per element and
// the block's image size into its group sum) -> smaq_pack_scan_kernel (group prefixes, header) ->
// smaq_emit_kernel (each block's image at its prefix). No workgroup waits on another.
// SMQ_PACK_SINGLE (and wider codes) take ONE packing launch instead:
//   * each workgroup owns a block of SMQ_PACK_BLOCK = 4096 elements (16 per lane, 4 x dwordx4),
//     quantises them with the same element code as the simulated round trip (smaq_quant), and
//     builds the block image in LDS: outlier mask and the element-order code stream (LDS ORs;
//     ranks from DPP wave scans + per-wave segment prefixes);
//   * blocks are compacted into one dense stream by a decoupled look-back scan: workgroup b packs
//     block b (index order; SMQ_PACK_TICKETED takes ids from an atomic ticket instead), publishes
//     its size, and wave 0 reads up to 64 predecessors' status words per step until it meets an
//     inclusive prefix. Status words are single 64-bit relaxed agent-scope atomics carrying their
//     value, so no fences are needed; a bounded spin turns a would-be hang into header.error;
//   * the block image is written with coalesced stores at its prefix, escapes directly, and the
//     block's word offset into the directory (random-access decode).
// Both give the same bytes.
// decompress = one launch, one workgroup per block: block image -> LDS, mask prefix popcounts,
//   per-element plane reads, escapes via an LDS bitmask + O(1) rank in the block's sorted list,
//   then smaq_dequant — the same arithmetic as the simulated round trip, so the result is
//   bit-identical to smq_smaq_apply for the same statistics and random stream.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "smaq_elem.h"
#include "smaq_host.h"
#include "smq.h"
#include "smq_common.h"

namespace smq {
namespace {

constexpr int kPB = SMQ_PACK_BLOCK;
constexpr int kMaskWords = kPB / 32;            // 128
constexpr int kHdrWords = 1 + kMaskWords;       // w[0] + mask
constexpr int kMaxWidth = 24;                   // widest code (num_bits - 1)
constexpr int kStageWords = kHdrWords + (kMaxWidth * kPB) / 32 + 2;
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;       // ~0.5 s of polling before giving up

static_assert(sizeof(SmqPackedHeader) == 128, "packed header layout");

struct PackArgs {
  const void* x;
  int64_t n;
  SmqPackedHeader* hdr;
  uint64_t* dir;
  uint32_t* data;
  const SmqSmaqStats* stats;
  uint64_t* status;          // [n_blocks] block aggregates
  uint64_t* gstatus;         // [n_groups] group aggregates / inclusive prefixes
  uint32_t* counter;
  float thr, r_main, r_out;
  double inv_r_main, inv_r_out;
  uint32_t key;
  uint64_t offset;
  int wm, wo, bm, bo;
  uint32_t n_blocks;
  uint32_t n_full;           // blocks of SMQ_PACK_BLOCK elements (the main launch)
  int ticketed;              // SMQ_PACK_TICKETED: block ids from an atomic ticket
  uint32_t flags;
  int place_atomic;          // measurement knob (SMQ_PACK_PLACE=atomic): see smq_smaq_compress
  uint32_t stage_words;      // LDS stage (w[0], mask, code stream) for these widths; q values follow
  unsigned long long* cursor;
  // streaming packer (smaq_code_kernel / smaq_pack_scan_kernel / smaq_emit_kernel)
  uint16_t* rec;             // [n_blocks * SMQ_PACK_BLOCK] element records
  uint32_t* meta;            // [n_blocks] n_out | n_esc << 16
  uint32_t* gsum;            // [n_groups] image words of each group of kGroup blocks
  uint64_t* gpre;            // [n_groups] exclusive prefix of gsum
  uint32_t n_groups;
};

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Plane code of one element (smq.h rules), branch-free; esc = the code does not fit the budget.
__device__ __forceinline__ uint32_t classify(float q, bool hi, bool lo, int wm, int wo, bool& esc) {
  const bool o = hi | lo;
  const float lim = (float)(1 << (wm - 1));
  const bool ok_m = (q >= -lim) && (q <= lim - 1.0f);          // false for NaN
  const float mag = hi ? q : -q;                                // hi: q >= 0, lo: q <= 0
  const bool ok_o = (mag >= 0.0f) && (mag <= (float)((1 << (wo - 1)) - 1));
  const uint32_t code_m = (uint32_t)(int32_t)q & ((1u << wm) - 1u);
  const uint32_t code_o = (lo ? (1u << (wo - 1)) : 0u) | (ok_o ? (uint32_t)(int32_t)mag : 0u);
  const bool ok = o ? ok_o : ok_m;
  esc = !ok;
  return o ? code_o : (ok_m ? code_m : 0u);
}

constexpr int kGroup = 64;  // blocks per look-back group (one status word per lane)

// Poll until lanes [0, count) hold a published status (flag != 0); returns this lane's value.
__device__ __forceinline__ uint64_t wait_all(const PackArgs& A, const uint64_t* st, int count,
                                             uint32_t& spins) {
  const int lane = threadIdx.x & (kWave - 1);
  for (;;) {
    const uint64_t v = lane < count ? ld_sc1_u64(st + lane) : kAgg;
    if (!__ballot((v >> 62) == 0ull)) return v;
    if (++spins >= kSpinLimit) {
      if (lane == 0) atomicOr(&A.hdr->error, 1u);  // give up: the stream is marked broken
      return v;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Two-level decoupled look-back (wave 0). Returns the exclusive prefix (words) of block b.
// Level 1: the blocks of b's group of 64 publish their sizes (one window read). Level 2: the
// group's last block publishes the group aggregate, walks back over group words (64 groups =
// 4096 blocks per read) to the nearest inclusive prefix and publishes its own; every block of the
// group walks the same group words. A single-level scan advances one 64-block window per memory
// round trip (~1 us): 65536 blocks took 1.1 ms; two levels move 4096 blocks per round trip.
__device__ uint64_t look_back(const PackArgs& A, uint32_t b, uint64_t size) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t g = b / kGroup, i = b % kGroup;
  const bool last = (i == kGroup - 1) || (b == A.n_blocks - 1);
  uint32_t spins = 0;
  if (lane == 0) st_sc1_u64(A.status + b, kAgg | size);
  // level 1: sizes of the group's earlier blocks
  uint64_t lp = 0;
  if (i > 0) {
    const uint64_t v = wait_all(A, A.status + (uint64_t)g * kGroup, (int)i, spins);
    lp = wave_sum_u64(lane < (int)i ? (v & kValMask) : 0ull);
  }
  if (last && lane == 0) st_sc1_u64(A.gstatus + g, (g == 0 ? kIncl : kAgg) | (lp + size));
  // level 2: prefix of the groups before g
  uint64_t gp = 0;
  if (g > 0) {
    int64_t j = (int64_t)g - 1;
    for (;;) {
      const int64_t idx = j - lane;
      const uint64_t v = idx >= 0 ? ld_sc1_u64(A.gstatus + idx) : kIncl;  // before group 0: 0
      const uint32_t flag = (uint32_t)(v >> 62);
      const uint64_t incl = __ballot(flag == 2u);
      const uint64_t invalid = __ballot(flag == 0u);
      const int first = incl ? __builtin_ctzll(incl) : 64;
      const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);  // lanes 0..first
      if ((invalid & need) && ++spins < kSpinLimit) {
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      if (spins >= kSpinLimit && lane == 0) atomicOr(&A.hdr->error, 1u);
      gp += wave_sum_u64(lane <= first ? (v & kValMask) : 0ull);
      if (first < 64 || spins >= kSpinLimit) break;
      j -= 64;
    }
    if (last && lane == 0) st_sc1_u64(A.gstatus + g, kIncl | (gp + lp + size));
  }
  return gp + lp;
}

// OR a code chunk (< 2^32) at bit pos of an LDS bit stream (two words; ORing 0 is harmless).
__device__ __forceinline__ void or_bits(uint32_t* base, uint32_t pos, uint32_t chunk) {
  const uint64_t v = (uint64_t)chunk << (pos & 31u);
  atomicOr(base + (pos >> 5), (uint32_t)v);
  atomicOr(base + (pos >> 5) + 1, (uint32_t)(v >> 32));
}

// FULL: the block holds SMQ_PACK_BLOCK elements (every block but a ragged last one).
// WM / WO: code widths compiled in (0: runtime widths). With WO <= 8 a lane's four codes form one
// chunk of at most 28 bits written by two LDS ORs.
template <int RM, int TIN, bool SUB, bool VEC, bool FULL, int WM, int WO>
__device__ __forceinline__ void pack_body(const PackArgs& A, const ElemConsts& c, uint32_t b,
                                          uint32_t* stage, float* qlds) {
  __shared__ uint32_t seg_cnt[2][16];
  __shared__ uint32_t seg_pre[2][17];
  __shared__ uint64_t s_prefix;
  constexpr bool kChunk = WO > 0 && WO <= 8;
  const int wm = WM > 0 ? WM : A.wm, wo = WO > 0 ? WO : A.wo;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  uint32_t* codes_lds = stage + kHdrWords;

  // 1. codes of this lane's 16 elements: local index el = 1024 k + 4 tid + i. Every q also goes to
  //    LDS (one 16-B store per float4): the escape list reads it back after the scan (re-deriving
  //    it cost a reload + the element chain; keeping it in registers cost occupancy)
  uint32_t code[16];
  uint32_t om[4], xm[4];
  // all four 16-B loads of the lane in flight before any element is processed
  float xv[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    if (VEC && (FULL || el + 3 < n_el)) {
      const float4 t = load4_stream<TIN>(A.x, (e0 + el) >> 2);
      xv[k][0] = t.x; xv[k][1] = t.y; xv[k][2] = t.z; xv[k][3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        xv[k][i] = (FULL || el + i < n_el) ? load1<TIN>(A.x, e0 + el + i) : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    float u[4] = {0.f, 0.f, 0.f, 0.f};
    const float* v = xv[k];
    const bool full4 = FULL || el + 3 < n_el;
    if (RM == kRoundHash) {
      const uint64_t ctr = A.offset + c.rng_off + (uint64_t)(e0 + el);
      if (full4) {
        rng_hu4(A.key, ctr, u[0], u[1], u[2], u[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (el + i < n_el) u[i] = rng_hu(A.key, ctr + i);
      }
    }
    om[k] = 0u;
    xm[k] = 0u;
    float qk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hi, lo, esc = false;
      const float q = smaq_quant<RM, false, TIN, SUB>(v[i], u[i], c, hi, lo);
      const bool valid = FULL || el + i < n_el;
      code[4 * k + i] = valid ? classify(q, hi, lo, wm, wo, esc) : 0u;
      qk[i] = q;
      om[k] |= (uint32_t)((hi | lo) && valid) << i;
      xm[k] |= (uint32_t)(esc && valid) << i;
    }
    *reinterpret_cast<float4*>(qlds + el) = make_float4(qk[0], qk[1], qk[2], qk[3]);
  }

  // 2. outlier / escape ranks: per 256-element segment s = 4 k + wave, lane prefixes by ballots;
  //    mask words from nibbles (8 lanes per word) by three xor-shuffles
  uint32_t pre_o[4], pre_x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t cnt = (uint32_t)__popc(om[k]) | ((uint32_t)__popc(xm[k]) << 16);
    const uint32_t incl = wave_incl_scan_u32(cnt);
    const uint32_t ex = incl - cnt;
    pre_o[k] = ex & 0xffffu;
    pre_x[k] = ex >> 16;
    const uint32_t mw = group8_or_to_last(om[k] << (4 * (lane & 7)));
    if ((lane & 7) == 7) stage[1 + ((1024 * k + 4 * (tid - 7)) >> 5)] = mw;
    if (lane == kWave - 1) {
      seg_cnt[0][4 * k + w] = incl & 0xffffu;
      seg_cnt[1][4 * k + w] = incl >> 16;
    }
  }
  const uint32_t code_cap = A.stage_words - kHdrWords;
  for (uint32_t i = tid; i < code_cap; i += kBlock) codes_lds[i] = 0u;
  __syncthreads();
  if (tid < 2) {
    uint32_t run = 0;
    for (int s = 0; s < 16; ++s) {
      seg_pre[tid][s] = run;
      run += seg_cnt[tid][s];
    }
    seg_pre[tid][16] = run;
  }
  __syncthreads();
  const uint32_t n_out = seg_pre[0][16], n_esc = seg_pre[1][16];
  const uint32_t code_words = ((uint32_t)wm * (uint32_t)n_el + (uint32_t)(wo - wm) * n_out + 31u) / 32u;
  const uint32_t img_words = kHdrWords + code_words;
  const uint64_t size = (uint64_t)img_words + 2ull * n_esc;

  // 3. wave 0 starts the look-back; every lane ORs its codes into the LDS code stream at
  //    pos(el) = wm * el + (wo - wm) * (outliers before el)
  if (A.place_atomic) {
    if (tid == 0) s_prefix = atomicAdd(A.cursor, (unsigned long long)size);
  } else if (w == 0) {
    const uint64_t p = look_back(A, b, size);
    if (lane == 0) s_prefix = p;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t el0 = 1024u * k + 4u * tid;
    if (!FULL && (int)el0 >= n_el) continue;
    const uint32_t r0 = seg_pre[0][4 * k + w] + pre_o[k];
    const uint32_t pos0 = (uint32_t)wm * el0 + (uint32_t)(wo - wm) * r0;
    if (kChunk) {
      uint32_t chunk = 0u, off = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        chunk |= code[4 * k + i] << off;  // invalid tail elements carry code 0, width wm
        off += ((om[k] >> i) & 1u) ? (uint32_t)wo : (uint32_t)wm;
      }
      or_bits(codes_lds, pos0, chunk);
    } else {
      uint32_t off = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        or_bits(codes_lds, pos0 + off, code[4 * k + i]);
        off += ((om[k] >> i) & 1u) ? (uint32_t)wo : (uint32_t)wm;
      }
    }
  }
  __syncthreads();

  // 4. the block image at its prefix, its escapes and directory entry
  const uint64_t P = s_prefix;
  uint32_t* out = A.data + P;
  for (uint32_t i = tid; i < img_words; i += kBlock)
    out[i] = i == 0 ? (n_out | (n_esc << 16)) : stage[i];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!xm[k]) continue;
    const uint32_t base_x = seg_pre[1][4 * k + w] + pre_x[k];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!((xm[k] >> i) & 1u)) continue;
      const uint32_t r = base_x + __popc(xm[k] & ((1u << i) - 1u));
      out[img_words + 2 * r] = 1024u * k + 4u * tid + i;
      out[img_words + 2 * r + 1] = __float_as_uint(qlds[1024u * k + 4u * tid + i]);
    }
  }
  if (tid == 0) {
    // directory entry: word offset (38 bits) | n_out << 38 | n_esc << 51 (decoder: no dependent
    // load of w[0] before the block image)
    A.dir[b] = P | ((uint64_t)n_out << 38) | ((uint64_t)n_esc << 51);
    if (!A.place_atomic && b == A.n_blocks - 1) {
      A.hdr->data_words = P + size;
      A.hdr->total_bytes = sizeof(SmqPackedHeader) + 8ull * A.n_blocks + 4ull * (P + size);
    }
    if (b == 0) {
      SmqPackedHeader* h = A.hdr;
      h->magic = SMQ_PACK_MAGIC;
      h->version = SMQ_PACK_VERSION;
      h->n = A.n;
      h->block_elems = kPB;
      h->n_blocks = A.n_blocks;
      h->num_bits_main = A.bm;
      h->num_bits_outlier = A.bo;
      h->flags = A.flags;
      h->thr = A.thr;
      h->range_main = A.r_main;
      h->range_outlier = A.r_out;
      h->mean = c.mean;
      h->std_dev = c.sd;
      h->inv_range_main = A.inv_r_main;
      h->inv_range_outlier = A.inv_r_out;
    }
  }
}

// One kernel per (widths, full/ragged), chosen on the host, each with ONE body: with the eight
// (quot_check x full x widths) bodies in one kernel the uniform constants spilled 568 SGPRs
// (v_writelane / v_readlane traffic on the VALU) and took 104 VGPRs.
// FULL: the main launch, blocks of SMQ_PACK_BLOCK elements. !FULL: the ragged last
// block, launched as one workgroup after the main launch (its look-back finds every predecessor
// published).
template <int RM, int TIN, bool VEC, bool FULL, int WM, int WO>
__global__ __launch_bounds__(kBlock) void smaq_pack_kernel(PackArgs A) {
  extern __shared__ uint32_t pack_lds[];  // [stage_words] stage, then [kPB] q values
  uint32_t* stage = pack_lds;
  float* qlds = reinterpret_cast<float*>(pack_lds + A.stage_words);
  uint32_t b;
  if (FULL) {
    if (A.ticketed) {  // block ids in start order: predecessors are resident by construction
      __shared__ uint32_t s_b;
      if (threadIdx.x == 0) {
        const uint32_t id = atomicAdd(A.counter, 1u);
        if (id == A.n_full - 1) atomicExch(A.counter, 0u);  // every id is taken: reset for reuse
        s_b = id;
      }
      __syncthreads();
      b = s_b;
    } else {  // index order (see SMQ_PACK_TICKETED in smq.h)
      b = blockIdx.x;
    }
  } else {
    b = A.n_blocks - 1;
  }
  ElemConsts c;
  const float cthr = (TIN == kF32) ? A.thr : round_in<TIN>(A.thr);  // z is compared in its type
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  // SUB = true regardless of stats->quot_check: the IEEE re-division of a subnormal quotient is
  // exact either way, and one body (no device-side dispatch) keeps the constants in registers
  pack_body<RM, TIN, true, VEC, FULL, WM, WO>(A, c, b, stage, qlds);
}

template <int RM, int TIN>
void launch_pack(const PackArgs& A, bool vec, size_t lds, hipStream_t st) {
  const bool w57 = A.wm == 5 && A.wo == 7;  // the default 6/8-bit budget, widths compiled in
  const dim3 grid(A.n_full), block(kBlock);
  if (A.n_full > 0) {
    if (vec) {
      if (w57) hipLaunchKernelGGL((smaq_pack_kernel<RM, TIN, true, true, 5, 7>), grid, block, lds, st, A);
      else hipLaunchKernelGGL((smaq_pack_kernel<RM, TIN, true, true, 0, 0>), grid, block, lds, st, A);
    } else {
      if (w57) hipLaunchKernelGGL((smaq_pack_kernel<RM, TIN, false, true, 5, 7>), grid, block, lds, st, A);
      else hipLaunchKernelGGL((smaq_pack_kernel<RM, TIN, false, true, 0, 0>), grid, block, lds, st, A);
    }
  }
  if (A.n_full < A.n_blocks)
    hipLaunchKernelGGL((smaq_pack_kernel<RM, TIN, false, false, 0, 0>), dim3(1), block, lds, st, A);
}

// ---- streaming packer (the default when both code widths are <= kRecCodeBits) ----------------
// The single packing launch above chains load -> quantise -> rank scan -> look-back -> image per
// block in one workgroup; PMC showed it latency-bound (57 % of wave time in s_waitcnt / barriers,
// VALU ~50 % busy). Here the same bytes come from three plain streaming launches, none of which
// waits on another workgroup:
//   1. smaq_code_kernel — one workgroup per block quantises its elements with pack_body's element
//      code (same smaq_quant / classify) and writes one 16-bit record per element: bit 15 outlier,
//      bit 14 escape; a plane code in bits 0-13, or for an escape the side (z < -T) in bit 13 and q
//      in bits 0-12 (two's complement; kRecBig = q outside [-4095, 4095] or not finite: the emitter
//      re-derives q from x). It adds the block's image size to its group sum (one atomic per
//      workgroup, 64 blocks per group) and stores n_out | n_esc.
//   2. smaq_pack_scan_kernel — one workgroup: exclusive scan of the group sums (zeroed by a
//      memset before phase 1), writes the header.
//   3. smaq_emit_kernel — one workgroup per block: prefix = its group's prefix + the sizes of its
//      group predecessors (one load per lane), records -> ranks -> LDS code stream -> block image.
// Traffic: 4 B/elem read + 2 B/elem records written, 2 B/elem records read + the stream written.
constexpr int kRecCodeBits = 14;
constexpr int kRecBig = -4096;

__device__ __forceinline__ uint32_t block_image_words(int wm, int wo, uint32_t n_el, uint32_t n_out) {
  return (uint32_t)kHdrWords + ((uint32_t)wm * n_el + (uint32_t)(wo - wm) * n_out + 31u) / 32u;
}

// Record of one element: classify()'s plane code / escape decision in integer ops (fewer selects).
// v = q + 2^(wm-1) for a main (fits: v < 2^wm), |q| on the element's side for an outlier (fits:
// v < 2^(wo-1)); |q| > 2^24, inf and NaN always escape (widths are at most 14 bits here). An
// escape record carries q when |q| <= 4095, else kRecBig (the emitter re-derives q).
__device__ __forceinline__ uint32_t record_of(float q, bool hi, bool lo, int wm, int wo, bool& esc) {
  const bool o = hi | lo;
  const int qi = (__builtin_fabsf(q) <= 0x1p24f) ? (int)q : -(1 << 30);
  const uint32_t half_m = 1u << (wm - 1), side = 1u << (wo - 1);
  const uint32_t v = (uint32_t)(lo ? -qi : (o ? qi : qi + (int)half_m));
  const uint32_t lim = o ? side : 2u * half_m;
  esc = !(v < lim);
  const uint32_t code = o ? ((lo ? side : 0u) | v) : (v ^ half_m);
  const int qe = ((uint32_t)(qi + 4095) <= 8190u) ? qi : kRecBig;
  return esc ? (0x4000u | ((uint32_t)o << 15) | ((uint32_t)lo << 13) | ((uint32_t)qe & 0x1fffu))
             : (((uint32_t)o << 15) | code);
}

// Records of one lane's 16 elements (smaq_code_kernel); returns its outliers | escapes << 16.
template <int RM, int TIN, bool FULL, bool SUB>
__device__ __forceinline__ uint32_t code_records(const PackArgs& A, const ElemConsts& c,
                                                 const float (&xv)[4][4], int64_t e0, int n_el,
                                                 int wm, int wo) {
  const int tid = threadIdx.x;
  uint32_t cnt = 0;  // outliers (bits 0-15) | escapes (bits 16-31) of this lane's elements
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    const bool full4 = FULL || el + 3 < n_el;
    float u[4] = {0.f, 0.f, 0.f, 0.f};
    if (RM == kRoundHash) {
      const uint64_t ctr = A.offset + c.rng_off + (uint64_t)(e0 + el);
      if (full4) {
        rng_hu4(A.key, ctr, u[0], u[1], u[2], u[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (el + i < n_el) u[i] = rng_hu(A.key, ctr + i);
      }
    }
    uint32_t r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hi, lo, esc;
      const float q = smaq_quant<RM, false, TIN, SUB>(xv[k][i], u[i], c, hi, lo);
      r[i] = record_of(q, hi, lo, wm, wo, esc);
      const bool o = hi | lo;
      const bool valid = FULL || el + i < n_el;
      cnt += valid ? ((uint32_t)o | ((uint32_t)esc << 16)) : 0u;
    }
    uint16_t* dst = A.rec + e0 + el;
    if (full4) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(r[0] | (r[1] << 16), r[2] | (r[3] << 16));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (el + i < n_el) dst[i] = (uint16_t)r[i];
    }
  }
  return cnt;
}

// One workgroup per block (half-block workgroups, the second to finish adding the block's size,
// measured 357 vs 338 us at 256M).
template <int RM, int TIN, bool VEC, bool FULL, int WM, int WO>
__global__ __launch_bounds__(kBlock) void smaq_code_kernel(PackArgs A) {
  __shared__ uint32_t s_cnt[kBlock / kWave];
  const int wm = WM > 0 ? WM : A.wm, wo = WO > 0 ? WO : A.wo;
  // blocks in reverse address order: the statistics sweep just read x front to back, so its tail
  // is still in the Infinity Cache (331 vs 335 us); the emitter then walks forward
  const uint32_t b = FULL ? A.n_full - 1 - blockIdx.x : A.n_blocks - 1;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  ElemConsts c;
  const float cthr = (TIN == kF32) ? A.thr : round_in<TIN>(A.thr);
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  float xv[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    if (VEC && (FULL || el + 3 < n_el)) {
      const float4 t = load4_stream<TIN>(A.x, (e0 + el) >> 2);
      xv[k][0] = t.x; xv[k][1] = t.y; xv[k][2] = t.z; xv[k][3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        xv[k][i] = (FULL || el + i < n_el) ? load1<TIN>(A.x, e0 + el + i) : 0.f;
    }
  }
  // the subnormal-quotient check only where quot_check_for() asks for it (one uniform branch
  // per workgroup; the x loads above are already in flight)
  const uint32_t cnt = A.stats->quot_check
      ? code_records<RM, TIN, FULL, true>(A, c, xv, e0, n_el, wm, wo)
      : code_records<RM, TIN, FULL, false>(A, c, xv, e0, n_el, wm, wo);
  const uint32_t tot = wave_total_u32(cnt);
  if (lane == 0) s_cnt[w] = tot;
  __syncthreads();
  if (tid == 0) {
    const uint32_t t = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
    A.meta[b] = t;
    atomicAdd(A.gsum + b / kGroup,
              block_image_words(wm, wo, (uint32_t)n_el, t & 0xffffu) + 2u * (t >> 16));
  }
}

constexpr int kScanThreads = 1024;

__global__ __launch_bounds__(kScanThreads) void smaq_pack_scan_kernel(PackArgs A) {
  __shared__ uint64_t s_wave[kScanThreads / kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  uint64_t carry = 0;
  for (uint32_t base = 0; base < A.n_groups; base += 4u * kScanThreads) {
    uint32_t v[4];
    uint64_t loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t g = base + 4u * tid + j;
      v[j] = g < A.n_groups ? A.gsum[g] : 0u;
      loc += v[j];
    }
    uint64_t inc = loc;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint64_t t = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += t;
    }
    if (lane == kWave - 1) s_wave[w] = inc;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kScanThreads / kWave; ++i) {
      const uint64_t s = s_wave[i];
      wpre += i < w ? s : 0ull;
      total += s;
    }
    uint64_t run = carry + wpre + (inc - loc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t g = base + 4u * tid + j;
      if (g < A.n_groups) A.gpre[g] = run;
      run += v[j];
    }
    carry += total;
    __syncthreads();
  }
  if (tid == 0) {
    SmqPackedHeader* h = A.hdr;
    const SmqSmaqStats* st = A.stats;
    h->magic = SMQ_PACK_MAGIC;
    h->version = SMQ_PACK_VERSION;
    h->n = A.n;
    h->block_elems = kPB;
    h->n_blocks = A.n_blocks;
    h->num_bits_main = A.bm;
    h->num_bits_outlier = A.bo;
    h->flags = A.flags;
    h->thr = A.thr;
    h->range_main = A.r_main;
    h->range_outlier = A.r_out;
    h->mean = st->mean;
    h->std_dev = st->std_dev;
    h->inv_range_main = A.inv_r_main;
    h->inv_range_outlier = A.inv_r_out;
    h->data_words = carry;
    h->total_bytes = sizeof(SmqPackedHeader) + 8ull * A.n_blocks + 4ull * carry;
    h->error = 0u;
#pragma unroll
    for (int i = 0; i < 9; ++i) h->reserved[i] = 0u;
  }
}

// q of one element re-derived from x (an escape whose q does not fit its record: |q| > 4095, inf,
// NaN), with pack_body's element code.
template <int RM, int TIN>
__device__ __forceinline__ float rederive_q(const PackArgs& A, int64_t e) {
  ElemConsts c;
  const float cthr = (TIN == kF32) ? A.thr : round_in<TIN>(A.thr);
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  const float u = (RM == kRoundHash) ? rng_hu(A.key, A.offset + c.rng_off + (uint64_t)e) : 0.0f;
  bool hi, lo;
  return smaq_quant<RM, false, TIN, true>(load1<TIN>(A.x, e), u, c, hi, lo);
}

// OR a code chunk of up to 64 bits at bit pos of an LDS bit stream (two or three words; the third
// only when bits land there, so it never passes the image; ORing 0 into the second is harmless).
__device__ __forceinline__ void or_bits64(uint32_t* base, uint32_t pos, uint64_t chunk) {
  const uint32_t sft = pos & 31u, w0 = pos >> 5;
  const uint64_t lo = chunk << sft;
  const uint32_t hi = sft ? (uint32_t)(chunk >> (64u - sft)) : 0u;
  atomicOr(base + w0, (uint32_t)lo);
  atomicOr(base + w0 + 1, (uint32_t)(lo >> 32));
  if (hi) atomicOr(base + w0 + 2, hi);
}

// OR of each aligned group of 4 lanes, complete in the group's last lane (lane & 3 == 3).
__device__ __forceinline__ uint32_t group4_or_to_last(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  return v;
}

// Emitter lane layout: lane t of the workgroup owns elements 2048 k + 8 t + i (k = 0, 1; i < 8), so
// its 8 records per k are one 16-B load (8-B loads of 4 records ran at ~0.6x the 16-B rate) and one
// 64-bit code chunk; segment 4 k + w (wave w) covers 512 consecutive elements.
constexpr int kEmitK = 2;
constexpr int kEmitE = 8;

template <int RM, int TIN, bool FULL, int WM, int WO>
__global__ __launch_bounds__(kBlock) void smaq_emit_kernel(PackArgs A) {
  extern __shared__ uint32_t stage[];  // [stage_words]: w[0], mask, code stream
  __shared__ uint32_t seg_cnt[kEmitK * kBlock / kWave];
  __shared__ uint64_t s_prefix;
  constexpr bool kChunk = WO > 0 && WO <= 8;
  const int wm = WM > 0 ? WM : A.wm, wo = WO > 0 ? WO : A.wo;
  const uint32_t b = FULL ? blockIdx.x : A.n_blocks - 1;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  uint32_t* codes_lds = stage + kHdrWords;

  // records of this lane's 16 elements, two per register
  uint32_t rw[kEmitK][4];
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    const int el = 2048 * k + kEmitE * tid;
    if (FULL || el + kEmitE <= n_el) {
      const uint4 t = *reinterpret_cast<const uint4*>(A.rec + e0 + el);
      rw[k][0] = t.x;
      rw[k][1] = t.y;
      rw[k][2] = t.z;
      rw[k][3] = t.w;
    } else {
      uint32_t r[kEmitE];
#pragma unroll
      for (int i = 0; i < kEmitE; ++i) r[i] = (el + i < n_el) ? (uint32_t)A.rec[e0 + el + i] : 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) rw[k][j] = r[2 * j] | (r[2 * j + 1] << 16);
    }
  }
  // block prefix: the group's prefix + the sizes of the group's earlier (full) blocks
  if (w == 0) {
    const uint32_t g = b / kGroup, j = g * kGroup + lane;
    uint32_t sz = 0u;
    if (j < b) {
      const uint32_t t = A.meta[j];
      sz = block_image_words(wm, wo, kPB, t & 0xffffu) + 2u * (t >> 16);
    }
    sz = wave_total_u32(sz);
    if (lane == 0) s_prefix = A.gpre[g] + sz;
  }

  auto rec = [&](int k, int i) -> uint32_t { return (rw[k][i >> 1] >> (16 * (i & 1))) & 0xffffu; };
  // outlier / escape bits per 8-element group (the codes themselves are decoded when placed)
  uint32_t om[kEmitK], xm[kEmitK];
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    om[k] = 0u;
    xm[k] = 0u;
#pragma unroll
    for (int i = 0; i < kEmitE; ++i) {
      const uint32_t r = rec(k, i);
      om[k] |= (r >> 15) << i;
      xm[k] |= ((r >> 14) & 1u) << i;
    }
  }
  auto code_of = [&](int k, int i) -> uint32_t {
    const uint32_t r = rec(k, i);
    const uint32_t side_code = ((r >> 13) & (r >> 15) & 1u) << (wo - 1);
    return ((r >> 14) & 1u) ? side_code : (r & 0x3fffu);
  };

  // ranks, mask words and the LDS code stream: outlier and escape counts packed in one word (each
  // <= 512 per wave) and scanned together by DPP; a mask word is the OR of 4 lanes' bytes, written
  // by each group's last lane
  uint32_t pre_o[kEmitK], pre_x[kEmitK];
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    const uint32_t cnt = (uint32_t)__popc(om[k]) | ((uint32_t)__popc(xm[k]) << 16);
    const uint32_t incl = wave_incl_scan_u32(cnt);
    const uint32_t ex = incl - cnt;
    pre_o[k] = ex & 0xffffu;
    pre_x[k] = ex >> 16;
    const uint32_t mw = group4_or_to_last(om[k] << (8 * (lane & 3)));
    if ((lane & 3) == 3) stage[1 + ((2048 * k + kEmitE * (tid - 3)) >> 5)] = mw;
    if (lane == kWave - 1) seg_cnt[4 * k + w] = incl;
  }
  const uint32_t code_cap = A.stage_words - kHdrWords;
  for (uint32_t i = tid; i < code_cap; i += kBlock) codes_lds[i] = 0u;
  __syncthreads();
  // every wave derives its segment prefixes from the 8 counts itself (no serial scan and no
  // second barrier): segment 4 k + w starts after segments 0 .. 4 k + w - 1 (lane s < 8 holds
  // segment s's counts packed as outliers | escapes << 16, each <= 2048)
  const uint32_t own = lane < kEmitK * 4 ? seg_cnt[lane] : 0u;
  uint32_t incl = own;  // lanes 0-7 scanned by DPP row shifts
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xf, 0xf, false);
  const uint32_t excl = incl - own;
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, kEmitK * 4 - 1);
  const uint32_t n_out = tot & 0xffffu, n_esc = tot >> 16;
  uint32_t base_o[kEmitK], base_x[kEmitK];
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    const uint32_t b4 = (uint32_t)__builtin_amdgcn_readlane((int)excl, 4 * k + w);
    base_o[k] = b4 & 0xffffu;
    base_x[k] = b4 >> 16;
  }
  const uint32_t img_words = block_image_words(wm, wo, (uint32_t)n_el, n_out);
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    const uint32_t el0 = 2048u * k + kEmitE * tid;
    if (!FULL && (int)el0 >= n_el) continue;
    const uint32_t r0 = base_o[k] + pre_o[k];
    const uint32_t pos0 = (uint32_t)wm * el0 + (uint32_t)(wo - wm) * r0;
    if (kChunk) {
      uint64_t chunk = 0u;
      uint32_t off = 0u;
#pragma unroll
      for (int i = 0; i < kEmitE; ++i) {
        chunk |= (uint64_t)code_of(k, i) << off;
        off += ((om[k] >> i) & 1u) ? (uint32_t)wo : (uint32_t)wm;
      }
      or_bits64(codes_lds, pos0, chunk);
    } else {
      uint32_t off = 0u;
#pragma unroll
      for (int i = 0; i < kEmitE; ++i) {
        or_bits(codes_lds, pos0 + off, code_of(k, i));
        off += ((om[k] >> i) & 1u) ? (uint32_t)wo : (uint32_t)wm;
      }
    }
  }
  __syncthreads();

  // the block image at its prefix, its escapes and directory entry
  const uint64_t P = s_prefix;
  uint32_t* out = A.data + P;
  for (uint32_t i = tid; i < img_words; i += kBlock)
    out[i] = i == 0 ? (n_out | (n_esc << 16)) : stage[i];
#pragma unroll
  for (int k = 0; k < kEmitK; ++k) {
    if (!xm[k]) continue;
    const uint32_t bx = base_x[k] + pre_x[k];
#pragma unroll
    for (int i = 0; i < kEmitE; ++i) {
      if (!((xm[k] >> i) & 1u)) continue;
      const uint32_t el = 2048u * k + kEmitE * tid + i;
      const uint32_t r = bx + __popc(xm[k] & ((1u << i) - 1u));
      const int qi = (int)((rec(k, i) & 0x1fffu) << 19) >> 19;
      const float q = qi == kRecBig ? rederive_q<RM, TIN>(A, e0 + el) : (float)qi;
      out[img_words + 2 * r] = el;
      out[img_words + 2 * r + 1] = __float_as_uint(q);
    }
  }
  if (tid == 0) A.dir[b] = P | ((uint64_t)n_out << 38) | ((uint64_t)n_esc << 51);
}

template <int RM, int TIN>
void launch_streaming_pack(const PackArgs& A, bool vec, size_t stage_lds, hipStream_t st) {
  const bool w57 = A.wm == 5 && A.wo == 7;
  const dim3 grid(A.n_full), block(kBlock);
  if (A.n_full > 0) {
    if (vec) {
      if (w57) hipLaunchKernelGGL((smaq_code_kernel<RM, TIN, true, true, 5, 7>), grid, block, 0, st, A);
      else hipLaunchKernelGGL((smaq_code_kernel<RM, TIN, true, true, 0, 0>), grid, block, 0, st, A);
    } else {
      if (w57) hipLaunchKernelGGL((smaq_code_kernel<RM, TIN, false, true, 5, 7>), grid, block, 0, st, A);
      else hipLaunchKernelGGL((smaq_code_kernel<RM, TIN, false, true, 0, 0>), grid, block, 0, st, A);
    }
  }
  if (A.n_full < A.n_blocks)
    hipLaunchKernelGGL((smaq_code_kernel<RM, TIN, false, false, 0, 0>), dim3(1), block, 0, st, A);
  hipLaunchKernelGGL(smaq_pack_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, A);
  if (A.n_full > 0) {
    if (w57) hipLaunchKernelGGL((smaq_emit_kernel<RM, TIN, true, 5, 7>), grid, block, stage_lds, st, A);
    else hipLaunchKernelGGL((smaq_emit_kernel<RM, TIN, true, 0, 0>), grid, block, stage_lds, st, A);
  }
  if (A.n_full < A.n_blocks)
    hipLaunchKernelGGL((smaq_emit_kernel<RM, TIN, false, 0, 0>), dim3(1), block, stage_lds, st, A);
}

// SMQ_PACK_PLACE=atomic: the stream size is the cursor (written after the packing launch).
__global__ void smaq_pack_total_kernel(SmqPackedHeader* h, const unsigned long long* cursor,
                                       uint32_t n_blocks) {
  if (threadIdx.x == 0) {
    h->data_words = *cursor;
    h->total_bytes = sizeof(SmqPackedHeader) + 8ull * n_blocks + 4ull * *cursor;
  }
}

struct UnpackArgs {
  const SmqPackedHeader* hdr;
  const uint64_t* dir;
  const uint32_t* data;
  float* y;
  int64_t n;
  int vec;
  int reverse;  // blocks in reverse order (smq_smaq_decompress)
};

// Escapes before element el of a block: the list is sorted by element index (lower bound).
__device__ __forceinline__ uint32_t escapes_below(const uint32_t* esc, uint32_t n_esc, uint32_t el) {
  uint32_t lo = 0, hi = n_esc;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (esc[2 * mid] < el) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Decode one code (width wm main / wo outlier) to q and the outlier sides.
__device__ __forceinline__ float decode_code(uint32_t v, bool is_o, int wm, int wo, bool& hi,
                                             bool& lo) {
  const uint32_t side_bit = 1u << (wo - 1);
  const uint32_t cm = v & ((1u << wm) - 1u);
  const float qm = (float)(((int32_t)(cm << (32 - wm))) >> (32 - wm));  // sign-extend
  const int mag = (int)(v & (side_bit - 1u));
  lo = is_o && (v & side_bit);
  hi = is_o && !(v & side_bit);
  return is_o ? (float)(lo ? -mag : mag) : qm;
}

// pc / epc / esc_mask: kMaskWords LDS words each, declared once by the kernel (a __shared__ array
// inside this template is one allocation PER INSTANTIATION: 16 bodies took 37 KB of LDS per
// workgroup, 4 workgroups per CU)
// Decode table of narrow codes (both widths <= 8 bits: the 6/8-bit default): every main code
// (2^wm) and outlier code (2^wo) de-quantised once per block by smaq_dequant into LDS, so an
// element costs a table read instead of decode + fp64 reciprocal product + de-normalisation
// (the PMC count of the decoder was 37 VALU per element, VALU-bound). Same arithmetic, same bits.
constexpr int kLutMax = 512;

template <bool AP, bool SQ, bool FULL, int WM, int WO>
__device__ __forceinline__ void unpack_body(const UnpackArgs& A, const ElemConsts& c, uint32_t b,
                                            uint64_t dent, int wm_rt, int wo_rt, uint32_t* stage,
                                            uint32_t* pc, uint32_t* epc, uint32_t* esc_mask,
                                            float* lut) {
  constexpr bool kWindow = WO > 0 && WO <= 8;  // a lane's 4 codes fit one 32-bit window
  constexpr bool kLut = kWindow && WM > 0 && WM <= 8;
  const int wm = WM > 0 ? WM : wm_rt, wo = WO > 0 ? WO : wo_rt;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  // dent = the block's directory entry: offset | n_out << 38 | n_esc << 51
  const uint32_t* blk = A.data + (dent & ((1ull << 38) - 1ull));
  const uint32_t n_out = (uint32_t)(dent >> 38) & 0x1fffu, n_esc = (uint32_t)(dent >> 51);
  const uint32_t code_words = ((uint32_t)wm * (uint32_t)n_el + (uint32_t)(wo - wm) * n_out + 31u) / 32u;
  const uint32_t img_words = kHdrWords + code_words;
  // the image and (when they fit) the escape list in one coalesced copy: 16-B windows
  // (dwordx4 loads from the image's 16-B line on, every load of a lane issued before its LDS
  // stores; the last window is clipped to the block with dword loads, so nothing past the stream
  // is read); word i of the block lands in stage[sh + i]
  const bool esc_lds = img_words + 2u * n_esc <= (uint32_t)kStageWords;
  const uint32_t copy_words = esc_lds ? img_words + 2u * n_esc : img_words;
  {
    const uintptr_t a = (uintptr_t)blk;
    const uint32_t sh = (uint32_t)((a >> 2) & 3u);
    const uint4* src = reinterpret_cast<const uint4*>(a - 4u * sh);
    const uint32_t nvec = (sh + copy_words + 3u) >> 2;
    constexpr int kR = (kStageWords + 3 + 4 * kBlock - 1) / (4 * kBlock);
    uint4 w[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t v = (uint32_t)tid + (uint32_t)r * kBlock;
      if (v >= nvec) continue;
      if (4u * v + 4u <= sh + copy_words) {
        w[r] = src[v];
      } else {  // the clipped last window
        uint32_t q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int idx = (int)(4u * v) + k - (int)sh;
          q[k] = (idx >= 0 && idx < (int)copy_words) ? blk[idx] : 0u;
        }
        w[r] = make_uint4(q[0], q[1], q[2], q[3]);
      }
    }
    if (kLut) {  // while the image is in flight: the block's decode table
      for (int i = tid; i < (1 << WM) + (1 << WO); i += kBlock) {
        bool hi = false, lo = false;
        float q;
        if (i < (1 << WM)) {
          q = (float)(((int32_t)((uint32_t)i << (32 - WM))) >> (32 - WM));  // sign-extend
        } else {
          const uint32_t v = (uint32_t)(i - (1 << WM));
          lo = (v >> (WO - 1)) & 1u;
          hi = !lo;
          const int mag = (int)(v & ((1u << (WO - 1)) - 1u));
          q = (float)(lo ? -mag : mag);
        }
        lut[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
      }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const uint32_t v = (uint32_t)tid + (uint32_t)r * kBlock;
      if (v < nvec) reinterpret_cast<uint4*>(stage)[v] = w[r];
    }
    stage += sh;
  }
  if (tid < kMaskWords) esc_mask[tid] = 0u;
  __syncthreads();
  const uint32_t* esc = esc_lds ? stage + img_words : blk + img_words;
  if (tid < kWave) {  // wave 0: exclusive popcount prefix of the 128 outlier-mask words
    const uint32_t a = __popc(stage[1 + 2 * lane]), bb = __popc(stage[2 + 2 * lane]);
    const uint32_t ex = wave_incl_scan_u32(a + bb) - (a + bb);
    pc[2 * lane] = ex;
    pc[2 * lane + 1] = ex + a;
  } else if (tid < kWave + kMaskWords) {  // waves 1-2: escapes before each mask word
    const uint32_t wi = (uint32_t)tid - kWave;
    epc[wi] = n_esc ? escapes_below(esc, n_esc, 32u * wi) : 0u;
  }
  for (uint32_t i = tid; i < n_esc; i += kBlock) {
    const uint32_t el = esc[2 * i];
    atomicOr(esc_mask + (el >> 5), 1u << (el & 31));
  }
  __syncthreads();
  const uint32_t* bits = stage + kHdrWords;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el0 = 1024 * k + 4 * tid;
    if (!FULL && el0 >= n_el) break;
    const uint32_t mw = stage[1 + (el0 >> 5)], em = esc_mask[el0 >> 5];
    const uint32_t ebase = epc[el0 >> 5];
    const uint32_t sh0 = (uint32_t)el0 & 31u;
    const uint32_t r0 = pc[el0 >> 5] + __popc(mw & ((1u << sh0) - 1u));
    const uint32_t nib = (mw >> sh0) & 15u, enib = (em >> sh0) & 15u;
    const uint32_t pos0 = (uint32_t)wm * (uint32_t)el0 + (uint32_t)(wo - wm) * r0;
    uint32_t window = 0u;
    if (kWindow)
      window = __builtin_amdgcn_alignbit(bits[(pos0 >> 5) + 1], bits[pos0 >> 5], pos0 & 31u);
    float o[4];
    uint32_t off = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool is_o = (nib >> i) & 1u;
      uint32_t v;
      if (kWindow) {
        v = window >> off;
      } else {
        const uint32_t pos = pos0 + off;
        v = __builtin_amdgcn_alignbit(bits[(pos >> 5) + 1], bits[pos >> 5], pos & 31u);
      }
      off += is_o ? (uint32_t)wo : (uint32_t)wm;
      if (kLut) {
        o[i] = lut[is_o ? (1u << WM) + (v & ((1u << WO) - 1u)) : (v & ((1u << WM) - 1u))];
        if (__builtin_expect((enib >> i) & 1u, 0)) {  // an escape: its q from the list
          bool hi, lo;
          decode_code(v, is_o, wm, wo, hi, lo);
          const uint32_t sh = (uint32_t)(el0 + i) & 31u;
          const float q = __uint_as_float(esc[2u * (ebase + __popc(em & ((1u << sh) - 1u))) + 1u]);
          o[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
        }
        continue;
      }
      bool hi, lo;
      float q = decode_code(v, is_o, wm, wo, hi, lo);
      if (__builtin_expect((enib >> i) & 1u, 0)) {  // rank among the block's escapes: O(1)
        const uint32_t sh = (uint32_t)(el0 + i) & 31u;
        q = __uint_as_float(esc[2u * (ebase + __popc(em & ((1u << sh) - 1u))) + 1u]);
      }
      o[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
    }
    float* y = A.y + e0 + el0;
    if (A.vec && (FULL || el0 + 3 < n_el)) {
      store_stream(reinterpret_cast<float4*>(y), make_float4(o[0], o[1], o[2], o[3]));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (FULL || el0 + i < n_el) y[i] = o[i];
    }
  }
}

__global__ __launch_bounds__(kBlock) void smaq_unpack_kernel(UnpackArgs A) {
  __shared__ __attribute__((aligned(16))) uint32_t stage[kStageWords + 4];  // + the 16-B shift
  __shared__ uint32_t pc[kMaskWords], epc[kMaskWords], esc_mask[kMaskWords];
  __shared__ float lut[kLutMax];
  // the directory entry is requested together with the header (not behind its checks): the
  // header -> directory -> image chain becomes two round trips
  const uint32_t b = A.reverse ? gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const uint64_t dent = A.dir[b];
  const SmqPackedHeader* h = A.hdr;
  if (h->magic != SMQ_PACK_MAGIC || h->version != SMQ_PACK_VERSION || h->n != A.n) return;
  const int wm = h->num_bits_main - 1, wo = h->num_bits_outlier - 1;
  if (wm < 1 || wm > kMaxWidth || wo < 2 || wo > kMaxWidth) return;
  ElemConsts c;
  c.mean = h->mean;
  c.sd = h->std_dev;
  c.thr = h->thr;
  c.nthr = -h->thr;
  c.zh = 0.0f * c.nthr;
  c.zl = 0.0f * c.thr;
  c.r_main = h->range_main;
  c.r_out = h->range_outlier;
  c.inv_r_main = h->inv_range_main;
  c.inv_r_out = h->inv_range_outlier;
  const uint32_t f = h->flags;
  const bool full = (int64_t)(b + 1) * kPB <= A.n;
  const bool w57 = wm == 5 && wo == 7;
#define SMQ_UNPACK_W(APV, SQV, FULLV)                                                 \
  do {                                                                                \
    if (w57) unpack_body<APV, SQV, FULLV, 5, 7>(A, c, b, dent, wm, wo, stage, pc, epc, esc_mask, lut); \
    else unpack_body<APV, SQV, FULLV, 0, 0>(A, c, b, dent, wm, wo, stage, pc, epc, esc_mask, lut);     \
  } while (0)
#define SMQ_UNPACK(APV, SQV)                                  \
  do {                                                        \
    if (full) SMQ_UNPACK_W(APV, SQV, true);                   \
    else SMQ_UNPACK_W(APV, SQV, false);                       \
  } while (0)
  if (f & 2u) {
    if (f & 1u) SMQ_UNPACK(true, true); else SMQ_UNPACK(false, true);
  } else {
    if (f & 1u) SMQ_UNPACK(true, false); else SMQ_UNPACK(false, false);
  }
#undef SMQ_UNPACK
#undef SMQ_UNPACK_W
}

inline bool aligned_to(const void* p, unsigned a) { return ((uintptr_t)p & (a - 1)) == 0; }

inline int64_t n_blocks_of(int64_t n) { return (n + kPB - 1) / kPB; }

size_t pack_ws_status_offset(int64_t n) {
  return (smaq_stats_ws_bytes(n) + 63) & ~(size_t)63;
}

// workspace: statistics | counter (64 B) | look-back status words | cursor (64 B) | streaming
// packer: records (2 B/elem) | meta [nb] | group sums [ng] | prefixes [ng]
size_t pack_ws_stream_offset(int64_t n) {
  const size_t nb = (size_t)n_blocks_of(n < 1 ? 1 : n);
  const size_t ng = (nb + kGroup - 1) / kGroup;
  return (pack_ws_status_offset(n) + 64 + 8 * nb + 8 * ng + 64 + 255) & ~(size_t)255;
}

}  // namespace
}  // namespace smq

using namespace smq;

extern "C" {

size_t smq_smaq_pack_bound(int64_t n, int num_bits_main, int num_bits_outlier) {
  if (n < 1) return sizeof(SmqPackedHeader);
  const int wmax = (num_bits_main > num_bits_outlier ? num_bits_main : num_bits_outlier) - 1;
  const size_t nb = (size_t)n_blocks_of(n);
  const size_t per_block = kHdrWords + ((size_t)wmax * kPB + 31) / 32 + 1 + 2 * (size_t)kPB;
  return sizeof(SmqPackedHeader) + 8 * nb + 4 * nb * per_block;
}

size_t smq_smaq_pack_workspace_bytes(int64_t n) {
  const size_t nb = (size_t)n_blocks_of(n < 1 ? 1 : n);
  const size_t ng = (nb + kGroup - 1) / kGroup;
  return pack_ws_stream_offset(n) + 2 * nb * kPB + 4 * nb + 4 * (ng + 1) + 8 * ng;
}

int smq_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* packed,
                      size_t packed_bytes, void* ws, size_t ws_bytes, void* stream) {
  return smq_smaq_compress_ex(x, dtype, n, p, packed, packed_bytes, ws, ws_bytes, 0u, stream);
}

int smq_smaq_compress_ex(const void* x, int dtype, int64_t n, const SmqSmaqParams* p,
                         void* packed, size_t packed_bytes, void* ws, size_t ws_bytes,
                         uint32_t flags, void* stream) {
  int rc = smaq_validate(p, dtype);
  if (rc) return rc;
  if (n < 1 || !x || !packed) {
    set_error("compress: n must be >= 1, x and packed non-NULL");
    return SMQ_ERR_INVALID;
  }
  if (p->num_bits_main < 2 || p->num_bits_main > kMaxWidth + 1 || p->num_bits_outlier < 3 ||
      p->num_bits_outlier > kMaxWidth + 1) {
    set_error("compress: needs 2 <= num_bits_main <= %d and 3 <= num_bits_outlier <= %d",
              kMaxWidth + 1, kMaxWidth + 1);
    return SMQ_ERR_INVALID;
  }
  if (!(p->main_std_dev_threshold > 0.0f)) {
    set_error("compress: needs main_std_dev_threshold > 0 (outlier sides must be exclusive)");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma) {
    set_error("compress: the BatchNorm variant is not supported by the packed container");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source != SMQ_STATS_WORKSPACE && p->stats_source != SMQ_STATS_SAMPLED &&
      p->stats_source != SMQ_STATS_SAMPLED_DEVICE) {
    set_error("compress: statistics must be SMQ_STATS_WORKSPACE or SMQ_STATS_SAMPLED(_DEVICE)");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = n_blocks_of(n);
  if (nb > 0xffffffffLL) {
    set_error("compress: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  const size_t bound = smq_smaq_pack_bound(n, p->num_bits_main, p->num_bits_outlier);
  if (packed_bytes < bound) {
    set_error("compress: packed buffer too small: need %zu bytes (smq_smaq_pack_bound), got %zu",
              bound, packed_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  if (!ws || ws_bytes < smq_smaq_pack_workspace_bytes(n)) {
    set_error("compress: workspace too small: need %zu bytes, got %zu",
              smq_smaq_pack_workspace_bytes(n), ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  rc = prepare_stats(x, dtype, n, p, ws, ws_bytes, st);
  if (rc) return rc;
  char* wb = (char*)ws;
  const size_t so = pack_ws_status_offset(n);
  PackArgs A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.n = n;
  A.hdr = (SmqPackedHeader*)packed;
  A.dir = (uint64_t*)((char*)packed + sizeof(SmqPackedHeader));
  A.data = (uint32_t*)((char*)packed + sizeof(SmqPackedHeader) + 8 * (size_t)nb);
  A.stats = (const SmqSmaqStats*)ws;
  A.counter = (uint32_t*)(wb + so);
  A.status = (uint64_t*)(wb + so + 64);
  A.gstatus = A.status + nb;
  const size_t ng = ((size_t)nb + kGroup - 1) / kGroup;
  A.cursor = (unsigned long long*)(A.gstatus + ng);
  A.n_groups = (uint32_t)ng;
  A.rec = (uint16_t*)(wb + pack_ws_stream_offset(n));
  A.meta = (uint32_t*)(A.rec + (size_t)nb * kPB);
  A.gsum = A.meta + nb;
  A.gpre = (uint64_t*)(((uintptr_t)(A.gsum + ng) + 7) & ~(uintptr_t)7);
  // measurement knob: place blocks by one atomicAdd (valid, decodable stream; block ORDER then
  // depends on timing, so the bytes are not reproducible) instead of the ordered look-back
  static const int place_env = [] {
    const char* e = getenv("SMQ_PACK_PLACE");
    return (e && !strcmp(e, "atomic")) ? 1 : 0;
  }();
  A.place_atomic = place_env;
  A.thr = p->main_std_dev_threshold;
  A.r_main = p->range_main;
  A.r_out = p->range_outlier;
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  A.inv_r_main = R.inv_main;
  A.inv_r_out = R.inv_out;
  A.key = rng_key(p->seed);
  A.offset = p->offset;
  A.bm = p->num_bits_main;
  A.bo = p->num_bits_outlier;
  A.wm = A.bm - 1;
  A.wo = A.bo - 1;
  A.n_blocks = (uint32_t)nb;
  A.n_full = (uint32_t)(n / kPB);
  A.ticketed = (flags & SMQ_PACK_TICKETED) ? 1 : 0;
  A.flags = (p->all_positive ? 1u : 0u) | (R.safe_q ? 2u : 0u);
  // stage: w[0] + mask + the code stream at its widest (every element an outlier) + 1 word of
  // slack for the two-word ORs, rounded to 4 words so the q values after it are 16-B aligned
  A.stage_words = (uint32_t)(kHdrWords + (A.wo * kPB + 31) / 32 + 1 + 3) & ~3u;
  const size_t lds_bytes = 4 * ((size_t)A.stage_words + kPB);
  const bool vec = aligned_to(x, dtype == SMQ_DTYPE_F32 ? 16 : 8);
  const bool sr = p->stochastic_rounding != 0;
  const bool streaming = !(flags & (SMQ_PACK_TICKETED | SMQ_PACK_SINGLE)) && !A.place_atomic &&
                         A.wm <= kRecCodeBits && A.wo <= kRecCodeBits;
  if (streaming) {
    // the group sums start at zero: their place in the workspace moves with n, so a previous call
    // with another n may have left records there
    if (hipMemsetAsync(A.gsum, 0, 4 * (size_t)A.n_groups, st) != hipSuccess) {
      set_error("compress: hipMemsetAsync failed");
      return SMQ_ERR_LAUNCH;
    }
    const size_t stage_lds = 4 * (size_t)A.stage_words;
    if (dtype == SMQ_DTYPE_F32) {
      if (sr) launch_streaming_pack<kRoundHash, kF32>(A, vec, stage_lds, st);
      else launch_streaming_pack<kRoundTrunc, kF32>(A, vec, stage_lds, st);
    } else if (dtype == SMQ_DTYPE_F16) {
      if (sr) launch_streaming_pack<kRoundHash, kF16>(A, vec, stage_lds, st);
      else launch_streaming_pack<kRoundTrunc, kF16>(A, vec, stage_lds, st);
    } else {
      if (sr) launch_streaming_pack<kRoundHash, kBF16>(A, vec, stage_lds, st);
      else launch_streaming_pack<kRoundTrunc, kBF16>(A, vec, stage_lds, st);
    }
    return check_launch("smaq_code_kernel / smaq_emit_kernel");
  }
  if (hipMemsetAsync(A.status, 0, 8 * ((size_t)nb + ng) + 64, st) != hipSuccess ||
      hipMemsetAsync(A.hdr, 0, sizeof(SmqPackedHeader), st) != hipSuccess) {
    set_error("compress: hipMemsetAsync failed");
    return SMQ_ERR_LAUNCH;
  }
  if (dtype == SMQ_DTYPE_F32) {
    if (sr) launch_pack<kRoundHash, kF32>(A, vec, lds_bytes, st);
    else launch_pack<kRoundTrunc, kF32>(A, vec, lds_bytes, st);
  } else if (dtype == SMQ_DTYPE_F16) {
    if (sr) launch_pack<kRoundHash, kF16>(A, vec, lds_bytes, st);
    else launch_pack<kRoundTrunc, kF16>(A, vec, lds_bytes, st);
  } else {
    if (sr) launch_pack<kRoundHash, kBF16>(A, vec, lds_bytes, st);
    else launch_pack<kRoundTrunc, kBF16>(A, vec, lds_bytes, st);
  }
  if (A.place_atomic)
    hipLaunchKernelGGL(smaq_pack_total_kernel, dim3(1), dim3(kWave), 0, st, A.hdr, A.cursor,
                       A.n_blocks);
  return check_launch("smaq_pack_kernel");
}

int smq_smaq_decompress(const void* packed, float* y, int64_t n, void* stream) {
  if (n < 1 || !packed || !y) {
    set_error("decompress: n must be >= 1, packed and y non-NULL");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = n_blocks_of(n);
  if (nb > 0xffffffffLL) {
    set_error("decompress: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  UnpackArgs A;
  A.hdr = (const SmqPackedHeader*)packed;
  A.dir = (const uint64_t*)((const char*)packed + sizeof(SmqPackedHeader));
  A.data = (const uint32_t*)((const char*)packed + sizeof(SmqPackedHeader) + 8 * (size_t)nb);
  A.y = y;
  A.n = n;
  A.vec = aligned_to(y, 16) ? 1 : 0;
  // blocks in reverse order: the emitter writes the stream front to back, so a decompress soon
  // after the compress finds the stream's tail (~the Infinity Cache's size) still cached; 256M
  // back to back: 252 -> 234 us (tools/unpack_rev.sh, two interleaved rounds; the compress after
  // it then sweeps its statistics 16 us slower, so the bench's round trip is unchanged). A stream
  // that has left the cache decodes alike in either order. Measurement knob SMQ_UNPACK_REVERSE=0.
  static const int rev = [] {
    const char* e = getenv("SMQ_UNPACK_REVERSE");
    return e ? atoi(e) : 1;
  }();
  A.reverse = rev;
  hipLaunchKernelGGL(smaq_unpack_kernel, dim3((unsigned)nb), dim3(kBlock), 0,
                     (hipStream_t)stream, A);
  return check_launch("smaq_unpack_kernel");
}

}  // extern "C"
