// Packed SmaQ container, format version 2 (include/smq.h "Packed SmaQ container"),
// on gfx950.
//
// The codes are smart.py's own (smart.py:144-169, the same smaq_quant as the simulated round trip);
// the container splits every block of SMQ_PACK_BLOCK = 4096 elements into
//   * a FIXED section (outlier mask + a plane of wm = num_bits_main - 1 bits per element: the low
//     wm bits of each code), whose size does not depend on the data, so block b's lands at b * F
//     words without knowing any other block, and
//   * a VARIABLE section (the outliers' remaining wo - wm code bits, then the escape list), small
//     (~0.09 B/element at 6/8 bits), placed by a prefix over the blocks.
// compress = statistics (smaq.hip) + three launches, none of which waits on another workgroup:
//   smaq_pack_block_kernel  one workgroup per block: x -> codes (registers) -> mask / plane / outlier
//                           ranks in LDS -> the fixed section straight into the stream, the variable
//                           section into a per-block scratch slot (kVarCap words), its size into the
//                           block's group sum;
//   smaq_pack_scan_kernel   one workgroup: exclusive prefix of the group sums, the header;
//   smaq_pack_var_kernel    one workgroup per group of 64 blocks: directory entries, the variable
//                           sections copied from scratch to their prefix; a block whose section
//                           outgrew its slot (escape-heavy data) is re-coded from x right there.
// HBM traffic: x read once (4 B/elem), the stream written once (0.93 B/elem at 6/8 bits on N(0,1)),
// plus the variable sections through scratch (~0.18 B/elem). The round-1/2 container (version 1)
// interleaved codes of two widths in element order, so every block needed its prefix before its
// first code could be placed: 2 B/elem of records went to HBM and back (1.45x the algorithmic
// bytes).
// Up to 2048 blocks (8,388,608 elements: the activation sizes) both directions are ONE launch after
// the statistics: smaq_pack_lb_kernel codes a block and places its variable section by a decoupled
// look-back over the blocks before it (no scratch, no var launch), smaq_unpack_small_kernel decodes
// the full, big and short last blocks in one grid. Same bytes, same values.
// decompress = one launch, one workgroup per block: fixed section + variable section -> LDS, mask
//   prefix popcounts for the outlier ranks, escapes via an LDS bitmask + O(1) rank, then
//   smaq_dequant (or a per-block table of it for narrow codes) — the same arithmetic as the
//   simulated round trip, so the result is bit-identical to smq_smaq_apply for the same
//   statistics and random stream.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "smaq_elem.h"
#include "smaq_host.h"
#include "smaq_pack_common.h"
#include "smaq_small.h"
#include "smq.h"
#include "smq_common.h"

namespace smq {
namespace {

struct PackArgs {
  const void* x;
  int64_t n;
  SmqPackedHeader* hdr;
  uint32_t* fixed;           // n_blocks * F words
  uint64_t* dir;             // n_blocks entries
  uint32_t* var;             // variable region
  const SmqSmaqStats* stats;
  uint32_t* scratch;         // n_blocks * kVarCap words
  uint32_t* meta;            // [n_blocks] n_out | n_esc << 16 | kMetaRecode
  uint32_t* gsum;            // [n_groups] variable words of each group of kGroup blocks
  uint64_t* gpre;            // [n_groups] exclusive prefix of gsum
  float thr, r_main, r_out;
  double inv_r_main, inv_r_out;
  uint32_t key;
  uint64_t offset;
  int wm, wo, bm, bo;
  uint32_t n_blocks;
  uint32_t n_full;           // blocks of SMQ_PACK_BLOCK elements
  uint32_t n_groups;
  uint32_t flags;
  uint32_t lds_words;        // dynamic LDS of the packing kernels (PackLds::words)
  uint32_t inline_scan;      // the var kernel sums the group prefixes itself (no scan launch)
  uint32_t forward;          // blocks in address order (measurement knob SMQ_PACK_FORWARD)
  uint64_t cap_words;        // words of the variable region (+ BN table) the buffer holds: a
                             // section that would end past it is not written
  uint32_t lb;               // one launch: the blocks' variable offsets by a look-back (pack_lookback)
  unsigned long long* lb_status;  // [n_blocks] status granules, zeroed by the statistics launch
  const float* bn_gamma;     // BN variant (general packer only), else NULL
  const float* bn_beta;
  int64_t bn_channels, bn_inner;
  uint32_t* notify;          // total_bytes also here (notify_total), or NULL
};

// smart.py:151-169 for one element, as smaq_quant computes it (same IEEE ops in the same order, so
// the same q), in the packer's branch-free form: the scalars term is a select, since with T > 0
// (a packer precondition) hi and lo exclude each other and (hi ? -T : -0.0) + (lo ? T : +0.0) is
// -T, T or +0.0 exactly. Returns q; o = outlier, lo = below -T.
template <int RM, int TIN, bool SUB>
__device__ __forceinline__ float pack_quant(float v, float u, const ElemConsts& c, bool& o, bool& lo) {
  const float dm = round_in<TIN>(v - c.mean);           // data - mean
  float z = div_by_const(dm, c.inv_sc);                 // / std.clamp(...)
  if (SUB && __builtin_expect(__builtin_amdgcn_classf(z, 0x90), 0)) z = dm / c.sc;
  z = round_in<TIN>(z);
  const bool hi = z > c.cthr;
  lo = z < c.cnthr;
  o = hi | lo;
  const float a = hi ? c.nthr : (lo ? c.thr : 0.0f);    // scalars
  const float r = o ? c.r_out : c.r_main;               // ranges
  const float d = (z + a) * r;
  if (RM == kRoundTrunc) return truncf(d);
  const float f = floorf(d);                            // _round_stochastic
  const float fr = d - f;
  float t = __builtin_fmaf(u, -0x1p-24f, fr) + 0.5f;
  t = relu_t(t);
  return f + __builtin_rintf(t);
}

// The general packer's element (EXT kernels: the BN variant, T_m <= 0): smaq_quant itself, the
// apply's own function, with the BN term of element e. The mask bit is "exactly one side" (o); an
// element with both sides (T_m < 0) codes as a main element; lo_side = below -T_m alone.
template <int RM, int TIN, bool SUB>
__device__ __forceinline__ float ext_quant(const PackArgs& A, float v, float u, const ElemConsts& c,
                                           int64_t e, bool& o, bool& lo_side) {
  bool hi, lo;
  float q;
  if (A.bn_gamma) {
    const int64_t ch = (e / A.bn_inner) % A.bn_channels;
    q = smaq_quant<RM, true, TIN, SUB>(v, u, c, hi, lo, BnTerm{A.bn_gamma[ch], A.bn_beta[ch]});
  } else {
    q = smaq_quant<RM, false, TIN, SUB>(v, u, c, hi, lo);
  }
  o = hi != lo;
  lo_side = lo && !hi;
  return q;
}

// The packer's z-score threshold: in the input type, but fp32 for BN (the parameters promote).
template <int TIN>
__device__ __forceinline__ float pack_cthr(const PackArgs& A) {
  return (TIN == kF32 || A.bn_gamma) ? A.thr : round_in<TIN>(A.thr);
}

// Keep a (uniform) value in a VGPR: an empty asm the compiler cannot see through.
#define PIN_VGPR(v) asm volatile("" : "+v"(v))

// meta bit: the block's variable section is not in its scratch slot (re-code it)
constexpr uint32_t kMetaRecode = 1u << 31;

// Dynamic LDS of the packing kernels (words): the fixed image (mask, plane), the outlier-bit
// stream, the 16 segments' escape lists {element, q bits}, the 16 segment counts.
struct PackLds {
  static uint32_t words(int wm, int we) {
    return fixed_words(wm) + 128u * (uint32_t)we + 2u * kSegs * kSegEsc + kSegs + 4u;
  }
};

__device__ void write_header(const PackArgs& A, uint64_t carry, int tid, int nthr);
template <int RM, int TIN, bool EXT>
__device__ void recode_var_section(const PackArgs& A, uint32_t b, uint64_t var_dst, uint32_t* ext,
                                   uint32_t* s_cnt);

// Blocks up to which the packer runs as ONE launch (smaq_pack_lb_kernel): 2048 blocks = 8,388,608
// elements, the activation sizes (below it the scratch round trip and the var launch are latency).
#ifndef SMQ_LB_MAX_BLOCKS  // (experiment builds: tools/build_variant.py -DSMQ_LB_MAX_BLOCKS=...)
#define SMQ_LB_MAX_BLOCKS 2048
#endif
constexpr uint32_t kLbMaxBlocks = SMQ_LB_MAX_BLOCKS;
constexpr int kLbWin = kBlock;  // predecessors examined per round trip (one per thread)

// Decoupled look-back (one launch, blocks in index order; a workgroup only waits on blocks of lower
// index, dispatched before it, so no co-residency is assumed): block b publishes its section's
// words as an aggregate the moment they are counted, looks back over windows of kLbWin predecessors
// for the nearest inclusive prefix (every block between it and b holding its aggregate), and
// publishes its own inclusive prefix. A status granule is ONE 64-bit sc1 store, (flag << 32) |
// words, flag 1 = aggregate, 2 = inclusive, 0 = not yet: the statistics launch of the same call
// cleared them (a generation tag kept in the workspace instead was clobbered when calls of other
// sizes laid the workspace out differently, and stale granules passed for the current call's).
// Returns the words of the blocks before b (every thread).
__device__ __forceinline__ uint64_t pack_lookback(const PackArgs& A, uint32_t b, uint32_t own) {
  __shared__ unsigned long long s_bi[kBlock / kWave], s_bv[kBlock / kWave];
  __shared__ unsigned long long s_sum[kBlock / kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  if (tid == 0) st_sc1_u64(A.lb_status + b, ((b == 0 ? 2ull : 1ull) << 32) | own);
  if (b == 0) return 0;
  uint64_t acc = 0;
  int64_t hi = (int64_t)b - 1;
  for (;;) {
    // thread t looks at block hi - t (t = 0: the nearest)
    const int64_t j = hi - tid;
    const uint64_t g = j >= 0 ? ld_sc1_u64(A.lb_status + j) : 0ull;
    const bool valid = j >= 0 && (g >> 32) != 0u;
    const bool incl = valid && (g >> 32) == 2u;
    const unsigned long long bi = __ballot(incl), bv = __ballot(valid);
    if (lane == 0) {
      s_bi[w] = bi;
      s_bv[w] = bv;
    }
    lds_barrier();
    // the nearest inclusive, and whether every block before it (in this window) is valid
    int t_i = kLbWin;
    bool ok = true;
#pragma unroll
    for (int v = 0; v < kBlock / kWave; ++v) {
      const unsigned long long vi = s_bi[v], vv = s_bv[v];
      if (t_i == kLbWin) {
        if (vi) {
          const int c = __builtin_ctzll(vi);
          t_i = kWave * v + c;
          const unsigned long long below = c ? ((1ull << c) - 1ull) : 0ull;
          ok = ok && (vv & below) == below;
        } else {
          // blocks before 0 (j < 0) never occur without an inclusive nearer: block 0 is one
          ok = ok && vv == ~0ull;
        }
      }
    }
    lds_barrier();  // (the next round's writes of s_bi / s_bv)
    if (!ok) {  // a block between is still coding: look again
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    // the words of blocks t <= t_i of this window (t_i itself: its inclusive prefix)
    uint64_t v = (tid <= t_i) ? (g & 0xffffffffull) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    if (lane == 0) s_sum[w] = v;
    lds_barrier();
    uint64_t tot = 0;
#pragma unroll
    for (int u = 0; u < kBlock / kWave; ++u) tot += s_sum[u];
    lds_barrier();
    acc += tot;
    if (t_i < kLbWin) break;
    hi -= kLbWin;
  }
  if (tid == 0) st_sc1_u64(A.lb_status + b, (2ull << 32) | (acc + own));
  return acc;
}

// One block (smaq_pack_block_kernel): codes of its elements, its fixed image in LDS -> the stream
// at b * F, outlier ranks and escapes -> the variable section in the block's scratch slot (unless
// it outgrows kVarCap or a segment's escape list: then the var kernel re-codes the block), the
// section's size -> meta / the group sum.
// EXT: the general element (ext_quant; instantiated with runtime widths only).
// LB: the single-launch packer (smaq_pack_lb_kernel): the section goes straight to its place in the
// variable region (offset by pack_lookback, directory entry written here; an escape-heavy block is
// re-coded to it at once), no scratch slot, meta or group sum; the last block writes the header.
template <int RM, int TIN, bool VEC, bool FULL, bool SUB, int WM, int WO, bool EXT, bool LB = false>
__device__ __forceinline__ void pack_block_body(const PackArgs& A, uint32_t b, uint32_t* lds) {
  constexpr int kWE = (WM > 0 && WO > 0) ? (WO > WM ? WO - WM : 0) : -1;  // -1: runtime
  const int wm = WM > 0 ? WM : A.wm, wo = WO > 0 ? WO : A.wo;
  const int we = kWE >= 0 ? kWE : (wo > wm ? wo - wm : 0);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  const uint32_t F = fixed_words(wm);
  uint32_t* mask = lds;
  uint32_t* plane = lds + kMaskWords;
  uint32_t* ext = lds + F;
  uint32_t* elist = ext + 128 * we;                  // [kSegs][kSegEsc][2]
  uint32_t* seg = elist + 2 * kSegs * kSegEsc;
  ElemConsts c;
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, pack_cthr<TIN>(A));
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
  // the plane and the outlier-bit stream are built by ORs: clear them while the loads are in flight
  for (uint32_t i = tid; i < 128u * (uint32_t)(wm + we); i += kBlock) plane[i] = 0u;
  lds_barrier();

  uint32_t nibs = 0u;      // per slot k: outlier nibble (bits 4k..4k+3)
  uint32_t pre[4];         // wave-exclusive outliers | escapes << 16 before this lane, per slot
  uint64_t ech[4];         // this lane's outlier bits above the plane, in element order (we <= 16;
                           // we == 2: its 8-lane group's run, in the group's last lane)
  uint32_t gfirst[4];      // we == 2: wave-local rank of the group's first outlier
  uint32_t ev[4][4];       // the same per element (we > 16 only)
  const uint32_t pmask = (wm >= 32) ? 0xffffffffu : ((1u << wm) - 1u);
  const uint32_t hm = 1u << (wm - 1), side = 1u << (wo - 1), lim_m = 2u * hm;
  // per-thread constants of the slot loop: the mask word this lane's group writes, and where its
  // 4 * wm plane bits start (the same bit offset in every slot: 1024 * wm is a multiple of 32)
  const uint32_t msh = 4u * (uint32_t)(lane & 7);
  const bool mwriter = (lane & 7) == 7;
  const uint32_t ppos0 = 4u * (uint32_t)wm * (uint32_t)tid;
  const uint32_t pw0 = ppos0 >> 5, psft = ppos0 & 31u;
  const QuadRun R = quad_run(A.key, A.offset + c.rng_off + (uint64_t)e0, kPB / 4);
  // the selects of pack_quant take two non-inline operands (T_m / r_main / r_out are SGPR values):
  // without a VGPR copy the compiler re-materialises one per slot (v_mov_b32) — pinned once here
  PIN_VGPR(c.thr);
  PIN_VGPR(c.r_main);
  PIN_VGPR(c.r_out);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    const bool full4 = FULL || el + 3 < n_el;
    float u[4] = {0.f, 0.f, 0.f, 0.f};
    if (RM == kRoundHash) {
      const uint64_t ctr = A.offset + c.rng_off + (uint64_t)(e0 + el);
      if (full4) {
        rng_hu4_run(R, 256u * (uint32_t)k + (uint32_t)tid, u[0], u[1], u[2], u[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (el + i < n_el) u[i] = rng_hu(A.key, ctr + i);
      }
    }
    uint32_t code[4], on = 0u, en = 0u;
    float qv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool o, lo, esc;
      if (EXT)
        qv[i] = ext_quant<RM, TIN, SUB>(A, xv[k][i], u[i], c, e0 + el + i, o, lo);
      else
        qv[i] = pack_quant<RM, TIN, SUB>(xv[k][i], u[i], c, o, lo);
      code[i] = code_sel(qv[i], o, lo, hm, side, lim_m, esc);
      const bool valid = FULL || el + i < n_el;
      if (!FULL) code[i] = valid ? code[i] : 0u;
      on |= ((FULL || valid) && o) ? (1u << i) : 0u;
      en |= ((FULL || valid) && esc) ? (1u << i) : 0u;
    }
    nibs |= on << (4 * k);
    // mask word of 32 elements = the nibbles of 8 consecutive lanes
    const uint32_t mw = group8_or_to_last(on << msh);
    if (mwriter) mask[32 * k + (tid >> 3)] = mw;
    // plane: the low wm bits of the 4 codes at bit wm * el
    if (4 * wm <= 32) {
      uint32_t ch = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) ch |= (code[i] & pmask) << (wm * i);
      uint32_t* pw = plane + pw0 + 32u * (uint32_t)wm * (uint32_t)k;
      atomicOr(pw, ch << psft);
      if (psft + 4u * (uint32_t)wm > 32u) atomicOr(pw + 1, ch >> (32u - psft));
    } else if (wm <= 16) {
      uint64_t ch = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) ch |= (uint64_t)(code[i] & pmask) << (wm * i);
      if (ch) or_bits64(plane, (uint32_t)wm * (uint32_t)el, ch);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const uint64_t ch = (uint64_t)(code[i] & pmask) | ((uint64_t)(code[i + 1] & pmask) << wm);
        if (ch) or_bits64(plane, (uint32_t)wm * (uint32_t)(el + i), ch);
      }
    }
    // outlier bits above the plane, in element order
    ech[k] = 0u;
    if (we > 0) {
      if (4 * we <= 32) {
        // code >> wm is 0 for a main element (its code has wm bits), so only the shifts depend on
        // which slots are outliers: slot i's bits start at we * (outliers among slots < i)
        const uint32_t s1 = (uint32_t)we * (on & 1u);
        const uint32_t s2 = (uint32_t)we * (uint32_t)__popc(on & 3u);
        const uint32_t s3 = (uint32_t)we * (uint32_t)__popc(on & 7u);
        ech[k] = (code[0] >> wm) | ((code[1] >> wm) << s1) | ((code[2] >> wm) << s2) |
                 ((code[3] >> wm) << s3);
      } else if (we <= 16) {
        uint32_t sft = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((on >> i) & 1u) {
            ech[k] |= (uint64_t)(code[i] >> wm) << sft;
            sft += (uint32_t)we;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) ev[k][i] = code[i] >> wm;
      }
    }
    const uint32_t cnt = (uint32_t)__popc(on) | ((uint32_t)__popc(en) << 16);
    const uint32_t incl = wave_incl_scan_u32(cnt);
    pre[k] = incl - cnt;
    if (lane == kWave - 1) seg[4 * k + w] = incl;
    if (kWE == 2) {
      // 2-bit outlier codes: the 8 lanes of a group own consecutive ranks, so their bits form one
      // run of <= 64 bits: assemble it in the group's last lane (DPP ORs), which alone ORs it into
      // the stream after the barrier — one lane per 8 instead of every lane ORing a few bits into
      // words its neighbours hit too (the LDS atomics serialised: 60 us of 425 at 256M)
      const uint32_t po = pre[k] & 0xffffu;
      const uint32_t first = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane & ~7), (int)po);
      const uint64_t ch = (uint64_t)(uint32_t)ech[k] << (2u * (po - first));
      const uint32_t glo = group8_or_to_last((uint32_t)ch), ghi = group8_or_to_last((uint32_t)(ch >> 32));
      ech[k] = ((uint64_t)ghi << 32) | glo;
      gfirst[k] = first;
    }
    // escapes (rare) go to the segment's list at their wave-local rank
    if (__builtin_expect(en != 0u, 0)) {
      uint32_t r = pre[k] >> 16;
      uint32_t* L = elist + 2 * kSegEsc * (4 * k + w);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((en >> i) & 1u) {
          if (r < (uint32_t)kSegEsc) {
            const float qe = qv[i];
            L[2 * r] = (uint32_t)(el + i);
            L[2 * r + 1] = qe == qe ? __float_as_uint(qe) : 0x7fc00000u;  // one NaN pattern
          }
          ++r;
        }
      }
    }
  }
  lds_barrier();
  // segment 4 k + w covers elements 1024 k + 256 w .. + 255: its base = the counts of the segments
  // before it (lanes 0-15 scan the 16 counts by DPP row shifts; every wave does it itself)
  const uint32_t own = lane < kSegs ? seg[lane] : 0u;
  uint32_t sincl = own;
  sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x111, 0xf, 0xf, false);
  sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x112, 0xf, 0xf, false);
  sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x114, 0xf, 0xf, false);
  sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x118, 0xf, 0xf, false);
  const uint32_t sexcl = sincl - own;
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)sincl, kSegs - 1);
  const bool seg_over = __ballot(lane < kSegs && (own >> 16) > (uint32_t)kSegEsc) != 0ull;
  const uint32_t n_out = tot & 0xffffu, n_esc = tot >> 16;
  const uint32_t n_ext = ext_words(we, n_out);
  const uint32_t var_words = n_ext + 2u * n_esc;
  const bool fits = !seg_over && var_words <= (uint32_t)kVarCap;
  uint32_t* dst = A.scratch + (size_t)b * kVarCap;
  uint64_t vbase = 0;  // LB: the section's word offset in the variable region
  if (LB) {
    vbase = pack_lookback(A, b, var_words);
    dst = A.var + vbase;
    if (tid == 0)
      A.dir[b] = vbase | ((uint64_t)n_out << 38) | ((uint64_t)n_esc << 51);
  }
  const bool room = !LB || vbase + var_words <= A.cap_words;  // (a capacity-bounded stream)
  if (we > 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t on = (nibs >> (4 * k)) & 15u;
      if (kWE != 2 && !on) continue;
      const uint32_t sbase = (uint32_t)__builtin_amdgcn_readlane((int)sexcl, 4 * k + w);
      if (kWE == 2) {
        if ((lane & 7) == 7 && ech[k]) or_bits64(ext, 2u * ((sbase & 0xffffu) + gfirst[k]), ech[k]);
        continue;
      }
      const uint32_t r_out = (sbase + pre[k]) & 0xffffu;
      if (4 * we <= 32) {
        or_bits32(ext, (uint32_t)we * r_out, (uint32_t)ech[k]);
      } else if (we <= 16) {
        or_bits64(ext, (uint32_t)we * r_out, ech[k]);
      } else {
        uint32_t r = r_out;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((on >> i) & 1u) or_bits64(ext, (uint32_t)we * r++, ev[k][i]);
      }
    }
  }
  // escapes: thread t copies entries t % 16 and t % 16 + 16 of segment t / 16 to their rank
  if (fits && room && n_esc) {
    const int s = tid >> 4;
    const uint32_t sb = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * s, (int)sexcl) >> 16;
    const uint32_t sc = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * s, (int)own) >> 16;
    const uint32_t* L = elist + 2 * kSegEsc * s;
#pragma unroll
    for (int jj = 0; jj < kSegEsc; jj += 16) {
      const uint32_t j = (uint32_t)(tid & 15) + (uint32_t)jj;
      if (j < sc) {
        dst[n_ext + 2u * (sb + j)] = L[2 * j];
        dst[n_ext + 2u * (sb + j) + 1u] = L[2 * j + 1];
      }
    }
  }
  lds_barrier();
  // the fixed section (mask + plane, F words, a multiple of 4) at b * F, 16-B stores
  uint4* fdst = reinterpret_cast<uint4*>(A.fixed + (size_t)b * F);
  const uint4* fsrc = reinterpret_cast<const uint4*>(lds);
  for (uint32_t i = tid; i < F / 4u; i += kBlock) fdst[i] = fsrc[i];
  if (!LB && tid == 0) {
    A.meta[b] = n_out | (n_esc << 16) | (fits ? 0u : kMetaRecode);
    atomicAdd(A.gsum + b / kGroup, var_words);
  }
  if (fits && room)
    for (uint32_t i = tid; i < n_ext; i += kBlock) dst[i] = ext[i];
  if (LB && !fits && room)  // escape-heavy: re-coded from x to its place (its LDS: ext, elist)
    recode_var_section<RM, TIN, EXT>(A, b, vbase, ext, elist);
  if (LB && b == A.n_blocks - 1)  // every block's inclusive prefix is out: the header
    write_header(A, vbase + var_words, tid, kBlock);
}

// One workgroup per full block, in reverse address order: the statistics sweep just read x front
// to back, so its tail is still in the Infinity Cache. The short last block has its own launch.
template <int RM, int TIN, bool VEC, bool FULL, int WM, int WO, bool EXT>
__global__ __launch_bounds__(kBlock) void smaq_pack_block_kernel(PackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t b = FULL ? (A.forward ? blockIdx.x : A.n_full - 1 - blockIdx.x) : A.n_blocks - 1;
  // the subnormal-quotient check only where quot_check_for() asks for it (one uniform branch)
  if (A.stats->quot_check)
    pack_block_body<RM, TIN, VEC, FULL, true, WM, WO, EXT>(A, b, lds);
  else
    pack_block_body<RM, TIN, VEC, FULL, false, WM, WO, EXT>(A, b, lds);
}

// The single launch up to kLbMaxBlocks blocks: blocks in index order (the look-back's), the short
// last block in the same grid.
template <int RM, int TIN, bool VEC, int WM, int WO, bool EXT>
__global__ __launch_bounds__(kBlock) void smaq_pack_lb_kernel(PackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t b = blockIdx.x;
  const bool full = b < A.n_full;
  if (A.stats->quot_check) {
    if (full) pack_block_body<RM, TIN, VEC, true, true, WM, WO, EXT, true>(A, b, lds);
    else pack_block_body<RM, TIN, false, false, true, WM, WO, EXT, true>(A, b, lds);
  } else {
    if (full) pack_block_body<RM, TIN, VEC, true, false, WM, WO, EXT, true>(A, b, lds);
    else pack_block_body<RM, TIN, false, false, false, WM, WO, EXT, true>(A, b, lds);
  }
}

constexpr int kScanThreads = 1024;
// up to this many groups of kGroup blocks (2048 groups: 537M elements) the var kernel's workgroups
// sum the group prefixes themselves (<= 2048 loads each, 8 KB from L2) instead of waiting for a
// one-workgroup scan launch (4.9 us at 256M)
constexpr uint32_t kInlineScanGroups = 2048;

__device__ void write_header(const PackArgs& A, uint64_t carry, int tid, int nthr);

// Inline scan: the sum of the group sums before group g, and of all of them (every thread of the
// workgroup takes part; the values fit 32 bits: <= 2048 groups of <= 64 * 11,136 words).
__device__ __forceinline__ uint32_t group_prefix(const PackArgs& A, uint32_t g, uint32_t& total) {
  __shared__ uint32_t s_p[kBlock / kWave], s_t[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  uint32_t p = 0u, t = 0u;
  for (uint32_t i = threadIdx.x; i < A.n_groups; i += kBlock) {
    const uint32_t v = A.gsum[i];
    t += v;
    p += i < g ? v : 0u;
  }
  p = wave_total_u32(p);
  t = wave_total_u32(t);
  if (lane == 0) {
    s_p[w] = p;
    s_t[w] = t;
  }
  __syncthreads();
  p = (s_p[0] + s_p[1]) + (s_p[2] + s_p[3]);
  total = (s_t[0] + s_t[1]) + (s_t[2] + s_t[3]);
  __syncthreads();
  return p;
}

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
  write_header(A, carry, tid, kScanThreads);
}

// The header, the directory's padding entry and the BN table (after the variable region of
// `carry` words): thread 0 the header, all nthr threads the table.
__device__ void write_header(const PackArgs& A, uint64_t carry, int tid, int nthr) {
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
    const uint64_t bn_words = A.bn_gamma ? 2ull * (uint64_t)A.bn_channels : 0ull;
    h->total_bytes = sizeof(SmqPackedHeader) + 8ull * dir_entries(A.n_blocks) +
                     4ull * A.n_blocks * fixed_words(A.wm) + 4ull * (carry + bn_words);
    notify_total(A.notify, h->total_bytes);
    h->error = 0u;
    h->bn_channels = A.bn_gamma ? (uint32_t)A.bn_channels : 0u;
    h->bn_inner = A.bn_gamma ? A.bn_inner : 0;
    h->mean_f64 = 0.0;
    h->std_dev_f64 = 0.0;
    h->reserved[0] = h->reserved[1] = 0u;
    if (A.n_blocks & 1u) A.dir[A.n_blocks] = 0ull;  // the directory's padding entry
  }
  if (A.bn_gamma && carry + 2ull * (uint64_t)A.bn_channels <= A.cap_words) {
    // the BN table after the variable region (which the var kernel fills next)
    float* t = reinterpret_cast<float*>(A.var + carry);
    for (int64_t i = tid; i < A.bn_channels; i += nthr) {
      t[i] = A.bn_gamma[i];
      t[A.bn_channels + i] = A.bn_beta[i];
    }
  }
}

// The variable section of block b re-coded from x straight to the stream at var_dst (a block whose
// section outgrew its scratch slot, or, in the one-launch packer, more than kSegEsc escapes in a
// 256-element segment: real activations give such blocks when a channel sits far from the tensor's
// mean). 16 passes of 256 consecutive elements, one per thread; outlier and escape ranks by wave
// ballots and the passes' running totals; the outlier bits are ORed into LDS (ext, 128 * we words)
// and copied out at the end, the escapes are written directly. Slow per block, but its few
// registers keep the var kernel's copy path and the one-launch packer at their occupancy. (Round 5,
// measured, not kept: a register-resident form — every load in flight, two barriers — cut a
// re-coded block's time, but inlined it raised the var launch from 18.4 to 24.8 us at 256M and the
// one-launch packer from 67 to 89 VGPRs for the same device time per ResNet-34 step; called out of
// line, the var launch took 46 us.)
template <int RM, int TIN, bool EXT>
__device__ void recode_var_section(const PackArgs& A, uint32_t b, uint64_t var_dst, uint32_t* ext,
                                   uint32_t* s_cnt) {
  const int wm = A.wm, wo = A.wo, we = wo > wm ? wo - wm : 0;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)min((int64_t)kPB, A.n - e0);
  ElemConsts c;
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, pack_cthr<TIN>(A));
  const uint32_t hm = 1u << (wm - 1), side = 1u << (wo - 1);
  for (uint32_t i = tid; i < 128u * (uint32_t)we; i += kBlock) ext[i] = 0u;
  __syncthreads();
  // pass 0 counts the block's outliers (its escapes follow the outlier bits: ext_words(we, n_out)
  // words); pass 1 places the outlier bits and writes the escapes
  uint32_t n_out = 0u;
#pragma unroll 1
  for (int pass = we > 0 ? 0 : 1; pass < 2; ++pass) {
    uint32_t r_out = 0u, r_esc = 0u;
    uint32_t* out = A.var + var_dst + ext_words(we, n_out);
#pragma unroll 1
    for (int j = 0; j < kPB / kBlock; ++j) {
      const int el = j * kBlock + tid;
      bool o = false, lo = false, esc = false;
      float q = 0.0f;
      uint32_t code = 0u;
      if (el < n_el) {
        const float u = (RM == kRoundHash) ? rng_hu(A.key, A.offset + c.rng_off + (uint64_t)(e0 + el)) : 0.0f;
        q = EXT ? ext_quant<RM, TIN, true>(A, load1<TIN>(A.x, e0 + el), u, c, e0 + el, o, lo)
                : pack_quant<RM, TIN, true>(load1<TIN>(A.x, e0 + el), u, c, o, lo);
        code = code_sel(q, o, lo, hm, side, 2u * hm, esc);
      }
      const unsigned long long bo = __ballot(o), be = __ballot(esc);
      const uint32_t ro = __builtin_amdgcn_mbcnt_hi((uint32_t)(bo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bo, 0u));
      const uint32_t re = __builtin_amdgcn_mbcnt_hi((uint32_t)(be >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)be, 0u));
      if (lane == 0) s_cnt[w] = (uint32_t)__popcll(bo) | ((uint32_t)__popcll(be) << 16);
      __syncthreads();
      uint32_t before = 0u, tot = 0u;
#pragma unroll
      for (int v = 0; v < kBlock / kWave; ++v) {
        const uint32_t t = s_cnt[v];
        before += v < w ? t : 0u;
        tot += t;
      }
      __syncthreads();
      if (pass == 1) {
        const uint32_t ko = r_out + (before & 0xffffu) + ro, ke = r_esc + (before >> 16) + re;
        if (o && we > 0) or_bits32(ext, (uint32_t)we * ko, code >> wm);  // we <= 23 bits
        if (esc) {
          out[2u * ke] = (uint32_t)el;
          out[2u * ke + 1u] = q == q ? __float_as_uint(q) : 0x7fc00000u;
        }
      }
      r_out += tot & 0xffffu;
      r_esc += tot >> 16;
    }
    n_out = r_out;
  }
  __syncthreads();
  uint32_t* out = A.var + var_dst;
  for (uint32_t i = tid; i < ext_words(we, n_out); i += kBlock) out[i] = ext[i];
}

// One workgroup per group of kGroup blocks: each wave requests the sections of its 16 blocks from
// their scratch slots (a lane holds words lane, lane + 64, lane + 128, lane + 192 of each), the
// workgroup sums the group prefix meanwhile, every wave turns the 64 sizes into offsets (DPP scan;
// wave 0 writes the directory entries) and stores its blocks' sections; blocks whose section
// outgrew the slot are re-coded from x (pack_recode_blocks, the workgroups after the groups).
template <int RM, int TIN, bool EXT>
__device__ void pack_recode_blocks(const PackArgs& A, uint32_t wg, uint32_t per, uint32_t* lds);

// Workgroups [0, n_groups): one group of kGroup blocks each (the copy described above); the
// workgroups after them re-code the escape-heavy blocks (pack_recode_blocks), one launch for both.
template <int RM, int TIN, int WM, int WO, bool EXT>
__global__ __launch_bounds__(kBlock) void smaq_pack_var_kernel(PackArgs A, uint32_t per) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];  // re-code: 128 * we words
  if (blockIdx.x >= A.n_groups) {
    pack_recode_blocks<RM, TIN, EXT>(A, blockIdx.x - A.n_groups, per, lds);
    return;
  }
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int wm = WM > 0 ? WM : A.wm, wo = WO > 0 ? WO : A.wo;
  const int we = wo > wm ? wo - wm : 0;
  const uint32_t g = blockIdx.x;
  const uint32_t b0 = g * kGroup;
  const uint32_t nb = min((uint32_t)kGroup, A.n_blocks - b0);
  // every wave: the group's 64 sizes (one meta word per lane), then the first 256 words of its 16
  // blocks' sections requested at once — in flight while the group prefix is summed (round 5: the
  // copy had waited for the prefix and gone 4 blocks per round trip, 24-25 us at 256M)
  uint32_t sz = 0u, t = 0u, fsz = 0u;  // fsz: the section's size; sz: the words copied here
  if ((uint32_t)lane < nb) {
    const uint32_t m = A.meta[b0 + lane];
    t = m & ~kMetaRecode;
    fsz = ext_words(we, t & 0xffffu) + 2u * (t >> 16);
    sz = (m & kMetaRecode) ? 0u : fsz;  // a re-coded block is written by pack_recode_blocks
  }
  constexpr int kB = kGroup / (kBlock / kWave);  // 16 blocks per wave
  constexpr int kW = 4;  // words per lane and block in the first round (256: most sections at 6/8 bits)
  uint32_t v[kB][kW];
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    const uint32_t j = (uint32_t)(w * kB + q);
    const uint32_t szq = (uint32_t)__builtin_amdgcn_readlane((int)sz, (int)j);
    const uint32_t* src = A.scratch + (size_t)(b0 + j) * kVarCap;
#pragma unroll
    for (int r = 0; r < kW; ++r) {
      const uint32_t i = (uint32_t)lane + (uint32_t)r * kWave;
      if (i < szq) v[q][r] = src[i];
    }
  }
  uint64_t ibase = 0;
  if (A.inline_scan) {
    uint32_t total;
    ibase = group_prefix(A, g, total);
    if (g == 0) write_header(A, total, tid, kBlock);
  }
  // offsets and directory entries: every wave holds the 64 sizes (no LDS hand-off)
  const uint64_t base = A.inline_scan ? ibase : A.gpre[g];
  const uint32_t fex = wave_incl_scan_u32(fsz) - fsz;
  if (w == 0 && (uint32_t)lane < nb)
    A.dir[b0 + lane] = (base + fex) | ((uint64_t)(t & 0xffffu) << 38) | ((uint64_t)(t >> 16) << 51);
  uint32_t* out = A.var + base;
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    const uint32_t j = (uint32_t)(w * kB + q);
    const uint32_t o0 = (uint32_t)__builtin_amdgcn_readlane((int)fex, (int)j);
    uint32_t szq = (uint32_t)__builtin_amdgcn_readlane((int)sz, (int)j);
    if (base + o0 + szq > A.cap_words) szq = 0u;  // past the buffer (a capacity-bounded stream)
    const uint32_t* src = A.scratch + (size_t)(b0 + j) * kVarCap;
#pragma unroll
    for (int r = 0; r < kW; ++r) {
      const uint32_t i = (uint32_t)lane + (uint32_t)r * kWave;
      if (i < szq) out[o0 + i] = v[q][r];
    }
    for (uint32_t i = (uint32_t)lane + kW * kWave; i < szq; i += kWave) out[o0 + i] = src[i];
  }
}

// Blocks whose variable section outgrew the scratch slot (escape-heavy data: a channel of an
// activation far from the tensor's mean escapes as a whole), re-coded from x: one workgroup per
// `per` consecutive blocks (per = 1 up to 1024 blocks), so the re-coded blocks of a tensor run in
// parallel — the var kernel's workgroups had re-coded their group's blocks one after another
// (a CIFAR ResNet activation: up to 0.7 ms per call). A block's offset: its group's prefix plus the
// sizes of the group's blocks before it (from meta).
template <int RM, int TIN, bool EXT>
__device__ void pack_recode_blocks(const PackArgs& A, uint32_t wg, uint32_t per, uint32_t* lds) {
  __shared__ uint32_t s_cnt[2 * kWave + 1];
  __shared__ uint32_t list[kBlock];
  __shared__ uint32_t n_list;
  __shared__ uint64_t s_dst;
  const int lane = threadIdx.x & (kWave - 1);
  const int we = A.wo > A.wm ? A.wo - A.wm : 0;
  // the workgroup's blocks' flags in one round of loads (per <= kBlock), the re-code list in LDS
  if (threadIdx.x == 0) n_list = 0u;
  __syncthreads();
  const uint32_t bt = wg * per + threadIdx.x;
  if (threadIdx.x < per && bt < A.n_blocks && (A.meta[bt] & kMetaRecode))
    list[atomicAdd(&n_list, 1u)] = bt;
  __syncthreads();
  const uint32_t m = n_list;
  for (uint32_t i = 0; i < m; ++i) {
    const uint32_t b = list[i];
    uint64_t gbase = 0;
    if (A.inline_scan) {
      uint32_t total;
      gbase = group_prefix(A, b / kGroup, total);
    }
    if (threadIdx.x < kWave) {
      const uint32_t g = b / kGroup, b0 = g * kGroup;
      uint32_t sz = 0u;
      if (b0 + (uint32_t)lane < b) {
        const uint32_t t = A.meta[b0 + lane] & ~kMetaRecode;
        sz = ext_words(we, t & 0xffffu) + 2u * (t >> 16);
      }
      const uint32_t before = wave_incl_scan_u32(sz);
      if (lane == kWave - 1) s_dst = (A.inline_scan ? gbase : A.gpre[g]) + before;
    }
    __syncthreads();
    const uint32_t t = A.meta[b] & ~kMetaRecode;
    if (s_dst + ext_words(we, t & 0xffffu) + 2u * (t >> 16) <= A.cap_words)
      recode_var_section<RM, TIN, EXT>(A, b, s_dst, lds, s_cnt);
    __syncthreads();
  }
}

// workgroups of the per-block rare-path launches (re-code, big-block decode): about 1024, at least
// one block each
__host__ __device__ inline uint32_t rare_per(uint32_t nb) {
  const uint32_t p = nb > 1024u ? (nb + 1023u) / 1024u : 1u;
  return p < (uint32_t)kBlock ? p : (uint32_t)kBlock;
}

template <int RM, int TIN, int WM, int WO, bool EXT>
void launch_pack_w(const PackArgs& A, bool vec, hipStream_t st) {
  const size_t lds = 4 * (size_t)A.lds_words;
  if constexpr (!EXT) {  // (the general element keeps the three-launch form: A.lb is 0 there)
    if (A.lb && vec) {  // (an unaligned x keeps the three-launch form too)
      hipLaunchKernelGGL((smaq_pack_lb_kernel<RM, TIN, true, WM, WO, false>), dim3(A.n_blocks),
                         dim3(kBlock), lds, st, A);
      return;
    }
  }
  if (A.n_full > 0) {
    if (vec)
      hipLaunchKernelGGL((smaq_pack_block_kernel<RM, TIN, true, true, WM, WO, EXT>), dim3(A.n_full),
                         dim3(kBlock), lds, st, A);
    else
      hipLaunchKernelGGL((smaq_pack_block_kernel<RM, TIN, false, true, WM, WO, EXT>),
                         dim3(A.n_full), dim3(kBlock), lds, st, A);
  }
  if (A.n_full < A.n_blocks)
    hipLaunchKernelGGL((smaq_pack_block_kernel<RM, TIN, false, false, WM, WO, EXT>), dim3(1),
                       dim3(kBlock), lds, st, A);
  if (!A.inline_scan)
    hipLaunchKernelGGL(smaq_pack_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, A);
  const int we = A.wo > A.wm ? A.wo - A.wm : 0;
  const uint32_t per = rare_per(A.n_blocks);
  hipLaunchKernelGGL((smaq_pack_var_kernel<RM, TIN, WM, WO, EXT>),
                     dim3(A.n_groups + (A.n_blocks + per - 1) / per), dim3(kBlock),
                     4 * 128 * (size_t)(we > 0 ? we : 1), st, A, per);
}

// ext: the BN variant or T_m <= 0 (ext_quant, runtime widths); else the packer's own element.
template <int RM, int TIN>
void launch_pack(const PackArgs& A, bool vec, bool ext, hipStream_t st) {
  if (ext) launch_pack_w<RM, TIN, 0, 0, true>(A, vec, st);
  else if (A.wm == 5 && A.wo == 7) launch_pack_w<RM, TIN, 5, 7, false>(A, vec, st);  // 6/8-bit default
  else launch_pack_w<RM, TIN, 0, 0, false>(A, vec, st);
}

// ---- decoder ------------------------------------------------------------------------------------
struct UnpackArgs {
  const SmqPackedHeader* hdr;
  const uint64_t* dir;
  const uint32_t* fixed;     // the fixed region (its place depends on n only)
  const uint32_t* var;       // the variable region: from the caller's widths, or (NULL) from the
                             // header's (one more dependent load at the start of every workgroup)
  float* y;
  int64_t n;
  int wm, wo;                // the caller's widths (smq_smaq_decompress_ex), else 0
  int vec;
  int reverse;  // blocks in reverse order (measurement knob SMQ_UNPACK_REVERSE=1)
  uint32_t nb;         // blocks
  uint32_t n_full;     // blocks of SMQ_PACK_BLOCK elements
  uint32_t lds_bytes;  // dynamic LDS of the launch (the widths' need, or the widest)
  uint32_t big_per;    // smaq_unpack_big_kernel: full blocks per workgroup (rare_per, <= kBlock)
  uint32_t per;        // full blocks per workgroup of the main body (1 .. kUnpackPer)
};

// Decode table of narrow codes (both widths <= 8 bits: the 6/8-bit default): every main code
// (2^wm) and outlier code (2^wo) de-quantised once per block by smaq_dequant into LDS, so an
// element costs a table read instead of decode + fp64 reciprocal product + de-normalisation. Same
// arithmetic, same bits.
constexpr int kLutMax = 512;

// q and the outlier sides of a full code (plane bits | outlier bits << wm). both: a mask-0
// element has both sides (SMQ_PACK_FLAG_BOTH_SIDES, T_m < 0).
__device__ __forceinline__ float decode_code(uint32_t v, bool is_o, int wm, int wo, bool both,
                                             bool& hi, bool& lo) {
  const uint32_t side_bit = 1u << (wo - 1);
  const uint32_t cm = v & ((1u << wm) - 1u);
  const float qm = (float)(((int32_t)(cm << (32 - wm))) >> (32 - wm));  // sign-extend
  const int mag = (int)(v & (side_bit - 1u));
  const bool sb = (v & side_bit) != 0u;
  lo = is_o ? sb : both;
  hi = is_o ? !sb : both;
  return is_o ? (float)(sb ? -mag : mag) : qm;
}

// A BN stream's table (SMQ_PACK_FLAG_BN): gamma[c], beta[c] of element e, c = (e / inner) % C
// (C, inner < 2^31). Per block the channel c0 and run offset r0 of its first element (two 64-bit
// divisions per block); an element j of the block then needs 32-bit ones only (a 64-bit division
// per element took 14 more VGPRs in the default decoder than it has).
struct BnTable {
  const float* gamma;
  const float* beta;
  uint32_t channels, inner;
  uint32_t c0, r0;
  __device__ __forceinline__ void block(int64_t e0) {
    c0 = (uint32_t)((e0 / inner) % channels);
    r0 = (uint32_t)(e0 % inner);
  }
  // channel and run offset of block element j
  __device__ __forceinline__ void locate(uint32_t j, uint32_t& ch, uint32_t& r) const {
    const uint32_t t = r0 + j, k = t / inner;
    r = t - k * inner;
    ch = (c0 + k) % channels;
  }
  // the next element's
  __device__ __forceinline__ void step(uint32_t& ch, uint32_t& r) const {
    if (++r == inner) {
      r = 0u;
      if (++ch == channels) ch = 0u;
    }
  }
  __device__ __forceinline__ BnTerm term(uint32_t ch) const { return BnTerm{gamma[ch], beta[ch]}; }
};

// dynamic LDS of the decoder (words): fixed image, variable section (when it fits kVarCap), mask
// prefix counts, escape bitmask and its prefix counts, decode table
constexpr uint32_t kUnpackLdsWords = 128u * (kMaxWidth + 1) + kVarCap + 4u + 3u * kMaskWords + kLutMax;
__host__ __device__ inline uint32_t unpack_lds_words(int wm) {
  return fixed_words(wm) + kVarCap + 4u + 3u * kMaskWords + kLutMax;
}
// blocks per decoder workgroup: both blocks' loads are in flight before the first is decoded (at
// 8 workgroups per CU one block each left ~4 KB of loads in flight per workgroup)
constexpr int kUnpackPer = 2;

// Where a block's sections are (from its directory entry and the widths).
struct UnpackGeom {
  uint32_t F, n_out, n_esc, n_ext, var_words, sh, nvec;
  bool var_lds;
  const uint32_t* vsrc;
  const uint4* fsrc;
};

__device__ __forceinline__ UnpackGeom unpack_geom(const UnpackArgs& A, uint32_t b, uint64_t dent,
                                                  int wm, int we) {
  UnpackGeom G;
  G.F = fixed_words(wm);
  G.n_out = (uint32_t)(dent >> 38) & 0x1fffu;
  G.n_esc = (uint32_t)(dent >> 51);
  G.n_ext = ext_words(we, G.n_out);
  G.var_words = G.n_ext + 2u * G.n_esc;
  G.vsrc = A.var + (dent & ((1ull << 38) - 1ull));
  G.var_lds = G.var_words <= (uint32_t)kVarCap;
  G.sh = (uint32_t)(((uintptr_t)G.vsrc >> 2) & 3u);
  G.nvec = G.var_lds ? (G.sh + G.var_words + 3u) >> 2 : 0u;
  G.fsrc = reinterpret_cast<const uint4*>(A.fixed + (size_t)b * G.F);
  return G;
}

// The loads of one block — its fixed section (one 16-B load per lane covers F <= 1024 words, i.e.
// wm <= 7; wider planes copy the rest in unpack_decode) and its variable section (16-B windows from
// its line on, the last window clipped with dword loads, so nothing past the stream is read) —
// issued, not waited for: a workgroup requests both of its blocks' bytes before it decodes one.
struct UnpackLoads {
  uint4 f0, vv;
};

__device__ __forceinline__ UnpackLoads unpack_issue(const UnpackGeom& G) {
  const int tid = threadIdx.x;
  UnpackLoads L;
  L.f0 = make_uint4(0u, 0u, 0u, 0u);
  if ((uint32_t)tid < G.F / 4u) L.f0 = G.fsrc[tid];
  L.vv = make_uint4(0u, 0u, 0u, 0u);
  constexpr int kRV = (kVarCap + 4 + 4 * kBlock - 1) / (4 * kBlock);
  static_assert(kRV == 1, "one 16-B window per lane covers the variable section");
  if ((uint32_t)tid < G.nvec) {
    // (pointer arithmetic, not an integer round trip: it stays a global pointer, no flat loads)
    const uint4* src = reinterpret_cast<const uint4*>(G.vsrc - G.sh);
    if (4u * tid + 4u <= G.sh + G.var_words) {
      L.vv = src[tid];
    } else {
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = (int)(4u * tid) + k - (int)G.sh;
        q[k] = (idx >= 0 && idx < (int)G.var_words) ? G.vsrc[idx] : 0u;
      }
      L.vv = make_uint4(q[0], q[1], q[2], q[3]);
    }
  }
  return L;
}

// Decode one block whose loads unpack_issue requested (the decode table, if any, is in LDS).
// BN: the stream's BatchNorm table applies (the decode table then holds values before it).
// M (where the variable section is read from): kVarLds — the block's section fits kVarCap and is
// in LDS, read through an LDS pointer; kVarMem — it does not, read from the stream; kVarAny — either,
// chosen per block. Through a pointer that may be global or LDS the reads are flat loads, and a flat
// load waits (vmcnt) for every store its wave has in flight: each 4-element slot with an outlier
// waited for the previous slot's output store. The full-block launch therefore decodes only kVarLds
// blocks, and a second launch (smaq_unpack_big_kernel) the rare others.
enum UnpackVarMode { kVarAny = 0, kVarLds = 1, kVarMem = 2 };

template <bool AP, bool SQ, bool FULL, int WM, int WO, bool BN, int M>
__device__ __forceinline__ void unpack_decode(const UnpackArgs& A, const ElemConsts& c, uint32_t b,
                                              const UnpackGeom& G, const UnpackLoads& L, int wm_rt,
                                              int wo_rt, bool both, BnTable bt,
                                              uint32_t* lds) {
  constexpr bool kLut = WM > 0 && WM <= 8 && WO > 0 && WO <= 8;
  constexpr bool kWide = kLut && M == kVarLds && WO > WM;
  const int wm = WM > 0 ? WM : wm_rt, wo = WO > 0 ? WO : wo_rt;
  const int we = wo > wm ? wo - wm : 0;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = FULL ? kPB : (int)(A.n - e0);
  if (BN) bt.block(e0);
  const uint32_t F = G.F, n_esc = G.n_esc, n_ext = G.n_ext, sh = G.sh, nvec = G.nvec;
  const bool var_lds = G.var_lds;
  const uint32_t* vsrc = G.vsrc;
  const uint4* fsrc = G.fsrc;
  const uint32_t nf4 = F / 4u;
  uint32_t* fx = lds;                    // [F]: mask, plane
  uint32_t* vs = lds + F;                // [kVarCap + 4]: outlier bits, escapes (16-B shifted)
  uint32_t* pc = vs + kVarCap + 4;       // [128] outliers before each mask word
  uint32_t* esc_mask = pc + kMaskWords;  // [128]
  uint32_t* epc = esc_mask + kMaskWords; // [128] escapes before each mask word
  float* lut = reinterpret_cast<float*>(epc + kMaskWords);
  if (tid < kMaskWords) esc_mask[tid] = 0u;
  if ((uint32_t)tid < nf4) reinterpret_cast<uint4*>(fx)[tid] = L.f0;
  for (uint32_t i = tid + kBlock; i < nf4; i += kBlock) reinterpret_cast<uint4*>(fx)[i] = fsrc[i];
  if ((uint32_t)tid < nvec) reinterpret_cast<uint4*>(vs)[tid] = L.vv;
  __syncthreads();
  const uint32_t* ext = M == kVarLds ? vs + sh : (M == kVarMem ? vsrc : (var_lds ? vs + sh : vsrc));
  const uint32_t* esc = ext + n_ext;
  if (tid < kWave) {  // wave 0: exclusive popcount prefix of the 128 outlier-mask words
    const uint32_t a = __popc(fx[2 * lane]), bb = __popc(fx[2 * lane + 1]);
    const uint32_t ex = wave_incl_scan_u32(a + bb) - (a + bb);
    pc[2 * lane] = ex;
    pc[2 * lane + 1] = ex + a;
  } else if (tid < kWave + kMaskWords) {  // waves 1-2: escapes before each mask word (lower
    const uint32_t wi = (uint32_t)tid - kWave;  // bound in the list, which is in element order)
    uint32_t lo = 0u, hi = n_esc;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (esc[2 * mid] < 32u * wi) lo = mid + 1u; else hi = mid;
    }
    epc[wi] = lo;
  }
  for (uint32_t i = tid; i < n_esc; i += kBlock) {
    const uint32_t el = esc[2 * i];
    atomicOr(esc_mask + (el >> 5), 1u << (el & 31));
  }
  __syncthreads();
  const uint32_t* plane = fx + kMaskWords;
  const uint32_t pm = (1u << wm) - 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el0 = 1024 * k + 4 * tid;
    if (!FULL && el0 >= n_el) break;
    const uint32_t wi = (uint32_t)el0 >> 5, sh0 = (uint32_t)el0 & 31u;
    const uint32_t mw = fx[wi], em = esc_mask[wi];
    const uint32_t nib = (mw >> sh0) & 15u, enib = (em >> sh0) & 15u;
    // plane codes: the lane's 4 * wm bits from bit wm * el0
    uint32_t cd[4];
    const uint32_t p0 = (uint32_t)wm * (uint32_t)el0;
    if (4 * wm <= 32) {
      const uint32_t win = __builtin_amdgcn_alignbit(plane[(p0 >> 5) + 1], plane[p0 >> 5], p0 & 31u);
#pragma unroll
      for (int i = 0; i < 4; ++i) cd[i] = (win >> (wm * i)) & pm;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t p = p0 + (uint32_t)(wm * i);
        cd[i] = __builtin_amdgcn_alignbit(plane[(p >> 5) + 1], plane[p >> 5], p & 31u) & pm;
      }
    }
    // kWide (narrow codes, variable section in LDS): every element's table index straight from the
    // bits, without branches — the plane code, the we bits at its would-be outlier rank, and the mask
    // bit on top; main entries of the table repeat over the we bits (unpack_lut<.., true>), so a main
    // element's (meaningless) bits there select the same value.
    uint32_t idx[4];
    if constexpr (kWide) {
      constexpr uint32_t kWE = (uint32_t)(WO - WM), kEmk = (1u << kWE) - 1u;
      const uint32_t r = pc[wi] + __popc(mw & ((1u << sh0) - 1u));
      const uint32_t p = kWE * r;  // (the word after the section is still LDS of this workgroup)
      const uint32_t win = __builtin_amdgcn_alignbit(ext[(p >> 5) + 1], ext[p >> 5], p & 31u);
      const uint32_t sft[4] = {0u, kWE * (nib & 1u), kWE * (uint32_t)__popc(nib & 3u),
                               kWE * (uint32_t)__popc(nib & 7u)};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        idx[i] = cd[i] | (((win >> sft[i]) & kEmk) << WM) | (((nib >> i) & 1u) << WO);
    }
    // outlier bits above the plane: we bits per outlier from bit we * rank
    if (!kWide && we > 0 && nib) {
      uint32_t r = pc[wi] + __popc(mw & ((1u << sh0) - 1u));
      const uint32_t emk = (we >= 32) ? 0xffffffffu : ((1u << we) - 1u);
      // (the word after the last holds no bits of it; not read past the section when it lives
      // in memory)
      auto ext_hi = [&](uint32_t wd) -> uint32_t { return wd < n_ext ? ext[wd] : 0u; };
      if (4 * we <= 32) {
        const uint32_t p = (uint32_t)we * r;
        const uint32_t win = __builtin_amdgcn_alignbit(ext_hi((p >> 5) + 1), ext[p >> 5], p & 31u);
        uint32_t s = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((nib >> i) & 1u) {
            cd[i] |= ((win >> s) & emk) << wm;
            s += (uint32_t)we;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((nib >> i) & 1u) {
            const uint32_t p = (uint32_t)we * r++;
            cd[i] |= (__builtin_amdgcn_alignbit(ext_hi((p >> 5) + 1), ext[p >> 5], p & 31u) & emk) << wm;
          }
        }
      }
    }
    float o[4];
    uint32_t bch = 0u, brun = 0u;  // BN: the element's channel and offset in its run
    if (BN) bt.locate((uint32_t)el0, bch, brun);
    if constexpr (kWide && !BN) {
      // the four table reads, then (rarely) the slot's escapes
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = lut[idx[i]];
      if (__builtin_expect(enib != 0u, 0)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (!((enib >> i) & 1u)) continue;
          bool hi, lo;
          decode_code(idx[i], (nib >> i) & 1u, wm, wo, both, hi, lo);
          const uint32_t s = sh0 + (uint32_t)i;
          const float q = __uint_as_float(esc[2u * (epc[wi] + __popc(em & ((1u << s) - 1u))) + 1u]);
          o[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (kWide && !BN) break;
      const bool is_o = (nib >> i) & 1u;
      bool hi, lo;
      float q;
      if (BN && i > 0) bt.step(bch, brun);
      const BnTerm bn = BN ? bt.term(bch) : BnTerm{1.0f, 0.0f};
      if (kLut) {
        o[i] = kWide ? lut[idx[i]] : lut[is_o ? (1u << WM) + cd[i] : cd[i]];
        if (__builtin_expect(!((enib >> i) & 1u), 1)) {
          if (BN) {  // smaq_dequant's last two statements on the table's value
            o[i] = (o[i] * bn.gamma) + bn.beta;
            if (AP) o[i] = (o[i] < 0.0f) ? 0.0f : o[i];
          }
          continue;
        }
        decode_code(kWide ? idx[i] : cd[i], is_o, wm, wo, both, hi, lo);
      } else {
        q = decode_code(cd[i], is_o, wm, wo, both, hi, lo);
        if (__builtin_expect(!((enib >> i) & 1u), 1)) {
          o[i] = smaq_dequant<BN, AP, SQ>(q, hi, lo, c, bn);
          continue;
        }
      }
      // an escape: its q from the list, rank in O(1)
      const uint32_t s = sh0 + (uint32_t)i;
      q = __uint_as_float(esc[2u * (epc[wi] + __popc(em & ((1u << s) - 1u))) + 1u]);
      o[i] = smaq_dequant<BN, AP, SQ>(q, hi, lo, c, bn);
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

// Decode table of narrow codes (kLut), once per workgroup: every main and outlier code de-quantised.
// WIDE (the branch-free indexing of unpack_decode): 2^(WO+1) entries, index = mask bit << WO | the
// WO code bits; a main element's index carries WO - WM further bits above its code, so its entry
// repeats over them.
template <bool AP, bool SQ, int WM, int WO, bool WIDE = false>
__device__ __forceinline__ void unpack_lut(const ElemConsts& c, bool both, uint32_t* lds,
                                           uint32_t F) {
  static_assert(!WIDE || (2 << WO) <= kLutMax, "decode table size");
  constexpr int kMain = WIDE ? (1 << WO) : (1 << WM);  // entries before the outlier codes
  float* lut = reinterpret_cast<float*>(lds + F + kVarCap + 4 + 3 * kMaskWords);
  for (int i = threadIdx.x; i < kMain + (1 << WO); i += kBlock) {
    bool hi = both, lo = both;
    float q;
    if (i < kMain) {
      const uint32_t cm = (uint32_t)i & ((1u << WM) - 1u);
      q = (float)(((int32_t)(cm << (32 - WM))) >> (32 - WM));  // sign-extend
    } else {
      const uint32_t v = (uint32_t)(i - kMain);
      lo = (v >> (WO - 1)) & 1u;
      hi = !lo;
      const int mag = (int)(v & ((1u << (WO - 1)) - 1u));
      q = (float)(lo ? -mag : mag);
    }
    lut[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
  }
}

// The workgroup's kUnpackPer consecutive blocks: every block's loads first, the decode table while
// they are in flight, then the blocks one after another (an LDS barrier between them).
template <bool AP, bool SQ, bool FULL, int WM, int WO, bool BN, int M>
__device__ __forceinline__ void unpack_blocks(const UnpackArgs& A, const ElemConsts& c, uint32_t b0,
                                              int nblk, const uint64_t* dent, int wm, int wo,
                                              bool both, const BnTable& bt, uint32_t* lds) {
  constexpr bool kLut = WM > 0 && WM <= 8 && WO > 0 && WO <= 8;
  const int we = wo > wm ? wo - wm : 0;
  if constexpr (BN) {
    // the BN variant one block at a time: no second block's loads held in registers while the
    // table terms are (the default decoder keeps its 67 VGPRs, 7 waves per SIMD)
    for (int i = 0; i < nblk; ++i) {
      if (i > 0) __syncthreads();
      const UnpackGeom G = unpack_geom(A, b0 + i, dent[i], wm, we);
      const UnpackLoads L = unpack_issue(G);
      if constexpr (kLut)
        if (i == 0) unpack_lut<false, SQ, WM, WO, (M == kVarLds && WO > WM)>(c, both, lds, G.F);
      if ((M == kVarLds && !G.var_lds) || (M == kVarMem && G.var_lds)) continue;  // the other launch's
      unpack_decode<AP, SQ, FULL, WM, WO, BN, M>(A, c, b0 + i, G, L, wm, wo, both, bt, lds);
    }
    return;
  }
  UnpackGeom G[kUnpackPer];
  UnpackLoads L[kUnpackPer];
#pragma unroll
  for (int i = 0; i < kUnpackPer; ++i)
    if (i < nblk) {
      G[i] = unpack_geom(A, b0 + i, dent[i], wm, we);
      L[i] = unpack_issue(G[i]);
    }
  if constexpr (kLut) unpack_lut<AP, SQ, WM, WO, (M == kVarLds && WO > WM)>(c, both, lds, G[0].F);
#pragma unroll
  for (int i = 0; i < kUnpackPer; ++i) {
    if (i >= nblk) break;
    if (i > 0) __syncthreads();  // the previous block's LDS reads are done
    if ((M == kVarLds && !G[i].var_lds) || (M == kVarMem && G[i].var_lds)) continue;
    unpack_decode<AP, SQ, FULL, WM, WO, BN, M>(A, c, b0 + i, G[i], L[i], wm, wo, both, bt, lds);
  }
}

// The widths a decoder launch works with: the caller's, else the header's (false: a corrupt header).
__device__ __forceinline__ bool unpack_widths(UnpackArgs& A, int& wm, int& wo) {
  const SmqPackedHeader* h = A.hdr;
  if (A.var) {  // widths from the caller: the fixed and variable sections' addresses do not wait
    wm = A.wm;  // for the header; a stream of other widths (or n, magic) is left alone
    wo = A.wo;
    return true;
  }
  wm = h->num_bits_main - 1;
  wo = h->num_bits_outlier - 1;
  if (wm < 1 || wm > kMaxWidth || wo < 2 || wo > kMaxWidth) return false;
  A.var = A.fixed + (size_t)A.nb * fixed_words(wm);
  return true;
}

// nblk blocks from b0 (directory entries dent) with the header's constants and flags.
template <int WM, int WO, bool FULL, int M>
__device__ __forceinline__ void unpack_run(UnpackArgs A, uint32_t b0, int nblk, const uint64_t* dent,
                                           uint32_t* lds) {
  const SmqPackedHeader* h = A.hdr;
  int wm, wo;
  if (!unpack_widths(A, wm, wo)) return;
  if (h->magic != SMQ_PACK_MAGIC || h->version != SMQ_PACK_VERSION || h->n != A.n ||
      h->num_bits_main != wm + 1 || h->num_bits_outlier != wo + 1 ||
      unpack_lds_words(wm) * 4u > A.lds_bytes || (WM > 0 && (wm != WM || wo != WO)))
    return;
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
  const bool both = (f & SMQ_PACK_FLAG_BOTH_SIDES) != 0u;
  BnTable bt;
  bt.gamma = reinterpret_cast<const float*>(A.var + h->data_words);
  bt.channels = h->bn_channels;
  bt.beta = bt.gamma + bt.channels;
  bt.inner = (uint32_t)h->bn_inner;
  bt.c0 = bt.r0 = 0u;
#define SMQ_UNPACK(APV, SQV, BNV) \
  unpack_blocks<APV, SQV, FULL, WM, WO, BNV, M>(A, c, b0, nblk, dent, wm, wo, both, bt, lds)
  if (f & SMQ_PACK_FLAG_BN) {  // the BN variant
    if (bt.channels < 1 || bt.channels > 0x7fffffffu || h->bn_inner < 1 || h->bn_inner > 0x7fffffff)
      return;
    if (f & SMQ_PACK_FLAG_SAFE_Q) {
      if (f & SMQ_PACK_FLAG_ALL_POSITIVE) SMQ_UNPACK(true, true, true); else SMQ_UNPACK(false, true, true);
    } else {
      if (f & SMQ_PACK_FLAG_ALL_POSITIVE) SMQ_UNPACK(true, false, true); else SMQ_UNPACK(false, false, true);
    }
  } else if (f & SMQ_PACK_FLAG_SAFE_Q) {
    if (f & SMQ_PACK_FLAG_ALL_POSITIVE) SMQ_UNPACK(true, true, false); else SMQ_UNPACK(false, true, false);
  } else {
    if (f & SMQ_PACK_FLAG_ALL_POSITIVE) SMQ_UNPACK(true, false, false); else SMQ_UNPACK(false, false, false);
  }
#undef SMQ_UNPACK
}

// FULL: the full blocks [0, n_full), kUnpackPer per workgroup, those whose variable section is in
// LDS (kVarLds); else the one short last block (kVarAny).
// WM / WO: the 6/8-bit default's widths, or 0 (any widths, from the caller or the header).
template <int WM, int WO, bool FULL>
__device__ __forceinline__ void unpack_main_body(const UnpackArgs& A, uint32_t g, uint32_t* lds) {
  const uint32_t b0 = FULL ? g * A.per : A.nb - 1;
  const int nblk = FULL ? (int)min(A.per, A.n_full - b0) : 1;
  // the stream is this call's (magic, n) before any directory entry is read: a caller's n beyond
  // the stream's would index past its directory (one scalar load; the rest of the header is
  // checked in unpack_run)
  if (A.hdr->magic != SMQ_PACK_MAGIC || A.hdr->n != A.n) return;
  uint64_t dent[kUnpackPer];
#pragma unroll
  for (int i = 0; i < kUnpackPer; ++i) dent[i] = i < nblk ? A.dir[b0 + i] : 0ull;
  unpack_run<WM, WO, FULL, FULL ? kVarLds : kVarAny>(A, b0, nblk, dent, lds);
}

template <int WM, int WO, bool FULL>
__global__ __launch_bounds__(kBlock) void smaq_unpack_kernel(UnpackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  unpack_main_body<WM, WO, FULL>(A, A.reverse ? gridDim.x - 1 - blockIdx.x : blockIdx.x, lds);
}

// The full blocks whose variable section outgrew kVarCap (escape-heavy data; none on N(0,1)):
// kBlock directory entries per workgroup, the listed blocks decoded from the stream one by one.
// wg: the workgroup's index among the big-block workgroups; list / n_list: its LDS list
template <int WM, int WO>
__device__ __forceinline__ void unpack_big_body(const UnpackArgs& A, uint32_t wg, uint32_t* lds,
                                                uint32_t* list, uint32_t& n_list) {
  int wm, wo;
  UnpackArgs W = A;
  if (!unpack_widths(W, wm, wo)) return;
  if (A.hdr->magic != SMQ_PACK_MAGIC || A.hdr->n != A.n) return;  // before the directory reads
  const int we = wo > wm ? wo - wm : 0;
  if (threadIdx.x == 0) n_list = 0u;
  __syncthreads();
  const uint32_t b = wg * A.big_per + threadIdx.x;
  if (threadIdx.x < A.big_per && b < A.n_full) {
    const uint64_t d = A.dir[b];
    const uint32_t n_out = (uint32_t)(d >> 38) & 0x1fffu, n_esc = (uint32_t)(d >> 51);
    if (ext_words(we, n_out) + 2u * n_esc > (uint32_t)kVarCap) list[atomicAdd(&n_list, 1u)] = b;
  }
  __syncthreads();
  const uint32_t m = n_list;
  for (uint32_t i = 0; i < m; ++i) {
    __syncthreads();  // the previous block's LDS reads are done
    const uint64_t d = A.dir[list[i]];
    unpack_run<WM, WO, true, kVarMem>(A, list[i], 1, &d, lds);
  }
}

template <int WM, int WO>
__global__ __launch_bounds__(kBlock) void smaq_unpack_big_kernel(UnpackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t list[kBlock];
  __shared__ uint32_t n_list;
  unpack_big_body<WM, WO>(A, blockIdx.x, lds, list, n_list);
}

// Streams of up to kLbMaxBlocks blocks (the activation sizes): the decode in ONE launch instead of
// two or three — workgroups [0, main_g) decode kUnpackPer full blocks each, [main_g, main_g + big_g)
// the big blocks, the last one (if n is not a multiple of the block) the short final block. Its
// registers are the three bodies' maximum, which a single wave of workgroups can afford.
template <int WM, int WO>
__global__ __launch_bounds__(kBlock) void smaq_unpack_small_kernel(UnpackArgs A, uint32_t main_g,
                                                                  uint32_t big_g) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t list[kBlock];
  __shared__ uint32_t n_list;
  const uint32_t bx = blockIdx.x;
  if (bx < main_g) unpack_main_body<WM, WO, true>(A, bx, lds);
  else if (bx < main_g + big_g) unpack_big_body<WM, WO>(A, bx - main_g, lds, list, n_list);
  else unpack_main_body<WM, WO, false>(A, 0, lds);
}

inline bool aligned_to(const void* p, unsigned a) { return ((uintptr_t)p & (a - 1)) == 0; }

inline int64_t n_blocks_of(int64_t n) { return (n + kPB - 1) / kPB; }

// workspace: statistics | meta [nb] | group sums [ng] | group prefixes [ng] | scratch [nb][kVarCap]
struct PackWs {
  size_t meta, gsum, gpre, scratch, total;
  // k: device-drawn samples (0: none); above SMQ_MAX_DEVICE_SAMPLES the statistics region holds
  // the multi-workgroup draw (smq_smaq_workspace_bytes_sampled)
  explicit PackWs(int64_t n, int64_t k = 0) {
    const size_t nb = (size_t)n_blocks_of(n < 1 ? 1 : n);
    const size_t ng = (nb + kGroup - 1) / kGroup;
    size_t st = smaq_stats_ws_bytes(n);
    if (k > SMQ_MAX_DEVICE_SAMPLES) {
      const size_t big = smq_smaq_workspace_bytes_sampled(n, k);
      st = big > st ? big : st;
    }
    meta = (st + 255) & ~(size_t)255;
    gsum = meta + 4 * nb;
    gpre = (gsum + 4 * ng + 7) & ~(size_t)7;
    scratch = (gpre + 8 * ng + 255) & ~(size_t)255;
    total = scratch + 4 * (size_t)kVarCap * nb;
  }
};

}  // namespace
}  // namespace smq

using namespace smq;

extern "C" {

size_t smq_smaq_pack_bound(int64_t n, int num_bits_main, int num_bits_outlier) {
  if (n < 1) return sizeof(SmqPackedHeader);
  const int wm = num_bits_main - 1, wo = num_bits_outlier - 1;
  const size_t we = wo > wm ? (size_t)(wo - wm) : 0;
  const size_t nb = (size_t)n_blocks_of(n);
  // every element an outlier and escaped
  const size_t per_block = fixed_words(wm < 1 ? 1 : wm) + 2 + 128 * we + 2 * (size_t)kPB;
  return sizeof(SmqPackedHeader) + 8 * (size_t)dir_entries((int64_t)nb) + 4 * nb * per_block;
}

size_t smq_smaq_pack_bound_bn(int64_t n, int num_bits_main, int num_bits_outlier,
                              int64_t bn_channels) {
  return smq_smaq_pack_bound(n, num_bits_main, num_bits_outlier) +
         8 * (size_t)(bn_channels > 0 ? bn_channels : 0);
}

size_t smq_smaq_pack_workspace_bytes(int64_t n) { return PackWs(n).total; }

size_t smq_smaq_pack_workspace_bytes_sampled(int64_t n, int64_t num_samples) {
  const int64_t k = num_samples < n ? num_samples : n;
  if (k > SMQ_MAX_DRAW_SAMPLES) return 0;
  return PackWs(n, k).total;
}

int smq_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* packed,
                      size_t packed_bytes, void* ws, size_t ws_bytes, void* stream) {
  return smq_smaq_compress_ex(x, dtype, n, p, packed, packed_bytes, ws, ws_bytes, 0u, stream);
}

}  // extern "C"

// An event to order a second stream after the first (a small per-thread ring: a wait enqueued on
// the second stream captures the event's state at that moment, so the event is free to be recorded
// again by a later call).
static hipEvent_t fork_event() {
  constexpr int kRing = 16;
  thread_local hipEvent_t ring[kRing] = {};
  thread_local int next = 0;
  hipEvent_t& e = ring[next];
  next = (next + 1) % kRing;
  if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
  return e;
}

// smq_smaq_compress_ex (y == NULL: the statistics launch first) and smq_smaq_roundtrip_compress
// (y != NULL: SmartFP's round trip into y first, whose statistics record the packer then reads;
// packed_bytes may be below the bound, down to the stream's fixed part).
// pst: the stream of the packing launches (NULL: st); a different one waits for st's statistics by
// an event (smq_smaq_roundtrip_compress_ex).
static int compress_impl(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, float* y,
                         void* packed, size_t packed_bytes, void* ws, size_t ws_bytes,
                         hipStream_t st, hipStream_t pst = nullptr, uint32_t* notify = nullptr) {
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
  if (p->main_std_dev_threshold != p->main_std_dev_threshold) {
    set_error("compress: main_std_dev_threshold is NaN");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1 ||
                      p->bn_channels > 0x7fffffffLL || p->bn_inner > 0x7fffffffLL)) {
    set_error("compress: BN variant needs bn_beta, 1 <= bn_channels, bn_inner < 2^31");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source != SMQ_STATS_WORKSPACE && p->stats_source != SMQ_STATS_SAMPLED &&
      p->stats_source != SMQ_STATS_SAMPLED_DEVICE) {
    set_error("compress: statistics must be SMQ_STATS_WORKSPACE or SMQ_STATS_SAMPLED(_DEVICE)");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = n_blocks_of(n);
  if (nb > 0x7fffffffLL) {
    set_error("compress: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  const size_t bound = smq_smaq_pack_bound_bn(n, p->num_bits_main, p->num_bits_outlier,
                                              p->bn_gamma ? p->bn_channels : 0);
  const size_t fixed = smq_smaq_pack_fixed_bytes(n, p->num_bits_main);
  if (packed_bytes < (y ? fixed : bound)) {
    set_error("compress: packed buffer too small: need %zu bytes (%s), got %zu",
              y ? fixed : bound,
              y ? "smq_smaq_pack_fixed_bytes" : (p->bn_gamma ? "smq_smaq_pack_bound_bn"
                                                             : "smq_smaq_pack_bound"),
              packed_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t k_draw = p->stats_source == SMQ_STATS_SAMPLED_DEVICE
                             ? (p->num_samples < n ? p->num_samples : n) : 0;
  const PackWs L(n, k_draw);
  if (!ws || ws_bytes < L.total) {
    set_error("compress: workspace too small: need %zu bytes, got %zu", L.total, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  // the statistics own the first region (sized for the multi-workgroup draw above 4096 samples)
  char* wb = (char*)ws;
  const uint32_t n_groups = (uint32_t)(((size_t)nb + kGroup - 1) / kGroup);
  // up to kLbMaxBlocks blocks (16-B aligned x, the packer's own element): ONE packing launch with
  // a look-back whose status granules (start of the scratch region) must start at zero; else the
  // three launches, whose group sums must. Either way the statistics launch clears them.
  const bool vec = aligned_to(x, dtype == SMQ_DTYPE_F32 ? 16 : 8);
  const bool lb = (uint32_t)nb <= kLbMaxBlocks && vec &&
                  !(p->bn_gamma || !(p->main_std_dev_threshold > 0.0f));
  uint32_t* zero = lb ? (uint32_t*)(wb + L.scratch) : (uint32_t*)(wb + L.gsum);
  const uint32_t zero_n = lb ? 2u * (uint32_t)nb : n_groups;
  bool zeroed = false;
  if (y && lb && (!pst || pst == st)) {
    // the round trip's single launch writes the stream too (smaq_fused.hip PACK): x read once
    const int wm = p->num_bits_main - 1;
    FusedPackCall k;
    k.hdr = (SmqPackedHeader*)packed;
    k.dir = (uint64_t*)((char*)packed + sizeof(SmqPackedHeader));
    k.fixed = (uint32_t*)(k.dir + dir_entries(nb));
    k.var = k.fixed + (size_t)nb * fixed_words(wm);
    k.cap_words = packed_bytes >= bound ? ~0ull : (uint64_t)((packed_bytes - fixed) / 4);
    k.n_blocks = (uint32_t)nb;
    k.notify = notify;
    const RangeRecips R0 = range_recips(p->range_main, p->range_outlier);
    k.flags = (p->all_positive ? SMQ_PACK_FLAG_ALL_POSITIVE : 0u) |
              (R0.safe_q ? SMQ_PACK_FLAG_SAFE_Q : 0u);
    rc = roundtrip_pack_fused(x, dtype, y, n, p, ws, L.meta, k, st);
    if (rc != kFusedPackDeclined) return rc;
  }
  if (y)
    rc = roundtrip_for_pack(x, dtype, y, n, p, ws, L.meta, st, zero, zero_n, &zeroed);
  else
    rc = prepare_stats(x, dtype, n, p, ws, L.meta, st, zero, zero_n, &zeroed);
  if (rc) return rc;
  PackArgs A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.n = n;
  A.bm = p->num_bits_main;
  A.bo = p->num_bits_outlier;
  A.wm = A.bm - 1;
  A.wo = A.bo - 1;
  const int we = A.wo > A.wm ? A.wo - A.wm : 0;
  A.hdr = (SmqPackedHeader*)packed;
  A.dir = (uint64_t*)((char*)packed + sizeof(SmqPackedHeader));
  A.fixed = (uint32_t*)(A.dir + dir_entries(nb));
  A.var = A.fixed + (size_t)nb * fixed_words(A.wm);
  A.cap_words = packed_bytes >= bound ? ~0ull : (uint64_t)((packed_bytes - fixed) / 4);
  A.stats = (const SmqSmaqStats*)ws;
  A.meta = (uint32_t*)(wb + L.meta);
  A.gsum = (uint32_t*)(wb + L.gsum);
  A.gpre = (uint64_t*)(wb + L.gpre);
  A.scratch = (uint32_t*)(wb + L.scratch);
  A.n_groups = n_groups;
  A.inline_scan = n_groups <= kInlineScanGroups ? 1u : 0u;
  static const int fwd_env = [] {
    const char* e = knob_env("SMQ_PACK_FORWARD");
    return e ? atoi(e) : 0;
  }();
  A.forward = fwd_env ? 1u : 0u;
  A.thr = p->main_std_dev_threshold;
  A.r_main = p->range_main;
  A.r_out = p->range_outlier;
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  A.inv_r_main = R.inv_main;
  A.inv_r_out = R.inv_out;
  A.key = rng_key(p->seed);
  A.offset = p->offset;
  A.n_blocks = (uint32_t)nb;
  A.n_full = (uint32_t)(n / kPB);
  A.bn_gamma = p->bn_gamma;
  A.bn_beta = p->bn_beta;
  A.bn_channels = p->bn_gamma ? p->bn_channels : 0;
  A.bn_inner = p->bn_gamma ? p->bn_inner : 0;
  A.flags = (p->all_positive ? SMQ_PACK_FLAG_ALL_POSITIVE : 0u) | (R.safe_q ? SMQ_PACK_FLAG_SAFE_Q : 0u) |
            (A.thr < 0.0f ? SMQ_PACK_FLAG_BOTH_SIDES : 0u) | (p->bn_gamma ? SMQ_PACK_FLAG_BN : 0u);
  const bool ext = p->bn_gamma || !(A.thr > 0.0f);
  A.lds_words = PackLds::words(A.wm, we);
  const bool sr = p->stochastic_rounding != 0;
  A.lb = lb ? 1u : 0u;
  A.lb_status = (unsigned long long*)(wb + L.scratch);
  A.notify = notify;
  if (!zeroed) fill_async(zero, 0u, zero_n, st);  // (sampled statistics: smq_common.h)
  if (pst && pst != st) {  // the packing launches on their own stream, behind the statistics
    const hipEvent_t ev = fork_event();
    if (!ev || hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(pst, ev, 0) != hipSuccess) {
      set_error("roundtrip_compress: cannot order the pack stream after the statistics");
      return SMQ_ERR_LAUNCH;
    }
    st = pst;
  }
  if (dtype == SMQ_DTYPE_F32) {
    if (sr) launch_pack<kRoundHash, kF32>(A, vec, ext, st);
    else launch_pack<kRoundTrunc, kF32>(A, vec, ext, st);
  } else if (dtype == SMQ_DTYPE_F16) {
    if (sr) launch_pack<kRoundHash, kF16>(A, vec, ext, st);
    else launch_pack<kRoundTrunc, kF16>(A, vec, ext, st);
  } else {
    if (sr) launch_pack<kRoundHash, kBF16>(A, vec, ext, st);
    else launch_pack<kRoundTrunc, kBF16>(A, vec, ext, st);
  }
  return check_launch("smaq_pack_block_kernel / smaq_pack_var_kernel");
}

extern "C" {

int smq_smaq_compress_ex(const void* x, int dtype, int64_t n, const SmqSmaqParams* p,
                         void* packed, size_t packed_bytes, void* ws, size_t ws_bytes,
                         uint32_t flags, void* stream) {
  (void)flags;  // SMQ_PACK_TICKETED / SMQ_PACK_SINGLE: accepted, one packer (see smq.h)
  return compress_impl(x, dtype, n, p, nullptr, packed, packed_bytes, ws, ws_bytes,
                       (hipStream_t)stream);
}

size_t smq_smaq_pack_fixed_bytes(int64_t n, int num_bits_main) {
  if (n < 1) return sizeof(SmqPackedHeader);
  const int wm = num_bits_main - 1;
  const int64_t nb = n_blocks_of(n);
  return sizeof(SmqPackedHeader) + 8 * (size_t)dir_entries(nb) +
         4 * (size_t)nb * fixed_words(wm < 1 ? 1 : wm);
}

int smq_smaq_roundtrip_compress(const void* x, int dtype, float* y, int64_t n,
                                const SmqSmaqParams* p, void* packed, size_t packed_bytes,
                                void* ws, size_t ws_bytes, void* stream) {
  if (!y) {
    set_error("roundtrip_compress: y must be a device pointer");
    return SMQ_ERR_INVALID;
  }
  return compress_impl(x, dtype, n, p, y, packed, packed_bytes, ws, ws_bytes,
                       (hipStream_t)stream);
}

int smq_smaq_roundtrip_compress_ex(const void* x, int dtype, float* y, int64_t n,
                                   const SmqSmaqParams* p, void* packed, size_t packed_bytes,
                                   void* ws, size_t ws_bytes, void* stream, void* pack_stream) {
  if (!y) {
    set_error("roundtrip_compress: y must be a device pointer");
    return SMQ_ERR_INVALID;
  }
  return compress_impl(x, dtype, n, p, y, packed, packed_bytes, ws, ws_bytes,
                       (hipStream_t)stream, (hipStream_t)pack_stream);
}

uint32_t* smq_notify_alloc(int64_t count) {
  if (count < 1 || count > (1ll << 28)) {
    set_error("notify_alloc: count must be in [1, 2^28]");
    return nullptr;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)count * 4,
                    hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess ||
      !p) {
    set_error("notify_alloc: hipHostMalloc of %lld words failed", (long long)count);
    return nullptr;
  }
  void* d = nullptr;  // kernels write the words through the host address: it must be the device's
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || d != p) {
    (void)hipHostFree(p);
    set_error("notify_alloc: host-mapped memory has a different device address");
    return nullptr;
  }
  uint32_t* w = (uint32_t*)p;
  for (int64_t i = 0; i < count; ++i) w[i] = SMQ_NOTIFY_PENDING;
  return w;
}

void smq_notify_free(uint32_t* words) {
  if (words) (void)hipHostFree(words);
}

int smq_smaq_roundtrip_compress_notify(const void* x, int dtype, float* y, int64_t n,
                                       const SmqSmaqParams* p, void* packed, size_t packed_bytes,
                                       void* ws, size_t ws_bytes, uint32_t* notify, void* stream) {
  if (!y) {
    set_error("roundtrip_compress: y must be a device pointer");
    return SMQ_ERR_INVALID;
  }
  if (((uintptr_t)notify & 3u) != 0) {
    set_error("roundtrip_compress_notify: notify must be 4-byte aligned");
    return SMQ_ERR_INVALID;
  }
  return compress_impl(x, dtype, n, p, y, packed, packed_bytes, ws, ws_bytes,
                       (hipStream_t)stream, nullptr, notify);
}

static int decompress_impl(const void* packed, float* y, int64_t n, int bm, int bo, void* stream) {
  if (n < 1 || !packed || !y) {
    set_error("decompress: n must be >= 1, packed and y non-NULL");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = n_blocks_of(n);
  if (nb > 0x7fffffffLL) {
    set_error("decompress: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  if (bm && (bm < 2 || bm > kMaxWidth + 1 || bo < 3 || bo > kMaxWidth + 1)) {
    set_error("decompress: needs 2 <= num_bits_main <= %d and 3 <= num_bits_outlier <= %d",
              kMaxWidth + 1, kMaxWidth + 1);
    return SMQ_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  UnpackArgs A;
  A.hdr = (const SmqPackedHeader*)packed;
  A.dir = (const uint64_t*)((const char*)packed + sizeof(SmqPackedHeader));
  A.fixed = (const uint32_t*)(A.dir + dir_entries(nb));
  A.wm = bm ? bm - 1 : 0;
  A.wo = bo ? bo - 1 : 0;
  A.var = bm ? A.fixed + (size_t)nb * fixed_words(A.wm) : nullptr;
  A.y = y;
  A.n = n;
  A.vec = aligned_to(y, 16) ? 1 : 0;
  // blocks in index order: the packer writes the fixed sections in reverse block order, so the
  // head of the stream is the part still in the Infinity Cache right after a compress (256M: 325 ->
  // 293 us). Measurement knob SMQ_UNPACK_REVERSE=1.
  static const int rev = [] {
    const char* e = knob_env("SMQ_UNPACK_REVERSE");
    return e ? atoi(e) : 0;
  }();
  A.reverse = rev;
  A.nb = (uint32_t)nb;
  A.n_full = (uint32_t)(n / kPB);
  A.lds_bytes = 4u * (bm ? unpack_lds_words(A.wm) : kUnpackLdsWords);
  // big blocks (a variable section beyond the LDS window: escape-heavy data) are decoded one after
  // another by their workgroup: about 1024 workgroups, so a tensor's big blocks decode in parallel
  A.big_per = rare_per(A.n_full);
  if (A.big_per > (uint32_t)kBlock) A.big_per = kBlock;
  // up to 1024 blocks (the activation sizes: 64 - 1024 blocks, a fraction of the chip's 8 decoder
  // workgroups per CU) one block per workgroup, so a small stream's blocks decode side by side;
  // above, two (both blocks' loads in flight before the first is decoded)
  A.per = A.nb <= 1024u ? 1u : (uint32_t)kUnpackPer;
  const unsigned grid = (unsigned)((A.n_full + A.per - 1) / A.per);
  const bool w57 = bm == 6 && bo == 8;  // the default widths, known from the caller
  const unsigned big_g = grid ? (unsigned)((A.n_full + A.big_per - 1) / A.big_per) : 0u;
  const bool small = A.nb <= kLbMaxBlocks;  // one launch (smaq_unpack_small_kernel)
  const unsigned small_g = grid + big_g + (A.n_full < A.nb ? 1u : 0u);
#define SMQ_UNPACK_LAUNCH(WMV, WOV)                                                                \
  do {                                                                                            \
    if (small) {                                                                                  \
      hipLaunchKernelGGL((smaq_unpack_small_kernel<WMV, WOV>), dim3(small_g), dim3(kBlock),        \
                         A.lds_bytes, st, A, grid, big_g);                                        \
      break;                                                                                      \
    }                                                                                             \
    if (grid) {                                                                                   \
      hipLaunchKernelGGL((smaq_unpack_kernel<WMV, WOV, true>), dim3(grid), dim3(kBlock),           \
                         A.lds_bytes, st, A);                                                     \
      hipLaunchKernelGGL((smaq_unpack_big_kernel<WMV, WOV>), dim3((A.n_full + A.big_per - 1) / A.big_per), \
                         dim3(kBlock), A.lds_bytes, st, A);                                       \
    }                                                                                             \
    if (A.n_full < A.nb)                                                                          \
      hipLaunchKernelGGL((smaq_unpack_kernel<WMV, WOV, false>), dim3(1), dim3(kBlock), A.lds_bytes, \
                         st, A);                                                                  \
  } while (0)
  if (w57) SMQ_UNPACK_LAUNCH(5, 7);
  else SMQ_UNPACK_LAUNCH(0, 0);
#undef SMQ_UNPACK_LAUNCH
  return check_launch("smaq_unpack_kernel");
}

int smq_smaq_decompress(const void* packed, float* y, int64_t n, void* stream) {
  return decompress_impl(packed, y, n, 0, 0, stream);
}

int smq_smaq_decompress_ex(const void* packed, float* y, int64_t n, int num_bits_main,
                           int num_bits_outlier, void* stream) {
  if (num_bits_main == 0) {
    set_error("decompress_ex: num_bits_main / num_bits_outlier required");
    return SMQ_ERR_INVALID;
  }
  return decompress_impl(packed, y, n, num_bits_main, num_bits_outlier, stream);
}

}  // extern "C"
