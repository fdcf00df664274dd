// Packed SmaQ container (include/smq.h "Packed SmaQ container") on gfx950.
//
// compress = statistics (smaq.hip, full or sampled) + ONE packing launch:
//   * each workgroup owns a block of SMQ_PACK_BLOCK = 4096 elements (16 per lane, 4 x dwordx4),
//     quantises them with the same element code as the simulated round trip (smaq_quant), and
//     builds the block image in LDS: outlier mask, main plane, outlier plane (LDS atomics for the
//     bit-packed codes; ranks from wave ballots + a 16-segment scan);
//   * blocks are compacted into one dense stream by a decoupled look-back scan: a workgroup takes
//     its block id from an atomic ticket (so every predecessor is already resident), publishes its
//     size, and wave 0 reads up to 64 predecessors' status words per step until it meets an
//     inclusive prefix. Status words are single 64-bit relaxed agent-scope atomics carrying their
//     value, so no fences are needed; a bounded spin turns a would-be hang into header.error;
//   * the block image is written with coalesced stores at its prefix, escapes directly, and the
//     block's word offset into the directory (random-access decode).
// decompress = one launch, one workgroup per block: block image -> LDS, mask prefix popcounts,
//   per-element plane reads, escapes via an LDS bitmask + binary search of the block's sorted list,
//   then smaq_dequant — the same arithmetic as the simulated round trip, so the result is
//   bit-identical to smq_smaq_apply for the same statistics and random stream.
#include <hip/hip_runtime.h>
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
  uint64_t* status;
  uint32_t* counter;
  float thr, r_main, r_out;
  double inv_r_main, inv_r_out;
  uint32_t key;
  uint64_t offset;
  int wm, wo, bm, bo;
  uint32_t n_blocks;
  uint32_t flags;
};

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive wave prefix of small per-lane counts (< 2^BITS) and the wave total, by bit-sliced
// ballots.
template <int BITS>
__device__ __forceinline__ uint32_t wave_prefix_small(uint32_t v, uint32_t& total) {
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int j = 0; j < BITS; ++j) {
    const uint64_t bal = __ballot((v >> j) & 1u);
    pre += mbcnt64(bal) << j;
    tot += (uint32_t)__popcll(bal) << j;
  }
  total = tot;
  return pre;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// OR a width-bit code into an LSB-first bit stream in LDS (codes may straddle two words).
__device__ __forceinline__ void put_bits(uint32_t* base, uint32_t pos, uint32_t code, int width) {
  const uint32_t w = pos >> 5, sh = pos & 31u;
  atomicOr(base + w, code << sh);
  if (sh + (uint32_t)width > 32u) atomicOr(base + w + 1, code >> (32u - sh));
}

__device__ __forceinline__ uint32_t get_bits(const uint32_t* base, uint32_t pos, int width) {
  const uint32_t w = pos >> 5, sh = pos & 31u;
  uint32_t v = base[w] >> sh;
  if (sh + (uint32_t)width > 32u) v |= base[w + 1] << (32u - sh);
  return v & ((1u << width) - 1u);
}

// Plane code of one element (smq.h rules); esc = the code does not fit the budget.
__device__ __forceinline__ uint32_t classify(float q, bool hi, bool lo, int wm, int wo, bool& esc) {
  if (!(hi | lo)) {
    const float lim = (float)(1 << (wm - 1));
    const bool ok = (q >= -lim) && (q <= lim - 1.0f);  // false for NaN
    esc = !ok;
    return ok ? ((uint32_t)(int32_t)q & ((1u << wm) - 1u)) : 0u;
  }
  const float mag_max = (float)((1 << (wo - 1)) - 1);
  const uint32_t side = lo ? (1u << (wo - 1)) : 0u;
  const bool ok = hi ? (q >= 0.0f && q <= mag_max) : (q <= 0.0f && -q <= mag_max);
  esc = !ok;
  return ok ? (side | (uint32_t)(int32_t)(hi ? q : -q)) : side;
}

// Decoupled look-back (wave 0). Returns the exclusive prefix (words) of block b.
__device__ uint64_t look_back(const PackArgs& A, uint32_t b, uint64_t size) {
  const int lane = threadIdx.x & (kWave - 1);
  if (b == 0) {
    if (lane == 0) st_sc1_u64(A.status, kIncl | size);
    return 0;
  }
  if (lane == 0) st_sc1_u64(A.status + b, kAgg | size);
  uint64_t acc = 0;
  int64_t j = (int64_t)b - 1;
  uint32_t spins = 0;
  for (;;) {
    const int64_t idx = j - lane;
    const uint64_t v = idx >= 0 ? ld_sc1_u64(A.status + idx) : kIncl;  // before block 0: 0
    const uint32_t flag = (uint32_t)(v >> 62);
    const uint64_t incl = __ballot(flag == 2u);
    const uint64_t invalid = __ballot(flag == 0u);
    const int first = incl ? __builtin_ctzll(incl) : 64;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);  // lanes 0..first
    if (invalid & need) {
      if (++spins < kSpinLimit) {
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      if (lane == 0) atomicOr(&A.hdr->error, 1u);  // give up: the stream is marked broken
    }
    acc += wave_sum_u64(lane <= first ? (v & kValMask) : 0ull);
    if (first < 64 || spins >= kSpinLimit) break;
    j -= 64;
  }
  if (lane == 0) st_sc1_u64(A.status + b, kIncl | (acc + size));
  return acc;
}

template <int RM, int TIN, bool SUB, bool VEC>
__device__ __forceinline__ void pack_body(const PackArgs& A, const ElemConsts& c, uint32_t b,
                                          uint32_t* stage) {
  __shared__ uint32_t seg_cnt[2][16];
  __shared__ uint32_t seg_pre[2][17];
  __shared__ uint64_t s_prefix;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)(A.n - e0 < kPB ? A.n - e0 : kPB);

  // 1. codes of this lane's 16 elements: local index el = 1024 k + 4 tid + c
  uint32_t code[16];
  float qv[16];
  uint32_t om[4] = {0, 0, 0, 0}, xm[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el = 1024 * k + 4 * tid;
    float v[4] = {0.f, 0.f, 0.f, 0.f}, u[4] = {0.f, 0.f, 0.f, 0.f};
    const bool full = el + 3 < n_el;
    if (VEC && full) {
      const float4 t = load4<TIN>(A.x, (e0 + el) >> 2);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (el + i < n_el) v[i] = load1<TIN>(A.x, e0 + el + i);
    }
    if (RM == kRoundHash) {
      const uint64_t ctr = A.offset + (uint64_t)(e0 + el);
      if (full) {
        rng_hu4(A.key, ctr, u[0], u[1], u[2], u[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (el + i < n_el) u[i] = rng_hu(A.key, ctr + i);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hi = false, lo = false, esc = false;
      float q = 0.f;
      uint32_t cd = 0;
      if (el + i < n_el) {
        q = smaq_quant<RM, false, TIN, SUB>(v[i], u[i], c, hi, lo);
        cd = classify(q, hi, lo, A.wm, A.wo, esc);
      }
      code[4 * k + i] = cd;
      qv[4 * k + i] = q;
      om[k] |= (uint32_t)(hi | lo) << i;
      xm[k] |= (uint32_t)esc << i;
    }
  }

  // 2. ranks: per 256-element segment s = 4 k + wave, exclusive lane prefixes by ballots
  uint32_t pre_o[4], pre_x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t to, tx;
    pre_o[k] = wave_prefix_small<3>(__popc(om[k]), to);
    pre_x[k] = wave_prefix_small<3>(__popc(xm[k]), tx);
    if (lane == 0) {
      seg_cnt[0][4 * k + w] = to;
      seg_cnt[1][4 * k + w] = tx;
    }
  }
  for (int i = tid; i < kStageWords; i += kBlock) stage[i] = 0u;
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
  const uint32_t n_main = (uint32_t)n_el - n_out;
  const uint32_t main_words = (A.wm * n_main + 31u) / 32u;
  const uint32_t out_words = (A.wo * n_out + 31u) / 32u;
  const uint32_t img_words = kHdrWords + main_words + out_words;
  const uint64_t size = (uint64_t)img_words + 2ull * n_esc;

  // 3. wave 0 starts the look-back while the other waves build the block image
  if (w == 0) {
    const uint64_t p = look_back(A, b, size);
    if (lane == 0) s_prefix = p;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el0 = 1024 * k + 4 * tid;
    if (om[k]) atomicOr(stage + 1 + (el0 >> 5), om[k] << (el0 & 31));
    const uint32_t base_o = seg_pre[0][4 * k + w] + pre_o[k];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int el = el0 + i;
      if (el >= n_el) continue;
      const uint32_t r_out = base_o + __popc(om[k] & ((1u << i) - 1u));
      if ((om[k] >> i) & 1u)
        put_bits(stage + kHdrWords + main_words, r_out * A.wo, code[4 * k + i], A.wo);
      else
        put_bits(stage + kHdrWords, ((uint32_t)el - r_out) * A.wm, code[4 * k + i], A.wm);
    }
  }
  __syncthreads();

  // 4. the block image, its escapes and its directory entry at the prefix
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
      out[img_words + 2 * r] = (uint32_t)(1024 * k + 4 * tid + i);
      out[img_words + 2 * r + 1] = __float_as_uint(qv[4 * k + i]);
    }
  }
  if (tid == 0) {
    A.dir[b] = P;
    if (b == A.n_blocks - 1) {
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

template <int RM, int TIN, bool VEC>
__global__ __launch_bounds__(kBlock) void smaq_pack_kernel(PackArgs A) {
  __shared__ uint32_t stage[kStageWords];
  __shared__ uint32_t s_b;
  if (threadIdx.x == 0) {
    const uint32_t id = atomicAdd(A.counter, 1u);  // block ids in start order
    if (id == A.n_blocks - 1) atomicExch(A.counter, 0u);  // every id is taken: reset for reuse
    s_b = id;
  }
  __syncthreads();
  const uint32_t b = s_b;
  ElemConsts c;
  const float cthr = (TIN == kF32) ? A.thr : round_in<TIN>(A.thr);  // z is compared in its type
  init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  if (A.stats->quot_check)
    pack_body<RM, TIN, true, VEC>(A, c, b, stage);
  else
    pack_body<RM, TIN, false, VEC>(A, c, b, stage);
}

struct UnpackArgs {
  const SmqPackedHeader* hdr;
  const uint64_t* dir;
  const uint32_t* data;
  float* y;
  int64_t n;
  int vec;
};

__device__ __forceinline__ float find_escape(const uint32_t* esc, uint32_t n_esc, uint32_t el) {
  uint32_t lo = 0, hi = n_esc;  // entries sorted by element index
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (esc[2 * mid] <= el) lo = mid; else hi = mid;
  }
  return __uint_as_float(esc[2 * lo + 1]);
}

template <bool AP, bool SQ>
__device__ __forceinline__ void unpack_body(const UnpackArgs& A, const ElemConsts& c, uint32_t b,
                                            int wm, int wo, uint32_t* stage) {
  __shared__ uint32_t pc[kMaskWords];
  __shared__ uint32_t esc_mask[kMaskWords];
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)(A.n - e0 < kPB ? A.n - e0 : kPB);
  const uint32_t* blk = A.data + A.dir[b];
  const uint32_t w0 = blk[0];
  const uint32_t n_out = w0 & 0xffffu, n_esc = w0 >> 16;
  const uint32_t main_words = (wm * ((uint32_t)n_el - n_out) + 31u) / 32u;
  const uint32_t out_words = (wo * n_out + 31u) / 32u;
  const uint32_t img_words = kHdrWords + main_words + out_words;
  for (uint32_t i = tid; i < img_words; i += kBlock) stage[i] = blk[i];
  if (tid < kMaskWords) esc_mask[tid] = 0u;
  __syncthreads();
  if (tid < kWave) {  // exclusive popcount prefix of the 128 mask words
    const uint32_t a = __popc(stage[1 + 2 * lane]), bb = __popc(stage[2 + 2 * lane]);
    uint32_t tot;
    const uint32_t ex = wave_prefix_small<7>(a + bb, tot);
    pc[2 * lane] = ex;
    pc[2 * lane + 1] = ex + a;
  }
  const uint32_t* esc = blk + img_words;
  for (uint32_t i = tid; i < n_esc; i += kBlock) {
    const uint32_t el = esc[2 * i];
    atomicOr(esc_mask + (el >> 5), 1u << (el & 31));
  }
  __syncthreads();
  const uint32_t* mplane = stage + kHdrWords;
  const uint32_t* oplane = stage + kHdrWords + main_words;
  const uint32_t side_bit = 1u << (wo - 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int el0 = 1024 * k + 4 * tid;
    if (el0 >= n_el) break;
    const uint32_t mw = stage[1 + (el0 >> 5)], em = esc_mask[el0 >> 5], base = pc[el0 >> 5];
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t el = (uint32_t)(el0 + i);
      const uint32_t sh = el & 31u;
      const uint32_t r_out = base + __popc(mw & ((1u << sh) - 1u));
      bool hi = false, lo = false;
      float q;
      if ((mw >> sh) & 1u) {
        const uint32_t cd = get_bits(oplane, r_out * wo, wo);
        const int mag = (int)(cd & (side_bit - 1u));
        lo = (cd & side_bit) != 0u;
        hi = !lo;
        q = (float)(lo ? -mag : mag);
      } else {
        const uint32_t cd = get_bits(mplane, (el - r_out) * wm, wm);
        q = (float)(((int32_t)(cd << (32 - wm))) >> (32 - wm));  // sign-extend wm bits
      }
      if (__builtin_expect((em >> sh) & 1u, 0)) q = find_escape(esc, n_esc, el);
      o[i] = smaq_dequant<false, AP, SQ>(q, hi, lo, c);
    }
    float* y = A.y + e0 + el0;
    if (A.vec && el0 + 3 < n_el) {
      store_nt(reinterpret_cast<float4*>(y), make_float4(o[0], o[1], o[2], o[3]));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (el0 + i < n_el) y[i] = o[i];
    }
  }
}

__global__ __launch_bounds__(kBlock) void smaq_unpack_kernel(UnpackArgs A) {
  __shared__ uint32_t stage[kStageWords];
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
  const uint32_t b = blockIdx.x;
  if (f & 2u) {
    if (f & 1u) unpack_body<true, true>(A, c, b, wm, wo, stage);
    else unpack_body<false, true>(A, c, b, wm, wo, stage);
  } else {
    if (f & 1u) unpack_body<true, false>(A, c, b, wm, wo, stage);
    else unpack_body<false, false>(A, c, b, wm, wo, stage);
  }
}

inline bool aligned_to(const void* p, unsigned a) { return ((uintptr_t)p & (a - 1)) == 0; }

inline int64_t n_blocks_of(int64_t n) { return (n + kPB - 1) / kPB; }

size_t pack_ws_status_offset(int64_t n) {
  return (smaq_stats_ws_bytes(n) + 63) & ~(size_t)63;
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
  return pack_ws_status_offset(n) + 64 + 8 * nb;
}

int smq_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* packed,
                      size_t packed_bytes, void* ws, size_t ws_bytes, void* stream) {
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
  if (p->stats_source != SMQ_STATS_WORKSPACE && p->stats_source != SMQ_STATS_SAMPLED) {
    set_error("compress: statistics must be SMQ_STATS_WORKSPACE or SMQ_STATS_SAMPLED");
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
  A.flags = (p->all_positive ? 1u : 0u) | (R.safe_q ? 2u : 0u);
  if (hipMemsetAsync(A.status, 0, 8 * (size_t)nb, st) != hipSuccess ||
      hipMemsetAsync(A.hdr, 0, sizeof(SmqPackedHeader), st) != hipSuccess) {
    set_error("compress: hipMemsetAsync failed");
    return SMQ_ERR_LAUNCH;
  }
  const bool vec = aligned_to(x, dtype == SMQ_DTYPE_F32 ? 16 : 8);
  const bool sr = p->stochastic_rounding != 0;
#define SMQ_PACK(RMV, TINV)                                                                   \
  do {                                                                                         \
    if (vec)                                                                                   \
      hipLaunchKernelGGL((smaq_pack_kernel<RMV, TINV, true>), dim3((unsigned)nb), dim3(kBlock), \
                         0, st, A);                                                            \
    else                                                                                       \
      hipLaunchKernelGGL((smaq_pack_kernel<RMV, TINV, false>), dim3((unsigned)nb),             \
                         dim3(kBlock), 0, st, A);                                              \
  } while (0)
#define SMQ_PACK_T(TINV)                                  \
  do {                                                    \
    if (sr) SMQ_PACK(kRoundHash, TINV); else SMQ_PACK(kRoundTrunc, TINV); \
  } while (0)
  if (dtype == SMQ_DTYPE_F32) SMQ_PACK_T(kF32);
  else if (dtype == SMQ_DTYPE_F16) SMQ_PACK_T(kF16);
  else SMQ_PACK_T(kBF16);
#undef SMQ_PACK_T
#undef SMQ_PACK
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
  hipLaunchKernelGGL(smaq_unpack_kernel, dim3((unsigned)nb), dim3(kBlock), 0,
                     (hipStream_t)stream, A);
  return check_launch("smaq_unpack_kernel");
}

}  // extern "C"
