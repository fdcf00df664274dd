// smaq_pack_f64.hip — float64 tensors in the packed SmaQ container (flag SMQ_PACK_FLAG_F64), gfx950.
//
// Reference: smart_compress/compress/smart.py:110-190 on a float64 tensor — the fp64 chain of
// smq_smaq_roundtrip_f64 (fp64.hip, smaq_f64.h: z, q and the de-quantisation in fp64, the scalars and
// ranges the fp32 values). The container is smaq_pack.hip's format version 2 (include/smq.h) with
// three words per escape (q as float64 bits), the statistics as doubles in the header and a BN table
// of doubles, so decompress_f64(compress_f64(x)) equals the fp64 round trip bit for bit.
//
// Not bandwidth-tuned (like the other fp64 kernels: fp64 SmaQ is a correctness path). compress =
// the fp64 statistics (launch_stats_f64) + three launches, none waiting on another workgroup:
//   pack_f64_count_kernel  one workgroup per block: codes, per-block outlier / escape counts (meta);
//   pack_f64_scan_kernel   one workgroup: the blocks' variable-section sizes -> directory (prefix
//                          offsets), header, BN table;
//   pack_f64_write_kernel  one workgroup per block: the codes again (the fp64 chain is cheaper to
//                          recompute than to park), the fixed section and the outlier bits through
//                          LDS, the escapes straight to their final place, both sections stored.
// decompress = one launch, one workgroup per block (unpack_f64_kernel): the fixed section and an
// escape map in LDS, outlier ranks by prefix popcounts, smaq_dequant_f64 per element.
#include <hip/hip_runtime.h>
#include <string.h>

#include "smaq_elem.h"
#include "smaq_f64.h"
#include "smaq_host.h"
#include "smq.h"
#include "smq_common.h"

namespace smq {
namespace {

constexpr int kPB = SMQ_PACK_BLOCK;      // elements per block
constexpr int kMaskWords = kPB / 32;
constexpr int kPasses = kPB / kBlock;     // 16 passes of 256 consecutive elements
constexpr uint32_t kEscWords = 3;         // {element, q low word, q high word}
constexpr int kScanThreads = 1024;
constexpr uint64_t kNaN64 = 0x7ff8000000000000ull;

__host__ __device__ inline int64_t dir_entries(int64_t nb) { return (nb + 1) & ~(int64_t)1; }
__host__ __device__ inline uint32_t fixed_words(int wm) { return kMaskWords + 128u * (uint32_t)wm; }
__host__ __device__ inline uint32_t ext_words(int we, uint32_t n_out) {
  return ((uint32_t)we * n_out + 31u) / 32u;
}

struct F64PackArgs {
  const double* x;
  int64_t n;
  const SmqSmaqStatsF64* stats;  // the workspace header (launch_stats_f64)
  SmqPackedHeader* hdr;
  uint64_t* dir;
  uint32_t* fixed;
  uint32_t* var;
  uint32_t* meta;                // [n_blocks] n_out | n_esc << 16
  const double* bn_gamma;        // BN streams (fp64 parameters), else NULL
  const double* bn_beta;
  int64_t bn_channels, bn_inner;
  SmqSmaqParams p;               // by value: the flag constants (elem_f64_consts)
  uint32_t key;
  uint64_t offset;
  int wm, wo;
  uint32_t n_blocks, flags;
};

// smart.py:144-169 for element e: q, the mask bit (exactly one side; T_m < 0 also gives elements
// with both sides, coded as main) and the lower side.
template <int RM, bool BN>
__device__ __forceinline__ double f64_q(const F64PackArgs& A, const ElemF64& c, uint64_t off,
                                        int64_t e, bool& o, bool& los) {
  const double u = RM == kRoundHash ? (double)smaq_u24(A.key, off + (uint64_t)e) : 0.0;
  double g = 1.0, b = 0.0;
  if (BN) {
    const int64_t ch = (e / A.bn_inner) % A.bn_channels;
    g = A.bn_gamma[ch];
    b = A.bn_beta[ch];
  }
  bool hi, lo;
  const double q = smaq_quant_f64<RM, BN>(A.x[e], u, c, hi, lo, g, b);
  o = hi != lo;
  los = lo && !hi;
  return q;
}

// The code of an element (include/smq.h format rules; cpu_codecs.hip pack_block_host restates them):
// main: wm-bit two's complement q; outlier: side bit (lower side) over |q|; a q outside the budget
// (or inf / NaN) escapes with code 0 (main) or its side bit alone (outlier).
__host__ __device__ __forceinline__ uint32_t f64_code(double q, bool o, bool los, int wm, int wo,
                                                      bool& esc) {
  const double hm = (double)(1u << (wm - 1)), mag_max = (double)((1u << (wo - 1)) - 1u);
  bool ok;
  if (o) ok = los ? (q <= 0.0 && -q <= mag_max) : (q >= 0.0 && q <= mag_max);
  else ok = q >= -hm && q <= hm - 1.0;
  esc = !ok;
  const int64_t qi = ok ? (int64_t)q : 0;
  if (o) {
    const uint32_t side = (uint32_t)los << (wo - 1);
    return ok ? (side | (uint32_t)(los ? -qi : qi)) : side;
  }
  return ok ? ((uint32_t)qi & ((1u << wm) - 1u)) : 0u;
}

__device__ __forceinline__ void or_bits(uint32_t* base, uint32_t pos, uint32_t v) {  // v < 2^24
  const uint32_t sft = pos & 31u, w0 = pos >> 5;
  atomicOr(base + w0, v << sft);
  if (sft && (v >> (32u - sft))) atomicOr(base + w0 + 1, v >> (32u - sft));
}

__device__ __forceinline__ uint32_t get_bits(const uint32_t* w, uint32_t pos, int width) {
  const uint32_t sft = pos & 31u, w0 = pos >> 5;
  uint64_t v = w[w0] >> sft;
  if (sft + (uint32_t)width > 32u) v |= (uint64_t)w[w0 + 1] << (32u - sft);
  return (uint32_t)(v & ((1ull << width) - 1ull));
}

template <int RM, bool BN>
__global__ __launch_bounds__(kBlock) void pack_f64_count_kernel(F64PackArgs A) {
  __shared__ uint32_t s_cnt[kBlock / kWave];
  const uint32_t b = blockIdx.x;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)min((int64_t)kPB, A.n - e0);
  const SmqSmaqStatsF64 st = *A.stats;
  const ElemF64 c = elem_f64_consts(st, A.p);
  const uint64_t off = A.offset + st.rng_offset;
  uint32_t no = 0u, ne = 0u;
  for (int j = 0; j < kPasses; ++j) {
    const int el = j * kBlock + (int)threadIdx.x;
    if (el >= n_el) break;
    bool o, los, esc;
    const double q = f64_q<RM, BN>(A, c, off, e0 + el, o, los);
    (void)f64_code(q, o, los, A.wm, A.wo, esc);
    no += o ? 1u : 0u;
    ne += esc ? 1u : 0u;
  }
  const uint32_t t = wave_sum_u32(no | (ne << 16));
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (lane == 0) s_cnt[w] = t;
  __syncthreads();
  if (threadIdx.x == 0) A.meta[b] = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
}

// One workgroup: the directory (each block's variable-section offset: an exclusive prefix of the
// sizes ext_words(we, n_out) + 3 n_esc, in 4096-block steps), the header and the BN table.
__global__ __launch_bounds__(kScanThreads) void pack_f64_scan_kernel(F64PackArgs A) {
  __shared__ uint64_t s_wave[kScanThreads / kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int we = A.wo > A.wm ? A.wo - A.wm : 0;
  uint64_t carry = 0;
  for (uint32_t base = 0; base < A.n_blocks; base += 4u * kScanThreads) {
    uint32_t m[4], sz[4];
    uint64_t loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t bb = base + 4u * (uint32_t)tid + (uint32_t)j;
      m[j] = bb < A.n_blocks ? A.meta[bb] : 0u;
      sz[j] = ext_words(we, m[j] & 0xffffu) + kEscWords * (m[j] >> 16);
      loc += sz[j];
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
      const uint32_t bb = base + 4u * (uint32_t)tid + (uint32_t)j;
      if (bb < A.n_blocks)
        A.dir[bb] = run | ((uint64_t)(m[j] & 0xffffu) << 38) | ((uint64_t)(m[j] >> 16) << 51);
      run += sz[j];
    }
    carry += total;
    __syncthreads();
  }
  if (tid == 0) {
    const SmqSmaqStatsF64 st = *A.stats;
    SmqPackedHeader* h = A.hdr;
    h->magic = SMQ_PACK_MAGIC;
    h->version = SMQ_PACK_VERSION;
    h->n = A.n;
    h->block_elems = kPB;
    h->n_blocks = A.n_blocks;
    h->num_bits_main = A.wm + 1;
    h->num_bits_outlier = A.wo + 1;
    h->flags = A.flags;
    h->thr = A.p.main_std_dev_threshold;
    h->range_main = A.p.range_main;
    h->range_outlier = A.p.range_outlier;
    h->mean = (float)st.mean;
    h->std_dev = (float)st.std_dev;
    h->inv_range_main = 1.0 / (double)A.p.range_main;
    h->inv_range_outlier = 1.0 / (double)A.p.range_outlier;
    h->data_words = carry;
    const uint64_t bn_words = A.bn_gamma ? 4ull * (uint64_t)A.bn_channels : 0ull;
    h->total_bytes = sizeof(SmqPackedHeader) + 8ull * dir_entries(A.n_blocks) +
                     4ull * A.n_blocks * fixed_words(A.wm) + 4ull * (carry + bn_words);
    h->error = 0u;
    h->bn_channels = A.bn_gamma ? (uint32_t)A.bn_channels : 0u;
    h->bn_inner = A.bn_gamma ? A.bn_inner : 0;
    h->mean_f64 = st.mean;
    h->std_dev_f64 = st.std_dev;
    h->reserved[0] = h->reserved[1] = 0u;
    if (A.n_blocks & 1u) A.dir[A.n_blocks] = 0ull;  // the directory's padding entry
  }
  if (A.bn_gamma) {  // fp64 gammas then betas, after the variable region
    double* t = reinterpret_cast<double*>(A.var + carry);
    for (int64_t i = tid; i < A.bn_channels; i += kScanThreads) {
      t[i] = A.bn_gamma[i];
      t[A.bn_channels + i] = A.bn_beta[i];
    }
  }
}

// The codes again; the fixed section (mask by wave ballots, plane by LDS ORs) and the outliers' bits
// above the plane (LDS ORs at their rank) are stored at the end, the escapes directly at their rank.
template <int RM, bool BN>
__global__ __launch_bounds__(kBlock) void pack_f64_write_kernel(F64PackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];  // fixed section, outlier bits
  __shared__ uint32_t s_cnt[kBlock / kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int wm = A.wm, wo = A.wo, we = wo > wm ? wo - wm : 0;
  const uint32_t b = blockIdx.x;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)min((int64_t)kPB, A.n - e0);
  const uint32_t F = fixed_words(wm);
  const uint64_t d = A.dir[b];
  const uint64_t vbase = d & ((1ull << 38) - 1ull);
  const uint32_t n_ext = ext_words(we, (uint32_t)(d >> 38) & 0x1fffu);
  uint32_t* mask = lds;
  uint32_t* plane = lds + kMaskWords;
  uint32_t* ext = lds + F;
  for (uint32_t i = tid; i < F + 128u * (uint32_t)we; i += kBlock) lds[i] = 0u;
  __syncthreads();
  const SmqSmaqStatsF64 st = *A.stats;
  const ElemF64 c = elem_f64_consts(st, A.p);
  const uint64_t off = A.offset + st.rng_offset;
  const uint32_t pmask = (1u << wm) - 1u;
  uint32_t* escs = A.var + vbase + n_ext;
  uint32_t r_out = 0u, r_esc = 0u;
  for (int j = 0; j < kPasses; ++j) {
    const int el = j * kBlock + tid;
    bool o = false, los = false, esc = false;
    double q = 0.0;
    uint32_t code = 0u;
    if (el < n_el) {
      q = f64_q<RM, BN>(A, c, off, e0 + el, o, los);
      code = f64_code(q, o, los, wm, wo, esc);
    }
    const unsigned long long bo = __ballot(o), be = __ballot(esc);
    if (lane == 0) {  // elements j * 256 + w * 64 .. + 63: mask words 8 j + 2 w, + 1
      mask[8 * j + 2 * w] = (uint32_t)bo;
      mask[8 * j + 2 * w + 1] = (uint32_t)(bo >> 32);
    }
    if (code & pmask) or_bits(plane, (uint32_t)wm * (uint32_t)el, code & pmask);
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
    if (o && we > 0 && (code >> wm)) or_bits(ext, (uint32_t)we * (r_out + (before & 0xffffu) + ro), code >> wm);
    if (esc) {
      const uint32_t k = r_esc + (before >> 16) + re;
      const uint64_t qb = q == q ? __builtin_bit_cast(uint64_t, q) : kNaN64;  // one NaN pattern
      escs[kEscWords * k] = (uint32_t)el;
      escs[kEscWords * k + 1] = (uint32_t)qb;
      escs[kEscWords * k + 2] = (uint32_t)(qb >> 32);
    }
    r_out += tot & 0xffffu;
    r_esc += tot >> 16;
  }
  __syncthreads();
  uint32_t* fdst = A.fixed + (size_t)b * F;
  for (uint32_t i = tid; i < F; i += kBlock) fdst[i] = lds[i];
  for (uint32_t i = tid; i < n_ext; i += kBlock) A.var[vbase + i] = ext[i];
}

struct F64UnpackArgs {
  const uint8_t* stream;
  double* y;
  int64_t n;
  int wm, wo;
  uint32_t n_blocks;
};

// One block: fixed section and an escape map (element -> escape index + 1) in LDS, the mask words'
// prefix popcounts for the outlier ranks, then smaq_dequant_f64 per element (BN / all_positive from
// the header's flags: uniform branches). A stream that is not this call's (magic, n, widths, the
// F64 flag) is left undecoded before any directory entry is read.
__global__ __launch_bounds__(kBlock) void unpack_f64_kernel(F64UnpackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];  // fixed section
  __shared__ uint16_t escmap[kPB];
  __shared__ uint32_t mpre[kMaskWords];
  __shared__ uint32_t s_w0;
  const int tid = threadIdx.x;
  const int wm = A.wm, wo = A.wo, we = wo > wm ? wo - wm : 0;
  const SmqPackedHeader* h = reinterpret_cast<const SmqPackedHeader*>(A.stream);
  if (h->magic != SMQ_PACK_MAGIC || h->version != SMQ_PACK_VERSION || h->n != A.n ||
      h->num_bits_main != wm + 1 || h->num_bits_outlier != wo + 1 ||
      !(h->flags & SMQ_PACK_FLAG_F64))
    return;
  const bool bn = (h->flags & SMQ_PACK_FLAG_BN) != 0;
  const bool ap = (h->flags & SMQ_PACK_FLAG_ALL_POSITIVE) != 0;
  const uint64_t* dir = reinterpret_cast<const uint64_t*>(A.stream + sizeof(SmqPackedHeader));
  const uint32_t* fixed = reinterpret_cast<const uint32_t*>(dir + dir_entries(A.n_blocks));
  const uint32_t F = fixed_words(wm);
  const uint32_t* var = fixed + (size_t)A.n_blocks * F;
  const uint32_t b = blockIdx.x;
  const int64_t e0 = (int64_t)b * kPB;
  const int n_el = (int)min((int64_t)kPB, A.n - e0);
  const uint64_t d = dir[b];
  const uint64_t vbase = d & ((1ull << 38) - 1ull);
  const uint32_t n_out = (uint32_t)(d >> 38) & 0x1fffu, n_esc = (uint32_t)(d >> 51);
  const uint32_t n_ext = ext_words(we, n_out);
  const uint32_t* ex = var + vbase;
  const uint32_t* escs = ex + n_ext;
  const uint32_t* fsrc = fixed + (size_t)b * F;
  for (uint32_t i = tid; i < F; i += kBlock) lds[i] = fsrc[i];
  for (int i = tid; i < kPB; i += kBlock) escmap[i] = 0;
  __syncthreads();
  if (tid < kMaskWords) {  // exclusive prefix popcounts of the 128 mask words (two waves)
    const uint32_t cnt = (uint32_t)__popc(lds[tid]);
    const uint32_t inc = wave_incl_scan_u32(cnt);
    if (tid == kWave - 1) s_w0 = inc;
    mpre[tid] = inc - cnt;
  }
  for (uint32_t i = tid; i < n_esc; i += kBlock) escmap[escs[kEscWords * i] & (kPB - 1)] = (uint16_t)(i + 1u);
  __syncthreads();
  if (tid >= kWave && tid < kMaskWords) mpre[tid] += s_w0;
  __syncthreads();
  ElemF64 c;
  memset(&c, 0, sizeof(c));
  c.mean = h->mean_f64;
  c.sd = h->std_dev_f64;
  const float thr = h->thr;
  c.sthr = (double)thr;
  c.snthr = -c.sthr;
  c.zh = (double)(0.0f * -thr);
  c.zl = (double)(0.0f * thr);
  c.r_main = (double)h->range_main;
  c.r_out = (double)h->range_outlier;
  const bool both = (h->flags & SMQ_PACK_FLAG_BOTH_SIDES) != 0;
  const double* gam = nullptr;
  const double* bet = nullptr;
  if (bn) {
    gam = reinterpret_cast<const double*>(var + h->data_words);
    bet = gam + h->bn_channels;
  }
  const uint32_t* mask = lds;
  const uint32_t* plane = lds + kMaskWords;
  for (int j = 0; j < kPasses; ++j) {
    const int el = j * kBlock + tid;
    if (el >= n_el) break;
    const uint32_t mw = mask[el >> 5], bit = (uint32_t)el & 31u;
    uint32_t code = get_bits(plane, (uint32_t)wm * (uint32_t)el, wm);
    double q;
    bool hi, lo;
    if ((mw >> bit) & 1u) {
      const uint32_t rank = mpre[el >> 5] + (uint32_t)__popc(mw & ((1u << bit) - 1u));
      if (we > 0) code |= get_bits(ex, (uint32_t)we * rank, we) << wm;
      const uint32_t side = (code >> (wo - 1)) & 1u;
      const double mag = (double)(code & ((1u << (wo - 1)) - 1u));
      q = side ? -mag : mag;
      hi = side == 0u;
      lo = side != 0u;
    } else {
      q = (double)((code >= (1u << (wm - 1))) ? (int32_t)code - (1 << wm) : (int32_t)code);
      hi = lo = both;
    }
    const uint32_t ei = escmap[el];
    if (ei) {
      const uint32_t* e3 = escs + kEscWords * (ei - 1u);
      q = __builtin_bit_cast(double, (uint64_t)e3[1] | ((uint64_t)e3[2] << 32));
    }
    // smaq_dequant_f64<BN, AP>'s chain with the flags as uniform branches (the same ops)
    double out = smaq_dequant_f64<false, false>(q, hi, lo, c, 1.0, 0.0);
    if (bn) {
      const int64_t ch = ((e0 + el) / h->bn_inner) % (int64_t)h->bn_channels;
      out = (out * gam[ch]) + bet[ch];
    }
    if (ap) out = (out < 0.0) ? 0.0 : out;
    A.y[e0 + el] = out;
  }
}

inline bool aligned8(const void* p) { return ((uintptr_t)p & 7u) == 0; }

}  // namespace

// workspace: the fp64 statistics region (the unpacked round trip's, incl. a large draw) | meta [nb]
static size_t f64_ws_meta(int64_t n, int64_t k) {
  size_t st = smq_smaq_workspace_bytes(n);
  if (k > SMQ_MAX_DEVICE_SAMPLES) {
    const size_t big = smq_smaq_workspace_bytes_sampled(n, k);
    st = big > st ? big : st;
  }
  return (st + 255) & ~(size_t)255;
}

}  // namespace smq

using namespace smq;

extern "C" {

size_t smq_smaq_pack_bound_f64(int64_t n, int num_bits_main, int num_bits_outlier,
                               int64_t bn_channels) {
  if (n < 1) return sizeof(SmqPackedHeader);
  const int wm = num_bits_main - 1, wo = num_bits_outlier - 1;
  const size_t we = wo > wm ? (size_t)(wo - wm) : 0;
  const size_t nb = (size_t)((n + kPB - 1) / kPB);
  // every element an outlier and escaped
  const size_t per_block = fixed_words(wm < 1 ? 1 : wm) + 128 * we + kEscWords * (size_t)kPB;
  return sizeof(SmqPackedHeader) + 8 * (size_t)dir_entries((int64_t)nb) + 4 * nb * per_block +
         16 * (size_t)(bn_channels > 0 ? bn_channels : 0);
}

size_t smq_smaq_pack_workspace_bytes_f64(int64_t n, int64_t num_samples) {
  if (n < 1) n = 1;
  const int64_t k = num_samples < n ? num_samples : n;
  if (k > SMQ_MAX_DRAW_SAMPLES) return 0;
  return f64_ws_meta(n, k) + 4 * (size_t)((n + kPB - 1) / kPB);
}

int smq_smaq_compress_f64(const double* x, int64_t n, const SmqSmaqParams* p, void* packed,
                          size_t packed_bytes, void* ws, size_t ws_bytes, void* stream) {
  int rc = smaq_validate(p, SMQ_DTYPE_F32);
  if (rc) return rc;
  if (n < 1 || !x || !packed || !aligned8(x)) {
    set_error("compress_f64: n >= 1 and non-NULL, 8-B aligned x and packed required");
    return SMQ_ERR_INVALID;
  }
  if (p->num_bits_main < 2 || p->num_bits_main > 25 || p->num_bits_outlier < 3 ||
      p->num_bits_outlier > 25) {
    set_error("compress_f64: needs 2 <= num_bits_main <= 25 and 3 <= num_bits_outlier <= 25");
    return SMQ_ERR_INVALID;
  }
  if (p->main_std_dev_threshold_f64 == 0.0 || !(p->clamp_hi_f64 > 0.0)) {
    set_error("compress_f64: params.main_std_dev_threshold_f64 / clamp_*_f64 unset");
    return SMQ_ERR_INVALID;
  }
  if (p->main_std_dev_threshold_f64 != p->main_std_dev_threshold_f64) {
    set_error("compress_f64: main_std_dev_threshold is NaN");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source != SMQ_STATS_WORKSPACE && p->stats_source != SMQ_STATS_SAMPLED &&
      p->stats_source != SMQ_STATS_SAMPLED_DEVICE) {
    set_error("compress_f64: statistics must be SMQ_STATS_WORKSPACE or SMQ_STATS_SAMPLED(_DEVICE)");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1 ||
                      p->bn_channels > 0x7fffffffLL)) {
    set_error("compress_f64: BN variant needs bn_beta, 1 <= bn_channels < 2^31, bn_inner >= 1");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = (n + kPB - 1) / kPB;
  if (nb > 0x7fffffffLL) {
    set_error("compress_f64: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  const size_t bound = smq_smaq_pack_bound_f64(n, p->num_bits_main, p->num_bits_outlier,
                                               p->bn_gamma ? p->bn_channels : 0);
  if (packed_bytes < bound) {
    set_error("compress_f64: packed buffer too small: need %zu bytes (smq_smaq_pack_bound_f64), "
              "got %zu", bound, packed_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t k = p->stats_source == SMQ_STATS_SAMPLED_DEVICE
                        ? (p->num_samples < n ? p->num_samples : n) : 0;
  const size_t need = smq_smaq_pack_workspace_bytes_f64(n, k);
  if (!ws || need == 0 || ws_bytes < need) {
    set_error("compress_f64: workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  rc = launch_stats_f64(x, n, p, nullptr, ws, ws_bytes, st);
  if (rc) return rc;
  F64PackArgs A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.n = n;
  A.stats = (const SmqSmaqStatsF64*)ws;
  A.hdr = (SmqPackedHeader*)packed;
  A.dir = (uint64_t*)((char*)packed + sizeof(SmqPackedHeader));
  A.wm = p->num_bits_main - 1;
  A.wo = p->num_bits_outlier - 1;
  A.fixed = (uint32_t*)(A.dir + dir_entries(nb));
  A.var = A.fixed + (size_t)nb * fixed_words(A.wm);
  A.meta = (uint32_t*)((char*)ws + f64_ws_meta(n, k));
  A.bn_gamma = reinterpret_cast<const double*>(p->bn_gamma);
  A.bn_beta = reinterpret_cast<const double*>(p->bn_beta);
  A.bn_channels = p->bn_gamma ? p->bn_channels : 0;
  A.bn_inner = p->bn_gamma ? p->bn_inner : 0;
  A.p = *p;
  A.key = rng_key(p->seed);
  A.offset = p->offset;
  A.n_blocks = (uint32_t)nb;
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  A.flags = SMQ_PACK_FLAG_F64 | (p->all_positive ? SMQ_PACK_FLAG_ALL_POSITIVE : 0u) |
            (R.safe_q ? SMQ_PACK_FLAG_SAFE_Q : 0u) |
            (p->main_std_dev_threshold < 0.0f ? SMQ_PACK_FLAG_BOTH_SIDES : 0u) |
            (p->bn_gamma ? SMQ_PACK_FLAG_BN : 0u);
  const int we = A.wo > A.wm ? A.wo - A.wm : 0;
  const size_t lds = 4 * ((size_t)fixed_words(A.wm) + 128 * (size_t)we);
  const dim3 grid((unsigned)nb), block(kBlock);
  const bool sr = p->stochastic_rounding != 0, bn = p->bn_gamma != nullptr;
#define SMQ_F64_PACK(RMV, BNV)                                                                  \
  do {                                                                                          \
    hipLaunchKernelGGL((pack_f64_count_kernel<RMV, BNV>), grid, block, 0, st, A);               \
    hipLaunchKernelGGL(pack_f64_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, A);            \
    hipLaunchKernelGGL((pack_f64_write_kernel<RMV, BNV>), grid, block, lds, st, A);             \
  } while (0)
  if (sr) {
    if (bn) SMQ_F64_PACK(kRoundHash, true); else SMQ_F64_PACK(kRoundHash, false);
  } else {
    if (bn) SMQ_F64_PACK(kRoundTrunc, true); else SMQ_F64_PACK(kRoundTrunc, false);
  }
#undef SMQ_F64_PACK
  return check_launch("pack_f64 kernels");
}

int smq_smaq_decompress_f64(const void* packed, double* y, int64_t n, int num_bits_main,
                            int num_bits_outlier, void* stream) {
  if (n < 1 || !packed || !y || !aligned8(y)) {
    set_error("decompress_f64: n must be >= 1, packed and (8-B aligned) y non-NULL");
    return SMQ_ERR_INVALID;
  }
  if (num_bits_main < 2 || num_bits_main > 25 || num_bits_outlier < 3 || num_bits_outlier > 25) {
    set_error("decompress_f64: needs 2 <= num_bits_main <= 25 and 3 <= num_bits_outlier <= 25");
    return SMQ_ERR_INVALID;
  }
  const int64_t nb = (n + kPB - 1) / kPB;
  if (nb > 0x7fffffffLL) {
    set_error("decompress_f64: tensor too large (%lld elements)", (long long)n);
    return SMQ_ERR_INVALID;
  }
  F64UnpackArgs A;
  A.stream = (const uint8_t*)packed;
  A.y = y;
  A.n = n;
  A.wm = num_bits_main - 1;
  A.wo = num_bits_outlier - 1;
  A.n_blocks = (uint32_t)nb;
  const size_t lds = 4 * (size_t)fixed_words(A.wm);
  hipLaunchKernelGGL(unpack_f64_kernel, dim3((unsigned)nb), dim3(kBlock), lds,
                     (hipStream_t)stream, A);
  return check_launch("unpack_f64_kernel");
}

}  // extern "C"
