// fp64.hip — float64 tensors through the SmaQ round trip, float_quantize and S2FP8 (gfx950).
//
// The reference's codecs are plain torch ops, so a float64 tensor runs them in fp64:
//   smart.py:130-182   mean / std (or range-std, or sampled) in fp64; (x - mean) / std.clamp(1e-38,
//                      1e38) with the clamp bounds and the outlier threshold as Python doubles; the
//                      bool*float scalars and the torch.where ranges are fp32 tensors (torch's
//                      default dtype) whose values promote into the fp64 chain; rand_like draws fp64
//                      uniforms; the output is fp64.
//   quantization.py:187-204 / qtorch 0.2.0: the quantiser works on fp32 words; precision 16 hands it
//                      x.float(). At precision 32 qtorch's kernel reads data_ptr<float>() and raises
//                      on fp64 — here it is dtype-generic: zeros_like(x) (fp64) filled with the
//                      quantised fp32(x).
//   s2fp8.py:27-48     log2 statistics, alpha, beta, 2^beta and |x|^alpha * 2^beta in fp64; the
//                      inverse in fp64 (precision 32) or, where float_quantize returns half
//                      (precision 16), in half as torch computes it, times the fp64 signs.
// Every fp64 op of those chains is one IEEE op here in the same order (-ffp-contract=off; `/` is the
// correctly rounded fp64 division), so for the same statistics and uniforms the outputs are the
// fp64 restatement's (oracle/smaq.py dtype "f64") bit for bit. Statistics are fp64 sums in a fixed
// order: within a few ulp of torch's (a different summation order).
//
// These are not bandwidth-tuned kernels (fp64 SmaQ moves 24 B per element against fp32's 12): plain
// coalesced 8-B element accesses, 4 per lane in flight, one launch per phase.
#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "qtorch.h"
#include "smaq_elem.h"
#include "smaq_f64.h"
#include "smaq_host.h"
#include "smq_common.h"

namespace smq {

constexpr int kF64Per = 4;            // elements per lane per tile
constexpr int kF64StatsGridCap = 1024;

struct alignas(32) PartialF64 {
  double s1, s2, mn, mx;
};
static_assert(SmaqWsLayout::kPartials + sizeof(PartialF64) * kF64StatsGridCap <= SMQ_WS_SAMPLES_OFFSET,
              "fp64 partials overflow the partials region");
static_assert(sizeof(SmqSmaqStatsF64) <= SMQ_WS_OUTLIER_SLOTS_OFFSET, "fp64 header too large");

__device__ __forceinline__ double wave_min_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}

// Workgroup reduction of a PartialF64 (fixed order); result valid in thread 0.
__device__ __forceinline__ void block_reduce_f64(PartialF64& a) {
  __shared__ PartialF64 sh[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  a.s1 = wave_sum(a.s1);
  a.s2 = wave_sum(a.s2);
  a.mn = wave_min_f64(a.mn);
  a.mx = wave_max_f64(a.mx);
  if (lane == 0) sh[wave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.s1 = (sh[0].s1 + sh[1].s1) + (sh[2].s1 + sh[3].s1);
    a.s2 = (sh[0].s2 + sh[1].s2) + (sh[2].s2 + sh[3].s2);
    a.mn = fmin(fmin(sh[0].mn, sh[1].mn), fmin(sh[2].mn, sh[3].mn));
    a.mx = fmax(fmax(sh[0].mx, sh[1].mx), fmax(sh[2].mx, sh[3].mx));
  }
  __syncthreads();
}

struct StatsF64Args {
  const double* x;
  int64_t n;              // elements of the tensor (the stream advance of a call)
  int64_t count;          // elements the statistics cover (n, or k samples)
  const int64_t* pick;    // sampled: the gathered indices (NULL: x[0 .. n))
  int biased;
  int use_range;
  double clamp_lo, clamp_hi, range_coef;
  unsigned long long* rng_ctr;
  PartialF64* parts;
  SmqSmaqStatsF64* hdr;
};

__device__ __forceinline__ double stats_f64_shift(const StatsF64Args& A) {
  if (A.pick) return A.x[A.pick[0]];
  return median3_f64(A.x[0], A.x[A.n >> 1], A.x[A.n - 1]);
}

// Per-workgroup shifted sums over x[0 .. n) (pick == NULL) or over the gathered samples.
__global__ __launch_bounds__(kBlock) void smaq_f64_stats_kernel(StatsF64Args A) {
  const double shift = stats_f64_shift(A);
  PartialF64 acc{0.0, 0.0, INFINITY, -INFINITY};
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.count; i += stride) {
    const double v = A.pick ? A.x[A.pick[i]] : A.x[i];
    const double d = v - shift;
    acc.s1 += d;
    acc.s2 = fma(d, d, acc.s2);
    acc.mn = fmin(acc.mn, v);
    acc.mx = fmax(acc.mx, v);
  }
  block_reduce_f64(acc);
  if (threadIdx.x == 0) A.parts[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void smaq_f64_finalize_kernel(StatsF64Args A, int g) {
  PartialF64 acc{0.0, 0.0, INFINITY, -INFINITY};
  for (int b = threadIdx.x; b < g; b += kBlock) {
    const PartialF64 q = A.parts[b];
    acc.s1 += q.s1;
    acc.s2 += q.s2;
    acc.mn = fmin(acc.mn, q.mn);
    acc.mx = fmax(acc.mx, q.mx);
  }
  block_reduce_f64(acc);
  if (threadIdx.x == 0) {
    SmqSmaqStatsF64 st;
    finalize_f64(acc.s1, acc.s2, acc.mn, acc.mx, A.count, stats_f64_shift(A), A.biased != 0,
                 A.use_range != 0, A.clamp_lo, A.clamp_hi, A.range_coef, &st);
    unsigned long long base = 0ull;
    if (A.rng_ctr) {  // graph-safe stream: snapshot for this call, advance by n
      base = *A.rng_ctr;
      *A.rng_ctr = base + (unsigned long long)A.n;
    }
    st.rng_offset = base;
    *A.hdr = st;
  }
}

// Sampled statistics of up to SMQ_MAX_DEVICE_SAMPLES indices by one workgroup: host-given
// (SMQ_STATS_SAMPLED) or drawn here (Floyd, draw_picks) and recorded at SMQ_WS_SAMPLES_OFFSET.
// Mean, then the biased second moment about it (smart.py:86-91), in fp64.
struct SmallSampleF64Args {
  StatsF64Args S;
  int k;
  int draw;               // 1: Floyd draw at the call's stream position
  uint32_t key;
  uint64_t offset;
  int64_t* idx_out;
  int64_t host_idx[SMQ_MAX_SAMPLES];
};

__global__ __launch_bounds__(kBlock) void smaq_f64_sample_kernel(SmallSampleF64Args A) {
  __shared__ DrawLds L;
  __shared__ double shs[kBlock / kWave];
  const int k = A.k;
  if (A.draw) {
    __shared__ unsigned long long pos_s;
    if (threadIdx.x == 0) pos_s = A.offset + (A.S.rng_ctr ? *A.S.rng_ctr : 0ull);
    __syncthreads();
    draw_picks(A.S.n, k, A.key, pos_s, L);
  } else {
    for (int i = threadIdx.x; i < k; i += kBlock) L.pick[i] = A.host_idx[i];
    __syncthreads();
  }
  double s = 0.0, mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < k; i += kBlock) {
    const int64_t e = L.pick[i];
    if (A.idx_out) A.idx_out[i] = e;
    const double v = A.S.x[e];
    s += v;
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  s = wave_sum(s);
  if (lane == 0) shs[wave] = s;
  __syncthreads();
  const double mean = ((shs[0] + shs[1]) + (shs[2] + shs[3])) / (double)k;
  double m2 = 0.0;
  for (int i = threadIdx.x; i < k; i += kBlock) {
    const double d = A.S.x[L.pick[i]] - mean;
    m2 = fma(d, d, m2);
  }
  PartialF64 acc{0.0, m2, mn, mx};
  block_reduce_f64(acc);
  if (threadIdx.x == 0) {
    SmqSmaqStatsF64 st;
    finalize_f64(0.0, acc.s2, acc.mn, acc.mx, k, mean, true, A.S.use_range != 0, A.S.clamp_lo,
                 A.S.clamp_hi, A.S.range_coef, &st);
    unsigned long long base = 0ull;
    if (A.S.rng_ctr) {
      base = *A.S.rng_ctr;
      *A.S.rng_ctr = base + (unsigned long long)A.S.n;
    }
    st.rng_offset = base;
    *A.S.hdr = st;
  }
}

// SMQ_STATS_INJECTED: mean and raw_std from the caller, the ==0 rule and the clamp derived.
__global__ void smaq_f64_inject_kernel(const SmqSmaqStatsF64* in, StatsF64Args A) {
  if (threadIdx.x == 0) {
    SmqSmaqStatsF64 st = *in;
    const double sd = st.raw_std;
    const double std_dev = (sd == 0.0) ? 1.0 : sd;
    double sc = std_dev < A.clamp_lo ? A.clamp_lo : std_dev;
    sc = sc > A.clamp_hi ? A.clamp_hi : sc;
    st.std_dev = std_dev;
    st.std_clamped = sc;
    unsigned long long base = 0ull;
    if (A.rng_ctr) {
      base = *A.rng_ctr;
      *A.rng_ctr = base + (unsigned long long)A.n;
    }
    st.rng_offset = base;
    *A.hdr = st;
  }
}

struct ApplyF64Args {
  const double* x;
  double* y;
  int64_t n;
  const double* uniforms;
  const SmqSmaqStatsF64* hdr;
  unsigned long long* out_slots;
  SmqSmaqParams p;  // by value: the constants and BN pointers
  uint32_t key;
  int count;
};

template <int RM, bool BN, bool AP>
__global__ __launch_bounds__(kBlock) void smaq_f64_apply_kernel(ApplyF64Args A) {
  __shared__ uint32_t sh_cnt[kBlock / kWave];
  const SmqSmaqStatsF64 st = *A.hdr;
  const ElemF64 c = elem_f64_consts(st, A.p);
  const uint64_t off = A.p.offset + st.rng_offset;
  const double* gam = reinterpret_cast<const double*>(A.p.bn_gamma);
  const double* bet = reinterpret_cast<const double*>(A.p.bn_beta);
  const int64_t e0 = (int64_t)blockIdx.x * (kBlock * kF64Per) + threadIdx.x;
  double v[kF64Per], u[kF64Per];
#pragma unroll
  for (int j = 0; j < kF64Per; ++j) {
    const int64_t e = e0 + j * kBlock;
    v[j] = e < A.n ? A.x[e] : 0.0;
    u[j] = 0.0;
    if (RM == kRoundUniform && e < A.n) u[j] = A.uniforms[e];
  }
  uint32_t n_out = 0;
#pragma unroll
  for (int j = 0; j < kF64Per; ++j) {
    const int64_t e = e0 + j * kBlock;
    if (e >= A.n) continue;
    double uu = u[j];
    if (RM == kRoundHash) uu = (double)smaq_u24(A.key, off + (uint64_t)e);
    double g = 1.0, b = 0.0;
    if (BN) {
      const int64_t ch = (e / A.p.bn_inner) % A.p.bn_channels;
      g = gam[ch];
      b = bet[ch];
    }
    bool o;
    A.y[e] = smaq_elem_f64<RM, BN, AP>(v[j], uu, c, o, g, b);
    n_out += o ? 1u : 0u;
  }
  if (A.count) {
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const uint32_t t = wave_sum_u32(n_out);
    if (lane == 0) sh_cnt[wave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long s = (unsigned long long)sh_cnt[0] + sh_cnt[1] + sh_cnt[2] + sh_cnt[3];
      if (s) atomicAdd(A.out_slots + (blockIdx.x & (SMQ_WS_OUTLIER_SLOTS - 1)), s);
    }
  }
}

}  // namespace smq

// The statistics of an fp64 call into the workspace header (SmqSmaqStatsF64 at offset 0): full,
// sampled (host-given or device-drawn, any k) or injected (smaq_host.h; the packed codec's too).
int smq::launch_stats_f64(const double* x, int64_t n, const SmqSmaqParams* p,
                          const SmqSmaqStatsF64* stats_in, void* ws, size_t ws_bytes,
                          hipStream_t st) {
  int rc = SMQ_OK;
  char* wb = (char*)ws;
  StatsF64Args S;
  memset(&S, 0, sizeof(S));
  S.x = x;
  S.n = n;
  S.count = n;
  S.use_range = p->use_range_std_dev;
  S.clamp_lo = p->clamp_lo_f64;
  S.clamp_hi = p->clamp_hi_f64;
  S.rng_ctr = (unsigned long long*)p->offset_counter;
  S.parts = (PartialF64*)(wb + SmaqWsLayout::kPartials);
  S.hdr = (SmqSmaqStatsF64*)wb;
  auto coef = [&](int64_t cnt) {
    return p->range_std_coef_f64 >= 0.0 ? p->range_std_coef_f64 : 1.0 / sqrt(2.0 * log((double)cnt));
  };
  switch (p->stats_source) {
    case SMQ_STATS_WORKSPACE: {
      S.range_coef = coef(n);
      const int g = (int)std::min<int64_t>(kF64StatsGridCap, (n + 16 * kBlock - 1) / (16 * kBlock));
      hipLaunchKernelGGL(smaq_f64_stats_kernel, dim3(g), dim3(kBlock), 0, st, S);
      hipLaunchKernelGGL(smaq_f64_finalize_kernel, dim3(1), dim3(kBlock), 0, st, S, g);
      break;
    }
    case SMQ_STATS_SAMPLED:
    case SMQ_STATS_SAMPLED_DEVICE: {
      const int64_t k = p->num_samples < n ? p->num_samples : n;
      const bool draw = p->stats_source == SMQ_STATS_SAMPLED_DEVICE;
      const int64_t cap = draw ? SMQ_MAX_DRAW_SAMPLES : SMQ_MAX_SAMPLES;
      if (k < 1 || k > cap) {
        set_error("smaq f64: sampled statistics need 1 <= k <= %lld", (long long)cap);
        return SMQ_ERR_INVALID;
      }
      S.count = k;
      S.biased = 1;
      S.range_coef = coef(k);
      if (draw && k > SMQ_MAX_DEVICE_SAMPLES) {
        LargeDrawArgs D;
        int g = 0;
        rc = launch_large_draw(n, k, p, ws, ws_bytes, st, &D, &g);
        if (rc) return rc;
        S.pick = D.pick;
        S.parts = (PartialF64*)D.parts;  // room for kDrawGridCap StatPartial (32 B) entries
        static_assert(sizeof(PartialF64) == sizeof(StatPartial), "partial sizes");
        hipLaunchKernelGGL(smaq_f64_stats_kernel, dim3(g), dim3(kBlock), 0, st, S);
        hipLaunchKernelGGL(smaq_f64_finalize_kernel, dim3(1), dim3(kBlock), 0, st, S, g);
        break;
      }
      SmallSampleF64Args A;
      memset(&A, 0, sizeof(A));
      A.S = S;
      A.k = (int)k;
      A.draw = draw ? 1 : 0;
      if (draw) {
        A.key = rng_key(p->seed ^ kDrawSalt);
        A.offset = p->offset;
        A.idx_out = (int64_t*)(wb + SMQ_WS_SAMPLES_OFFSET);
      } else {
        for (int j = 0; j < (int)k; ++j) {
          if (p->sample_idx[j] < 0 || p->sample_idx[j] >= n) {
            set_error("smaq f64: sample_idx[%d] out of range", j);
            return SMQ_ERR_INVALID;
          }
          A.host_idx[j] = p->sample_idx[j];
        }
      }
      hipLaunchKernelGGL(smaq_f64_sample_kernel, dim3(1), dim3(kBlock), 0, st, A);
      break;
    }
    default: {
      if (!stats_in) {
        set_error("smaq f64: SMQ_STATS_INJECTED needs stats_in");
        return SMQ_ERR_INVALID;
      }
      hipLaunchKernelGGL(smaq_f64_inject_kernel, dim3(1), dim3(kWave), 0, st, stats_in, S);
    }
  }
  return check_launch("smaq_f64 statistics");
}

namespace smq {

static int smaq_f64_impl(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                         const double* uniforms, const SmqSmaqStatsF64* stats_in, void* ws,
                         size_t ws_bytes, hipStream_t st) {
  int rc = smaq_validate(p, SMQ_DTYPE_F32);
  if (rc) return rc;
  if (n < 1 || !x || !y) {
    set_error("smaq f64: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (p->main_std_dev_threshold_f64 == 0.0 || !(p->clamp_hi_f64 > 0.0)) {
    set_error("smaq f64: params.main_std_dev_threshold_f64 / clamp_*_f64 unset "
              "(smq_smaq_params_set fills them)");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1)) {
    set_error("smaq f64: batch-norm parameters incomplete");
    return SMQ_ERR_INVALID;
  }
  if (!ws || ws_bytes < smq_smaq_workspace_bytes(n)) {
    set_error("smaq f64: workspace too small: need %zu bytes", smq_smaq_workspace_bytes(n));
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t tiles = (n + kBlock * kF64Per - 1) / (kBlock * kF64Per);
  if (tiles > 0x7fffffffLL) {
    set_error("smaq f64: tensor too large");
    return SMQ_ERR_INVALID;
  }
  rc = launch_stats_f64(x, n, p, stats_in, ws, ws_bytes, st);
  if (rc) return rc;
  char* wb = (char*)ws;
  ApplyF64Args A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.y = y;
  A.n = n;
  A.uniforms = uniforms;
  A.hdr = (const SmqSmaqStatsF64*)wb;
  A.out_slots = (unsigned long long*)(wb + SmaqWsLayout::kSlots);
  A.p = *p;
  A.key = rng_key(p->seed);
  A.count = p->count_outliers;
  if (p->count_outliers) fill_async(A.out_slots, 0ull, SMQ_WS_OUTLIER_SLOTS, st);
  const int rm = !p->stochastic_rounding ? kRoundTrunc : (uniforms ? kRoundUniform : kRoundHash);
  const bool bn = p->bn_gamma != nullptr, ap = p->all_positive != 0;
  const dim3 grid((unsigned)tiles);
#define SMQ_F64_APPLY(RMV)                                                                              \
  do {                                                                                                  \
    if (bn) { if (ap) hipLaunchKernelGGL((smaq_f64_apply_kernel<RMV, true, true>), grid, dim3(kBlock), 0, st, A); \
              else hipLaunchKernelGGL((smaq_f64_apply_kernel<RMV, true, false>), grid, dim3(kBlock), 0, st, A); } \
    else { if (ap) hipLaunchKernelGGL((smaq_f64_apply_kernel<RMV, false, true>), grid, dim3(kBlock), 0, st, A); \
           else hipLaunchKernelGGL((smaq_f64_apply_kernel<RMV, false, false>), grid, dim3(kBlock), 0, st, A); } \
  } while (0)
  if (rm == kRoundHash) SMQ_F64_APPLY(kRoundHash);
  else if (rm == kRoundUniform) SMQ_F64_APPLY(kRoundUniform);
  else SMQ_F64_APPLY(kRoundTrunc);
#undef SMQ_F64_APPLY
  return check_launch("smaq_f64_apply_kernel");
}

// ---- float_quantize of fp64 data ------------------------------------------------------------------
struct FqF64Args {
  const double* x;
  void* y;
  int64_t n;
  const uint32_t* rand_bits;
  const uint64_t* ctr;
  uint32_t key;
  uint64_t offset;
  int exp_bits, man_bits, sr, check_inf;
  float max_value;
};

template <bool HOUT>
__global__ __launch_bounds__(kBlock) void fq_f64_kernel(FqF64Args A) {
  const uint64_t off = A.offset + (A.ctr ? *A.ctr : 0ull);
  const int64_t e0 = (int64_t)blockIdx.x * (kBlock * kF64Per) + threadIdx.x;
#pragma unroll
  for (int j = 0; j < kF64Per; ++j) {
    const int64_t e = e0 + j * kBlock;
    if (e >= A.n) continue;
    const uint32_t r = !A.sr ? 0u : (A.rand_bits ? A.rand_bits[e] : rng_u32(A.key, off + (uint64_t)e));
    float q = qtorch_quant((float)A.x[e], r, A.exp_bits, A.man_bits, A.sr != 0);
    if (A.check_inf && fabsf(q - A.max_value) <= FLT_EPSILON) q = INFINITY;
    if (HOUT) static_cast<__half*>(A.y)[e] = __float2half_rn(q);
    else static_cast<double*>(A.y)[e] = (double)q;
  }
}

__global__ void fq_f64_bump_kernel(uint64_t* ctr, uint64_t n) {
  if (threadIdx.x == 0) *ctr += n;
}

int float_quant_f64(const double* x, void* y, int dtype_out, int64_t n, int exp_bits, int man_bits,
                    int rounding, int check_inf, const uint32_t* rand_bits, uint64_t seed,
                    uint64_t offset, uint64_t* offset_counter, float max_value, hipStream_t st) {
  if (dtype_out != SMQ_DTYPE_F64 && dtype_out != SMQ_DTYPE_F16) {
    set_error("float_quant: fp64 input takes dtype_out SMQ_DTYPE_F64 or SMQ_DTYPE_F16 (got %d)",
              dtype_out);
    return SMQ_ERR_INVALID;
  }
  if (n == 0) return SMQ_OK;
  FqF64Args A;
  A.x = x;
  A.y = y;
  A.n = n;
  A.rand_bits = rand_bits;
  A.ctr = offset_counter;
  A.key = rng_key(seed);
  A.offset = offset;
  A.exp_bits = exp_bits;
  A.man_bits = man_bits;
  A.sr = rounding == SMQ_ROUND_STOCHASTIC ? 1 : 0;
  A.check_inf = check_inf;
  A.max_value = max_value;
  const dim3 grid((unsigned)((n + kBlock * kF64Per - 1) / (kBlock * kF64Per)));
  if (dtype_out == SMQ_DTYPE_F16) hipLaunchKernelGGL(fq_f64_kernel<true>, grid, dim3(kBlock), 0, st, A);
  else hipLaunchKernelGGL(fq_f64_kernel<false>, grid, dim3(kBlock), 0, st, A);
  if (offset_counter)
    hipLaunchKernelGGL(fq_f64_bump_kernel, dim3(1), dim3(kWave), 0, st, offset_counter, (uint64_t)n);
  return check_launch("fq_f64_kernel");
}

// ---- S2FP8 of fp64 data -------------------------------------------------------------------------
struct alignas(16) S2PartF64 {
  double s, m;
};

struct S2F64Args {
  const double* x;
  double* y;
  int64_t n;
  S2PartF64* parts;
  SmqS2fp8StatsF64* hdr;
  const SmqS2fp8StatsF64* stats_in;
  uint64_t* rng_ctr;
  const uint32_t* rand_bits;
  uint32_t key;
  uint64_t offset;
  int check_inf, out_mode;
  float max_value;
};

__global__ __launch_bounds__(kBlock) void s2fp8_f64_stats_kernel(S2F64Args A) {
  __shared__ S2PartF64 sh[kBlock / kWave];
  double s = 0.0, m = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n;
       i += (int64_t)gridDim.x * kBlock) {
    const double l = s2_log_f64(A.x[i]);
    s += l;
    m = nan_max_f64(m, l);
  }
  s = wave_sum(s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = nan_max_f64(m, __shfl_xor(m, o, kWave));
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) sh[wave] = S2PartF64{s, m};
  __syncthreads();
  if (threadIdx.x == 0)
    A.parts[blockIdx.x] = S2PartF64{(sh[0].s + sh[1].s) + (sh[2].s + sh[3].s),
                                    nan_max_f64(nan_max_f64(sh[0].m, sh[1].m),
                                                nan_max_f64(sh[2].m, sh[3].m))};
}

__global__ __launch_bounds__(kWave) void s2fp8_f64_derive_kernel(S2F64Args A, int g) {
  if (threadIdx.x != 0) return;
  SmqS2fp8StatsF64 st;
  memset(&st, 0, sizeof(st));
  if (A.stats_in) {
    s2_derive_f64(A.stats_in->mu * (double)A.n, A.stats_in->m, A.n, &st);
    st.mu = A.stats_in->mu;  // as given (mu * n / n need not round back)
    const double alpha = (1.0 / (st.m - st.mu)) * 15.0;
    st.alpha = alpha;
    st.beta = (-alpha) * st.mu;
    st.beta_pow2 = pow(2.0, st.beta);
    st.inv_beta_pow2 = 1.0 / st.beta_pow2;
    st.inv_alpha = 1.0 / alpha;
  } else {
    double s = 0.0, m = -INFINITY;
    for (int b = 0; b < g; ++b) {
      s += A.parts[b].s;
      m = nan_max_f64(m, A.parts[b].m);
    }
    s2_derive_f64(s, m, A.n, &st);
  }
  uint64_t base = 0ull;
  if (A.rng_ctr) {
    base = *A.rng_ctr;
    *A.rng_ctr = base + (uint64_t)A.n;
  }
  st.rng_offset = base;
  *A.hdr = st;
}

template <bool P16>
__global__ __launch_bounds__(kBlock) void s2fp8_f64_apply_kernel(S2F64Args A) {
  const SmqS2fp8StatsF64 s = *A.hdr;
  const uint64_t off = A.offset + s.rng_offset;
  const int64_t e0 = (int64_t)blockIdx.x * (kBlock * kF64Per) + threadIdx.x;
#pragma unroll
  for (int j = 0; j < kF64Per; ++j) {
    const int64_t e = e0 + j * kBlock;
    if (e >= A.n) continue;
    const uint32_t r = A.rand_bits ? A.rand_bits[e] : rng_u32(A.key, off + (uint64_t)e);
    A.y[e] = s2_elem_f64<P16>(A.x[e], r, s, A.check_inf, A.max_value, A.out_mode);
  }
}

}  // namespace smq

using namespace smq;

extern "C" {

int smq_smaq_roundtrip_f64(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                           const double* uniforms, const SmqSmaqStatsF64* stats_in, void* ws,
                           size_t ws_bytes, void* stream) {
  return smaq_f64_impl(x, y, n, p, uniforms, stats_in, ws, ws_bytes, (hipStream_t)stream);
}

int smq_s2fp8_roundtrip_f64(const double* x, double* y, int64_t n, int precision, int check_inf,
                            const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                            uint64_t* offset_counter, const SmqS2fp8StatsF64* stats_in, void* ws,
                            size_t ws_bytes, uint32_t flags, void* stream) {
  if (n < 1 || !x || !y) {
    set_error("s2fp8 f64: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (precision != 16 && precision != 32) {
    set_error("s2fp8 f64: precision must be 16 or 32 (got %d)", precision);
    return SMQ_ERR_INVALID;
  }
  if (flags & ~(SMQ_S2FP8_OUT_Y | SMQ_S2FP8_OUT_T | SMQ_S2FP8_EXACT_POW | SMQ_S2FP8_SPLIT)) {
    set_error("s2fp8 f64: unsupported flags 0x%x", flags);
    return SMQ_ERR_INVALID;
  }
  if ((flags & SMQ_S2FP8_OUT_Y) && (flags & SMQ_S2FP8_OUT_T)) {
    set_error("s2fp8 f64: SMQ_S2FP8_OUT_Y and SMQ_S2FP8_OUT_T are exclusive");
    return SMQ_ERR_INVALID;
  }
  const int out_mode = (flags & SMQ_S2FP8_OUT_Y) ? 1 : ((flags & SMQ_S2FP8_OUT_T) ? 2 : 0);
  if (out_mode && precision != 32) {
    set_error("s2fp8 f64: SMQ_S2FP8_OUT_* need precision 32");
    return SMQ_ERR_INVALID;
  }
  // header + at most 1024 partials: within smq_s2fp8_workspace_bytes (53,504 B)
  const int g = (int)std::min<int64_t>(1024, (n + 16 * kBlock - 1) / (16 * kBlock));
  const size_t need = 256 + sizeof(S2PartF64) * (size_t)g;
  static_assert(sizeof(SmqS2fp8StatsF64) <= 256, "fp64 S2FP8 header");
  if (!ws || ws_bytes < need || ws_bytes < smq_s2fp8_workspace_bytes(n)) {
    set_error("s2fp8 f64: workspace too small: need %zu bytes", smq_s2fp8_workspace_bytes(n));
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t tiles = (n + kBlock * kF64Per - 1) / (kBlock * kF64Per);
  if (tiles > 0x7fffffffLL) {
    set_error("s2fp8 f64: tensor too large");
    return SMQ_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  S2F64Args A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.y = y;
  A.n = n;
  A.hdr = (SmqS2fp8StatsF64*)ws;
  A.parts = (S2PartF64*)((char*)ws + 256);
  A.stats_in = stats_in;
  A.rng_ctr = offset_counter;
  A.rand_bits = rand_bits;
  A.key = rng_key(seed);
  A.offset = offset;
  A.check_inf = check_inf;
  A.out_mode = out_mode;
  A.max_value = smq_float_quant_max_value(5, 2);
  if (!stats_in) hipLaunchKernelGGL(s2fp8_f64_stats_kernel, dim3(g), dim3(kBlock), 0, st, A);
  hipLaunchKernelGGL(s2fp8_f64_derive_kernel, dim3(1), dim3(kWave), 0, st, A, g);
  if (precision == 16)
    hipLaunchKernelGGL(s2fp8_f64_apply_kernel<true>, dim3((unsigned)tiles), dim3(kBlock), 0, st, A);
  else
    hipLaunchKernelGGL(s2fp8_f64_apply_kernel<false>, dim3((unsigned)tiles), dim3(kBlock), 0, st, A);
  return check_launch("s2fp8_f64_apply_kernel");
}

}  // extern "C"
