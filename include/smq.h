/*
 * smq.h — C-ABI of the MI355X (gfx950) SmaQ / FP8 / S2FP8 round-trip library (libsmq.so).
 *
 * Plain C: raw device pointers, sizes, and an opaque stream handle (a hipStream_t passed as
 * void*, e.g. torch.cuda.current_stream().cuda_stream). No torch types, no HIP headers needed
 * by a caller. Every entry point is re-entrant, never synchronises the host, and launches all of
 * its work on the given stream, so it can be called from the autograd engine's device thread and
 * captured into a hipGraph.
 *
 * Each compute entry point replaces an ATen op sequence inside a reference plugin
 * (paths relative to nimashoghi/smart-quantization):
 *
 *   smq_smaq_stats_f32      smart_compress/compress/smart.py:130-134, 86-91, 100-108, 151-152
 *                           (mean / unbiased std, range-std, sampled stats, std==0 -> 1)
 *   smq_smaq_apply_f32      smart_compress/compress/smart.py:154-182
 *                           (z-score, outlier split, N-bit scale, stochastic/trunc rounding,
 *                            dequantisation, all_positive) + the outlier count of 184-188
 *   smq_smaq_roundtrip_f32  smart.py:130-182 (stats + apply, two launches, no host sync)
 *   smq_smaq_multi_f32      smart.py:110-190 applied to a list of tensors in two launches
 *                           (the per-parameter calls of util/pytorch/optimizer.py:79-127)
 *   smq_float_quant_f32     smart_compress/util/pytorch/quantization.py:187-204 and the
 *                           qtorch 0.2.0 float_quantize it calls (quantization.py:3) —
 *                           used by compress/fp8.py:31, fp16.py:31, bf16.py:31
 *   smq_s2fp8_roundtrip_f32 smart_compress/compress/s2fp8.py:27-48
 *   smq_s2fp8_roundtrip     the same with quantization.py:187-204's precision-16 branch
 *   smq_smaq_compress /     the packed SmaQ container: the codes smart.py:154-169
 *   smq_smaq_decompress     computes, stored in the [outlier flag][sign][N-2 magnitude] layout
 *                           of README.md:25-28 (6 bits per main element, 8 per outlier by
 *                           default) with an escape list for codes outside the budget, so
 *                           decompress(compress(x)) is bit-identical to smart.py:171-182
 *
 * Errors: every function returns SMQ_OK (0) or a negative SMQ_ERR_* code; the message of the
 * last failure on the calling thread is returned by smq_last_error(). Nothing aborts.
 *
 * Workspaces are caller-allocated device memory and must not be used by two streams at the same
 * time. They need no initialisation: every cross-workgroup arrival counter is a 64-bit word tagged
 * with a per-call value (high half) and a count (low half). A call whose tag does not match the
 * word it finds (an unzeroed buffer, a call that never finished) re-installs its own tag with one
 * compare-and-swap instead of miscounting, so one bad call cannot poison later statistics.
 */
#ifndef SMQ_H_
#define SMQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMQ_ABI_VERSION 8

#define SMQ_OK 0
#define SMQ_ERR_INVALID -1  /* bad argument */
#define SMQ_ERR_WORKSPACE -2 /* workspace missing or too small */
#define SMQ_ERR_LAUNCH -3   /* HIP reported an error on launch */

#define SMQ_MAX_SAMPLES 64            /* host-given indices (SMQ_STATS_SAMPLED) */
#define SMQ_MAX_DEVICE_SAMPLES 4096   /* device-drawn indices (SMQ_STATS_SAMPLED_DEVICE) */

/* Single-tensor SmaQ workspace layout (bytes): [0, 64) SmqSmaqStats header, [64, 128) scratch,
 * [128, 640) SMQ_WS_OUTLIER_SLOTS uint64 outlier-count slots
 * (params.count_outliers: the count is their sum; spread so 10^5 workgroups do not serialise on
 * one address), [640, SMQ_WS_SAMPLES_OFFSET) the statistics partials, then the
 * SMQ_MAX_DEVICE_SAMPLES int64 indices the last SMQ_STATS_SAMPLED_DEVICE call drew (in draw
 * order; read them after the stream has reached the call), then 64 tagged arrival counters, then
 * at SMQ_WS_FUSED_OFFSET the single-launch round trip's exchange region (generation word, arrival
 * word, epoch-tagged partial granules; smq_smaq_roundtrip on tensors up to 8,388,611 elements). */
#define SMQ_WS_OUTLIER_SLOTS_OFFSET 128
#define SMQ_WS_OUTLIER_SLOTS 64
#define SMQ_WS_SAMPLES_OFFSET 66176
#define SMQ_WS_FUSED_OFFSET 99584

/* Device-drawn samples beyond SMQ_MAX_DEVICE_SAMPLES, up to SMQ_MAX_DRAW_SAMPLES: the draw runs
 * across workgroups (smaq.hip, "multi-workgroup draw") and needs
 * smq_smaq_workspace_bytes_sampled(n, k) bytes; its k indices land at SMQ_WS_LARGE_SAMPLES_OFFSET
 * (int64, draw order) instead of SMQ_WS_SAMPLES_OFFSET. The indices are the same Floyd draw either
 * way (smq_smaq_draw_samples / oracle/rng.py floyd_indices). */
#define SMQ_MAX_DRAW_SAMPLES (1 << 28)
#define SMQ_WS_LARGE_SAMPLES_OFFSET 199168

/* Where smq_smaq_apply_f32 takes (mean, std) from. */
#define SMQ_STATS_WORKSPACE 0 /* written by smq_smaq_stats_f32 into the workspace header */
#define SMQ_STATS_SAMPLED 1   /* computed in-kernel from params.sample_idx (smart.py:86-91) */
#define SMQ_STATS_INJECTED 2  /* read from the stats_in device pointer (parity tests) */
/* k = min(n, num_samples) <= SMQ_MAX_DRAW_SAMPLES distinct indices drawn ON THE DEVICE by
 * Floyd's algorithm from (seed, offset + graph-safe stream position), a fresh set per call and per
 * hipGraph replay, replacing torch.randperm(n)[:k] (smart.py:88); mean / biased std of the gathered
 * elements as smart.py:86-91. smq_smaq_draw_samples is the host mirror of the draw. */
#define SMQ_STATS_SAMPLED_DEVICE 3

/* Input element types of the SmaQ entry points with a dtype argument. fp16 / bf16 inputs follow
 * the reference's dtype flow: statistics and z-score in the input type, the rest of the chain
 * (and the output) in fp32 (smart.py:154-172 with torch type promotion). */
#define SMQ_DTYPE_F32 0
#define SMQ_DTYPE_F16 1
#define SMQ_DTYPE_BF16 2
/* fp64 tensors: the _f64 entry points (SmaQ, S2FP8) and smq_float_quant / smq_cpu_float_quant.
 * The reference computes fp64 data in fp64 (smart.py:130-182 under torch's type flow: statistics,
 * z-score, rounding and de-quantisation in fp64; the bool*float scalars and ranges tensors hold fp32
 * values) and returns fp64. */
#define SMQ_DTYPE_F64 3

/* Rounding modes of smq_float_quant_f32 (qtorch float_quantize rounding=...). */
#define SMQ_ROUND_NEAREST 0
#define SMQ_ROUND_STOCHASTIC 1

/*
 * SmaQ parameters. Fill with smq_smaq_params_init() (reference defaults, smart.py:11-84) and
 * override fields as the hparams Namespace says. Floating constants are the fp32 roundings of the
 * Python doubles the reference computes (smart.py:72-84).
 */
typedef struct SmqSmaqParams {
  int32_t num_bits_main;        /* --num_bits_main (6) */
  int32_t num_bits_outlier;     /* --num_bits_outlier (8) */
  float main_std_dev_threshold; /* fp32(T_m) (1.0) */
  float range_main;             /* fp32((2^(bm-2)-1)/T_m)             smart.py:76-78 */
  float range_outlier;          /* fp32((2^(bo-2)-1)/(T_o-T_m))       smart.py:72-75 */
  float clamp_lo;               /* fp32(1e-38) or fp32(1e-4) at precision 16, smart.py:80-84 */
  float clamp_hi;               /* fp32(1e38)  or fp32(1e4) */
  float range_std_coef;         /* C = 1/sqrt(2 ln n) for --use_range_std_dev; <0: library computes it (fp32) */
  int32_t stochastic_rounding;  /* 1 = smart.py:93-98, 0 = trunc (smart.py:168-169) */
  int32_t all_positive;         /* clamp_min(0) after dequantisation (smart.py:181-182) */
  int32_t use_range_std_dev;    /* --use_range_std_dev */
  int32_t stats_source;         /* SMQ_STATS_* */
  int32_t count_outliers;       /* accumulate the outlier count into the workspace header */
  int32_t num_samples;          /* k = min(n, --num_samples): entries of sample_idx used
                                   (SMQ_STATS_SAMPLED) or indices drawn (SMQ_STATS_SAMPLED_DEVICE) */
  uint64_t seed;                /* counter-based RNG key (stochastic rounding) */
  uint64_t offset;              /* RNG counter of element 0; element i uses offset + i */
  /* --use_batch_norm (smart.py:136-149, 174-179): per-channel (x - beta[c]) / gamma[c] before the
   * z-score and y * gamma[c] + beta[c] after de-quantisation, c = (i / bn_inner) % bn_channels
   * (channel dim 1 of NCHW; bn_channels = 1 for --bn_scalar_params). NULL gamma = off. */
  const float* bn_gamma;        /* device [bn_channels] */
  const float* bn_beta;         /* device [bn_channels] */
  int64_t bn_channels;
  int64_t bn_inner;             /* H * W */
  int64_t sample_idx[SMQ_MAX_SAMPLES]; /* distinct flat indices for SMQ_STATS_SAMPLED */
  /* Graph-safe random stream: if non-NULL, a device uint64 holding the stream position. The first
   * kernel of the call reads it into the statistics record (SmqSmaqStats.rng_offset) and advances
   * it by n; element i then draws counter offset + rng_offset + i. Nothing on the host changes
   * between calls, so a captured hipGraph replays with fresh, consecutive random streams. */
  uint64_t* offset_counter;
  /* fp64 inputs (smq_smaq_roundtrip_f64, smq_cpu_smaq_roundtrip_f64): the Python doubles the
   * reference compares and clamps fp64 data with (smart.py:82-84, 154-156); smq_smaq_params_set
   * fills them. The scalars / ranges tensors stay fp32 values (torch's default dtype). */
  double main_std_dev_threshold_f64; /* T_m */
  double clamp_lo_f64;               /* 1e-38 (1e-4 at precision 16) */
  double clamp_hi_f64;               /* 1e38 (1e4 at precision 16) */
  double range_std_coef_f64;         /* C = 1/sqrt(2 log n) in fp64 (smart.py:103-105 with
                                        type_as(range_) = double); < 0: the library computes it */
} SmqSmaqParams;

/*
 * Header of a SmaQ workspace (first 64 bytes). Written on the device; read it after the stream
 * has reached the call (e.g. by the Python wrapper's lazy log_size).
 */
typedef struct SmqSmaqStats {
  float mean;          /* data.mean() */
  float std_dev;       /* std after the `std == 0 -> 1` rule (used by the de-normalisation) */
  float std_clamped;   /* std_dev.clamp(clamp_lo, clamp_hi) (used by the normalisation) */
  float raw_std;       /* std before the `std == 0` rule */
  float min_val;       /* min / max (valid in range-std mode) */
  float max_val;
  uint32_t n_used;     /* elements the statistics were computed over */
  uint32_t quot_check; /* library-internal: 1 if (x - mean) / std_clamped can need the IEEE
                          subnormal path (see smaq_elem.h quot_check_for) */
  unsigned long long n_outlier; /* multi-tensor calls: this tensor's outlier count (single-tensor
                                   calls: see SMQ_WS_OUTLIER_SLOTS_OFFSET) */
  double inv_std_clamped;      /* RN64(1 / std_clamped); written by the library (injected stats:
                                  ignored, the library derives it and quot_check itself) */
  unsigned long long rng_offset; /* the call's stream position when params.offset_counter is set
                                    (else 0), added to params.offset by the element kernels */
  float inv_std_clamped_f32;    /* RN32(1 / std_clamped); written by the library (half inputs:
                                   the z-score quotient, smaq_elem.h half_quot) */
  uint32_t reserved;
} SmqSmaqStats;

/* Header of the workspace of an fp64 SmaQ call ([0, 80) of the single-tensor layout; the outlier
 * slots stay at SMQ_WS_OUTLIER_SLOTS_OFFSET). Also the record of SMQ_STATS_INJECTED for the _f64
 * entry points (mean and raw_std read; the rest derived). */
typedef struct SmqSmaqStatsF64 {
  double mean;        /* data.mean() */
  double std_dev;     /* std after the `std == 0 -> 1` rule */
  double std_clamped; /* std_dev.clamp(clamp_lo_f64, clamp_hi_f64) */
  double raw_std;     /* std before the `std == 0` rule */
  double min_val, max_val; /* valid in range-std mode */
  uint32_t n_used;
  uint32_t reserved0;
  unsigned long long rng_offset; /* as SmqSmaqStats.rng_offset */
  unsigned long long reserved[2];
} SmqSmaqStatsF64;

/* One tensor of a multi-tensor call. x holds n elements of the call's dtype; y (fp32) may alias x
 * for fp32 inputs (in-place, the optimizer path). */
typedef struct SmqTensorDesc {
  const void* x;
  float* y;
  int64_t n;
  int32_t all_positive;
  float range_std_coef; /* --use_range_std_dev: C for this tensor (n, or k samples, in its dtype,
                           as the reference's torch ops give it: see SmqSmaqParams.range_std_coef);
                           negative: the library's fp32 1 / sqrt(2 ln n). Unused otherwise. */
  uint64_t rng_offset; /* RNG counter of element 0, relative to params.offset */
} SmqTensorDesc;

/* Header of an S2FP8 workspace. */
typedef struct SmqS2fp8Stats {
  float mu;        /* mean(log2|x|), zeros counted as 0 (s2fp8.py:35-40) */
  float m;         /* max(log2|x|) */
  float alpha;     /* 15 / (m - mu) */
  float beta;      /* -alpha * mu */
  float beta_pow2; /* 2 ** beta */
  float inv_beta_pow2;
  float inv_alpha;
  uint32_t n_used;
  uint64_t rng_offset; /* random-stream position of element 0 relative to the call's offset:
                          the snapshot of *offset_counter (graph-safe mode), else 0 */
  uint32_t reserved[6];
} SmqS2fp8Stats;

/* Header of an fp64 S2FP8 workspace: the reference's fp64 values (s2fp8.py:35-43). */
typedef struct SmqS2fp8StatsF64 {
  double mu, m, alpha, beta, beta_pow2, inv_beta_pow2, inv_alpha;
  uint32_t n_used;
  uint32_t reserved0;
  uint64_t rng_offset;
  uint64_t reserved[3];
} SmqS2fp8StatsF64;

/* ---- library ---- */
int smq_abi_version(void);
const char* smq_last_error(void);

/* Fill p with the reference defaults (smart.py:11-84, precision 32). */
void smq_smaq_params_init(SmqSmaqParams* p);
/* Recompute range_main / range_outlier / clamp_* from bit widths, thresholds and precision. */
int smq_smaq_params_set(SmqSmaqParams* p, int num_bits_main, int num_bits_outlier,
                        double main_std_dev_threshold, double outlier_std_dev_threshold,
                        int precision);
/* Draw k = min(n, num_samples) <= SMQ_MAX_SAMPLES distinct indices in [0, n) into p->sample_idx
 * (host; a deterministic function of (seed, offset)): the same Floyd draw the device performs for
 * SMQ_STATS_SAMPLED_DEVICE at stream position offset. Replaces torch.randperm(n)[:k], smart.py:88. */
int smq_smaq_draw_samples(SmqSmaqParams* p, int64_t n, int num_samples);

/* ---- SmaQ single tensor ---- */
size_t smq_smaq_workspace_bytes(int64_t n);
/* Workspace of a call on n elements with k = min(n, num_samples) device-drawn samples
 * (SMQ_STATS_SAMPLED_DEVICE): smq_smaq_workspace_bytes(n) for k <= SMQ_MAX_DEVICE_SAMPLES, more for
 * the multi-workgroup draw above it (k <= SMQ_MAX_DRAW_SAMPLES; 0 for larger k). */
size_t smq_smaq_workspace_bytes_sampled(int64_t n, int64_t num_samples);
int smq_smaq_stats_f32(const float* x, int64_t n, const SmqSmaqParams* p, void* ws,
                       size_t ws_bytes, void* stream);
/* uniforms: optional device array of n U[0,1) floats replacing the in-kernel RNG (parity tests
 * replay torch.rand_like draws, smart.py:94). stats_in: device pointer, SMQ_STATS_INJECTED only. */
int smq_smaq_apply_f32(const float* x, float* y, int64_t n, const SmqSmaqParams* p,
                       const float* uniforms, const SmqSmaqStats* stats_in, void* ws,
                       size_t ws_bytes, void* stream);
int smq_smaq_roundtrip_f32(const float* x, float* y, int64_t n, const SmqSmaqParams* p,
                           const float* uniforms, void* ws, size_t ws_bytes, void* stream);

/* Same as the _f32 entry points for an input x of element type `dtype` (SMQ_DTYPE_*); the output
 * y is always fp32. For SMQ_DTYPE_F16 / BF16 params.clamp_lo/hi and range_std_coef are the values
 * the reference's torch ops produce in that dtype (the library rounds clamp bounds to it). */
int smq_smaq_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                   size_t ws_bytes, void* stream);
int smq_smaq_apply(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                   const float* uniforms, const SmqSmaqStats* stats_in, void* ws, size_t ws_bytes,
                   void* stream);
/* The round trip as one entry point, always with the same output, header and stream position as
 * smq_smaq_stats + smq_smaq_apply (both statistics paths compute the same partials and reduce them
 * in one fixed order):
 *  - up to 8,388,611 elements (full statistics, fp32 / fp16 / bf16 x 16-B / 8-B aligned, y 16-B
 *    aligned, no BN term, no injected uniforms): ONE launch that holds the tensor in registers
 *    (smaq_fused.hip: every workgroup publishes its statistics partial, gathers all of them, reduces
 *    them and transforms its registers; 8 B/elem of HBM traffic);
 *  - otherwise up to 12M elements (aligned x / y, no BN term): two launches, the statistics' final
 *    reduction deferred to every apply workgroup;
 *  - above: the statistics launch's last workgroup finalises, then the apply launch. */
int smq_smaq_roundtrip(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                       const float* uniforms, void* ws, size_t ws_bytes, void* stream);
/* smq_smaq_roundtrip with path flags (tests and measurement; every path gives the same bytes). */
#define SMQ_SMAQ_SPLIT 1u     /* no single launch: the two-launch path (deferred reduction) */
#define SMQ_SMAQ_NO_DEFER 2u  /* two launches, the statistics launch finalises the header */
#define SMQ_SMAQ_TEST_LATE 4u /* single launch: half of the workgroups start ~500 us late and the
                                 others take missing partials after 20 us (no co-residency) */
int smq_smaq_roundtrip_ex(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                          const float* uniforms, void* ws, size_t ws_bytes, uint32_t flags,
                          void* stream);

/* ---- --measure_compression_ratio without a host synchronisation ----
 * The reference logs, per SmartFP call, new_size = sum(is_outlier) * num_bits_outlier +
 * sum(~is_outlier) * num_bits_main and compression_ratio = orig_size / new_size with orig_size =
 * 32 n (smart.py:184-188, base.py:72-102), converting each to a Python float (a device->host sync
 * per call). These entry points leave the values on the device, as fp64 (exact: < 2^53), for the
 * logger to read when it consumes them. */
typedef struct SmqSizeRecord {
  unsigned long long slots[8];   /* per residue b % 8 of the workgroups: outlier-count partial (low
                                    40 bits) and arrivals (above); ZERO on entry (a fresh record per
                                    call) */
  unsigned long long arrived;    /* residues counted: ZERO on entry */
  unsigned long long reserved[3];
  double n_outlier;              /* written by the call: sum(is_outlier) */
  double new_size;               /* n_outlier * bo + (n - n_outlier) * bm */
  double compression_ratio;      /* orig_size / new_size (IEEE fp64 division: Python's int / int) */
  double orig_size;              /* 32 n */
} SmqSizeRecord;
/* smq_smaq_roundtrip (params.count_outliers is implied) whose outlier count and log_size values
 * land in rec: the single launch counts into rec->slots and its last workgroup writes the values
 * (no extra launch); the other paths count into the workspace slots and one small launch reads
 * them (smq_smaq_size_metrics). rec: device memory, zero-initialised, used by this call only. */
int smq_smaq_roundtrip_counted(const void* x, int dtype, float* y, int64_t n,
                               const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                               SmqSizeRecord* rec, void* stream);
/* The log_size values of the last count_outliers call on the single-tensor workspace ws (n its
 * element count) into rec->n_outlier .. orig_size (rec's other fields are not touched). */
int smq_smaq_size_metrics(const void* ws, int64_t n, int num_bits_main, int num_bits_outlier,
                          SmqSizeRecord* rec, void* stream);
/* The same for the `count` tensors of a multi-tensor call (their statistics records in its
 * workspace, n[t] their element counts, a device int64 array): out[4t .. 4t+3] = n_outlier,
 * new_size, compression_ratio, orig_size of tensor t (fp64, device). */
int smq_smaq_multi_size_metrics(const void* ws, const int64_t* n, int count, int num_bits_main,
                                int num_bits_outlier, double* out, void* stream);
/* fp64 data (smart.py:130-182 on a float64 tensor): statistics, z-score, stochastic or truncating
 * rounding and de-quantisation in fp64, output fp64; every stats_source (k of SMQ_STATS_SAMPLED_DEVICE
 * up to SMQ_MAX_DRAW_SAMPLES with a workspace of smq_smaq_workspace_bytes_sampled), BN
 * (params.bn_gamma / bn_beta then point at fp64 arrays), all_positive, count_outliers.
 * uniforms: optional n fp64 U[0,1) values (torch.rand_like of fp64 data); else the counter RNG's
 * u = (h >> 8) * 2^-24. stats_in: SMQ_STATS_INJECTED only. Header: SmqSmaqStatsF64 at offset 0. */
int smq_smaq_roundtrip_f64(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                           const double* uniforms, const SmqSmaqStatsF64* stats_in, void* ws,
                           size_t ws_bytes, void* stream);

/* ---- SmaQ multi tensor ---- */
/* A plan is a descriptor table plus a chunk map. smq_smaq_multi_plan_build writes it into a host
 * buffer of smq_smaq_multi_plan_bytes; the caller uploads a device copy once and reuses both while
 * the tensor list (pointers and sizes) is unchanged. Tensors with n < min_size must be left out
 * (the reference returns them untouched, smart.py:123-128). */
size_t smq_smaq_multi_plan_bytes(const int64_t* sizes, int count);
int smq_smaq_multi_plan_build(const SmqTensorDesc* descs, int count, void* host_plan,
                              size_t plan_bytes);
size_t smq_smaq_multi_workspace_bytes(const int64_t* sizes, int count);
/* Two launches for the whole list. Statistics of tensor t land in ((SmqSmaqStats*)ws)[t]:
 * SMQ_STATS_WORKSPACE (full statistics, with --use_range_std_dev the range form), or
 * SMQ_STATS_SAMPLED_DEVICE (k = min(n, num_samples) indices per tensor drawn on the device at
 * position offset + snapshot + rng_offset: the draw of a single-tensor call at that offset). The
 * inputs are all of element type `dtype` (SMQ_DTYPE_*), outputs fp32; fp16 / bf16 inputs cannot be
 * updated in place. No BN variant. host_plan is read for its header and descriptors (with
 * params.offset_counter the call advances the counter by max(rng_offset + n) over the tensors;
 * tensor t draws offset + snapshot + rng_offset + i). A multi call equals the sequence of
 * single-tensor calls at those offsets, bit for bit. */
int smq_smaq_multi(const void* dev_plan, const void* host_plan, int dtype, const SmqSmaqParams* p,
                   void* ws, size_t ws_bytes, void* stream);
/* smq_smaq_multi with dtype SMQ_DTYPE_F32. */
int smq_smaq_multi_f32(const void* dev_plan, const void* host_plan, const SmqSmaqParams* p,
                       void* ws, size_t ws_bytes, void* stream);

/* ---- qtorch-style float quantisation (FP8 E5M2, FP16, BF16, any exp/man) ---- */
/* rand_bits: optional device array of n uint32 random words (qtorch's randint_like draws);
 * else the counter-based RNG keyed by (seed, offset + i) is used. check_inf: quantization.py:195-199. */
int smq_float_quant_f32(const float* x, float* y, int64_t n, int exp_bits, int man_bits,
                        int rounding, int check_inf, const uint32_t* rand_bits, uint64_t seed,
                        uint64_t offset, void* stream);
/* The same for any element types: x is SMQ_DTYPE_F32 / F16 / BF16 (quantised as its exact fp32
 * value), y is SMQ_DTYPE_F32 or SMQ_DTYPE_F16 (RN conversion of the fp32 result: the `.half()` of
 * quantization.py:201-202, fused). offset_counter: optional device uint64 holding the stream
 * position; when given, element i draws counter offset + *offset_counter + i and the call
 * advances *offset_counter by n on the stream (graph-safe: nothing is read on the host). */
int smq_float_quant(const void* x, int dtype_in, void* y, int dtype_out, int64_t n, int exp_bits,
                    int man_bits, int rounding, int check_inf, const uint32_t* rand_bits,
                    uint64_t seed, uint64_t offset, uint64_t* offset_counter, void* stream);
/* dtype_in SMQ_DTYPE_F64: each element is quantised as its fp32 rounding (the precision-16 branch's
 * x.float(), quantization.py:190-191; qtorch 0.2.0's kernel itself reads data_ptr<float>() and
 * raises on fp64, so at precision 32 this is the dtype-generic extension: zeros_like(x) filled with
 * the quantised values), written as fp64 (dtype_out SMQ_DTYPE_F64) or fp16 (the `.half()`). */
/* fp32 value of qtorch nearest-quantising FLT_MAX (quantization.py:138-150), host only. */
float smq_float_quant_max_value(int exp_bits, int man_bits);

/* ---- S2FP8 ---- */
size_t smq_s2fp8_workspace_bytes(int64_t n);
/* stats_in: optional device SmqS2fp8Stats whose mu and m are used instead of computing them. */
int smq_s2fp8_roundtrip_f32(const float* x, float* y, int64_t n, int check_inf,
                            const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                            const SmqS2fp8Stats* stats_in, void* ws, size_t ws_bytes,
                            void* stream);

/* S2FP8 for an input of element type `dtype` (SMQ_DTYPE_*) at Lightning precision 16 or 32.
 * precision 32 needs fp32 input (identical to smq_s2fp8_roundtrip_f32). precision 16 follows the
 * reference's dtypes: statistics and |x|^alpha * 2^beta in the input type, float_quantize returns
 * half (quantization.py:201-202), the inverse power runs in half; y is fp16 for fp16 inputs and
 * fp32 for fp32 / bf16 inputs (torch promotion of `... * signs`, s2fp8.py:48). The SmqS2fp8Stats
 * fields hold the input-type values (exact in fp32). offset_counter: as for smq_float_quant
 * (snapshot in SmqS2fp8Stats.rng_offset, taken by the first launch). */
int smq_s2fp8_roundtrip(const void* x, int dtype, void* y, int64_t n, int precision,
                        int check_inf, const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                        uint64_t* offset_counter, const SmqS2fp8Stats* stats_in, void* ws,
                        size_t ws_bytes, void* stream);

/* Flags of smq_s2fp8_roundtrip_ex. OUT_Y / OUT_T (test aids, precision 32 only) write the
 * quantiser's input Y = |x|^alpha * 2^beta or its E5M2 quantisation T (after check_inf) instead of
 * the round-trip output: the S2FP8 parity contract is the E5M2 code of Y (s2fp8.py:45-47).
 * EXACT_POW computes both powers with the accurate (<= 1 ulp) library powf, as the reference's
 * torch.pow does, instead of the hardware exp2(p * log2 x) form (a few ulp; slower ALU, same
 * memory traffic).
 * fp32 precision-32 calls on 16-B-aligned x / y with the statistics computed (stats_in NULL) and no
 * rand_bits run as ONE launch when the tensor fits a resident grid's registers (n <= 4,194,304:
 * 256 chunks of <= 4 float4 per lane of 1024 threads); otherwise, or with SPLIT, as two (statistics
 * partials, then transform). Both give the same bytes: the same chunks and summation order.
 * TEST_LATE (test aid, single launch only): the upper half of the workgroups start ~500 us late
 * and the others take their unclaimed chunks after 20 us, exercising the path that keeps the
 * single launch free of any co-residency assumption. The single launch leaves
 * SmqS2fp8Stats.reserved[0] = 0 (it has no give-up path: a workgroup that waited long for a
 * partial computes it itself). */
#define SMQ_S2FP8_OUT_Y 1u
#define SMQ_S2FP8_OUT_T 2u
#define SMQ_S2FP8_EXACT_POW 4u
#define SMQ_S2FP8_SPLIT 8u
#define SMQ_S2FP8_TEST_LATE 16u
int smq_s2fp8_roundtrip_ex(const void* x, int dtype, void* y, int64_t n, int precision,
                           int check_inf, const uint32_t* rand_bits, uint64_t seed,
                           uint64_t offset, uint64_t* offset_counter,
                           const SmqS2fp8Stats* stats_in, void* ws, size_t ws_bytes,
                           uint32_t flags, void* stream);

/* S2FP8 of fp64 data (s2fp8.py:27-48 in fp64): log2 statistics, alpha, beta, 2^beta and |x|^alpha *
 * 2^beta in fp64; float_quantize of that as for smq_float_quant with SMQ_DTYPE_F64 input. Precision
 * 32 (dtype-generic quantiser): the inverse in fp64. Precision 16: float_quantize returns half and
 * the inverse runs in half as torch does (the 0-dim fp64 reciprocal of 2^beta enters the product at
 * fp32, the exponent 1/alpha rounded to half), times the fp64 signs: y is fp64 either way.
 * flags: SMQ_S2FP8_OUT_Y / OUT_T (precision 32). Three launches (statistics partials, derive,
 * transform); header SmqS2fp8StatsF64 at offset 0 of ws (smq_s2fp8_workspace_bytes(n) bytes). */
int smq_s2fp8_roundtrip_f64(const double* x, double* y, int64_t n, int precision, int check_inf,
                            const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                            uint64_t* offset_counter, const SmqS2fp8StatsF64* stats_in, void* ws,
                            size_t ws_bytes, uint32_t flags, void* stream);

/* ---- CPU tensors ----
 * The codecs on host pointers, for tensors that live on the CPU (the reference's plugins run on
 * any device; BASELINE config 1 is a CPU run). Same argument meaning as the device entry points,
 * minus the stream; n_threads <= 0 uses all hardware threads (at most 256; the library reads no
 * environment variable). Each element uses the device path's arithmetic, so
 * for the same statistics and random stream the SmaQ and float_quant outputs are the device's
 * bytes; statistics are fp64 sums in a fixed order independent of the thread count. S2FP8 uses the
 * C library's powf / log2f (the device's SMQ_S2FP8_EXACT_POW semantics). */
/* Threads the library's CPU pool has started so far (the calling thread included); it grows to
 * what the calls ask for. */
int smq_cpu_threads(void);
/* SmaQ round trip; ws: host buffer of smq_smaq_workspace_bytes(n) bytes that receives the
 * SmqSmaqStats header, the outlier count (slot 0 of SMQ_WS_OUTLIER_SLOTS, when
 * params.count_outliers) and the drawn indices (SMQ_STATS_SAMPLED_DEVICE: the same Floyd draw as the
 * device, any k <= SMQ_MAX_DRAW_SAMPLES; above SMQ_MAX_DEVICE_SAMPLES the buffer is
 * smq_smaq_workspace_bytes_sampled(n, k) bytes and the indices land at SMQ_WS_LARGE_SAMPLES_OFFSET).
 * params.bn_gamma / bn_beta / offset_counter and
 * uniforms / stats_in are host pointers here. */
int smq_cpu_smaq_roundtrip(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                           const float* uniforms, const SmqSmaqStats* stats_in, void* ws,
                           size_t ws_bytes, int n_threads);
/* smq_float_quant on host pointers (no offset_counter). */
int smq_cpu_float_quant(const void* x, int dtype_in, void* y, int dtype_out, int64_t n,
                        int exp_bits, int man_bits, int rounding, int check_inf,
                        const uint32_t* rand_bits, uint64_t seed, uint64_t offset, int n_threads);
/* smq_s2fp8_roundtrip_ex on host pointers; ws (optional, >= 64 bytes) receives SmqS2fp8Stats.
 * flags: OUT_Y / OUT_T as on the device; EXACT_POW and SPLIT are accepted and change nothing. */
int smq_cpu_s2fp8_roundtrip(const void* x, int dtype, void* y, int64_t n, int precision,
                            int check_inf, const uint32_t* rand_bits, uint64_t seed,
                            uint64_t offset, const SmqS2fp8Stats* stats_in, void* ws,
                            size_t ws_bytes, uint32_t flags, int n_threads);

/* The fp64 codecs on host pointers (see the device entry points). */
int smq_cpu_smaq_roundtrip_f64(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                               const double* uniforms, const SmqSmaqStatsF64* stats_in, void* ws,
                               size_t ws_bytes, int n_threads);
int smq_cpu_s2fp8_roundtrip_f64(const double* x, double* y, int64_t n, int precision,
                                int check_inf, const uint32_t* rand_bits, uint64_t seed,
                                uint64_t offset, const SmqS2fp8StatsF64* stats_in, void* ws,
                                size_t ws_bytes, uint32_t flags, int n_threads);

/* ---- host reference helpers shared with the oracle (pure functions, no GPU) ---- */
uint32_t smq_rng_u32(uint64_t seed, uint64_t counter);
/* SmaQ's stochastic-rounding draw of counter `counter` (an integer < 2^24; the uniform is it times
 * 2^-24): the top 24 bits of quad_word(key, counter >> 2) * an odd multiplier of counter & 3 — one
 * hash per four consecutive counters (oracle/rng.py smaq_u24 restates it). */
uint32_t smq_smaq_u24(uint64_t seed, uint64_t counter);
/* Half inputs (dtype SMQ_DTYPE_F16 / BF16, no BN term): the two-op fp32 quotient the apply launch
 * uses for q / range, out[0..3] = {h_main, l_main, h_outlier, l_outlier} with h = RN32(1 / r),
 * l = RN32(1 / r - h), q / r == fmaf(q, h, q * l). Returns 1 when that equals the IEEE quotient for
 * every code the flags can produce (every half z-score; floor + 0/1/2 when stochastic, else trunc),
 * 0 when the launch keeps the fp64 form. oracle/csrc/half_div_check.c (qr mode) restates it. */
int smq_half_quot_split(int dtype, float main_std_dev_threshold, float range_main,
                        float range_outlier, int stochastic_rounding, float* out);


/* ---------------------------------------------------------------------------------------------
 * Packed SmaQ container (format version 2)
 *
 * stream = SmqPackedHeader (128 B)
 *        | directory: n_blocks x uint64 (bits 0-37: word offset of the block's VARIABLE section in
 *          the variable region, 38-50: n_out, 51-63: n_esc), padded with one zero entry when
 *          n_blocks is odd
 *        | fixed region: n_blocks x F words, F = 128 + 128 * wm (block b's at b * F; 16-B aligned)
 *        | variable region: the blocks' variable sections, in block order
 * (every region's place but the variable one's depends on n alone; the variable one's on wm too)
 * block  = SMQ_PACK_BLOCK elements (the last one may be shorter: its absent elements code 0);
 *   wm = num_bits_main - 1, wo = num_bits_outlier - 1, we = max(0, wo - wm);
 *   code of an element: main: wm-bit two's-complement q; outlier: wo bits, top bit = side (1: z < -T,
 *   the code is -q; 0: z > T, the code is q), the rest = |q|; an element whose code does not fit
 *   the budget (|q| too large, a negative q for z > T, a positive q for z < -T, inf / NaN) is an
 *   escape: its code is 0 (main) or the side bit alone (outlier), its q is in the escape list.
 *   fixed section:  w[0 .. 127]  outlier mask: bit (e % 32) of word e / 32 = element e is an outlier
 *                   w[128 ..]    plane: the low wm bits of element e's code at bit wm * e, LSB-first
 *   variable section: the outliers' code bits above the plane (we bits each, in element order,
 *                   LSB-first: ceil(we * n_out / 32) words), then n_esc x {element index in the
 *                   block, q as float32 bits (any NaN q as 0x7fc00000)} in element order
 * Size: the same bits as an element-order stream of wm-bit main and wo-bit outlier codes, but the
 * fixed section can be written the moment its block is coded (no prefix over earlier blocks).
 *        | BatchNorm table (flag SMQ_PACK_FLAG_BN only): bn_channels gammas then bn_channels betas
 *          (fp32), right after the variable region (word data_words of it)
 * Decoding: q -> (q / range) - scalars, * std + mean (smart.py:171-182), then * gamma[c] + beta[c]
 * with c = (element / bn_inner) % bn_channels for a BN stream (smart.py:174-179), bit-identical to
 * smq_smaq_apply for the same statistics, BN parameters, rounding mode and random stream.
 * Thresholds: T_m >= 0 makes the sides exclusive (mask bit = outlier). T_m < 0 (flag
 * SMQ_PACK_FLAG_BOTH_SIDES) adds a third state, z above T_m and below -T_m at once (smart.py:157-158
 * both true: scalars -T_m + T_m, range_outlier): such an element has mask bit 0 and codes as a main
 * element (wm-bit two's complement q) that the decoder de-quantises with both sides set.
 * float64 streams (flag SMQ_PACK_FLAG_F64; smq_smaq_compress_f64): the codes of the fp64 chain
 * (smart.py on a float64 tensor: z, q and the de-quantisation in fp64, scalars and ranges the fp32
 * values), the same sections, with three words per escape {element index, q as float64 bits low
 * word, high word} (any NaN q as 0x7ff8000000000000), the statistics as doubles (header
 * mean_f64 / std_dev_f64) and a BN table of fp64 gammas then betas; decoded to float64.
 * ------------------------------------------------------------------------------------------- */
#define SMQ_PACK_MAGIC 0x50514d53u /* "SMQP" */
#define SMQ_PACK_VERSION 2u
#define SMQ_PACK_BLOCK 4096

typedef struct SmqPackedHeader {
  uint32_t magic;             /* SMQ_PACK_MAGIC */
  uint32_t version;           /* SMQ_PACK_VERSION */
  int64_t n;                  /* elements */
  uint32_t block_elems;       /* SMQ_PACK_BLOCK */
  uint32_t n_blocks;
  int32_t num_bits_main, num_bits_outlier;
  uint32_t flags;             /* bit 0: all_positive, bit 1: IEEE q / range (absurd ranges),
                                 SMQ_PACK_FLAG_BOTH_SIDES, SMQ_PACK_FLAG_BN */
  float thr;                  /* T_m (fp32) */
  float range_main, range_outlier;
  float mean, std_dev;        /* de-normalisation statistics (std after the ==0 rule) */
  double inv_range_main, inv_range_outlier;
  uint64_t data_words;        /* size of the data region in uint32 words */
  uint64_t total_bytes;       /* header + directory + data */
  uint32_t error;             /* 0 (no packing launch waits on another workgroup) */
  uint32_t bn_channels;       /* BN streams: channels of the table (1: scalar parameters), else 0 */
  int64_t bn_inner;           /* BN streams: elements per channel run (H * W of NCHW), else 0 */
  double mean_f64, std_dev_f64; /* float64 streams (SMQ_PACK_FLAG_F64): the statistics, else 0 */
  uint32_t reserved[2];
} SmqPackedHeader;

#define SMQ_PACK_FLAG_ALL_POSITIVE 1u
#define SMQ_PACK_FLAG_SAFE_Q 2u
#define SMQ_PACK_FLAG_BOTH_SIDES 4u /* T_m < 0: a mask-0 element has both outlier sides */
#define SMQ_PACK_FLAG_BN 8u         /* the BatchNorm table follows the variable region */
#define SMQ_PACK_FLAG_F64 16u       /* float64 stream: 3-word escapes, fp64 statistics / BN table */

/* Worst-case stream size (every element an outlier and escaped) for n elements; the stream's real
 * size is header.total_bytes. */
size_t smq_smaq_pack_bound(int64_t n, int num_bits_main, int num_bits_outlier);
/* The same for a BN stream of bn_channels channels (+ 8 bytes per channel for its table). */
size_t smq_smaq_pack_bound_bn(int64_t n, int num_bits_main, int num_bits_outlier,
                              int64_t bn_channels);
/* Workspace of smq_smaq_compress: statistics, per-block sizes, group sums / prefixes and a
 * 3 KiB scratch slot per block for its variable section (0.75 B per element); needs no
 * initialisation. */
size_t smq_smaq_pack_workspace_bytes(int64_t n);
/* Statistics (full / sampled / range, params as smq_smaq_stats) then the packing launches: codes,
 * fixed sections and variable-section sizes (one workgroup per block), a scan of the group sizes
 * (header), the variable sections moved to their prefix (one workgroup per 64 blocks; a block
 * whose section outgrew its scratch slot is re-coded from x there). Up to 2048 blocks (8,388,608
 * elements; 16-B aligned x, T_m > 0, no BN term) the packing is ONE launch instead: each block
 * finds its variable section's offset by a decoupled look-back over the blocks before it and
 * writes it in place; the bytes are the same. The host is never synchronised; the stream incl.
 * header.total_bytes is written on the device. packed_bytes >= smq_smaq_pack_bound (smq_smaq_pack_bound_bn with params->bn_gamma:
 * the BN variant, whose parameters are copied into the stream). Any threshold but NaN. */
int smq_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* params,
                      void* packed, size_t packed_bytes, void* workspace, size_t workspace_bytes,
                      void* stream);
/* Packing flags of smq_smaq_compress_ex, kept for ABI compatibility with format version 1 (whose
 * single-launch look-back packer they selected): accepted and without effect — there is one packer
 * and it gives the same bytes whatever the flags. */
#define SMQ_PACK_TICKETED 1u
#define SMQ_PACK_SINGLE 2u
int smq_smaq_compress_ex(const void* x, int dtype, int64_t n, const SmqSmaqParams* params,
                         void* packed, size_t packed_bytes, void* workspace,
                         size_t workspace_bytes, uint32_t flags, void* stream);
/* Bytes of a stream's parts that do not depend on the data: header, directory, fixed region. */
size_t smq_smaq_pack_fixed_bytes(int64_t n, int num_bits_main);
/* y = smq_smaq_roundtrip(x) AND the stream of the same call (the codes whose decoding is y, bit for
 * bit): one statistics pass (the single launch up to 8,388,611 elements, else the statistics and
 * apply launches) whose record the packing launches then read — no statistics launch of their own,
 * no decode of the stream to get y. The random stream advances once (n counters), as for either
 * call alone. Same params, workspace (smq_smaq_pack_workspace_bytes[_sampled]) and statistics
 * sources as smq_smaq_compress; x must not alias y. packed_bytes may be anything from
 * smq_smaq_pack_fixed_bytes up: a variable section (or the BN table) that would end past the
 * buffer is not written, and header.total_bytes > packed_bytes then tells the caller that the
 * stream did not fit (it must not be decoded). With packed_bytes >= smq_smaq_pack_bound[_bn] the
 * stream equals smq_smaq_compress's byte for byte. Reference: smart.py:110-190 (y) and its
 * log_size codes (smart.py:184-188) kept for real (README.md:25-28). */
int smq_smaq_roundtrip_compress(const void* x, int dtype, float* y, int64_t n,
                                const SmqSmaqParams* params, void* packed, size_t packed_bytes,
                                void* workspace, size_t workspace_bytes, void* stream);
/* The same with the packing launches on pack_stream (NULL or == stream: one stream): they wait for
 * stream's statistics by an event and then overlap what the caller enqueues on stream next (y is
 * ready on stream as usual). The caller orders every reader of the stream after pack_stream and
 * keeps x, packed and the workspace alive (and the workspace unused by other calls) until
 * pack_stream has passed them. */
int smq_smaq_roundtrip_compress_ex(const void* x, int dtype, float* y, int64_t n,
                                   const SmqSmaqParams* params, void* packed, size_t packed_bytes,
                                   void* workspace, size_t workspace_bytes, void* stream,
                                   void* pack_stream);
/* smq_smaq_roundtrip_compress whose launch that writes the header also stores header.total_bytes
 * into *notify as a 32-bit value (SMQ_NOTIFY_SATURATED when it is 2^32 - 1 or more; NULL: none),
 * by a system-scope store: with notify in host-mapped coherent memory (hipHostMalloc with
 * hipHostMallocCoherent) the host sees whether the stream fitted its buffer as soon as the launch
 * has written it — no event, no copy, no synchronisation. The caller sets *notify to
 * SMQ_NOTIFY_PENDING before the call. notify must be 4-byte aligned. Reference: the log_size
 * total (smart.py:184-188) PackedActivations needs to drop the fp32 activation (README.md:25). */
#define SMQ_NOTIFY_PENDING 0xFFFFFFFFu
#define SMQ_NOTIFY_SATURATED 0xFFFFFFFEu
int smq_smaq_roundtrip_compress_notify(const void* x, int dtype, float* y, int64_t n,
                                       const SmqSmaqParams* params, void* packed,
                                       size_t packed_bytes, void* workspace,
                                       size_t workspace_bytes, uint32_t* notify, void* stream);
/* count notify words in host-mapped coherent memory (hipHostMalloc, coherent | mapped | portable:
 * one address for the host and every device), each set to SMQ_NOTIFY_PENDING; NULL on failure. Free
 * with smq_notify_free once no launch that may still write them is in flight. */
uint32_t* smq_notify_alloc(int64_t count);
void smq_notify_free(uint32_t* words);
/* Decode a stream of n elements into y (fp32). n must equal the header's n (a stream with another
 * n or a bad magic leaves y untouched). */
int smq_smaq_decompress(const void* packed, float* y, int64_t n, void* stream);
/* The same with the stream's bit widths given by the caller (who compressed it, e.g. with its
 * hparams): the fixed and variable regions are located without waiting for the header (256M:
 * ~6 % faster). A stream whose header records other widths leaves y untouched. */
int smq_smaq_decompress_ex(const void* packed, float* y, int64_t n, int num_bits_main,
                           int num_bits_outlier, void* stream);
/* Workspace of smq_smaq_compress / smq_cpu_smaq_compress with SMQ_STATS_SAMPLED_DEVICE and
 * num_samples samples (above SMQ_MAX_DEVICE_SAMPLES the multi-workgroup draw's region comes first:
 * smart.py:86-91 for any k the unpacked codec takes). Equals smq_smaq_pack_workspace_bytes(n) for
 * num_samples <= SMQ_MAX_DEVICE_SAMPLES. */
size_t smq_smaq_pack_workspace_bytes_sampled(int64_t n, int64_t num_samples);
/* Host twins for CPU tensors (host pointers; smart.py:110-190 runs on any device): the same
 * statistics as smq_cpu_smaq_roundtrip, the same codes and the same stream layout as
 * smq_smaq_compress — byte for byte the device stream whenever the statistics agree (they are fp64
 * sums in another fixed order: equal but for rare last-bit cases) — and its decoder, which reads
 * any version-2 stream. Synchronous, on n_threads threads; workspace as smq_smaq_compress's first
 * region (smq_smaq_workspace_bytes[_sampled] bytes: the statistics header is left at its start). */
int smq_cpu_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* params,
                          void* packed, size_t packed_bytes, void* workspace,
                          size_t workspace_bytes, int n_threads);
int smq_cpu_smaq_decompress(const void* packed, float* y, int64_t n, int n_threads);

/* float64 tensors (smart.py:110-190 on a float64 tensor: the fp64 chain of smq_smaq_roundtrip_f64)
 * in a float64 stream (flag SMQ_PACK_FLAG_F64): decompress_f64(compress_f64(x)) equals
 * smq_smaq_roundtrip_f64(x) bit for bit for the same statistics and random stream. Statistics:
 * params.stats_source SMQ_STATS_WORKSPACE, _SAMPLED or _SAMPLED_DEVICE (params' *_f64 fields set);
 * rounding: hash or truncation; BN parameters (bn_gamma / bn_beta) as doubles. Not bandwidth-tuned:
 * statistics, a counting launch (codes per block), a one-workgroup scan (directory, header) and a
 * writing launch that recomputes the codes and stores both sections at their final places. */
size_t smq_smaq_pack_bound_f64(int64_t n, int num_bits_main, int num_bits_outlier,
                               int64_t bn_channels);
size_t smq_smaq_pack_workspace_bytes_f64(int64_t n, int64_t num_samples);
int smq_smaq_compress_f64(const double* x, int64_t n, const SmqSmaqParams* params, void* packed,
                          size_t packed_bytes, void* workspace, size_t workspace_bytes,
                          void* stream);
/* The widths the stream was written with (a stream that is not a float64 stream of n elements and
 * these widths is left undecoded: y unchanged). */
int smq_smaq_decompress_f64(const void* packed, double* y, int64_t n, int num_bits_main,
                            int num_bits_outlier, void* stream);
/* Host twins (the same bytes as the device stream whenever the statistics agree). */
int smq_cpu_smaq_compress_f64(const double* x, int64_t n, const SmqSmaqParams* params,
                              void* packed, size_t packed_bytes, void* workspace,
                              size_t workspace_bytes, int n_threads);
int smq_cpu_smaq_decompress_f64(const void* packed, double* y, int64_t n, int n_threads);

#ifdef __cplusplus
}
#endif

#endif /* SMQ_H_ */
