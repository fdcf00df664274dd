// cpu_codecs.hip — the same codecs on CPU tensors (host pointers), for callers whose tensors live on
// the host: the reference's plugins run on whatever device the tensor is on (smart.py:110-190,
// quantization.py:187-204, s2fp8.py:27-48 are plain torch ops), and BASELINE config 1 is a CPU
// run. Host code only (this translation unit has no kernels); it is built with the rest of
// libsmq.so so that it shares the element arithmetic's helpers (counter RNG, Floyd draw, qtorch
// bit code) with the device path.
//
// Every element is computed with the device path's arithmetic in the same order, so for the same
// statistics and random stream the bytes are the same as the GPU's (SmaQ, float_quantize):
//   * z = (x - mean) / std_clamped and q / range as IEEE fp32 divisions — the device's
//     RN32(RN64(a * RN64(1/b))) equals them (smaq_elem.h div_by_const, proven exact);
//   * SR draws u = smaq_u24(key, offset + i), t = fma(u, -2^-24, fr) + 0.5 (one rounding);
//   * fp16 / bf16 inputs follow the torch type flow with the same round-to-nearest-even steps.
// Statistics are fp64 sums in a fixed order (per 64K-element task, combined in task order: the
// result does not depend on the thread count); the device sums in another fixed order, so mean /
// std can differ from the GPU's in the last fp32 bit in rare cases (both are within 1 ulp of the
// exact value, tests/test_cpu_codecs.py).
// S2FP8 powers use the C library's powf / log2f (the device's SMQ_S2FP8_EXACT_POW semantics).
//
// Parallelism: a process-wide pool of std::threads (no OpenMP runtime next to torch's); the
// calling thread takes part. Work is split into fixed 64K-element tasks.
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "qtorch.h"
#include "smaq_elem.h"
#include "smaq_f64.h"
#include "smaq_host.h"
#include "smq_common.h"

namespace smq {
namespace cpu {

constexpr int64_t kTask = 1 << 16;  // elements per task

// ---- thread pool ----------------------------------------------------------------------------------
// Workers are started on demand (a call asking for T threads makes sure T - 1 exist, at most
// kMaxThreads - 1): the library reads no environment variable for its thread count; the caller
// passes it (the Python host: torch's intra-op thread count).
constexpr int kMaxThreads = 256;

class Pool {
 public:
  Pool() = default;
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size() + 1; }

  // fn(task) for task in [0, n_tasks) on up to n_threads threads (the caller included)
  void run(int64_t n_tasks, int n_threads, const std::function<void(int64_t)>& fn) {
    std::lock_guard<std::mutex> one_job(job_mu_);
    grow(std::min<int64_t>((int64_t)std::max(n_threads, 1) - 1, n_tasks - 1));
    int helpers = std::min<int64_t>((int64_t)std::max(n_threads, 1) - 1, n_tasks - 1);
    helpers = std::max(0, std::min(helpers, (int)workers_.size()));
    if (helpers == 0) {
      for (int64_t t = 0; t < n_tasks; ++t) fn(t);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_tasks_ = n_tasks;
      next_.store(0, std::memory_order_relaxed);
      active_ = helpers;
      pending_ = helpers;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const int64_t t = next_.fetch_add(1, std::memory_order_relaxed);
      if (t >= n_tasks_) return;
      (*fn_)(t);
    }
  }
  // called under job_mu_: no job is running, so a new worker starts from the current generation
  void grow(int64_t want) {
    want = std::min<int64_t>(want, kMaxThreads - 1);
    uint64_t g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      g = gen_;
    }
    while ((int64_t)workers_.size() < want) {
      const int i = (int)workers_.size();
      workers_.emplace_back([this, i, g] { loop(i, g); });
    }
  }
  void loop(int idx, uint64_t seen) {
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        if (idx >= active_) continue;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_tasks_ = 0;
  std::atomic<int64_t> next_{0};
  int active_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

static Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: no join at exit
  return *p;
}

// n_threads <= 0: the machine's hardware threads (capped)
static int threads_for(int n_threads) {
  if (n_threads > 0) return std::min(n_threads, kMaxThreads);
  const unsigned hc = std::thread::hardware_concurrency();
  return hc ? (int)std::min(hc, (unsigned)kMaxThreads) : 1;
}

template <class F>
static void parallel_tasks(int64_t n, int n_threads, F&& f) {
  const int64_t tasks = (n + kTask - 1) / kTask;
  const std::function<void(int64_t)> fn = [&](int64_t t) {
    const int64_t i0 = t * kTask;
    f(t, i0, std::min(n, i0 + kTask));
  };
  pool().run(tasks, threads_for(n_threads), fn);
}

// ---- element types ------------------------------------------------------------------------------
static inline float h2f(uint16_t h) {  // fp16 -> fp32 (exact)
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  if (e == 0x1fu) return u2f(s | 0x7f800000u | (m << 13));
  if (e == 0) return m ? (s ? -1.0f : 1.0f) * (float)m * 0x1p-24f : u2f(s);
  return u2f(s | ((e + 112u) << 23) | (m << 13));
}

static inline uint16_t f2h(float f) {  // fp32 -> fp16, round to nearest even
  const uint32_t x = f2u(f), s = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(s | 0x7c00u | (ax > 0x7f800000u ? (0x200u | ((ax >> 13) & 0x3ffu)) : 0u));
  if (ax >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);  // rounds to inf
  if (ax < 0x38800000u) {                                   // fp16 subnormal (or zero)
    const float t = u2f(ax) * 0x1p24f;                      // exact; < 2^10
    return (uint16_t)(s | (uint32_t)rintf(t));              // RN-even (0x400 = smallest normal)
  }
  const uint32_t r = ax - 0x38000000u;  // rebias 127 -> 15
  return (uint16_t)(s | ((r + 0x0fffu + ((r >> 13) & 1u)) >> 13));
}

static inline float bf2f(uint16_t h) { return u2f((uint32_t)h << 16); }

static inline float round_bf16(float v) {  // RN-even to bf16, as an fp32 value
  const uint32_t u = f2u(v);
  if ((u & 0x7fffffffu) > 0x7f800000u) return u2f((u | 0x00400000u) & 0xffff0000u);
  return u2f((u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
}

template <int T>
static inline float rin(float v) {  // round_in<T> on the host
  if (T == kF16) return h2f(f2h(v));
  if (T == kBF16) return round_bf16(v);
  return v;
}

template <int T>
static inline float ld(const void* p, int64_t i) {
  if (T == kF32) return static_cast<const float*>(p)[i];
  if (T == SMQ_DTYPE_F64) return (float)static_cast<const double*>(p)[i];  // the x.float() RN
  const uint16_t h = static_cast<const uint16_t*>(p)[i];
  return T == kF16 ? h2f(h) : bf2f(h);
}

static inline float hash_u24(uint32_t key, uint64_t ctr) {  // rng_hu: smaq_u24 as a float
  return (float)smaq_u24(key, ctr);
}

// ---- SmaQ statistics ----------------------------------------------------------------------------
struct Moments {
  double s1 = 0.0, s2 = 0.0;
  float mn = INFINITY, mx = -INFINITY;
};

// Shifted fp64 sums of one task: 8 interleaved chains (element i of the task in chain i % 8),
// combined in a fixed order.
template <int T>
static Moments task_moments(const void* x, int64_t i0, int64_t i1, double shift) {
  double a1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mn[8], mx[8];
  for (int j = 0; j < 8; ++j) {
    mn[j] = INFINITY;
    mx[j] = -INFINITY;
  }
  int64_t i = i0;
  for (; i + 8 <= i1; i += 8) {
    for (int j = 0; j < 8; ++j) {
      const float v = ld<T>(x, i + j);
      const double d = (double)v - shift;
      a1[j] += d;
      a2[j] = fma(d, d, a2[j]);
      mn[j] = fminf(mn[j], v);
      mx[j] = fmaxf(mx[j], v);
    }
  }
  for (int j = 0; i < i1; ++i, ++j) {
    const float v = ld<T>(x, i);
    const double d = (double)v - shift;
    a1[j] += d;
    a2[j] = fma(d, d, a2[j]);
    mn[j] = fminf(mn[j], v);
    mx[j] = fmaxf(mx[j], v);
  }
  Moments m;
  m.s1 = ((a1[0] + a1[1]) + (a1[2] + a1[3])) + ((a1[4] + a1[5]) + (a1[6] + a1[7]));
  m.s2 = ((a2[0] + a2[1]) + (a2[2] + a2[3])) + ((a2[4] + a2[5]) + (a2[6] + a2[7]));
  for (int j = 0; j < 8; ++j) {
    m.mn = fminf(m.mn, mn[j]);
    m.mx = fmaxf(m.mx, mx[j]);
  }
  return m;
}

// smaq_elem.h finalize_stats on the host (the same formulas).
template <int T>
static void finalize(double s1, double s2, float mn, float mx, int64_t n, double shift, bool biased,
                     bool range, float clamp_lo, float clamp_hi, float range_coef,
                     SmqSmaqStats* out) {
  const double nd = (double)n;
  const double mean = shift + s1 / nd;
  float sd;
  if (range) {
    sd = rin<T>(rin<T>(mx - mn) * range_coef);
  } else {
    double var = (s2 - s1 * (s1 / nd)) / (biased ? nd : (nd - 1.0));
    if (var < 0.0) var = 0.0;
    sd = rin<T>((float)sqrt(var));
  }
  const float std_dev = (sd == 0.0f) ? 1.0f : sd;
  const float lo = rin<T>(clamp_lo), hi = rin<T>(clamp_hi);
  float sc = std_dev < lo ? lo : std_dev;
  sc = sc > hi ? hi : sc;
  memset(out, 0, sizeof(*out));
  out->mean = rin<T>((float)mean);
  out->std_dev = std_dev;
  out->std_clamped = sc;
  out->raw_std = sd;
  out->min_val = mn;
  out->max_val = mx;
  out->n_used = (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n);
  out->inv_std_clamped = 1.0 / (double)sc;
  out->inv_std_clamped_f32 = (float)out->inv_std_clamped;
  out->quot_check = quot_check_for(sc);
}

template <int T>
static void full_stats(const void* x, int64_t n, const SmqSmaqParams* p, float range_coef,
                       int n_threads, SmqSmaqStats* out) {
  const float k0 = ld<T>(x, 0), k1 = ld<T>(x, n >> 1), k2 = ld<T>(x, n - 1);
  const double shift = (double)fmaxf(fminf(k0, k1), fminf(fmaxf(k0, k1), k2));  // as the device
  std::vector<Moments> part((size_t)((n + kTask - 1) / kTask));
  parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
    part[(size_t)t] = task_moments<T>(x, i0, i1, shift);
  });
  Moments tot;
  for (const Moments& m : part) {
    tot.s1 += m.s1;
    tot.s2 += m.s2;
    tot.mn = fminf(tot.mn, m.mn);
    tot.mx = fmaxf(tot.mx, m.mx);
  }
  finalize<T>(tot.s1, tot.s2, tot.mn, tot.mx, n, shift, false, p->use_range_std_dev != 0,
              p->clamp_lo, p->clamp_hi, range_coef, out);
}

// smart.py:86-91 over k given indices: mean, biased std (shift = mean, as the device)
template <int T>
static void sampled_stats(const void* x, const int64_t* idx, int64_t k, const SmqSmaqParams* p,
                          float range_coef, SmqSmaqStats* out) {
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = 0; i < k; ++i) {
    const float v = ld<T>(x, idx[i]);
    s += (double)v;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  const double mean = s / (double)k;
  double m2 = 0.0;
  for (int64_t i = 0; i < k; ++i) {
    const double d = (double)ld<T>(x, idx[i]) - mean;
    m2 = fma(d, d, m2);
  }
  finalize<T>(0.0, m2, mn, mx, k, mean, true, p->use_range_std_dev != 0, p->clamp_lo, p->clamp_hi,
              range_coef, out);
}

// The device draw (smaq_elem.h Floyd, smq_smaq_draw_samples) for any k <= SMQ_MAX_DRAW_SAMPLES.
static void floyd_draw(uint64_t seed, uint64_t pos, int64_t n, int64_t k, int64_t* out) {
  const uint32_t key = rng_key(seed ^ kDrawSalt);
  std::unordered_set<int64_t> seen;
  seen.reserve((size_t)(2 * k));
  for (int i = 0; i < (int)k; ++i) {
    int64_t t = floyd_candidate(key, pos, n, (int)k, i);
    if (!seen.insert(t).second) {
      t = n - k + i;
      seen.insert(t);
    }
    out[i] = t;
  }
}

// ---- SmaQ element pass --------------------------------------------------------------------------
struct SmaqCtx {
  const void* x;
  float* y;
  const float* uniforms;
  const float* bn_gamma;
  const float* bn_beta;
  int64_t bn_channels, bn_inner;
  float mean, sd, sc, thr, nthr, cthr, cnthr, zh, zl, r_main, r_out;
  uint32_t key;
  uint64_t off;  // params.offset + stream snapshot
};

// smart.py:144-182 for elements [i0, i1): smaq_quant + smaq_dequant with the device's arithmetic.
// RM: kRoundHash / kRoundUniform / kRoundTrunc. Returns the outliers among them.
template <int T, int RM, bool BN, bool AP>
static uint64_t smaq_task(const SmaqCtx& c, int64_t i0, int64_t i1) {
  constexpr int TZ = BN ? kF32 : T;
  uint64_t n_out = 0;
  for (int64_t i = i0; i < i1; ++i) {
    float v = ld<T>(c.x, i);
    float g = 1.0f, bb = 0.0f;
    if (BN) {
      const int64_t ch = (i / c.bn_inner) % c.bn_channels;
      g = c.bn_gamma[ch];
      bb = c.bn_beta[ch];
      v = (v - bb) / g;
    }
    const float dm = rin<TZ>(v - c.mean);
    const float z = rin<TZ>(dm / c.sc);
    const bool hi = z > c.cthr, lo = z < c.cnthr, o = hi || lo;
    const float a = (hi ? c.nthr : c.zh) + (lo ? c.thr : c.zl);
    const float r = o ? c.r_out : c.r_main;
    const float d = (z + a) * r;
    float q;
    if (RM == kRoundTrunc) {
      q = truncf(d);
    } else {
      const float f = floorf(d);
      const float fr = d - f;
      float t;
      if (RM == kRoundHash)
        t = fmaf(hash_u24(c.key, c.off + (uint64_t)i), -0x1p-24f, fr) + 0.5f;
      else
        t = (fr - c.uniforms[i]) + 0.5f;
      t = (t < 0.0f) ? 0.0f : t;
      q = f + rintf(t);
    }
    float out = q / r - a;
    out = out * c.sd;
    out = out + c.mean;
    if (BN) {
      out = out * g;
      out = out + bb;
    }
    if (AP) out = (out < 0.0f) ? 0.0f : out;
    c.y[i] = out;
    n_out += o ? 1u : 0u;
  }
  return n_out;
}

template <int T>
static uint64_t smaq_pass(const SmaqCtx& c, int64_t n, int rm, bool bn, bool ap, int n_threads) {
  std::vector<uint64_t> part((size_t)((n + kTask - 1) / kTask));
  auto go = [&](auto rm_c, auto bn_c, auto ap_c) {
    parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
      part[(size_t)t] = smaq_task<T, decltype(rm_c)::value, decltype(bn_c)::value,
                                  decltype(ap_c)::value>(c, i0, i1);
    });
  };
  using H = std::integral_constant<int, kRoundHash>;
  using U = std::integral_constant<int, kRoundUniform>;
  using R = std::integral_constant<int, kRoundTrunc>;
  using Y = std::true_type;
  using N = std::false_type;
  if (rm == kRoundHash) {
    if (bn) { if (ap) go(H(), Y(), Y()); else go(H(), Y(), N()); }
    else { if (ap) go(H(), N(), Y()); else go(H(), N(), N()); }
  } else if (rm == kRoundUniform) {
    if (bn) { if (ap) go(U(), Y(), Y()); else go(U(), Y(), N()); }
    else { if (ap) go(U(), N(), Y()); else go(U(), N(), N()); }
  } else {
    if (bn) { if (ap) go(R(), Y(), Y()); else go(R(), Y(), N()); }
    else { if (ap) go(R(), N(), Y()); else go(R(), N(), N()); }
  }
  uint64_t tot = 0;
  for (uint64_t v : part) tot += v;
  return tot;
}

static float range_coef_host(const SmqSmaqParams* p, int64_t n) {
  if (p->range_std_coef >= 0.0f) return p->range_std_coef;
  const float lg = logf((float)n);
  return 1.0f / sqrtf(2.0f * lg);
}

// The call's statistics (full, host-given or drawn samples, injected) into *st; *base = the host
// mirror of the graph-safe stream position (params.offset_counter), not yet advanced.
template <int T>
static int host_stats(const void* x, int64_t n, const SmqSmaqParams* p,
                      const SmqSmaqStats* stats_in, char* ws, size_t ws_bytes, int n_threads,
                      SmqSmaqStats* out, uint64_t* base_out) {
  SmqSmaqStats& st = *out;
  // a host uint64 stream position (graph-safe mirror), advanced by n only once the call is
  // validated: a rejected call consumes no stream positions, like the device entry points
  const uint64_t base = p->offset_counter ? *p->offset_counter : 0ull;
  *base_out = base;
  switch (p->stats_source) {
    case SMQ_STATS_WORKSPACE:
      full_stats<T>(x, n, p, range_coef_host(p, n), n_threads, &st);
      break;
    case SMQ_STATS_SAMPLED: {
      const int64_t k = std::min<int64_t>(p->num_samples, n);
      if (k < 1 || k > SMQ_MAX_SAMPLES) {
        set_error("cpu smaq: num_samples must be in [1, %d] for SMQ_STATS_SAMPLED", SMQ_MAX_SAMPLES);
        return SMQ_ERR_INVALID;
      }
      for (int64_t i = 0; i < k; ++i)
        if (p->sample_idx[i] < 0 || p->sample_idx[i] >= n) {
          set_error("cpu smaq: sample index %lld out of range", (long long)p->sample_idx[i]);
          return SMQ_ERR_INVALID;
        }
      sampled_stats<T>(x, p->sample_idx, k, p, range_coef_host(p, k), &st);
      break;
    }
    case SMQ_STATS_SAMPLED_DEVICE: {
      const int64_t k = std::min<int64_t>(p->num_samples, n);
      if (k < 1 || k > SMQ_MAX_DRAW_SAMPLES) {
        set_error("cpu smaq: num_samples must be in [1, %d]", SMQ_MAX_DRAW_SAMPLES);
        return SMQ_ERR_INVALID;
      }
      if (ws_bytes < smq_smaq_workspace_bytes_sampled(n, k)) {
        set_error("cpu smaq: workspace too small for %lld samples: need %zu bytes", (long long)k,
                  smq_smaq_workspace_bytes_sampled(n, k));
        return SMQ_ERR_WORKSPACE;
      }
      int64_t* idx = reinterpret_cast<int64_t*>(
          ws + (k > SMQ_MAX_DEVICE_SAMPLES ? SMQ_WS_LARGE_SAMPLES_OFFSET : SMQ_WS_SAMPLES_OFFSET));
      floyd_draw(p->seed, p->offset + base, n, k, idx);
      sampled_stats<T>(x, idx, k, p, range_coef_host(p, k), &st);
      break;
    }
    default: {  // SMQ_STATS_INJECTED: mean / std from stats_in, the rest derived
      if (!stats_in) {
        set_error("cpu smaq: SMQ_STATS_INJECTED needs stats_in");
        return SMQ_ERR_INVALID;
      }
      st = *stats_in;
      st.inv_std_clamped = 1.0 / (double)st.std_clamped;
      st.inv_std_clamped_f32 = (float)st.inv_std_clamped;
      st.quot_check = quot_check_for(st.std_clamped);
    }
  }
  return SMQ_OK;
}

template <int T>
static int smaq_roundtrip(const void* x, float* y, int64_t n, const SmqSmaqParams* p,
                          const float* uniforms, const SmqSmaqStats* stats_in, char* ws,
                          size_t ws_bytes, int n_threads) {
  SmqSmaqStats st;
  uint64_t base = 0;
  const int rc = host_stats<T>(x, n, p, stats_in, ws, ws_bytes, n_threads, &st, &base);
  if (rc) return rc;
  if (p->offset_counter) *p->offset_counter = base + (uint64_t)n;
  st.rng_offset = base;
  SmaqCtx c;
  c.x = x;
  c.y = y;
  c.uniforms = uniforms;
  c.bn_gamma = p->bn_gamma;
  c.bn_beta = p->bn_beta;
  c.bn_channels = p->bn_channels;
  c.bn_inner = p->bn_inner;
  c.mean = st.mean;
  c.sd = st.std_dev;
  c.sc = st.std_clamped;
  c.thr = p->main_std_dev_threshold;
  c.nthr = -c.thr;
  const bool bn = p->bn_gamma != nullptr;
  c.cthr = bn ? c.thr : rin<T>(c.thr);
  c.cnthr = -c.cthr;
  c.zh = 0.0f * c.nthr;
  c.zl = 0.0f * c.thr;
  c.r_main = p->range_main;
  c.r_out = p->range_outlier;
  c.key = rng_key(p->seed);
  c.off = p->offset + base;
  const int rm = !p->stochastic_rounding ? kRoundTrunc : (uniforms ? kRoundUniform : kRoundHash);
  const uint64_t n_out = smaq_pass<T>(c, n, rm, bn, p->all_positive != 0, n_threads);
  if (p->count_outliers) st.n_outlier = n_out;
  memcpy(ws, &st, sizeof(st));
  uint64_t* slots = reinterpret_cast<uint64_t*>(ws + SMQ_WS_OUTLIER_SLOTS_OFFSET);
  for (int i = 0; i < SMQ_WS_OUTLIER_SLOTS; ++i) slots[i] = 0;
  if (p->count_outliers) slots[0] = n_out;
  return SMQ_OK;
}

// ---- packed container (include/smq.h "Packed SmaQ container", format version 2) -----------------
// The host twin of smq_smaq_compress / smq_smaq_decompress (smaq_pack.hip): the same codes (the
// quantisation of smaq_task, i.e. the device's smaq_quant), the same block layout, the same bytes
// for the same statistics and random stream (oracle/smaq_packed.py restates the format; the GPU
// tests compare the two libraries' streams). Tasks of kPackTaskBlocks blocks: every block's fixed
// section is written in place, its variable section into a per-block buffer that is copied to its
// prefix-sum place once all sizes are known.
constexpr int kPB = SMQ_PACK_BLOCK;
constexpr int kPackTaskBlocks = 16;

static inline size_t pk_fixed_words(int wm) { return 128 + (size_t)wm * (kPB / 32); }
static inline int64_t pk_dir_entries(int64_t nb) { return nb + (nb & 1); }

// LSB-first bit writer over uint32 words (zeroed by the caller)
static inline void put_bits(uint32_t* w, uint64_t bitpos, uint32_t v, int width) {
  const uint64_t word = bitpos >> 5;
  const int sh = (int)(bitpos & 31);
  w[word] |= v << sh;
  if (sh + width > 32) w[word + 1] |= v >> (32 - sh);
}

static inline uint32_t get_bits(const uint32_t* w, uint64_t bitpos, int width) {
  const uint64_t word = bitpos >> 5;
  const int sh = (int)(bitpos & 31);
  uint64_t v = w[word] >> sh;
  if (sh + width > 32) v |= (uint64_t)w[word + 1] << (32 - sh);
  return (uint32_t)(v & ((1ull << width) - 1ull));
}

struct PackHostCtx {
  SmaqCtx c;
  int wm, wo, we, rm;
  int64_t n;
};

// smart.py:144-169 for element i: q and the two sides (smaq_task's quantisation)
template <int T, int RM, bool BN>
static inline float quant_host(const SmaqCtx& c, int64_t i, bool& hi, bool& lo) {
  constexpr int TZ = BN ? kF32 : T;
  float v = ld<T>(c.x, i);
  if (BN) {
    const int64_t ch = (i / c.bn_inner) % c.bn_channels;
    v = (v - c.bn_beta[ch]) / c.bn_gamma[ch];
  }
  const float dm = rin<TZ>(v - c.mean);
  const float z = rin<TZ>(dm / c.sc);
  hi = z > c.cthr;
  lo = z < c.cnthr;
  const bool o = hi || lo;
  const float a = (hi ? c.nthr : c.zh) + (lo ? c.thr : c.zl);
  const float r = o ? c.r_out : c.r_main;
  const float d = (z + a) * r;
  if (RM == kRoundTrunc) return truncf(d);
  const float f = floorf(d);
  const float fr = d - f;
  float t;
  if (RM == kRoundHash)
    t = fmaf(hash_u24(c.key, c.off + (uint64_t)i), -0x1p-24f, fr) + 0.5f;
  else
    t = (fr - c.uniforms[i]) + 0.5f;
  t = (t < 0.0f) ? 0.0f : t;
  return f + rintf(t);
}

// One block: its fixed section written at fx (fk words, zeroed here), its variable section
// appended to var; *n_out / *n_esc as the directory records them.
template <int T, int RM, bool BN>
static void pack_block_host(const PackHostCtx& P, int64_t b, uint32_t* fx,
                            std::vector<uint32_t>& var, uint32_t* n_out, uint32_t* n_esc) {
  const int wm = P.wm, wo = P.wo, we = P.we;
  const int64_t e0 = b * kPB, m = std::min<int64_t>(kPB, P.n - e0);
  memset(fx, 0, 4 * pk_fixed_words(wm));
  uint32_t* plane = fx + 128;
  const float main_lo = -ldexpf(1.0f, wm - 1), main_hi = ldexpf(1.0f, wm - 1) - 1.0f;
  const float mag_max = ldexpf(1.0f, wo - 1) - 1.0f;
  const uint32_t wmask = (uint32_t)((1ull << wm) - 1ull);
  std::vector<uint32_t> ext;  // outlier code bits above the plane, element order
  std::vector<uint32_t> esc;  // {index, q bits}
  for (int64_t e = 0; e < m; ++e) {
    bool hi, lo;
    const float q = quant_host<T, RM, BN>(P.c, e0 + e, hi, lo);
    const bool o = hi != lo;
    const bool h1 = hi && o, l1 = lo && o;
    bool ok;
    if (o) ok = h1 ? (q >= 0.0f && q <= mag_max) : (q <= 0.0f && -q <= mag_max);
    else ok = q >= main_lo && q <= main_hi;
    const int64_t qi = ok ? (int64_t)q : 0;
    uint32_t code;
    if (o) {
      const uint32_t side = (uint32_t)l1 << (wo - 1);
      code = ok ? (side | (uint32_t)(h1 ? qi : -qi)) : side;
      fx[e >> 5] |= 1u << (e & 31);
      if (we > 0) ext.push_back(code >> wm);
    } else {
      code = ok ? ((uint32_t)qi & wmask) : 0u;
    }
    put_bits(plane, (uint64_t)e * (uint64_t)wm, code & wmask, wm);
    if (!ok) {
      esc.push_back((uint32_t)e);
      esc.push_back(q != q ? 0x7fc00000u : f2u(q));
    }
  }
  *n_out = (uint32_t)ext.size();
  if (we == 0) {  // (no outlier bits above the plane: count the mask)
    uint32_t c = 0;
    for (int w = 0; w < 128; ++w) c += (uint32_t)__builtin_popcount(fx[w]);
    *n_out = c;
  }
  *n_esc = (uint32_t)(esc.size() / 2);
  const size_t ext_words = ((size_t)we * ext.size() + 31) / 32;
  const size_t at = var.size();
  var.resize(at + ext_words, 0u);
  for (size_t k = 0; k < ext.size(); ++k) put_bits(var.data() + at, (uint64_t)k * we, ext[k], we);
  var.insert(var.end(), esc.begin(), esc.end());
}

template <int T>
static int pack_host(const void* x, int64_t n, const SmqSmaqParams* p, uint8_t* out,
                     size_t out_bytes, char* ws, size_t ws_bytes, int n_threads) {
  SmqSmaqStats st;
  uint64_t base = 0;
  int rc = host_stats<T>(x, n, p, nullptr, ws, ws_bytes, n_threads, &st, &base);
  if (rc) return rc;
  if (p->offset_counter) *p->offset_counter = base + (uint64_t)n;
  st.rng_offset = base;
  memcpy(ws, &st, sizeof(st));  // the header the device packer leaves in its workspace
  PackHostCtx P;
  SmaqCtx& c = P.c;
  memset(&c, 0, sizeof(c));
  c.x = x;
  c.bn_gamma = p->bn_gamma;
  c.bn_beta = p->bn_beta;
  c.bn_channels = p->bn_channels;
  c.bn_inner = p->bn_inner;
  c.mean = st.mean;
  c.sd = st.std_dev;
  c.sc = st.std_clamped;
  c.thr = p->main_std_dev_threshold;
  c.nthr = -c.thr;
  const bool bn = p->bn_gamma != nullptr;
  c.cthr = bn ? c.thr : rin<T>(c.thr);
  c.cnthr = -c.cthr;
  c.zh = 0.0f * c.nthr;
  c.zl = 0.0f * c.thr;
  c.r_main = p->range_main;
  c.r_out = p->range_outlier;
  c.key = rng_key(p->seed);
  c.off = p->offset + base;
  P.wm = p->num_bits_main - 1;
  P.wo = p->num_bits_outlier - 1;
  P.we = P.wo > P.wm ? P.wo - P.wm : 0;
  P.n = n;
  const int rm = p->stochastic_rounding ? kRoundHash : kRoundTrunc;
  const int64_t nb = (n + kPB - 1) / kPB;
  const size_t fk = pk_fixed_words(P.wm);
  SmqPackedHeader* hdr = reinterpret_cast<SmqPackedHeader*>(out);
  uint64_t* dir = reinterpret_cast<uint64_t*>(out + sizeof(SmqPackedHeader));
  uint32_t* fixed = reinterpret_cast<uint32_t*>(dir + pk_dir_entries(nb));
  std::vector<std::vector<uint32_t>> var((size_t)nb);
  std::vector<uint32_t> nout((size_t)nb), nesc((size_t)nb);
  const int64_t tasks = (nb + kPackTaskBlocks - 1) / kPackTaskBlocks;
  const std::function<void(int64_t)> fn = [&](int64_t t) {
    const int64_t b1 = std::min(nb, (t + 1) * kPackTaskBlocks);
    for (int64_t b = t * kPackTaskBlocks; b < b1; ++b) {
      uint32_t* fx = fixed + (size_t)b * fk;
      auto& v = var[(size_t)b];
      if (rm == kRoundHash) {
        if (bn) pack_block_host<T, kRoundHash, true>(P, b, fx, v, &nout[b], &nesc[b]);
        else pack_block_host<T, kRoundHash, false>(P, b, fx, v, &nout[b], &nesc[b]);
      } else {
        if (bn) pack_block_host<T, kRoundTrunc, true>(P, b, fx, v, &nout[b], &nesc[b]);
        else pack_block_host<T, kRoundTrunc, false>(P, b, fx, v, &nout[b], &nesc[b]);
      }
    }
  };
  pool().run(tasks, threads_for(n_threads), fn);
  uint64_t off = 0;
  for (int64_t b = 0; b < nb; ++b) {
    dir[b] = off | ((uint64_t)nout[b] << 38) | ((uint64_t)nesc[b] << 51);
    off += var[(size_t)b].size();
  }
  if (nb & 1) dir[nb] = 0;
  uint32_t* vr = fixed + (size_t)nb * fk;
  const size_t bn_words = bn ? 2 * (size_t)p->bn_channels : 0;
  const size_t total = sizeof(SmqPackedHeader) + 8 * (size_t)pk_dir_entries(nb) +
                       4 * ((size_t)nb * fk + off + bn_words);
  if (total > out_bytes) {  // (cannot happen below smq_smaq_pack_bound; checked all the same)
    set_error("cpu compress: stream of %zu bytes exceeds the buffer (%zu)", total, out_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  uint64_t at = 0;
  for (int64_t b = 0; b < nb; ++b) {
    const auto& v = var[(size_t)b];
    if (!v.empty()) memcpy(vr + at, v.data(), 4 * v.size());
    at += v.size();
  }
  if (bn) {
    float* tab = reinterpret_cast<float*>(vr + off);
    memcpy(tab, p->bn_gamma, 4 * (size_t)p->bn_channels);
    memcpy(tab + p->bn_channels, p->bn_beta, 4 * (size_t)p->bn_channels);
  }
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  SmqPackedHeader h;
  memset(&h, 0, sizeof(h));
  h.magic = SMQ_PACK_MAGIC;
  h.version = SMQ_PACK_VERSION;
  h.n = n;
  h.block_elems = kPB;
  h.n_blocks = (uint32_t)nb;
  h.num_bits_main = p->num_bits_main;
  h.num_bits_outlier = p->num_bits_outlier;
  h.flags = (p->all_positive ? SMQ_PACK_FLAG_ALL_POSITIVE : 0u) | (R.safe_q ? SMQ_PACK_FLAG_SAFE_Q : 0u) |
            (c.thr < 0.0f ? SMQ_PACK_FLAG_BOTH_SIDES : 0u) | (bn ? SMQ_PACK_FLAG_BN : 0u);
  h.thr = c.thr;
  h.range_main = p->range_main;
  h.range_outlier = p->range_outlier;
  h.mean = st.mean;
  h.std_dev = st.std_dev;
  h.inv_range_main = R.inv_main;
  h.inv_range_outlier = R.inv_out;
  h.data_words = off;
  h.total_bytes = total;
  h.bn_channels = bn ? (uint32_t)p->bn_channels : 0u;
  h.bn_inner = bn ? p->bn_inner : 0;
  memcpy(hdr, &h, sizeof(h));
  return SMQ_OK;
}

// The decoder (smq_smaq_decompress on the host): every block's codes, outlier bits and escapes
// back to q and the sides, then smart.py:171-182 (and the BN term, all_positive) as smaq_dequant.
static int unpack_host(const uint8_t* in, float* y, int64_t n, int n_threads) {
  SmqPackedHeader h;
  memcpy(&h, in, sizeof(h));
  if (h.magic != SMQ_PACK_MAGIC || h.version != SMQ_PACK_VERSION || h.n != n ||
      h.block_elems != (uint32_t)kPB || h.n_blocks != (uint32_t)((n + kPB - 1) / kPB) ||
      h.num_bits_main < 2 || h.num_bits_main > 25 || h.num_bits_outlier < 3 ||
      h.num_bits_outlier > 25) {
    set_error("cpu decompress: not a version-%u stream of %lld elements", SMQ_PACK_VERSION,
              (long long)n);
    return SMQ_ERR_INVALID;
  }
  const int wm = h.num_bits_main - 1, wo = h.num_bits_outlier - 1, we = wo > wm ? wo - wm : 0;
  const int64_t nb = h.n_blocks;
  const size_t fk = pk_fixed_words(wm);
  const uint64_t* dir = reinterpret_cast<const uint64_t*>(in + sizeof(SmqPackedHeader));
  const uint32_t* fixed = reinterpret_cast<const uint32_t*>(dir + pk_dir_entries(nb));
  const uint32_t* vr = fixed + (size_t)nb * fk;
  const bool bn = (h.flags & SMQ_PACK_FLAG_BN) != 0, ap = (h.flags & 1u) != 0;
  const bool both = (h.flags & SMQ_PACK_FLAG_BOTH_SIDES) != 0;
  const float* g = bn ? reinterpret_cast<const float*>(vr + h.data_words) : nullptr;
  const float* bb = bn ? g + h.bn_channels : nullptr;
  const float thr = h.thr, nthr = -thr, zh = 0.0f * nthr, zl = 0.0f * thr;
  const int64_t tasks = (nb + kPackTaskBlocks - 1) / kPackTaskBlocks;
  const std::function<void(int64_t)> fn = [&](int64_t t) {
    std::vector<float> qb(kPB);
    std::vector<uint8_t> sides(kPB);  // bit 0: hi, bit 1: lo
    const uint8_t both2 = both ? 3 : 0;
    const int64_t b1 = std::min(nb, (t + 1) * kPackTaskBlocks);
    for (int64_t b = t * kPackTaskBlocks; b < b1; ++b) {
      const int64_t e0 = b * kPB, m = std::min<int64_t>(kPB, n - e0);
      const uint64_t d = dir[b];
      const uint64_t vbase = d & ((1ull << 38) - 1ull);
      const uint32_t n_out = (uint32_t)((d >> 38) & 0x1fffu), n_esc = (uint32_t)(d >> 51);
      const uint32_t* fx = fixed + (size_t)b * fk;
      const uint32_t* ext = vr + vbase;
      const uint32_t* esc = ext + ((size_t)we * n_out + 31) / 32;
      uint32_t rank = 0;
      for (int64_t e = 0; e < m; ++e) {
        uint32_t code = get_bits(fx + 128, (uint64_t)e * wm, wm);
        if ((fx[e >> 5] >> (e & 31)) & 1u) {  // outlier: side bit on top of |q|
          if (we > 0) code |= get_bits(ext, (uint64_t)rank * we, we) << wm;
          ++rank;
          const uint32_t side = (code >> (wo - 1)) & 1u;
          const float mag = (float)(code & ((1u << (wo - 1)) - 1u));
          qb[(size_t)e] = side ? -mag : mag;
          sides[(size_t)e] = side ? 2 : 1;
        } else {  // main: wm-bit two's complement
          qb[(size_t)e] = (float)((code >= (1u << (wm - 1))) ? (int32_t)code - (1 << wm)
                                                             : (int32_t)code);
          sides[(size_t)e] = both2;
        }
      }
      for (uint32_t k = 0; k < n_esc; ++k)
        if (esc[2 * k] < (uint32_t)m) qb[esc[2 * k]] = u2f(esc[2 * k + 1]);
      for (int64_t e = 0; e < m; ++e) {
        const bool hi = sides[(size_t)e] & 1, lo = sides[(size_t)e] & 2;
        const float a = (hi ? nthr : zh) + (lo ? thr : zl);
        const float r = (hi || lo) ? h.range_outlier : h.range_main;
        float out = qb[(size_t)e] / r - a;
        out = out * h.std_dev;
        out = out + h.mean;
        if (bn) {
          const int64_t ch = ((e0 + e) / h.bn_inner) % (int64_t)h.bn_channels;
          out = out * g[ch];
          out = out + bb[ch];
        }
        if (ap) out = (out < 0.0f) ? 0.0f : out;
        y[e0 + e] = out;
      }
    }
  };
  pool().run(tasks, threads_for(n_threads), fn);
  return SMQ_OK;
}

// ---- float_quantize -----------------------------------------------------------------------------
template <int TIN, bool HOUT>
static void float_quant_pass(const void* x, void* y, int64_t n, int eb, int mb, bool sr,
                             int check_inf, const uint32_t* rand_bits, uint32_t key,
                             uint64_t offset, float max_value, int n_threads) {
  parallel_tasks(n, n_threads, [&](int64_t, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint32_t r = !sr ? 0u : (rand_bits ? rand_bits[i] : rng_u32(key, offset + (uint64_t)i));
      float q = qtorch_quant(ld<TIN>(x, i), r, eb, mb, sr);
      if (check_inf && fabsf(q - max_value) <= FLT_EPSILON) q = INFINITY;
      if (HOUT) static_cast<uint16_t*>(y)[i] = f2h(q);
      else static_cast<float*>(y)[i] = q;
    }
  });
}

// ---- S2FP8 ----------------------------------------------------------------------------------------
static inline float nan_max_h(float a, float b) { return (b > a || b != b) ? b : a; }

template <int TIN>
static void s2_derive(float mu, float m, uint32_t n_used, SmqS2fp8Stats* o) {
  const float alpha = rin<TIN>(rin<TIN>(1.0f / rin<TIN>(m - mu)) * 15.0f);
  const float beta = rin<TIN>((-alpha) * mu);
  const float bp2 = rin<TIN>((float)exp2((double)beta));
  o->mu = mu;
  o->m = m;
  o->alpha = alpha;
  o->beta = beta;
  o->beta_pow2 = bp2;
  o->inv_beta_pow2 = rin<TIN>(1.0f / bp2);
  o->inv_alpha = rin<TIN>(1.0f / alpha);
  o->n_used = n_used;
}

template <int TIN>
static inline float s2_log_h(float v) {
  const float a = fabsf(v);
  return a == 0.0f ? a : rin<TIN>(log2f(a));
}

template <int TIN>
static void s2_stats(const void* x, int64_t n, int n_threads, SmqS2fp8Stats* o) {
  struct P {
    double s;
    float m;
  };
  std::vector<P> part((size_t)((n + kTask - 1) / kTask));
  parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float mx = -INFINITY;
    for (int64_t i = i0; i < i1; ++i) {
      const float l = s2_log_h<TIN>(ld<TIN>(x, i));
      a[(i - i0) & 7] += (double)l;
      mx = nan_max_h(mx, l);
    }
    part[(size_t)t] = P{((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])), mx};
  });
  double s = 0.0;
  float m = -INFINITY;
  for (const P& q : part) {
    s += q.s;
    m = nan_max_h(m, q.m);
  }
  const float mu = rin<TIN>((float)(s / (double)n));
  s2_derive<TIN>(mu, m, (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n), o);
}

// s2fp8.py:45-48 (precision 32; out_mode 1 / 2: Y / T as the device's OUT_Y / OUT_T)
static inline float s2_elem32(float xv, uint32_t r, const SmqS2fp8Stats& s, int check_inf,
                              float max_value, int out_mode) {
  const float sgn = (xv > 0.0f) ? 1.0f : ((xv < 0.0f) ? -1.0f : 0.0f);
  float Y = powf(fabsf(xv), s.alpha);
  Y = Y * s.beta_pow2;
  if (out_mode == 1) return Y;
  float T = qtorch_quant(Y, r, 5, 2, true);
  if (check_inf && fabsf(T - max_value) <= FLT_EPSILON) T = INFINITY;
  if (out_mode == 2) return T;
  return powf(T * s.inv_beta_pow2, s.inv_alpha) * sgn;
}

// precision 16 (quantization.py:187-204 half branch): forward in TIN, inverse in half
template <int TIN>
static inline float s2_elem16(float xv, uint32_t r, const SmqS2fp8Stats& s, int check_inf,
                              float max_value) {
  // powers rounded to a half type: the correctly rounded float power (double pow, then float),
  // which the reference's torch half pow reproduces (tests/golden f64_s2fp8_p16_powcase); fp32 data
  // keeps powf (its Y is not rounded further)
  float Y = TIN == kF32 ? powf(fabsf(xv), s.alpha) : (float)pow((double)fabsf(xv), (double)s.alpha);
  Y = rin<TIN>(rin<TIN>(Y) * s.beta_pow2);
  float T = qtorch_quant(Y, r, 5, 2, true);
  if (check_inf && fabsf(T - max_value) <= FLT_EPSILON) T = INFINITY;
  const float t1 = rin<kF16>(T * s.inv_beta_pow2);
  const float t2 = rin<kF16>((float)pow((double)t1, (double)rin<kF16>(s.inv_alpha)));
  if (xv > 0.0f) return t2;
  if (xv < 0.0f) return u2f(f2u(t2) ^ 0x80000000u);
  return t2 * 0.0f;
}

template <int TIN>
static void s2_pass(const void* x, void* y, int64_t n, bool p16, bool hout, int check_inf,
                    const uint32_t* rand_bits, uint32_t key, uint64_t off, const SmqS2fp8Stats& s,
                    int out_mode, int n_threads) {
  const float max_value = qtorch_quant(FLT_MAX, 0u, 5, 2, false);
  parallel_tasks(n, n_threads, [&](int64_t, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint32_t r = rand_bits ? rand_bits[i] : rng_u32(key, off + (uint64_t)i);
      const float xv = ld<TIN>(x, i);
      const float v = p16 ? s2_elem16<TIN>(xv, r, s, check_inf, max_value)
                          : s2_elem32(xv, r, s, check_inf, max_value, out_mode);
      if (hout) static_cast<uint16_t*>(y)[i] = f2h(v);
      else static_cast<float*>(y)[i] = v;
    }
  });
}


// ---- fp64 tensors (smaq_f64.h holds the shared finaliser and element transforms) -----------------
// The statistics of an fp64 call (full / sampled / injected) and the stream position it takes
// (*base; params.offset_counter advanced by n).
static int stats_f64(const double* x, int64_t n, const SmqSmaqParams* p,
                     const SmqSmaqStatsF64* stats_in, char* ws, size_t ws_bytes, int n_threads,
                     SmqSmaqStatsF64* out, uint64_t* base_out) {
  SmqSmaqStatsF64 st;
  memset(&st, 0, sizeof(st));
  const uint64_t base = p->offset_counter ? *p->offset_counter : 0ull;
  auto coef = [&](int64_t cnt) {
    return p->range_std_coef_f64 >= 0.0 ? p->range_std_coef_f64 : 1.0 / sqrt(2.0 * log((double)cnt));
  };
  const bool range = p->use_range_std_dev != 0;
  switch (p->stats_source) {
    case SMQ_STATS_WORKSPACE: {
      const double shift = median3_f64(x[0], x[n >> 1], x[n - 1]);
      struct M { double s1, s2, mn, mx; };
      std::vector<M> part((size_t)((n + kTask - 1) / kTask));
      parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
        double a1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        double mn = INFINITY, mx = -INFINITY;
        for (int64_t i = i0; i < i1; ++i) {
          const double d = x[i] - shift;
          a1[(i - i0) & 7] += d;
          a2[(i - i0) & 7] = fma(d, d, a2[(i - i0) & 7]);
          mn = fmin(mn, x[i]);
          mx = fmax(mx, x[i]);
        }
        part[(size_t)t] = M{((a1[0] + a1[1]) + (a1[2] + a1[3])) + ((a1[4] + a1[5]) + (a1[6] + a1[7])),
                            ((a2[0] + a2[1]) + (a2[2] + a2[3])) + ((a2[4] + a2[5]) + (a2[6] + a2[7])),
                            mn, mx};
      });
      M tot{0.0, 0.0, INFINITY, -INFINITY};
      for (const M& m : part) {
        tot.s1 += m.s1;
        tot.s2 += m.s2;
        tot.mn = fmin(tot.mn, m.mn);
        tot.mx = fmax(tot.mx, m.mx);
      }
      finalize_f64(tot.s1, tot.s2, tot.mn, tot.mx, n, shift, false, range, p->clamp_lo_f64,
                   p->clamp_hi_f64, coef(n), &st);
      break;
    }
    case SMQ_STATS_SAMPLED:
    case SMQ_STATS_SAMPLED_DEVICE: {
      const bool draw = p->stats_source == SMQ_STATS_SAMPLED_DEVICE;
      const int64_t k = std::min<int64_t>(p->num_samples, n);
      const int64_t cap = draw ? SMQ_MAX_DRAW_SAMPLES : SMQ_MAX_SAMPLES;
      if (k < 1 || k > cap) {
        set_error("cpu smaq f64: num_samples must be in [1, %lld]", (long long)cap);
        return SMQ_ERR_INVALID;
      }
      const int64_t* idx = p->sample_idx;
      if (draw) {
        if (ws_bytes < smq_smaq_workspace_bytes_sampled(n, k)) {
          set_error("cpu smaq f64: workspace too small for %lld samples", (long long)k);
          return SMQ_ERR_WORKSPACE;
        }
        int64_t* out = reinterpret_cast<int64_t*>(
            ws + (k > SMQ_MAX_DEVICE_SAMPLES ? SMQ_WS_LARGE_SAMPLES_OFFSET : SMQ_WS_SAMPLES_OFFSET));
        floyd_draw(p->seed, p->offset + base, n, k, out);
        idx = out;
      } else {
        for (int64_t i = 0; i < k; ++i)
          if (idx[i] < 0 || idx[i] >= n) {
            set_error("cpu smaq f64: sample index %lld out of range", (long long)idx[i]);
            return SMQ_ERR_INVALID;
          }
      }
      double sum = 0.0, mn = INFINITY, mx = -INFINITY;
      for (int64_t i = 0; i < k; ++i) {
        const double v = x[idx[i]];
        sum += v;
        mn = fmin(mn, v);
        mx = fmax(mx, v);
      }
      const double mean = sum / (double)k;
      double m2 = 0.0;
      for (int64_t i = 0; i < k; ++i) {
        const double d = x[idx[i]] - mean;
        m2 = fma(d, d, m2);
      }
      finalize_f64(0.0, m2, mn, mx, k, mean, true, range, p->clamp_lo_f64, p->clamp_hi_f64, coef(k),
                   &st);
      break;
    }
    default: {
      if (!stats_in) {
        set_error("cpu smaq f64: SMQ_STATS_INJECTED needs stats_in");
        return SMQ_ERR_INVALID;
      }
      st = *stats_in;
      const double sd = st.raw_std;
      const double std_dev = (sd == 0.0) ? 1.0 : sd;
      double sc = std_dev < p->clamp_lo_f64 ? p->clamp_lo_f64 : std_dev;
      sc = sc > p->clamp_hi_f64 ? p->clamp_hi_f64 : sc;
      st.std_dev = std_dev;
      st.std_clamped = sc;
    }
  }
  if (p->offset_counter) *p->offset_counter = base + (uint64_t)n;
  st.rng_offset = base;
  *out = st;
  *base_out = base;
  return SMQ_OK;
}

static int smaq_roundtrip_f64(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                              const double* uniforms, const SmqSmaqStatsF64* stats_in, char* ws,
                              size_t ws_bytes, int n_threads) {
  SmqSmaqStatsF64 st;
  uint64_t base = 0;
  const int rc = stats_f64(x, n, p, stats_in, ws, ws_bytes, n_threads, &st, &base);
  if (rc) return rc;
  const ElemF64 c = elem_f64_consts(st, *p);
  const uint32_t key = rng_key(p->seed);
  const uint64_t off = p->offset + base;
  const double* gam = reinterpret_cast<const double*>(p->bn_gamma);
  const double* bet = reinterpret_cast<const double*>(p->bn_beta);
  const int rm = !p->stochastic_rounding ? kRoundTrunc : (uniforms ? kRoundUniform : kRoundHash);
  const bool bn = p->bn_gamma != nullptr, ap = p->all_positive != 0;
  std::vector<uint64_t> part((size_t)((n + kTask - 1) / kTask));
  auto go = [&](auto rm_c, auto bn_c, auto ap_c) {
    constexpr int RM = decltype(rm_c)::value;
    constexpr bool BN = decltype(bn_c)::value, AP = decltype(ap_c)::value;
    parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
      uint64_t cnt = 0;
      for (int64_t i = i0; i < i1; ++i) {
        double u = 0.0, g = 1.0, b = 0.0;
        if (RM == kRoundHash) u = (double)smaq_u24(key, off + (uint64_t)i);
        if (RM == kRoundUniform) u = uniforms[i];
        if (BN) {
          const int64_t ch = (i / p->bn_inner) % p->bn_channels;
          g = gam[ch];
          b = bet[ch];
        }
        bool o;
        y[i] = smaq_elem_f64<RM, BN, AP>(x[i], u, c, o, g, b);
        cnt += o ? 1u : 0u;
      }
      part[(size_t)t] = cnt;
    });
  };
  using H = std::integral_constant<int, kRoundHash>;
  using U = std::integral_constant<int, kRoundUniform>;
  using R = std::integral_constant<int, kRoundTrunc>;
  using Y = std::true_type;
  using N = std::false_type;
  if (rm == kRoundHash) {
    if (bn) { if (ap) go(H(), Y(), Y()); else go(H(), Y(), N()); }
    else { if (ap) go(H(), N(), Y()); else go(H(), N(), N()); }
  } else if (rm == kRoundUniform) {
    if (bn) { if (ap) go(U(), Y(), Y()); else go(U(), Y(), N()); }
    else { if (ap) go(U(), N(), Y()); else go(U(), N(), N()); }
  } else {
    if (bn) { if (ap) go(R(), Y(), Y()); else go(R(), Y(), N()); }
    else { if (ap) go(R(), N(), Y()); else go(R(), N(), N()); }
  }
  uint64_t n_out = 0;
  for (uint64_t v : part) n_out += v;
  memcpy(ws, &st, sizeof(st));
  uint64_t* slots = reinterpret_cast<uint64_t*>(ws + SMQ_WS_OUTLIER_SLOTS_OFFSET);
  for (int i = 0; i < SMQ_WS_OUTLIER_SLOTS; ++i) slots[i] = 0;
  if (p->count_outliers) slots[0] = n_out;
  return SMQ_OK;
}

static void s2_stats_f64(const double* x, int64_t n, int n_threads, SmqS2fp8StatsF64* o) {
  struct P {
    double s, m;
  };
  std::vector<P> part((size_t)((n + kTask - 1) / kTask));
  parallel_tasks(n, n_threads, [&](int64_t t, int64_t i0, int64_t i1) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double mx = -INFINITY;
    for (int64_t i = i0; i < i1; ++i) {
      const double l = s2_log_f64(x[i]);
      a[(i - i0) & 7] += l;
      mx = nan_max_f64(mx, l);
    }
    part[(size_t)t] = P{((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])), mx};
  });
  double s = 0.0, m = -INFINITY;
  for (const P& q : part) {
    s += q.s;
    m = nan_max_f64(m, q.m);
  }
  s2_derive_f64(s, m, n, o);
}
// ---- float64 streams (flag SMQ_PACK_FLAG_F64; smaq_pack_f64.hip is the device twin) -------------
// The fp64 chain's codes (smaq_quant_f64) in the version-2 sections, escapes {element, q low word,
// q high word}, the statistics as doubles in the header, an fp64 BN table.
static inline uint32_t code_f64(double q, bool o, bool los, int wm, int wo, bool& esc) {
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

struct PackF64Ctx {
  const double* x;
  const double* gam;
  const double* bet;
  int64_t channels, inner, n;
  ElemF64 c;
  uint32_t key;
  uint64_t off;
  int wm, wo, we;
};

template <int RM, bool BN>
static void pack_block_host_f64(const PackF64Ctx& P, int64_t b, uint32_t* fx,
                                std::vector<uint32_t>& var, uint32_t* n_out, uint32_t* n_esc) {
  const int wm = P.wm, wo = P.wo, we = P.we;
  const int64_t e0 = b * kPB, m = std::min<int64_t>(kPB, P.n - e0);
  memset(fx, 0, 4 * pk_fixed_words(wm));
  uint32_t* plane = fx + 128;
  const uint32_t wmask = (uint32_t)((1ull << wm) - 1ull);
  std::vector<uint32_t> ext, esc;
  uint32_t no = 0;
  for (int64_t e = 0; e < m; ++e) {
    const int64_t i = e0 + e;
    const double u = RM == kRoundHash ? (double)smaq_u24(P.key, P.off + (uint64_t)i) : 0.0;
    double g = 1.0, bb = 0.0;
    if (BN) {
      const int64_t ch = (i / P.inner) % P.channels;
      g = P.gam[ch];
      bb = P.bet[ch];
    }
    bool hi, lo, es;
    const double q = smaq_quant_f64<RM, BN>(P.x[i], u, P.c, hi, lo, g, bb);
    const bool o = hi != lo, los = lo && !hi;
    const uint32_t code = code_f64(q, o, los, wm, wo, es);
    if (o) {
      fx[e >> 5] |= 1u << (e & 31);
      ++no;
      if (we > 0) ext.push_back(code >> wm);
    }
    put_bits(plane, (uint64_t)e * (uint64_t)wm, code & wmask, wm);
    if (es) {
      const uint64_t qb = q != q ? 0x7ff8000000000000ull : __builtin_bit_cast(uint64_t, q);
      esc.push_back((uint32_t)e);
      esc.push_back((uint32_t)qb);
      esc.push_back((uint32_t)(qb >> 32));
    }
  }
  *n_out = no;
  *n_esc = (uint32_t)(esc.size() / 3);
  const size_t ext_w = ((size_t)we * ext.size() + 31) / 32;
  const size_t at = var.size();
  var.resize(at + ext_w, 0u);
  for (size_t k = 0; k < ext.size(); ++k) put_bits(var.data() + at, (uint64_t)k * we, ext[k], we);
  var.insert(var.end(), esc.begin(), esc.end());
}

static int pack_host_f64(const double* x, int64_t n, const SmqSmaqParams* p, uint8_t* out,
                         size_t out_bytes, char* ws, size_t ws_bytes, int n_threads) {
  SmqSmaqStatsF64 st;
  uint64_t base = 0;
  const int rc = stats_f64(x, n, p, nullptr, ws, ws_bytes, n_threads, &st, &base);
  if (rc) return rc;
  memcpy(ws, &st, sizeof(st));  // the header the device packer leaves in its workspace
  PackF64Ctx P;
  P.x = x;
  P.gam = reinterpret_cast<const double*>(p->bn_gamma);
  P.bet = reinterpret_cast<const double*>(p->bn_beta);
  P.channels = p->bn_channels;
  P.inner = p->bn_inner;
  P.n = n;
  P.c = elem_f64_consts(st, *p);
  P.key = rng_key(p->seed);
  P.off = p->offset + base;
  P.wm = p->num_bits_main - 1;
  P.wo = p->num_bits_outlier - 1;
  P.we = P.wo > P.wm ? P.wo - P.wm : 0;
  const bool bn = p->bn_gamma != nullptr, sr = p->stochastic_rounding != 0;
  const int64_t nb = (n + kPB - 1) / kPB;
  const size_t fk = pk_fixed_words(P.wm);
  uint64_t* dir = reinterpret_cast<uint64_t*>(out + sizeof(SmqPackedHeader));
  uint32_t* fixed = reinterpret_cast<uint32_t*>(dir + pk_dir_entries(nb));
  std::vector<std::vector<uint32_t>> var((size_t)nb);
  std::vector<uint32_t> nout((size_t)nb), nesc((size_t)nb);
  const int64_t tasks = (nb + kPackTaskBlocks - 1) / kPackTaskBlocks;
  const std::function<void(int64_t)> fn = [&](int64_t t) {
    const int64_t b1 = std::min(nb, (t + 1) * kPackTaskBlocks);
    for (int64_t b = t * kPackTaskBlocks; b < b1; ++b) {
      uint32_t* fx = fixed + (size_t)b * fk;
      auto& v = var[(size_t)b];
      if (sr) {
        if (bn) pack_block_host_f64<kRoundHash, true>(P, b, fx, v, &nout[b], &nesc[b]);
        else pack_block_host_f64<kRoundHash, false>(P, b, fx, v, &nout[b], &nesc[b]);
      } else {
        if (bn) pack_block_host_f64<kRoundTrunc, true>(P, b, fx, v, &nout[b], &nesc[b]);
        else pack_block_host_f64<kRoundTrunc, false>(P, b, fx, v, &nout[b], &nesc[b]);
      }
    }
  };
  pool().run(tasks, threads_for(n_threads), fn);
  uint64_t off = 0;
  for (int64_t b = 0; b < nb; ++b) {
    dir[b] = off | ((uint64_t)nout[b] << 38) | ((uint64_t)nesc[b] << 51);
    off += var[(size_t)b].size();
  }
  if (nb & 1) dir[nb] = 0;
  uint32_t* vr = fixed + (size_t)nb * fk;
  const size_t bn_words = bn ? 4 * (size_t)p->bn_channels : 0;
  const size_t total = sizeof(SmqPackedHeader) + 8 * (size_t)pk_dir_entries(nb) +
                       4 * ((size_t)nb * fk + off + bn_words);
  if (total > out_bytes) {
    set_error("cpu compress_f64: stream of %zu bytes exceeds the buffer (%zu)", total, out_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  uint64_t at = 0;
  for (int64_t b = 0; b < nb; ++b) {
    const auto& v = var[(size_t)b];
    if (!v.empty()) memcpy(vr + at, v.data(), 4 * v.size());
    at += v.size();
  }
  if (bn) {
    double* tab = reinterpret_cast<double*>(vr + off);
    memcpy(tab, p->bn_gamma, 8 * (size_t)p->bn_channels);
    memcpy(tab + p->bn_channels, p->bn_beta, 8 * (size_t)p->bn_channels);
  }
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  SmqPackedHeader h;
  memset(&h, 0, sizeof(h));
  h.magic = SMQ_PACK_MAGIC;
  h.version = SMQ_PACK_VERSION;
  h.n = n;
  h.block_elems = kPB;
  h.n_blocks = (uint32_t)nb;
  h.num_bits_main = p->num_bits_main;
  h.num_bits_outlier = p->num_bits_outlier;
  h.flags = SMQ_PACK_FLAG_F64 | (p->all_positive ? SMQ_PACK_FLAG_ALL_POSITIVE : 0u) |
            (R.safe_q ? SMQ_PACK_FLAG_SAFE_Q : 0u) |
            (p->main_std_dev_threshold < 0.0f ? SMQ_PACK_FLAG_BOTH_SIDES : 0u) |
            (bn ? SMQ_PACK_FLAG_BN : 0u);
  h.thr = p->main_std_dev_threshold;
  h.range_main = p->range_main;
  h.range_outlier = p->range_outlier;
  h.mean = (float)st.mean;
  h.std_dev = (float)st.std_dev;
  h.inv_range_main = 1.0 / (double)p->range_main;
  h.inv_range_outlier = 1.0 / (double)p->range_outlier;
  h.data_words = off;
  h.total_bytes = total;
  h.bn_channels = bn ? (uint32_t)p->bn_channels : 0u;
  h.bn_inner = bn ? p->bn_inner : 0;
  h.mean_f64 = st.mean;
  h.std_dev_f64 = st.std_dev;
  memcpy(out, &h, sizeof(h));
  return SMQ_OK;
}

static int unpack_host_f64(const uint8_t* in, double* y, int64_t n, int n_threads) {
  SmqPackedHeader h;
  memcpy(&h, in, sizeof(h));
  if (h.magic != SMQ_PACK_MAGIC || h.version != SMQ_PACK_VERSION || h.n != n ||
      h.block_elems != (uint32_t)kPB || h.n_blocks != (uint32_t)((n + kPB - 1) / kPB) ||
      !(h.flags & SMQ_PACK_FLAG_F64) || h.num_bits_main < 2 || h.num_bits_main > 25 ||
      h.num_bits_outlier < 3 || h.num_bits_outlier > 25) {
    set_error("cpu decompress_f64: not a version-%u float64 stream of %lld elements",
              SMQ_PACK_VERSION, (long long)n);
    return SMQ_ERR_INVALID;
  }
  const int wm = h.num_bits_main - 1, wo = h.num_bits_outlier - 1, we = wo > wm ? wo - wm : 0;
  const int64_t nb = h.n_blocks;
  const size_t fk = pk_fixed_words(wm);
  const uint64_t* dir = reinterpret_cast<const uint64_t*>(in + sizeof(SmqPackedHeader));
  const uint32_t* fixed = reinterpret_cast<const uint32_t*>(dir + pk_dir_entries(nb));
  const uint32_t* vr = fixed + (size_t)nb * fk;
  const bool bn = (h.flags & SMQ_PACK_FLAG_BN) != 0, ap = (h.flags & 1u) != 0;
  const bool both = (h.flags & SMQ_PACK_FLAG_BOTH_SIDES) != 0;
  const double* g = bn ? reinterpret_cast<const double*>(vr + h.data_words) : nullptr;
  const double* bb = bn ? g + h.bn_channels : nullptr;
  ElemF64 c;
  memset(&c, 0, sizeof(c));
  c.mean = h.mean_f64;
  c.sd = h.std_dev_f64;
  c.sthr = (double)h.thr;
  c.snthr = -c.sthr;
  c.zh = (double)(0.0f * -h.thr);
  c.zl = (double)(0.0f * h.thr);
  c.r_main = (double)h.range_main;
  c.r_out = (double)h.range_outlier;
  const int64_t tasks = (nb + kPackTaskBlocks - 1) / kPackTaskBlocks;
  const std::function<void(int64_t)> fn = [&](int64_t t) {
    std::vector<double> qb(kPB);
    std::vector<uint8_t> sides(kPB);  // bit 0: hi, bit 1: lo
    const uint8_t both2 = both ? 3 : 0;
    const int64_t b1 = std::min(nb, (t + 1) * kPackTaskBlocks);
    for (int64_t b = t * kPackTaskBlocks; b < b1; ++b) {
      const int64_t e0 = b * kPB, m = std::min<int64_t>(kPB, n - e0);
      const uint64_t d = dir[b];
      const uint64_t vbase = d & ((1ull << 38) - 1ull);
      const uint32_t n_out = (uint32_t)((d >> 38) & 0x1fffu), n_esc = (uint32_t)(d >> 51);
      const uint32_t* fx = fixed + (size_t)b * fk;
      const uint32_t* ext = vr + vbase;
      const uint32_t* esc = ext + ((size_t)we * n_out + 31) / 32;
      uint32_t rank = 0;
      for (int64_t e = 0; e < m; ++e) {
        uint32_t code = get_bits(fx + 128, (uint64_t)e * wm, wm);
        if ((fx[e >> 5] >> (e & 31)) & 1u) {
          if (we > 0) code |= get_bits(ext, (uint64_t)rank * we, we) << wm;
          ++rank;
          const uint32_t side = (code >> (wo - 1)) & 1u;
          const double mag = (double)(code & ((1u << (wo - 1)) - 1u));
          qb[(size_t)e] = side ? -mag : mag;
          sides[(size_t)e] = side ? 2 : 1;
        } else {
          qb[(size_t)e] = (double)((code >= (1u << (wm - 1))) ? (int32_t)code - (1 << wm)
                                                              : (int32_t)code);
          sides[(size_t)e] = both2;
        }
      }
      for (uint32_t k = 0; k < n_esc; ++k)
        if (esc[3 * k] < (uint32_t)m)
          qb[esc[3 * k]] = __builtin_bit_cast(double, (uint64_t)esc[3 * k + 1] |
                                                          ((uint64_t)esc[3 * k + 2] << 32));
      for (int64_t e = 0; e < m; ++e) {
        const bool hi = sides[(size_t)e] & 1, lo = sides[(size_t)e] & 2;
        double out = smaq_dequant_f64<false, false>(qb[(size_t)e], hi, lo, c, 1.0, 0.0);
        if (bn) {
          const int64_t ch = ((e0 + e) / h.bn_inner) % (int64_t)h.bn_channels;
          out = (out * g[ch]) + bb[ch];
        }
        if (ap) out = (out < 0.0) ? 0.0 : out;
        y[e0 + e] = out;
      }
    }
  };
  pool().run(tasks, threads_for(n_threads), fn);
  return SMQ_OK;
}

}  // namespace cpu
}  // namespace smq

using namespace smq;

extern "C" {

int smq_cpu_threads(void) { return cpu::pool().size(); }

int smq_cpu_smaq_roundtrip(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                           const float* uniforms, const SmqSmaqStats* stats_in, void* ws,
                           size_t ws_bytes, int n_threads) {
  int rc = smaq_validate(p, dtype);
  if (rc) return rc;
  if (n < 1 || !x || !y) {
    set_error("cpu smaq: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (!ws || ws_bytes < smq_smaq_workspace_bytes(n)) {
    set_error("cpu smaq: workspace too small: need %zu bytes", smq_smaq_workspace_bytes(n));
    return SMQ_ERR_WORKSPACE;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1)) {
    set_error("cpu smaq: batch-norm parameters incomplete");
    return SMQ_ERR_INVALID;
  }
  char* w = static_cast<char*>(ws);
  if (dtype == SMQ_DTYPE_F32) return cpu::smaq_roundtrip<kF32>(x, y, n, p, uniforms, stats_in, w, ws_bytes, n_threads);
  if (dtype == SMQ_DTYPE_F16) return cpu::smaq_roundtrip<kF16>(x, y, n, p, uniforms, stats_in, w, ws_bytes, n_threads);
  return cpu::smaq_roundtrip<kBF16>(x, y, n, p, uniforms, stats_in, w, ws_bytes, n_threads);
}

int smq_cpu_smaq_compress(const void* x, int dtype, int64_t n, const SmqSmaqParams* p,
                          void* packed, size_t packed_bytes, void* ws, size_t ws_bytes,
                          int n_threads) {
  int rc = smaq_validate(p, dtype);
  if (rc) return rc;
  if (n < 1 || !x || !packed) {
    set_error("cpu compress: n must be >= 1, x and packed non-NULL");
    return SMQ_ERR_INVALID;
  }
  if (p->num_bits_main < 2 || p->num_bits_main > 25 || p->num_bits_outlier < 3 ||
      p->num_bits_outlier > 25) {
    set_error("cpu compress: needs 2 <= num_bits_main <= 25 and 3 <= num_bits_outlier <= 25");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1)) {
    set_error("cpu compress: batch-norm parameters incomplete");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source == SMQ_STATS_INJECTED) {
    set_error("cpu compress: computes its statistics (SMQ_STATS_WORKSPACE or _SAMPLED*)");
    return SMQ_ERR_INVALID;
  }
  const size_t bound = smq_smaq_pack_bound_bn(n, p->num_bits_main, p->num_bits_outlier,
                                              p->bn_gamma ? p->bn_channels : 0);
  if (packed_bytes < bound) {
    set_error("cpu compress: packed buffer too small: need %zu bytes, got %zu", bound, packed_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t k = p->stats_source == SMQ_STATS_SAMPLED_DEVICE
                        ? std::min<int64_t>(p->num_samples, n) : 0;
  const size_t need = k > 0 ? smq_smaq_workspace_bytes_sampled(n, k) : smq_smaq_workspace_bytes(n);
  if (!ws || ws_bytes < need) {
    set_error("cpu compress: workspace too small: need %zu bytes", need);
    return SMQ_ERR_WORKSPACE;
  }
  uint8_t* out = static_cast<uint8_t*>(packed);
  char* w = static_cast<char*>(ws);
  if (dtype == SMQ_DTYPE_F32) return cpu::pack_host<kF32>(x, n, p, out, packed_bytes, w, ws_bytes, n_threads);
  if (dtype == SMQ_DTYPE_F16) return cpu::pack_host<kF16>(x, n, p, out, packed_bytes, w, ws_bytes, n_threads);
  return cpu::pack_host<kBF16>(x, n, p, out, packed_bytes, w, ws_bytes, n_threads);
}

int smq_cpu_smaq_decompress(const void* packed, float* y, int64_t n, int n_threads) {
  if (n < 1 || !packed || !y) {
    set_error("cpu decompress: n must be >= 1, packed and y non-NULL");
    return SMQ_ERR_INVALID;
  }
  return cpu::unpack_host(static_cast<const uint8_t*>(packed), y, n, n_threads);
}

int smq_cpu_smaq_compress_f64(const double* x, int64_t n, const SmqSmaqParams* p, void* packed,
                              size_t packed_bytes, void* ws, size_t ws_bytes, int n_threads) {
  int rc = smaq_validate(p, SMQ_DTYPE_F32);
  if (rc) return rc;
  if (n < 1 || !x || !packed) {
    set_error("cpu compress_f64: n must be >= 1, x and packed non-NULL");
    return SMQ_ERR_INVALID;
  }
  if (p->num_bits_main < 2 || p->num_bits_main > 25 || p->num_bits_outlier < 3 ||
      p->num_bits_outlier > 25) {
    set_error("cpu compress_f64: needs 2 <= num_bits_main <= 25 and 3 <= num_bits_outlier <= 25");
    return SMQ_ERR_INVALID;
  }
  if (p->main_std_dev_threshold_f64 == 0.0 || !(p->clamp_hi_f64 > 0.0)) {
    set_error("cpu compress_f64: params.main_std_dev_threshold_f64 / clamp_*_f64 unset");
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1)) {
    set_error("cpu compress_f64: batch-norm parameters incomplete");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source == SMQ_STATS_INJECTED) {
    set_error("cpu compress_f64: computes its statistics (SMQ_STATS_WORKSPACE or _SAMPLED*)");
    return SMQ_ERR_INVALID;
  }
  const size_t bound = smq_smaq_pack_bound_f64(n, p->num_bits_main, p->num_bits_outlier,
                                               p->bn_gamma ? p->bn_channels : 0);
  if (packed_bytes < bound) {
    set_error("cpu compress_f64: packed buffer too small: need %zu bytes, got %zu", bound,
              packed_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  const int64_t k = p->stats_source == SMQ_STATS_SAMPLED_DEVICE
                        ? std::min<int64_t>(p->num_samples, n) : 0;
  const size_t need = k > 0 ? smq_smaq_workspace_bytes_sampled(n, k) : smq_smaq_workspace_bytes(n);
  if (!ws || ws_bytes < need) {
    set_error("cpu compress_f64: workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  return cpu::pack_host_f64(x, n, p, static_cast<uint8_t*>(packed), packed_bytes,
                            static_cast<char*>(ws), ws_bytes, n_threads);
}

int smq_cpu_smaq_decompress_f64(const void* packed, double* y, int64_t n, int n_threads) {
  if (n < 1 || !packed || !y) {
    set_error("cpu decompress_f64: n must be >= 1, packed and y non-NULL");
    return SMQ_ERR_INVALID;
  }
  return cpu::unpack_host_f64(static_cast<const uint8_t*>(packed), y, n, n_threads);
}

int smq_cpu_float_quant(const void* x, int dtype_in, void* y, int dtype_out, int64_t n,
                        int exp_bits, int man_bits, int rounding, int check_inf,
                        const uint32_t* rand_bits, uint64_t seed, uint64_t offset, int n_threads) {
  if (n < 0 || (n > 0 && (!x || !y))) {
    set_error("cpu float_quant: bad tensor arguments");
    return SMQ_ERR_INVALID;
  }
  if (dtype_in != SMQ_DTYPE_F32 && dtype_in != SMQ_DTYPE_F16 && dtype_in != SMQ_DTYPE_BF16 &&
      dtype_in != SMQ_DTYPE_F64) {
    set_error("cpu float_quant: dtype_in must be SMQ_DTYPE_F32, _F16, _BF16 or _F64 (got %d)", dtype_in);
    return SMQ_ERR_INVALID;
  }
  const bool dout = dtype_in == SMQ_DTYPE_F64 && dtype_out == SMQ_DTYPE_F64;
  if (!dout && dtype_out != SMQ_DTYPE_F16 && (dtype_out != SMQ_DTYPE_F32 || dtype_in == SMQ_DTYPE_F64)) {
    set_error("cpu float_quant: dtype_out must be SMQ_DTYPE_F32 or _F16 (_F64 or _F16 for fp64 "
              "input; got %d)", dtype_out);
    return SMQ_ERR_INVALID;
  }
  if (exp_bits < 2 || exp_bits > 8 || man_bits < 0 || man_bits > 22) {
    set_error("cpu float_quant: exp_bits in [2,8] and man_bits in [0,22] required (got %d,%d)",
              exp_bits, man_bits);
    return SMQ_ERR_INVALID;
  }
  if (rounding != SMQ_ROUND_NEAREST && rounding != SMQ_ROUND_STOCHASTIC) {
    set_error("cpu float_quant: rounding must be SMQ_ROUND_NEAREST or SMQ_ROUND_STOCHASTIC");
    return SMQ_ERR_INVALID;
  }
  if (n == 0) return SMQ_OK;
  const bool sr = rounding == SMQ_ROUND_STOCHASTIC, hout = dtype_out == SMQ_DTYPE_F16;
  const float mv = qtorch_quant(FLT_MAX, 0u, exp_bits, man_bits, false);
  const uint32_t key = rng_key(seed);
#define SMQ_CFQ(T, H) \
  cpu::float_quant_pass<T, H>(x, y, n, exp_bits, man_bits, sr, check_inf, rand_bits, key, offset, mv, n_threads)
  if (dout) {
    cpu::parallel_tasks(n, n_threads, [&](int64_t, int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i) {
        const uint32_t r = !sr ? 0u : (rand_bits ? rand_bits[i] : rng_u32(key, offset + (uint64_t)i));
        float q = qtorch_quant((float)static_cast<const double*>(x)[i], r, exp_bits, man_bits, sr);
        if (check_inf && fabsf(q - mv) <= FLT_EPSILON) q = INFINITY;
        static_cast<double*>(y)[i] = (double)q;
      }
    });
  } else if (dtype_in == SMQ_DTYPE_F64) SMQ_CFQ(SMQ_DTYPE_F64, true);
  else if (dtype_in == SMQ_DTYPE_F32) { if (hout) SMQ_CFQ(kF32, true); else SMQ_CFQ(kF32, false); }
  else if (dtype_in == SMQ_DTYPE_F16) { if (hout) SMQ_CFQ(kF16, true); else SMQ_CFQ(kF16, false); }
  else { if (hout) SMQ_CFQ(kBF16, true); else SMQ_CFQ(kBF16, false); }
#undef SMQ_CFQ
  return SMQ_OK;
}

int smq_cpu_s2fp8_roundtrip(const void* x, int dtype, void* y, int64_t n, int precision,
                            int check_inf, const uint32_t* rand_bits, uint64_t seed,
                            uint64_t offset, const SmqS2fp8Stats* stats_in, void* ws,
                            size_t ws_bytes, uint32_t flags, int n_threads) {
  if (n < 1 || !x || !y) {
    set_error("cpu s2fp8: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (dtype != SMQ_DTYPE_F32 && dtype != SMQ_DTYPE_F16 && dtype != SMQ_DTYPE_BF16) {
    set_error("cpu s2fp8: dtype must be SMQ_DTYPE_F32, _F16 or _BF16 (got %d)", dtype);
    return SMQ_ERR_INVALID;
  }
  if (precision != 16 && precision != 32) {
    set_error("cpu s2fp8: precision must be 16 or 32 (got %d)", precision);
    return SMQ_ERR_INVALID;
  }
  if (precision == 32 && dtype != SMQ_DTYPE_F32) {
    set_error("cpu s2fp8: precision 32 quantises the tensor as is and needs fp32 input");
    return SMQ_ERR_INVALID;
  }
  if (flags & ~(SMQ_S2FP8_OUT_Y | SMQ_S2FP8_OUT_T | SMQ_S2FP8_EXACT_POW | SMQ_S2FP8_SPLIT)) {
    set_error("cpu s2fp8: unsupported flags 0x%x", flags);
    return SMQ_ERR_INVALID;
  }
  const int out_mode = (flags & SMQ_S2FP8_OUT_Y) ? 1 : ((flags & SMQ_S2FP8_OUT_T) ? 2 : 0);
  if ((flags & SMQ_S2FP8_OUT_Y) && (flags & SMQ_S2FP8_OUT_T)) {
    set_error("cpu s2fp8: SMQ_S2FP8_OUT_Y and SMQ_S2FP8_OUT_T are exclusive");
    return SMQ_ERR_INVALID;
  }
  if (out_mode && precision != 32) {
    set_error("cpu s2fp8: SMQ_S2FP8_OUT_* need precision 32");
    return SMQ_ERR_INVALID;
  }
  SmqS2fp8Stats s;
  memset(&s, 0, sizeof(s));
  const uint32_t n_used = (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n);
  if (dtype == SMQ_DTYPE_F32) {
    if (stats_in) cpu::s2_derive<kF32>(stats_in->mu, stats_in->m, n_used, &s);
    else cpu::s2_stats<kF32>(x, n, n_threads, &s);
  } else if (dtype == SMQ_DTYPE_F16) {
    if (stats_in) cpu::s2_derive<kF16>(stats_in->mu, stats_in->m, n_used, &s);
    else cpu::s2_stats<kF16>(x, n, n_threads, &s);
  } else {
    if (stats_in) cpu::s2_derive<kBF16>(stats_in->mu, stats_in->m, n_used, &s);
    else cpu::s2_stats<kBF16>(x, n, n_threads, &s);
  }
  const bool p16 = precision == 16, hout = p16 && dtype == SMQ_DTYPE_F16;
  const uint32_t key = rng_key(seed);
  if (dtype == SMQ_DTYPE_F32)
    cpu::s2_pass<kF32>(x, y, n, p16, hout, check_inf, rand_bits, key, offset, s, out_mode, n_threads);
  else if (dtype == SMQ_DTYPE_F16)
    cpu::s2_pass<kF16>(x, y, n, p16, hout, check_inf, rand_bits, key, offset, s, out_mode, n_threads);
  else
    cpu::s2_pass<kBF16>(x, y, n, p16, hout, check_inf, rand_bits, key, offset, s, out_mode, n_threads);
  if (ws && ws_bytes >= sizeof(s)) memcpy(ws, &s, sizeof(s));
  return SMQ_OK;
}

}  // extern "C"

extern "C" {

int smq_cpu_smaq_roundtrip_f64(const double* x, double* y, int64_t n, const SmqSmaqParams* p,
                               const double* uniforms, const SmqSmaqStatsF64* stats_in, void* ws,
                               size_t ws_bytes, int n_threads) {
  int rc = smaq_validate(p, SMQ_DTYPE_F32);
  if (rc) return rc;
  if (n < 1 || !x || !y) {
    set_error("cpu smaq f64: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (p->main_std_dev_threshold_f64 == 0.0 || !(p->clamp_hi_f64 > 0.0)) {
    set_error("cpu smaq f64: params.main_std_dev_threshold_f64 / clamp_*_f64 unset");
    return SMQ_ERR_INVALID;
  }
  if (!ws || ws_bytes < smq_smaq_workspace_bytes(n)) {
    set_error("cpu smaq f64: workspace too small: need %zu bytes", smq_smaq_workspace_bytes(n));
    return SMQ_ERR_WORKSPACE;
  }
  if (p->bn_gamma && (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1)) {
    set_error("cpu smaq f64: batch-norm parameters incomplete");
    return SMQ_ERR_INVALID;
  }
  return cpu::smaq_roundtrip_f64(x, y, n, p, uniforms, stats_in, static_cast<char*>(ws), ws_bytes,
                                 n_threads);
}

int smq_cpu_s2fp8_roundtrip_f64(const double* x, double* y, int64_t n, int precision,
                                int check_inf, const uint32_t* rand_bits, uint64_t seed,
                                uint64_t offset, const SmqS2fp8StatsF64* stats_in, void* ws,
                                size_t ws_bytes, uint32_t flags, int n_threads) {
  if (n < 1 || !x || !y) {
    set_error("cpu s2fp8 f64: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (precision != 16 && precision != 32) {
    set_error("cpu s2fp8 f64: precision must be 16 or 32 (got %d)", precision);
    return SMQ_ERR_INVALID;
  }
  if (flags & ~(SMQ_S2FP8_OUT_Y | SMQ_S2FP8_OUT_T | SMQ_S2FP8_EXACT_POW | SMQ_S2FP8_SPLIT)) {
    set_error("cpu s2fp8 f64: unsupported flags 0x%x", flags);
    return SMQ_ERR_INVALID;
  }
  if ((flags & SMQ_S2FP8_OUT_Y) && (flags & SMQ_S2FP8_OUT_T)) {
    set_error("cpu s2fp8 f64: SMQ_S2FP8_OUT_Y and SMQ_S2FP8_OUT_T are exclusive");
    return SMQ_ERR_INVALID;
  }
  const int out_mode = (flags & SMQ_S2FP8_OUT_Y) ? 1 : ((flags & SMQ_S2FP8_OUT_T) ? 2 : 0);
  if (out_mode && precision != 32) {
    set_error("cpu s2fp8 f64: SMQ_S2FP8_OUT_* need precision 32");
    return SMQ_ERR_INVALID;
  }
  SmqS2fp8StatsF64 s;
  memset(&s, 0, sizeof(s));
  if (stats_in) {
    s2_derive_f64(stats_in->mu * (double)n, stats_in->m, n, &s);
    s.mu = stats_in->mu;
    const double alpha = (1.0 / (s.m - s.mu)) * 15.0;
    s.alpha = alpha;
    s.beta = (-alpha) * s.mu;
    s.beta_pow2 = pow(2.0, s.beta);
    s.inv_beta_pow2 = 1.0 / s.beta_pow2;
    s.inv_alpha = 1.0 / alpha;
  } else {
    cpu::s2_stats_f64(x, n, n_threads, &s);
  }
  const float mv = qtorch_quant(FLT_MAX, 0u, 5, 2, false);
  const uint32_t key = rng_key(seed);
  const bool p16 = precision == 16;
  cpu::parallel_tasks(n, n_threads, [&](int64_t, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint32_t r = rand_bits ? rand_bits[i] : rng_u32(key, offset + (uint64_t)i);
      y[i] = p16 ? s2_elem_f64<true>(x[i], r, s, check_inf, mv, 0)
                 : s2_elem_f64<false>(x[i], r, s, check_inf, mv, out_mode);
    }
  });
  if (ws && ws_bytes >= sizeof(s)) memcpy(ws, &s, sizeof(s));
  return SMQ_OK;
}

}  // extern "C"
