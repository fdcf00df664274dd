// smaq.hip — SmaQ compress->decompress round trip for gfx950 (MI355X).
//
// Reference: smart_compress/compress/smart.py:110-190 (SmartFP.__call__). The reference issues
// ~24 ATen kernels and one host sync per call; here a call is two launches and no sync:
//
//   smaq_stats_kernel  one HBM read (4 B/elem): shifted fp64 sums (+ fp32 min/max in range-std
//                      mode) per workgroup; the last workgroup to arrive reduces the partials in a
//                      fixed order and writes SmqSmaqStats (mean, std, std==0->1, clamp) into the
//                      workspace header.                            smart.py:130-134, 100-108, 151-152
//   smaq_apply_kernel  read + write (8 B/elem), float4 (dwordx4) coalesced streams, per element:
//                      z-score, main/outlier split, N-bit scale, stochastic rounding from the
//                      counter-based RNG (or trunc), de-quantisation, all_positive.  smart.py:154-182
//
// smq_smaq_roundtrip on tensors up to kDeferMaxN elements defers the statistics' final reduction:
// the statistics launch only stores its partials, and every apply workgroup reduces them itself in
// one fixed order (defer_consts) — no workgroup of either launch waits on another.
//
// Sampled statistics (smart.py:86-91) need no stats launch: every workgroup of the apply kernel
// gathers the k <= 64 sampled elements itself (L2-resident after the first workgroup) and reduces
// them in the same fixed order, so the whole call is ONE launch of 8 B/elem.
#include <math.h>
#include <stdarg.h>

#include <algorithm>
#include <atomic>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "smq_common.h"
#include "smaq_elem.h"
#include "smaq_host.h"
#include "smaq_small.h"

namespace smq {

// ------------------------------------------------------------------------------------------------
// error reporting
// ------------------------------------------------------------------------------------------------
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return SMQ_ERR_LAUNCH;
  }
  return SMQ_OK;
}

ArriveTag arrive_tag(const void* ws, hipStream_t st) {
  // one running tag per slot; workspaces hashing to the same slot only mispredict (one CAS)
  static std::atomic<uint32_t> slots[256];
  const uint64_t h = ((uint64_t)(uintptr_t)ws >> 6) * 0x9e3779b97f4a7c15ull;
  const uint32_t v = slots[h >> 56].fetch_add(1u, std::memory_order_relaxed);
  ArriveTag t;
  t.tag = (v % 0x7fffffffu) + 1u;  // [1, 2^31 - 1]: never the 0 of a zeroed workspace
  t.next = (t.tag % 0x7fffffffu) + 1u;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive)
    t.next = t.tag;  // replays of the captured call reuse this tag
  return t;
}

// measurement knob SMQ_HALF_TILE=0: fp16 / bf16 inputs keep 8-B loads (grid-stride statistics
// sweep, one float4 of elements per apply slot)
static bool half_tile_env() {
  static const bool v = [] {
    const char* e = knob_env("SMQ_HALF_TILE");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

static int grid_for(int64_t work_items, int per_block_items, int cap) {
  int64_t g = (work_items + per_block_items - 1) / per_block_items;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// Memory shapes measured on MI355X (tools/membench.hip, tools/statsbench.hip, profiles/): a read
// stream wants the whole grid sweeping the buffer in address order with ONE front: grid-stride
// single loads over ~2k workgroups, or (better, r04) tile-stride over 512 workgroups where each
// step of a workgroup is one contiguous 16 KiB tile and the next tile's loads are in flight while
// the current one is summed; several loads per lane at grid-stride distance open several sweep
// fronts (-20 %). A read+write stream is fastest as flat contiguous tiles, one per workgroup; with
// the stochastic-rounding ALU chain 2 vector slots per lane beat 1 and 4 (cold-cache sweep,
// profiles/r02_kbench_cold_tile*.json), truncation prefers 1.
constexpr int kStatsGridCap = 2048;  // also the number of fp64 partials the last workgroup sums
constexpr int kStatsTileGrid = 512;  // tile-stride sweep: 2 workgroups per CU (launch_stats)
// Deferred statistics (defer_consts): at most kDeferMaxG statistics workgroups, whose partials
// every apply workgroup loads (4 per lane of wave 0), on tensors of at most kDeferMaxN elements.
// Back-to-back smq_smaq_roundtrip calls, fp32, us per call, off -> on (tools/defer_exp.sh, two
// interleaved rounds): 64K 9.1 -> 8.0; 256K 9.4 -> 8.4; 1M 11.5 -> 10.2; 2M 13.2 -> 11.7; 4M 16.9 ->
// 15.1; 8M 26.0 -> 23.6; 16M 40.1 -> 44.0; 32M 66.5 -> 79.6 (there the apply grid's partial
// loads and the 256-workgroup sweep cost more than the hand-off they replace).
constexpr int kDeferMaxG = 256;
static_assert(kDeferMaxG == kSmallMaxG, "reduce_partials_w0 reduces <= kSmallMaxG partials");
constexpr int64_t kDeferMaxN = 12ll << 20;
// plain-load tail of an nt sweep (launch_stats): the Infinity Cache's size. 256M headline, two
// interleaved rounds, ms/step: tail 0: 0.497 / 0.497; 128: 0.495 / 0.491; 160: 0.488 / 0.486;
// 192: 0.484-0.490; 224: 0.488 / 0.489; 256: 0.488-0.492; 320: 0.484 / 0.488 (tools/tail_exp.sh)
constexpr int64_t kStatsPlainTailMB = 256;
constexpr int64_t kStatsNtMinMB = 512;  // non-temporal statistics loads from this tensor size on

static inline bool aligned(const void* p, unsigned a) { return ((uintptr_t)p & (a - 1)) == 0; }

template <bool RANGE, int TIN, bool TILE = false, bool NT = false>
__global__ __launch_bounds__(kBlock) void smaq_stats_kernel(const void* __restrict__ x, int64_t n,
                                                            int vec, FinalizeArgs fin,
                                                            StatPartial* __restrict__ partials,
                                                            unsigned long long* counter,
                                                            ArriveTag tag, SmqSmaqStats* out,
                                                            int64_t nt_end, double* def_rec) {
  __shared__ uint32_t arrive_slot;
  clear_aux(fin);
  // Shift = median of three fixed elements: keeps sum(x-K)^2 - (sum(x-K))^2/n well conditioned
  // unless the mean is > 2^14 standard deviations away from all three.
  const float k0 = load1<TIN>(x, 0), k1 = load1<TIN>(x, n >> 1), k2 = load1<TIN>(x, n - 1);
  const float kmed = fmaxf(fminf(k0, k1), fminf(fmaxf(k0, k1), k2));
  const double shift = (double)kmed;

  // four independent fp64 chains (one per vector component) so the adds of one iteration do not
  // serialise behind each other while the next load is in flight
  StatAcc acc, ay, az, aw;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (TIN != kF32 && vec == 2 && TILE) {
    // fp16 / bf16 on a 16-B aligned pointer: the same tile-stride sweep with one 16-B load of 8
    // elements per lane and slot (tiles of kBlock * 4 such loads, the next tile's in flight)
    const int64_t n8 = n >> 3;
    constexpr int64_t kT = (int64_t)kBlock * 4;
    const int64_t tstride = (int64_t)gridDim.x * kT;
    int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x;
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * kBlock < n8) cur[u] = static_cast<const uint4*>(x)[t + u * kBlock];
    for (; t < n8; t += tstride) {
      const int64_t tn = t + tstride;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tn + u * kBlock < n8) nxt[u] = static_cast<const uint4*>(x)[tn + u * kBlock];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (t + u * kBlock < n8) {
          float4 a, b;
          const uint2 lo = make_uint2(cur[u].x, cur[u].y), hi = make_uint2(cur[u].z, cur[u].w);
          a = load4<TIN>(&lo, 0);
          b = load4<TIN>(&hi, 0);
          acc.add<RANGE>(a.x, shift);
          ay.add<RANGE>(a.y, shift);
          az.add<RANGE>(a.z, shift);
          aw.add<RANGE>(a.w, shift);
          acc.add<RANGE>(b.x, shift);
          ay.add<RANGE>(b.y, shift);
          az.add<RANGE>(b.z, shift);
          aw.add<RANGE>(b.w, shift);
        }
        cur[u] = nxt[u];
      }
    }
    i = (n8 << 3) + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  } else if (vec && TILE) {
    // tile-stride: workgroup w sweeps tiles w, w + G, ... of kBlock * 4 float4 (16 KiB, one
    // contiguous piece per workgroup and step, one front across the grid); the next tile's four
    // loads are issued before the current tile is consumed (8 loads per lane in flight at most)
    const int64_t nv = n >> 2;
    constexpr int64_t kT = (int64_t)kBlock * 4;
    const int64_t tstride = (int64_t)gridDim.x * kT;
    int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x;
    float4 cur[4], nxt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t + u * kBlock < nv)
        cur[u] = (NT && t + u * kBlock < nt_end) ? load4_stream<TIN>(x, t + u * kBlock)
                                                 : load4<TIN>(x, t + u * kBlock);
    for (; t < nv; t += tstride) {
      const int64_t tn = t + tstride;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tn + u * kBlock < nv)
          nxt[u] = (NT && tn + u * kBlock < nt_end) ? load4_stream<TIN>(x, tn + u * kBlock)
                                                    : load4<TIN>(x, tn + u * kBlock);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (t + u * kBlock < nv) {
          acc.add<RANGE>(cur[u].x, shift);
          ay.add<RANGE>(cur[u].y, shift);
          az.add<RANGE>(cur[u].z, shift);
          aw.add<RANGE>(cur[u].w, shift);
        }
        cur[u] = nxt[u];
      }
    }
    i = (nv << 2) + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  } else if (vec) {
    const int64_t nv = n >> 2;
    for (; i < nv; i += stride) {  // one load in flight per lane: a single sweep front
      const float4 v = load4<TIN>(x, i);
      acc.add<RANGE>(v.x, shift);
      ay.add<RANGE>(v.y, shift);
      az.add<RANGE>(v.z, shift);
      aw.add<RANGE>(v.w, shift);
    }
    i = (nv << 2) + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  }
  for (; i < n; i += stride) acc.add<RANGE>(load1<TIN>(x, i), shift);
  acc.s1 = (acc.s1 + ay.s1) + (az.s1 + aw.s1);
  acc.s2 = (acc.s2 + ay.s2) + (az.s2 + aw.s2);
  if (RANGE) {
    acc.mn = fminf(fminf(acc.mn, ay.mn), fminf(az.mn, aw.mn));
    acc.mx = fmaxf(fmaxf(acc.mx, ay.mx), fmaxf(az.mx, aw.mx));
  }

  block_reduce_stats<RANGE>(acc);
  if (gridDim.x == 1) {  // a single workgroup finalises without a hand-off
    if (threadIdx.x == 0)
      finalize_stats<RANGE, TIN>(acc.s1, acc.s2, acc.mn, acc.mx, n, shift, false, fin, out);
    return;
  }
  if (def_rec) {  // deferred statistics: the apply launch reduces the partials (defer_consts)
    if (threadIdx.x == 0) {
      StatPartial* p = partials + blockIdx.x;
      p->s1 = acc.s1;
      p->s2 = acc.s2;
      if (RANGE) {
        p->mn = acc.mn;
        p->mx = acc.mx;
      }
      if (blockIdx.x == 0) {  // the shift, and the call's graph-safe stream position
        unsigned long long base = 0ull;
        if (fin.rng_ctr) {
          base = *fin.rng_ctr;
          *fin.rng_ctr = base + (unsigned long long)fin.rng_n;
        }
        def_rec[0] = shift;
        def_rec[1] = __builtin_bit_cast(double, base);
      }
    }
    return;
  }
  if (threadIdx.x == 0) {
    StatPartial* p = partials + blockIdx.x;
    st_sc1_f64(&p->s1, acc.s1);
    st_sc1_f64(&p->s2, acc.s2);
    if (RANGE) st_sc1_f32x2(&p->mn, acc.mn, acc.mx);
  }
  const uint32_t prev = block_arrive_tagged(counter + (tag.tag & (SmaqWsLayout::kTagWords - 1)),
                                            tag.tag, &arrive_slot);
  if (prev != gridDim.x - 1) return;

  // Last workgroup: ordered reduction of all partials (deterministic for a given n). Every load
  // of a lane is issued before any is consumed: a loop that adds as it loads waits out one memory
  // round trip per partial (8 serial ~1.5 us trips at 2048 partials). Grids of <= kDeferMaxG
  // reduce in the deferred path's order (reduce_partials_w0), so smq_smaq_stats + smq_smaq_apply
  // and the deferred smq_smaq_roundtrip produce the same statistics bit for bit.
  if ((int)gridDim.x <= kDeferMaxG) {
    if (threadIdx.x < kWave) {
      double t1, t2;
      float tmn, tmx;
      reduce_partials_w0<true>(partials, gridDim.x, RANGE, t1, t2, tmn, tmx);
      if (threadIdx.x == 0) {
        finalize_stats<RANGE, TIN>(t1, t2, tmn, tmx, n, shift, false, fin, out);
        arrive_reset(counter + (tag.next & (SmaqWsLayout::kTagWords - 1)), tag.next);
      }
    }
    return;
  }
  constexpr int K = kStatsGridCap / kBlock;
  double s1v[K], s2v[K];
  float mnv[K], mxv[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int b = threadIdx.x + i * kBlock;
    if (b < (int)gridDim.x) {
      const StatPartial* p = partials + b;
      s1v[i] = ld_sc1_f64(&p->s1);
      s2v[i] = ld_sc1_f64(&p->s2);
      if (RANGE) ld_sc1_f32x2(&p->mn, mnv[i], mxv[i]);
    }
  }
  StatAcc tot;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    if (threadIdx.x + i * kBlock < (int)gridDim.x) {
      tot.s1 += s1v[i];
      tot.s2 += s2v[i];
      if (RANGE) {
        tot.mn = fminf(tot.mn, mnv[i]);
        tot.mx = fmaxf(tot.mx, mxv[i]);
      }
    }
  }
  block_reduce_stats<RANGE>(tot);
  if (threadIdx.x == 0) {
    finalize_stats<RANGE, TIN>(tot.s1, tot.s2, tot.mn, tot.mx, n, shift, false, fin, out);
    // the next call's tag, count 0, in the word that call will use
    arrive_reset(counter + (tag.next & (SmaqWsLayout::kTagWords - 1)), tag.next);
  }
}

struct ApplyArgs {
  const void* x;
  float* y;
  int64_t n;
  const float* uniforms;
  const SmqSmaqStats* stats;     // workspace header or injected
  SmqSmaqStats* ws_stats;        // sampled-stats destination
  unsigned long long* out_slots; // outlier count slots
  float thr, r_main, r_out, clamp_lo, clamp_hi, range_coef;
  double inv_r_main, inv_r_out;  // host-computed reciprocals of the ranges
  int safe_q;
  QuotSplit qs;                  // half inputs without BN: the checked two-op quotient (qs.ok)
  unsigned long long* rng_ctr;   // params.offset_counter (graph-safe stream) or NULL
  uint32_t key;
  int all_pos;
  int count;
  int use_range;
  int k;                         // sampled mode
  int reverse;                   // tile order (see smaq_apply_kernel)
  int nt_loads;                  // non-temporal x loads (tensors >= kStatsNtMinMB only)
  uint64_t offset;
  const float* bn_gamma;         // BN variant
  const float* bn_beta;
  int64_t bn_channels, bn_inner;
  const StatPartial* def_parts;  // deferred statistics (defer_consts): the statistics launch's
  const double* def_rec;         // partials and {shift, stream position}; def_g partials, 0 = off
  int def_g;
  int64_t sample_idx[SMQ_MAX_SAMPLES];
};

// Deferred statistics (smq_smaq_roundtrip on tensors up to kDeferMaxN elements): the statistics
// launch leaves only its workgroup partials, and every apply workgroup reduces them itself — in
// one fixed order, so every workgroup (and every call on the same n) gets the same totals — and
// finalises. This replaces the hand-off in which the last statistics workgroup to arrive reduces
// and finalises (partial store, arrival atomic, partial loads, header store: ~5 us of dependent
// round trips, the larger part of a statistics launch on an activation-sized tensor). Wave 0
// loads the partials after the workgroup's x loads are in flight and finalises in lane 0; the
// other waves wait at an LDS-only barrier, their loads still outstanding. Workgroup 0 also
// writes the header (log_size, read_stats).
template <int TIN>
__device__ __forceinline__ void defer_consts(const ApplyArgs& A, ElemConsts& c, uint64_t& off,
                                          float cthr) {
  __shared__ SmqSmaqStats sh;
  if (threadIdx.x < kWave) {
    const int l = threadIdx.x;
    double s1, s2;
    float mn, mx;
    reduce_partials_w0<false>(A.def_parts, A.def_g, A.use_range, s1, s2, mn, mx);
    if (l == 0) {
      const FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, nullptr, 0};
      SmqSmaqStats st;
      if (A.use_range) finalize_stats<true, TIN>(s1, s2, mn, mx, A.n, A.def_rec[0], false, f, &st);
      else finalize_stats<false, TIN>(s1, s2, mn, mx, A.n, A.def_rec[0], false, f, &st);
      st.rng_offset = __builtin_bit_cast(uint64_t, A.def_rec[1]);
      sh = st;
      if (blockIdx.x == 0) *A.ws_stats = st;
    }
  }
  lds_barrier();
  init_consts(c, &sh, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  off = A.offset + sh.rng_offset;
}

template <bool BN>
__device__ __forceinline__ BnTerm bn_term(const ApplyArgs& A, int64_t e) {
  if (!BN) return BnTerm{1.0f, 0.0f};
  const int64_t ch = (e / A.bn_inner) % A.bn_channels;
  return BnTerm{A.bn_gamma[ch], A.bn_beta[ch]};
}

// Sampled statistics (smart.py:86-91): mean and biased std (or range-std) of the k gathered
// elements, by ONE wave into the workspace header; the apply launch reads them like full stats.
template <int TIN>
__global__ __launch_bounds__(kWave) void smaq_sample_stats_kernel(ApplyArgs A) {
  const int lane = threadIdx.x;
  const bool valid = lane < A.k;
  const float v = valid ? load1<TIN>(A.x, A.sample_idx[lane]) : 0.0f;
  const double kd = (double)A.k;
  const double mean = wave_sum(valid ? (double)v : 0.0) / kd;
  const double dv = valid ? ((double)v - mean) : 0.0;
  const double m2 = wave_sum(dv * dv);
  const float mn = wave_min(valid ? v : INFINITY);
  const float mx = wave_max(valid ? v : -INFINITY);
  if (lane == 0) {
    SmqSmaqStats st;
    FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, A.rng_ctr, A.n};
    // finalize_stats takes shifted sums: shift = mean, s1 = 0, s2 = m2 (biased)
    if (A.use_range)
      finalize_stats<true, TIN>(0.0, m2, mn, mx, A.k, mean, true, f, &st);
    else
      finalize_stats<false, TIN>(0.0, m2, mn, mx, A.k, mean, true, f, &st);
    *A.ws_stats = st;
  }
}

// Device-drawn sampled statistics (SMQ_STATS_SAMPLED_DEVICE): one workgroup draws k indices
// (Floyd, smaq_elem.h draw_sample_stats) from the call's stream position and writes the statistics.
struct DrawArgs {
  const void* x;
  int64_t n;
  int k;
  int use_range;
  uint32_t key;                   // rng_key(seed ^ kDrawSalt)
  uint64_t offset;                // params.offset
  unsigned long long* rng_ctr;    // params.offset_counter or NULL
  float clamp_lo, clamp_hi, range_coef;
  SmqSmaqStats* ws_stats;
  int64_t* idx_out;               // workspace, SMQ_MAX_DEVICE_SAMPLES entries
};

template <int TIN>
__global__ __launch_bounds__(kBlock) void smaq_draw_stats_kernel(DrawArgs A) {
  __shared__ DrawLds L;
  __shared__ unsigned long long pos_s;
  if (threadIdx.x == 0) pos_s = A.offset + (A.rng_ctr ? *A.rng_ctr : 0ull);
  __syncthreads();
  // the finaliser snapshots the graph-safe position and advances it by n
  const FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, A.rng_ctr, A.n};
  draw_sample_stats<TIN>(A.x, A.n, A.k, A.key, pos_s, A.use_range, f, A.ws_stats, A.idx_out, L);
}

// ------------------------------------------------------------------------------------------------
// Multi-workgroup draw (k > SMQ_MAX_DEVICE_SAMPLES; smart.py:86-91 takes any k = min(n, num_samples)).
// The same Floyd picks as draw_picks. A step whose candidate t_i no other candidate equals and that
// lies below n - k keeps t_i: every earlier pick is another candidate or a substitute j_m >= n - k.
// Only the other steps — "suspects": a candidate repeated among the candidates, or one in
// [n - k, n) — can be substituted, and their outcome depends on earlier suspects alone (a
// non-suspect pick never equals a suspect's candidate or any j). So:
//   draw_candidates (grid): t_i into pick[], and into a hash set that marks repeated keys;
//   draw_suspects   (grid): a bitmap of the suspect steps (each 32-step word stored once);
//   draw_resolve    (one wave): the suspects in draw order, 64 at a time — a lookup of each
//                   candidate among the earlier chunks' final picks (a second hash set), then
//                   the in-chunk order by readlane / compare — writing the final picks back;
//   draw_gather     (grid): shifted fp64 sums / extrema of the gathered samples per workgroup;
//   draw_finalize   (one workgroup): fixed-order total, finalize_stats (biased), the header.
// Without repeats (k^2 << n) the resolve pass only walks the bitmap.
// ------------------------------------------------------------------------------------------------
constexpr unsigned long long kEmptyKey = ~0ull;

__global__ __launch_bounds__(kBlock) void smaq_draw_candidates_kernel(LargeDrawArgs A) {
  const uint64_t pos = A.offset + (A.rng_ctr ? *A.rng_ctr : 0ull);
  const uint32_t mask = (1u << A.bits) - 1u;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.k;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t t = floyd_candidate(A.key, pos, A.n, (int)A.k, (int)i);
    A.pick[i] = t;
    for (uint32_t s = pick_hash(t, A.bits);; s = (s + 1) & mask) {
      const unsigned long long prev = atomicCAS(A.hkey + s, kEmptyKey, (unsigned long long)t);
      if (prev == kEmptyKey) break;
      if (prev == (unsigned long long)t) {
        atomicOr(A.hdup + s, 1u);
        break;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void smaq_draw_suspects_kernel(LargeDrawArgs A) {
  const uint32_t mask = (1u << A.bits) - 1u;
  const int64_t span = (A.k + kWave - 1) / kWave * kWave;  // whole waves: every word stored once
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < span;
       i += (int64_t)gridDim.x * kBlock) {
    bool sus = false;
    if (i < A.k) {
      const int64_t t = A.pick[i];
      sus = t >= A.n - A.k;
      if (!sus) {
        uint32_t s = pick_hash(t, A.bits);
        while (A.hkey[s] != (unsigned long long)t) s = (s + 1) & mask;
        sus = A.hdup[s] != 0u;
      }
    }
    const uint64_t b = __ballot(sus);
    const int lane = threadIdx.x & (kWave - 1);
    if ((lane & 31) == 0 && i < A.k) A.susp[i >> 5] = (uint32_t)(b >> lane);
  }
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__global__ __launch_bounds__(kWave) void smaq_draw_resolve_kernel(LargeDrawArgs A) {
  __shared__ int32_t list[kWave * 32];  // suspect steps of one 64-word window of the bitmap
  const int lane = threadIdx.x;
  const uint32_t mask = (1u << A.bits) - 1u;
  const int64_t words = (A.k + 31) / 32, base_j = A.n - A.k;
  for (int64_t w0 = 0; w0 < words; w0 += kWave) {
    const int64_t w = w0 + lane;
    uint32_t b = w < words ? A.susp[w] : 0u;
    const uint32_t c = (uint32_t)__builtin_popcount(b);
    const uint32_t incl = wave_incl_scan_u32(c);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    if (total == 0) continue;
    for (uint32_t o = incl - c; b; b &= b - 1) list[o++] = (int32_t)(w * 32 + __builtin_ctz(b));
    __syncthreads();
    for (uint32_t c0 = 0; c0 < total; c0 += kWave) {
      const uint32_t m = c0 + lane;
      const bool act = m < total;
      const int64_t i = act ? list[m] : 0;
      const int64_t t = act ? A.pick[i] : -1;
      bool dup = false;
      if (act) {  // among the final picks of earlier chunks (sc1 loads: the L1 may hold old lines)
        for (uint32_t s = pick_hash(t, A.bits);; s = (s + 1) & mask) {
          const unsigned long long e = ld_sc1_u64(A.h2key + s);
          if (e == kEmptyKey) break;
          if (e == (unsigned long long)t) {
            dup = true;
            break;
          }
        }
      }
      const int cnt = (int)min((uint32_t)kWave, total - c0);
      int64_t p = t;
      for (int l = 0; l < cnt; ++l) {  // step l is final once the earlier lanes' picks are known
        if (lane == l && dup) p = base_j + i;
        const int64_t pl = readlane_i64(p, l);
        if (lane > l && t == pl) dup = true;
      }
      if (act) {
        A.pick[i] = p;
        for (uint32_t s = pick_hash(p, A.bits);; s = (s + 1) & mask)
          if (atomicCAS(A.h2key + s, kEmptyKey, (unsigned long long)p) == kEmptyKey) break;
      }
    }
    __syncthreads();
  }
}

template <int TIN, bool RANGE>
__global__ __launch_bounds__(kBlock) void smaq_draw_gather_kernel(LargeDrawArgs A) {
  const double shift = (double)load1<TIN>(A.x, A.pick[0]);  // step 0 is never substituted
  StatAcc acc;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.k;
       i += (int64_t)gridDim.x * kBlock)
    acc.add<RANGE>(load1<TIN>(A.x, A.pick[i]), shift);
  block_reduce_stats<RANGE>(acc);
  if (threadIdx.x == 0) {
    StatPartial& q = A.parts[blockIdx.x];
    q.s1 = acc.s1;
    q.s2 = acc.s2;
    q.mn = acc.mn;
    q.mx = acc.mx;
  }
}

template <int TIN, bool RANGE>
__global__ __launch_bounds__(kBlock) void smaq_draw_finalize_kernel(LargeDrawArgs A, int g) {
  StatAcc acc;
  for (int b = threadIdx.x; b < g; b += kBlock) {  // per-thread partials in a fixed order
    const StatPartial& q = A.parts[b];
    acc.s1 += q.s1;
    acc.s2 += q.s2;
    acc.mn = fminf(acc.mn, q.mn);
    acc.mx = fmaxf(acc.mx, q.mx);
  }
  block_reduce_stats<RANGE>(acc);
  if (threadIdx.x == 0) {
    const double shift = (double)load1<TIN>(A.x, A.pick[0]);
    // the finaliser snapshots the graph-safe position and advances it by n
    const FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, A.rng_ctr, A.n};
    SmqSmaqStats st;
    finalize_stats<RANGE, TIN>(acc.s1, acc.s2, acc.mn, acc.mx, A.k, shift, true, f, &st);
    *A.ws_stats = st;
  }
}

// Injected statistics (parity tests, callers with their own mean/std): copy the record into the
// workspace header with the fp64 reciprocal the element transform reads.
__global__ void smaq_prep_injected_kernel(const SmqSmaqStats* in, SmqSmaqStats* out,
                                          unsigned long long* rng_ctr, int64_t n) {
  if (threadIdx.x == 0) {
    SmqSmaqStats s = *in;
    s.inv_std_clamped = 1.0 / (double)s.std_clamped;
    s.inv_std_clamped_f32 = (float)s.inv_std_clamped;
    s.quot_check = quot_check_for(s.std_clamped);
    s.rng_offset = 0ull;
    if (rng_ctr) {
      s.rng_offset = *rng_ctr;
      *rng_ctr = s.rng_offset + (unsigned long long)n;
    }
    *out = s;
  }
}

// One workgroup's share of the apply launch. TV = float4 slots per lane per tile: flat tiles of
// kBlock * TV float4 dispatched in (reverse) address order, one front across the grid.
// SUB: see quot_check_for. The unaligned (!VEC) variant always keeps the subnormal check and
// divides q / range by IEEE division (the launcher routes safe_q calls to it).
template <int RM, bool VEC, bool BN, int TIN, int TV, bool AP, bool SUB, bool DEF = false,
          bool QF = false>
__device__ __forceinline__ uint32_t apply_body(const ApplyArgs& A, ElemConsts& c, uint64_t off,
                                               float cthr) {
  constexpr int kTileElems = kBlock * TV * 4;
  uint32_t n_out = 0;
  const int64_t n = A.n;
  if (VEC) {
    // Tiles run in REVERSE address order after a forward statistics sweep of the same tensor:
    // the last ~256 MB of x are then still in the Infinity Cache (MALL) when this launch starts.
    float4* __restrict__ y4 = reinterpret_cast<float4*>(A.y);
    const float4* __restrict__ u4 = reinterpret_cast<const float4*>(A.uniforms);
    const int64_t nv = n >> 2;
    const int64_t tile = A.reverse ? (int64_t)(gridDim.x - 1 - blockIdx.x) : (int64_t)blockIdx.x;
    const int64_t t0 = tile * (kBlock * TV) + threadIdx.x;
    // fp16 inputs (no BN term) in pairs of raw halves: smaq_elem_f16x2 (interleaved A/B at 256M:
    // apply 5.15 -> 5.34 TB/s event-timed, profiles/r3c_ab_f16pk.txt)
    constexpr bool RAW16 = !BN && TIN == kF16;
    float4 v[TV], uu[TV];
    uint2 hv[TV];
#pragma unroll
    for (int u = 0; u < TV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j < nv) {
        if constexpr (RAW16) hv[u] = static_cast<const uint2*>(A.x)[j];
        else v[u] = A.nt_loads ? load4_stream<TIN>(A.x, j) : load4<TIN>(A.x, j);
        if (RM == kRoundUniform) uu[u] = u4[j];
      }
    }
    if (DEF) defer_consts<TIN>(A, c, off, cthr);  // with this tile's loads in flight
    const QuadRun R = quad_run(A.key, off, (uint64_t)nv);
#pragma unroll
    for (int u = 0; u < TV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j >= nv) continue;
      float u0 = 0.0f, u1 = 0.0f, u2 = 0.0f, u3 = 0.0f;
      if (RM == kRoundHash) {
        rng_hu4_run(R, (uint32_t)j, u0, u1, u2, u3);
      } else if (RM == kRoundUniform) {
        u0 = uu[u].x; u1 = uu[u].y; u2 = uu[u].z; u3 = uu[u].w;
      }
      bool b0, b1, b2, b3;
      float4 o;
      if constexpr (RAW16) {
        smaq_elem_f16x2<RM, AP, QF>(hv[u].x, u0, u1, c, o.x, o.y, b0, b1);
        smaq_elem_f16x2<RM, AP, QF>(hv[u].y, u2, u3, c, o.z, o.w, b2, b3);
      } else {
        o.x = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC, QF>(v[u].x, u0, c, b0, bn_term<BN>(A, 4 * j + 0));
        o.y = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC, QF>(v[u].y, u1, c, b1, bn_term<BN>(A, 4 * j + 1));
        o.z = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC, QF>(v[u].z, u2, c, b2, bn_term<BN>(A, 4 * j + 2));
        o.w = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC, QF>(v[u].w, u3, c, b3, bn_term<BN>(A, 4 * j + 3));
      }
      n_out += (unsigned)b0 + (unsigned)b1 + (unsigned)b2 + (unsigned)b3;
      store_stream(y4 + j, o);
    }
    // ragged tail (n % 4 elements): the workgroup owning the last tile
    if (tile == gridDim.x - 1 && threadIdx.x < (int)(n & 3)) {
      const int64_t e = (nv << 2) + threadIdx.x;
      float uf = 0.0f;
      if (RM == kRoundHash) uf = rng_hu(A.key, off + (uint64_t)e);
      if (RM == kRoundUniform) uf = A.uniforms[e];
      bool bt;
      A.y[e] = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC, QF>(load1<TIN>(A.x, e), uf, c, bt, bn_term<BN>(A, e));
      n_out += (unsigned)bt;
    }
  } else {
    // unaligned pointers: the same tile of kTileElems elements with element accesses
    const int64_t e0 = (int64_t)blockIdx.x * kTileElems + threadIdx.x;
#pragma unroll 4
    for (int k = 0; k < kTileElems / kBlock; ++k) {
      const int64_t e = e0 + (int64_t)k * kBlock;
      if (e >= n) break;
      float uf = 0.0f;
      if (RM == kRoundHash) uf = rng_hu(A.key, off + (uint64_t)e);
      if (RM == kRoundUniform) uf = A.uniforms[e];
      bool bt;
      A.y[e] = smaq_elem<RM, BN, TIN, AP, SUB || !VEC, !VEC>(load1<TIN>(A.x, e), uf, c, bt, bn_term<BN>(A, e));
      n_out += (unsigned)bt;
    }
  }
  return n_out;
}

// RM = rounding mode, TIN = input element type, TV = float4 slots per lane per tile.
template <int RM, bool VEC, bool BN, int TIN, int TV>
__global__ __launch_bounds__(kBlock) void smaq_apply_kernel(ApplyArgs A) {
  __shared__ uint32_t sh_cnt[kBlock / kWave];
  ElemConsts c;
  const float cthr = (BN || TIN == kF32) ? A.thr : round_in<TIN>(A.thr);
  // uniform per launch: pick the body once (all_positive, subnormal-quotient check)
  uint32_t n_out;
  if (VEC && !BN && A.def_g) {
    // deferred statistics: quot_check is not known before the loads, keep the check
    n_out = A.all_pos ? apply_body<RM, VEC, BN, TIN, TV, true, true, VEC && !BN>(A, c, 0, cthr)
                      : apply_body<RM, VEC, BN, TIN, TV, false, true, VEC && !BN>(A, c, 0, cthr);
  } else {
    init_consts(c, A.stats, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
    const uint64_t off = A.offset + A.stats->rng_offset;  // + graph-safe stream position
    constexpr bool kQF = VEC && !BN && TIN != kF32;  // (SUB has no effect on half z-scores)
    if (kQF && A.qs.ok) {
      c.qs = A.qs;
      n_out = A.all_pos ? apply_body<RM, VEC, BN, TIN, TV, true, true, false, kQF>(A, c, off, cthr)
                        : apply_body<RM, VEC, BN, TIN, TV, false, true, false, kQF>(A, c, off, cthr);
    } else if (!VEC) {
      n_out = A.all_pos ? apply_body<RM, VEC, BN, TIN, TV, true, true>(A, c, off, cthr)
                        : apply_body<RM, VEC, BN, TIN, TV, false, true>(A, c, off, cthr);
    } else if (A.stats->quot_check) {
      n_out = A.all_pos ? apply_body<RM, VEC, BN, TIN, TV, true, true>(A, c, off, cthr)
                        : apply_body<RM, VEC, BN, TIN, TV, false, true>(A, c, off, cthr);
    } else {
      n_out = A.all_pos ? apply_body<RM, VEC, BN, TIN, TV, true, false>(A, c, off, cthr)
                        : apply_body<RM, VEC, BN, TIN, TV, false, false>(A, c, off, cthr);
    }
  }

  if (A.count) {  // outlier count for log_size (smart.py:184-188): one atomic per workgroup,
                  // spread over SMQ_WS_OUTLIER_SLOTS addresses
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

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static int validate_params(const SmqSmaqParams* p) {
  if (!p) {
    set_error("params is NULL");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source < 0 || p->stats_source > 3) {
    set_error("stats_source %d invalid", p->stats_source);
    return SMQ_ERR_INVALID;
  }
  return SMQ_OK;
}

static float range_coef_for(const SmqSmaqParams* p, int64_t n) {
  // 0 is a real value (fp16 data with n > 65504: half(n) = inf -> C = 0 -> std 0 -> 1)
  if (p->range_std_coef >= 0.0f) return p->range_std_coef;
  // smart.py:101-106: C = 1 / sqrt(2.0 * log(tensor(n).float())) in fp32 ops
  const float lg = logf((float)n);
  const float t = 2.0f * lg;
  return 1.0f / sqrtf(t);
}

static size_t stats_ws_bytes(int64_t n) {
  (void)n;
  static_assert(SmaqWsLayout::kPartials + sizeof(StatPartial) * (size_t)kStatsGridCap ==
                    SMQ_WS_SAMPLES_OFFSET, "smq.h SMQ_WS_SAMPLES_OFFSET");
  return SmaqWsLayout::kTotal;
}

static int check_dtype(int dtype) {
  if (dtype != SMQ_DTYPE_F32 && dtype != SMQ_DTYPE_F16 && dtype != SMQ_DTYPE_BF16) {
    set_error("dtype %d is not one of SMQ_DTYPE_F32/F16/BF16", dtype);
    return SMQ_ERR_INVALID;
  }
  return SMQ_OK;
}

// def_g != NULL: deferred statistics (defer_consts) — *def_g = the number of partials left for the
// apply launch, or 0 when a single workgroup finalised the header itself.
// zero / zero_n: words the launch clears on the way (FinalizeArgs::zero).
static int launch_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                        size_t ws_bytes, hipStream_t st, int* def_g = nullptr,
                        SmqSmaqStats* out = nullptr, uint32_t* zero = nullptr,
                        uint32_t zero_n = 0) {
  // (the single launch's exchange region above the tag counters is not needed here)
  const size_t need = SmaqWsLayout::kTagCounters + 8 * (size_t)SmaqWsLayout::kTagWords;
  if (!ws || ws_bytes < need) {
    set_error("workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  char* base = (char*)ws;
  SmqSmaqStats* hdr = out ? out : (SmqSmaqStats*)base;
  unsigned long long* counter = (unsigned long long*)(base + SmaqWsLayout::kTagCounters);
  StatPartial* partials = (StatPartial*)(base + SmaqWsLayout::kPartials);
  const int vec = aligned(x, dtype == SMQ_DTYPE_F32 ? 16 : 8) ? 1 : 0;
  if (n <= kSmallMaxN && !out) {
    // activation-sized tensors: the partition the single launch uses (smaq_small.h), so every path
    // gives the same statistics bit for bit
    const FinalizeArgs fin{p->clamp_lo, p->clamp_hi, range_coef_for(p, n),
                           (unsigned long long*)p->offset_counter, n, zero, zero_n};
    return launch_stats_small(x, dtype, n, vec != 0, p->use_range_std_dev != 0, fin, ws, st,
                              def_g != nullptr, def_g);
  }
  // fp32 sweeps tile-stride (smaq_stats_kernel<.., TILE>) on at most kStatsTileGrid workgroups;
  // measured on the 256M headline (bench, 3 interleaved rounds): grid-stride at 2048 workgroups
  // 0.542 ms/step; tile-stride at 1024 / 768 / 640 / 512 / 384 / 256 workgroups 0.529 / 0.528 /
  // 0.528 / 0.515 / 0.522 / 0.589 — at 512 (2 per CU, 8 dwordx4 per lane in flight) the sweep
  // takes 169 us instead of 184, and the apply launch after it 335 us instead of 352. fp16 / bf16
  // inputs on a 16-B aligned x sweep tile-stride too, with one 16-B load of 8 elements per lane and
  // slot (256M: 112 -> 90 us, 0.422-0.431 -> 0.407-0.408 ms/step fp16, tools/half_tile.sh; with
  // 8-B loads the tile form had lost, 0.636 vs 0.463); an 8-B aligned x keeps the grid-stride sweep.
  static const int tile_env = [] {  // measurement knob SMQ_STATS_TILE=0: grid-stride sweep
    const char* e = knob_env("SMQ_STATS_TILE");
    return e ? atoi(e) : 1;
  }();
  // half inputs take the tile sweep with 16-B loads when x is 16-B aligned (vec = 2)
  const bool x16 = dtype != SMQ_DTYPE_F32 && aligned(x, 16) && half_tile_env();
  const bool tile = tile_env != 0 && (dtype == SMQ_DTYPE_F32 || x16);
  const int vec_arg = x16 ? 2 : vec;
  static const int grid_env = [] {  // measurement knob SMQ_STATS_GRID (64 .. kStatsGridCap)
    const char* e = knob_env("SMQ_STATS_GRID");
    const int v = e ? atoi(e) : 0;
    return (v >= 64 && v <= kStatsGridCap) ? v : 0;
  }();
  const int cap = grid_env ? grid_env : (tile ? kStatsTileGrid : kStatsGridCap);
  // >= 16K elements per workgroup: mid-size tensors (activations, 1-30M elements) are bound by
  // the arrival of their workgroups, not by bandwidth; at 256M the cap decides
  static const int per_wg = [] {  // measurement knob SMQ_STATS_PER_WG (elements, >= 1024)
    const char* e = knob_env("SMQ_STATS_PER_WG");
    const int v = e ? atoi(e) : kBlock * 4 * 16;
    return v >= kBlock * 4 ? v : kBlock * 4 * 16;
  }();
  // tensors the deferred path may take use its grid cap in EVERY statistics launch, so the
  // partials (and, through reduce_partials_w0, the totals) are the same in both paths
  const bool defer_size = n <= kDeferMaxN || def_g;
  const int grid = grid_for(n, per_wg, defer_size && cap > kDeferMaxG ? kDeferMaxG : cap);
  double* def_rec = nullptr;
  ArriveTag tag{};
  if (def_g) {
    *def_g = grid > 1 ? grid : 0;
    if (grid > 1) def_rec = (double*)(base + SmaqWsLayout::kDeferRec);
  }
  // the host's tag prediction follows the calls that use the arrival counter
  if (!def_rec) tag = arrive_tag(ws, st);
  FinalizeArgs fin{p->clamp_lo, p->clamp_hi, range_coef_for(p, n),
                   (unsigned long long*)p->offset_counter, n, zero, zero_n};
  // non-temporal loads only for tensors well beyond the Infinity Cache: there they keep the
  // sweep from thrashing it (1 GiB: 0.506-0.508 -> 0.499-0.502 ms/step); up to 256 MiB the apply
  // launch re-reads x from the cache the plain loads filled (64 / 128 / 256 MiB tensors: 0.047 /
  // 0.075 / 0.131 ms/step plain against 0.051 / 0.080 / 0.138 nt; tools/ntsize_exp.sh)
  static const int64_t nt_min_bytes = [] {  // measurement knob SMQ_STATS_NT_MIN_MB
    const char* e = knob_env("SMQ_STATS_NT_MIN_MB");
    return (int64_t)(e ? atoll(e) : kStatsNtMinMB) << 20;
  }();
  const bool nt = tile && 4 * n >= nt_min_bytes;
  // with nt loads, the last plain_tail bytes of the sweep still load plain, so they stay in the
  // Infinity Cache for the apply launch, which walks its tiles from the end (measurement knob
  // SMQ_STATS_PLAIN_TAIL_MB)
  static const int64_t plain_tail = [] {
    const char* e = knob_env("SMQ_STATS_PLAIN_TAIL_MB");
    return (int64_t)(e ? atoll(e) : kStatsPlainTailMB) << 20;
  }();
  const int64_t nt_end = (n >> 2) - plain_tail / 16;
#define SMQ_STATS(RANGE, TIN)                                                                       \
  do {                                                                                              \
    if (tile && nt)                                                                                 \
      hipLaunchKernelGGL((smaq_stats_kernel<RANGE, TIN, true, true>), dim3(grid), dim3(kBlock), 0,  \
                         st, x, n, vec_arg, fin, partials, counter, tag, hdr, nt_end, def_rec);         \
    else if (tile)                                                                                  \
      hipLaunchKernelGGL((smaq_stats_kernel<RANGE, TIN, true>), dim3(grid), dim3(kBlock), 0, st, x, \
                         n, vec_arg, fin, partials, counter, tag, hdr, nt_end, def_rec);                \
    else                                                                                            \
      hipLaunchKernelGGL((smaq_stats_kernel<RANGE, TIN>), dim3(grid), dim3(kBlock), 0, st, x, n,    \
                         vec_arg, fin, partials, counter, tag, hdr, nt_end, def_rec);                   \
  } while (0)
  if (dtype == SMQ_DTYPE_F32) {
    if (p->use_range_std_dev) SMQ_STATS(true, kF32); else SMQ_STATS(false, kF32);
  } else if (dtype == SMQ_DTYPE_F16) {
    if (p->use_range_std_dev) SMQ_STATS(true, kF16); else SMQ_STATS(false, kF16);
  } else {
    if (p->use_range_std_dev) SMQ_STATS(true, kBF16); else SMQ_STATS(false, kBF16);
  }
#undef SMQ_STATS
  return check_launch("smaq_stats_kernel");
}

// Float4 slots per lane per tile for the stochastic-rounding kernels (env SMQ_APPLY_TILE = 1 | 2,
// measurement knob). 2: two loads in flight per lane hide the longer SR element chain (256M, r03:
// 0.358 vs 0.368 ms) and halve the outlier-count atomics; truncation always uses 1.
static int sr_tile_v() {
  static const int v = [] {
    const char* e = knob_env("SMQ_APPLY_TILE");
    return (e && atoi(e) == 1) ? 1 : 2;
  }();
  return v;
}

template <int TIN>
static void launch_apply_t(const ApplyArgs& A, int rm, bool vec, bool bn, int tv, int grid,
                           hipStream_t st) {
#define SMQ_APPLY(RMV, VECV, BNV, TVV)                                                         \
  hipLaunchKernelGGL((smaq_apply_kernel<RMV, VECV, BNV, TIN, TVV>), dim3(grid), dim3(kBlock), 0, \
                     st, A)
#define SMQ_APPLY_RM(VECV, BNV)                                         \
  do {                                                                  \
    if (rm == kRoundHash) SMQ_APPLY(kRoundHash, VECV, BNV, 1);          \
    else if (rm == kRoundUniform) SMQ_APPLY(kRoundUniform, VECV, BNV, 1); \
    else SMQ_APPLY(kRoundTrunc, VECV, BNV, 1);                          \
  } while (0)
  if (vec && !bn && rm == kRoundHash && tv == 2) {
    SMQ_APPLY(kRoundHash, true, false, 2);
  } else if (TIN != kF32 && vec && !bn && rm == kRoundHash && tv == 4) {
    SMQ_APPLY(kRoundHash, true, false, 4);
  } else if (vec) {
    if (bn) SMQ_APPLY_RM(true, true); else SMQ_APPLY_RM(true, false);
  } else {
    if (bn) SMQ_APPLY_RM(false, true); else SMQ_APPLY_RM(false, false);
  }
#undef SMQ_APPLY_RM
#undef SMQ_APPLY
}

static int fill_sampled(ApplyArgs& A, const SmqSmaqParams* p, int64_t n) {
  const int64_t k = p->num_samples < n ? p->num_samples : n;
  if (k < 1 || k > SMQ_MAX_SAMPLES) {
    set_error("sampled stats need 1 <= k <= %d, got %lld", SMQ_MAX_SAMPLES, (long long)k);
    return SMQ_ERR_INVALID;
  }
  for (int j = 0; j < (int)k; ++j) {
    if (p->sample_idx[j] < 0 || p->sample_idx[j] >= n) {
      set_error("sample_idx[%d] = %lld out of range [0, %lld)", j, (long long)p->sample_idx[j],
                (long long)n);
      return SMQ_ERR_INVALID;
    }
    A.sample_idx[j] = p->sample_idx[j];
  }
  A.k = (int)k;
  A.range_coef = range_coef_for(p, k);
  return SMQ_OK;
}

static void launch_sample_stats(const ApplyArgs& A, int dtype, hipStream_t st) {
  if (dtype == SMQ_DTYPE_F32)
    hipLaunchKernelGGL(smaq_sample_stats_kernel<kF32>, dim3(1), dim3(kWave), 0, st, A);
  else if (dtype == SMQ_DTYPE_F16)
    hipLaunchKernelGGL(smaq_sample_stats_kernel<kF16>, dim3(1), dim3(kWave), 0, st, A);
  else
    hipLaunchKernelGGL(smaq_sample_stats_kernel<kBF16>, dim3(1), dim3(kWave), 0, st, A);
}

// Host side of the multi-workgroup draw: checks, memsets of the two hash sets, the three draw
// launches. Fills *A (x, statistics fields and ws_stats are the caller's).
int launch_large_draw(int64_t n, int64_t k, const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                      hipStream_t st, LargeDrawArgs* A, int* grid) {
  const LargeDrawLayout L(k);
  const size_t need = SMQ_WS_LARGE_SAMPLES_OFFSET + L.total;
  if (!ws || ws_bytes < need) {
    set_error("workspace too small for %lld device-drawn samples: need %zu bytes "
              "(smq_smaq_workspace_bytes_sampled), got %zu", (long long)k, need, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  char* r = (char*)ws + SMQ_WS_LARGE_SAMPLES_OFFSET;
  memset(A, 0, sizeof(*A));
  A->n = n;
  A->k = k;
  A->key = rng_key(p->seed ^ kDrawSalt);
  A->offset = p->offset;
  A->rng_ctr = (unsigned long long*)p->offset_counter;
  A->bits = L.bits;
  A->pick = (int64_t*)(r + L.pick);
  A->hkey = (unsigned long long*)(r + L.hkey);
  A->hdup = (uint32_t*)(r + L.hdup);
  A->h2key = (unsigned long long*)(r + L.h2key);
  A->susp = (uint32_t*)(r + L.susp);
  A->parts = (StatPartial*)(r + L.parts);
  const size_t slots = (size_t)1 << L.bits;
  fill_async(A->hkey, ~0ull, slots, st);
  fill_async(A->hdup, 0u, slots, st);
  fill_async(A->h2key, ~0ull, slots, st);
  const int g = (int)std::min<int64_t>(kDrawGridCap, (k + 4 * kBlock - 1) / (4 * kBlock));
  hipLaunchKernelGGL(smaq_draw_candidates_kernel, dim3(g), dim3(kBlock), 0, st, *A);
  hipLaunchKernelGGL(smaq_draw_suspects_kernel, dim3(g), dim3(kBlock), 0, st, *A);
  hipLaunchKernelGGL(smaq_draw_resolve_kernel, dim3(1), dim3(kWave), 0, st, *A);
  *grid = g;
  return check_launch("smaq_draw_resolve_kernel");
}

size_t large_draw_ws_bytes(int64_t k) {
  return SMQ_WS_LARGE_SAMPLES_OFFSET + LargeDrawLayout(k).total;
}

static int launch_draw_stats_large(const void* x, int dtype, int64_t n, int64_t k,
                                   const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                                   hipStream_t st) {
  LargeDrawArgs A;
  int g = 0;
  const int rc = launch_large_draw(n, k, p, ws, ws_bytes, st, &A, &g);
  if (rc) return rc;
  A.x = x;
  A.clamp_lo = p->clamp_lo;
  A.clamp_hi = p->clamp_hi;
  A.range_coef = range_coef_for(p, k);
  A.ws_stats = (SmqSmaqStats*)ws;
#define SMQ_DRAW_STATS(TIN, RANGE)                                                                  \
  do {                                                                                            \
    hipLaunchKernelGGL((smaq_draw_gather_kernel<TIN, RANGE>), dim3(g), dim3(kBlock), 0, st, A);    \
    hipLaunchKernelGGL((smaq_draw_finalize_kernel<TIN, RANGE>), dim3(1), dim3(kBlock), 0, st, A, g); \
  } while (0)
  const bool rg = p->use_range_std_dev != 0;
  if (dtype == SMQ_DTYPE_F32) { if (rg) SMQ_DRAW_STATS(kF32, true); else SMQ_DRAW_STATS(kF32, false); }
  else if (dtype == SMQ_DTYPE_F16) { if (rg) SMQ_DRAW_STATS(kF16, true); else SMQ_DRAW_STATS(kF16, false); }
  else { if (rg) SMQ_DRAW_STATS(kBF16, true); else SMQ_DRAW_STATS(kBF16, false); }
#undef SMQ_DRAW_STATS
  return check_launch("smaq_draw_finalize_kernel");
}

static int launch_draw_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p,
                             void* ws, size_t ws_bytes, hipStream_t st) {
  const int64_t k = p->num_samples < n ? p->num_samples : n;
  if (k < 1 || k > SMQ_MAX_DRAW_SAMPLES) {
    set_error("device-drawn sampled stats need 1 <= k <= %d, got %lld", SMQ_MAX_DRAW_SAMPLES,
              (long long)k);
    return SMQ_ERR_INVALID;
  }
  if (k > SMQ_MAX_DEVICE_SAMPLES) return launch_draw_stats_large(x, dtype, n, k, p, ws, ws_bytes, st);
  const size_t need = SMQ_WS_SAMPLES_OFFSET + 8 * (size_t)SMQ_MAX_DEVICE_SAMPLES;
  if (!ws || ws_bytes < need) {
    set_error("workspace too small for device-drawn samples: need %zu bytes, got %zu", need,
              ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  DrawArgs D;
  D.x = x;
  D.n = n;
  D.k = (int)k;
  D.use_range = p->use_range_std_dev;
  D.key = rng_key(p->seed ^ kDrawSalt);
  D.offset = p->offset;
  D.rng_ctr = (unsigned long long*)p->offset_counter;
  D.clamp_lo = p->clamp_lo;
  D.clamp_hi = p->clamp_hi;
  D.range_coef = range_coef_for(p, k);
  D.ws_stats = (SmqSmaqStats*)ws;
  D.idx_out = (int64_t*)((char*)ws + SMQ_WS_SAMPLES_OFFSET);
  if (dtype == SMQ_DTYPE_F32)
    hipLaunchKernelGGL(smaq_draw_stats_kernel<kF32>, dim3(1), dim3(kBlock), 0, st, D);
  else if (dtype == SMQ_DTYPE_F16)
    hipLaunchKernelGGL(smaq_draw_stats_kernel<kF16>, dim3(1), dim3(kBlock), 0, st, D);
  else
    hipLaunchKernelGGL(smaq_draw_stats_kernel<kBF16>, dim3(1), dim3(kBlock), 0, st, D);
  return check_launch("smaq_draw_stats_kernel");
}

static int launch_apply(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                        const float* uniforms, const SmqSmaqStats* stats_in, void* ws,
                        size_t ws_bytes, hipStream_t st, int def_g = 0) {
  if (!ws || ws_bytes < SmaqWsLayout::kPartials) {
    set_error("workspace too small: need >= %zu bytes", (size_t)SmaqWsLayout::kPartials);
    return SMQ_ERR_WORKSPACE;
  }
  ApplyArgs A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.y = y;
  A.n = n;
  A.uniforms = uniforms;
  A.ws_stats = (SmqSmaqStats*)ws;
  A.stats = (p->stats_source == SMQ_STATS_INJECTED) ? stats_in : (const SmqSmaqStats*)ws;
  A.thr = p->main_std_dev_threshold;
  A.r_main = p->range_main;
  A.r_out = p->range_outlier;
  A.clamp_lo = p->clamp_lo;
  A.clamp_hi = p->clamp_hi;
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  A.inv_r_main = R.inv_main;
  A.inv_r_out = R.inv_out;
  A.safe_q = R.safe_q;
  A.key = rng_key(p->seed);
  A.offset = p->offset;
  A.rng_ctr = (unsigned long long*)p->offset_counter;
  A.all_pos = p->all_positive;
  A.count = p->count_outliers;
  A.use_range = p->use_range_std_dev;
  // half inputs: the fp32 quotient form when every reachable code checks (measurement knob
  // SMQ_HALF_QF=0 keeps the fp64 form)
  static const int qf_env = [] {
    const char* e = knob_env("SMQ_HALF_QF");
    return e ? atoi(e) : 1;
  }();
  if (dtype != SMQ_DTYPE_F32 && !p->bn_gamma && !def_g && qf_env)
    A.qs = quot_split_for(dtype, A.thr, A.r_main, A.r_out,
                          p->stochastic_rounding ? kRoundHash : kRoundTrunc);
  if (def_g) {  // the statistics launch left def_g partials (launch_stats)
    A.def_parts = (const StatPartial*)((const char*)ws + SmaqWsLayout::kPartials);
    A.def_rec = (const double*)((const char*)ws + SmaqWsLayout::kDeferRec);
    A.def_g = def_g;
    A.range_coef = range_coef_for(p, n);
  }
  if (p->bn_gamma) {
    if (!p->bn_beta || p->bn_channels < 1 || p->bn_inner < 1) {
      set_error("BN variant needs bn_beta, bn_channels >= 1 and bn_inner >= 1");
      return SMQ_ERR_INVALID;
    }
    A.bn_gamma = p->bn_gamma;
    A.bn_beta = p->bn_beta;
    A.bn_channels = p->bn_channels;
    A.bn_inner = p->bn_inner;
  }
  if (p->stats_source == SMQ_STATS_INJECTED && !stats_in) {
    set_error("SMQ_STATS_INJECTED needs stats_in");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source == SMQ_STATS_SAMPLED) {
    const int rc = fill_sampled(A, p, n);
    if (rc) return rc;
  }
  const int rm = !p->stochastic_rounding ? kRoundTrunc : (uniforms ? kRoundUniform : kRoundHash);
  const bool vec = aligned(x, dtype == SMQ_DTYPE_F32 ? 16 : 8) && aligned(y, 16) &&
                   (rm != kRoundUniform || aligned(uniforms, 16)) && !A.safe_q;
  A.out_slots = (unsigned long long*)((char*)ws + SmaqWsLayout::kSlots);
  if (p->count_outliers) fill_async(A.out_slots, 0ull, SMQ_WS_OUTLIER_SLOTS, st);
  static const int rev_env = [] {
    const char* e = knob_env("SMQ_APPLY_REVERSE");
    return e ? atoi(e) : 1;
  }();
  // reverse only pays after a forward statistics sweep of the same tensor
  A.reverse = (p->stats_source == SMQ_STATS_WORKSPACE) ? rev_env : 0;
  // non-temporal loads only where they do not forfeit Infinity-Cache hits: a tensor that fits is
  // re-read from the cache (multi-tensor chunks, same policy: nt loads 86.5 vs 80.8 us per step)
  static const int64_t apply_nt_min = [] {
    const char* e = knob_env("SMQ_STATS_NT_MIN_MB");
    return (int64_t)(e ? atoll(e) : kStatsNtMinMB) << 20;
  }();
  A.nt_loads = (int64_t)(dtype == SMQ_DTYPE_F32 ? 4 : 2) * n >= apply_nt_min ? 1 : 0;
  int tv = (rm == kRoundHash && vec && !A.bn_gamma) ? sr_tile_v() : 1;
  // half inputs: 8-B loads, so twice the slots for the bytes in flight per lane of fp32. 256M,
  // interleaved rounds, ms/step (tools/half_tv.sh, tools/ab_env.sh): bf16 2 slots 0.401-0.404,
  // 4 slots 0.384-0.390; fp16 (round 3, with the fp32-reciprocal z-score, half_quot) 4 slots
  // 0.4005-0.406 vs 2 slots 0.408-0.422 (round 2, before half_quot: no gain from 4)
  static const int half_tv = [] {  // measurement knob SMQ_HALF_TV (2 | 4): both half types
    const char* e = knob_env("SMQ_HALF_TV");
    return e ? (atoi(e) == 4 ? 4 : 2) : 0;
  }();
  if (tv == 2 && dtype != SMQ_DTYPE_F32)
    tv = half_tv ? half_tv : 4;
  const int64_t tile_elems = (int64_t)kBlock * 4 * tv;
  const int64_t tiles = (n + tile_elems - 1) / tile_elems;
  if (tiles > 0x7fffffffLL) {
    set_error("tensor too large: %lld elements", (long long)n);
    return SMQ_ERR_INVALID;
  }
  const int grid = (int)tiles;
  if (p->stats_source == SMQ_STATS_INJECTED) {
    hipLaunchKernelGGL(smaq_prep_injected_kernel, dim3(1), dim3(kWave), 0, st, stats_in,
                       A.ws_stats, A.rng_ctr, n);
    A.stats = A.ws_stats;
  }
  if (p->stats_source == SMQ_STATS_SAMPLED) {
    launch_sample_stats(A, dtype, st);
    A.stats = A.ws_stats;
  }
  if (p->stats_source == SMQ_STATS_SAMPLED_DEVICE) {
    const int rc = launch_draw_stats(x, dtype, n, p, ws, ws_bytes, st);
    if (rc) return rc;
    A.stats = A.ws_stats;
  }
  const bool bn = A.bn_gamma != nullptr;
  if (dtype == SMQ_DTYPE_F32) launch_apply_t<kF32>(A, rm, vec, bn, tv, grid, st);
  else if (dtype == SMQ_DTYPE_F16) launch_apply_t<kF16>(A, rm, vec, bn, tv, grid, st);
  else launch_apply_t<kBF16>(A, rm, vec, bn, tv, grid, st);
  return check_launch("smaq_apply_kernel");
}

static int check_tensor_args(const void* x, const float* y, int64_t n) {
  if (n < 1) {
    set_error("n must be >= 1 (got %lld); the caller passes n < min_size through", (long long)n);
    return SMQ_ERR_INVALID;
  }
  if (!x || !y) {
    set_error("x and y must be device pointers");
    return SMQ_ERR_INVALID;
  }
  return SMQ_OK;
}

// Statistics for a consumer other than the apply kernel (the packed codec): full or sampled
// statistics of x into the workspace header (smaq_host.h).
int prepare_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                  size_t ws_bytes, hipStream_t st, uint32_t* zero, uint32_t zero_n, bool* zeroed) {
  if (zeroed) *zeroed = false;
  if (p->stats_source == SMQ_STATS_WORKSPACE) {
    if (zeroed) *zeroed = zero != nullptr;
    return launch_stats(x, dtype, n, p, ws, ws_bytes, st, nullptr, nullptr, zero, zero_n);
  }
  if (p->stats_source == SMQ_STATS_SAMPLED_DEVICE)
    return launch_draw_stats(x, dtype, n, p, ws, ws_bytes, st);
  if (p->stats_source != SMQ_STATS_SAMPLED) {
    set_error("this entry point computes its statistics (SMQ_STATS_WORKSPACE or _SAMPLED*)");
    return SMQ_ERR_INVALID;
  }
  if (!ws || ws_bytes < SmaqWsLayout::kPartials) {
    set_error("workspace too small: need >= %zu bytes", (size_t)SmaqWsLayout::kPartials);
    return SMQ_ERR_WORKSPACE;
  }
  ApplyArgs A;
  memset(&A, 0, sizeof(A));
  A.x = x;
  A.n = n;
  A.ws_stats = (SmqSmaqStats*)ws;
  A.clamp_lo = p->clamp_lo;
  A.clamp_hi = p->clamp_hi;
  A.use_range = p->use_range_std_dev;
  A.rng_ctr = (unsigned long long*)p->offset_counter;
  const int rc = fill_sampled(A, p, n);
  if (rc) return rc;
  launch_sample_stats(A, dtype, st);
  return check_launch("smaq_sample_stats_kernel");
}

size_t smaq_stats_ws_bytes(int64_t n) { return stats_ws_bytes(n); }
int stats_into(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
               size_t ws_bytes, hipStream_t st, SmqSmaqStats* out) {
  return launch_stats(x, dtype, n, p, ws, ws_bytes, st, nullptr, out);
}
int smaq_validate(const SmqSmaqParams* p, int dtype) {
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  return rc;
}

}  // namespace smq

using namespace smq;

extern "C" {

int smq_abi_version(void) { return SMQ_ABI_VERSION; }
const char* smq_last_error(void) { return g_err; }

uint32_t smq_rng_u32(uint64_t seed, uint64_t counter) { return rng_u32(rng_key(seed), counter); }
uint32_t smq_smaq_u24(uint64_t seed, uint64_t counter) { return smaq_u24(rng_key(seed), counter); }

int smq_half_quot_split(int dtype, float thr, float r_main, float r_out, int stochastic_rounding,
                        float* out) {
  if (dtype != SMQ_DTYPE_F16 && dtype != SMQ_DTYPE_BF16) return 0;
  const QuotSplit s = quot_split_compute(dtype, thr, r_main, r_out,
                                         stochastic_rounding ? kRoundHash : kRoundTrunc);
  if (out) {
    out[0] = s.hm;
    out[1] = s.lm;
    out[2] = s.ho;
    out[3] = s.lo;
  }
  return s.ok;
}

void smq_smaq_params_init(SmqSmaqParams* p) {
  memset(p, 0, sizeof(*p));
  smq_smaq_params_set(p, 6, 8, 1.0, 2.5, 32);
  p->stochastic_rounding = 1;
  p->num_samples = 16;
  p->stats_source = SMQ_STATS_WORKSPACE;
  p->range_std_coef = -1.0f;  // library computes the fp32 coefficient
}

int smq_smaq_params_set(SmqSmaqParams* p, int num_bits_main, int num_bits_outlier,
                        double main_thr, double outlier_thr, int precision) {
  if (!p) {
    set_error("params is NULL");
    return SMQ_ERR_INVALID;
  }
  if (main_thr == 0.0 || outlier_thr - main_thr == 0.0) {
    set_error("thresholds give a division by zero (smart.py:72-78)");
    return SMQ_ERR_INVALID;
  }
  p->num_bits_main = num_bits_main;
  p->num_bits_outlier = num_bits_outlier;
  p->main_std_dev_threshold = (float)main_thr;
  // Python: ((2 ** (bits - 2)) - 1) / threshold, in double, rounded to fp32 when used.
  p->range_outlier = (float)((pow(2.0, num_bits_outlier - 2) - 1.0) / (outlier_thr - main_thr));
  p->range_main = (float)((pow(2.0, num_bits_main - 2) - 1.0) / main_thr);
  p->clamp_lo = precision == 16 ? 1e-4f : 1e-38f;
  p->clamp_hi = precision == 16 ? 1e4f : 1e38f;
  p->main_std_dev_threshold_f64 = main_thr;
  p->clamp_lo_f64 = precision == 16 ? 1e-4 : 1e-38;
  p->clamp_hi_f64 = precision == 16 ? 1e4 : 1e38;
  p->range_std_coef_f64 = -1.0;
  return SMQ_OK;
}

int smq_smaq_draw_samples(SmqSmaqParams* p, int64_t n, int num_samples) {
  if (!p || n < 1 || num_samples < 1) {
    set_error("draw_samples: bad arguments");
    return SMQ_ERR_INVALID;
  }
  const int64_t k = num_samples < n ? num_samples : n;
  if (k > SMQ_MAX_SAMPLES) {
    set_error("num_samples %d exceeds SMQ_MAX_SAMPLES", num_samples);
    return SMQ_ERR_INVALID;
  }
  // Floyd's algorithm, the draw smaq_draw_stats_kernel performs at stream position p->offset
  const uint32_t key = rng_key(p->seed ^ kDrawSalt);
  for (int i = 0; i < (int)k; ++i) {
    int64_t t = floyd_candidate(key, p->offset, n, (int)k, i);
    for (int q = 0; q < i; ++q)
      if (p->sample_idx[q] == t) {
        t = n - k + i;
        break;
      }
    p->sample_idx[i] = t;
  }
  p->num_samples = (int32_t)k;
  return SMQ_OK;
}

size_t smq_smaq_workspace_bytes(int64_t n) { return stats_ws_bytes(n); }

size_t smq_smaq_workspace_bytes_sampled(int64_t n, int64_t num_samples) {
  static_assert(SMQ_WS_LARGE_SAMPLES_OFFSET >= SmaqWsLayout::kTagCounters + 8 * SmaqWsLayout::kTagWords,
                "smq.h SMQ_WS_LARGE_SAMPLES_OFFSET overlaps the fixed layout");
  const int64_t k = num_samples < n ? num_samples : n;
  if (k <= SMQ_MAX_DEVICE_SAMPLES) return stats_ws_bytes(n);
  if (k > SMQ_MAX_DRAW_SAMPLES) return 0;
  return large_draw_ws_bytes(k);
}

int smq_smaq_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                   size_t ws_bytes, void* stream) {
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  if (rc) return rc;
  if (n < 1 || !x) {
    set_error("stats: n must be >= 1 and x non-NULL");
    return SMQ_ERR_INVALID;
  }
  return launch_stats(x, dtype, n, p, ws, ws_bytes, (hipStream_t)stream);
}

int smq_smaq_apply(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                   const float* uniforms, const SmqSmaqStats* stats_in, void* ws, size_t ws_bytes,
                   void* stream) {
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  if (!rc) rc = check_tensor_args(x, y, n);
  if (rc) return rc;
  return launch_apply(x, dtype, y, n, p, uniforms, stats_in, ws, ws_bytes, (hipStream_t)stream);
}

// Deferred statistics need the vector apply body without the BN term (defer_consts).
static bool defer_eligible(const void* x, int dtype, const float* y, int64_t n,
                           const SmqSmaqParams* p, const float* uniforms) {
  static const int64_t max_n = [] {  // measurement knob SMQ_DEFER_MAX_N (elements; 0 = off)
    const char* e = knob_env("SMQ_DEFER_MAX_N");
    return e ? (int64_t)atoll(e) : kDeferMaxN;
  }();
  if (n > max_n || p->bn_gamma) return false;
  if (!aligned(x, dtype == SMQ_DTYPE_F32 ? 16 : 8) || !aligned(y, 16)) return false;
  if (p->stochastic_rounding && uniforms && !aligned(uniforms, 16)) return false;
  return !range_recips(p->range_main, p->range_outlier).safe_q;
}

// The single launch (smaq_fused.hip) needs the vector body without the BN term, the in-kernel
// random draws and its workspace region.
static bool fused_eligible(const void* x, int dtype, const float* y, int64_t n,
                           const SmqSmaqParams* p, const float* uniforms, size_t ws_bytes) {
  static const bool on = [] {  // measurement knob SMQ_FUSED=0: the two-launch paths
    const char* e = knob_env("SMQ_FUSED");
    return e ? atoi(e) != 0 : true;
  }();
  if (!on || n < 4 || n > kSmallMaxN || p->bn_gamma) return false;
  if (p->stochastic_rounding && uniforms) return false;
  if (ws_bytes < SmaqWsLayout::kTotal) return false;
  if (!aligned(x, dtype == SMQ_DTYPE_F32 ? 16 : 8) || !aligned(y, 16)) return false;
  return !range_recips(p->range_main, p->range_outlier).safe_q;
}

int smq_smaq_roundtrip_ex(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                          const float* uniforms, void* ws, size_t ws_bytes, uint32_t flags,
                          void* stream) {
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  if (!rc) rc = check_tensor_args(x, y, n);
  if (rc) return rc;
  if (flags & ~(SMQ_SMAQ_SPLIT | SMQ_SMAQ_NO_DEFER | SMQ_SMAQ_TEST_LATE)) {
    set_error("roundtrip: unknown flags 0x%x", flags);
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source == SMQ_STATS_WORKSPACE && !(flags & (SMQ_SMAQ_SPLIT | SMQ_SMAQ_NO_DEFER)) &&
      ws && fused_eligible(x, dtype, y, n, p, uniforms, ws_bytes)) {
    const RangeRecips R = range_recips(p->range_main, p->range_outlier);
    FusedCall c{x, dtype, y, n, p, range_coef_for(p, n), R.inv_main, R.inv_out, ws,
                (flags & SMQ_SMAQ_TEST_LATE) ? 1 : 0, ws_bytes};
    return launch_fused(c, (hipStream_t)stream);
  }
  int def_g = 0;
  if (p->stats_source == SMQ_STATS_WORKSPACE) {
    const bool defer = !(flags & SMQ_SMAQ_NO_DEFER) && defer_eligible(x, dtype, y, n, p, uniforms);
    rc = launch_stats(x, dtype, n, p, ws, ws_bytes, (hipStream_t)stream,
                      defer ? &def_g : nullptr);
    if (rc) return rc;
  } else if (p->stats_source == SMQ_STATS_INJECTED) {
    set_error("roundtrip: use smq_smaq_apply for injected statistics");
    return SMQ_ERR_INVALID;
  }
  return launch_apply(x, dtype, y, n, p, uniforms, nullptr, ws, ws_bytes, (hipStream_t)stream,
                      def_g);
}

int smq_smaq_roundtrip(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                       const float* uniforms, void* ws, size_t ws_bytes, void* stream) {
  return smq_smaq_roundtrip_ex(x, dtype, y, n, p, uniforms, ws, ws_bytes, 0u, stream);
}

// --measure_compression_ratio on the device (smart.py:184-188, base.py:72-102): the single launch
// counts into the caller's zeroed record and its last workgroup writes the values; every other path
// counts into the workspace slots, then smaq_size_metrics_kernel reads them.
int smq_smaq_roundtrip_counted(const void* x, int dtype, float* y, int64_t n,
                               const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                               SmqSizeRecord* rec, void* stream) {
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  if (!rc) rc = check_tensor_args(x, y, n);
  if (rc) return rc;
  if (!rec) {
    set_error("roundtrip_counted: rec must be a device pointer");
    return SMQ_ERR_INVALID;
  }
  SmqSmaqParams q = *p;
  q.count_outliers = 1;
  if (q.stats_source == SMQ_STATS_WORKSPACE && ws && fused_eligible(x, dtype, y, n, &q, nullptr,
                                                                   ws_bytes)) {
    const RangeRecips R = range_recips(q.range_main, q.range_outlier);
    FusedCall c{x, dtype, y, n, &q, range_coef_for(&q, n), R.inv_main, R.inv_out, ws, 0, ws_bytes};
    c.rec = rec;
    return launch_fused(c, (hipStream_t)stream);
  }
  rc = smq_smaq_roundtrip_ex(x, dtype, y, n, &q, nullptr, ws, ws_bytes, 0u, stream);
  if (rc) return rc;
  return smq_smaq_size_metrics(ws, n, q.num_bits_main, q.num_bits_outlier, rec, stream);
}

}  // extern "C"

namespace smq {

// n_out = the sum of `slots` uint64 counts (one wave); the log_size values into rec.
__global__ __launch_bounds__(kWave) void smaq_size_metrics_kernel(
    const unsigned long long* __restrict__ slots, int nslots, int64_t n, int bm, int bo,
    SmqSizeRecord* rec) {
  unsigned long long v = 0;
  for (int i = threadIdx.x; i < nslots; i += kWave) v += slots[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  if (threadIdx.x == 0) {
    const double no = (double)v;
    const double ns = no * (double)bo + (double)(n - (int64_t)v) * (double)bm;
    const double orig = 32.0 * (double)n;
    rec->n_outlier = no;
    rec->new_size = ns;
    rec->compression_ratio = orig / ns;
    rec->orig_size = orig;
  }
}

// Multi-tensor call: tensor t's n_outlier from its statistics record, one thread per tensor.
__global__ __launch_bounds__(256) void smaq_multi_size_metrics_kernel(
    const SmqSmaqStats* __restrict__ st, const int64_t* __restrict__ n, int count, int bm, int bo,
    double* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= count) return;
  const unsigned long long v = st[t].n_outlier;
  const int64_t nt = n[t];
  const double no = (double)v;
  const double ns = no * (double)bo + (double)(nt - (int64_t)v) * (double)bm;
  const double orig = 32.0 * (double)nt;
  out[4 * t] = no;
  out[4 * t + 1] = ns;
  out[4 * t + 2] = orig / ns;
  out[4 * t + 3] = orig;
}

}  // namespace smq

extern "C" {

int smq_smaq_size_metrics(const void* ws, int64_t n, int num_bits_main, int num_bits_outlier,
                          SmqSizeRecord* rec, void* stream) {
  if (!ws || !rec || n < 1) {
    set_error("size_metrics: ws and rec must be device pointers, n >= 1");
    return SMQ_ERR_INVALID;
  }
  hipLaunchKernelGGL(smaq_size_metrics_kernel, dim3(1), dim3(kWave), 0, (hipStream_t)stream,
                     (const unsigned long long*)((const char*)ws + SmaqWsLayout::kSlots),
                     (int)SMQ_WS_OUTLIER_SLOTS, n, num_bits_main, num_bits_outlier, rec);
  return check_launch("smaq_size_metrics_kernel");
}

int smq_smaq_multi_size_metrics(const void* ws, const int64_t* n, int count, int num_bits_main,
                                int num_bits_outlier, double* out, void* stream) {
  if (count < 0 || (count > 0 && (!ws || !n || !out))) {
    set_error("multi_size_metrics: ws, n and out must be device pointers");
    return SMQ_ERR_INVALID;
  }
  if (count == 0) return SMQ_OK;
  hipLaunchKernelGGL(smaq_multi_size_metrics_kernel, dim3((unsigned)((count + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, (const SmqSmaqStats*)ws, n, count,
                     num_bits_main, num_bits_outlier, out);
  return check_launch("smaq_multi_size_metrics_kernel");
}

int smq_smaq_stats_f32(const float* x, int64_t n, const SmqSmaqParams* p, void* ws,
                       size_t ws_bytes, void* stream) {
  return smq_smaq_stats(x, SMQ_DTYPE_F32, n, p, ws, ws_bytes, stream);
}

int smq_smaq_apply_f32(const float* x, float* y, int64_t n, const SmqSmaqParams* p,
                       const float* uniforms, const SmqSmaqStats* stats_in, void* ws,
                       size_t ws_bytes, void* stream) {
  return smq_smaq_apply(x, SMQ_DTYPE_F32, y, n, p, uniforms, stats_in, ws, ws_bytes, stream);
}

int smq_smaq_roundtrip_f32(const float* x, float* y, int64_t n, const SmqSmaqParams* p,
                           const float* uniforms, void* ws, size_t ws_bytes, void* stream) {
  return smq_smaq_roundtrip(x, SMQ_DTYPE_F32, y, n, p, uniforms, ws, ws_bytes, stream);
}

}  // extern "C"

namespace smq {

int roundtrip_pack_fused(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                         void* ws, size_t ws_bytes, const FusedPackCall& k, hipStream_t st) {
  static const bool on = [] {  // measurement knob SMQ_FUSED_PACK=0: the round trip + packer launches
    const char* e = knob_env("SMQ_FUSED_PACK");
    return e ? atoi(e) != 0 : true;
  }();
  if (!on || p->stats_source != SMQ_STATS_WORKSPACE || !ws ||
      !fused_eligible(x, dtype, y, n, p, nullptr, ws_bytes))
    return kFusedPackDeclined;
  const RangeRecips R = range_recips(p->range_main, p->range_outlier);
  FusedCall c{x, dtype, y, n, p, range_coef_for(p, n), R.inv_main, R.inv_out, ws, 0, ws_bytes};
  return launch_fused_pack(c, k, st);
}

int roundtrip_for_pack(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                       void* ws, size_t ws_bytes, hipStream_t st, uint32_t* zero, uint32_t zero_n,
                       bool* zeroed) {
  *zeroed = false;
  int rc = validate_params(p);
  if (!rc) rc = check_dtype(dtype);
  if (!rc) rc = check_tensor_args(x, y, n);
  if (rc) return rc;
  if (p->stats_source == SMQ_STATS_INJECTED) {
    set_error("roundtrip_compress: statistics must be computed (not SMQ_STATS_INJECTED)");
    return SMQ_ERR_INVALID;
  }
  if (p->stats_source == SMQ_STATS_WORKSPACE && ws &&
      fused_eligible(x, dtype, y, n, p, nullptr, ws_bytes)) {
    // the single launch: its workgroup 0 writes the record to the header and clears `zero`
    const RangeRecips R = range_recips(p->range_main, p->range_outlier);
    FusedCall c{x, dtype, y, n, p, range_coef_for(p, n), R.inv_main, R.inv_out, ws, 0, ws_bytes,
                zero, zero_n};
    *zeroed = zero != nullptr;
    return launch_fused(c, st);
  }
  if (p->stats_source == SMQ_STATS_WORKSPACE) {  // finalised into the header, never deferred
    rc = launch_stats(x, dtype, n, p, ws, ws_bytes, st, nullptr, nullptr, zero, zero_n);
    if (rc) return rc;
    *zeroed = zero != nullptr;
  }
  return launch_apply(x, dtype, y, n, p, nullptr, nullptr, ws, ws_bytes, st);
}

}  // namespace smq
