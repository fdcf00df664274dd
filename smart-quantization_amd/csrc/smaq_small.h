// smaq_small.h — the statistics partition of SmaQ tensors up to kSmallMaxN elements, shared by the
// single-launch round trip (smaq_fused.hip smaq_fused_kernel), the statistics launch of the
// two-launch paths (smaq_fused.hip smaq_stats_small_kernel) and the multi-tensor statistics
// (smaq_multi.hip), so that every path computes the same fp64 partials and totals bit for bit.
// Reference: smart_compress/compress/smart.py:100-108, 130-134 (data.mean(), data.std()).
//
// The partition is a function of n alone:
//   float4 groups j (elements 4j .. 4j+3), nv = n / 4;
//   V = ceil(nv / (kSmallMaxG * kSmallT)) groups per lane (1 .. kSmallMaxV);
//   G = ceil(nv / (V * kSmallT)) partials (<= kSmallMaxG).
// Partial b is the sum over kSmallT "lanes": lane t holds the groups (b V + u) kSmallT + t,
// u = 0 .. V-1 (those < nv), and in partial G-1 lane t < n % 4 also element 4 nv + t. Per lane:
// four fp64 chains of shifted sums (StatAcc::add, one chain per group component, in u order; the
// tail element last, on chain 0), lane value (c0 + c1) + (c2 + c3); per wave of 64 lanes the
// ascending DPP butterfly (wave_sum_asc); the 16 wave values combined as
//   S = 0; for w = 0, 4, 8, 12: S += (v[w] + v[w+1]) + (v[w+2] + v[w+3]).
// min / max are order-free (fminf / fmaxf, NaN ignored like the big sweep). The totals are then
// reduce_partials_w0's order over the G partials (smaq.hip), or the partial itself when G == 1.
// Every path computes a partial with a 1024-thread workgroup, thread t = lane t.
#pragma once

#include "smaq_elem.h"

namespace smq {

constexpr int kSmallT = 1024;    // lanes per partial (threads of the native workgroup)
constexpr int kSmallMaxV = 8;    // float4 groups per lane (registers of the single launch)
constexpr int kSmallMaxG = 256;  // partials (four per lane of reduce_partials_w0's wave)
constexpr int64_t kSmallMaxN = (int64_t)kSmallMaxG * kSmallT * kSmallMaxV * 4 + 3;  // 8,388,611
constexpr int kSmallWaves = kSmallT / kWave;

struct SmallGeom {
  int V, G;
};

__host__ __device__ __forceinline__ SmallGeom small_geom(int64_t n) {
  const int64_t nv = n >> 2;
  const int64_t per_v = (int64_t)kSmallMaxG * kSmallT;
  int64_t V = (nv + per_v - 1) / per_v;
  if (V < 1) V = 1;
  const int64_t G = nv > 0 ? (nv + V * kSmallT - 1) / (V * kSmallT) : 1;
  return SmallGeom{(int)V, (int)G};
}

// The shift of the shifted sums (every statistics path): median of x[0], x[n/2], x[n-1].
template <int TIN>
__device__ __forceinline__ double stats_shift(const void* x, int64_t n) {
  const float k0 = load1<TIN>(x, 0), k1 = load1<TIN>(x, n >> 1), k2 = load1<TIN>(x, n - 1);
  return (double)fmaxf(fminf(k0, k1), fminf(fmaxf(k0, k1), k2));
}

// One float4 group from memory: 16-B (fp32) / 8-B (half) load when x is aligned for it, else four
// element loads (the same values).
template <int TIN>
__device__ __forceinline__ float4 small_group(const void* x, int64_t j, bool vec) {
  if (vec) return load4<TIN>(x, j);
  return make_float4(load1<TIN>(x, 4 * j), load1<TIN>(x, 4 * j + 1), load1<TIN>(x, 4 * j + 2),
                     load1<TIN>(x, 4 * j + 3));
}

// The V float4 groups of lane t of partial b from memory (every load in flight before any is used).
template <int TIN, int MAXV>
__device__ __forceinline__ void small_lane_load(const void* x, int64_t n, int V, int b, int t,
                                                bool vec, float4 (&g)[MAXV]) {
  const int64_t nv = n >> 2;
  const int64_t base = (int64_t)b * V * kSmallT + t;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    const int64_t j = base + (int64_t)u * kSmallT;
    if (u < V && j < nv) g[u] = small_group<TIN>(x, j, vec);
  }
}

// The lane value of lane t of partial b from its groups g (entries past nv ignored).
template <int TIN, int MAXV, bool RANGE = true>
__device__ __forceinline__ StatAcc small_lane_sum(const void* x, int64_t n, int V, int G, int b,
                                                  int t, const float4 (&g)[MAXV], double shift) {
  const int64_t nv = n >> 2;
  const int64_t base = (int64_t)b * V * kSmallT + t;
  StatAcc c0, c1, c2, c3;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    if (u >= V) break;
    if (base + (int64_t)u * kSmallT >= nv) continue;
    c0.add<RANGE>(g[u].x, shift);
    c1.add<RANGE>(g[u].y, shift);
    c2.add<RANGE>(g[u].z, shift);
    c3.add<RANGE>(g[u].w, shift);
  }
  if (b == G - 1 && t < (int)(n & 3)) c0.add<RANGE>(load1<TIN>(x, (nv << 2) + t), shift);
  StatAcc r;
  r.s1 = (c0.s1 + c1.s1) + (c2.s1 + c3.s1);
  r.s2 = (c0.s2 + c1.s2) + (c2.s2 + c3.s2);
  r.mn = fminf(fminf(c0.mn, c1.mn), fminf(c2.mn, c3.mn));
  r.mx = fmaxf(fmaxf(c0.mx, c1.mx), fmaxf(c2.mx, c3.mx));
  return r;
}

// The same value with one group in flight at a time (few registers: the single launch's rare
// path that computes a missing partial while its own registers stay live).
template <int TIN>
__device__ __forceinline__ StatAcc small_lane_seq(const void* x, int64_t n, int V, int G, int b,
                                                  int t, double shift, bool vec = true) {
  const int64_t nv = n >> 2;
  const int64_t base = (int64_t)b * V * kSmallT + t;
  StatAcc c0, c1, c2, c3;
#pragma unroll 1
  for (int u = 0; u < V; ++u) {
    const int64_t j = base + (int64_t)u * kSmallT;
    if (j >= nv) break;
    const float4 g = small_group<TIN>(x, j, vec);
    c0.add<true>(g.x, shift);
    c1.add<true>(g.y, shift);
    c2.add<true>(g.z, shift);
    c3.add<true>(g.w, shift);
  }
  if (b == G - 1 && t < (int)(n & 3)) c0.add<true>(load1<TIN>(x, (nv << 2) + t), shift);
  StatAcc r;
  r.s1 = (c0.s1 + c1.s1) + (c2.s1 + c3.s1);
  r.s2 = (c0.s2 + c1.s2) + (c2.s2 + c3.s2);
  r.mn = fminf(fminf(c0.mn, c1.mn), fminf(c2.mn, c3.mn));
  r.mx = fmaxf(fmaxf(c0.mx, c1.mx), fmaxf(c2.mx, c3.mx));
  return r;
}

template <int TIN, int MAXV>
__device__ __forceinline__ StatAcc small_lane(const void* x, int64_t n, int V, int G, int b, int t,
                                              bool vec, double shift) {
  float4 g[MAXV];
  small_lane_load<TIN, MAXV>(x, n, V, b, t, vec, g);
  return small_lane_sum<TIN, MAXV>(x, n, V, G, b, t, g, shift);
}

// Wave value of 64 lane values (every lane gets it); the extrema only with range-std (their
// reduction order does not matter, so any path may skip or compute them).
__device__ __forceinline__ StatAcc small_wave(StatAcc a, bool range = true) {
  a.s1 = wave_sum_asc(a.s1);
  a.s2 = wave_sum_asc(a.s2);
  if (range) {
    a.mn = wave_min_dpp(a.mn);
    a.mx = wave_max_dpp(a.mx);
  }
  return a;
}

// LDS of the 16 wave values of one partial.
struct SmallWaveLds {
  double s1[kSmallWaves], s2[kSmallWaves];
  float mn[kSmallWaves], mx[kSmallWaves];
};

__device__ __forceinline__ StatAcc small_combine(const SmallWaveLds& w) {
  StatAcc r;
#pragma unroll
  for (int i = 0; i < kSmallWaves; i += 4) {
    r.s1 += (w.s1[i] + w.s1[i + 1]) + (w.s1[i + 2] + w.s1[i + 3]);
    r.s2 += (w.s2[i] + w.s2[i + 1]) + (w.s2[i + 2] + w.s2[i + 3]);
    r.mn = fminf(r.mn, fminf(fminf(w.mn[i], w.mn[i + 1]), fminf(w.mn[i + 2], w.mn[i + 3])));
    r.mx = fmaxf(r.mx, fmaxf(fmaxf(w.mx[i], w.mx[i + 1]), fmaxf(w.mx[i + 2], w.mx[i + 3])));
  }
  return r;
}

// The 4 / V partials b0 .. (those < G) of a tensor with V <= 4 by a 1024-thread workgroup, the
// native partial shape (thread t = lane t: smaq_stats_small_kernel's lane function and wave
// butterfly, one butterfly per wave and partial), every load of the run in flight at once (4 float4
// per thread): partial b0 + p's 16 wave values in W[p]; valid after the trailing barrier.
template <int TIN, int V, bool RANGE>
__device__ __forceinline__ void small_waves_1024_runs(const void* x, int64_t n, int G, int b0,
                                                      bool vec, double shift, SmallWaveLds* W) {
  static_assert(V >= 1 && V <= 4, "runs of partials: V <= 4");
  constexpr int P = 4 / V;
  const int wave = threadIdx.x / kWave, l = threadIdx.x & (kWave - 1);
  float4 g[P][V];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if (b0 + p >= G) break;
    small_lane_load<TIN, V>(x, n, V, b0 + p, threadIdx.x, vec, g[p]);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if (b0 + p >= G) break;
    const StatAcc w = small_wave(
        small_lane_sum<TIN, V, RANGE>(x, n, V, G, b0 + p, threadIdx.x, g[p], shift), RANGE);
    if (l == 0) {
      W[p].s1[wave] = w.s1;
      W[p].s2[wave] = w.s2;
      W[p].mn[wave] = w.mn;
      W[p].mx[wave] = w.mx;
    }
  }
  __syncthreads();
}

// Partial b0 alone the same way with one group per lane in flight (small_lane_seq: few registers;
// for V > 4 where holding all V groups would spill at two 1024-thread workgroups per CU).
template <int TIN, bool RANGE>
__device__ __forceinline__ void small_waves_1024_seq(const void* x, int64_t n, int V, int G, int b0,
                                                     bool vec, double shift, SmallWaveLds* W) {
  const int wave = threadIdx.x / kWave, l = threadIdx.x & (kWave - 1);
  const StatAcc w =
      small_wave(small_lane_seq<TIN>(x, n, V, G, b0, threadIdx.x, shift, vec), RANGE);
  if (l == 0) {
    W[0].s1[wave] = w.s1;
    W[0].s2[wave] = w.s2;
    W[0].mn[wave] = w.mn;
    W[0].mx[wave] = w.mx;
  }
  __syncthreads();
}

// Wave-0 reduction of g <= kSmallMaxG statistics partials in ONE fixed order: lane l sums
// partials 4l, 4l + 1, 4l + 2, 4l + 3 in that order (from 0.0), then the ascending DPP butterfly. Used by the
// deferred path (every apply workgroup, plain loads: the partials come from an earlier launch) and by
// the last statistics workgroup of a grid of <= kDeferMaxG (sc1 loads: same launch), so both give
// the same fp64 totals bit for bit. Every load is issued before any is consumed. Call from wave 0
// (all 64 lanes); the result is wave-uniform.
template <bool SC1>
__device__ __forceinline__ void reduce_partials_w0(const StatPartial* parts, int g, bool range,
                                                   double& s1, double& s2, float& mn, float& mx) {
  constexpr int K = kSmallMaxG / kWave;
  const int l = threadIdx.x & (kWave - 1);
  double2 sv[K];
  float2 mv[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int b = K * l + i;
    if (b < g) {
      if (SC1) {
        sv[i].x = ld_sc1_f64(&parts[b].s1);
        sv[i].y = ld_sc1_f64(&parts[b].s2);
        if (range) ld_sc1_f32x2(&parts[b].mn, mv[i].x, mv[i].y);
      } else {
        sv[i] = *reinterpret_cast<const double2*>(&parts[b].s1);
        if (range) mv[i] = *reinterpret_cast<const float2*>(&parts[b].mn);
      }
    }
  }
  s1 = 0.0;
  s2 = 0.0;
  mn = INFINITY;
  mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    if (K * l + i < g) {
      s1 += sv[i].x;
      s2 += sv[i].y;
      if (range) {
        mn = fminf(mn, mv[i].x);
        mx = fmaxf(mx, mv[i].y);
      }
    }
  }
  s1 = wave_sum_asc(s1);
  s2 = wave_sum_asc(s2);
  if (range) {
    mn = wave_min(mn);
    mx = wave_max(mx);
  }
}

// ---- host side (smaq_fused.hip) --------------------------------------------------------------------
// Statistics launch of a tensor of n <= kSmallMaxN elements in this partition (one 1024-thread
// workgroup per partial). defer: leave the G partials (and {shift, stream position}) for a deferring
// apply launch, *def_g = G (0 when G == 1 finalised the header itself); else the last workgroup
// reduces them (reduce_partials_w0) into the header.
int launch_stats_small(const void* x, int dtype, int64_t n, bool vec, bool range,
                       const FinalizeArgs& fin, void* ws, hipStream_t st, bool defer, int* def_g);

// The single-launch round trip (smaq_fused_kernel); the caller checked eligibility (smaq.hip).
struct FusedCall {
  const void* x;
  int dtype;
  float* y;
  int64_t n;
  const SmqSmaqParams* p;
  float range_coef;
  double inv_r_main, inv_r_out;
  void* ws;
  int test_late;
  size_t ws_bytes;
  uint32_t* zero = nullptr;  // words the launch clears (the packer's group sums), or NULL
  uint32_t zero_n = 0;
  SmqSizeRecord* rec = nullptr;  // smq_smaq_roundtrip_counted: count into it, last workgroup
                                 // writes the log_size values (no fill, no extra launch)
};
int launch_fused(const FusedCall& c, hipStream_t st);

// The single launch that also writes the call's packed stream (smq_smaq_roundtrip_compress,
// smaq_fused.hip PACK): the stream's regions (include/smq.h "Packed SmaQ container").
struct FusedPackCall {
  SmqPackedHeader* hdr;
  uint64_t* dir;
  uint32_t* fixed;
  uint32_t* var;
  uint64_t cap_words;  // words of the variable region the buffer holds
  uint32_t n_blocks, flags;
  uint32_t* notify;     // total_bytes also here (smq_smaq_roundtrip_compress_notify), or NULL
};
constexpr int kFusedPackDeclined = 1;  // not this call's shape: nothing launched
int launch_fused_pack(const FusedCall& c, const FusedPackCall& k, hipStream_t st);

}  // namespace smq
