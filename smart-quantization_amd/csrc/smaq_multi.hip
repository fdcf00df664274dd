// smaq_multi.hip — SmaQ over a list of tensors in two launches (gfx950).
//
// Reference: the per-parameter SmartFP calls of smart_compress/util/pytorch/optimizer.py:79-127
// (grads, weights, momenta), each of which runs smart.py:110-190 separately (~24 ATen launches
// + 1 host sync per tensor; a ResNet-34 step has 148 such tensors, median 256 elements).
//
// Design: a multi call computes, per tensor, EXACTLY what a single-tensor call computes — the same
// statistics partials, reduced in the same order, the same element transform at the same counter
// offsets — so its outputs equal the per-tensor calls' bit for bit by construction.
//   statistics of tensors up to kSmallMaxN elements (smaq_small.h): one launch for all of them; a
//            workgroup computes a run of consecutive partials of one tensor (each the 1024-lane
//            partial of the single-tensor partition, emulated with four lanes per thread), stores
//            them and arrives on the tensor's counter; the tensor's last workgroup reduces its
//            partials in reduce_partials_w0's order and finalises.
//   statistics of larger tensors: the single-tensor statistics launch itself (smaq.hip
//            launch_stats), one per such tensor, into the tensor's record.
//   apply: per 4096-element chunk, the tensor's SmqSmaqStats + the element transform of smaq.hip,
//            RNG counter = params.offset + desc.rng_offset + element index (so a multi call equals
//            the sequence of single-tensor calls at those offsets, and a plan is reusable).
// y may alias x: every element is read once by the apply launch before it is written.
//
// Statistics variants (params): full (the statistics launch above; with --use_range_std_dev it also
// carries min / max), or SMQ_STATS_SAMPLED_DEVICE: one workgroup per tensor draws its k indices
// (Floyd, smaq_elem.h draw_sample_stats) at position offset + snapshot + desc.rng_offset — the
// draw a single-tensor call at that offset makes — instead of the sweep. Input element types:
// fp32, fp16, bf16 (one per call; outputs fp32 like the single-tensor path, so y may alias x only
// for fp32).
#include <stdlib.h>
#include <string.h>

#include "smq_common.h"
#include "smaq_elem.h"
#include "smaq_host.h"
#include "smaq_small.h"

namespace smq {

// Elements per workgroup, separately for the two launches (knobs SMQ_MULTI_CHUNK / _STATS_CHUNK,
// multiples of 4096). Measured on the ResNet-34 set (42.5M elements, 148 tensors): the statistics
// launch wants few, long chunks (each chunk's partial hand-off is a store-drain + atomic round
// trip: 8K chunks 62 us, 32K chunks 34 us; with the next 16 KiB step prefetched, r04: 32K 32.6 us,
// 64K 30.7 us, 128K 38.3 us), the apply launch wants many short ones (8K 60 us, 32K 80 us; with
// sc0 sc1 nt output stores the whole step: 4K 79.9 us, 8K 82.3 us). A statistics workgroup takes
// as many whole partials of its tensor as fit its chunk (at least one).
constexpr int64_t kDefaultChunk = 4096;
// workspace region of the single-tensor statistics launches of the large tensors
constexpr size_t kBigWsBytes = (SmaqWsLayout::kTagCounters + 8 * SmaqWsLayout::kTagWords + 255) &
                               ~(size_t)255;
constexpr size_t kSnapBytes = 64;  // workspace slot: the call's random-stream snapshot

struct MultiHeader {
  int32_t count;
  int32_t n_chunks;       // apply chunks
  int64_t chunk;
  int32_t n_stat_chunks;  // statistics chunks (their records follow the apply chunk records)
  int32_t n_partials;     // statistics partials of the small tensors
  int64_t stat_chunk;
};

// Everything one workgroup needs, in ONE 64-B record (uniform per workgroup -> two s_load_dwordx8):
// no dependent descriptor loads stand between the launch and the first data load.
struct ChunkDesc {
  const void* x;        // tensor base (element type: the call's dtype)
  float* y;
  int64_t n;            // tensor elements
  int64_t begin, end;   // apply: element range of this chunk; statistics: its partials [begin, end)
  uint64_t rng_offset;  // tensor's RNG offset relative to params.offset
  int32_t tensor;
  int32_t first_chunk;  // apply: global index of the tensor's first chunk; statistics: of its first
                        // partial in the partial array
  int32_t n_chunks;     // chunks of this tensor (statistics: workgroups arriving on its counter)
  int32_t all_positive;
};

static_assert(sizeof(MultiHeader) == 32, "plan header");
static_assert(sizeof(ChunkDesc) == 64, "chunk desc");

struct MultiArgs {
  const MultiHeader* hdr;
  const SmqTensorDesc* descs;
  const ChunkDesc* chunks;       // apply chunks
  const ChunkDesc* stat_chunks;  // statistics chunks
  const int32_t* final_rec;      // [count] first statistics record of a tensor to finalize, or -1
  SmqSmaqStats* stats;       // [count]
  unsigned long long* counters;  // [count] tagged arrival counters (block_arrive_tagged)
  ArriveTag tag;
  uint64_t* rng_snap;        // stream position of this call relative to offset (graph-safe mode)
  uint64_t* rng_ctr;         // params.offset_counter (NULL: host-managed offsets)
  uint64_t rng_span;         // elements this call draws: max(desc.rng_offset + n)
  StatPartial* partials;     // [n_chunks]
  float thr, r_main, r_out, clamp_lo, clamp_hi;
  int k;                     // SMQ_STATS_SAMPLED_DEVICE: samples per tensor (min(n, k) used)
  uint32_t draw_key;         // rng_key(seed ^ kDrawSalt)
  int advance_in_apply;      // sampled: the apply launch advances *rng_ctr (see the draw kernel)
  int use_range;             // --use_range_std_dev
  double inv_r_main, inv_r_out;
  int safe_q;
  uint32_t key;
  uint64_t offset;           // params.offset; tensor t draws from offset + desc.rng_offset + i
  int sr;
  int count_outliers;
};

// range-std coefficient of tensor t (desc.range_std_coef; negative: the fp32 1 / sqrt(2 ln n))
__device__ __forceinline__ float multi_range_coef(const MultiArgs& A, int t, int64_t n) {
  const float c = A.descs[t].range_std_coef;
  return c >= 0.0f ? c : 1.0f / sqrtf(2.0f * logf((float)n));
}

// Statistics of the tensors up to kSmallMaxN elements: one 1024-thread workgroup (two per CU) per
// record of partials_per_wg partials of the single-tensor partition (smaq_small.h): the native
// partial shape, smaq_stats_small_kernel's lane function, wave butterfly and combine. A tensor of
// one partial finalises in place; otherwise the partials are stored (plain) and
// smaq_multi_final_kernel reduces them.
template <int TIN, bool RANGE>
__global__ __launch_bounds__(kSmallT, 8) void smaq_multi_stats_kernel(MultiArgs A) {
  __shared__ SmallWaveLds W[8];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // one snapshot + advance per call
    uint64_t o = 0;
    if (A.rng_ctr) {
      o = *A.rng_ctr;
      *A.rng_ctr = o + A.rng_span;
    }
    *A.rng_snap = o;
  }
  const ChunkDesc ch = A.stat_chunks[blockIdx.x];
  const void* __restrict__ x = ch.x;
  const int64_t n = ch.n;
  const SmallGeom g = small_geom(n);
  const int G = g.G, b0 = (int)ch.begin, end = (int)ch.end;
  const double shift = stats_shift<TIN>(x, n);
  const bool vec = ((uintptr_t)x & (TIN == kF32 ? 15u : 7u)) == 0;
  switch (g.V) {
    case 1: small_waves_1024_runs<TIN, 1, RANGE>(x, n, G, b0, vec, shift, W); break;
    case 2: small_waves_1024_runs<TIN, 2, RANGE>(x, n, G, b0, vec, shift, W); break;
    case 3: small_waves_1024_runs<TIN, 3, RANGE>(x, n, G, b0, vec, shift, W); break;
    case 4: small_waves_1024_runs<TIN, 4, RANGE>(x, n, G, b0, vec, shift, W); break;
    default: small_waves_1024_seq<TIN, RANGE>(x, n, g.V, G, b0, vec, shift, W);
  }
  if (G == 1) {
    if (threadIdx.x == 0) {
      const FinalizeArgs fin{A.clamp_lo, A.clamp_hi,
                             RANGE ? multi_range_coef(A, ch.tensor, n) : 0.0f};
      const StatAcc r = small_combine(W[0]);
      finalize_stats<RANGE, TIN>(r.s1, r.s2, r.mn, r.mx, n, shift, false, fin,
                                 &A.stats[ch.tensor]);
    }
    return;
  }
  if (b0 + (int)threadIdx.x < end) {  // one partial per thread
    const int k = b0 + (int)threadIdx.x;
    const StatAcc r = small_combine(W[threadIdx.x]);
    StatPartial* q = A.partials + ch.first_chunk + k;
    q->s1 = r.s1;
    q->s2 = r.s2;
    q->mn = r.mn;
    q->mx = r.mx;
  }
}

// The totals of every small tensor of more than one partial (one workgroup per tensor, its first
// statistics record from the plan's table): reduce_partials_w0's order over its
// partials, stored by the statistics launch just before (plain loads: a launch boundary between),
// then the finalisation — the single-tensor call's statistics, bit for bit. Its own launch (5 us at
// C5): the last-arriving statistics workgroup reducing instead needs every workgroup's partial
// stores released before its arrival (sc1 stores + atomic: 45.7 us for the sweep against 40.7 +
// 4.8; plain stores + a release fence: 111 us), and every apply workgroup reducing its tensor's
// partials itself cost the apply 8 us.
template <int TIN, bool RANGE>
__global__ __launch_bounds__(kWave) void smaq_multi_final_kernel(MultiArgs A) {
  const int rec = A.final_rec[blockIdx.x];
  if (rec < 0) return;  // a large tensor, or one partial: its statistics are final already
  const ChunkDesc ch = A.stat_chunks[rec];
  const int64_t n = ch.n;
  const int G = small_geom(n).G;
  const double shift = stats_shift<TIN>(ch.x, n);
  double t1, t2;
  float tmn, tmx;
  reduce_partials_w0<false>(A.partials + ch.first_chunk, G, true, t1, t2, tmn, tmx);
  if (threadIdx.x == 0) {
    const FinalizeArgs fin{A.clamp_lo, A.clamp_hi,
                           RANGE ? multi_range_coef(A, ch.tensor, n) : 0.0f};
    finalize_stats<RANGE, TIN>(t1, t2, tmn, tmx, n, shift, false, fin, &A.stats[ch.tensor]);
  }
}

// Only the call's stream snapshot (no tensor of the call is small enough for the statistics launch
// above, which takes it otherwise).
__global__ void smaq_multi_snap_kernel(MultiArgs A) {
  if (threadIdx.x == 0) {
    uint64_t o = 0;
    if (A.rng_ctr) {
      o = *A.rng_ctr;
      *A.rng_ctr = o + A.rng_span;
    }
    *A.rng_snap = o;
  }
}

// SMQ_STATS_SAMPLED_DEVICE: one workgroup per tensor. Every workgroup reads the graph-safe position
// (nobody writes it during this launch); workgroup 0 records it for the apply launch, whose
// workgroup 0 then advances it (apply workgroups read only the record).
template <int TIN>
__global__ __launch_bounds__(kBlock) void smaq_multi_draw_kernel(MultiArgs A) {
  __shared__ DrawLds L;
  const int t = blockIdx.x;
  const SmqTensorDesc d = A.descs[t];
  const uint64_t snap = A.rng_ctr ? *A.rng_ctr : 0ull;
  if (t == 0 && threadIdx.x == 0) *A.rng_snap = snap;
  const int k = (int64_t)A.k < d.n ? A.k : (int)d.n;
  const FinalizeArgs f{A.clamp_lo, A.clamp_hi,
                       A.descs[t].range_std_coef >= 0.0f ? A.descs[t].range_std_coef
                                                         : 1.0f / sqrtf(2.0f * logf((float)k))};
  draw_sample_stats<TIN>(d.x, d.n, k, A.draw_key, A.offset + snap + d.rng_offset,
                         A.use_range, f, &A.stats[t], nullptr, L);
}

// all_positive varies per tensor here (one chunk = one tensor): a per-element select.
template <int RM, int TIN, bool SUB, bool SQ>
__device__ __forceinline__ float elem_ap(float v, float u, const ElemConsts& c, bool all_pos,
                                         bool& b) {
  const float o = smaq_elem<RM, false, TIN, false, SUB, SQ>(v, u, c, b);
  return (all_pos && o < 0.0f) ? 0.0f : o;  // clamp_min(0.0)
}

// One chunk. SUB: subnormal-quotient check (per tensor, quot_check_for); SQ: RangeRecips::safe_q.
// pre: the first step's data, loaded by the caller before the tensor's statistics arrive.
template <bool SR, int TIN, bool SUB, bool SQ>
__device__ __forceinline__ unsigned long long multi_chunk(const MultiArgs& A, const ChunkDesc& ch,
                                                          const ElemConsts& c, bool all_pos,
                                                          bool vec, const float4 (&pre)[4],
                                                          uint64_t off) {
  const void* __restrict__ x = ch.x;
  float* y = ch.y;  // may alias x (fp32)
  unsigned long long n_out = 0;
  constexpr int RM = SR ? kRoundHash : kRoundTrunc;
  if (vec) {
    float4* y4 = reinterpret_cast<float4*>(y);
    const int64_t b4 = ch.begin >> 2, e4 = ch.end >> 2;
    for (int64_t t0 = b4; t0 < e4; t0 += 4 * kBlock) {  // 16 KiB per step, 4 dwordx4 per lane
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = t0 + threadIdx.x + u * kBlock;
      if (t0 == b4) v[u] = pre[u];
      else if (j < e4) v[u] = load4<TIN>(x, j);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = t0 + threadIdx.x + u * kBlock;
      if (j >= e4) continue;
      const uint64_t ctr = off + ch.rng_offset + ((uint64_t)j << 2);
      float u0 = 0.f, u1 = 0.f, u2 = 0.f, u3 = 0.f;
      if (SR) rng_hu4(A.key, ctr, u0, u1, u2, u3);
      bool b0, b1, b2, b3;
      float4 o;
      o.x = elem_ap<RM, TIN, SUB, SQ>(v[u].x, u0, c, all_pos, b0);
      o.y = elem_ap<RM, TIN, SUB, SQ>(v[u].y, u1, c, all_pos, b1);
      o.z = elem_ap<RM, TIN, SUB, SQ>(v[u].z, u2, c, all_pos, b2);
      o.w = elem_ap<RM, TIN, SUB, SQ>(v[u].w, u3, c, all_pos, b3);
      n_out += (unsigned)b0 + (unsigned)b1 + (unsigned)b2 + (unsigned)b3;
      store_stream(y4 + j, o);
    }
    }
    if (threadIdx.x < (int)(ch.end - (e4 << 2))) {
      const int64_t e = (e4 << 2) + threadIdx.x;
      const float u = SR ? rng_hu(A.key, off + ch.rng_offset + (uint64_t)e) : 0.f;
      bool b;
      y[e] = elem_ap<RM, TIN, SUB, SQ>(load1<TIN>(x, e), u, c, all_pos, b);
      n_out += (unsigned)b;
    }
  } else {
    for (int64_t j = ch.begin + threadIdx.x; j < ch.end; j += kBlock) {
      const float u = SR ? rng_hu(A.key, off + ch.rng_offset + (uint64_t)j) : 0.f;
      bool b;
      y[j] = elem_ap<RM, TIN, SUB, SQ>(load1<TIN>(x, j), u, c, all_pos, b);
      n_out += (unsigned)b;
    }
  }
  return n_out;
}

template <bool SR, bool SQ, int TIN>
__global__ __launch_bounds__(kBlock) void smaq_multi_apply_kernel(MultiArgs A) {
  __shared__ unsigned long long sh_cnt[kBlock / kWave];
  const ChunkDesc ch = A.chunks[blockIdx.x];
  // the first 16 KiB of the chunk is requested before the statistics (they do not depend on them)
  const bool vec = (((uintptr_t)ch.x & (TIN == kF32 ? 15u : 7u)) | ((uintptr_t)ch.y & 15u)) == 0;
  float4 pre[4];
  if (vec) {
    const int64_t b4 = ch.begin >> 2, e4 = ch.end >> 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = b4 + threadIdx.x + u * kBlock;
      pre[u] = j < e4 ? load4<TIN>(ch.x, j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (A.advance_in_apply && blockIdx.x == 0 && threadIdx.x == 0 && A.rng_ctr)
    *A.rng_ctr = *A.rng_snap + A.rng_span;  // sampled: the draw launch only recorded the position
  const SmqSmaqStats* st = &A.stats[ch.tensor];
  ElemConsts c;
  const float cthr = TIN == kF32 ? A.thr : round_in<TIN>(A.thr);
  init_consts(c, st, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  const bool all_pos = ch.all_positive != 0;
  const uint64_t off = A.offset + *A.rng_snap;  // + the call's snapshot (0 unless graph-safe)
  const unsigned long long n_out =
      st->quot_check ? multi_chunk<SR, TIN, true, SQ>(A, ch, c, all_pos, vec, pre, off)
                     : multi_chunk<SR, TIN, false, SQ>(A, ch, c, all_pos, vec, pre, off);
  if (A.count_outliers) {
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const double t = wave_sum((double)n_out);
    if (lane == 0) sh_cnt[wave] = (unsigned long long)t;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long s = sh_cnt[0] + sh_cnt[1] + sh_cnt[2] + sh_cnt[3];
      if (s) atomicAdd((unsigned long long*)&A.stats[ch.tensor].n_outlier, s);
    }
  }
}

static int64_t chunk_elems() {
  static const int64_t c = [] {
    const char* e = knob_env("SMQ_MULTI_CHUNK");
    const int64_t v = e ? atoll(e) : kDefaultChunk;
    return (v >= 4096 && v % 4096 == 0) ? v : kDefaultChunk;
  }();
  return c;
}

static int64_t chunks_of(int64_t n, int64_t c) { return (n + c - 1) / c; }

struct PlanSizes {
  size_t hdr, descs, chunks, stat_chunks, final_tab, total;
  int64_t n_chunks, n_stat_chunks, n_partials;
  bool big;  // a tensor above kSmallMaxN (its statistics: the single-tensor launch)
};

// Partials per statistics workgroup (1024 threads, the partial's native shape, two per CU): 4 / V
// at V <= 4, i.e. 4 float4 groups per thread, all in flight at once; else 1 (loaded a group at a
// time: holding V > 4 groups spills at that occupancy). Not a reduction-order parameter:
// every partial is stored and reduced in one order whatever the grouping. (Measured at C5: a
// 256-thread workgroup walking 16 partials one 12-KB step of loads ahead at a time, 139 us; 256
// threads with four lanes each, a run of 4 / V partials in flight, 41 us — of which 22.6 us of
// VALU alone, four wave butterflies per partial and wave: repo:tools/multi_exp.sh.)
static int64_t partials_per_wg(int64_t n) {
  const int V = small_geom(n).V;
  return V <= 4 ? 4 / V : 1;
}

static bool plan_sizes(const int64_t* sizes, int count, PlanSizes* ps) {
  int64_t nc = 0, ns = 0, np = 0;
  bool big = false;
  for (int t = 0; t < count; ++t) {
    if (sizes[t] < 1) return false;
    nc += chunks_of(sizes[t], chunk_elems());
    if (sizes[t] > kSmallMaxN) {
      big = true;
      continue;
    }
    const int64_t G = small_geom(sizes[t]).G;
    np += G;
    ns += chunks_of(G, partials_per_wg(sizes[t]));
  }
  ps->n_chunks = nc;
  ps->n_stat_chunks = ns;
  ps->n_partials = np;
  ps->big = big;
  ps->hdr = sizeof(MultiHeader);
  ps->descs = ((sizeof(SmqTensorDesc) * (size_t)count) + 31) & ~(size_t)31;
  ps->chunks = sizeof(ChunkDesc) * (size_t)nc;
  ps->stat_chunks = sizeof(ChunkDesc) * (size_t)ns;
  ps->final_tab = ((sizeof(int32_t) * (size_t)count) + 63) & ~(size_t)63;
  ps->total = ps->hdr + ps->descs + ps->chunks + ps->stat_chunks + ps->final_tab;
  return true;
}

// Statistics records: per small tensor, runs of partials_per_wg partials.
static void fill_stat_chunks(ChunkDesc* ch, const SmqTensorDesc* descs, int count) {
  int32_t g = 0, part = 0;
  for (int t = 0; t < count; ++t) {
    const int64_t n = descs[t].n;
    if (n > kSmallMaxN) continue;
    const int64_t G = small_geom(n).G, per = partials_per_wg(n), wgs = chunks_of(G, per);
    for (int64_t c = 0; c < wgs; ++c, ++g) {
      ch[g].x = descs[t].x;
      ch[g].y = descs[t].y;
      ch[g].n = n;
      ch[g].begin = c * per;
      ch[g].end = (c + 1) * per < G ? (c + 1) * per : G;
      ch[g].rng_offset = descs[t].rng_offset;
      ch[g].tensor = t;
      ch[g].first_chunk = part;
      ch[g].n_chunks = (int32_t)wgs;
      ch[g].all_positive = descs[t].all_positive;
    }
    part += (int32_t)G;
  }
}

// Chunk records of one map (element chunks of C) for every tensor, starting at ch.
static void fill_chunks(ChunkDesc* ch, const SmqTensorDesc* descs, int count, int64_t C) {
  int32_t g = 0;
  for (int t = 0; t < count; ++t) {
    const int64_t nc = chunks_of(descs[t].n, C);
    const int32_t first = g;
    for (int64_t c = 0; c < nc; ++c, ++g) {
      ch[g].x = descs[t].x;
      ch[g].y = descs[t].y;
      ch[g].n = descs[t].n;
      ch[g].begin = c * C;
      ch[g].end = (c + 1) * C < descs[t].n ? (c + 1) * C : descs[t].n;
      ch[g].rng_offset = descs[t].rng_offset;
      ch[g].tensor = t;
      ch[g].first_chunk = first;
      ch[g].n_chunks = (int32_t)nc;
      ch[g].all_positive = descs[t].all_positive;
    }
  }
}

}  // namespace smq

using namespace smq;

extern "C" {

size_t smq_smaq_multi_plan_bytes(const int64_t* sizes, int count) {
  PlanSizes ps;
  if (!sizes || count < 1 || !plan_sizes(sizes, count, &ps)) return 0;
  return ps.total;
}

int smq_smaq_multi_plan_build(const SmqTensorDesc* descs, int count, void* host_plan,
                              size_t plan_bytes) {
  if (!descs || count < 1 || !host_plan) {
    set_error("multi_plan_build: bad arguments");
    return SMQ_ERR_INVALID;
  }
  int64_t* sizes = (int64_t*)malloc(sizeof(int64_t) * (size_t)count);
  for (int t = 0; t < count; ++t) {
    sizes[t] = descs[t].n;
    if (!descs[t].x || !descs[t].y || descs[t].n < 1) {
      free(sizes);
      set_error("multi_plan_build: tensor %d has NULL pointer or n < 1", t);
      return SMQ_ERR_INVALID;
    }
  }
  PlanSizes ps;
  plan_sizes(sizes, count, &ps);
  free(sizes);
  if (plan_bytes < ps.total) {
    set_error("multi_plan_build: plan buffer too small (%zu < %zu)", plan_bytes, ps.total);
    return SMQ_ERR_INVALID;
  }
  if (ps.n_chunks > 0x7fffffffLL) {
    set_error("multi_plan_build: too many chunks");
    return SMQ_ERR_INVALID;
  }
  char* base = (char*)host_plan;
  memset(base, 0, ps.total);
  MultiHeader* h = (MultiHeader*)base;
  h->count = count;
  h->n_chunks = (int32_t)ps.n_chunks;
  h->chunk = chunk_elems();
  h->n_stat_chunks = (int32_t)ps.n_stat_chunks;
  h->n_partials = (int32_t)ps.n_partials;
  h->stat_chunk = 0;  // statistics records are runs of partials_per_wg partials
  memcpy(base + ps.hdr, descs, sizeof(SmqTensorDesc) * (size_t)count);
  fill_chunks((ChunkDesc*)(base + ps.hdr + ps.descs), descs, count, h->chunk);
  ChunkDesc* sc = (ChunkDesc*)(base + ps.hdr + ps.descs + ps.chunks);
  fill_stat_chunks(sc, descs, count);
  // per tensor: its first statistics record when the finalize launch reduces its partials (a
  // small tensor of more than one partial), else -1
  int32_t* fin = (int32_t*)(base + ps.hdr + ps.descs + ps.chunks + ps.stat_chunks);
  for (int t = 0; t < count; ++t) fin[t] = -1;
  for (int64_t r = 0; r < ps.n_stat_chunks; ++r)
    if (sc[r].begin == 0 && small_geom(sc[r].n).G > 1) fin[sc[r].tensor] = (int32_t)r;
  return SMQ_OK;
}

static size_t multi_ws_bytes(int count, int64_t n_partials, bool big) {
  const size_t stats = sizeof(SmqSmaqStats) * (size_t)count;
  const size_t counters = ((sizeof(uint64_t) * (size_t)count) + 63) & ~(size_t)63;
  const size_t parts = (sizeof(StatPartial) * (size_t)n_partials + 255) & ~(size_t)255;
  return ((stats + counters + kSnapBytes + 255) & ~(size_t)255) + parts + (big ? kBigWsBytes : 0);
}

size_t smq_smaq_multi_workspace_bytes(const int64_t* sizes, int count) {
  PlanSizes ps;
  if (!sizes || count < 1 || !plan_sizes(sizes, count, &ps)) return 0;
  return multi_ws_bytes(count, ps.n_partials, ps.big);
}

}  // extern "C"

template <int TIN>
static int launch_multi(const MultiArgs& A, bool sampled, bool range, int n_stat_chunks,
                        int count, int n_chunks, hipStream_t st) {
  if (sampled) {
    hipLaunchKernelGGL((smaq_multi_draw_kernel<TIN>), dim3(count), dim3(kBlock), 0, st, A);
  } else if (n_stat_chunks == 0) {  // only large tensors: their statistics are launched already
    hipLaunchKernelGGL(smaq_multi_snap_kernel, dim3(1), dim3(kWave), 0, st, A);
  } else if (range) {
    hipLaunchKernelGGL((smaq_multi_stats_kernel<TIN, true>), dim3(n_stat_chunks), dim3(kSmallT), 0,
                       st, A);
    hipLaunchKernelGGL((smaq_multi_final_kernel<TIN, true>), dim3(count), dim3(kWave), 0, st, A);
  } else {
    hipLaunchKernelGGL((smaq_multi_stats_kernel<TIN, false>), dim3(n_stat_chunks), dim3(kSmallT),
                       0, st, A);
    hipLaunchKernelGGL((smaq_multi_final_kernel<TIN, false>), dim3(count), dim3(kWave), 0, st, A);
  }
  int rc = check_launch(sampled ? "smaq_multi_draw_kernel" : "smaq_multi_stats_kernel");
  if (rc) return rc;
#define SMQ_MULTI_APPLY(SRV, SQV) \
  hipLaunchKernelGGL((smaq_multi_apply_kernel<SRV, SQV, TIN>), dim3(n_chunks), dim3(kBlock), 0, st, A)
  if (A.sr) {
    if (A.safe_q) SMQ_MULTI_APPLY(true, true); else SMQ_MULTI_APPLY(true, false);
  } else {
    if (A.safe_q) SMQ_MULTI_APPLY(false, true); else SMQ_MULTI_APPLY(false, false);
  }
#undef SMQ_MULTI_APPLY
  return check_launch("smaq_multi_apply_kernel");
}

extern "C" int smq_smaq_multi(const void* dev_plan, const void* host_plan, int dtype,
                              const SmqSmaqParams* p, void* ws, size_t ws_bytes, void* stream) {
  if (!dev_plan || !host_plan) {
    set_error("multi: dev_plan and host_plan are required");
    return SMQ_ERR_INVALID;
  }
  const MultiHeader* hh = (const MultiHeader*)host_plan;
  const int count = hh->count;
  const int n_chunks = hh->n_chunks;
  const int n_stat_chunks = hh->n_stat_chunks;
  const int n_partials = hh->n_partials;
  if (!dev_plan || count < 1 || n_chunks < 1 || n_stat_chunks < 0 || !p || !ws) {
    set_error("multi: bad arguments");
    return SMQ_ERR_INVALID;
  }
  if (dtype != SMQ_DTYPE_F32 && dtype != SMQ_DTYPE_F16 && dtype != SMQ_DTYPE_BF16) {
    set_error("multi: dtype %d is not one of SMQ_DTYPE_F32/F16/BF16", dtype);
    return SMQ_ERR_INVALID;
  }
  const bool sampled = p->stats_source == SMQ_STATS_SAMPLED_DEVICE;
  if (p->stats_source != SMQ_STATS_WORKSPACE && !sampled) {
    set_error("multi: statistics must be SMQ_STATS_WORKSPACE or SMQ_STATS_SAMPLED_DEVICE");
    return SMQ_ERR_INVALID;
  }
  if (sampled && (p->num_samples < 1 || p->num_samples > SMQ_MAX_DEVICE_SAMPLES)) {
    set_error("multi: device-drawn sampled stats need 1 <= num_samples <= %d",
              SMQ_MAX_DEVICE_SAMPLES);
    return SMQ_ERR_INVALID;
  }
  if (p->bn_gamma) {
    set_error("multi: the BN variant is per activation tensor (smq_smaq_apply)");
    return SMQ_ERR_INVALID;
  }
  const SmqTensorDesc* hd = (const SmqTensorDesc*)((const char*)host_plan + sizeof(MultiHeader));
  bool big = false;
  for (int t = 0; t < count && !big; ++t) big = hd[t].n > kSmallMaxN;
  const size_t stats = sizeof(SmqSmaqStats) * (size_t)count;
  const size_t counters = ((sizeof(uint64_t) * (size_t)count) + 63) & ~(size_t)63;
  const size_t need = multi_ws_bytes(count, n_partials, big);
  if (ws_bytes < need) {
    set_error("multi: workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    return SMQ_ERR_WORKSPACE;
  }
  if (dtype != SMQ_DTYPE_F32) {  // fp32 outputs: an in-place half tensor cannot hold them
    for (int t = 0; t < count; ++t)
      if ((const void*)hd[t].x == (const void*)hd[t].y) {
        set_error("multi: tensor %d: fp16 / bf16 inputs write fp32 outputs, y cannot alias x", t);
        return SMQ_ERR_INVALID;
      }
  }
  const char* pb = (const char*)dev_plan;
  const size_t descs_bytes = ((sizeof(SmqTensorDesc) * (size_t)count) + 31) & ~(size_t)31;
  MultiArgs A;
  memset(&A, 0, sizeof(A));
  A.hdr = (const MultiHeader*)pb;
  A.descs = (const SmqTensorDesc*)(pb + sizeof(MultiHeader));
  A.chunks = (const ChunkDesc*)(pb + sizeof(MultiHeader) + descs_bytes);
  A.stat_chunks = A.chunks + n_chunks;
  A.final_rec = reinterpret_cast<const int32_t*>(A.stat_chunks + n_stat_chunks);
  char* wb = (char*)ws;
  A.stats = (SmqSmaqStats*)wb;
  A.counters = (unsigned long long*)(wb + stats);
  A.tag = arrive_tag(ws, (hipStream_t)stream);
  A.rng_snap = (uint64_t*)(wb + stats + counters);
  const size_t parts_at = (stats + counters + kSnapBytes + 255) & ~(size_t)255;
  A.partials = (StatPartial*)(wb + parts_at);
  A.rng_ctr = p->offset_counter;
  uint64_t span = 0;  // the stream span of the call, from the host copy of the descriptors
  if (A.rng_ctr) {
    for (int t = 0; t < count; ++t) {
      const uint64_t e = hd[t].rng_offset + (uint64_t)hd[t].n;
      span = e > span ? e : span;
    }
  }
  A.rng_span = span;
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
  A.sr = p->stochastic_rounding;
  A.count_outliers = p->count_outliers;
  A.use_range = p->use_range_std_dev;
  A.k = sampled ? p->num_samples : 0;
  A.draw_key = rng_key(p->seed ^ kDrawSalt);
  A.advance_in_apply = sampled ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  const bool range = p->use_range_std_dev != 0;
  if (big && !sampled) {
    // tensors above kSmallMaxN: the single-tensor statistics launch, into the tensor's record (its
    // own partition and reduction order, so the statistics are a single call's); no stream
    // position is taken here (the element kernels read the call's snapshot)
    char* bws = wb + parts_at + ((sizeof(StatPartial) * (size_t)n_partials + 255) & ~(size_t)255);
    for (int t = 0; t < count; ++t) {
      if (hd[t].n <= kSmallMaxN) continue;
      SmqSmaqParams q = *p;
      q.offset_counter = nullptr;
      q.range_std_coef = hd[t].range_std_coef;
      const int rc = stats_into(hd[t].x, dtype, hd[t].n, &q, bws, kBigWsBytes, st, &A.stats[t]);
      if (rc) return rc;
    }
  }
  if (dtype == SMQ_DTYPE_F32)
    return launch_multi<kF32>(A, sampled, range, n_stat_chunks, count, n_chunks, st);
  if (dtype == SMQ_DTYPE_F16)
    return launch_multi<kF16>(A, sampled, range, n_stat_chunks, count, n_chunks, st);
  return launch_multi<kBF16>(A, sampled, range, n_stat_chunks, count, n_chunks, st);
}

extern "C" int smq_smaq_multi_f32(const void* dev_plan, const void* host_plan,
                                  const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                                  void* stream) {
  return smq_smaq_multi(dev_plan, host_plan, SMQ_DTYPE_F32, p, ws, ws_bytes, stream);
}
