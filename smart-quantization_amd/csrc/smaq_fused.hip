// smaq_fused.hip — SmaQ compress->decompress round trip of activation-sized tensors in ONE launch
// (gfx950), and the statistics launch of the two-launch paths for the same sizes.
//
// Reference: smart_compress/compress/smart.py:110-190 (SmartFP.__call__), called per module output
// and per grad-map by util/pytorch/autograd.py:30-42 — tensors of 10^5 .. 8.4 * 10^6 elements
// (CIFAR ResNet-34 at batch 128: 132 forward calls, the largest 128x64x32x32). At these sizes the
// two-launch shape (statistics sweep, then a transform that re-reads x) pays a kernel boundary, a
// second launch ramp and a second read of x; the call is latency-bound, not bandwidth-bound.
//
// smaq_fused_kernel: workgroup b (1024 threads) loads its chunk of the smaq_small.h partition — V
// float4 groups per lane — into registers ONCE, computes the chunk's statistics partial exactly as
// the two-launch statistics launch does (smaq_stats_small_kernel, same lanes, same chains, same
// butterflies), publishes it, waits until every chunk's partial is there, reduces them in
// reduce_partials_w0's order, finalises (smart.py:130-134, 100-108, 151-152), and transforms its
// registers (smart.py:154-182). 8 B/elem of HBM traffic (x read once, y written); the statistics,
// outputs and stream position equal smq_smaq_stats + smq_smaq_apply bit for bit by construction.
//
// Hand-off (cdna_hip_programming.md Guideline 16 R2, as the single-launch S2FP8 in float_quant.hip):
// a partial is 4 (6 with range-std: + min, max) aligned 8-byte granules {epoch, 32-bit word}, each
// ONE relaxed agent-scope (sc1) store, written to 8 replicas (replica r is polled by the workgroups
// b % 8 == r, spreading 256 readers over 8x the memory channels). A replica is dense (partial k's
// words at k * words): every thread re-reads the two words it owns while any is missing, so a wave
// load is 512 consecutive bytes (4 lines, not 64) — 12 KB per pass in 96 lines. The epoch is
// (generation << 1) | 1: every workgroup reads the generation word at its start; the arrival words
// (eight per residue b % 8, one on top: same-address atomics serialise at ~12 ns each, so 256 adds
// on one word would cost ~3 us) are tagged with the generation, added to after the gather and
// looked at after the transform; the last arrival advances the generation, the graph-safe stream
// counter and re-arms the arrival words. Calls on one workspace are serialised by the stream, so
// consecutive calls — eager or replayed from a graph — see consecutive generations and never a
// stale granule of an earlier call as their own.
//
// No co-residency assumption: a workgroup that has waited kFusedStealTicks computes the partials it
// still misses itself, from memory (a partial is a pure function of its chunk: duplicates store the
// same bytes), so a grid that is only partly resident (other kernels holding CUs) still finishes.
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "smq_common.h"
#include "smaq_elem.h"
#include "smaq_pack_common.h"
#include "smaq_small.h"

namespace smq {

constexpr int kFusedRep = SmaqWsLayout::kFusedRep;
constexpr int kFusedWords = SmaqWsLayout::kFusedWords;
constexpr uint64_t kFusedStealTicks = 20000;  // s_memrealtime at 100 MHz: 200 us
// dynamic LDS request (one workgroup per CU): the parked groups (V > 4) and then the rounding
// draws of the first fused_draw_groups(V) groups, 16 KiB per group
constexpr int kFusedLdsGroups = 9;
constexpr int kFusedLds = kFusedLdsGroups * 16 * 1024;
// groups whose rounding draws are hashed during the gather into LDS (V >= 4; V <= 3 keeps them in
// registers): as many as fit next to the parked groups
// (V = 8: 5 of its 8 groups would fit, and measured 19.41 -> 19.53 us at 8M: left in the transform)
__host__ __device__ constexpr int fused_draw_groups(int V) {
  return (V < 4 || V > 7) ? 0 : (V < kFusedLdsGroups - (V - 4) ? V : kFusedLdsGroups - (V - 4));
}
// the launch's dynamic LDS: the parked groups and the draws, at least 88 KiB (one workgroup per CU)
__host__ __device__ constexpr int fused_lds_bytes(int V) {
  return ((V > 4 ? V - 4 : 0) + fused_draw_groups(V)) * 16 * 1024 > 88 * 1024
             ? ((V > 4 ? V - 4 : 0) + fused_draw_groups(V)) * 16 * 1024
             : 88 * 1024;
}
constexpr int kSubStride = (int)(SmaqWsLayout::kFusedSubStride / 8);  // residue words (u64 units)

// ------------------------------------------------------------------------------------------------
// statistics launch of the two-launch paths (smq_smaq_stats, and smq_smaq_roundtrip when the single
// launch does not apply): one workgroup per partial
// ------------------------------------------------------------------------------------------------
template <int TIN>
__global__ __launch_bounds__(kSmallT) void smaq_stats_small_kernel(const void* __restrict__ x,
                                                                   int64_t n, int V, int vec,
                                                                   int range, FinalizeArgs fin,
                                                                   StatPartial* partials,
                                                                   unsigned long long* counter,
                                                                   ArriveTag tag,
                                                                   SmqSmaqStats* out,
                                                                   double* def_rec) {
  __shared__ SmallWaveLds W;
  __shared__ uint32_t arrive_slot;
  clear_aux(fin);
  const int G = gridDim.x, b = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const double shift = stats_shift<TIN>(x, n);
  const StatAcc w = small_wave(small_lane<TIN, kSmallMaxV>(x, n, V, G, b, threadIdx.x, vec != 0,
                                                           shift));
  if (lane == 0) {
    W.s1[wave] = w.s1;
    W.s2[wave] = w.s2;
    W.mn[wave] = w.mn;
    W.mx[wave] = w.mx;
  }
  __syncthreads();
  if (G == 1) {  // the partial is the total: finalise without a hand-off
    if (threadIdx.x == 0) {
      const StatAcc a = small_combine(W);
      if (range) finalize_stats<true, TIN>(a.s1, a.s2, a.mn, a.mx, n, shift, false, fin, out);
      else finalize_stats<false, TIN>(a.s1, a.s2, a.mn, a.mx, n, shift, false, fin, out);
    }
    return;
  }
  if (def_rec) {  // deferred statistics: every apply workgroup reduces the partials (defer_consts)
    if (threadIdx.x == 0) {
      const StatAcc a = small_combine(W);
      StatPartial* p = partials + b;
      p->s1 = a.s1;
      p->s2 = a.s2;
      p->mn = a.mn;
      p->mx = a.mx;
      if (b == 0) {  // the shift, and the call's graph-safe stream position
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
    const StatAcc a = small_combine(W);
    StatPartial* p = partials + b;
    st_sc1_f64(&p->s1, a.s1);
    st_sc1_f64(&p->s2, a.s2);
    st_sc1_f32x2(&p->mn, a.mn, a.mx);
  }
  const uint32_t prev = block_arrive_tagged(counter + (tag.tag & (SmaqWsLayout::kTagWords - 1)),
                                            tag.tag, &arrive_slot);
  if (prev != (uint32_t)G - 1) return;
  if (threadIdx.x < kWave) {
    double t1, t2;
    float tmn, tmx;
    reduce_partials_w0<true>(partials, G, true, t1, t2, tmn, tmx);
    if (threadIdx.x == 0) {
      if (range) finalize_stats<true, TIN>(t1, t2, tmn, tmx, n, shift, false, fin, out);
      else finalize_stats<false, TIN>(t1, t2, tmn, tmx, n, shift, false, fin, out);
      arrive_reset(counter + (tag.next & (SmaqWsLayout::kTagWords - 1)), tag.next);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// the single launch
// ------------------------------------------------------------------------------------------------
struct FusedArgs {
  const void* x;
  float* y;
  int64_t n, nv;
  int G;
  uint32_t key;
  uint64_t offset;
  uint64_t* ctr;                 // graph-safe stream position (nullable)
  SmqSmaqStats* hdr;
  uint32_t* gen;                 // generation word
  unsigned long long* left;      // residues whose workgroups are all past the wait (tagged)
  unsigned long long* sub;       // workgroups b % 8 == s past the wait: word s * kSubStride
  unsigned long long* gran;      // [kFusedRep][kSmallMaxG][kFusedWords] granules
  unsigned long long* out_slots; // outlier-count slots (count)
  float thr, r_main, r_out, clamp_lo, clamp_hi, range_coef;
  double inv_r_main, inv_r_out;
  int all_pos, count, range, test_late;
  int poll_sleep;   // s_sleep between poll passes
  uint64_t* trace;  // experiment builds (-DSMQ_FUSED_TRACE=1): 16 timestamps per workgroup
  uint32_t* zero;   // cleared by workgroup 0 (the packer's group sums: roundtrip_compress), or NULL
  uint32_t zero_n;
  unsigned long long* rec_gran;  // counted call, full statistics: [G] epoch-tagged counts (or NULL)
  SmqSizeRecord* rec;  // counted call (count = 1, out_slots = rec->slots): the last workgroup to
                       // have added its count writes the log_size values
  int bm, bo;
  // PACK variant (smq_smaq_roundtrip_compress): the call's packed stream, written from registers
  struct {
    SmqPackedHeader* hdr;
    uint64_t* dir;
    uint32_t* fixed;
    uint32_t* var;
    uint64_t cap_words;        // words of the variable region the buffer holds
    uint32_t n_blocks, flags;
    unsigned long long* look;  // [G] epoch-tagged aggregates: replica 0, granules 1024 + b
    uint32_t lds_off;          // word offset of the pack area in the dynamic LDS
    uint32_t* notify;          // total_bytes also here (notify_total), or NULL
  } pk;
};

// The log_size values of a counted call from its n_outlier (smart.py:184-188, base.py:84-88).
__device__ __forceinline__ void size_record_finish(SmqSizeRecord* rec, uint64_t n_out, int64_t n,
                                                   int bm, int bo) {
  const double no = (double)n_out;
  const double ns = no * (double)bo + (double)(n - (int64_t)n_out) * (double)bm;  // exact (< 2^53)
  const double orig = 32.0 * (double)n;
  rec->n_outlier = no;
  rec->new_size = ns;
  rec->compression_ratio = orig / ns;
  rec->orig_size = orig;
}

// Counted call: this workgroup's count s AND its arrival in ONE returning atomic on its residue's
// slot (count in the low 40 bits, arrivals above: 32 same-address atomics per word at G = 256
// instead of 256 on one word, ~12 ns each); the last of a residue then arrives on the top word, and
// the last of those (every slot add has returned before its residue's top add was issued) sums the
// slots' counts and writes the values.
constexpr int kRecArrShift = 40;
__device__ __forceinline__ void size_record_arrive(SmqSizeRecord* rec, unsigned long long s, int b,
                                                   int G, int64_t n, int bm, int bo) {
  if (G == 1) {
    size_record_finish(rec, s, n, bm, bo);
    return;
  }
  const int r = b & 7;
  const unsigned long long prev = __hip_atomic_fetch_add(
      rec->slots + r, s + (1ull << kRecArrShift), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int in_res = G / 8 + (r < (G & 7) ? 1 : 0);  // workgroups b < G with b % 8 == r
  if ((int)(prev >> kRecArrShift) != in_res - 1) return;
  const int residues = G < 8 ? G : 8;
  const unsigned long long top = __hip_atomic_fetch_add(&rec->arrived, 1ull, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
  if (top != (unsigned long long)residues - 1ull) return;
  unsigned long long t = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    t += __hip_atomic_load(rec->slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
         ((1ull << kRecArrShift) - 1ull);
  size_record_finish(rec, t, n, bm, bo);
}

// s_memrealtime stamps (100 MHz) of workgroup milestones, experiment builds only
#ifndef SMQ_FUSED_TRACE
#define SMQ_FUSED_TRACE 0
#endif
// The thread that issues this workgroup's arrivals: wave 1's lane 0, so a wait for an atomic's
// return never holds wave 0 (the reduce and finalise) or the barrier after it.
constexpr int kArriveThread = kWave;
#if SMQ_FUSED_TRACE
#define FSTAMP(i)                                                                   \
  do {                                                                              \
    if (A.trace && threadIdx.x == 0)                                                \
      A.trace[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define FSTAMP(i) \
  do {            \
  } while (0)
#endif

// s_sleep between poll passes (units of 64 clocks; a compile-time immediate, so a small switch)
__device__ __forceinline__ void fused_sleep(int s) {
  switch (s) {
    case 0: break;
    case 1: __builtin_amdgcn_s_sleep(1); break;
    case 2: __builtin_amdgcn_s_sleep(2); break;
    case 4: __builtin_amdgcn_s_sleep(4); break;
    case 8: __builtin_amdgcn_s_sleep(8); break;
    default: __builtin_amdgcn_s_sleep(16); break;
  }
}

// The partial of chunk k by the whole workgroup from the lanes' groups g; valid in wave 0 (the
// next writer of W, fused_steal, runs behind a barrier wave 0 reaches after reading it).
template <int TIN, int V>
__device__ __forceinline__ StatAcc fused_partial(const FusedArgs& A, int k, const float4 (&g)[V],
                                                 double shift, SmallWaveLds& W) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const StatAcc w = small_wave(small_lane_sum<TIN, V>(A.x, A.n, V, A.G, k, threadIdx.x, g, shift),
                               A.range != 0);
  if (lane == 0) {
    W.s1[wave] = w.s1;
    W.s2[wave] = w.s2;
    W.mn[wave] = w.mn;
    W.mx[wave] = w.mx;
  }
  lds_barrier();
  StatAcc r;
  if (wave == 0) r = small_combine(W);
  return r;
}

// The rare path: partial k computed from memory by the whole workgroup (one group per lane in
// flight), every thread gets it. Not inlined: its registers would otherwise add to the kernel's
// peak (the chunk held in registers stays live across it); a call costs register saves only on
// this path.
template <int TIN>
__device__ __noinline__ StatAcc fused_steal(const void* x, int64_t n, int V, int G, int k,
                                            double shift, SmallWaveLds* W) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const StatAcc w = small_wave(small_lane_seq<TIN>(x, n, V, G, k, threadIdx.x, shift), true);
  if (lane == 0) {
    W->s1[wave] = w.s1;
    W->s2[wave] = w.s2;
    W->mn[wave] = w.mn;
    W->mx[wave] = w.mx;
  }
  lds_barrier();
  const StatAcc r = small_combine(*W);
  lds_barrier();
  return r;
}

// Word c of a partial: s1 low / high, s2 low / high, min, max.
__device__ __forceinline__ uint32_t partial_word(const StatAcc& a, int c) {
  const uint64_t b1 = __builtin_bit_cast(uint64_t, a.s1), b2 = __builtin_bit_cast(uint64_t, a.s2);
  switch (c) {
    case 0: return (uint32_t)b1;
    case 1: return (uint32_t)(b1 >> 32);
    case 2: return (uint32_t)b2;
    case 3: return (uint32_t)(b2 >> 32);
    case 4: return __builtin_bit_cast(uint32_t, a.mn);
    default: return __builtin_bit_cast(uint32_t, a.mx);
  }
}

// Lanes 0 .. kFusedRep * words - 1 of wave 0 store partial k's granules (nobody waits for them).
__device__ __forceinline__ void fused_publish(const StatAcc& a, const FusedArgs& A, int k,
                                              uint32_t epoch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int words = A.range ? 6 : 4;
  if (lane >= kFusedRep * words) return;
  const int r = words == 4 ? lane >> 2 : (lane * 43) >> 8;  // lane / words (lane < 48)
  const int c = lane - r * words;
  const uint32_t word = partial_word(a, c);
  st_sc1_u64(A.gran + (size_t)r * kSmallMaxG * kFusedWords + (size_t)k * words + c,
             ((unsigned long long)epoch << 32) | word);
}

__device__ __forceinline__ float rfl(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ double rfl(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void uniform_consts(ElemConsts& c) {
  c.mean = rfl(c.mean);
  c.sd = rfl(c.sd);
  c.sc = rfl(c.sc);
  c.inv_sc = rfl(c.inv_sc);
  c.inv_sc32 = rfl(c.inv_sc32);
  c.zh = rfl(c.zh);
  c.zl = rfl(c.zl);
}

// The element transform of the registers (smart.py:154-182) and their stores. PRE: the rounding
// draws uu were computed ahead (during the gather); DL > 0: those of groups u < DL likewise, but
// they wait in LDS (park[(VP + u) * kSmallT + t], behind the VP parked groups); else they are
// hashed here.
template <int RM, int V, int TIN, bool AP, bool SUB, bool PRE, int DL = 0>
__device__ __forceinline__ uint32_t fused_transform(const FusedArgs& A, const float4 (&vr)[V],
                                                    const float4* park, const float (&uu)[V][4],
                                                    const ElemConsts& c, int64_t base,
                                                    uint64_t off) {
  constexpr int VR = V < 4 ? V : 4;
  uint32_t n_out = 0;
  float4* __restrict__ y4 = reinterpret_cast<float4*>(A.y);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int64_t j = base + (int64_t)u * kSmallT;
    if (j >= A.nv) continue;
    const float4 x4 = u < VR ? vr[u] : park[(u - VR) * kSmallT + threadIdx.x];
    float u0 = uu[u][0], u1 = uu[u][1], u2 = uu[u][2], u3 = uu[u][3];
    if (u < DL) {
      const float4 w = park[((V > 4 ? V - 4 : 0) + u) * kSmallT + threadIdx.x];
      u0 = w.x;
      u1 = w.y;
      u2 = w.z;
      u3 = w.w;
    } else if (RM == kRoundHash && !PRE) {
      rng_hu4(A.key, off + ((uint64_t)j << 2), u0, u1, u2, u3);
    }
    bool b0, b1, b2, b3;
    float4 o;
    o.x = smaq_elem<RM, false, TIN, AP, SUB, false>(x4.x, u0, c, b0);
    o.y = smaq_elem<RM, false, TIN, AP, SUB, false>(x4.y, u1, c, b1);
    o.z = smaq_elem<RM, false, TIN, AP, SUB, false>(x4.z, u2, c, b2);
    o.w = smaq_elem<RM, false, TIN, AP, SUB, false>(x4.w, u3, c, b3);
    n_out += (unsigned)b0 + (unsigned)b1 + (unsigned)b2 + (unsigned)b3;
    store_stream(y4 + j, o);
  }
  return n_out;
}

template <int RM, int TIN, bool AP, bool SUB>
__device__ __forceinline__ uint32_t fused_tail(const FusedArgs& A, const ElemConsts& c,
                                               uint64_t off) {
  const int64_t e = (A.nv << 2) + threadIdx.x;
  const float u = RM == kRoundHash ? rng_hu(A.key, off + (uint64_t)e) : 0.0f;
  bool bt;
  A.y[e] = smaq_elem<RM, false, TIN, AP, SUB, false>(load1<TIN>(A.x, e), u, c, bt);
  return (uint32_t)bt;
}

// ------------------------------------------------------------------------------------------------
// PACK: the single launch that also writes the call's packed stream (smq_smaq_roundtrip_compress:
// PackedActivations' forward call, util/pytorch/saved.py; format: include/smq.h "Packed SmaQ
// container"). Group u of workgroup b IS block b * V + u of the format (4096 elements, thread t
// holding elements 4t .. 4t+3 of it, wave w its rank segment w), so right after the transform has
// computed a group's codes (the apply's own smaq_quant) the workgroup builds the block from
// registers: the outlier mask (DPP group ORs), the wm-bit code plane (LDS ORs) -> the fixed section
// at its index-determined place; the outlier bits above the plane and the escapes (wave scans + the
// 16 segment counts) -> the block's variable section, kept in LDS. After its V blocks the workgroup
// publishes their total size as ONE epoch-tagged granule (the statistics granules' epoch: no
// clearing), sums the granules of the workgroups before it (dispatched earlier: no co-residency
// assumption) and stores its sections and directory entries at that prefix; the last workgroup
// writes the header. The stream is byte for byte the one the look-back packer
// (smaq_pack_lb_kernel) writes after the same round trip — x is read once for y AND the stream.
// ------------------------------------------------------------------------------------------------
// Escapes a block's LDS section holds: every element up to 3 groups per lane (the dynamic LDS is
// free there), kPkEscV4 at 4 (the rounding draws hold 64 KiB of it); a block with more is re-coded
// from x into its place.
constexpr int kPkEscV4 = 256;
__host__ __device__ inline uint32_t pk_esc_cap(int V) { return V <= 3 ? (uint32_t)kPB : (uint32_t)kPkEscV4; }
__host__ __device__ inline uint32_t pk_var_words(int we, int V) {
  return 128u * (uint32_t)we + 2u * pk_esc_cap(V);
}
// pack area (words): two fixed images (mask + plane), the 16 segment counts, 4 x 4 words of block
// meta, 4 uint64 of the prefix reduction, 4 x 16 wave totals, then the V variable sections
// (outlier bits, escapes)
__host__ __device__ inline uint32_t pk_seg_off(int wm) { return 2u * fixed_words(wm); }
__host__ __device__ inline uint32_t pk_meta_off(int wm) { return pk_seg_off(wm) + kSegs; }
__host__ __device__ inline uint32_t pk_red_off(int wm) { return pk_meta_off(wm) + 16u; }
__host__ __device__ inline uint32_t pk_tot_off(int wm) { return pk_red_off(wm) + 8u; }
__host__ __device__ inline uint32_t pk_var_off(int wm) { return pk_tot_off(wm) + 64u; }
__host__ __device__ inline uint32_t pk_lds_words(int wm, int we, int V) {
  return pk_var_off(wm) + (uint32_t)V * pk_var_words(we, V);
}

// Block B's variable section re-coded from x straight to dst (a block with more escapes than its
// LDS section holds): 4 passes of 1024 consecutive elements, outlier / escape ranks by wave ballots
// and the passes' running totals (smaq_pack.hip recode_var_section for a 1024-thread workgroup).
// ext: 128 * we words of LDS, s_cnt: 16 words.
template <int RM, int TIN>
__device__ __forceinline__ void fused_recode(const FusedArgs& A, const ElemConsts& c, uint64_t off,
                                          uint32_t B, uint32_t* dst, uint32_t* ext,
                                          uint32_t* s_cnt, int wm, int wo) {
  const int we = wo > wm ? wo - wm : 0;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int64_t e0 = (int64_t)B * kPB;
  const int n_el = (int)min((int64_t)kPB, A.n - e0);
  const uint32_t hm = 1u << (wm - 1), side = 1u << (wo - 1);
  for (uint32_t i = tid; i < 128u * (uint32_t)we; i += kSmallT) ext[i] = 0u;
  __syncthreads();
  uint32_t n_out = 0u;
#pragma unroll 1
  for (int pass = we > 0 ? 0 : 1; pass < 2; ++pass) {
    uint32_t r_out = 0u, r_esc = 0u;
    uint32_t* out = dst + ext_words(we, n_out);
#pragma unroll 1
    for (int jj = 0; jj < kPB / kSmallT; ++jj) {
      const int el = jj * kSmallT + tid;
      bool o = false, esc = false;
      float q = 0.0f;
      uint32_t code = 0u;
      if (el < n_el) {
        const float u = (RM == kRoundHash) ? rng_hu(A.key, off + (uint64_t)(e0 + el)) : 0.0f;
        bool hi, lo;
        q = smaq_quant<RM, false, TIN, true>(load1<TIN>(A.x, e0 + el), u, c, hi, lo);
        o = hi | lo;
        code = code_sel(q, o, lo, hm, side, 2u * hm, esc);
      }
      const unsigned long long bo = __ballot(o), be = __ballot(esc);
      const uint32_t ro = __builtin_amdgcn_mbcnt_hi((uint32_t)(bo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bo, 0u));
      const uint32_t re = __builtin_amdgcn_mbcnt_hi((uint32_t)(be >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)be, 0u));
      if (lane == 0) s_cnt[w] = (uint32_t)__popcll(bo) | ((uint32_t)__popcll(be) << 16);
      __syncthreads();
      uint32_t before = 0u, tot = 0u;
#pragma unroll
      for (int v = 0; v < kSmallWaves; ++v) {
        const uint32_t t = s_cnt[v];
        before += v < w ? t : 0u;
        tot += t;
      }
      __syncthreads();
      if (pass == 1) {
        const uint32_t ko = r_out + (before & 0xffffu) + ro, ke = r_esc + (before >> 16) + re;
        if (o && we > 0) or_bits32(ext, (uint32_t)we * ko, code >> wm);
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
  for (uint32_t i = tid; i < ext_words(we, n_out); i += kSmallT) dst[i] = ext[i];
}

// The transform of the registers (fused_transform) that also packs every group as its block.
// Returns the outliers counted (the log_size count, as fused_transform).
template <int RM, int V, int TIN, bool AP, bool SUB, bool PRE, int DL, int WM, int WO>
__device__ __forceinline__ uint32_t fused_transform_pack(const FusedArgs& A, const float4 (&vr)[V],
                                                         const float4* park, const float (&uu)[V][4],
                                                         const ElemConsts& c, int64_t base,
                                                         uint64_t off, uint32_t* pk,
                                                         uint32_t epoch) {
  constexpr int VR = V < 4 ? V : 4;
  constexpr int kWE = (WM > 0 && WO > 0) ? (WO > WM ? WO - WM : 0) : -1;
  const int wm = WM > 0 ? WM : A.bm - 1, wo = WO > 0 ? WO : A.bo - 1;
  const int we = kWE >= 0 ? kWE : (wo > wm ? wo - wm : 0);
  const uint32_t F = fixed_words(wm), VA = pk_var_words(we, V);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  uint32_t* seg = pk + pk_seg_off(wm);
  uint32_t* meta = pk + pk_meta_off(wm);  // [4][4]: words, n_out | n_esc << 16, fits
  const uint32_t pmask = (1u << wm) - 1u;
  const uint32_t hm = 1u << (wm - 1), side = 1u << (wo - 1), lim_m = 2u * hm;
  const uint32_t msh = 4u * (uint32_t)(lane & 7);
  const bool mwriter = (lane & 7) == 7;
  const uint32_t ppos0 = 4u * (uint32_t)wm * (uint32_t)tid;
  const uint32_t pw0 = ppos0 >> 5, psft = ppos0 & 31u;
  uint32_t n_out_all = 0;
  float4* __restrict__ y4 = reinterpret_cast<float4*>(A.y);
  // Phase A: every group's codes and its blocks' sizes first, so the workgroup's aggregate goes
  // out before the stream is built — the wait for the predecessors' aggregates then overlaps the
  // y stores and the block images (phase B). q and the sides stay in registers between the phases.
  float qa[V][4];
  uint32_t hla[V];  // bit i: z > T of element i, bit 4 + i: z < -T
  uint32_t* tots = pk + pk_tot_off(wm);  // [V][16] wave totals: outliers | escapes << 16
#pragma unroll
  for (int u = 0; u < V; ++u) {
    hla[u] = 0u;
    qa[u][0] = qa[u][1] = qa[u][2] = qa[u][3] = 0.0f;
    const uint32_t B = (uint32_t)blockIdx.x * (uint32_t)V + (uint32_t)u;
    if (B >= A.pk.n_blocks) break;  // (uniform: the grid's last workgroup may hold fewer blocks)
    const int64_t j = base + (int64_t)u * kSmallT;
    const bool valid = j < A.nv;
    const float4 x4 = u < VR ? vr[u] : park[(u - VR) * kSmallT + threadIdx.x];
    float u0 = uu[u][0], u1 = uu[u][1], u2 = uu[u][2], u3 = uu[u][3];
    if (u < DL) {
      const float4 wv = park[((V > 4 ? V - 4 : 0) + u) * kSmallT + threadIdx.x];
      u0 = wv.x;
      u1 = wv.y;
      u2 = wv.z;
      u3 = wv.w;
    } else if (RM == kRoundHash && !PRE) {
      rng_hu4(A.key, off + ((uint64_t)j << 2), u0, u1, u2, u3);
    }
    const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
    const float us[4] = {u0, u1, u2, u3};
    uint32_t cnt = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hi, lo, esc;
      qa[u][i] = smaq_quant<RM, false, TIN, SUB>(xs[i], us[i], c, hi, lo);
      hla[u] |= (hi ? 1u << i : 0u) | (lo ? 16u << i : 0u);
      (void)code_sel(qa[u][i], hi | lo, lo, hm, side, lim_m, esc);
      cnt += valid ? ((hi | lo) ? 1u : 0u) + (esc ? 0x10000u : 0u) : 0u;
    }
    const uint32_t wt = wave_sum_u32(cnt);
    if (lane == 0) tots[16 * u + w] = wt;
  }
  lds_barrier();
  if (tid == 0 && blockIdx.x + 1 < A.G) {  // (the last workgroup's aggregate is nobody's prefix)
    uint32_t agg = 0u;
    for (int u = 0; u < V; ++u) {
      if ((uint32_t)blockIdx.x * (uint32_t)V + (uint32_t)u >= A.pk.n_blocks) break;
      uint32_t t = 0u;
#pragma unroll
      for (int ww = 0; ww < kSmallWaves; ++ww) t += tots[16 * u + ww];
      agg += ext_words(we, t & 0xffffu) + 2u * (t >> 16);
    }
    st_sc1_u64(A.pk.look + blockIdx.x, ((unsigned long long)epoch << 32) | agg);
  }
  // Phase B: per block, y and the block's image from the registers
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const uint32_t B = (uint32_t)blockIdx.x * (uint32_t)V + (uint32_t)u;
    if (B >= A.pk.n_blocks) break;
    const int64_t j = base + (int64_t)u * kSmallT;
    const bool valid = j < A.nv;
    float ys[4];
    uint32_t code[4], on = 0u, en = 0u;
    float qv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool esc;
      const bool hi = (hla[u] >> i) & 1u, lo = (hla[u] >> (4 + i)) & 1u;
      qv[i] = qa[u][i];
      ys[i] = smaq_dequant<false, AP, false, false>(qv[i], hi, lo, c);
      const bool o = hi | lo;
      code[i] = valid ? code_sel(qv[i], o, lo, hm, side, lim_m, esc) : 0u;
      on |= (valid && o) ? (1u << i) : 0u;
      en |= (valid && esc) ? (1u << i) : 0u;
    }
    if (valid) {
      store_stream(y4 + j, make_float4(ys[0], ys[1], ys[2], ys[3]));
      n_out_all += (uint32_t)__popc(on);
    }
    uint32_t* img = pk + (uint32_t)(u & 1) * F;
    uint32_t* mask = img;
    uint32_t* plane = img + kMaskWords;
    uint32_t* var = pk + pk_var_off(wm) + (uint32_t)u * VA;
    // outlier mask: the nibbles of 8 consecutive lanes make a word
    const uint32_t mw = group8_or_to_last(on << msh);
    if (mwriter) mask[tid >> 3] = mw;
    // plane: the low wm bits of the 4 codes at bit wm * 4t
    if (4 * wm <= 32) {
      uint32_t ch = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) ch |= (code[i] & pmask) << (wm * i);
      atomicOr(plane + pw0, ch << psft);
      if (psft + 4u * (uint32_t)wm > 32u) atomicOr(plane + pw0 + 1, ch >> (32u - psft));
    } else if (wm <= 16) {
      uint64_t ch = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) ch |= (uint64_t)(code[i] & pmask) << (wm * i);
      if (ch) or_bits64(plane, ppos0, ch);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const uint64_t ch = (uint64_t)(code[i] & pmask) | ((uint64_t)(code[i + 1] & pmask) << wm);
        if (ch) or_bits64(plane, (uint32_t)wm * (uint32_t)(4 * tid + i), ch);
      }
    }
    // outlier bits above the plane, in element order
    uint64_t ech = 0u;
    uint32_t ev[4] = {0u, 0u, 0u, 0u};
    if (we > 0) {
      if (4 * we <= 32) {
        const uint32_t s1 = (uint32_t)we * (on & 1u);
        const uint32_t s2 = (uint32_t)we * (uint32_t)__popc(on & 3u);
        const uint32_t s3 = (uint32_t)we * (uint32_t)__popc(on & 7u);
        ech = (code[0] >> wm) | ((code[1] >> wm) << s1) | ((code[2] >> wm) << s2) |
              ((code[3] >> wm) << s3);
      } else if (we <= 16) {
        uint32_t sft = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((on >> i) & 1u) {
            ech |= (uint64_t)(code[i] >> wm) << sft;
            sft += (uint32_t)we;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) ev[i] = code[i] >> wm;
      }
    }
    const uint32_t cnt = (uint32_t)__popc(on) | ((uint32_t)__popc(en) << 16);
    const uint32_t incl = wave_incl_scan_u32(cnt);
    const uint32_t pre = incl - cnt;
    if (lane == kWave - 1) seg[w] = incl;
    uint32_t gfirst = 0u;
    if (kWE == 2) {  // the 8 lanes of a group own consecutive ranks: one run in the last lane
      const uint32_t po = pre & 0xffffu;
      gfirst = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane & ~7), (int)po);
      const uint64_t ch = (uint64_t)(uint32_t)ech << (2u * (po - gfirst));
      const uint32_t glo = group8_or_to_last((uint32_t)ch), ghi = group8_or_to_last((uint32_t)(ch >> 32));
      ech = ((uint64_t)ghi << 32) | glo;
    }
    lds_barrier();
    // the other image's plane for the next block (its last reader, block u - 1's fixed store, is
    // behind the barrier above; its first writer, block u + 1, behind the one below)
    if (u + 1 < V) {
      uint32_t* np = pk + (uint32_t)((u + 1) & 1) * F + kMaskWords;
      for (uint32_t i = tid; i < 128u * (uint32_t)wm; i += kSmallT) np[i] = 0u;
    }
    // segment bases (lanes 0-15 of every wave scan the 16 counts by DPP row shifts)
    const uint32_t own = lane < kSegs ? seg[lane] : 0u;
    uint32_t sincl = own;
    sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x111, 0xf, 0xf, false);
    sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x112, 0xf, 0xf, false);
    sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x114, 0xf, 0xf, false);
    sincl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sincl, 0x118, 0xf, 0xf, false);
    const uint32_t sexcl = sincl - own;
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)sincl, kSegs - 1);
    const uint32_t n_o = tot & 0xffffu, n_e = tot >> 16;
    const uint32_t n_ext = ext_words(we, n_o);
    const bool fits = n_e <= pk_esc_cap(V);
    const uint32_t sbase = (uint32_t)__builtin_amdgcn_readlane((int)sexcl, w);
    if (we > 0 && (kWE == 2 || on)) {
      if (kWE == 2) {
        if (mwriter && ech) or_bits64(var, 2u * ((sbase & 0xffffu) + gfirst), ech);
      } else {
        const uint32_t r_out = (sbase + pre) & 0xffffu;
        if (4 * we <= 32) {
          or_bits32(var, (uint32_t)we * r_out, (uint32_t)ech);
        } else if (we <= 16) {
          or_bits64(var, (uint32_t)we * r_out, ech);
        } else {
          uint32_t r = r_out;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if ((on >> i) & 1u) or_bits64(var, (uint32_t)we * r++, ev[i]);
        }
      }
    }
    // escapes (their q still in registers): each straight to its rank in the block's list
    if (__builtin_expect(en != 0u, 0) && fits) {
      uint32_t r = (sbase >> 16) + (pre >> 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((en >> i) & 1u) {
          const float qe = qv[i];
          var[n_ext + 2u * r] = 4u * (uint32_t)tid + (uint32_t)i;
          var[n_ext + 2u * r + 1u] = qe == qe ? __float_as_uint(qe) : 0x7fc00000u;
          ++r;
        }
      }
    }
    if (tid == 0) {
      meta[4 * u] = n_ext + 2u * n_e;
      meta[4 * u + 1] = n_o | (n_e << 16);
      meta[4 * u + 2] = fits ? 1u : 0u;
    }
    lds_barrier();
    // the fixed section (mask + plane, F words) at B * F, 16-B stores
    uint4* fdst = reinterpret_cast<uint4*>(A.pk.fixed + (size_t)B * F);
    const uint4* fsrc = reinterpret_cast<const uint4*>(img);
    for (uint32_t i = tid; i < F / 4u; i += kSmallT) fdst[i] = fsrc[i];
  }
  return n_out_all;
}

// After the transform: the workgroup's blocks' variable sections and directory entries at the
// prefix of the workgroups before it, the header by the last one.
template <int RM, int V, int TIN>
__device__ __forceinline__ void fused_pack_finish(const FusedArgs& A, const ElemConsts& c,
                                                  uint64_t off, uint32_t epoch,
                                                  const SmqSmaqStats& st, uint32_t* pk) {
  const int wm = A.bm - 1, wo = A.bo - 1, we = wo > wm ? wo - wm : 0;
  const uint32_t VA = pk_var_words(we, V);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const int b = blockIdx.x, G = A.G;
  const uint32_t* meta = pk + pk_meta_off(wm);
  unsigned long long* s_red = reinterpret_cast<unsigned long long*>(pk + pk_red_off(wm));
  const uint32_t B0 = (uint32_t)b * (uint32_t)V;
  const int nbk = (int)min((uint32_t)V, A.pk.n_blocks - B0);
  // the aggregates of workgroups 0 .. b-1 (dispatched before this one; published by their phase
  // A, fused_transform_pack), one per thread
  unsigned long long v = 0ull;
  if (tid < b) {
    for (;;) {
      const unsigned long long g = ld_sc1_u64(A.pk.look + tid);
      if ((uint32_t)(g >> 32) == epoch) {
        v = g & 0xffffffffull;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (b > 0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    if (lane == 0 && w < 4) s_red[w] = v;  // (b < 256: waves 0-3 hold the aggregates)
  }
  lds_barrier();
  uint64_t vb = b > 0 ? (uint64_t)(s_red[0] + s_red[1] + s_red[2] + s_red[3]) : 0ull;
  for (int u = 0; u < nbk; ++u) {
    const uint32_t B = B0 + (uint32_t)u;
    const uint32_t words = meta[4 * u], cnt = meta[4 * u + 1];
    if (tid == 0)
      A.pk.dir[B] = vb | ((uint64_t)(cnt & 0xffffu) << 38) | ((uint64_t)(cnt >> 16) << 51);
    if (vb + words <= A.pk.cap_words) {  // (a capacity-bounded stream: sections past it unwritten)
      uint32_t* src = pk + pk_var_off(wm) + (uint32_t)u * VA;
      uint32_t* dst = A.pk.var + vb;
      if (meta[4 * u + 2]) {
        for (uint32_t i = tid; i < words; i += kSmallT) dst[i] = src[i];
      } else {  // more escapes than its LDS section holds: re-coded from x (its area as scratch)
        fused_recode<RM, TIN>(A, c, off, B, dst, src, pk + pk_seg_off(wm), wm, wo);
      }
    }
    vb += words;
  }
  if (b == G - 1 && tid == 0) {  // every workgroup's aggregate is in vb: the header
    SmqPackedHeader* h = A.pk.hdr;
    h->magic = SMQ_PACK_MAGIC;
    h->version = SMQ_PACK_VERSION;
    h->n = A.n;
    h->block_elems = kPB;
    h->n_blocks = A.pk.n_blocks;
    h->num_bits_main = A.bm;
    h->num_bits_outlier = A.bo;
    h->flags = A.pk.flags;
    h->thr = A.thr;
    h->range_main = A.r_main;
    h->range_outlier = A.r_out;
    h->mean = st.mean;
    h->std_dev = st.std_dev;
    h->inv_range_main = A.inv_r_main;
    h->inv_range_outlier = A.inv_r_out;
    h->data_words = vb;
    h->total_bytes = sizeof(SmqPackedHeader) + 8ull * dir_entries(A.pk.n_blocks) +
                     4ull * A.pk.n_blocks * fixed_words(wm) + 4ull * vb;
    notify_total(A.pk.notify, h->total_bytes);
    h->error = 0u;
    h->bn_channels = 0u;
    h->bn_inner = 0;
    h->mean_f64 = 0.0;
    h->std_dev_f64 = 0.0;
    h->reserved[0] = h->reserved[1] = 0u;
    if (A.pk.n_blocks & 1u) A.pk.dir[A.pk.n_blocks] = 0ull;  // the directory's padding entry
  }
}

template <int RM, int V, int TIN, bool PACK = false, int PWM = 0, int PWO = 0>
__global__ __launch_bounds__(kSmallT) void smaq_fused_kernel(FusedArgs A) {
  __shared__ SmallWaveLds W;
  __shared__ SmqSmaqStats sst;
  __shared__ float4 u0lds[V <= 4 ? V : 1][kWave];  // wave 0's rounding draws (PRE)
  __shared__ uint32_t sh_cnt[kSmallWaves];
  // the gathered partials' words, word c of partial k = 4l + q at (4c + q) * 64 + l: the reduction's
  // lane l reads them bank-conflict free
  __shared__ uint32_t pw[kSmallMaxG * kFusedWords];
  __shared__ int smiss[kSmallWaves];
  const int b = blockIdx.x, G = A.G;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t base = (int64_t)b * V * kSmallT + threadIdx.x;
  const uint64_t steal_ticks = A.test_late ? 2000 : kFusedStealTicks;
  FSTAMP(0);
  if (A.zero && b == 0)
    for (uint32_t i = threadIdx.x; i < A.zero_n; i += kSmallT) A.zero[i] = 0u;
  if (A.test_late && 2 * b >= G && G > 1) {  // test aid: half of the grid starts ~500 us late
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 50000) __builtin_amdgcn_s_sleep(127);
  }
  // this chunk into registers (branch-free: indices past the end re-read the last group and are
  // ignored), so every load is in flight before the first wait
  float4 v[V];
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int64_t j = base + (int64_t)u * kSmallT;
    v[u] = load4<TIN>(A.x, j < A.nv ? j : A.nv - 1);
  }
  // groups VR .. V-1 wait in LDS (dynamic, park[(u - VR) * kSmallT + t]) once the statistics have
  // consumed them: registers for more than four groups would spill across the gather
  constexpr int VR = V < 4 ? V : 4;
  extern __shared__ float4 park[];
  uint32_t* pk = reinterpret_cast<uint32_t*>(park) + A.pk.lds_off;  // (PACK)
  if constexpr (PACK) {  // the planes and outlier-bit areas are built by ORs: zero, loads in flight
    const int wm = A.bm - 1, we = A.bo > A.bm ? A.bo - A.bm : 0;
    uint32_t* plane0 = pk + kMaskWords;  // (image 1's plane: in block 0's iteration)
    for (uint32_t i = threadIdx.x; i < 128u * (uint32_t)wm; i += kSmallT) plane0[i] = 0u;
    for (int u = 0; u < V; ++u) {
      uint32_t* ext = pk + pk_var_off(wm) + (uint32_t)u * pk_var_words(we, V);
      for (uint32_t i = threadIdx.x; i < 128u * (uint32_t)we; i += kSmallT) ext[i] = 0u;
    }
  }
  const double shift = stats_shift<TIN>(A.x, A.n);
  const uint32_t gen = G > 1 ? ld_sc1_u32(A.gen) : 0u;
  const uint64_t ctr_word = A.ctr ? ld_sc1_u64(A.ctr) : 0ull;
  const uint64_t off0 = ctr_word;
  const uint32_t epoch = (gen << 1) | 1u;
  // materialised here: both reads have returned before this workgroup can be counted past the
  // wait (after which the last workgroup may advance them)
  asm volatile("" ::"v"(off0), "v"(epoch));
  const uint64_t off = A.offset + off0;

  const StatAcc part = fused_partial<TIN, V>(A, b, v, shift, W);
  FSTAMP(1);
#pragma unroll
  for (int u = VR; u < V; ++u) park[(u - VR) * kSmallT + threadIdx.x] = v[u];
  if (G > 1 && wave == 0) fused_publish(part, A, b, epoch);

  // the rounding draws depend on the stream position only: every wave computes its own now (wave
  // 0's by waves 4..4+V-1, handed over in LDS), before it polls for the partials. Above 3
  // groups per lane they would hold 4V more VGPRs across the gather: at V = 4 they wait in the
  // (then unused) parking LDS instead, above it they are hashed in the transform.
  constexpr bool PRE = RM == kRoundHash && V <= 3;
  constexpr int DL = RM == kRoundHash ? fused_draw_groups(V) : 0;
  constexpr int VP = V > 4 ? V - 4 : 0;
  float uu[V][4];
#pragma unroll
  for (int u = 0; u < V; ++u) uu[u][0] = uu[u][1] = uu[u][2] = uu[u][3] = 0.0f;
  if (PRE && wave != 0) {
#pragma unroll
    for (int u = 0; u < V; ++u)
      rng_hu4(A.key, off + ((uint64_t)(base + (int64_t)u * kSmallT) << 2), uu[u][0], uu[u][1],
              uu[u][2], uu[u][3]);
    if (wave >= 4 && wave < 4 + V) {
      const int u = wave - 4;
      float4 w;
      rng_hu4(A.key, off + ((uint64_t)((int64_t)b * V * kSmallT + lane + (int64_t)u * kSmallT) << 2),
              w.x, w.y, w.z, w.w);
      u0lds[u][lane] = w;
    }
  }
  if (DL > 0) {  // (the launcher gives V >= 4 the dynamic LDS whatever G is)
    if (wave != 0) {
#pragma unroll
      for (int u = 0; u < DL; ++u) {
        float4 w;
        rng_hu4(A.key, off + ((uint64_t)(base + (int64_t)u * kSmallT) << 2), w.x, w.y, w.z, w.w);
        park[(VP + u) * kSmallT + threadIdx.x] = w;
      }
    }
    if (wave >= 4 && wave < 4 + DL) {  // wave 0's slot u
      const int u = wave - 4;
      float4 w;
      rng_hu4(A.key, off + ((uint64_t)((int64_t)b * V * kSmallT + lane + (int64_t)u * kSmallT) << 2),
              w.x, w.y, w.z, w.w);
      park[(VP + u) * kSmallT + lane] = w;
    }
  }

  unsigned long long left_old = 0;
  if (G > 1) {
    // every thread gathers the words t and t + 1024 of replica b % 8 (G * words words, dense:
    // partial k's word c at k * words + c), so each wave load reads 512 consecutive bytes, until
    // every granule carries the epoch; accepted words go to LDS (pw). One loop for the whole
    // workgroup: each wave waits (the first time until its words are there or its patience runs
    // out, afterwards one pass); a partial still missing then is computed by the whole workgroup
    // from memory and published, and the waves look again.
    const int words = A.range ? 6 : 4;
    const int total = G * words;
    const unsigned long long* rep =
        A.gran + (size_t)(b % kFusedRep) * kSmallMaxG * kFusedWords;
    const int i0 = threadIdx.x, i1 = threadIdx.x + kSmallT;
    uint32_t miss_bits = (i0 < total ? 1u : 0u) | (i1 < total ? 2u : 0u);
    // partial and word of granule i (i / words without a division: i < 1536), and its LDS slot
    auto part_of = [&](int i) { return words == 4 ? i >> 2 : (i * 43691) >> 18; };
    auto slot_of = [&](int i) {
      const int k = part_of(i), c = i - k * words;
      return ((c << 2) + (k & 3)) * kWave + (k >> 2);
    };
    const int sl0 = slot_of(i0), sl1 = slot_of(i1);
    bool stealing = false;
    for (;;) {
      const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
      uint32_t polls = 0;
      for (;;) {
        const unsigned long long g0 = (miss_bits & 1u) ? ld_sc1_u64(rep + i0) : 0ull;
        const unsigned long long g1 = (miss_bits & 2u) ? ld_sc1_u64(rep + i1) : 0ull;
        if ((miss_bits & 1u) && (uint32_t)(g0 >> 32) == epoch) {
          miss_bits &= ~1u;
          pw[sl0] = (uint32_t)g0;
        }
        if ((miss_bits & 2u) && (uint32_t)(g1 >> 32) == epoch) {
          miss_bits &= ~2u;
          pw[sl1] = (uint32_t)g1;
        }
        if (__all(miss_bits == 0u) || stealing) break;
        if ((++polls & 7) != 0) {
          fused_sleep(A.poll_sleep);
          continue;
        }
        if (__builtin_amdgcn_s_memrealtime() - t_start > steal_ticks) break;
        fused_sleep(A.poll_sleep);
      }
      // the first missing partial after b (cyclically)
      int miss = INT_MAX;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (!((miss_bits >> h) & 1u)) continue;
        const int k = part_of(h ? i1 : i0);
        int d = k - b;
        d += d < 0 ? G : 0;
        miss = min(miss, d);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) miss = min(miss, __shfl_xor(miss, o, kWave));
      if (lane == 0) smiss[wave] = miss;
      lds_barrier();
      int m = smiss[0];
#pragma unroll
      for (int w = 1; w < kSmallWaves; ++w) m = min(m, smiss[w]);
      if (m == INT_MAX) break;
      // the patience ran out: compute partial (m + b) % G from memory (one group per lane in
      // flight) and publish it
      const int k = m + b < G ? m + b : m + b - G;
      stealing = true;
      const StatAcc pk_acc = fused_steal<TIN>(A.x, A.n, V, G, k, shift, &W);
      if (wave == 0) fused_publish(pk_acc, A, k, epoch);
      // its words need no poll here (and the others' next pass may precede the stores)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = h ? i1 : i0;
        const int c = i - k * words;
        if (((miss_bits >> h) & 1u) && c >= 0 && c < words) {
          pw[h ? sl1 : sl0] = partial_word(pk_acc, c);
          miss_bits &= ~(1u << h);
        }
      }
    }
    FSTAMP(2);
    // count this workgroup past the wait now, on its residue's word (eight words of <= 32 arrivals
    // each instead of one word of 256: same-address atomics serialise at ~12 ns each); the
    // returned word is looked at only after the transform
    if (threadIdx.x == kArriveThread) left_old = arrive_tagged_issue(A.sub + (b & 7) * kSubStride);
    if (wave == 0) {
      // reduce_partials_w0's order: lane l adds partials 4l .. 4l+3 from 0.0, then one ascending
      // butterfly
      double s1 = 0.0, s2 = 0.0;
      float mn = INFINITY, mx = -INFINITY;
      // every word read first (one LDS round trip instead of one per partial; the words of
      // partials >= G are not used), then the adds in the same order, skipped ones as selects
      uint32_t wd[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) wd[q][c] = pw[(4 * c + q) * kWave + lane];  // word c at w[4c * 64]
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = 4 * lane + q < G;
        const double a1 = __builtin_bit_cast(double, ((uint64_t)wd[q][1] << 32) | wd[q][0]);
        const double a2 = __builtin_bit_cast(double, ((uint64_t)wd[q][3] << 32) | wd[q][2]);
        s1 = ok ? s1 + a1 : s1;
        s2 = ok ? s2 + a2 : s2;
      }
      if (A.range) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (4 * lane + q >= G) continue;
          const uint32_t* w = pw + q * kWave + lane;
          mn = fminf(mn, __builtin_bit_cast(float, w[16 * kWave]));
          mx = fmaxf(mx, __builtin_bit_cast(float, w[20 * kWave]));
        }
      }
      FSTAMP(10);
      s1 = wave_sum_asc(s1);
      s2 = wave_sum_asc(s2);
      if (A.range) {
        mn = wave_min_dpp(mn);
        mx = wave_max_dpp(mx);
      }
      FSTAMP(8);
      if (lane == 0) {
        const FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, nullptr, 0};
        SmqSmaqStats st;
        if (A.range) finalize_stats<true, TIN>(s1, s2, mn, mx, A.n, shift, false, f, &st);
        else finalize_stats<false, TIN>(s1, s2, mn, mx, A.n, shift, false, f, &st);
        st.rng_offset = off0;
        sst = st;
        FSTAMP(9);
        if (b == 0) *A.hdr = st;
      }
    }
  } else if (threadIdx.x == 0) {  // one chunk: the partial is the total
    const FinalizeArgs f{A.clamp_lo, A.clamp_hi, A.range_coef, nullptr, 0};
    SmqSmaqStats st;
    if (A.range) finalize_stats<true, TIN>(part.s1, part.s2, part.mn, part.mx, A.n, shift, false, f, &st);
    else finalize_stats<false, TIN>(part.s1, part.s2, part.mn, part.mx, A.n, shift, false, f, &st);
    st.rng_offset = off0;
    sst = st;
    *A.hdr = st;
    if (A.ctr) st_sc1_u64(A.ctr, off0 + (uint64_t)A.n);
  }
  lds_barrier();
  if (PRE && wave == 0) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const float4 w = u0lds[u][lane];
      uu[u][0] = w.x;
      uu[u][1] = w.y;
      uu[u][2] = w.z;
      uu[u][3] = w.w;
    }
  }
  FSTAMP(3);
  ElemConsts c;
  const float cthr = TIN == kF32 ? A.thr : round_in<TIN>(A.thr);
  init_consts(c, &sst, A.thr, A.r_main, A.r_out, A.inv_r_main, A.inv_r_out, cthr);
  uniform_consts(c);  // LDS reads land in VGPRs: the constants are wave-uniform, keep them in SGPRs
  const bool tail = b == G - 1 && threadIdx.x < (int)(A.n & 3);
  uint32_t n_out;
  if constexpr (PACK) {
    if (sst.quot_check) {
      n_out = A.all_pos
                  ? fused_transform_pack<RM, V, TIN, true, true, PRE, DL, PWM, PWO>(A, v, park, uu, c, base, off, pk, epoch)
                  : fused_transform_pack<RM, V, TIN, false, true, PRE, DL, PWM, PWO>(A, v, park, uu, c, base, off, pk, epoch);
    } else {
      n_out = A.all_pos
                  ? fused_transform_pack<RM, V, TIN, true, false, PRE, DL, PWM, PWO>(A, v, park, uu, c, base, off, pk, epoch)
                  : fused_transform_pack<RM, V, TIN, false, false, PRE, DL, PWM, PWO>(A, v, park, uu, c, base, off, pk, epoch);
    }
  } else if (sst.quot_check) {
    if (A.all_pos) {
      n_out = fused_transform<RM, V, TIN, true, true, PRE, DL>(A, v, park, uu, c, base, off);
      if (tail) n_out += fused_tail<RM, TIN, true, true>(A, c, off);
    } else {
      n_out = fused_transform<RM, V, TIN, false, true, PRE, DL>(A, v, park, uu, c, base, off);
      if (tail) n_out += fused_tail<RM, TIN, false, true>(A, c, off);
    }
  } else {
    if (A.all_pos) {
      n_out = fused_transform<RM, V, TIN, true, false, PRE, DL>(A, v, park, uu, c, base, off);
      if (tail) n_out += fused_tail<RM, TIN, true, false>(A, c, off);
    } else {
      n_out = fused_transform<RM, V, TIN, false, false, PRE, DL>(A, v, park, uu, c, base, off);
      if (tail) n_out += fused_tail<RM, TIN, false, false>(A, c, off);
    }
  }
  FSTAMP(4);
#if SMQ_FUSED_TRACE
  if (A.trace && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    A.trace[(size_t)blockIdx.x * 16 + 5] = __builtin_amdgcn_s_memrealtime();
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    A.trace[(size_t)blockIdx.x * 16 + 6] = xcc;
  }
#endif
  if (A.count) {  // outlier count for log_size (smart.py:184-188), spread over the slots
    const uint32_t t = wave_sum_u32(n_out);
    if (lane == 0) sh_cnt[wave] = t;
    lds_barrier();
    if (threadIdx.x == 0) {
      unsigned long long s = 0;
#pragma unroll
      for (int w = 0; w < kSmallWaves; ++w) s += sh_cnt[w];
      if (A.rec_gran && G > 1) {  // one epoch-tagged granule; the call's last workgroup sums them
        st_sc1_u64(A.rec_gran + b, ((uint64_t)epoch << 32) | (uint32_t)s);
        smiss[1] = (int)s;  // (its own count: the last workgroup does not read its granule back)
      }
      else if (A.rec) size_record_arrive(A.rec, s, b, G, A.n, A.bm, A.bo);
      else if (s) atomicAdd(A.out_slots + (b & (SMQ_WS_OUTLIER_SLOTS - 1)), s);
    }
  }
  if constexpr (PACK) fused_pack_finish<RM, V, TIN>(A, c, off, epoch, sst, pk);
  // the last workgroup of its residue arrives on the top word; the last residue's advances the
  // generation and the stream and re-arms the arrival words. Every workgroup has read the
  // generation, the stream position and the granules before its add.
  const bool last = G > 1 && threadIdx.x == kArriveThread &&
                    arrive_sharded_finish(A.left, A.sub, kSubStride, b, G, gen, left_old);
  if (A.rec_gran && G > 1) {
    // counted call: the last workgroup (every other one is past the gather, so running: no
    // co-residency question) sums the workgroups' count granules of this epoch into the record —
    // no returning atomic at every workgroup's end
    if (threadIdx.x == kArriveThread) smiss[0] = last ? 1 : 0;
    lds_barrier();
    if (smiss[0] && wave == 0) {
      // every granule's load issued before any is looked at (one round trip, not G / 64), then
      // the missing ones polled
      constexpr int K = kSmallMaxG / kWave;
      uint64_t g[K];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int k = lane + i * kWave;
        g[i] = (k < G && k != b) ? ld_sc1_u64(A.rec_gran + k) : ((uint64_t)epoch << 32);
      }
      unsigned long long tot = lane == 0 ? (unsigned long long)(uint32_t)smiss[1] : 0ull;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int k = lane + i * kWave;
        while ((uint32_t)(g[i] >> 32) != epoch) {
          fused_sleep(1);
          g[i] = ld_sc1_u64(A.rec_gran + k);
        }
        if (k < G && k != b) tot += (uint32_t)g[i];
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, kWave);
      if (lane == 0) size_record_finish(A.rec, tot, A.n, A.bm, A.bo);
    }
  }
  if (last) {
    st_sc1_u32(A.gen, gen + 1u);
    if (A.ctr) st_sc1_u64(A.ctr, off0 + (uint64_t)A.n);
    rearm_sharded(A.left, A.sub, kSubStride, gen + 1u);
  }
  FSTAMP(7);
}

// ------------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------------
int launch_stats_small(const void* x, int dtype, int64_t n, bool vec, bool range,
                       const FinalizeArgs& fin, void* ws, hipStream_t st, bool defer,
                       int* def_g) {
  const SmallGeom g = small_geom(n);
  char* base = (char*)ws;
  SmqSmaqStats* hdr = (SmqSmaqStats*)base;
  unsigned long long* counter = (unsigned long long*)(base + SmaqWsLayout::kTagCounters);
  StatPartial* partials = (StatPartial*)(base + SmaqWsLayout::kPartials);
  double* def_rec = nullptr;
  ArriveTag tag{};
  if (defer) {
    if (def_g) *def_g = g.G > 1 ? g.G : 0;
    if (g.G > 1) def_rec = (double*)(base + SmaqWsLayout::kDeferRec);
  }
  if (!def_rec) tag = arrive_tag(ws, st);  // the tag prediction follows the calls that arrive
  const dim3 grid((unsigned)g.G), block(kSmallT);
  const int vi = vec ? 1 : 0, ri = range ? 1 : 0;
  if (dtype == SMQ_DTYPE_F32)
    hipLaunchKernelGGL(smaq_stats_small_kernel<kF32>, grid, block, 0, st, x, n, g.V, vi, ri, fin,
                       partials, counter, tag, hdr, def_rec);
  else if (dtype == SMQ_DTYPE_F16)
    hipLaunchKernelGGL(smaq_stats_small_kernel<kF16>, grid, block, 0, st, x, n, g.V, vi, ri, fin,
                       partials, counter, tag, hdr, def_rec);
  else
    hipLaunchKernelGGL(smaq_stats_small_kernel<kBF16>, grid, block, 0, st, x, n, g.V, vi, ri, fin,
                       partials, counter, tag, hdr, def_rec);
  return check_launch("smaq_stats_small_kernel");
}

template <int RM, int V, int TIN>
static int launch_fused_v(const FusedArgs& F, hipStream_t st) {
  // one workgroup per CU: without the LDS request two small-V workgroups could share a CU while
  // another stays idle
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&smaq_fused_kernel<RM, V, TIN>),
      hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLds);
  if (attr != hipSuccess) {
    set_error("smaq_fused_kernel: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed: %s",
              hipGetErrorString(attr));
    return SMQ_ERR_LAUNCH;
  }
  // parking (V > 4): (V - 4) * 16 KiB; the rounding draws at V = 4: 64 KiB
  const int lds = (F.G > 1 || V >= 4) ? fused_lds_bytes(V) : 0;
  static_assert(kFusedLds >= (kSmallMaxV - 4) * kSmallT * 16, "LDS parking");
  static_assert(kFusedLds >= ((V > 4 ? V - 4 : 0) + fused_draw_groups(V)) * kSmallT * 16,
                "parked groups + rounding draws");
  static_assert(kFusedLds + 8 * 1024 <= 160 * 1024, "LDS of one workgroup (static part < 8 KiB)");
  hipLaunchKernelGGL((smaq_fused_kernel<RM, V, TIN>), dim3((unsigned)F.G), dim3(kSmallT), lds, st,
                     F);
  return check_launch("smaq_fused_kernel");
}

template <int RM, int TIN>
static int launch_fused_rm(const FusedArgs& F, int V, hipStream_t st) {
  switch (V) {
    case 1: return launch_fused_v<RM, 1, TIN>(F, st);
    case 2: return launch_fused_v<RM, 2, TIN>(F, st);
    case 3: return launch_fused_v<RM, 3, TIN>(F, st);
    case 4: return launch_fused_v<RM, 4, TIN>(F, st);
    case 5: return launch_fused_v<RM, 5, TIN>(F, st);
    case 6: return launch_fused_v<RM, 6, TIN>(F, st);
    case 7: return launch_fused_v<RM, 7, TIN>(F, st);
    default: return launch_fused_v<RM, 8, TIN>(F, st);
  }
}

static void fused_args(const FusedCall& c, FusedArgs& F) {
  const SmqSmaqParams* p = c.p;
  const SmallGeom g = small_geom(c.n);
  char* base = (char*)c.ws;
  memset(&F, 0, sizeof(F));
  F.x = c.x;
  F.y = c.y;
  F.n = c.n;
  F.nv = c.n >> 2;
  F.G = g.G;
  F.key = rng_key(p->seed);
  F.offset = p->offset;
  F.ctr = p->offset_counter;
  F.hdr = (SmqSmaqStats*)base;
  F.gen = (uint32_t*)(base + SmaqWsLayout::kFusedGen);
  F.left = (unsigned long long*)(base + SmaqWsLayout::kFusedLeft);
  F.sub = (unsigned long long*)(base + SmaqWsLayout::kFusedSub);
  F.gran = (unsigned long long*)(base + SmaqWsLayout::kFusedGran);
  F.out_slots = (unsigned long long*)(base + SmaqWsLayout::kSlots);
  F.thr = p->main_std_dev_threshold;
  F.r_main = p->range_main;
  F.r_out = p->range_outlier;
  F.clamp_lo = p->clamp_lo;
  F.clamp_hi = p->clamp_hi;
  F.range_coef = c.range_coef;
  F.inv_r_main = c.inv_r_main;
  F.inv_r_out = c.inv_r_out;
  F.all_pos = p->all_positive;
  F.count = p->count_outliers;
  F.range = p->use_range_std_dev;
  F.test_late = c.test_late;
  static const int poll_sleep = [] {  // measurement knob SMQ_FUSED_SLEEP (0, 1, 2, 4, 8, 16)
    const char* e = knob_env("SMQ_FUSED_SLEEP");
    return e ? atoi(e) : 2;
  }();
  F.poll_sleep = poll_sleep;
  F.trace = nullptr;
  F.zero = c.zero;
  F.zero_n = c.zero_n;
#if SMQ_FUSED_TRACE
  if (c.ws_bytes >= SmaqWsLayout::kTotal + 16 * 8 * (size_t)kSmallMaxG)
    F.trace = (uint64_t*)(base + SmaqWsLayout::kTotal);
#endif
  F.rec = c.rec;
  F.bm = p->num_bits_main;
  F.bo = p->num_bits_outlier;
  if (c.rec) F.count = 1;  // (the record's slots are zero: no fill)
  // the counts as granules in replica 1's spare words (behind its 4-word partials: the range form's
  // 6-word partials use them, so it keeps the record's atomics)
  F.rec_gran = (c.rec && !F.range) ? F.gran + SmaqWsLayout::kFusedRecGran : nullptr;
}

int launch_fused(const FusedCall& c, hipStream_t st) {
  const SmqSmaqParams* p = c.p;
  const SmallGeom g = small_geom(c.n);
  FusedArgs F;
  fused_args(c, F);
  if (!c.rec && p->count_outliers) fill_async(F.out_slots, 0ull, SMQ_WS_OUTLIER_SLOTS, st);
  const bool sr = p->stochastic_rounding != 0;
  if (c.dtype == SMQ_DTYPE_F32)
    return sr ? launch_fused_rm<kRoundHash, kF32>(F, g.V, st)
              : launch_fused_rm<kRoundTrunc, kF32>(F, g.V, st);
  if (c.dtype == SMQ_DTYPE_F16)
    return sr ? launch_fused_rm<kRoundHash, kF16>(F, g.V, st)
              : launch_fused_rm<kRoundTrunc, kF16>(F, g.V, st);
  return sr ? launch_fused_rm<kRoundHash, kBF16>(F, g.V, st)
            : launch_fused_rm<kRoundTrunc, kBF16>(F, g.V, st);
}

// ---- PACK (smq_smaq_roundtrip_compress) ---------------------------------------------------------
template <int RM, int V, int WM, int WO>
static int launch_fused_pack_v(FusedArgs& F, hipStream_t st) {
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&smaq_fused_kernel<RM, V, kF32, true, WM, WO>),
      hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLds);
  if (attr != hipSuccess) {
    set_error("smaq_fused_kernel (PACK): hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed: %s",
              hipGetErrorString(attr));
    return SMQ_ERR_LAUNCH;
  }
  const int wm = F.bm - 1, we = F.bo > F.bm ? F.bo - F.bm : 0;
  const int need = 4 * (int)(F.pk.lds_off + pk_lds_words(wm, we, V));
  const int lds = need > fused_lds_bytes(V) ? need : fused_lds_bytes(V);
  hipLaunchKernelGGL((smaq_fused_kernel<RM, V, kF32, true, WM, WO>), dim3((unsigned)F.G),
                     dim3(kSmallT), lds, st, F);
  return check_launch("smaq_fused_kernel (PACK)");
}

template <int RM, int WM, int WO>
static int launch_fused_pack_rm(FusedArgs& F, int V, hipStream_t st) {
  switch (V) {
    case 1: return launch_fused_pack_v<RM, 1, WM, WO>(F, st);
    case 2: return launch_fused_pack_v<RM, 2, WM, WO>(F, st);
    case 3: return launch_fused_pack_v<RM, 3, WM, WO>(F, st);
    default: return launch_fused_pack_v<RM, 4, WM, WO>(F, st);
  }
}

int launch_fused_pack(const FusedCall& c, const FusedPackCall& k, hipStream_t st) {
  const SmqSmaqParams* p = c.p;
  // fp32 x (16-B aligned: fused_eligible), whole float4 groups, full statistics without the
  // range form (its granules would overlap the aggregates'), T_m > 0, no BN term, V <= 4
  if (c.dtype != SMQ_DTYPE_F32 || (c.n & 3) || p->use_range_std_dev || p->bn_gamma ||
      !(p->main_std_dev_threshold > 0.0f) || c.rec)
    return kFusedPackDeclined;
  const SmallGeom g = small_geom(c.n);
  const int wm = p->num_bits_main - 1, wo = p->num_bits_outlier - 1;
  const int we = wo > wm ? wo - wm : 0;
  if (g.V > 4 || wm < 1 || wm > kMaxWidth || wo < 2 || wo > kMaxWidth) return kFusedPackDeclined;
  const uint32_t lds_off = (uint32_t)fused_draw_groups(g.V) * kSmallT * 4u;  // after the draws
  if (4ull * (lds_off + pk_lds_words(wm, we, g.V)) > (unsigned long long)kFusedLds)
    return kFusedPackDeclined;
  FusedArgs F;
  fused_args(c, F);
  F.pk.hdr = k.hdr;
  F.pk.dir = k.dir;
  F.pk.fixed = k.fixed;
  F.pk.var = k.var;
  F.pk.cap_words = k.cap_words;
  F.pk.n_blocks = k.n_blocks;
  F.pk.flags = k.flags;
  F.pk.notify = k.notify;
  F.pk.look = F.gran + SmaqWsLayout::kFusedPackLook;
  F.pk.lds_off = lds_off;
  if (p->count_outliers) fill_async(F.out_slots, 0ull, SMQ_WS_OUTLIER_SLOTS, st);
  const bool sr = p->stochastic_rounding != 0;
  if (wm == 5 && wo == 7)  // the 6/8-bit default
    return sr ? launch_fused_pack_rm<kRoundHash, 5, 7>(F, g.V, st)
              : launch_fused_pack_rm<kRoundTrunc, 5, 7>(F, g.V, st);
  return sr ? launch_fused_pack_rm<kRoundHash, 0, 0>(F, g.V, st)
            : launch_fused_pack_rm<kRoundTrunc, 0, 0>(F, g.V, st);
}

}  // namespace smq
