// Host-side helpers of smaq.hip shared with the packed codec (smaq_pack.hip). Internal.
#pragma once

#include <hip/hip_runtime.h>

#include "smq.h"

namespace smq {

// Full or sampled statistics of x into the workspace header (SmqSmaqStats at offset 0).
// zero / zero_n: words to clear on the way (full statistics only: *zeroed tells whether it did).
int prepare_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                  size_t ws_bytes, hipStream_t st, uint32_t* zero = nullptr, uint32_t zero_n = 0,
                  bool* zeroed = nullptr);
// smq_smaq_roundtrip (y = SmartFP(x)) whose statistics record ends in the workspace header for a
// packer that follows (smq_smaq_roundtrip_compress): the single launch where it applies, else the
// statistics launch without deferral and the apply. zero / zero_n as for prepare_stats.
int roundtrip_for_pack(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                       void* ws, size_t ws_bytes, hipStream_t st, uint32_t* zero, uint32_t zero_n,
                       bool* zeroed);
// smq_smaq_roundtrip_compress's y AND stream from one launch where its shape allows (the single
// launch's PACK variant, smaq_fused.hip): kFusedPackDeclined (smaq_small.h) when it does not —
// nothing enqueued then.
struct FusedPackCall;
int roundtrip_pack_fused(const void* x, int dtype, float* y, int64_t n, const SmqSmaqParams* p,
                         void* ws, size_t ws_bytes, const FusedPackCall& k, hipStream_t st);
// Full statistics of x (the single-tensor statistics launch, finalised by its last workgroup) into
// *out instead of the workspace header (multi-tensor calls: tensors above the small partition).
int stats_into(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
               size_t ws_bytes, hipStream_t st, SmqSmaqStats* out);
// Workspace bytes prepare_stats needs for n elements.
size_t smaq_stats_ws_bytes(int64_t n);
// The multi-workgroup Floyd draw of k > SMQ_MAX_DEVICE_SAMPLES indices (smaq.hip): memsets and the
// candidate / suspect / resolve launches on st; the picks are in A->pick (draw order) after them.
// *grid = the grid the gather of the samples should use (A->parts has room for it).
struct LargeDrawArgs;
int launch_large_draw(int64_t n, int64_t k, const SmqSmaqParams* p, void* ws, size_t ws_bytes,
                      hipStream_t st, LargeDrawArgs* A, int* grid);
size_t large_draw_ws_bytes(int64_t k);
// smq_float_quant of fp64 data (fp64.hip): arguments validated by the caller.
int float_quant_f64(const double* x, void* y, int dtype_out, int64_t n, int exp_bits, int man_bits,
                    int rounding, int check_inf, const uint32_t* rand_bits, uint64_t seed,
                    uint64_t offset, uint64_t* offset_counter, float max_value, hipStream_t st);
// Parameter block + dtype validation (sets the thread's last error).
int smaq_validate(const SmqSmaqParams* p, int dtype);
// The statistics of an fp64 call (full / sampled / injected) into the workspace header
// (SmqSmaqStatsF64 at offset 0; fp64.hip): the unpacked round trip's and the fp64 packer's.
int launch_stats_f64(const double* x, int64_t n, const SmqSmaqParams* p,
                     const SmqSmaqStatsF64* stats_in, void* ws, size_t ws_bytes, hipStream_t st);

}  // namespace smq
