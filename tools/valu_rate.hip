// VALU issue cost per wave instruction on gfx950, measured: a full-occupancy grid runs a loop of
// 8 independent chains of one instruction (inline asm, so the compiler cannot fold or reorder it);
// cycles per wave instruction per SIMD = elapsed clocks * SIMDs / wave instructions issued.
// hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && tools/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP8(INS)                                                                    \
  asm volatile(INS : "+v"(a0) : "v"(s)); asm volatile(INS : "+v"(a1) : "v"(s));     \
  asm volatile(INS : "+v"(a2) : "v"(s)); asm volatile(INS : "+v"(a3) : "v"(s));     \
  asm volatile(INS : "+v"(a4) : "v"(s)); asm volatile(INS : "+v"(a5) : "v"(s));     \
  asm volatile(INS : "+v"(a6) : "v"(s)); asm volatile(INS : "+v"(a7) : "v"(s));

constexpr int kIters = 2048;

#define KERNEL32(NAME, INS)                                                         \
  __global__ __launch_bounds__(256) void NAME(float* out, float seed) {             \
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, s = seed * 0.5f;                  \
    for (int i = 0; i < kIters; ++i) { OP8(INS) }                                   \
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;    \
  }

KERNEL32(k_add_f32, "v_add_f32 %0, %0, %1")
KERNEL32(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
KERNEL32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_xor_b32, "v_xor_b32 %0, %0, %1")
KERNEL32(k_cvt_f16, "v_cvt_f16_f32 %0, %1")
KERNEL32(k_floor_f32, "v_floor_f32 %0, %1")
KERNEL32(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %1")
KERNEL32(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %1")
KERNEL32(k_rndne_f32, "v_rndne_f32 %0, %1")
KERNEL32(k_max_f32, "v_max_f32 %0, %0, %1")
KERNEL32(k_lshl_or, "v_lshl_or_b32 %0, %1, 3, %0")
KERNEL32(k_exp_f32, "v_exp_f32 %0, %1")

// v_cndmask_b32 with a lane mask in an SGPR pair (as the compiler emits it after a v_cmp)
__global__ __launch_bounds__(256) void k_cndmask(float* out, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7, s = seed * 0.5f;
  const unsigned long long m = __ballot(threadIdx.x & 1);
#define CM(A) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(A) : "v"(s), "s"(m));
  for (int i = 0; i < kIters; ++i) { CM(a0) CM(a1) CM(a2) CM(a3) CM(a4) CM(a5) CM(a6) CM(a7) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// v_cmp_lt_f32 into an SGPR pair (VOP3 form)
__global__ __launch_bounds__(256) void k_cmp(float* out, float seed) {
  float a = seed + threadIdx.x, s = seed * 0.5f;
  unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0;
#define CP(M) asm volatile("v_cmp_lt_f32 %0, %1, %2" : "=s"(M) : "v"(a), "v"(s));
  for (int i = 0; i < kIters; ++i) { CP(m0) CP(m1) CP(m2) CP(m3) CP(m0) CP(m1) CP(m2) CP(m3) }
  out[blockIdx.x * 256 + threadIdx.x] = (float)(m0 ^ m1 ^ m2 ^ m3);
}

// 64-bit register operands
#define OP8D(INS)                                                                   \
  asm volatile(INS : "+v"(a0) : "v"(s)); asm volatile(INS : "+v"(a1) : "v"(s));     \
  asm volatile(INS : "+v"(a2) : "v"(s)); asm volatile(INS : "+v"(a3) : "v"(s));     \
  asm volatile(INS : "+v"(a4) : "v"(s)); asm volatile(INS : "+v"(a5) : "v"(s));     \
  asm volatile(INS : "+v"(a6) : "v"(s)); asm volatile(INS : "+v"(a7) : "v"(s));
#define KERNEL64(NAME, T, INS)                                                      \
  __global__ __launch_bounds__(256) void NAME(float* out, float seed) {             \
    T a0, a1, a2, a3, a4, a5, a6, a7, s;                                            \
    __builtin_memset(&a0, 0, sizeof(T)); a1 = a2 = a3 = a4 = a5 = a6 = a7 = s = a0; \
    for (int i = 0; i < kIters; ++i) { OP8D(INS) }                                  \
    float r;                                                                        \
    __builtin_memcpy(&r, &a0, 4);                                                   \
    out[blockIdx.x * 256 + threadIdx.x] = r + seed;                                 \
  }
typedef float f2 __attribute__((ext_vector_type(2)));
KERNEL64(k_pk_add_f32, f2, "v_pk_add_f32 %0, %0, %1")
KERNEL64(k_pk_fma_f32, f2, "v_pk_fma_f32 %0, %0, %1, %0")
KERNEL64(k_mul_f64, double, "v_mul_f64 %0, %0, %1")
KERNEL64(k_add_f64, double, "v_add_f64 %0, %0, %1")

__global__ __launch_bounds__(256) void k_cvt_f64(float* out, float seed) {
  float a[8];
  double d[8];
  for (int j = 0; j < 8; ++j) a[j] = seed + j + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[j]) : "v"(a[j]));
  }
  float r = 0;
  for (int j = 0; j < 8; ++j) r += (float)d[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef void (*KFn)(float*, float);
int main() {
  struct { const char* name; KFn fn; } ks[] = {
      {"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32}, {"v_mul_lo_u32", k_mul_lo_u32},
      {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_hi_u32", k_mul_hi_u32}, {"v_xor_b32", k_xor_b32},
      {"v_cvt_f16_f32", k_cvt_f16}, {"v_floor_f32", k_floor_f32}, {"v_cndmask_b32", k_cndmask},
      {"v_cmp_lt_f32", k_cmp}, {"v_cvt_i32_f32", k_cvt_i32_f32}, {"v_cvt_f32_u32", k_cvt_f32_u32},
      {"v_rndne_f32", k_rndne_f32}, {"v_max_f32", k_max_f32}, {"v_lshl_or_b32", k_lshl_or},
      {"v_exp_f32", k_exp_f32},
      {"v_pk_add_f32", k_pk_add_f32}, {"v_pk_fma_f32", k_pk_fma_f32}, {"v_mul_f64", k_mul_f64},
      {"v_add_f64", k_add_f64}, {"v_cvt_f64_f32", k_cvt_f64}};
  int cus = 0, clk_khz = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  float* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs %d, clock attribute %.0f MHz\n", cus, clk_khz / 1e3);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double wave_ins = (double)blocks * 4 * kIters * 8;
    const double per_simd = wave_ins / (cus * 4.0);
    printf("%-16s %.3f ms  %.2f ns per wave-instruction per SIMD  (%.2f cycles at 2.4 GHz)\n",
           k.name, best, best * 1e6 / per_simd, best * 1e6 / per_simd * 2.4);
  }
  return 0;
}
