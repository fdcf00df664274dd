// upcast_bench.hip — the HBM ceiling of the half-input apply's traffic shape: read 2 B/elem (fp16),
// write 4 B/elem (fp32), 256M elements, with trivial compute. Variants:
//   ld8_tvT   one 8-B load (4 halves) per lane and slot, T slots, 16-B `sc0 sc1 nt` stores (the
//             apply's current shape);
//   ld16_str  one 16-B load (8 halves) per lane, two 16-B stores at a 32-B lane stride;
//   ld16_xch  one 16-B load per lane, outputs exchanged with ds_bpermute so both stores are
//             coalesced (lane l stores elements 4l..4l+3 of each 256-element half);
//   wr_only   the stores alone (4 B/elem written, nothing read): the write ceiling.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/upcast_bench tools/upcast_bench.hip
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_nt(float4* p, float a, float b, float c, float d) {
  const f32x4 w = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ float h(uint32_t w, int hi) {
  return __half2float(__builtin_bit_cast(__half, (uint16_t)(hi ? (w >> 16) : (w & 0xffffu))));
}

template <int TV>
__global__ __launch_bounds__(256) void ld8(const uint2* __restrict__ x, float4* __restrict__ y, long nv) {
  const long t0 = (long)blockIdx.x * (256 * TV) + threadIdx.x;
  uint2 v[TV];
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long j = t0 + u * 256;
    if (j < nv) v[u] = x[j];
  }
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long j = t0 + u * 256;
    if (j < nv) st_nt(y + j, h(v[u].x, 0) * 1.5f, h(v[u].x, 1) * 1.5f, h(v[u].y, 0) * 1.5f, h(v[u].y, 1) * 1.5f);
  }
}

// 16-B loads of 8 halves, two stores at a 32-B lane stride
template <int TV>
__global__ __launch_bounds__(256) void ld16_str(const uint4* __restrict__ x, float4* __restrict__ y, long n8) {
  const long t0 = (long)blockIdx.x * (256 * TV) + threadIdx.x;
  uint4 v[TV];
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long j = t0 + u * 256;
    if (j < n8) v[u] = x[j];
  }
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long j = t0 + u * 256;
    if (j >= n8) continue;
    st_nt(y + 2 * j, h(v[u].x, 0), h(v[u].x, 1), h(v[u].y, 0), h(v[u].y, 1));
    st_nt(y + 2 * j + 1, h(v[u].z, 0), h(v[u].z, 1), h(v[u].w, 0), h(v[u].w, 1));
  }
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// 16-B loads of 8 halves; a wave's 512 elements: lane l holds 8l..8l+7. Store 0 writes elements
// 0..255 (lane l: 4l..4l+3, held by lane l/2, half l%2), store 1 elements 256..511 (lane 32 + l/2).
template <int TV>
__global__ __launch_bounds__(256) void ld16_xch(const uint4* __restrict__ x, float4* __restrict__ y, long n8) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long w0 = ((long)blockIdx.x * 4 + wave) * (64 * TV);  // first uint4 of this wave
  uint4 v[TV];
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long j = w0 + u * 64 + lane;
    if (j < n8) v[u] = x[j];
  }
#pragma unroll
  for (int u = 0; u < TV; ++u) {
    const long base = w0 + u * 64;
    if (base >= n8) continue;
    const int s0 = lane >> 1, s1 = 32 + (lane >> 1);
    const bool odd = lane & 1;
    // the dwords a lane stores depend on ITS parity (x,y or z,w of the source): pull all four
    const uint32_t ax = bperm(v[u].x, s0), ay = bperm(v[u].y, s0), az = bperm(v[u].z, s0), aw = bperm(v[u].w, s0);
    const uint32_t bx = bperm(v[u].x, s1), by = bperm(v[u].y, s1), bz = bperm(v[u].z, s1), bw = bperm(v[u].w, s1);
    const uint32_t p0 = odd ? az : ax, p1 = odd ? aw : ay, q0 = odd ? bz : bx, q1 = odd ? bw : by;
    float4* yw = y + base * 2;  // 512 floats = 128 float4 per wave-slot
    st_nt(yw + lane, h(p0, 0), h(p0, 1), h(p1, 0), h(p1, 1));
    st_nt(yw + 64 + lane, h(q0, 0), h(q0, 1), h(q1, 0), h(q1, 1));
  }
}

__global__ __launch_bounds__(256) void wr_only(float4* __restrict__ y, long nv) {
  const long t0 = (long)blockIdx.x * 512 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const long j = t0 + u * 256;
    if (j < nv) st_nt(y + j, 1.f, 2.f, 3.f, (float)j);
  }
}

int main() {
  const long n = 1L << 28;
  void *x, *y;
  CHECK(hipMalloc(&x, n * 2));
  CHECK(hipMalloc(&y, n * 4));
  CHECK(hipMemset(x, 0x3c, n * 2));
  CHECK(hipMemset(y, 0, n * 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch, double bytes) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e9, sum = 0;
    const int R = 20;
    for (int i = 0; i < R; ++i) {
      CHECK(hipEventRecord(a));
      launch();
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("{\"variant\": \"%s\", \"best_ms\": %.4f, \"avg_ms\": %.4f, \"GBps_best\": %.1f}\n", name,
           best, sum / R, bytes / best / 1e6);
  };
  const double up = 6.0 * n;
  run("ld8_tv2", [&] { hipLaunchKernelGGL(ld8<2>, dim3(n / 4 / 512), dim3(256), 0, 0, (const uint2*)x, (float4*)y, n / 4); }, up);
  run("ld8_tv4", [&] { hipLaunchKernelGGL(ld8<4>, dim3(n / 4 / 1024), dim3(256), 0, 0, (const uint2*)x, (float4*)y, n / 4); }, up);
  run("ld16_str_tv1", [&] { hipLaunchKernelGGL(ld16_str<1>, dim3(n / 8 / 256), dim3(256), 0, 0, (const uint4*)x, (float4*)y, n / 8); }, up);
  run("ld16_str_tv2", [&] { hipLaunchKernelGGL(ld16_str<2>, dim3(n / 8 / 512), dim3(256), 0, 0, (const uint4*)x, (float4*)y, n / 8); }, up);
  run("ld16_xch_tv1", [&] { hipLaunchKernelGGL(ld16_xch<1>, dim3(n / 8 / 256), dim3(256), 0, 0, (const uint4*)x, (float4*)y, n / 8); }, up);
  run("ld16_xch_tv2", [&] { hipLaunchKernelGGL(ld16_xch<2>, dim3(n / 8 / 512), dim3(256), 0, 0, (const uint4*)x, (float4*)y, n / 8); }, up);
  run("wr_only", [&] { hipLaunchKernelGGL(wr_only, dim3(n / 4 / 512), dim3(256), 0, 0, (float4*)y, n / 4); }, 4.0 * n);
  CHECK(hipFree(x));
  CHECK(hipFree(y));
  return 0;
}
