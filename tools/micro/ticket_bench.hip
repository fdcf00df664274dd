// Microbenchmark: cost of a per-workgroup ticket (one returning atomicAdd on ONE address) at the
// packed codec's grid (65536 workgroups of 256 threads), against the same grid without it and
// with one ticket per group of workgroups. Prints ms per launch (hipEvent, 20 launches).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void no_ticket(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}

__global__ void ticket(unsigned* ctr, unsigned* out) {
  __shared__ unsigned s;
  if (threadIdx.x == 0) s = atomicAdd(ctr, 1u);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// K workgroups share one ticket word among 8 spread counters (XCD-local rows, 256 B apart)
__global__ void ticket_spread(unsigned* ctr, unsigned* out) {
  __shared__ unsigned s;
  if (threadIdx.x == 0) s = atomicAdd(ctr + 64 * (blockIdx.x & 7), 1u);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// with a 16 KiB streaming read per workgroup (the packer's input) to see overlap
__global__ void ticket_load(unsigned* ctr, const float4* x, float* out) {
  __shared__ unsigned s;
  if (threadIdx.x == 0) s = atomicAdd(ctr, 1u);
  __syncthreads();
  const unsigned b = s;
  float acc = 0.f;
  for (int k = 0; k < 4; ++k) {
    const float4 v = x[(size_t)b * 1024 + k * 256 + threadIdx.x];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[b] = acc;
}

__global__ void plain_load(const float4* x, float* out) {
  const unsigned b = blockIdx.x;
  float acc = 0.f;
  for (int k = 0; k < 4; ++k) {
    const float4 v = x[(size_t)b * 1024 + k * 256 + threadIdx.x];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[b] = acc;
}

template <class F>
static float time_it(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  const unsigned G = 65536;
  unsigned *ctr, *out;
  float4* x;
  float* fo;
  hipMalloc(&ctr, 4096);
  hipMalloc(&out, 4 * G);
  hipMalloc(&x, (size_t)G * 16384);
  hipMalloc(&fo, 4 * G);
  hipMemset(ctr, 0, 4096);
  hipMemset(x, 0, (size_t)G * 16384);
  printf("no_ticket      %.4f ms\n", time_it([&] { hipLaunchKernelGGL(no_ticket, dim3(G), dim3(256), 0, 0, out); }));
  printf("ticket         %.4f ms\n", time_it([&] { hipLaunchKernelGGL(ticket, dim3(G), dim3(256), 0, 0, ctr, out); }));
  printf("ticket_spread8 %.4f ms\n", time_it([&] { hipLaunchKernelGGL(ticket_spread, dim3(G), dim3(256), 0, 0, ctr, out); }));
  printf("plain_load     %.4f ms\n", time_it([&] { hipLaunchKernelGGL(plain_load, dim3(G), dim3(256), 0, 0, x, fo); }));
  hipMemset(ctr, 0, 4096);
  printf("ticket_load    %.4f ms\n", time_it([&] { hipMemsetAsync(ctr, 0, 4); hipLaunchKernelGGL(ticket_load, dim3(G), dim3(256), 0, 0, ctr, x, fo); }));
  return 0;
}
