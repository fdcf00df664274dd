// membench.hip — measured HBM roofline on the box: streaming read-only and copy kernels over a
// 1 GiB fp32 buffer, in the access shapes the SmaQ kernels use (dwordx4 per lane, grid-stride or
// contiguous per-block chunks, default or nontemporal hints), timed with hipEvents.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride read, U loads in flight per thread
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_gs(const f32x4* __restrict__ x, long n4, float* out) {
  long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; i < n4; i += stride) acc += ld<NT>(x + i);
  float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[0] = s;  // keep live
}

// per-block contiguous chunk read
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_chunk(const f32x4* __restrict__ x, long n4, float* out) {
  long per = (n4 + gridDim.x - 1) / gridDim.x;
  long beg = (long)blockIdx.x * per, end = beg + per < n4 ? beg + per : n4;
  f32x4 acc = {0, 0, 0, 0};
  long i = beg + threadIdx.x;
  for (; i + (U - 1) * 256 < end; i += U * 256) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(x + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; i < end; i += 256) acc += ld<NT>(x + i);
  float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[0] = s;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_gs(const f32x4* __restrict__ x, f32x4* __restrict__ y,
                                               long n4) {
  long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(y + i + u * stride, v[u] * 1.0001f);
  }
  for (; i < n4; i += stride) st<NTS>(y + i, ld<NTL>(x + i) * 1.0001f);
}

// flat tiles: block b owns float4 [b*256*V, (b+1)*256*V); V coalesced sweeps of 4 KiB
template <int V, bool NTS>
__global__ __launch_bounds__(256) void copy_tile(const f32x4* __restrict__ x, f32x4* __restrict__ y,
                                                 long n4) {
  long base = (long)blockIdx.x * 256 * V + threadIdx.x;
  f32x4 v[V];
#pragma unroll
  for (int u = 0; u < V; ++u) {
    long i = base + u * 256;
    if (i < n4) v[u] = x[i];
  }
#pragma unroll
  for (int u = 0; u < V; ++u) {
    long i = base + u * 256;
    if (i < n4) st<NTS>(y + i, v[u] * 1.0001f);
  }
}
template <int V>
__global__ __launch_bounds__(256) void read_tile(const f32x4* __restrict__ x, long n4, float* out) {
  long base = (long)blockIdx.x * 256 * V + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < V; ++u) {
    long i = base + u * 256;
    if (i < n4) acc += x[i];
  }
  float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[0] = s;
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int r = 0; r < reps + 3; ++r) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (r >= 3) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : (1L << 28);
  long n4 = n / 4;
  f32x4 *x, *y;
  float* out;
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMalloc(&y, n * 4));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(x, 0, n * 4));
  CHECK(hipMemset(y, 0, n * 4));
  const double bytes = n * 4.0;
  printf("{\"n\": %ld, \"results\": [\n", n);
  bool first = true;
  auto rep = [&](const char* kind, const char* name, int grid, float ms, double b) {
    printf("%s{\"kind\": \"%s\", \"variant\": \"%s\", \"grid\": %d, \"ms\": %.5f, \"GBps\": %.1f}",
           first ? "" : ",\n", kind, name, grid, ms, b / ms / 1e6);
    first = false;
  };
  int grids[] = {1024, 2048, 4096, 8192, 16384};
#define RD(K, U, NT, NAME)                                                              \
  for (int g : grids) {                                                                  \
    float ms = time_ms([&] { hipLaunchKernelGGL((K<U, NT>), dim3(g), dim3(256), 0, 0, x, n4, out); }, 20); \
    rep("read", NAME, g, ms, bytes);                                                     \
  }
  RD(read_gs, 1, false, "gs_u1")
  RD(read_gs, 4, false, "gs_u4")
  RD(read_gs, 8, false, "gs_u8")
  RD(read_gs, 4, true, "gs_u4_nt")
  RD(read_chunk, 4, false, "chunk_u4")
  RD(read_chunk, 8, false, "chunk_u8")
#define CP(U, NTL, NTS, NAME)                                                           \
  for (int g : grids) {                                                                  \
    float ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<U, NTL, NTS>), dim3(g), dim3(256), 0, 0, x, y, n4); }, 20); \
    rep("copy", NAME, g, ms, 2 * bytes);                                                 \
  }
  CP(1, false, false, "u1")
  CP(4, false, false, "u4")
  CP(4, false, true, "u4_ntstore")
  CP(4, true, true, "u4_nt_both")
  CP(2, false, true, "u2_ntstore")
  // one float4 per thread, no grid-stride
  {
    int g = (int)std::min<long>(n4 / 256, 2147483647L);
    float ms = time_ms([&] { hipLaunchKernelGGL((copy_gs<1, false, false>), dim3(g), dim3(256), 0, 0, x, y, n4); }, 20);
    rep("copy", "flat_one_per_thread", g, ms, 2 * bytes);
    ms = time_ms([&] { hipLaunchKernelGGL((read_gs<1, false>), dim3(g), dim3(256), 0, 0, x, n4, out); }, 20);
    rep("read", "flat_one_per_thread", g, ms, bytes);
  }
#define TILE(V)                                                                            \
  {                                                                                        \
    int g = (int)((n4 + 256L * V - 1) / (256L * V));                                       \
    float ms = time_ms([&] { hipLaunchKernelGGL((copy_tile<V, false>), dim3(g), dim3(256), 0, 0, x, y, n4); }, 20); \
    rep("copy", "tile_v" #V, g, ms, 2 * bytes);                                            \
    ms = time_ms([&] { hipLaunchKernelGGL((copy_tile<V, true>), dim3(g), dim3(256), 0, 0, x, y, n4); }, 20); \
    rep("copy", "tile_v" #V "_ntstore", g, ms, 2 * bytes);                                 \
    ms = time_ms([&] { hipLaunchKernelGGL((read_tile<V>), dim3(g), dim3(256), 0, 0, x, n4, out); }, 20); \
    rep("read", "tile_v" #V, g, ms, bytes);                                                \
  }
  TILE(1) TILE(2) TILE(4) TILE(8) TILE(16)
  printf("\n]}\n");
  return 0;
}
