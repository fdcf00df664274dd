// statsbench.hip — which streaming shape suits the SmaQ statistics pass (fp64 shifted sums per
// element), and does a reversed apply sweep reuse the MALL after a forward statistics sweep?
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/statsbench tools/statsbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

struct Acc {
  double s1 = 0, s2 = 0;
  __device__ void add(float v, double k) {
    const double d = (double)v - k;
    s1 += d;
    s2 = fma(d, d, s2);
  }
};

__device__ void put(double2* part, Acc a, Acc b, Acc c, Acc d) {
  double s1 = (a.s1 + b.s1) + (c.s1 + d.s1), s2 = (a.s2 + b.s2) + (c.s2 + d.s2);
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + threadIdx.x / 64] = make_double2(s1, s2);
}

// grid-stride, PF = loads in flight per lane (software prefetch distance PF-1)
template <int PF>
__global__ __launch_bounds__(256) void st_gs(const float4* __restrict__ x, long n4, double k,
                                             double2* part) {
  Acc a, b, c, d;
  long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (PF == 1) {
    for (; i < n4; i += stride) {
      float4 v = x[i];
      a.add(v.x, k); b.add(v.y, k); c.add(v.z, k); d.add(v.w, k);
    }
  } else {
    float4 cur = i < n4 ? x[i] : make_float4(0, 0, 0, 0);
    bool have = i < n4;
    while (have) {
      const long nx = i + stride;
      float4 nxt = make_float4(0, 0, 0, 0);
      const bool hn = nx < n4;
      if (hn) nxt = x[nx];
      a.add(cur.x, k); b.add(cur.y, k); c.add(cur.z, k); d.add(cur.w, k);
      cur = nxt;
      have = hn;
      i = nx;
    }
  }
  put(part, a, b, c, d);
}

// flat tiles: V float4 per lane, block-contiguous
template <int V>
__global__ __launch_bounds__(256) void st_tile(const float4* __restrict__ x, long n4, double k,
                                               double2* part) {
  Acc a, b, c, d;
  long base = (long)blockIdx.x * 256 * V + threadIdx.x;
  float4 v[V];
#pragma unroll
  for (int u = 0; u < V; ++u) {
    long i = base + u * 256;
    v[u] = i < n4 ? x[i] : make_float4(0, 0, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < V; ++u) {
    a.add(v[u].x, k); b.add(v[u].y, k); c.add(v[u].z, k); d.add(v[u].w, k);
  }
  put(part, a, b, c, d);
}

// per-block contiguous chunk, one float4 per lane in flight
__global__ __launch_bounds__(256) void st_chunk(const float4* __restrict__ x, long n4, double k,
                                                double2* part) {
  Acc a, b, c, d;
  long per = (n4 + gridDim.x - 1) / gridDim.x;
  long beg = (long)blockIdx.x * per, end = beg + per < n4 ? beg + per : n4;
  for (long i = beg + threadIdx.x; i < end; i += 256) {
    float4 v = x[i];
    a.add(v.x, k); b.add(v.y, k); c.add(v.z, k); d.add(v.w, k);
  }
  put(part, a, b, c, d);
}

// fp32 read-only reference (membench read_gs<1>)
__global__ __launch_bounds__(256) void rd_gs(const float4* __restrict__ x, long n4, double k,
                                             double2* part) {
  float4 acc = make_float4(0, 0, 0, 0);
  long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 v = x[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) part[0] = make_double2(k, 0);
}

// copy tiles forward or reversed (block b handles tile b or grid-1-b)
template <bool REV>
__global__ __launch_bounds__(256) void cp_tile(const float4* __restrict__ x, float4* __restrict__ y,
                                               long n4) {
  long t = REV ? (long)(gridDim.x - 1 - blockIdx.x) : (long)blockIdx.x;
  long base = t * 256 * 4 + threadIdx.x;
  float4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    long i = base + u * 256;
    if (i < n4) v[u] = x[i];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    long i = base + u * 256;
    if (i < n4) {
      float4 w = v[u];
      w.x *= 1.0001f;
      __builtin_nontemporal_store(w.x, &y[i].x);
      __builtin_nontemporal_store(w.y, &y[i].y);
      __builtin_nontemporal_store(w.z, &y[i].z);
      __builtin_nontemporal_store(w.w, &y[i].w);
    }
  }
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
  float4 *x, *y, *z;
  double2* part;
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMalloc(&y, n * 4));
  CHECK(hipMalloc(&z, n * 4));
  CHECK(hipMalloc(&part, sizeof(double2) * 4 * (n4 / 256 + 1)));
  CHECK(hipMemset(x, 0x3c, n * 4));
  CHECK(hipMemset(z, 0x3c, n * 4));
  const double bytes = n * 4.0;
  const double k = 0.5;
  printf("{\"n\": %ld, \"results\": [\n", n);
  bool first = true;
  auto rep = [&](const char* name, int grid, float ms, double b) {
    printf("%s{\"variant\": \"%s\", \"grid\": %d, \"ms\": %.5f, \"GBps\": %.1f}", first ? "" : ",\n",
           name, grid, ms, b / ms / 1e6);
    first = false;
  };
  for (int g : {256, 512, 1024, 2048, 4096}) {
    rep("rd_gs_f32", g, time_ms([&] { hipLaunchKernelGGL(rd_gs, dim3(g), dim3(256), 0, 0, x, n4, k, part); }, 20), bytes);
    rep("st_gs_pf1", g, time_ms([&] { hipLaunchKernelGGL(st_gs<1>, dim3(g), dim3(256), 0, 0, x, n4, k, part); }, 20), bytes);
    rep("st_gs_pf2", g, time_ms([&] { hipLaunchKernelGGL(st_gs<2>, dim3(g), dim3(256), 0, 0, x, n4, k, part); }, 20), bytes);
    rep("st_chunk", g, time_ms([&] { hipLaunchKernelGGL(st_chunk, dim3(g), dim3(256), 0, 0, x, n4, k, part); }, 20), bytes);
  }
#define TILE(V) { int g = (int)((n4 + 256L * V - 1) / (256L * V)); \
    rep("st_tile_v" #V, g, time_ms([&] { hipLaunchKernelGGL(st_tile<V>, dim3(g), dim3(256), 0, 0, x, n4, k, part); }, 20), bytes); }
  TILE(1) TILE(2) TILE(4) TILE(8) TILE(16)
  // MALL reuse: forward read of x, then copy x->y forward or reversed (time the copy only);
  // a read of the unrelated buffer z first gives the cold reference.
  int gc = (int)((n4 + 1023) / 1024);
  for (int rev = 0; rev < 2; ++rev) {
    for (int warm = 0; warm < 2; ++warm) {
      std::vector<float> ts;
      for (int r = 0; r < 23; ++r) {
        hipLaunchKernelGGL(rd_gs, dim3(1024), dim3(256), 0, 0, warm ? x : z, n4, k, part);
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        CHECK(hipEventRecord(a));
        if (rev) hipLaunchKernelGGL(cp_tile<true>, dim3(gc), dim3(256), 0, 0, x, y, n4);
        else hipLaunchKernelGGL(cp_tile<false>, dim3(gc), dim3(256), 0, 0, x, y, n4);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) ts.push_back(ms);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
      }
      std::sort(ts.begin(), ts.end());
      char nm[64];
      snprintf(nm, sizeof nm, "copy_after_%s_read_%s", warm ? "same" : "other", rev ? "rev" : "fwd");
      rep(nm, gc, ts[ts.size() / 2], 2 * bytes);
    }
  }
  printf("\n]}\n");
  return 0;
}
