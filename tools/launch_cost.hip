// Host cost of one smq_smaq_roundtrip call (the library's enqueue: argument checks, parameter
// block, hipLaunchKernel) against a bare hipLaunchKernel of an empty kernel with the same
// argument size, both back to back on one stream without synchronisation (the device keeps up:
// 64K-element calls). Microseconds of host time per call.
//
// hipcc --offload-arch=gfx950 -O2 -I include tools/launch_cost.hip -L smart-quantization_amd/lib
//   -lsmq -Wl,-rpath,$PWD/smart-quantization_amd/lib -o tools/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "smq.h"

template <int B>
struct Args {
  char b[B];
};
template <int B>
__global__ void empty_kernel(Args<B>) {}

static double us_per(int reps, auto&& fn) {
  for (int i = 0; i < 200; ++i) fn();
  hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) fn();
  const auto t1 = std::chrono::steady_clock::now();
  hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  const int64_t n = 1 << 16;
  float *x, *y;
  void* ws;
  const size_t wsb = smq_smaq_workspace_bytes(n);
  hipMalloc(&x, 4 * n);
  hipMalloc(&y, 4 * n);
  hipMalloc(&ws, wsb);
  hipMemset(ws, 0, wsb);
  std::vector<float> h(n);
  for (int64_t i = 0; i < n; ++i) h[i] = (float)((i * 7919) % 1000) / 500.0f - 1.0f;
  hipMemcpy(x, h.data(), 4 * n, hipMemcpyHostToDevice);
  hipStream_t st;
  hipStreamCreate(&st);
  SmqSmaqParams p;
  smq_smaq_params_init(&p);
  p.seed = 1;
  const int reps = 20000;
  Args<256> big{};
  Args<16> a16{};
  Args<64> a64{};
  Args<1024> a1k{};
  const double t_empty = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<256>, dim3(16), dim3(1024), 0, st, big); });
  const double t_empty_small = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<256>, dim3(1), dim3(64), 0, st, big); });
  const double t16 = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<16>, dim3(16), dim3(256), 0, st, a16); });
  const double t64 = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<64>, dim3(16), dim3(256), 0, st, a64); });
  const double t1k = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<1024>, dim3(16), dim3(256), 0, st, a1k); });
  hipStream_t st2;
  hipStreamCreateWithFlags(&st2, hipStreamNonBlocking);
  const double t16nb = us_per(reps, [&] { hipLaunchKernelGGL(empty_kernel<16>, dim3(16), dim3(256), 0, st2, a16); });
  uint64_t off = 0;
  const double t_smaq = us_per(reps, [&] {
    p.offset = off;
    off += n;
    smq_smaq_roundtrip(x, SMQ_DTYPE_F32, y, n, &p, nullptr, ws, wsb, st);
  });
  const double t_err = us_per(reps, [&] { (void)hipGetLastError(); });
  // the same 256-B-argument launch through hipModuleLaunchKernel with the function handle looked up
  // once (hipLaunchKernel resolves the host stub on every call)
  hipFunction_t fn;
  (void)hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&empty_kernel<256>));
  size_t asz = sizeof(big);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &big, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz,
                 HIP_LAUNCH_PARAM_END};
  const double t_mod = us_per(reps, [&] {
    (void)hipModuleLaunchKernel(fn, 16, 1, 1, 1024, 1, 1, 0, st, nullptr, cfg);
  });
  void* kargs[] = {&big};
  const double t_lk = us_per(reps, [&] {
    (void)hipLaunchKernel(reinterpret_cast<const void*>(&empty_kernel<256>), dim3(16), dim3(1024),
                          kargs, 0, st);
  });
  std::printf("{\"module_launch_us\": %.3f, \"hipLaunchKernel_us\": %.3f}\n", t_mod, t_lk);
  std::printf("{\"empty_launch_us\": %.3f, \"empty_launch_1wg_us\": %.3f, \"smq_smaq_roundtrip_us\": %.3f, "
              "\"hipGetLastError_us\": %.3f, \"args16_us\": %.3f, \"args64_us\": %.3f, "
              "\"args1024_us\": %.3f, \"args16_nonblocking_us\": %.3f}\n", t_empty, t_empty_small,
              t_smaq, t_err, t16, t64, t1k, t16nb);
  return 0;
}
