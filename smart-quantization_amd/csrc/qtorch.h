// qtorch.h — qtorch 0.2.0 float_quantize bit helpers, host and device (float_quant.hip's kernels,
// cpu_codecs.hip's CPU path). qtorch is an un-vendored dependency of the reference
// (poetry.lock:773-781): quant_function.float_quantize -> float_kernel_stochastic /
// float_kernel_nearest + bit_helper round_bitwise_* / clip_exponent, restated here from its
// published algorithm (integer arithmetic on the fp32 bit pattern).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace smq {

// ---- qtorch bit helpers (restated) --------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
__host__ __device__ __forceinline__ float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

__host__ __device__ __forceinline__ uint32_t round_bitwise(uint32_t target, uint32_t rand_bits,
                                                           int man_bits, bool stochastic) {
  const uint32_t mask = (1u << (23 - man_bits)) - 1u;
  const uint32_t add = stochastic ? (rand_bits & mask) : (1u << (23 - man_bits - 1));
  return (target + add) & ~mask;
}

__host__ __device__ __forceinline__ uint32_t clip_exponent(int exp_bits, int man_bits,
                                                           uint32_t old_num, uint32_t q) {
  const int qexp = (int)((q << 1) >> 24);
  const int min_store = -((1 << (exp_bits - 1)) - 2) - 1 + 127;
  const int max_store = ((1 << (exp_bits - 1)) - 1) + 127;
  if (qexp > max_store) {
    const uint32_t max_man = ((0xffffffffu << 9) >> 9) >> (23 - man_bits) << (23 - man_bits);
    const uint32_t max_num = ((uint32_t)max_store << 23) | max_man;
    q = (old_num & 0x80000000u) | max_num;
  } else if (qexp < min_store) {
    const uint32_t min_num = (uint32_t)min_store << 23;
    const uint32_t middle = (uint32_t)(min_store - 1) << 23;
    const uint32_t uq = q & 0x7fffffffu;
    q = uq > middle ? ((old_num & 0x80000000u) | min_num) : 0u;
  }
  return q;
}

// qtorch float_kernel_{stochastic,nearest} for one element.
__host__ __device__ __forceinline__ float qtorch_quant(float a, uint32_t rand_bits, int exp_bits,
                                                      int man_bits, bool stochastic) {
  uint32_t target = f2u(a);
  const int target_exp = (int)((target << 1) >> 24) - 127;
  const int min_exp = -((1 << (exp_bits - 1)) - 2);
  if (target_exp < min_exp) {  // subnormal in the target format
    const uint32_t shift_bits = ((uint32_t)(127 + min_exp) << 23) | (target & 0x80000000u);
    const float shift = u2f(shift_bits);
    const float val = a + shift;
    const uint32_t qb = round_bitwise(f2u(val), rand_bits, man_bits, stochastic);
    return u2f(qb) - shift;
  }
  uint32_t qb = round_bitwise(target, rand_bits, man_bits, stochastic);
  qb = clip_exponent(exp_bits, man_bits, target, qb);
  return u2f(qb);
}

}  // namespace smq
