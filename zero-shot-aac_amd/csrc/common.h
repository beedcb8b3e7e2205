// Shared device/host helpers for the zsaac HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <string>
#include "../../include/zsaac.h"

namespace zs {

// ---------------------------------------------------------------- error plumbing
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...);

#define ZS_CHECK_HIP(expr)                                                          \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return ::zs::fail(ZS_ERR_HIP, "%s:%d %s -> %s", __FILE__, __LINE__, #expr,    \
                        hipGetErrorString(_e));                                     \
  } while (0)

#define ZS_REQUIRE(cond, ...)                                                       \
  do {                                                                              \
    if (!(cond)) return ::zs::fail(ZS_ERR_ARG, __VA_ARGS__);                        \
  } while (0)

#define ZS_LAUNCH_CHECK() ZS_CHECK_HIP(hipGetLastError())

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
__host__ __device__ inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------- bf16 helpers
typedef uint16_t bf16_t;  // storage type (raw bits)

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even; NaN kept NaN by the cast path of the compiler (v_cvt_pk_bf16_f32)
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

// two floats -> one dword of two bf16 (low = a), round-to-nearest-even: ONE v_cvt_pk_bf16_f32
// (two f2bf calls and an OR cost three instructions)
typedef __attribute__((ext_vector_type(2))) float cvt_f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 cvt_bf16x2_t;
__device__ __forceinline__ uint32_t pk2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((cvt_f32x2_t){a, b}, cvt_bf16x2_t));
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};
template <typename T> __device__ __forceinline__ float ldf(const T* p) { return Cvt<T>::to_f(*p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v) { *p = Cvt<T>::from_f(v); }
// 4 consecutive values in one store (16 B f32 / 8 B bf16; p aligned to that)
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void st4(bf16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(a, b), pk2bf(c, d));
}

// ---------------------------------------------------------------- wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum through LDS (blockDim multiple of 64, <= 1024)
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// order-preserving float -> uint32 key (larger float -> larger key)
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// activations (reference semantics)
enum Act { ACT_NONE = 0, ACT_GELU_ERF = 1, ACT_GELU_TANH = 2, ACT_RELU = 3, ACT_TANH = 4 };
__device__ __forceinline__ float act_apply(float x, int act) {
  switch (act) {
    case ACT_GELU_ERF: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
    case ACT_GELU_TANH: {
      // HF gelu_new: 0.5*x*(1+tanh(sqrt(2/pi)*(x+0.044715*x^3)))
      const float c = 0.7978845608028654f;
      return 0.5f * x * (1.0f + tanhf(c * (x + 0.044715f * x * x * x)));
    }
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

// GELU (erf form, nn.GELU default) with erf from Abramowitz & Stegun 7.1.26: one v_rcp, one v_exp
// and a degree-5 polynomial, no branches (ocml's erff is a piecewise polynomial whose branches
// diverge across a wave).  |gelu error| <= 2.2e-7 absolute over the whole line (checked against
// scipy in float64), far below bf16 rounding; used only where the result is stored as bf16.
__device__ __forceinline__ float gelu_erf_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float q = t * p * __expf(-z * z);          // = 1 - erf(z)
  return x * (x >= 0.f ? fmaf(-0.5f, q, 1.0f) : 0.5f * q);
}

// bf16-output epilogues: the same activations in cheaper forms whose error (a few f32 ulp) is far
// below bf16 rounding.  gelu_new = x * sigmoid(2u) exactly (0.5 * (1 + tanh u) = sigmoid(2u)),
// one v_exp_f32 + one reciprocal instead of tanhf; the f32 parity path keeps act_apply.
__device__ __forceinline__ float act_apply_fast(float x, int act) {
  if (act == ACT_GELU_TANH) {
    const float u2 = -1.5957691216057308f * (x + 0.044715f * x * x * x);   // -2*sqrt(2/pi)*(...)
    return x * __builtin_amdgcn_rcpf(1.0f + __expf(u2));
  }
  if (act == ACT_GELU_ERF) return gelu_erf_fast(x);
  return act_apply(x, act);
}

}  // namespace zs
