// Common device helpers for the DMA-YOLO gfx950 kernels.
//
// Storage convention (see DESIGN.md "Data layout"): every activation is NHWC with a
// per-pixel stride `ps` (elements between consecutive pixels), so a channel slice of a
// concat buffer is addressed by (base + c0, ps = Ctot).  Storage type T is float (parity
// mode) or bf16 (throughput mode); all arithmetic and reductions are fp32 (f64 for BN
// finalisation).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

// The C ABI declarations: every DMY_API definition below must match its declaration here, so a signature that
// drifts from include/dmayolo.h (and from the ctypes table checked against it, tests/test_abi.py) fails to compile.
#include "../../include/dmayolo.h"

typedef __hip_bfloat16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define DEV __device__ __forceinline__

template <typename T> struct Traits;
template <> struct Traits<float> {
  static constexpr int VW = 4;  // elements per 16-byte vector
};
template <> struct Traits<bf16> {
  static constexpr int VW = 8;
};

DEV float to_f(float x) { return x; }
DEV float to_f(bf16 x) { return __bfloat162float(x); }
template <typename T> DEV T from_f(float x);
template <> DEV float from_f<float>(float x) { return x; }
template <> DEV bf16 from_f<bf16>(float x) { return __float2bfloat16(x); }

// 16-byte vector <-> VW floats
template <typename T> DEV void unpack(const uint4& v, float* f) {
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int i = 0; i < Traits<T>::VW; ++i) f[i] = to_f(e[i]);
}
template <typename T> DEV uint4 pack(const float* f) {
  uint4 v;
  T* e = reinterpret_cast<T*>(&v);
#pragma unroll
  for (int i = 0; i < Traits<T>::VW; ++i) e[i] = from_f<T>(f[i]);
  return v;
}

// fast transcendental helpers: v_exp_f32 (via __expf) and v_rcp_f32 (1 ulp); the elementwise BN /
// activation kernels are VALU-bound with the accurate expf + IEEE division
DEV float rcp_(float x) { return __builtin_amdgcn_rcpf(x); }
DEV float sigmoidf_(float x) { return rcp_(1.0f + __expf(-x)); }

// N consecutive fp32 per-channel parameters (N % 4 == 0): 16-B loads when p is 16-B aligned, else scalar.  A
// streaming kernel loads its lane's channel parameters once; as 2 x N scalar loads they were the bulk of a short
// wave's VMEM stream (batch-1 LayerNorm: 19.4 -> 5.8 us with the 16-B form)
template <int N> DEV void ldf(const float* p, float* o) {
  if ((((uintptr_t)p) & 15) == 0) {
#pragma unroll
    for (int j = 0; j < N; j += 4) {
      const float4 a = *reinterpret_cast<const float4*>(p + j);
      o[j] = a.x; o[j + 1] = a.y; o[j + 2] = a.z; o[j + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = p[j];
  }
}

// Activation codes shared with the host (dmayolo/_lib.py ACT_*).
enum Act : int { ACT_NONE = 0, ACT_SILU = 1, ACT_HARDSWISH = 2, ACT_SIGMOID = 3, ACT_GELU = 4, ACT_RELU = 5 };

DEV float act_fwd(int act, float u) {
  switch (act) {
    case ACT_SILU: return u * sigmoidf_(u);
    case ACT_HARDSWISH: return u * fminf(fmaxf(u + 3.0f, 0.0f), 6.0f) / 6.0f;
    case ACT_SIGMOID: return sigmoidf_(u);
    case ACT_GELU: return 0.5f * u * (1.0f + erff(u * 0.70710678118654752f));
    case ACT_RELU: return fmaxf(u, 0.0f);
    default: return u;
  }
}
// act_fwd over N values with the activation switch hoisted out of the element loop: the per-element switch keeps every
// element's exp / rcp chain behind uniform branches, one dependent chain at a time, and measured 2.5-5x the conv time of
// the batch-1 eval epilogues; the expressions are act_fwd's, so the results are bit-identical
template <int N> DEV void act_fwd_n(int act, float* u) {
  switch (act) {
    case ACT_SILU:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = u[e] * sigmoidf_(u[e]);
      break;
    case ACT_RELU:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = fmaxf(u[e], 0.0f);
      break;
    case ACT_NONE: break;
    default:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = act_fwd(act, u[e]);
  }
}
// d act / d u at pre-activation u
DEV float act_grad(int act, float u) {
  switch (act) {
    case ACT_SILU: {
      const float s = sigmoidf_(u);
      return s * (1.0f + u * (1.0f - s));
    }
    case ACT_HARDSWISH:  // torch hardswish_backward: u<-3 -> 0, u<=3 -> u/3+0.5, else 1
      return u < -3.0f ? 0.0f : (u <= 3.0f ? u / 3.0f + 0.5f : 1.0f);
    case ACT_SIGMOID: {
      const float s = sigmoidf_(u);
      return s * (1.0f - s);
    }
    case ACT_RELU: return u > 0.0f ? 1.0f : 0.0f;  // torch threshold_backward (result > 0)
    case ACT_GELU: {
      const float kA = 0.70710678118654752f, kB = 0.3989422804014327f;  // 1/sqrt2, 1/sqrt(2pi)
      return 0.5f * (1.0f + erff(u * kA)) + u * kB * expf(-0.5f * u * u);
    }
    default: return 1.0f;
  }
}
// act_grad over N values in place (u -> d act / d u), the switch hoisted out of the element loop as in act_fwd_n
template <int N> DEV void act_grad_n(int act, float* u) {
  switch (act) {
    case ACT_SILU:
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float s = sigmoidf_(u[e]);
        u[e] = s * (1.0f + u[e] * (1.0f - s));
      }
      break;
    case ACT_RELU:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = u[e] > 0.0f ? 1.0f : 0.0f;
      break;
    case ACT_NONE:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = 1.0f;
      break;
    default:
#pragma unroll
      for (int e = 0; e < N; ++e) u[e] = act_grad(act, u[e]);
  }
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

DEV unsigned pack4_e4m3(float a, float b, float c, float d) {  // OCP e4m3fn, round to nearest even, saturated
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}
DEV float nanmax(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }

#define HIP_LAUNCH_CHECK() return (int)hipGetLastError()

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
static inline int grid_cap(long blocks, int cap = 4096) { return (int)(blocks < cap ? (blocks < 1 ? 1 : blocks) : cap); }

#define DMY_API extern "C" __attribute__((visibility("default")))
