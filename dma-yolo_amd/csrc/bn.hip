// BatchNorm2d (train: batch statistics; eval: running statistics) fused with the activation,
// NHWC.  Replaces nn.BatchNorm2d + nn.SiLU / nn.Hardswish of models/common.py:67-73 (Conv),
// :1168-1180 (CoorAttention.bn1+act), :1281-1307 (SCConv k2/k3/k4 BN, no act).
// BN semantics: torch batch_norm with eps/momentum from the module (utils/torch_utils.py:161-170
// sets 1e-3 / 0.03): normalise with the biased batch variance, update running_var with the
// unbiased one.  Batch sums arrive as per-row-block partials (written by the conv epilogue or by
// bn_stats below) and are finalised in f64.
#include "common.h"

namespace {

// -------- per-channel batch statistics from a stored activation (when no fused conv epilogue)
template <typename T>
__global__ void bn_stats_kernel(const T* __restrict__ z, long zps, long M, int C, int rows_per_block,
                                float* __restrict__ psum, float* __restrict__ psq) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  __shared__ float s1[4][64], s2[4][64];
  float a = 0.f, b = 0.f;
  if (c < C) {
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(M, r0 + rows_per_block);
    // independent loads in flight: the sums stay sequential per thread (same order)
#pragma unroll 8
    for (long m = r0 + ty; m < r1; m += 4) {
      float v = to_f(z[m * zps + c]);
      a += v;
      b += v * v;
    }
  }
  s1[ty][threadIdx.x & 63] = a;
  s2[ty][threadIdx.x & 63] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
    const int l = threadIdx.x;
    psum[(long)blockIdx.x * C + c] = s1[0][l] + s1[1][l] + s1[2][l] + s1[3][l];
    psq[(long)blockIdx.x * C + c] = s2[0][l] + s2[1][l] + s2[2][l] + s2[3][l];
  }
}

// -------- finalise: partial rows -> mean, invstd, scale, shift (+ running-stat update)
__global__ void bn_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psq, int P, int C,
                                   double count, const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ rmean, float* __restrict__ rvar, long long* nbt, float momentum,
                                   float eps, int update, float* __restrict__ mean, float* __restrict__ invstd,
                                   float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x;
  __shared__ double sa[256], sb[256];
  double a = 0.0, b = 0.0;
  // independent loads in flight: the sums stay sequential per thread (same order)
#pragma unroll 8
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    a += (double)psum[(long)p * C + c];
    b += (double)psq[(long)p * C + c];
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sa[threadIdx.x] += sa[threadIdx.x + s];
      sb[threadIdx.x] += sb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double mu = sa[0] / count;
    double var = sb[0] / count - mu * mu;
    if (var < 0) var = 0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[c] = (float)mu;
    invstd[c] = is;
    const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
    scale[c] = g * is;
    shift[c] = bb - (float)mu * g * is;
    if (update) {
      const double unb = count > 1 ? var * count / (count - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
      if (c == 0 && nbt) *nbt += 1;
    }
  }
}

// eval mode: scale/shift from running stats
__global__ void bn_eval_coef_kernel(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                    float eps, int C, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = 1.f / sqrtf(rvar[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - rmean[c] * g * is;
}

// Thread mapping shared by the vectorised kernels below: a block of 256 threads covers RB rows x
// CV channel-vectors (CV = C / VW, RB = 256 / CV); each thread keeps ONE channel-vector for the
// whole launch, so its per-channel coefficients live in registers and every access is a 16-B
// vector.  Rows are grid-strided.
struct RowMap {
  int cv, rr, RB, CV;
  DEV RowMap(int C, int VW) {
    CV = C / VW;
    RB = 256 / CV;
    cv = threadIdx.x % CV;
    rr = threadIdx.x / CV;
  }
  DEV bool active() const { return rr < RB; }
};

// -------- y = act(z * scale + shift) (+ res)
// U rows per thread and iteration, all loads issued before the arithmetic: U x 16 B (x2 with a residual) in flight
// per lane, where one row per iteration left the streaming kernels at 4.6-5.4 TB/s
template <typename T, int U = 1>
__global__ void __launch_bounds__(256) bn_act_fwd_vec(const T* __restrict__ z, long zps, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, int act, const T* __restrict__ res,
                                                      long rps, T* __restrict__ y, long yps, long M, int C, int rev) {
  constexpr int VW = Traits<T>::VW;
  RowMap rm(C, VW);
  if (!rm.active()) return;
  const int c0 = rm.cv * VW;
  float sc[VW], sh[VW];
  ldf<VW>(scale + c0, sc);
  ldf<VW>(shift + c0, sh);
  const long S = (long)gridDim.x * rm.RB;
  for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += S * U) {
    uint4 zv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long mu = rev ? M - 1 - (m + u * S) : m + u * S;
      if (m + u * S < M) {
        zv[u] = *reinterpret_cast<const uint4*>(z + mu * zps + c0);
        if (res) rv[u] = *reinterpret_cast<const uint4*>(res + mu * rps + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long mu = rev ? M - 1 - (m + u * S) : m + u * S;
      if (m + u * S >= M) break;
      float f[VW];
      unpack<T>(zv[u], f);
#pragma unroll
      for (int j = 0; j < VW; ++j) f[j] = f[j] * sc[j] + sh[j];
      act_fwd_n<VW>(act, f);
      if (res) {
        float r[VW];
        unpack<T>(rv[u], r);
#pragma unroll
        for (int j = 0; j < VW; ++j) f[j] += r[j];
      }
      *reinterpret_cast<uint4*>(y + mu * yps + c0) = pack<T>(f);
    }
  }
}

// Config 5 (fp8 forward convs) with delayed scaling: the producer of an e4m3 conv's input emits the e4m3 copy itself.
// y = act(z * scale + shift) (+ res) as bn_act_fwd_vec (bf16), plus y8[m][c] = e4m3(y * 448 / amax) dense, where amax
// is the PREVIOUS step's max |y| (the G block maxima `pmax` it left, reduced here by every block; block 0 records it
// in used[0] for the conv's dequantisation), and this step's block maxima go to nmax[blockIdx.x] for the next step.
// Values above the previous amax x headroom saturate at +-448 (delayed scaling); nsat (optional, G floats) receives
// each block's count of saturated elements, so the clipping a growing activation range causes is visible.
// A NaN anywhere makes the next amax NaN.
__global__ void __launch_bounds__(256) bn_act_fwd_f8_kernel(const bf16* __restrict__ z, long zps,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, int act,
                                                            const bf16* __restrict__ res, long rps, bf16* __restrict__ y,
                                                            long yps, long M, int C, unsigned char* __restrict__ y8,
                                                            const float* __restrict__ pmax, int G,
                                                            float* __restrict__ nmax, float* __restrict__ used,
                                                            float headroom, float* __restrict__ nsat) {
  __shared__ float red[4], rsat[4];
  float a = 0.f;
  for (int i = threadIdx.x; i < G; i += 256) a = nanmax(a, pmax[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a = nanmax(a, __shfl_xor(a, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  a = nanmax(nanmax(red[0], red[1]), nanmax(red[2], red[3]));
  __syncthreads();
  a *= headroom;
  if (blockIdx.x == 0 && threadIdx.x == 0) used[0] = a;
  const float inv = a > 0.f ? 448.f / a : 1.f, thr = a > 0.f ? a : 448.f;  // |v| > thr saturates
  RowMap rm(C, 8);
  float mx = 0.f, sat = 0.f;
  if (rm.active()) {
    const int c0 = rm.cv * 8;
    float sc[8], sh[8];
    ldf<8>(scale + c0, sc);
    ldf<8>(shift + c0, sh);
    for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += (long)gridDim.x * rm.RB) {
      float f[8];
      unpack<bf16>(*reinterpret_cast<const uint4*>(z + m * zps + c0), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * sc[j] + sh[j];
      act_fwd_n<8>(act, f);
      if (res) {
        float r[8];
        unpack<bf16>(*reinterpret_cast<const uint4*>(res + m * rps + c0), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += r[j];
      }
      const uint4 v = pack<bf16>(f);
      *reinterpret_cast<uint4*>(y + m * yps + c0) = v;
      unpack<bf16>(v, f);  // quantise the stored (bf16-rounded) value, as a separate pass over y would
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mx = nanmax(mx, fabsf(f[j]));
        sat += fabsf(f[j]) > thr ? 1.f : 0.f;
      }
      uint2 o;
      o.x = pack4_e4m3(f[0] * inv, f[1] * inv, f[2] * inv, f[3] * inv);
      o.y = pack4_e4m3(f[4] * inv, f[5] * inv, f[6] * inv, f[7] * inv);
      *reinterpret_cast<uint2*>(y8 + m * C + c0) = o;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = nanmax(mx, __shfl_xor(mx, o, 64));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sat += __shfl_xor(sat, o, 64);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = mx;
    rsat[threadIdx.x >> 6] = sat;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    nmax[blockIdx.x] = nanmax(nanmax(red[0], red[1]), nanmax(red[2], red[3]));
    if (nsat) nsat[blockIdx.x] = (rsat[0] + rsat[1]) + (rsat[2] + rsat[3]);
  }
}

template <typename T>
__global__ void bn_act_fwd_scalar(const T* __restrict__ z, long zps, const float* __restrict__ scale,
                                  const float* __restrict__ shift, int act, const T* __restrict__ res, long rps,
                                  T* __restrict__ y, long yps, long M, int C) {
  const long total = M * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / C;
    const int c = (int)(i % C);
    float v = act_fwd(act, to_f(z[m * zps + c]) * scale[c] + shift[c]);
    if (res) v += to_f(res[m * rps + c]);
    y[m * yps + c] = from_f<T>(v);
  }
}

// -------- backward reduce: per channel  sum(du), sum(du * xhat), du = dy * act'(u)
// also used (dy = z, act none, scale 1, shift 0, mean 0, invstd 1) as plain column sums
template <typename T, bool STATS, int U = 1>
__global__ void __launch_bounds__(256) bn_bwd_reduce_vec(const T* __restrict__ z, long zps, const T* __restrict__ dy,
                                                         long dps, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, int act, long M, int C,
                                                         float* __restrict__ pdb, float* __restrict__ pdg, int rev) {
  constexpr int VW = Traits<T>::VW;
  __shared__ float red[2][256 * VW];
  RowMap rm(C, VW);
  const int c0 = rm.cv * VW;
  float a[VW], b[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) { a[j] = 0.f; b[j] = 0.f; }
  if (rm.active()) {
    float sc[VW], sh[VW], mu[VW], is[VW];
    if (STATS) {
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        sc[j] = 1.f;
        sh[j] = 0.f;
        mu[j] = 0.f;
        is[j] = 1.f;
      }
    } else {
      ldf<VW>(scale + c0, sc);
      ldf<VW>(shift + c0, sh);
      ldf<VW>(mean + c0, mu);
      ldf<VW>(invstd + c0, is);
    }
    const long S = (long)gridDim.x * rm.RB;
    for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += S * U) {
      uint4 zv[U], gv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long mu = rev ? M - 1 - (m + u * S) : m + u * S;
        if (m + u * S < M) {
          zv[u] = *reinterpret_cast<const uint4*>(z + mu * zps + c0);
          if (!STATS) gv[u] = *reinterpret_cast<const uint4*>(dy + mu * dps + c0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {  // rows summed in the same order as one row per iteration
        if (m + u * S >= M) break;
        float zf[VW], gf[VW];
        unpack<T>(zv[u], zf);
        if (!STATS) unpack<T>(gv[u], gf);
        if (STATS) {  // plain column sums of z and z^2 (batch statistics / bias gradients)
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            a[j] += zf[j];
            b[j] += zf[j] * zf[j];
          }
        } else {
          float ag[VW];
#pragma unroll
          for (int j = 0; j < VW; ++j) ag[j] = zf[j] * sc[j] + sh[j];
          act_grad_n<VW>(act, ag);
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const float du = gf[j] * ag[j];
            a[j] += du;
            b[j] += du * (zf[j] - mu[j]) * is[j];
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    red[0][threadIdx.x * VW + j] = a[j];
    red[1][threadIdx.x * VW + j] = b[j];
  }
  __syncthreads();
  // one thread per channel sums the RB row groups
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int cv = c / VW, j = c % VW;
    float s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < rm.RB; ++r) {
      const int t = r * rm.CV + cv;
      s1 += red[0][t * VW + j];
      s2 += red[1][t * VW + j];
    }
    pdb[(long)blockIdx.x * C + c] = s1;
    pdg[(long)blockIdx.x * C + c] = s2;
  }
}

// dz = ca*du + cb + cc*xhat   (train);  eval: cb = cc = 0, ca = scale
template <typename T, int U = 1>
__global__ void __launch_bounds__(256) bn_bwd_apply_vec(const T* __restrict__ z, long zps, const T* __restrict__ dy,
                                                        long dps, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, int act,
                                                        const float* __restrict__ ca, const float* __restrict__ cb,
                                                        const float* __restrict__ cc, T* __restrict__ dz, long dzps,
                                                        long M, int C, int rev) {
  constexpr int VW = Traits<T>::VW;
  RowMap rm(C, VW);
  if (!rm.active()) return;
  const int c0 = rm.cv * VW;
  float sc[VW], sh[VW], k1[VW], k0[VW], k2[VW], t0[VW], t1[VW];
  ldf<VW>(scale + c0, sc);
  ldf<VW>(shift + c0, sh);
  ldf<VW>(ca + c0, k1);
  ldf<VW>(cc + c0, k2);
  ldf<VW>(invstd + c0, t0);
  ldf<VW>(cb + c0, k0);
  ldf<VW>(mean + c0, t1);
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    // dz = ca*du + cb + cc*(z - mean)*invstd = ca*du + k0 + k2*z
    k2[j] = k2[j] * t0[j];
    k0[j] = k0[j] - k2[j] * t1[j];
  }
  const long S = (long)gridDim.x * rm.RB;
  for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += S * U) {
    uint4 zv[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long mu = rev ? M - 1 - (m + u * S) : m + u * S;
      if (m + u * S < M) {
        zv[u] = *reinterpret_cast<const uint4*>(z + mu * zps + c0);
        gv[u] = *reinterpret_cast<const uint4*>(dy + mu * dps + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long mu = rev ? M - 1 - (m + u * S) : m + u * S;
      if (m + u * S >= M) break;
      float zf[VW], gf[VW], o[VW];
      unpack<T>(zv[u], zf);
      unpack<T>(gv[u], gf);
#pragma unroll
      for (int j = 0; j < VW; ++j) o[j] = zf[j] * sc[j] + sh[j];
      act_grad_n<VW>(act, o);
#pragma unroll
      for (int j = 0; j < VW; ++j) o[j] = k1[j] * (gf[j] * o[j]) + k0[j] + k2[j] * zf[j];
      *reinterpret_cast<uint4*>(dz + mu * dzps + c0) = pack<T>(o);
    }
  }
}

template <typename T>
__global__ void bn_bwd_apply_scalar(const T* __restrict__ z, long zps, const T* __restrict__ dy, long dps,
                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                    const float* __restrict__ mean, const float* __restrict__ invstd, int act,
                                    const float* __restrict__ ca, const float* __restrict__ cb,
                                    const float* __restrict__ cc, T* __restrict__ dz, long dzps, long M, int C) {
  const long total = M * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / C;
    const int c = (int)(i % C);
    const float zv = to_f(z[m * zps + c]);
    const float du = to_f(dy[m * dps + c]) * act_grad(act, zv * scale[c] + shift[c]);
    dz[m * dzps + c] = from_f<T>(ca[c] * du + cb[c] + cc[c] * (zv - mean[c]) * invstd[c]);
  }
}

// -------- backward reduce: per channel  sum(du), sum(du * xhat), du = dy * act'(u)
template <typename T>
__global__ void bn_bwd_reduce_kernel(const T* __restrict__ z, long zps, const T* __restrict__ dy, long dps,
                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                     const float* __restrict__ mean, const float* __restrict__ invstd, int act,
                                     long M, int C, int rows_per_block, float* __restrict__ pdb,
                                     float* __restrict__ pdg) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  __shared__ float s1[4][64], s2[4][64];
  float a = 0.f, b = 0.f;
  if (c < C) {
    const float sc = scale[c], sh = shift[c], mu = mean[c], is = invstd[c];
    const long r0 = (long)blockIdx.x * rows_per_block;
    const long r1 = min(M, r0 + rows_per_block);
    for (long m = r0 + ty; m < r1; m += 4) {
      const float zv = to_f(z[m * zps + c]);
      const float du = to_f(dy[m * dps + c]) * act_grad(act, zv * sc + sh);
      a += du;
      b += du * (zv - mu) * is;
    }
  }
  s1[ty][threadIdx.x & 63] = a;
  s2[ty][threadIdx.x & 63] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
    const int l = threadIdx.x;
    pdb[(long)blockIdx.x * C + c] = s1[0][l] + s1[1][l] + s1[2][l] + s1[3][l];
    pdg[(long)blockIdx.x * C + c] = s2[0][l] + s2[1][l] + s2[2][l] + s2[3][l];
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ pdb, const float* __restrict__ pdg, int P, int C,
                                       double count, const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ ca,
                                       float* __restrict__ cb, float* __restrict__ cc) {
  const int c = blockIdx.x;
  __shared__ double sa[256], sb[256];
  double a = 0.0, b = 0.0;
  // independent loads in flight: the sums stay sequential per thread (same order)
#pragma unroll 8
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    a += (double)pdb[(long)p * C + c];
    b += (double)pdg[(long)p * C + c];
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sa[threadIdx.x] += sa[threadIdx.x + s];
      sb[threadIdx.x] += sb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float db = (float)sa[0], dg = (float)sb[0];
    if (dbeta) dbeta[c] = db;
    if (dgamma) dgamma[c] = dg;
    const float g = gamma ? gamma[c] : 1.f;
    const float k = g * invstd[c];
    ca[c] = k;
    cb[c] = (float)(-(double)k * sa[0] / count);
    cc[c] = (float)(-(double)k * sb[0] / count);
  }
}

// two-stage column sums of [P][C] float partial pairs -> [S][C]
__global__ void colsum2_kernel(const float* __restrict__ a, const float* __restrict__ b, long P, int C, int rows_per,
                               float* __restrict__ oa, float* __restrict__ ob) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  __shared__ double s1[4][64], s2[4][64];
  double x = 0.0, y = 0.0;
  if (c < C) {
    const long r0 = (long)blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
    // independent loads in flight: the sums stay sequential per thread (same order)
#pragma unroll 8
    for (long r = r0 + ty; r < r1; r += 4) {
      x += a[r * C + c];
      y += b[r * C + c];
    }
  }
  s1[ty][threadIdx.x & 63] = x;
  s2[ty][threadIdx.x & 63] = y;
  __syncthreads();
  if (ty == 0 && c < C) {
    const int l = threadIdx.x;
    oa[(long)blockIdx.x * C + c] = (float)(s1[0][l] + s1[1][l] + s1[2][l] + s1[3][l]);
    ob[(long)blockIdx.x * C + c] = (float)(s2[0][l] + s2[1][l] + s2[2][l] + s2[3][l]);
  }
}

inline bool vec_ok(int VW, int C, long s1, long s2, long s3, const void* p1, const void* p2, const void* p3) {
  auto al = [](const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; };
  return C % VW == 0 && s1 % VW == 0 && s2 % VW == 0 && s3 % VW == 0 && al(p1) && al(p2) && al(p3);
}

}  // namespace

// grid of the vectorised streaming passes (blocks of 256 threads, RB rows per block and loop step), capped per kind
// (tools/gpu/bw_micro.py, profiles/r05/bn_grid_ab.log, M x C = 1.18M x 128 and 295k x 512 bf16): the reduce passes
// (bn_stats, bn_bwd_reduce: per-block partial rows) are fastest at 2048 blocks (5.0 -> 5.5 TB/s: fewer partial rows to
// write and sum), the elementwise ones (bn_act_fwd, bn_bwd_apply) at 16384 (apply 4.7 -> 5.2 TB/s, act 5.3 -> 5.5: more
// rows in flight per CU); 4096 for the rest.  Round 6 fixed the caps and removed their switches, with the unroll
// variants (DMY_BN_UNROLL 2 / 4, never faster than 1) and the row-order switch.
inline int vec_grid_cap(long M, int C, int VW, int cap) {
  const int RB = 256 / (C / VW);
  return grid_cap(ceil_div(M, (long)RB * 8), cap);
}
inline int vec_grid(long M, int C, int VW) { return vec_grid_cap(M, C, VW, 4096); }
inline int vec_grid_red(long M, int C, int VW) { return vec_grid_cap(M, C, VW, 2048); }
inline int vec_grid_ew(long M, int C, int VW) { return vec_grid_cap(M, C, VW, 16384); }
// row order of the streaming passes: bn_act_fwd and bn_bwd_apply walk M from the END.  A pass that reads a tensor in
// the reverse of the order its producer (or the previous pass) touched it starts on the lines still resident in the
// 256 MiB Infinity Cache instead of the ones evicted first: conv writes z -> act reads z backwards (tail hot) and writes
// y backwards -> the next conv reads y forwards (head hot); data-grad writes dy -> reduce reads dy, z forwards -> apply
// reads them backwards (tail hot) and writes dz backwards -> the conv's data-grad reads dz forwards (head hot).  Same-box
// A/B on DMA-1536 (profiles/r03/ab_bnorder.log): all forwards 147.0 / 146.9, reduce + act reversed 147.3 / 147.4, act +
// apply reversed (kept) 147.5 / 147.6 img/s (the tensors are 0.15-2.4 GB, so only their Infinity-Cache-sized ends
// benefit)
constexpr int kRevAct = 1, kRevReduce = 0, kRevApply = 1;

DMY_API int dmy_bn_partial_rows(long M) {
  long p = (M + 255) / 256;
  return (int)(p < 1024 ? (p < 1 ? 1 : p) : 1024);
}

DMY_API int dmy_bn_stats(int dtype, const void* z, long zps, long M, int C, float* psum, float* psq, void* stream) {
  const int VW = dtype ? 8 : 4;
  if (vec_ok(VW, C, zps, 0, 0, z, nullptr, nullptr) && C / VW <= 256) {
    const int g = vec_grid_red(M, C, VW);
    hipStream_t st = (hipStream_t)stream;
    if (dtype) bn_bwd_reduce_vec<bf16, true><<<g, 256, 0, st>>>((const bf16*)z, zps, (const bf16*)z, zps, nullptr, nullptr, nullptr, nullptr, 0, M, C, psum, psq, 0);
    else bn_bwd_reduce_vec<float, true><<<g, 256, 0, st>>>((const float*)z, zps, (const float*)z, zps, nullptr, nullptr, nullptr, nullptr, 0, M, C, psum, psq, 0);
    return (int)hipGetLastError();
  }
  const int P = dmy_bn_partial_rows(M);
  const int rpb = (int)((M + P - 1) / P);
  dim3 grid(P, ceil_div(C, 64));
  if (dtype) bn_stats_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>((const bf16*)z, zps, M, C, rpb, psum, psq);
  else bn_stats_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>((const float*)z, zps, M, C, rpb, psum, psq);
  return (int)hipGetLastError();
}

DMY_API int dmy_bn_finalize(const float* psum, const float* psq, int P, int C, double count, const float* gamma,
                            const float* beta, float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                            int update, float* mean, float* invstd, float* scale, float* shift, void* stream) {
  bn_finalize_kernel<<<C, 256, 0, (hipStream_t)stream>>>(psum, psq, P, C, count, gamma, beta, rmean, rvar, nbt,
                                                         momentum, eps, update, mean, invstd, scale, shift);
  return (int)hipGetLastError();
}

DMY_API int dmy_bn_eval_coef(const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                             int C, float* scale, float* shift, void* stream) {
  bn_eval_coef_kernel<<<ceil_div(C, 256), 256, 0, (hipStream_t)stream>>>(gamma, beta, rmean, rvar, eps, C, scale, shift);
  return (int)hipGetLastError();
}


DMY_API int dmy_bn_act_fwd(int dtype, const void* z, long zps, const float* scale, const float* shift, int act,
                           const void* res, long rps, void* y, long yps, long M, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int VW = dtype ? 8 : 4;
  const bool vec = vec_ok(VW, C, zps, yps, res ? rps : 0, z, y, res) && C / VW <= 256;
  if (vec) {
    const int g = vec_grid_ew(M, C, VW);
    if (dtype) bn_act_fwd_vec<bf16><<<g, 256, 0, st>>>((const bf16*)z, zps, scale, shift, act, (const bf16*)res, rps, (bf16*)y, yps, M, C, kRevAct);
    else bn_act_fwd_vec<float><<<g, 256, 0, st>>>((const float*)z, zps, scale, shift, act, (const float*)res, rps, (float*)y, yps, M, C, kRevAct);
  } else {
    const int g = grid_cap(ceil_div(M * C, 256), 8192);
    if (dtype) bn_act_fwd_scalar<bf16><<<g, 256, 0, st>>>((const bf16*)z, zps, scale, shift, act, (const bf16*)res, rps, (bf16*)y, yps, M, C);
    else bn_act_fwd_scalar<float><<<g, 256, 0, st>>>((const float*)z, zps, scale, shift, act, (const float*)res, rps, (float*)y, yps, M, C);
  }
  return (int)hipGetLastError();
}

DMY_API int dmy_bn_act_f8_blocks(void) { return 1024; }

DMY_API int dmy_bn_act_fwd_f8(const void* z, long zps, const float* scale, const float* shift, int act, const void* res,
                              long rps, void* y, long yps, long M, int C, void* y8, const float* pmax, float* nmax,
                              float* used, float headroom, float* nsat, void* stream) {
  if (C % 8 != 0 || C / 8 > 256 || !vec_ok(8, C, zps, yps, res ? rps : 0, z, y, res) || ((uintptr_t)y8 & 7) ||
      !(headroom >= 1.f))
    return (int)hipErrorInvalidValue;
  const int G = dmy_bn_act_f8_blocks();
  bn_act_fwd_f8_kernel<<<G, 256, 0, (hipStream_t)stream>>>((const bf16*)z, zps, scale, shift, act, (const bf16*)res, rps,
                                                          (bf16*)y, yps, M, C, (unsigned char*)y8, pmax, G, nmax, used,
                                                          headroom, nsat);
  return (int)hipGetLastError();
}

// Partial rows written by dmy_bn_bwd_reduce / dmy_bn_stats for these exact arguments.
DMY_API int dmy_bn_reduce_rows(int dtype, const void* z, long zps, const void* dy, long dps, long M, int C) {
  const int VW = dtype ? 8 : 4;
  if (vec_ok(VW, C, zps, dy ? dps : 0, 0, z, dy, nullptr) && C / VW <= 256) return vec_grid_red(M, C, VW);
  return dmy_bn_partial_rows(M);
}

DMY_API int dmy_bn_bwd_reduce(int dtype, const void* z, long zps, const void* dy, long dps, const float* scale,
                              const float* shift, const float* mean, const float* invstd, int act, long M, int C,
                              float* pdb, float* pdg, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int VW = dtype ? 8 : 4;
  if (vec_ok(VW, C, zps, dps, 0, z, dy, nullptr) && C / VW <= 256) {
    const int g = vec_grid_red(M, C, VW);
    if (dtype) bn_bwd_reduce_vec<bf16, false><<<g, 256, 0, st>>>((const bf16*)z, zps, (const bf16*)dy, dps, scale, shift, mean, invstd, act, M, C, pdb, pdg, kRevReduce);
    else bn_bwd_reduce_vec<float, false><<<g, 256, 0, st>>>((const float*)z, zps, (const float*)dy, dps, scale, shift, mean, invstd, act, M, C, pdb, pdg, kRevReduce);
    return (int)hipGetLastError();
  }
  const int P = dmy_bn_partial_rows(M);
  const int rpb = (int)((M + P - 1) / P);
  dim3 grid(P, ceil_div(C, 64));
  if (dtype)
    bn_bwd_reduce_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)z, zps, (const bf16*)dy, dps, scale, shift, mean, invstd, act, M, C, rpb, pdb, pdg);
  else
    bn_bwd_reduce_kernel<float><<<grid, 256, 0, st>>>((const float*)z, zps, (const float*)dy, dps, scale, shift, mean, invstd, act, M, C, rpb, pdb, pdg);
  return (int)hipGetLastError();
}

DMY_API int dmy_colsum2_rows(long P) { return (int)(P < 256 ? P : 256); }

DMY_API int dmy_colsum2(const float* a, const float* b, long P, int C, float* oa, float* ob, void* stream) {
  const int S = dmy_colsum2_rows(P);
  const int rows = (int)((P + S - 1) / S);
  dim3 grid(S, ceil_div(C, 64));
  colsum2_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a, b, P, C, rows, oa, ob);
  return (int)hipGetLastError();
}

DMY_API int dmy_bn_bwd_finalize(const float* pdb, const float* pdg, int P, int C, double count, const float* gamma,
                                const float* invstd, float* dgamma, float* dbeta, float* ca, float* cb, float* cc,
                                void* stream) {
  bn_bwd_finalize_kernel<<<C, 256, 0, (hipStream_t)stream>>>(pdb, pdg, P, C, count, gamma, invstd, dgamma, dbeta, ca,
                                                             cb, cc);
  return (int)hipGetLastError();
}

DMY_API int dmy_bn_bwd_apply(int dtype, const void* z, long zps, const void* dy, long dps, const float* scale,
                             const float* shift, const float* mean, const float* invstd, int act, const float* ca,
                             const float* cb, const float* cc, void* dz, long dzps, long M, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int VW = dtype ? 8 : 4;
  if (vec_ok(VW, C, zps, dps, dzps, z, dy, dz) && C / VW <= 256) {
    const int g = vec_grid_ew(M, C, VW);
    if (dtype) bn_bwd_apply_vec<bf16><<<g, 256, 0, st>>>((const bf16*)z, zps, (const bf16*)dy, dps, scale, shift, mean, invstd, act, ca, cb, cc, (bf16*)dz, dzps, M, C, kRevApply);
    else bn_bwd_apply_vec<float><<<g, 256, 0, st>>>((const float*)z, zps, (const float*)dy, dps, scale, shift, mean, invstd, act, ca, cb, cc, (float*)dz, dzps, M, C, kRevApply);
  } else {
    const int g = grid_cap(ceil_div(M * C, 256), 8192);
    if (dtype) bn_bwd_apply_scalar<bf16><<<g, 256, 0, st>>>((const bf16*)z, zps, (const bf16*)dy, dps, scale, shift, mean, invstd, act, ca, cb, cc, (bf16*)dz, dzps, M, C);
    else bn_bwd_apply_scalar<float><<<g, 256, 0, st>>>((const float*)z, zps, (const float*)dy, dps, scale, shift, mean, invstd, act, ca, cb, cc, (float*)dz, dzps, M, C);
  }
  return (int)hipGetLastError();
}

// out[c] (+)= sum_p part[p][c]   (bias gradients from bn_stats partials)
__global__ void reduce_rows_kernel(const float* __restrict__ part, int P, int C, float* __restrict__ out, int acc) {
  const int c = blockIdx.x;
  __shared__ double s[256];
  double a = 0.0;
  // independent loads in flight: the sums stay sequential per thread (same order)
#pragma unroll 8
  for (int p = threadIdx.x; p < P; p += blockDim.x) a += (double)part[(long)p * C + c];
  s[threadIdx.x] = a;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[c] = (acc ? out[c] : 0.f) + (float)s[0];
}

DMY_API int dmy_reduce_rows(const float* part, int P, int C, float* out, int accumulate, void* stream) {
  reduce_rows_kernel<<<C, 256, 0, (hipStream_t)stream>>>(part, P, C, out, accumulate);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- SCConv gate with k3's BatchNorm folded in
// SCConv (models/common.py:1279-1316): out = k3(x) * sigmoid(x + up(k2(x))), k3 = conv + BN (no activation).  Unfused,
// k3's BN costs a bn_act_fwd pass (read z3, write u3) in the forward and a bn_bwd_reduce pass (read du3, z3) in the
// backward, over the layer's largest tensors (64 channels @768^2 bs32: 2.4 GB each).  Here the gate reads z3 and applies
// k3's BN scale / shift itself (u3 = bf16(z3 * scale + shift): the value bn_act_fwd would have stored), and the gate's
// backward writes du3 AND k3's backward-reduce partials (sum du3, sum du3 * xhat3 over its rows; du3 as stored in
// bf16), one row per block, so k3's ConvBNActFn backward skips bn_bwd_reduce (functional.BnLink).  Thread layout of the
// BN streaming kernels (RowMap: a thread owns one 8-channel vector and walks rows), rows in order: deterministic.
namespace {
// (w, h, image) of NHWC pixel m: 32-bit divisions whenever the pixel count fits (the gate kernels' per-row index math
// was three 64-bit divisions per 8-channel vector)
DEV void pix_hwb(long m, int W, int H, bool small, int& w, int& h, int& b) {
  if (small) {
    const unsigned u = (unsigned)m, q = u / (unsigned)W;
    w = (int)(u - q * (unsigned)W);
    b = (int)(q / (unsigned)H);
    h = (int)(q - (unsigned)b * (unsigned)H);
  } else {
    w = (int)(m % W);
    h = (int)((m / W) % H);
    b = (int)(m / ((long)W * H));
  }
}

DEV int nearest_src_bn(int d, int in, int out) {  // ATen nearest index rule (= eltwise.hip nearest_src)
  if (out == in) return d;
  if (out == 2 * in) return d >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf(__fmul_rn((float)d, scale));
  return s < in - 1 ? s : in - 1;
}

__global__ void __launch_bounds__(256) scgate_bn_fwd_kernel(const bf16* __restrict__ x, long xps,
                                                            const bf16* __restrict__ z, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, const bf16* __restrict__ g,
                                                            bf16* __restrict__ out, int N, int H, int W, int C, int GH,
                                                            int GW) {
  constexpr int VW = 8;
  RowMap rm(C, VW);
  if (!rm.active()) return;
  const int c0 = rm.cv * VW;
  float sc[VW], sh[VW];
  ldf<VW>(scale + c0, sc);
  ldf<VW>(shift + c0, sh);
  const long M = (long)N * H * W, S = (long)gridDim.x * rm.RB;
  const bool small = M < (1L << 31);
  for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += S) {
    int w, h, b;
    pix_hwb(m, W, H, small, w, h, b);
    const long gp = ((long)b * GH + nearest_src_bn(h, GH, H)) * GW + nearest_src_bn(w, GW, W);
    const uint4 xv = *reinterpret_cast<const uint4*>(x + m * xps + c0);
    const uint4 zv = *reinterpret_cast<const uint4*>(z + m * C + c0);
    const uint4 gv = *reinterpret_cast<const uint4*>(g + gp * C + c0);
    float xf[VW], zf[VW], gf[VW], o[VW];
    unpack<bf16>(xv, xf);
    unpack<bf16>(zv, zf);
    unpack<bf16>(gv, gf);
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float u = to_f(from_f<bf16>(zf[j] * sc[j] + sh[j]));  // k3's BN output as bn_act_fwd stores it
      const float sg = sigmoidf_(to_f(from_f<bf16>(xf[j] + gf[j])));
      o[j] = u * to_f(from_f<bf16>(sg));
    }
    *reinterpret_cast<uint4*>(out + m * C + c0) = pack<bf16>(o);
  }
}

__global__ void __launch_bounds__(256) scgate_bn_bwd_kernel(
    const bf16* __restrict__ x, long xps, const bf16* __restrict__ z, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ invstd,
    const bf16* __restrict__ g, const bf16* __restrict__ dout, bf16* __restrict__ du3, bf16* __restrict__ dpre, int N,
    int H, int W, int C, int GH, int GW, float* __restrict__ pdb, float* __restrict__ pdg) {
  constexpr int VW = 8;
  __shared__ float red[2][256 * VW];
  RowMap rm(C, VW);
  const int c0 = rm.cv * VW;
  float a[VW], bsum[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) a[j] = bsum[j] = 0.f;
  if (rm.active()) {
    float sc[VW], sh[VW], mu[VW], is[VW];
    ldf<VW>(scale + c0, sc);
    ldf<VW>(shift + c0, sh);
    ldf<VW>(mean + c0, mu);
    ldf<VW>(invstd + c0, is);
    const long M = (long)N * H * W, S = (long)gridDim.x * rm.RB;
    const bool small = M < (1L << 31);
    for (long m = (long)blockIdx.x * rm.RB + rm.rr; m < M; m += S) {
      int w, h, b;
      pix_hwb(m, W, H, small, w, h, b);
      const long gp = ((long)b * GH + nearest_src_bn(h, GH, H)) * GW + nearest_src_bn(w, GW, W);
      const uint4 xv = *reinterpret_cast<const uint4*>(x + m * xps + c0);
      const uint4 zv = *reinterpret_cast<const uint4*>(z + m * C + c0);
      const uint4 gv = *reinterpret_cast<const uint4*>(g + gp * C + c0);
      const uint4 dv = *reinterpret_cast<const uint4*>(dout + m * C + c0);
      float xf[VW], zf[VW], gf[VW], df[VW], du[VW], dp[VW];
      unpack<bf16>(xv, xf);
      unpack<bf16>(zv, zf);
      unpack<bf16>(gv, gf);
      unpack<bf16>(dv, df);
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const float u = to_f(from_f<bf16>(zf[j] * sc[j] + sh[j]));
        const float sg = sigmoidf_(to_f(from_f<bf16>(xf[j] + gf[j])));
        dp[j] = df[j] * u * sg * (1.f - sg);
        du[j] = df[j] * sg;
      }
      const uint4 duv = pack<bf16>(du);
      *reinterpret_cast<uint4*>(du3 + m * C + c0) = duv;
      *reinterpret_cast<uint4*>(dpre + m * C + c0) = pack<bf16>(dp);
      float dr[VW];
      unpack<bf16>(duv, dr);  // the reduce sees du3 as stored, as bn_bwd_reduce would read it
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        a[j] += dr[j];
        bsum[j] += dr[j] * (zf[j] - mu[j]) * is[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    red[0][threadIdx.x * VW + j] = a[j];
    red[1][threadIdx.x * VW + j] = bsum[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int cv = c / VW, j = c % VW;
    float s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < rm.RB; ++r) {
      const int t = r * rm.CV + cv;
      s1 += red[0][t * VW + j];
      s2 += red[1][t * VW + j];
    }
    pdb[(long)blockIdx.x * C + c] = s1;
    pdg[(long)blockIdx.x * C + c] = s2;
  }
}
}  // namespace

static bool scgate_bn_ok(int C, long xps, const void* x, const void* z, const void* g, const void* o) {
  return C % 8 == 0 && C / 8 <= 256 && xps % 8 == 0 && vec_ok(8, C, xps, 0, 0, x, z, g) && vec_ok(8, C, 0, 0, 0, o, nullptr, nullptr);
}

DMY_API int dmy_scgate_bn_rows(int N, int H, int W, int C) { return vec_grid((long)N * H * W, C, 8); }

DMY_API int dmy_scgate_bn_fwd(const void* x, long xps, const void* z, const float* scale, const float* shift,
                              const void* g, void* out, int N, int H, int W, int C, int GH, int GW, void* stream) {
  if (!scgate_bn_ok(C, xps, x, z, g, out)) return (int)hipErrorInvalidValue;
  const int grid = dmy_scgate_bn_rows(N, H, W, C);
  scgate_bn_fwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16*)x, xps, (const bf16*)z, scale, shift,
                                                              (const bf16*)g, (bf16*)out, N, H, W, C, GH, GW);
  return (int)hipGetLastError();
}

DMY_API int dmy_scgate_bn_bwd(const void* x, long xps, const void* z, const float* scale, const float* shift,
                              const float* mean, const float* invstd, const void* g, const void* dout, void* du3,
                              void* dpre, int N, int H, int W, int C, int GH, int GW, float* pdb, float* pdg,
                              void* stream) {
  if (!scgate_bn_ok(C, xps, x, z, g, du3) || !vec_ok(8, C, 0, 0, 0, dout, dpre, nullptr)) return (int)hipErrorInvalidValue;
  const int grid = dmy_scgate_bn_rows(N, H, W, C);
  scgate_bn_bwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const bf16*)x, xps, (const bf16*)z, scale, shift, mean,
                                                              invstd, (const bf16*)g, (const bf16*)dout, (bf16*)du3,
                                                              (bf16*)dpre, N, H, W, C, GH, GW, pdb, pdg);
  return (int)hipGetLastError();
}
