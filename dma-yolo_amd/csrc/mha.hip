// Global multi-head self-attention of the config-5 C3TR block (models/common.py:312-355 ->
// nn.MultiheadAttention, torch/nn/functional.py multi_head_attention_forward), and the
// TransformerLayer dropout (common.py:328, nn.Dropout(0.1)).
//
// Tokens are the pixels of one image in (h, w) row-major order (TransformerBlock flattens
// x.flatten(2) -> [HW, b, c], common.py:353-355), so in our NHWC buffers the token i of image b
// is row b * L + i with stride `ps`; head h owns the channel columns [h d, h d + d).  q, k, v are
// the in-projected tensors (the in_proj / out_proj GEMMs run on the implicit-GEMM kernels).
//
//   O = softmax(scale Q K^T) V, scale = d^-1/2 (the reference scales q before the product);
//   saved for the backward: lse2 = log2-domain row log-sum-exp (max + log2 sum of exp2).
//   Backward (nothing L x L is stored; P is recomputed):
//     Dq = rowsum(dO * O);  dS = P (dP - Dq), dP = dO V^T;
//     dV = P^T dO;  dK = scale dS^T Q;  dQ = scale dS K.
//
// Two implementations:
//   * generic (fp32 math, any head dim <= 128, float or bf16 storage): one thread per query (or
//     key), keys streamed through L1; the parity path for fp32 storage.
//   * MFMA (bf16, head dim 32 / 64 / 128): flash-style, 16x16x32 bf16 MFMAs, K/V (or Q/dO) tiles
//     double-buffered in LDS.  S^T = K Q^T is computed with the K rows of each 16-row tile taken
//     in the order 8 (i >> 2) + 4 t + (i & 3), so a lane ends up holding P for 8 CONSECUTIVE keys of
//     one query: exactly the B fragment of O^T = V^T P^T.  The softmax statistics and the O^T
//     accumulator rows therefore belong to the same lane (query = lane & 15): no shuffles beyond
//     the 4-lane-group row reductions.
#include "common.h"

namespace {

struct MhaGeom {
  int B, L, nh, d;
  long qps, kps, vps, ops;  // token strides of q, k, v and of o / dO (and of dq, dk, dv)
  float scale;              // d^-1/2
};

constexpr float LOG2E = 1.4426950408889634f;

DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---------------------------------------------------------------- generic (fp32 math)
// grid (ceil(L / 64), nh, B), 64 threads; per-thread accumulators in LDS (d <= 128).
template <typename T>
__global__ void __launch_bounds__(64) mha_fwd_generic(const T* __restrict__ q, const T* __restrict__ k,
                                                      const T* __restrict__ v, T* __restrict__ o,
                                                      float* __restrict__ lse2, MhaGeom g) {
  __shared__ float acc[64 * 129];
  __shared__ float qs[64 * 129];
  const int t = threadIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int i = blockIdx.x * 64 + t;
  const bool live = i < g.L;
  const int d = g.d;
  float* a = acc + t * 129;
  float* qq = qs + t * 129;
  const long tb = (long)b * g.L;
  const float c = g.scale * LOG2E;
  for (int e = 0; e < d; ++e) {
    a[e] = 0.f;
    qq[e] = live ? to_f(q[(tb + i) * g.qps + h * d + e]) * c : 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < g.L; ++j) {
    const T* kr = k + (tb + j) * g.kps + h * d;
    float s = 0.f;
    for (int e = 0; e < d; ++e) s += qq[e] * to_f(kr[e]);
    const float mn = fmaxf(m, s);
    const float al = ex2(m - mn), p = ex2(s - mn);
    l = l * al + p;
    m = mn;
    const T* vr = v + (tb + j) * g.vps + h * d;
    for (int e = 0; e < d; ++e) a[e] = a[e] * al + p * to_f(vr[e]);
  }
  if (!live) return;
  const float inv = 1.f / l;
  for (int e = 0; e < d; ++e) o[(tb + i) * g.ops + h * d + e] = from_f<T>(a[e] * inv);
  lse2[((long)b * g.nh + h) * g.L + i] = m + __log2f(l);
}

// Dq[b][h][i] = sum_e dO * O over the head's columns; grid-stride over B * L * nh
template <typename T>
__global__ void mha_rowdot(const T* __restrict__ o, const T* __restrict__ dout, float* __restrict__ Dq, MhaGeom g) {
  const long total = (long)g.B * g.L * g.nh;
  for (long x = blockIdx.x * (long)blockDim.x + threadIdx.x; x < total; x += (long)gridDim.x * blockDim.x) {
    const int h = (int)(x % g.nh);
    const long bi = x / g.nh;  // b * L + i
    const int i = (int)(bi % g.L);
    const int b = (int)(bi / g.L);
    const T* op = o + bi * g.ops + h * g.d;
    const T* dp = dout + bi * g.ops + h * g.d;
    float s = 0.f;
    for (int e = 0; e < g.d; ++e) s += to_f(op[e]) * to_f(dp[e]);
    Dq[((long)b * g.nh + h) * g.L + i] = s;
  }
}

// dQ: one thread per query
template <typename T>
__global__ void __launch_bounds__(64) mha_bwd_dq_generic(const T* __restrict__ q, const T* __restrict__ k,
                                                         const T* __restrict__ v, const T* __restrict__ dout,
                                                         const float* __restrict__ lse2, const float* __restrict__ Dq,
                                                         T* __restrict__ dq, MhaGeom g) {
  __shared__ float qs[64 * 129], ds_[64 * 129], acc[64 * 129];
  const int t = threadIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int i = blockIdx.x * 64 + t;
  if (i >= g.L) return;  // no block-level sync below
  const int d = g.d;
  const long tb = (long)b * g.L;
  const float c = g.scale * LOG2E;
  float* qq = qs + t * 129;
  float* dd = ds_ + t * 129;
  float* a = acc + t * 129;
  for (int e = 0; e < d; ++e) {
    qq[e] = to_f(q[(tb + i) * g.qps + h * d + e]) * c;
    dd[e] = to_f(dout[(tb + i) * g.ops + h * d + e]);
    a[e] = 0.f;
  }
  const long row = ((long)b * g.nh + h) * g.L + i;
  const float L2 = lse2[row], Di = Dq[row];
  for (int j = 0; j < g.L; ++j) {
    const T* kr = k + (tb + j) * g.kps + h * d;
    const T* vr = v + (tb + j) * g.vps + h * d;
    float s = 0.f, dp = 0.f;
    for (int e = 0; e < d; ++e) {
      s += qq[e] * to_f(kr[e]);
      dp += dd[e] * to_f(vr[e]);
    }
    const float ds = ex2(s - L2) * (dp - Di);
    for (int e = 0; e < d; ++e) a[e] += ds * to_f(kr[e]);
  }
  for (int e = 0; e < d; ++e) dq[(tb + i) * g.ops + h * d + e] = from_f<T>(a[e] * g.scale);
}

// dK, dV: one thread per key (32 threads per block: two d x 32 accumulators + k, v rows in LDS)
template <typename T>
__global__ void __launch_bounds__(32) mha_bwd_dkdv_generic(const T* __restrict__ q, const T* __restrict__ k,
                                                           const T* __restrict__ v, const T* __restrict__ dout,
                                                           const float* __restrict__ lse2, const float* __restrict__ Dq,
                                                           T* __restrict__ dk, T* __restrict__ dv, MhaGeom g) {
  __shared__ float ks[32 * 129], vs[32 * 129], ak[32 * 129], av[32 * 129];
  const int t = threadIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int j = blockIdx.x * 32 + t;
  if (j >= g.L) return;
  const int d = g.d;
  const long tb = (long)b * g.L;
  const float c = g.scale * LOG2E;
  float* kk = ks + t * 129;
  float* vv = vs + t * 129;
  float* a1 = ak + t * 129;
  float* a2 = av + t * 129;
  for (int e = 0; e < d; ++e) {
    kk[e] = to_f(k[(tb + j) * g.kps + h * d + e]);
    vv[e] = to_f(v[(tb + j) * g.vps + h * d + e]);
    a1[e] = 0.f;
    a2[e] = 0.f;
  }
  const long rb = ((long)b * g.nh + h) * g.L;
  for (int i = 0; i < g.L; ++i) {
    const T* qr = q + (tb + i) * g.qps + h * d;
    const T* dr = dout + (tb + i) * g.ops + h * d;
    float s = 0.f, dp = 0.f;
    for (int e = 0; e < d; ++e) {
      s += to_f(qr[e]) * kk[e];
      dp += to_f(dr[e]) * vv[e];
    }
    const float p = ex2(s * c - lse2[rb + i]);
    const float ds = p * (dp - Dq[rb + i]);
    for (int e = 0; e < d; ++e) {
      a1[e] += ds * to_f(qr[e]);
      a2[e] += p * to_f(dr[e]);
    }
  }
  for (int e = 0; e < d; ++e) {
    dk[(tb + j) * g.ops + h * d + e] = from_f<T>(a1[e] * g.scale);
    dv[(tb + j) * g.ops + h * d + e] = from_f<T>(a2[e]);
  }
}

// ---------------------------------------------------------------- MFMA (bf16, D in {32, 64, 128})
typedef short s4v __attribute__((ext_vector_type(4)));
DEV f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// lane gets X[r][k0 + 8g .. +8), r = row (caller-chosen), g = lane >> 4
DEV bf16x8 rd_row(const bf16* X, int ld, int r, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(X + r * ld + k0 + 8 * (lane >> 4));
}
// lane gets X[k0 + 8g + e][r0 + (lane&15)], e = 0..7 (transposed read)
DEV bf16x8 rd_col(const bf16* X, int ld, int r0, int k0, int lane) {
  const int g = lane >> 4, il = lane & 15, qq = il >> 2, p = il & 3;
  const bf16* a0 = X + (k0 + 8 * g + qq) * ld + r0 + 4 * p;
  const bf16* a1 = X + (k0 + 8 * g + 4 + qq) * ld + r0 + 4 * p;
  s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a0));
  s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// permuted row of a 16-row tile: lane il of tile tt reads row 8 (il >> 2) + 4 tt + (il & 3)
DEV int prow(int il, int tt) { return 8 * (il >> 2) + 4 * tt + (il & 3); }
DEV short bfbits(float x) {
  bf16 h = __float2bfloat16(x);
  return *reinterpret_cast<short*>(&h);
}
// a global 16-B chunk of a token row (zeros past L)
DEV uint4 ld16(const bf16* base, long ps, int row, int L, int col) {
  if (row >= L) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(base + (long)row * ps + col);
}

// Stage a 64-token x D tile pair (two token matrices, e.g. K and V) through registers into LDS.
template <int D, int NT> struct Stage2 {
  static constexpr int CH = 64 * D / 8 / NT;  // 16-B chunks per thread per matrix
  uint4 ra[CH], rb[CH];
  DEV void load(const bf16* A, long aps, const bf16* Bm, long bps, int t0, int L, int tid) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int x = tid + c * NT, row = x / (D / 8), col = (x % (D / 8)) * 8;
      ra[c] = ld16(A, aps, t0 + row, L, col);
      rb[c] = ld16(Bm, bps, t0 + row, L, col);
    }
  }
  DEV void store(bf16* As, bf16* Bs, int tid) {
    constexpr int LD = D + 8;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int x = tid + c * NT, row = x / (D / 8), col = (x % (D / 8)) * 8;
      *reinterpret_cast<uint4*>(As + row * LD + col) = ra[c];
      *reinterpret_cast<uint4*>(Bs + row * LD + col) = rb[c];
    }
  }
};

// Forward: 4 waves x 32 queries per workgroup, keys in blocks of 64.
template <int D>
__global__ void __launch_bounds__(256) mha_fwd_mfma(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                    const bf16* __restrict__ v, bf16* __restrict__ o,
                                                    float* __restrict__ lse2, MhaGeom g) {
  constexpr int LD = D + 8, KC = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][64 * LD];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][64 * LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, il = lane & 15, gq = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const long tb = (long)b * g.L;
  const bf16* qb = q + tb * g.qps + h * D;
  const bf16* kb_ = k + tb * g.kps + h * D;
  const bf16* vb_ = v + tb * g.vps + h * D;
  const int q0 = blockIdx.x * 128 + w * 32;
  const float c = g.scale * LOG2E;
  // Q as the B operand of S^T = K Q^T: lane = query il of tile t, d = 32 kc + 8 gq ..
  bf16x8 qf[2][KC];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      uint4 u = ld16(qb, g.qps, q0 + 16 * t + il, g.L, 32 * kc + 8 * gq);
      qf[t][kc] = *reinterpret_cast<bf16x8*>(&u);
    }
  f32x4 O[2][DT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) O[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  const int nkb = (g.L + 63) / 64;
  Stage2<D, 256> st;
  st.load(kb_, g.kps, vb_, g.vps, 0, g.L, tid);
  st.store(Ks[0], Vs[0], tid);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) st.load(kb_, g.kps, vb_, g.vps, (kb + 1) * 64, g.L, tid);
    const bf16* K_ = Ks[kb & 1];
    const bf16* V_ = Vs[kb & 1];
    // S^T: [t][chunk c2][tile tt]; lane: query il, keys 32 c2 + 8 gq + 4 tt + r
    f32x4 S[2][2][2];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const bf16x8 kf = rd_row(K_, LD, 32 * c2 + prow(il, tt), 32 * kc, lane);
          a0 = mma(kf, qf[0][kc], a0);
          a1 = mma(kf, qf[1][kc], a1);
        }
        S[0][c2][tt] = a0;
        S[1][c2][tt] = a1;
      }
    const int kbase = kb * 64;
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float mx = -INFINITY;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kbase + 32 * c2 + 8 * gq + 4 * tt + r;
            const float s = key < g.L ? S[t][c2][tt][r] * c : -INFINITY;
            S[t][c2][tt][r] = s;
            mx = fmaxf(mx, s);
          }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[t], mx);
      const float al = ex2(m[t] - mn);
      float sum = 0.f;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = ex2(S[t][c2][tt][r] - mn);
            sum += p;
            pf[t][c2][4 * tt + r] = bfbits(p);
          }
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[t] = l[t] * al + sum;
      m[t] = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) O[t][dt] *= al;
    }
    // O^T[d][q] += sum_k V[k][d] P[q][k]
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const bf16x8 vf = rd_col(V_, LD, 16 * dt, 32 * c2, lane);
        O[0][dt] = mma(vf, pf[0][c2], O[0][dt]);
        O[1][dt] = mma(vf, pf[1][c2], O[1][dt]);
      }
    if (kb + 1 < nkb) st.store(Ks[(kb + 1) & 1], Vs[(kb + 1) & 1], tid);
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qi = q0 + 16 * t + il;
    if (qi >= g.L) continue;
    const float inv = 1.f / l[t];
    bf16* orow = o + (tb + qi) * g.ops + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      union { bf16 x[4]; uint2 u; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.x[r] = __float2bfloat16(O[t][dt][r] * inv);
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * gq) = pk.u;
    }
    if (gq == 0) lse2[((long)b * g.nh + h) * g.L + qi] = m[t] + __log2f(l[t]);
  }
}

// dQ: like the forward (4 waves x 32 queries), K / V tiles streamed; dS in registers is the B
// fragment of dQ^T = K^T dS^T.
template <int D>
__global__ void __launch_bounds__(256) mha_bwd_dq_mfma(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                       const bf16* __restrict__ v, const bf16* __restrict__ dout,
                                                       const float* __restrict__ lse2, const float* __restrict__ Dq,
                                                       bf16* __restrict__ dq, MhaGeom g) {
  constexpr int LD = D + 8, KC = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][64 * LD];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][64 * LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, il = lane & 15, gq = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const long tb = (long)b * g.L;
  const int q0 = blockIdx.x * 128 + w * 32;
  const float c = g.scale * LOG2E;
  bf16x8 qf[2][KC], df[2][KC];
  float L2[2], Di[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qi = q0 + 16 * t + il;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      uint4 u = ld16(q + tb * g.qps + h * D, g.qps, qi, g.L, 32 * kc + 8 * gq);
      qf[t][kc] = *reinterpret_cast<bf16x8*>(&u);
      uint4 u2 = ld16(dout + tb * g.ops + h * D, g.ops, qi, g.L, 32 * kc + 8 * gq);
      df[t][kc] = *reinterpret_cast<bf16x8*>(&u2);
    }
    const long row = ((long)b * g.nh + h) * g.L + (qi < g.L ? qi : 0);
    L2[t] = lse2[row];
    Di[t] = Dq[row];
  }
  f32x4 A[2][DT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) A[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (g.L + 63) / 64;
  Stage2<D, 256> st;
  const bf16* kb_ = k + tb * g.kps + h * D;
  const bf16* vb_ = v + tb * g.vps + h * D;
  st.load(kb_, g.kps, vb_, g.vps, 0, g.L, tid);
  st.store(Ks[0], Vs[0], tid);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) st.load(kb_, g.kps, vb_, g.vps, (kb + 1) * 64, g.L, tid);
    const bf16* K_ = Ks[kb & 1];
    const bf16* V_ = Vs[kb & 1];
    bf16x8 dsf[2][2];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      f32x4 S[2][2], P[2][2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const int r = 32 * c2 + prow(il, tt);
          const bf16x8 kf = rd_row(K_, LD, r, 32 * kc, lane);
          const bf16x8 vf = rd_row(V_, LD, r, 32 * kc, lane);
          s0 = mma(kf, qf[0][kc], s0);
          s1 = mma(kf, qf[1][kc], s1);
          p0 = mma(vf, df[0][kc], p0);
          p1 = mma(vf, df[1][kc], p1);
        }
        S[0][tt] = s0; S[1][tt] = s1; P[0][tt] = p0; P[1][tt] = p1;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kb * 64 + 32 * c2 + 8 * gq + 4 * tt + r;
            const float p = key < g.L ? ex2(S[t][tt][r] * c - L2[t]) : 0.f;
            dsf[t][c2][4 * tt + r] = bfbits(p * (P[t][tt][r] - Di[t]));
          }
    }
    // dQ^T[d][q] += sum_k K[k][d] dS[q][k]
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const bf16x8 kf = rd_col(K_, LD, 16 * dt, 32 * c2, lane);
        A[0][dt] = mma(kf, dsf[0][c2], A[0][dt]);
        A[1][dt] = mma(kf, dsf[1][c2], A[1][dt]);
      }
    if (kb + 1 < nkb) st.store(Ks[(kb + 1) & 1], Vs[(kb + 1) & 1], tid);
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qi = q0 + 16 * t + il;
    if (qi >= g.L) continue;
    bf16* row = dq + (tb + qi) * g.ops + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      union { bf16 x[4]; uint2 u; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.x[r] = __float2bfloat16(A[t][dt][r] * g.scale);
      *reinterpret_cast<uint2*>(row + 16 * dt + 4 * gq) = pk.u;
    }
  }
}

// dK, dV: 4 waves x 32 keys per workgroup, Q / dO tiles (64 queries) streamed with their lse2 and
// Dq.  S = Q K^T with permuted Q rows leaves a lane holding P[8 consecutive queries][key il]: the B
// fragment of dV^T = dO^T P and (as dS) of dK^T = Q^T dS.
template <int D>
__global__ void __launch_bounds__(256) mha_bwd_dkdv_mfma(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                         const bf16* __restrict__ v, const bf16* __restrict__ dout,
                                                         const float* __restrict__ lse2, const float* __restrict__ Dq,
                                                         bf16* __restrict__ dk, bf16* __restrict__ dv, MhaGeom g) {
  constexpr int LD = D + 8, KC = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16 Qs[2][64 * LD];
  __shared__ __attribute__((aligned(16))) bf16 Ds[2][64 * LD];
  __shared__ float Ls[2][64], Dd[2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, il = lane & 15, gq = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const long tb = (long)b * g.L;
  const long rb = ((long)b * g.nh + h) * g.L;
  const int k0 = blockIdx.x * 128 + w * 32;
  const float c = g.scale * LOG2E;
  bf16x8 kf[2][KC], vf[2][KC];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      uint4 u = ld16(k + tb * g.kps + h * D, g.kps, k0 + 16 * t + il, g.L, 32 * kc + 8 * gq);
      kf[t][kc] = *reinterpret_cast<bf16x8*>(&u);
      uint4 u2 = ld16(v + tb * g.vps + h * D, g.vps, k0 + 16 * t + il, g.L, 32 * kc + 8 * gq);
      vf[t][kc] = *reinterpret_cast<bf16x8*>(&u2);
    }
  f32x4 AK[2][DT], AV[2][DT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      AK[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      AV[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  const int nqb = (g.L + 63) / 64;
  Stage2<D, 256> st;
  const bf16* qb_ = q + tb * g.qps + h * D;
  const bf16* db_ = dout + tb * g.ops + h * D;
  float lv = 0.f, dvv = 0.f;
  st.load(qb_, g.qps, db_, g.ops, 0, g.L, tid);
  if (tid < 64) {
    lv = tid < g.L ? lse2[rb + tid] : 0.f;
    dvv = tid < g.L ? Dq[rb + tid] : 0.f;
  }
  st.store(Qs[0], Ds[0], tid);
  if (tid < 64) { Ls[0][tid] = lv; Dd[0][tid] = dvv; }
  __syncthreads();
  for (int qb = 0; qb < nqb; ++qb) {
    if (qb + 1 < nqb) {
      st.load(qb_, g.qps, db_, g.ops, (qb + 1) * 64, g.L, tid);
      if (tid < 64) {
        const int qi = (qb + 1) * 64 + tid;
        lv = qi < g.L ? lse2[rb + qi] : 0.f;
        dvv = qi < g.L ? Dq[rb + qi] : 0.f;
      }
    }
    const bf16* Q_ = Qs[qb & 1];
    const bf16* D_ = Ds[qb & 1];
    const float* Lq = Ls[qb & 1];
    const float* Dl = Dd[qb & 1];
    bf16x8 pf[2][2], dsf[2][2];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      f32x4 S[2][2], P[2][2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const int r = 32 * c2 + prow(il, tt);
          const bf16x8 qa = rd_row(Q_, LD, r, 32 * kc, lane);
          const bf16x8 da = rd_row(D_, LD, r, 32 * kc, lane);
          s0 = mma(qa, kf[0][kc], s0);
          s1 = mma(qa, kf[1][kc], s1);
          p0 = mma(da, vf[0][kc], p0);
          p1 = mma(da, vf[1][kc], p1);
        }
        S[0][tt] = s0; S[1][tt] = s1; P[0][tt] = p0; P[1][tt] = p1;
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 32 * c2 + 8 * gq + 4 * tt + r;  // query within the block
          const bool ok = qb * 64 + ql < g.L;
          const float lq = Lq[ql], dq_ = Dl[ql];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const float p = ok ? ex2(S[t][tt][r] * c - lq) : 0.f;
            pf[t][c2][4 * tt + r] = bfbits(p);
            dsf[t][c2][4 * tt + r] = bfbits(p * (P[t][tt][r] - dq_));
          }
        }
    }
    // dV^T[d][k] += sum_q dO[q][d] P[q][k];  dK^T[d][k] += sum_q Q[q][d] dS[q][k]
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const bf16x8 da = rd_col(D_, LD, 16 * dt, 32 * c2, lane);
        const bf16x8 qa = rd_col(Q_, LD, 16 * dt, 32 * c2, lane);
        AV[0][dt] = mma(da, pf[0][c2], AV[0][dt]);
        AV[1][dt] = mma(da, pf[1][c2], AV[1][dt]);
        AK[0][dt] = mma(qa, dsf[0][c2], AK[0][dt]);
        AK[1][dt] = mma(qa, dsf[1][c2], AK[1][dt]);
      }
    if (qb + 1 < nqb) {
      st.store(Qs[(qb + 1) & 1], Ds[(qb + 1) & 1], tid);
      if (tid < 64) { Ls[(qb + 1) & 1][tid] = lv; Dd[(qb + 1) & 1][tid] = dvv; }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kj = k0 + 16 * t + il;
    if (kj >= g.L) continue;
    bf16* rk = dk + (tb + kj) * g.ops + h * D;
    bf16* rv = dv + (tb + kj) * g.ops + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      union { bf16 x[4]; uint2 u; } pk, pv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pk.x[r] = __float2bfloat16(AK[t][dt][r] * g.scale);
        pv.x[r] = __float2bfloat16(AV[t][dt][r]);
      }
      *reinterpret_cast<uint2*>(rk + 16 * dt + 4 * gq) = pk.u;
      *reinterpret_cast<uint2*>(rv + 16 * dt + 4 * gq) = pv.u;
    }
  }
}

// ---------------------------------------------------------------- dropout (nn.Dropout, train mode)
// y = x * keep(seed, m, c) / (1 - p); the keep bit is a counter-based hash (splitmix64) of the
// element's (row, channel) index, so the backward regenerates the same mask from the seed.
DEV float u01(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps, long M, int C, float p,
                               const unsigned long long* __restrict__ seed_ptr) {
  const unsigned long long seed = *seed_ptr;  // device-resident: a graph replay reads the seed drawn for that replay
  const long total = M * C;
  const float sc = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / C;
    const int cc = (int)(i % C);
    const float v = to_f(x[m * xps + cc]);
    y[m * yps + cc] = from_f<T>(u01(seed, (unsigned long long)i) >= p ? v * sc : 0.f);
  }
}

inline bool mfma_ok(int dtype, const MhaGeom& g, const void* const* ps) {
  if (!dtype || !(g.d == 32 || g.d == 64 || g.d == 128)) return false;
  if (g.qps % 8 || g.kps % 8 || g.vps % 8 || g.ops % 8) return false;
  for (int i = 0; i < 7; ++i)
    if (ps[i] && ((uintptr_t)ps[i] & 15)) return false;
  return true;
}

}  // namespace

// ================================================================ C ABI (include/dmayolo.h)
DMY_API int dmy_mha_fwd(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps, void* o,
                        long ops, float* lse2, int B, int L, int nh, int d, float scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (B <= 0 || L <= 0) return 0;
  if (d <= 0 || d > 128 || nh <= 0) return (int)hipErrorInvalidValue;
  MhaGeom g{B, L, nh, d, qps, kps, vps, ops, scale};
  const void* ps[7] = {q, k, v, o, nullptr, nullptr, nullptr};
  if (mfma_ok(dtype, g, ps)) {
    const dim3 grid(ceil_div(L, 128), nh, B);
    const bf16 *Q = (const bf16*)q, *K = (const bf16*)k, *V = (const bf16*)v;
    if (d == 32) mha_fwd_mfma<32><<<grid, 256, 0, st>>>(Q, K, V, (bf16*)o, lse2, g);
    else if (d == 64) mha_fwd_mfma<64><<<grid, 256, 0, st>>>(Q, K, V, (bf16*)o, lse2, g);
    else mha_fwd_mfma<128><<<grid, 256, 0, st>>>(Q, K, V, (bf16*)o, lse2, g);
    return (int)hipGetLastError();
  }
  const dim3 grid(ceil_div(L, 64), nh, B);
  if (dtype) mha_fwd_generic<bf16><<<grid, 64, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse2, g);
  else mha_fwd_generic<float><<<grid, 64, 0, st>>>((const float*)q, (const float*)k, (const float*)v, (float*)o, lse2, g);
  return (int)hipGetLastError();
}

// dq / dk / dv use token stride `ops` (the stride of o / dO); Dq = fp32 workspace [B * nh * L]
DMY_API int dmy_mha_bwd(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps,
                        const void* o, const void* dout, long ops, const float* lse2, float* Dq, void* dq, void* dk,
                        void* dv, int B, int L, int nh, int d, float scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (B <= 0 || L <= 0) return 0;
  if (d <= 0 || d > 128 || nh <= 0) return (int)hipErrorInvalidValue;
  MhaGeom g{B, L, nh, d, qps, kps, vps, ops, scale};
  const int rg = grid_cap(ceil_div((long)B * L * nh, 256), 4096);
  if (dtype) mha_rowdot<bf16><<<rg, 256, 0, st>>>((const bf16*)o, (const bf16*)dout, Dq, g);
  else mha_rowdot<float><<<rg, 256, 0, st>>>((const float*)o, (const float*)dout, Dq, g);
  const void* ps[7] = {q, k, v, dout, dq, dk, dv};
  if (mfma_ok(dtype, g, ps)) {
    const dim3 grid(ceil_div(L, 128), nh, B);
    const bf16 *Q = (const bf16*)q, *K = (const bf16*)k, *V = (const bf16*)v, *DO = (const bf16*)dout;
#define MHA_BWD(D)                                                                                      \
    mha_bwd_dq_mfma<D><<<grid, 256, 0, st>>>(Q, K, V, DO, lse2, Dq, (bf16*)dq, g);                         \
    mha_bwd_dkdv_mfma<D><<<grid, 256, 0, st>>>(Q, K, V, DO, lse2, Dq, (bf16*)dk, (bf16*)dv, g);
    if (d == 32) { MHA_BWD(32) }
    else if (d == 64) { MHA_BWD(64) }
    else { MHA_BWD(128) }
#undef MHA_BWD
    return (int)hipGetLastError();
  }
  const dim3 g1(ceil_div(L, 64), nh, B), g2(ceil_div(L, 32), nh, B);
  if (dtype) {
    mha_bwd_dq_generic<bf16><<<g1, 64, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse2, Dq, (bf16*)dq, g);
    mha_bwd_dkdv_generic<bf16><<<g2, 32, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse2, Dq, (bf16*)dk, (bf16*)dv, g);
  } else {
    mha_bwd_dq_generic<float><<<g1, 64, 0, st>>>((const float*)q, (const float*)k, (const float*)v, (const float*)dout, lse2, Dq, (float*)dq, g);
    mha_bwd_dkdv_generic<float><<<g2, 32, 0, st>>>((const float*)q, (const float*)k, (const float*)v, (const float*)dout, lse2, Dq, (float*)dk, (float*)dv, g);
  }
  return (int)hipGetLastError();
}

// generic-path forward / backward regardless of dtype and head dim (test reference for the MFMA path)
DMY_API int dmy_mha_fwd_ref(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps,
                            void* o, long ops, float* lse2, int B, int L, int nh, int d, float scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (B <= 0 || L <= 0) return 0;
  if (d <= 0 || d > 128 || nh <= 0) return (int)hipErrorInvalidValue;
  MhaGeom g{B, L, nh, d, qps, kps, vps, ops, scale};
  const dim3 grid(ceil_div(L, 64), nh, B);
  if (dtype) mha_fwd_generic<bf16><<<grid, 64, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse2, g);
  else mha_fwd_generic<float><<<grid, 64, 0, st>>>((const float*)q, (const float*)k, (const float*)v, (float*)o, lse2, g);
  return (int)hipGetLastError();
}

// seed = state = splitmix64 step of the per-device generator state (one lane, vector store): launched on the
// stream before each dropout forward, so HIP-graph replays draw a fresh mask every step
__global__ void dropout_seed_kernel(unsigned long long* state, unsigned long long* seed) {
  if (threadIdx.x == 0) {
    const unsigned long long s = *state + 0x9E3779B97F4A7C15ull;
    *state = s;
    unsigned long long z = (s ^ (s >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    *seed = z ^ (z >> 31);
  }
}

DMY_API int dmy_dropout_seed(unsigned long long* state, unsigned long long* seed, void* stream) {
  dropout_seed_kernel<<<1, 64, 0, (hipStream_t)stream>>>(state, seed);
  return (int)hipGetLastError();
}

DMY_API int dmy_dropout(int dtype, const void* x, long xps, void* y, long yps, long M, int C, float p,
                        const unsigned long long* seed, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M * C == 0) return 0;
  if (!(p >= 0.f && p < 1.f)) return (int)hipErrorInvalidValue;
  const int g = grid_cap(ceil_div(M * C, 256), 8192);
  if (dtype) dropout_kernel<bf16><<<g, 256, 0, st>>>((const bf16*)x, xps, (bf16*)y, yps, M, C, p, seed);
  else dropout_kernel<float><<<g, 256, 0, st>>>((const float*)x, xps, (float*)y, yps, M, C, p, seed);
  return (int)hipGetLastError();
}
