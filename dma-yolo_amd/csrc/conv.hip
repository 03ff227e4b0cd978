// Implicit-GEMM convolution for gfx950 (forward, data-grad, weight-grad), NHWC activations.
//
// Replaces the ATen/MIOpen conv2d that the reference reaches from
//   models/cspcm.py:15-20 (YAML Conv), models/common.py:67-73 (Conv), :1279-1316 (SCConv k2/k3/k4),
//   :1158-1207 (CoorAttention 1x1 convs), :1257-1276 (SPPFCSPC), models/yolo.py:71 (Detect 1x1),
//   and nn.Linear in the Swin layers (:452-545, 97-117) as 1x1 convs over tokens.
//
// One GEMM core, three operand loaders:
//   fwd  : C[m=(b,oh,ow)][n=cout]      = sum_k A[m][k=(kh,kw,ci)]   * W[n][k]          (W = OHWI)
//   dgrad: C[m=(b,ih,iw)][n=ci]        = sum_k dY[m'(m,kh,kw)][co]  * Wt[n][k=(kh,kw,co)] (Wt = IHWO)
//   wgrad: C[m=cout][n=(kh,kw,ci)]     = sum_pix dY[pix][m] * X[pix shifted][ci]        (split-K over pixels)
// Tiles are staged global -> registers -> LDS ([row][k] with k contiguous, rows padded so the
// MFMA fragment reads are bank-conflict free), double-buffered with one barrier per K-step.
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16, f32 -> v_mfma_f32_16x16x4_f32 (exact fp32, parity mode).
#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int NT = 256;  // 4 waves, 2x2 over the block tile

template <typename T> struct LdsCfg;
template <> struct LdsCfg<bf16> { static constexpr int RS = BK + 8; };   // 80-B rows: conflict-free b128 reads
template <> struct LdsCfg<float> { static constexpr int RS = BK + 4; };  // 144-B rows

template <typename T, int BM, int BN> struct Tile {
  static constexpr int RS = LdsCfg<T>::RS;
  static constexpr int VW = Traits<T>::VW;
  static constexpr int STAGE = (BM + BN) * RS;  // elements per pipeline stage
  static constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 fragments per wave
};

// ---------------------------------------------------------------- MFMA over one staged K-step
template <int BM, int BN>
DEV void mma_step(const bf16* As, const bf16* Bs, f32x4 (&acc)[BM / 32][BN / 32], int wm, int wn, int lane) {
  constexpr int RS = LdsCfg<bf16>::RS, TM = BM / 32, TN = BN / 32;
  bf16x8 a[TM], b[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
    a[i] = *reinterpret_cast<const bf16x8*>(As + (wm * (BM / 2) + i * 16 + (lane & 15)) * RS + 8 * (lane >> 4));
#pragma unroll
  for (int j = 0; j < TN; ++j)
    b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * (BN / 2) + j * 16 + (lane & 15)) * RS + 8 * (lane >> 4));
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

template <int BM, int BN>
DEV void mma_step(const float* As, const float* Bs, f32x4 (&acc)[BM / 32][BN / 32], int wm, int wn, int lane) {
  constexpr int RS = LdsCfg<float>::RS, TM = BM / 32, TN = BN / 32;
#pragma unroll
  for (int kk = 0; kk < BK / 4; ++kk) {
    float a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = As[(wm * (BM / 2) + i * 16 + (lane & 15)) * RS + 4 * kk + (lane >> 4)];
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = Bs[(wn * (BN / 2) + j * 16 + (lane & 15)) * RS + 4 * kk + (lane >> 4)];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// ---------------------------------------------------------------- generic pipelined main loop
// Loader contract:  load(kt, ra, rb) issues global loads for K-tile kt into registers;
//                   store(As, Bs, ra, rb) writes them into one LDS stage.
template <typename T, int BM, int BN, class L>
DEV void mainloop(L& ld, int kt0, int kt1, T* lds, f32x4 (&acc)[BM / 32][BN / 32]) {
  using TT = Tile<T, BM, BN>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  uint4 ra[L::CA], rb[L::CB];
  if (kt0 >= kt1) return;
  ld.load(kt0, ra, rb);
  int buf = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    T* As = lds + buf * TT::STAGE;
    T* Bs = As + BM * TT::RS;
    ld.store(As, Bs, ra, rb);
    __syncthreads();
    if (kt + 1 < kt1) ld.load(kt + 1, ra, rb);
    mma_step<BM, BN>(As, Bs, acc, wm, wn, lane);
    buf ^= 1;
  }
}

// row-major [row][k] vector store into LDS
template <typename T, int RS> DEV void st_vec(T* base, int row, int col, const uint4& v) {
  *reinterpret_cast<uint4*>(base + row * RS + col) = v;
}
// transposed store: element e of the vector goes to [row0+e][col]
template <typename T, int RS> DEV void st_tr(T* base, int row0, int col, const uint4& v) {
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int i = 0; i < Traits<T>::VW; ++i) base[(row0 + i) * RS + col] = e[i];
}

struct Geom {
  int N, H, W, C;      // input activation (forward sense)
  int K, KH, KW, S, P;  // out channels, kernel, stride, pad
  int OH, OW;           // output spatial
  long xps, yps;        // pixel strides of x and y (elements)
};

// ---------------------------------------------------------------- forward loader
template <typename T, int BM, int BN, bool VEC, bool P1> struct FwdLoader {
  using TT = Tile<T, BM, BN>;
  static constexpr int VW = TT::VW, KV = BK / VW, RPP = NT / KV;  // rows per pass
  static constexpr int CA = BM / RPP, CB = BN / RPP;
  const T* x; const T* w; Geom g; long M; int Ktot;
  int kc, r0;
  long abase[CA]; int ih0[CA], iw0[CA]; bool aval[CA];
  int n0;
  DEV FwdLoader(const T* x_, const T* w_, const Geom& g_, long M_, long m0, int n0_) : x(x_), w(w_), g(g_), M(M_), n0(n0_) {
    Ktot = g.KH * g.KW * g.C;
    kc = threadIdx.x % KV;
    r0 = threadIdx.x / KV;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      long m = m0 + r0 + i * RPP;
      aval[i] = m < M;
      long mm = aval[i] ? m : 0;
      int ow = (int)(mm % g.OW);
      long t = mm / g.OW;
      int oh = (int)(t % g.OH);
      int b = (int)(t / g.OH);
      if (P1) { abase[i] = mm * g.xps; ih0[i] = 0; iw0[i] = 0; }
      else { abase[i] = (long)b * g.H * g.W * g.xps; ih0[i] = oh * g.S - g.P; iw0[i] = ow * g.S - g.P; }
    }
  }
  DEV T ld_a1(int i, int k) const {
    if (!aval[i] || k >= Ktot) return from_f<T>(0.f);
    if (P1) return x[abase[i] + k];
    int ci = k % g.C, t = k / g.C, kw = t % g.KW, kh = t / g.KW;
    int ih = ih0[i] + kh, iw = iw0[i] + kw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return from_f<T>(0.f);
    return x[abase[i] + ((long)ih * g.W + iw) * g.xps + ci];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
    const int k = kt * BK + kc * VW;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (aval[i] && k < Ktot) {
          if (P1) v = *reinterpret_cast<const uint4*>(x + abase[i] + k);
          else {
            int ci = k % g.C, t = k / g.C, kw = t % g.KW, kh = t / g.KW;
            int ih = ih0[i] + kh, iw = iw0[i] + kw;
            if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
              v = *reinterpret_cast<const uint4*>(x + abase[i] + ((long)ih * g.W + iw) * g.xps + ci);
          }
        }
        ra[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&ra[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = ld_a1(i, k + j);
      }
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      int n = n0 + r0 + i * RPP;
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n < g.K && k < Ktot) v = *reinterpret_cast<const uint4*>(w + (long)n * Ktot + k);
        rb[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&rb[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = (n < g.K && k + j < Ktot) ? w[(long)n * Ktot + k + j] : from_f<T>(0.f);
      }
    }
  }
  DEV void store(T* As, T* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) st_vec<T, TT::RS>(As, r0 + i * RPP, kc * VW, ra[i]);
#pragma unroll
    for (int i = 0; i < CB; ++i) st_vec<T, TT::RS>(Bs, r0 + i * RPP, kc * VW, rb[i]);
  }
};

// ---------------------------------------------------------------- data-grad loader
// A[m=(b,ih,iw)][k=(kh,kw,co)] = dy[b, (ih+P-kh)/S, (iw+P-kw)/S, co] when divisible and in range.
template <typename T, int BM, int BN, bool VEC, bool P1> struct DgradLoader {
  using TT = Tile<T, BM, BN>;
  static constexpr int VW = TT::VW, KV = BK / VW, RPP = NT / KV;
  static constexpr int CA = BM / RPP, CB = BN / RPP;
  const T* dy; const T* wt; Geom g; long M; int Ktot;
  int kc, r0, n0;
  long abase[CA]; int ih[CA], iw[CA]; bool aval[CA];
  DEV DgradLoader(const T* dy_, const T* wt_, const Geom& g_, long M_, long m0, int n0_) : dy(dy_), wt(wt_), g(g_), M(M_), n0(n0_) {
    Ktot = g.KH * g.KW * g.K;
    kc = threadIdx.x % KV;
    r0 = threadIdx.x / KV;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      long m = m0 + r0 + i * RPP;
      aval[i] = m < M;
      long mm = aval[i] ? m : 0;
      iw[i] = (int)(mm % g.W);
      long t = mm / g.W;
      ih[i] = (int)(t % g.H);
      int b = (int)(t / g.H);
      abase[i] = P1 ? mm * g.yps : (long)b * g.OH * g.OW * g.yps;
    }
  }
  DEV T ld_a1(int i, int k) const {
    if (!aval[i] || k >= Ktot) return from_f<T>(0.f);
    if (P1) return dy[abase[i] + k];
    int co = k % g.K, t = k / g.K, kw = t % g.KW, kh = t / g.KW;
    int hn = ih[i] + g.P - kh, wn = iw[i] + g.P - kw;
    if (hn < 0 || wn < 0 || hn % g.S || wn % g.S) return from_f<T>(0.f);
    int oh = hn / g.S, ow = wn / g.S;
    if (oh >= g.OH || ow >= g.OW) return from_f<T>(0.f);
    return dy[abase[i] + ((long)oh * g.OW + ow) * g.yps + co];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
    const int k = kt * BK + kc * VW;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (aval[i] && k < Ktot) {
          if (P1) v = *reinterpret_cast<const uint4*>(dy + abase[i] + k);
          else {
            int co = k % g.K, t = k / g.K, kw = t % g.KW, kh = t / g.KW;
            int hn = ih[i] + g.P - kh, wn = iw[i] + g.P - kw;
            if (hn >= 0 && wn >= 0 && (hn % g.S) == 0 && (wn % g.S) == 0) {
              int oh = hn / g.S, ow = wn / g.S;
              if (oh < g.OH && ow < g.OW)
                v = *reinterpret_cast<const uint4*>(dy + abase[i] + ((long)oh * g.OW + ow) * g.yps + co);
            }
          }
        }
        ra[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&ra[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = ld_a1(i, k + j);
      }
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      int n = n0 + r0 + i * RPP;
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n < g.C && k < Ktot) v = *reinterpret_cast<const uint4*>(wt + (long)n * Ktot + k);
        rb[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&rb[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = (n < g.C && k + j < Ktot) ? wt[(long)n * Ktot + k + j] : from_f<T>(0.f);
      }
    }
  }
  DEV void store(T* As, T* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) st_vec<T, TT::RS>(As, r0 + i * RPP, kc * VW, ra[i]);
#pragma unroll
    for (int i = 0; i < CB; ++i) st_vec<T, TT::RS>(Bs, r0 + i * RPP, kc * VW, rb[i]);
  }
};

// ---------------------------------------------------------------- weight-grad loader
// GEMM over pixels: A[m=co][pix] = dy[pix][co]; B[n=(kh,kw,ci)][pix] = x[pix shifted by (kh,kw)][ci].
// Global loads are coalesced along channels; the LDS stores transpose into [row][pix].
template <typename T, int BM, int BN, bool VECA, bool VECB> struct WgradLoader {
  using TT = Tile<T, BM, BN>;
  static constexpr int VW = TT::VW;
  static constexpr int AV = BM / VW, BV = BN / VW;  // vectors per pixel row
  static constexpr int CA = BK * AV / NT, CB = BK * BV / NT;
  const T* x; const T* dy; Geom g; long NP; int Ntot, m0, n0;
  DEV WgradLoader(const T* x_, const T* dy_, const Geom& g_, int m0_, int n0_) : x(x_), dy(dy_), g(g_), m0(m0_), n0(n0_) {
    NP = (long)g.N * g.OH * g.OW;
    Ntot = g.KH * g.KW * g.C;
  }
  DEV T ld_b1(long pix, int n) const {
    if (pix >= NP || n >= Ntot) return from_f<T>(0.f);
    int ow = (int)(pix % g.OW);
    long t = pix / g.OW;
    int oh = (int)(t % g.OH), b = (int)(t / g.OH);
    int ci = n % g.C, u = n / g.C, kw = u % g.KW, kh = u / g.KW;
    int ih = oh * g.S - g.P + kh, iw = ow * g.S - g.P + kw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return from_f<T>(0.f);
    return x[(((long)b * g.H + ih) * g.W + iw) * g.xps + ci];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      int c = threadIdx.x + i * NT;
      int pl = c / AV, cv = c % AV;
      long pix = (long)kt * BK + pl;
      int co = m0 + cv * VW;
      if (VECA) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (pix < NP && co < g.K) v = *reinterpret_cast<const uint4*>(dy + pix * g.yps + co);
        ra[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&ra[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = (pix < NP && co + j < g.K) ? dy[pix * g.yps + co + j] : from_f<T>(0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      int c = threadIdx.x + i * NT;
      int pl = c / BV, nv = c % BV;
      long pix = (long)kt * BK + pl;
      int n = n0 + nv * VW;
      if (VECB) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (pix < NP && n < Ntot) {
          int ow = (int)(pix % g.OW);
          long t = pix / g.OW;
          int oh = (int)(t % g.OH), b = (int)(t / g.OH);
          int ci = n % g.C, u = n / g.C, kw = u % g.KW, kh = u / g.KW;
          int ih = oh * g.S - g.P + kh, iw = ow * g.S - g.P + kw;
          if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
            v = *reinterpret_cast<const uint4*>(x + (((long)b * g.H + ih) * g.W + iw) * g.xps + ci);
        }
        rb[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&rb[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = ld_b1(pix, n + j);
      }
    }
  }
  DEV void store(T* As, T* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      int c = threadIdx.x + i * NT;
      st_tr<T, TT::RS>(As, (c % AV) * VW, c / AV, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      int c = threadIdx.x + i * NT;
      st_tr<T, TT::RS>(Bs, (c % BV) * VW, c / BV, rb[i]);
    }
  }
};

// ---------------------------------------------------------------- kernels
template <typename T, int BM, int BN, bool VEC, bool P1>
__global__ void __launch_bounds__(NT) conv_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      const float* __restrict__ bias, T* __restrict__ y,
                                                      float* __restrict__ psum, float* __restrict__ psq, Geom g) {
  using TT = Tile<T, BM, BN>;
  __shared__ __attribute__((aligned(16))) T lds[2 * TT::STAGE];
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  FwdLoader<T, BM, BN, VEC, P1> ld(x, w, g, M, m0, n0);
  f32x4 acc[TT::TM][TT::TN];
#pragma unroll
  for (int i = 0; i < TT::TM; ++i)
#pragma unroll
    for (int j = 0; j < TT::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (g.KH * g.KW * g.C + BK - 1) / BK;
  mainloop<T, BM, BN>(ld, 0, nk, lds, acc);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int j = 0; j < TT::TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = (bias != nullptr && n < g.K) ? bias[n] : 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < TT::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long m = m0 + wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        float v = acc[i][j][r] + bv;
        if (m < M && n < g.K) {
          y[m * g.yps + n] = from_f<T>(v);
          s1 += v;
          s2 += v * v;
        }
      }
    }
    if (psum != nullptr) {
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 16 && n < g.K) {
        const long row = (long)blockIdx.x * 2 + wm;
        psum[row * g.K + n] = s1;
        psq[row * g.K + n] = s2;
      }
    }
  }
}

template <typename T, int BM, int BN, bool VEC, bool P1>
__global__ void __launch_bounds__(NT) conv_dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ wt,
                                                        T* __restrict__ dx, int accumulate, Geom g) {
  using TT = Tile<T, BM, BN>;
  __shared__ __attribute__((aligned(16))) T lds[2 * TT::STAGE];
  const long M = (long)g.N * g.H * g.W;
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  DgradLoader<T, BM, BN, VEC, P1> ld(dy, wt, g, M, m0, n0);
  f32x4 acc[TT::TM][TT::TN];
#pragma unroll
  for (int i = 0; i < TT::TM; ++i)
#pragma unroll
    for (int j = 0; j < TT::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (g.KH * g.KW * g.K + BK - 1) / BK;
  mainloop<T, BM, BN>(ld, 0, nk, lds, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int j = 0; j < TT::TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < TT::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long m = m0 + wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        if (m < M && n < g.C) {
          T* p = dx + m * g.xps + n;
          float v = acc[i][j][r];
          if (accumulate) v += to_f(*p);
          *p = from_f<T>(v);
        }
      }
  }
}

template <typename T, int BM, int BN, bool VECA, bool VECB>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        float* __restrict__ dw, int kt_per_split, Geom g) {
  using TT = Tile<T, BM, BN>;
  __shared__ __attribute__((aligned(16))) T lds[2 * TT::STAGE];
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  WgradLoader<T, BM, BN, VECA, VECB> ld(x, dy, g, m0, n0);
  const long NP = (long)g.N * g.OH * g.OW;
  const int nk = (int)((NP + BK - 1) / BK);
  const int kt0 = blockIdx.z * kt_per_split;
  const int kt1 = min(nk, kt0 + kt_per_split);
  f32x4 acc[TT::TM][TT::TN];
#pragma unroll
  for (int i = 0; i < TT::TM; ++i)
#pragma unroll
    for (int j = 0; j < TT::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop<T, BM, BN>(ld, kt0, kt1, lds, acc);
  const int Ntot = g.KH * g.KW * g.C;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int j = 0; j < TT::TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < TT::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        if (m < g.K && n < Ntot) atomicAdd(dw + (long)m * Ntot + n, acc[i][j][r]);
      }
  }
}

// OIHW fp32 master weights -> T OHWI (forward B operand, input channels padded to Cp with zeros)
// and T IHWO (data-grad B operand).
template <typename T>
__global__ void wprep_kernel(const float* __restrict__ w, T* __restrict__ wf, T* __restrict__ wt, int K, int C, int Cp,
                             int KH, int KW) {
  const long total = (long)K * Cp * KH * KW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    long t = i / Cp;
    const int kw = (int)(t % KW);
    t /= KW;
    const int kh = (int)(t % KH);
    const int k = (int)(t / KH);
    const float v = c < C ? w[(((long)k * C + c) * KH + kh) * KW + kw] : 0.f;
    if (wf) wf[i] = from_f<T>(v);
    if (wt && c < C) wt[(((long)c * KH + kh) * KW + kw) * K + k] = from_f<T>(v);
  }
}

// OHWI fp32 grad accumulator (input channels padded to Cp) -> OIHW param-shaped gradient
__global__ void wgrad_to_oihw_kernel(const float* __restrict__ src, float* __restrict__ dst, int K, int C, int Cp,
                                     int KH, int KW) {
  const long total = (long)K * C * KH * KW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int kw = (int)(i % KW);
    long t = i / KW;
    int kh = (int)(t % KH);
    t /= KH;
    int c = (int)(t % C);
    int k = (int)(t / C);
    dst[i] = src[(((long)k * KH + kh) * KW + kw) * Cp + c];
  }
}

// ---------------------------------------------------------------- host dispatch
Geom make_geom(int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps) {
  Geom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.KH = KH; g.KW = KW; g.S = S; g.P = P;
  g.OH = OH; g.OW = OW; g.xps = xps; g.yps = yps;
  return g;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// tile choice shared by launch and partial-row query
inline bool big_tile(long M, int N) { return M >= 4096 && N > 64; }

template <typename T, int BM, int BN>
int launch_fwd(const T* x, const T* w, const float* b, T* y, float* ps, float* pq, const Geom& g, hipStream_t st) {
  constexpr int VW = Traits<T>::VW;
  const long M = (long)g.N * g.OH * g.OW;
  dim3 grid(ceil_div(M, BM), ceil_div(g.K, BN));
  const bool p1 = g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0;
  const bool vec = g.C % VW == 0 && g.xps % VW == 0 && aligned16(x);
  if (vec && p1) conv_fwd_kernel<T, BM, BN, true, true><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g);
  else if (vec) conv_fwd_kernel<T, BM, BN, true, false><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g);
  else if (p1) conv_fwd_kernel<T, BM, BN, false, true><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g);
  else conv_fwd_kernel<T, BM, BN, false, false><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g);
  return (int)hipGetLastError();
}

template <typename T, int BM, int BN>
int launch_dgrad(const T* dy, const T* wt, T* dx, int acc, const Geom& g, hipStream_t st) {
  constexpr int VW = Traits<T>::VW;
  const long M = (long)g.N * g.H * g.W;
  dim3 grid(ceil_div(M, BM), ceil_div(g.C, BN));
  const bool p1 = g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0;
  const bool vec = g.K % VW == 0 && g.yps % VW == 0 && aligned16(dy);
  if (vec && p1) conv_dgrad_kernel<T, BM, BN, true, true><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g);
  else if (vec) conv_dgrad_kernel<T, BM, BN, true, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g);
  else if (p1) conv_dgrad_kernel<T, BM, BN, false, true><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g);
  else conv_dgrad_kernel<T, BM, BN, false, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g);
  return (int)hipGetLastError();
}

template <typename T, int BM, int BN>
int launch_wgrad(const T* x, const T* dy, float* dw, const Geom& g, hipStream_t st) {
  constexpr int VW = Traits<T>::VW;
  const long NP = (long)g.N * g.OH * g.OW;
  const int Ntot = g.KH * g.KW * g.C;
  const int gm = ceil_div(g.K, BM), gn = ceil_div(Ntot, BN);
  const int nk = ceil_div(NP, BK);
  // split-K over pixels: aim for ~2048 blocks, >= 8 K-tiles per split
  int splits = 2048 / (gm * gn);
  if (splits < 1) splits = 1;
  int maxs = nk / 8;
  if (maxs < 1) maxs = 1;
  if (splits > maxs) splits = maxs;
  int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  dim3 grid(gm, gn, splits);
  const bool va = g.K % VW == 0 && g.yps % VW == 0 && aligned16(dy);
  const bool vb = g.C % VW == 0 && g.xps % VW == 0 && aligned16(x);
  (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * Ntot, st);
  if (va && vb) conv_wgrad_kernel<T, BM, BN, true, true><<<grid, NT, 0, st>>>(x, dy, dw, per, g);
  else if (va) conv_wgrad_kernel<T, BM, BN, true, false><<<grid, NT, 0, st>>>(x, dy, dw, per, g);
  else if (vb) conv_wgrad_kernel<T, BM, BN, false, true><<<grid, NT, 0, st>>>(x, dy, dw, per, g);
  else conv_wgrad_kernel<T, BM, BN, false, false><<<grid, NT, 0, st>>>(x, dy, dw, per, g);
  return (int)hipGetLastError();
}

template <typename T>
int conv_fwd_t(const void* x, const void* w, const float* b, void* y, float* ps, float* pq, const Geom& g, hipStream_t st) {
  const long M = (long)g.N * g.OH * g.OW;
  if (big_tile(M, g.K))
    return launch_fwd<T, 128, 128>((const T*)x, (const T*)w, b, (T*)y, ps, pq, g, st);
  return launch_fwd<T, 64, 64>((const T*)x, (const T*)w, b, (T*)y, ps, pq, g, st);
}
template <typename T>
int conv_dgrad_t(const void* dy, const void* wt, void* dx, int acc, const Geom& g, hipStream_t st) {
  const long M = (long)g.N * g.H * g.W;
  if (big_tile(M, g.C)) return launch_dgrad<T, 128, 128>((const T*)dy, (const T*)wt, (T*)dx, acc, g, st);
  return launch_dgrad<T, 64, 64>((const T*)dy, (const T*)wt, (T*)dx, acc, g, st);
}
template <typename T>
int conv_wgrad_t(const void* x, const void* dy, float* dw, const Geom& g, hipStream_t st) {
  if (g.K > 64 && g.KH * g.KW * g.C > 64) return launch_wgrad<T, 128, 128>((const T*)x, (const T*)dy, dw, g, st);
  return launch_wgrad<T, 64, 64>((const T*)x, (const T*)dy, dw, g, st);
}

}  // namespace

// ================================================================ C ABI (include/dmayolo.h)
DMY_API int dmy_conv_fwd_partial_rows(long M, int K) { return 2 * ceil_div(M, big_tile(M, K) ? 128 : 64); }

DMY_API int dmy_conv_fwd(int dtype, const void* x, const void* w, const float* bias, void* y, float* psum, float* psq,
                         int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW,
                         long yps, void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * OH * OW == 0 || K == 0) return 0;
  return dtype ? conv_fwd_t<bf16>(x, w, bias, y, psum, psq, g, (hipStream_t)stream)
               : conv_fwd_t<float>(x, w, bias, y, psum, psq, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int accumulate, int N, int H, int W,
                           int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps,
                           void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * H * W == 0 || C == 0) return 0;
  return dtype ? conv_dgrad_t<bf16>(dy, wt, dx, accumulate, g, (hipStream_t)stream)
               : conv_dgrad_t<float>(dy, wt, dx, accumulate, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_wgrad(int dtype, const void* x, const void* dy, float* dw_ohwi, int N, int H, int W, int C,
                           long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  return dtype ? conv_wgrad_t<bf16>(x, dy, dw_ohwi, g, (hipStream_t)stream)
               : conv_wgrad_t<float>(x, dy, dw_ohwi, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_wprep(int dtype, const float* w_oihw, void* w_ohwi, void* w_ihwo, int K, int C, int Cp, int KH,
                           int KW, void* stream) {
  const long total = (long)K * Cp * KH * KW;
  const int grid = grid_cap(ceil_div(total, 256), 1024);
  if (dtype) wprep_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (bf16*)w_ohwi, (bf16*)w_ihwo, K, C, Cp, KH, KW);
  else wprep_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (float*)w_ohwi, (float*)w_ihwo, K, C, Cp, KH, KW);
  return (int)hipGetLastError();
}

DMY_API int dmy_conv_wgrad_to_oihw(const float* dw_ohwi, float* dw_oihw, int K, int C, int Cp, int KH, int KW,
                                   void* stream) {
  const long total = (long)K * C * KH * KW;
  wgrad_to_oihw_kernel<<<grid_cap(ceil_div(total, 256), 1024), 256, 0, (hipStream_t)stream>>>(dw_ohwi, dw_oihw, K, C,
                                                                                               Cp, KH, KW);
  return (int)hipGetLastError();
}
