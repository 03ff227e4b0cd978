// Implicit-GEMM convolution for gfx950 (forward, data-grad, weight-grad), NHWC activations.
//
// Replaces the ATen/MIOpen conv2d that the reference reaches from
//   models/cspcm.py:15-20 (YAML Conv), models/common.py:67-73 (Conv), :1279-1316 (SCConv k2/k3/k4),
//   :1158-1207 (CoorAttention 1x1 convs), :1257-1276 (SPPFCSPC), models/yolo.py:71 (Detect 1x1),
//   and nn.Linear in the Swin layers (:452-545, 97-117) as 1x1 convs over tokens.
//
// One GEMM core, three operand loaders:
//   fwd  : C[m=(b,oh,ow)][n=cout]  = sum_k A[m][k=(kh,kw,ci)]  * W[n][k]            W  = OHWI
//   dgrad: C[m=(b,ih,iw)][n=ci]    = sum_k dY[m'(m,kh,kw)][co] * Wt[n][k=(kh,kw,co)] Wt = IHWO
//          stride-2 layers are split into the 4 output-parity classes so only live taps are
//          multiplied (sub-pixel decomposition; 4x less MFMA work for 3x3/s2).
//   wgrad: C[m=cout][n=(kh,kw,ci)] = sum_pix dY[pix][m] * X[pix shifted][ci]       split-K over pixels
// Staging: global -> registers -> LDS, two stages, one barrier per BK-deep step (BK = 64 bf16 / 32 f32).
//   "m-major" tiles ([row][k], k contiguous, 16-B row pad => conflict-free ds_read_b128 fragments);
//   "k-major" tiles ([k][row], as loaded from NHWC; wgrad) are read with ds_read_b64_tr_b16, the
//   16-B chunks XOR-swizzled per k-row so the transposed reads are bank-conflict free.
// Epilogues go through LDS so every global store / atomic is a 16-B vector or a 256-B wave segment.
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16, f32 -> v_mfma_f32_16x16x4_f32 (exact fp32, parity mode).
// Block ids are remapped so consecutive tiles sharing an A panel land on one XCD (L2 reuse).
#include <mutex>
#include "common.h"
#include <cstdlib>
#include <type_traits>
#include <atomic>
#include <cmath>

namespace {

constexpr int NT = 256;  // 4 waves, 2x2 over the block tile

template <typename T> struct Cfg;
template <> struct Cfg<bf16> {
  static constexpr int BK = 64, PADM = 8, PADK = 0;  // m-major rows 144 B; k-major rows unpadded (swizzled)
};
template <> struct Cfg<float> {
  static constexpr int BK = 32, PADM = 4, PADK = 16;
};

template <typename T, int BM, int BN, bool AK, bool BKM> struct Tile {
  static constexpr int BK = Cfg<T>::BK, VW = Traits<T>::VW;
  static constexpr int RSM = BK + Cfg<T>::PADM;  // m-major row stride (elements)
  static constexpr int A_ELEMS = AK ? BK * (BM + Cfg<T>::PADK) : BM * RSM;
  static constexpr int B_ELEMS = BKM ? BK * (BN + Cfg<T>::PADK) : BN * RSM;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int TM = BM / 32, TN = BN / 32;
  static constexpr int STAGE_BYTES = 2 * STAGE * (int)sizeof(T);
  static constexpr int CT_BYTES = BM * (BN + 8) * 4;  // C tile (largest epilogue use, fp32 worst case)
  static constexpr int LDS_BYTES = STAGE_BYTES > CT_BYTES ? STAGE_BYTES : CT_BYTES;
};

// ---------------------------------------------------------------- LDS placement helpers
// k-major tile [k][ROW] with ROW = BM (or BN) elements; bf16 16-B chunks XOR-swizzled per k-row
template <typename T, int ROW> DEV int kmaj_off(int k, int row) {
  if constexpr (sizeof(T) == 2) {
    constexpr int RB = ROW * 2;  // bytes per k-row
    const int c = row >> 3, w = row & 7;
    int key;
    if constexpr (RB >= 256) key = 2 * ((k & 3) | (((k >> 3) & 1) << 2));
    else key = 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
    return k * ROW + (((c ^ key) & (ROW / 8 - 1)) << 3) + w;
  } else {
    return k * (ROW + Cfg<float>::PADK) + row;
  }
}

// ---------------------------------------------------------------- fragment reads + MFMA
// bf16: A frag lane l = A[m0 + (l&15)][8(l>>4) .. +8)
template <int RSM> DEV bf16x8 frag_m(const bf16* base, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + (r0 + (lane & 15)) * RSM + k0 + 8 * (lane >> 4));
}
template <int ROW> DEV bf16x8 frag_k(const bf16* base, int r0, int k0, int lane) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3;
  const bf16* a0 = base + kmaj_off<bf16, ROW>(k0 + 8 * g + q, r0 + 4 * p);
  const bf16* a1 = base + kmaj_off<bf16, ROW>(k0 + 8 * g + 4 + q, r0 + 4 * p);
  s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
  s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <int BM, int BN, bool AK, bool BKM>
DEV void mma_step(const bf16* As, const bf16* Bs, f32x4 (&acc)[BM / 32][BN / 32], int wm, int wn, int lane) {
  using TT = Tile<bf16, BM, BN, AK, BKM>;
  constexpr int TM = TT::TM, TN = TT::TN;
#pragma unroll
  for (int ks = 0; ks < TT::BK; ks += 32) {
    bf16x8 a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r0 = wm * (BM / 2) + i * 16;
      a[i] = AK ? frag_k<BM>(As, r0, ks, lane) : frag_m<TT::RSM>(As, r0, ks, lane);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r0 = wn * (BN / 2) + j * 16;
      b[j] = BKM ? frag_k<BN>(Bs, r0, ks, lane) : frag_m<TT::RSM>(Bs, r0, ks, lane);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

template <int BM, int BN, bool AK, bool BKM>
DEV void mma_step(const float* As, const float* Bs, f32x4 (&acc)[BM / 32][BN / 32], int wm, int wn, int lane) {
  using TT = Tile<float, BM, BN, AK, BKM>;
  constexpr int TM = TT::TM, TN = TT::TN;
#pragma unroll
  for (int kk = 0; kk < TT::BK / 4; ++kk) {
    const int k = 4 * kk + (lane >> 4);
    float a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * (BM / 2) + i * 16 + (lane & 15);
      a[i] = AK ? As[kmaj_off<float, BM>(k, r)] : As[r * TT::RSM + k];
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wn * (BN / 2) + j * 16 + (lane & 15);
      b[j] = BKM ? Bs[kmaj_off<float, BN>(k, r)] : Bs[r * TT::RSM + k];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// ---------------------------------------------------------------- pipelined main loop
// Loader contract: load(kt, ra, rb) issues the global loads of K-tile kt into registers;
//                  store(As, Bs, ra, rb) writes them into one LDS stage.
template <typename T, int BM, int BN, bool AK, bool BKM, class L>
DEV void mainloop(L& ld, int kt0, int kt1, T* lds, f32x4 (&acc)[BM / 32][BN / 32]) {
  using TT = Tile<T, BM, BN, AK, BKM>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  uint4 ra[L::CA], rb[L::CB];
  if (kt0 >= kt1) return;
  ld.load(kt0, ra, rb);
  int buf = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    T* As = lds + buf * TT::STAGE;
    T* Bs = As + TT::A_ELEMS;
    ld.store(As, Bs, ra, rb);
    __syncthreads();
    if (kt + 1 < kt1) ld.load(kt + 1, ra, rb);
    mma_step<BM, BN, AK, BKM>(As, Bs, acc, wm, wn, lane);
    buf ^= 1;
  }
}

template <typename T, int RSM> DEV void st_m(T* base, int row, int col, const uint4& v) {
  *reinterpret_cast<uint4*>(base + row * RSM + col) = v;
}
template <typename T, int ROW> DEV void st_k(T* base, int k, int row0, const uint4& v) {
  *reinterpret_cast<uint4*>(base + kmaj_off<T, ROW>(k, row0)) = v;
}

struct Geom {
  int N, H, W, C;       // input activation (forward sense)
  int K, KH, KW, S, P;  // out channels, kernel, stride, pad
  int OH, OW;           // output spatial
  long xps, yps;        // pixel strides of x and y (elements)
  int oihw;             // weight-grad: write [K][C][KH][KW] (torch OIHW) instead of the GEMM view [K][KH][KW][C]
  int zeroed;           // weight-grad: the output is already zero (caller-cleared arena): no memset
  // weight-grad deterministic mode: split s stores its partial tile to dws[s * dws_slab + idx] (no atomics) and
  // wgrad_split_reduce sums the splits in index order; null = fp32 atomics into dw
  float* dws;
  long dws_slab;
  int* plan;            // non-null: only report the split count the dispatch would use (*plan), launch nothing
};

// weight-grad epilogue store: deterministic workspace slot of this split, or an fp32 atomic into dw
DEV void wgrad_out(const Geom& g, float* dw, int split, long idx, float v) {
  if (g.dws != nullptr) g.dws[(long)split * g.dws_slab + idx] = v;
  else atomicAdd(dw + idx, v);
}

// Inference epilogue (eval BatchNorm folded per channel + activation + residual, applied to the T-rounded
// conv output exactly as dmy_bn_act_fwd would read it back): y = act(z * scale + shift) (+ res).
// scale / shift may be null (1 / 0).  `on` = 0 leaves the plain (+bias) store.
struct Epi {
  const float* scale;
  const float* shift;
  const void* res;
  long rps;
  int act;
  int on;
};

// eval coefficients of the 8 consecutive channels n .. n + 7 (all < K): 16-B loads when the arrays are 16-B aligned
// (n % 8 == 0 at every call), scale 1 / shift 0 when absent
DEV void epi_coef8(const Epi& ep, int n, float (&sc)[8], float (&sh)[8]) {
  const bool vs = (((uintptr_t)ep.scale | (uintptr_t)ep.shift) & 15) == 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float4 a = make_float4(1.f, 1.f, 1.f, 1.f), b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vs) {
      if (ep.scale) a = *reinterpret_cast<const float4*>(ep.scale + n + 4 * h);
      if (ep.shift) b = *reinterpret_cast<const float4*>(ep.shift + n + 4 * h);
    } else {
      if (ep.scale) a = make_float4(ep.scale[n + 4 * h], ep.scale[n + 4 * h + 1], ep.scale[n + 4 * h + 2], ep.scale[n + 4 * h + 3]);
      if (ep.shift) b = make_float4(ep.shift[n + 4 * h], ep.shift[n + 4 * h + 1], ep.shift[n + 4 * h + 2], ep.shift[n + 4 * h + 3]);
    }
    sc[4 * h] = a.x; sc[4 * h + 1] = a.y; sc[4 * h + 2] = a.z; sc[4 * h + 3] = a.w;
    sh[4 * h] = b.x; sh[4 * h + 1] = b.y; sh[4 * h + 2] = b.z; sh[4 * h + 3] = b.w;
  }
}
// f = act(f * sc + sh) (+ r) over 8 values, the activation switch outside the element loop (act_fwd_n)
DEV void epi_apply8(int act, float (&f)[8], const float (&sc)[8], const float (&sh)[8], const float* r) {
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = f[e] * sc[e] + sh[e];
  act_fwd_n<8>(act, f);
  if (r != nullptr) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += r[e];
  }
}

template <typename T, int VW>
DEV void epi_store(const Epi& ep, const T* src, T* dst, int n, int K, long m, bool full) {
  if constexpr (sizeof(T) == 2 && VW == 8) {
    if (full) {  // 8 channels of a bf16 row: vector coefficient / residual loads, one hoisted activation switch
      float f[8], sc[8], sh[8], r8[8];
      unpack<T>(*reinterpret_cast<const uint4*>(src), f);
      epi_coef8(ep, n, sc, sh);
      const T* rp = ep.res != nullptr ? reinterpret_cast<const T*>(ep.res) + m * ep.rps + n : nullptr;
      if (rp != nullptr) {
        if ((((uintptr_t)rp) & 15) == 0) {
          unpack<T>(*reinterpret_cast<const uint4*>(rp), r8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) r8[j] = to_f(rp[j]);
        }
      }
      epi_apply8(ep.act, f, sc, sh, rp != nullptr ? r8 : nullptr);
      *reinterpret_cast<uint4*>(dst) = pack<T>(f);
      return;
    }
  }
  float f[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    if (n + j < K) {
      const float sc = ep.scale ? ep.scale[n + j] : 1.f, sh = ep.shift ? ep.shift[n + j] : 0.f;
      float v = act_fwd(ep.act, to_f(src[j]) * sc + sh);
      if (ep.res) v += to_f(reinterpret_cast<const T*>(ep.res)[m * ep.rps + n + j]);
      f[j] = v;
    } else {
      f[j] = 0.f;
    }
  }
  if (full) {
    *reinterpret_cast<uint4*>(dst) = pack<T>(f);
  } else {
    for (int j = 0; j < VW && n + j < K; ++j) dst[j] = from_f<T>(f[j]);
  }
}

// weight-grad GEMM column n = (kh * KW + kw) * C + c -> its offset inside one output row of dw
DEV long wgrad_col(const Geom& g, int n) {
  if (!g.oihw) return n;
  const int taps = g.KH * g.KW;
  return (long)(n % g.C) * taps + n / g.C;
}

// parity class of a stride-2 data-grad (blockIdx.y): output pixels with (ih%2, iw%2) == (a, b)
struct Parity {
  int a, b;      // parities
  int kh0, kw0;  // first live tap ( (a + P) & 1 )
  int nkh, nkw;  // live taps per dim
  int Hc, Wc;    // pixels of this class per image (rows / cols)
};
DEV Parity parity_class(const Geom& g, int cls) {
  Parity q;
  q.a = cls >> 1;
  q.b = cls & 1;
  q.kh0 = (q.a + g.P) & 1;
  q.kw0 = (q.b + g.P) & 1;
  q.nkh = (g.KH - q.kh0 + 1) / 2;
  q.nkw = (g.KW - q.kw0 + 1) / 2;
  q.Hc = (g.H - q.a + 1) / 2;
  q.Wc = (g.W - q.b + 1) / 2;
  return q;
}

// ---------------------------------------------------------------- forward loader (m-major A and B)
template <typename T, int BM, int BN, bool VEC, bool P1> struct FwdLoader {
  using TT = Tile<T, BM, BN, false, false>;
  static constexpr int BK = TT::BK, VW = TT::VW, KV = BK / VW, RPP = NT / KV;
  static constexpr int CA = BM / RPP, CB = BN / RPP;
  const T* x; const T* w; Geom g; long M; int Ktot;
  int kc, r0, n0;
  long abase[CA]; int ih0[CA], iw0[CA]; bool aval[CA];
  DEV FwdLoader(const T* x_, const T* w_, const Geom& g_, long M_, long m0, int n0_) : x(x_), w(w_), g(g_), M(M_), n0(n0_) {
    Ktot = g.KH * g.KW * g.C;
    kc = threadIdx.x % KV;
    r0 = threadIdx.x / KV;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const long m = m0 + r0 + i * RPP;
      aval[i] = m < M;
      const long mm = aval[i] ? m : 0;
      const int ow = (int)(mm % g.OW);
      const long t = mm / g.OW;
      const int oh = (int)(t % g.OH);
      const int b = (int)(t / g.OH);
      if (P1) { abase[i] = mm * g.xps; ih0[i] = 0; iw0[i] = 0; }
      else { abase[i] = (long)b * g.H * g.W * g.xps; ih0[i] = oh * g.S - g.P; iw0[i] = ow * g.S - g.P; }
    }
  }
  DEV T ld_a1(int i, int k) const {
    if (!aval[i] || k >= Ktot) return from_f<T>(0.f);
    if (P1) return x[abase[i] + k];
    const int ci = k % g.C, t = k / g.C, kw = t % g.KW, kh = t / g.KW;
    const int ih = ih0[i] + kh, iw = iw0[i] + kw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return from_f<T>(0.f);
    return x[abase[i] + ((long)ih * g.W + iw) * g.xps + ci];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
    const int k = kt * BK + kc * VW;
    int ci = 0, kh = 0, kw = 0;
    if (!P1) {
      ci = k % g.C;
      const int t = k / g.C;
      kw = t % g.KW;
      kh = t / g.KW;
    }
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (aval[i] && k < Ktot) {
          if (P1) v = *reinterpret_cast<const uint4*>(x + abase[i] + k);
          else {
            const int ih = ih0[i] + kh, iw = iw0[i] + kw;
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
      const int n = n0 + r0 + i * RPP;
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
    for (int i = 0; i < CA; ++i) st_m<T, TT::RSM>(As, r0 + i * RPP, kc * VW, ra[i]);
#pragma unroll
    for (int i = 0; i < CB; ++i) st_m<T, TT::RSM>(Bs, r0 + i * RPP, kc * VW, rb[i]);
  }
};

// ---------------------------------------------------------------- data-grad loader (m-major)
// S2: stride-2 parity class; m enumerates the class pixels, k = (live kh, live kw, co)
template <typename T, int BM, int BN, bool VEC, bool P1, bool S2> struct DgradLoader {
  using TT = Tile<T, BM, BN, false, false>;
  static constexpr int BK = TT::BK, VW = TT::VW, KV = BK / VW, RPP = NT / KV;
  static constexpr int CA = BM / RPP, CB = BN / RPP;
  const T* dy; const T* wt; Geom g; Parity q; long M; int Ktot, kc, r0, n0;
  long abase[CA]; int ih[CA], iw[CA]; bool aval[CA];
  DEV DgradLoader(const T* dy_, const T* wt_, const Geom& g_, const Parity& q_, long M_, long m0, int n0_)
      : dy(dy_), wt(wt_), g(g_), q(q_), M(M_), n0(n0_) {
    Ktot = S2 ? q.nkh * q.nkw * g.K : g.KH * g.KW * g.K;
    kc = threadIdx.x % KV;
    r0 = threadIdx.x / KV;
    const int Hm = S2 ? q.Hc : g.H, Wm = S2 ? q.Wc : g.W;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const long m = m0 + r0 + i * RPP;
      aval[i] = m < M;
      const long mm = aval[i] ? m : 0;
      const int x_ = (int)(mm % Wm);
      const long t = mm / Wm;
      const int y_ = (int)(t % Hm);
      const int b = (int)(t / Hm);
      ih[i] = S2 ? 2 * y_ + q.a : y_;
      iw[i] = S2 ? 2 * x_ + q.b : x_;
      abase[i] = P1 ? mm * g.yps : (long)b * g.OH * g.OW * g.yps;
    }
  }
  // tap index t (row-major over the (live) taps) -> kernel (kh, kw)
  DEV void tap(int t, int& kh, int& kw) const {
    if (S2) { kh = q.kh0 + 2 * (t / q.nkw); kw = q.kw0 + 2 * (t % q.nkw); }
    else { kh = t / g.KW; kw = t % g.KW; }
  }
  DEV bool src(int i, int kh, int kw, long& off) const {
    const int hn = ih[i] + g.P - kh, wn = iw[i] + g.P - kw;
    if (hn < 0 || wn < 0) return false;
    if (!S2 && g.S > 1 && ((hn % g.S) || (wn % g.S))) return false;
    const int oh = S2 ? (hn >> 1) : hn / g.S, ow = S2 ? (wn >> 1) : wn / g.S;
    if (oh >= g.OH || ow >= g.OW) return false;
    off = abase[i] + ((long)oh * g.OW + ow) * g.yps;
    return true;
  }
  DEV T ld_a1(int i, int k) const {
    if (!aval[i] || k >= Ktot) return from_f<T>(0.f);
    if (P1) return dy[abase[i] + k];
    int kh, kw;
    tap(k / g.K, kh, kw);
    long off;
    return src(i, kh, kw, off) ? dy[off + k % g.K] : from_f<T>(0.f);
  }
  DEV T ld_b1(int n, int k) const {
    if (n >= g.C || k >= Ktot) return from_f<T>(0.f);
    if (!S2) return wt[(long)n * Ktot + k];
    int kh, kw;
    tap(k / g.K, kh, kw);
    return wt[(((long)n * g.KH + kh) * g.KW + kw) * g.K + k % g.K];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
    const int k = kt * BK + kc * VW;
    const int co = k % g.K;
    int kh = 0, kw = 0;
    if (!P1) tap(k / g.K, kh, kw);
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (aval[i] && k < Ktot) {
          if (P1) v = *reinterpret_cast<const uint4*>(dy + abase[i] + k);
          else {
            long off;
            if (src(i, kh, kw, off)) v = *reinterpret_cast<const uint4*>(dy + off + co);
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
      const int n = n0 + r0 + i * RPP;
      if (VEC) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n < g.C && k < Ktot) {
          const long wo = S2 ? (((long)n * g.KH + kh) * g.KW + kw) * g.K + co : (long)n * Ktot + k;
          v = *reinterpret_cast<const uint4*>(wt + wo);
        }
        rb[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&rb[i]);
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = ld_b1(n, k + j);
      }
    }
  }
  DEV void store(T* As, T* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) st_m<T, TT::RSM>(As, r0 + i * RPP, kc * VW, ra[i]);
#pragma unroll
    for (int i = 0; i < CB; ++i) st_m<T, TT::RSM>(Bs, r0 + i * RPP, kc * VW, rb[i]);
  }
};

// ---------------------------------------------------------------- weight-grad loader (k-major A and B)
// A[k=pix][m=co] = dy[pix][co];  B[k=pix][n=(kh,kw,ci)] = x[pix shifted by (kh,kw)][ci]
template <typename T, int BM, int BN, bool VECA, bool VECB> struct WgradLoader {
  using TT = Tile<T, BM, BN, true, true>;
  static constexpr int BK = TT::BK, VW = TT::VW;
  static constexpr int AV = BM / VW, BV = BN / VW;  // vectors per pixel row
  static constexpr int CA = BK * AV / NT, CB = BK * BV / NT;
  const T* x; const T* dy; Geom g; long NP; int Ntot, m0, n0;
  // the n -> (kh, kw, ci) decomposition is fixed per thread across K-steps
  int b_kh[CB], b_kw[CB], b_ci[CB];
  bool b_ok[CB];
  DEV WgradLoader(const T* x_, const T* dy_, const Geom& g_, int m0_, int n0_) : x(x_), dy(dy_), g(g_), m0(m0_), n0(n0_) {
    NP = (long)g.N * g.OH * g.OW;
    Ntot = g.KH * g.KW * g.C;
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = threadIdx.x + i * NT;
      const int n = n0 + (c % BV) * VW;
      b_ok[i] = n < Ntot;
      b_ci[i] = n % g.C;
      const int u = n / g.C;
      b_kw[i] = u % g.KW;
      b_kh[i] = u / g.KW;
    }
  }
  DEV T ld_b1(long pix, int n) const {
    if (pix >= NP || n >= Ntot) return from_f<T>(0.f);
    const int ow = (int)(pix % g.OW);
    const long t = pix / g.OW;
    const int oh = (int)(t % g.OH), b = (int)(t / g.OH);
    const int ci = n % g.C, u = n / g.C, kw = u % g.KW, kh = u / g.KW;
    const int ih = oh * g.S - g.P + kh, iw = ow * g.S - g.P + kw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return from_f<T>(0.f);
    return x[(((long)b * g.H + ih) * g.W + iw) * g.xps + ci];
  }
  DEV void load(int kt, uint4* ra, uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = threadIdx.x + i * NT;
      const long pix = (long)kt * BK + c / AV;
      const int co = m0 + (c % AV) * VW;
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
      const int c = threadIdx.x + i * NT;
      const long pix = (long)kt * BK + c / BV;
      if (VECB) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (pix < NP && b_ok[i]) {
          const int ow = (int)(pix % g.OW);
          const long t = pix / g.OW;
          const int oh = (int)(t % g.OH), b = (int)(t / g.OH);
          const int ih = oh * g.S - g.P + b_kh[i], iw = ow * g.S - g.P + b_kw[i];
          if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
            v = *reinterpret_cast<const uint4*>(x + (((long)b * g.H + ih) * g.W + iw) * g.xps + b_ci[i]);
        }
        rb[i] = v;
      } else {
        T* e = reinterpret_cast<T*>(&rb[i]);
        const int n = n0 + (c % BV) * VW;
#pragma unroll
        for (int j = 0; j < VW; ++j) e[j] = ld_b1(pix, n + j);
      }
    }
  }
  DEV void store(T* As, T* Bs, const uint4* ra, const uint4* rb) const {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = threadIdx.x + i * NT;
      st_k<T, BM>(As, c / AV, (c % AV) * VW, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = threadIdx.x + i * NT;
      st_k<T, BN>(Bs, c / BV, (c % BV) * VW, rb[i]);
    }
  }
};

// ---------------------------------------------------------------- XCD-aware tile order
// Linear block id -> logical tile id such that each XCD (block id mod 8 under round-robin
// dispatch) walks a contiguous range of logical tiles; n-tiles of one m-panel are adjacent.
// Speed only: any placement is correct.  Bijective for every grid size.
DEV int xcd_remap(int id, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = id % 8, loc = id / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int BM, int BN> DEV void zero_acc(f32x4 (&acc)[BM / 32][BN / 32]) {
#pragma unroll
  for (int i = 0; i < BM / 32; ++i)
#pragma unroll
    for (int j = 0; j < BN / 32; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Write the accumulator tile (+bias) as T into LDS [BM][BN+8] (row-major) and return per-column
// sums / sums of squares of the fp32 values (rows < M) for the BN statistics.
template <typename T, int BM, int BN>
DEV void acc_to_lds(const f32x4 (&acc)[BM / 32][BN / 32], T* ct, const float* bias, int n0, int K, long m0, long M,
                    float* s1, float* s2) {
  constexpr int RS = BN + 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int j = 0; j < BN / 32; ++j) {
    const int c = wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = (bias != nullptr && n0 + c < K) ? bias[n0 + c] : 0.f;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < BM / 32; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        const float v = acc[i][j][r] + bv;
        ct[row * RS + c] = from_f<T>(v);
        if (m0 + row < M) {
          a += v;
          b += v * v;
        }
      }
    s1[j] = a;
    s2[j] = b;
  }
}

// ---------------------------------------------------------------- kernels
template <typename T, int BM, int BN, bool VEC, bool P1>
__global__ void __launch_bounds__(NT) conv_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      const float* __restrict__ bias, T* __restrict__ y,
                                                      float* __restrict__ psum, float* __restrict__ psq, Geom g,
                                                      int gm, int gn, Epi ep) {
  using TT = Tile<T, BM, BN, false, false>;
  __shared__ __attribute__((aligned(16))) char smem[TT::LDS_BYTES];
  T* lds = reinterpret_cast<T*>(smem);
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  FwdLoader<T, BM, BN, VEC, P1> ld(x, w, g, M, m0, n0);
  f32x4 acc[TT::TM][TT::TN];
  zero_acc<BM, BN>(acc);
  const int nk = (g.KH * g.KW * g.C + TT::BK - 1) / TT::BK;
  mainloop<T, BM, BN, false, false>(ld, 0, nk, lds, acc);
  __syncthreads();
  float s1[TT::TN], s2[TT::TN];
  acc_to_lds<T, BM, BN>(acc, lds, bias, n0, g.K, m0, M, s1, s2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
  if (psum != nullptr) {
#pragma unroll
    for (int j = 0; j < TT::TN; ++j) {
      float a = s1[j], b = s2[j];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
      if (lane < 16 && n < g.K) {
        const long row = (long)tm * 2 + wm;
        psum[row * g.K + n] = a;
        psq[row * g.K + n] = b;
      }
    }
  }
  __syncthreads();
  // coalesced 16-B stores of the staged tile
  constexpr int VW = TT::VW, RS = BN + 8, CPR = BN / VW;
  const bool vec = (g.yps % VW) == 0 && (g.K % VW) == 0 && ((((uintptr_t)y) & 15) == 0);
  for (int e = threadIdx.x; e < BM * CPR; e += NT) {
    const int row = e / CPR, cv = e % CPR;
    const long m = m0 + row;
    const int n = n0 + cv * VW;
    if (m >= M || n >= g.K) continue;
    const T* src = lds + row * RS + cv * VW;
    if (ep.on) {
      epi_store<T, VW>(ep, src, y + m * g.yps + n, n, g.K, m, vec && n + VW <= g.K);
      continue;
    }
    if (vec && n + VW <= g.K) {
      *reinterpret_cast<uint4*>(y + m * g.yps + n) = *reinterpret_cast<const uint4*>(src);
    } else {
      for (int j = 0; j < VW && n + j < g.K; ++j) y[m * g.yps + n + j] = src[j];
    }
  }
}

template <typename T, int BM, int BN, bool VEC, bool P1, bool S2>
__global__ void __launch_bounds__(NT) conv_dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ wt,
                                                        T* __restrict__ dx, int accumulate, Geom g, int gm, int gn) {
  using TT = Tile<T, BM, BN, false, false>;
  __shared__ __attribute__((aligned(16))) char smem[TT::LDS_BYTES];
  T* lds = reinterpret_cast<T*>(smem);
  const Parity q = parity_class(g, S2 ? (int)blockIdx.y : 0);
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = S2 ? (long)g.N * q.Hc * q.Wc : (long)g.N * g.H * g.W;
  const long m0 = (long)tm * BM;
  if (m0 >= M) return;  // a parity class can be smaller than the grid's M extent (block-uniform exit)
  const int n0 = tn * BN;
  DgradLoader<T, BM, BN, VEC, P1, S2> ld(dy, wt, g, q, M, m0, n0);
  f32x4 acc[TT::TM][TT::TN];
  zero_acc<BM, BN>(acc);
  const int Ktot = S2 ? q.nkh * q.nkw * g.K : g.KH * g.KW * g.K;
  const int nk = (Ktot + TT::BK - 1) / TT::BK;
  mainloop<T, BM, BN, false, false>(ld, 0, nk, lds, acc);
  __syncthreads();
  float s1[TT::TN], s2[TT::TN];
  acc_to_lds<T, BM, BN>(acc, lds, nullptr, n0, g.C, m0, M, s1, s2);
  __syncthreads();
  constexpr int VW = TT::VW, RS = BN + 8, CPR = BN / VW;
  const bool vec = (g.xps % VW) == 0 && (g.C % VW) == 0 && ((((uintptr_t)dx) & 15) == 0);
  const int Wm = S2 ? q.Wc : g.W, Hm = S2 ? q.Hc : g.H;
  for (int e = threadIdx.x; e < BM * CPR; e += NT) {
    const int row = e / CPR, cv = e % CPR;
    const long m = m0 + row;
    const int n = n0 + cv * VW;
    if (m >= M || n >= g.C) continue;
    long pix = m;
    if (S2) {
      const int xx = (int)(m % Wm);
      const long t = m / Wm;
      const int yy = (int)(t % Hm), b = (int)(t / Hm);
      pix = ((long)b * g.H + 2 * yy + q.a) * g.W + 2 * xx + q.b;
    }
    const T* src = lds + row * RS + cv * VW;
    T* dst = dx + pix * g.xps + n;
    if (vec && n + VW <= g.C) {
      if (accumulate) {
        float a[VW], b[VW];
        unpack<T>(*reinterpret_cast<const uint4*>(src), a);
        unpack<T>(*reinterpret_cast<const uint4*>(dst), b);
#pragma unroll
        for (int j = 0; j < VW; ++j) a[j] += b[j];
        *reinterpret_cast<uint4*>(dst) = pack<T>(a);
      } else {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
      }
    } else {
      for (int j = 0; j < VW && n + j < g.C; ++j)
        dst[j] = accumulate ? from_f<T>(to_f(src[j]) + to_f(dst[j])) : src[j];
    }
  }
}

template <typename T, int BM, int BN, bool VECA, bool VECB>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        float* __restrict__ dw, int kt_per_split, Geom g, int gm,
                                                        int gn) {
  using TT = Tile<T, BM, BN, true, true>;
  __shared__ __attribute__((aligned(16))) char smem[TT::LDS_BYTES];
  T* lds = reinterpret_cast<T*>(smem);
  // (tile, split) from the linear dispatch id: consecutive logical ids share an XCD, so all tiles of
  // a split (which read the same pixel chunk) run on one XCD and share its L2
  const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int tile = lin % (gm * gn), split = lin / (gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const int m0 = tm * BM, n0 = tn * BN;
  WgradLoader<T, BM, BN, VECA, VECB> ld(x, dy, g, m0, n0);
  const long NP = (long)g.N * g.OH * g.OW;
  const int nk = (int)((NP + TT::BK - 1) / TT::BK);
  const int kt0 = split * kt_per_split;
  const int kt1 = min(nk, kt0 + kt_per_split);
  f32x4 acc[TT::TM][TT::TN];
  zero_acc<BM, BN>(acc);
  mainloop<T, BM, BN, true, true>(ld, kt0, kt1, lds, acc);
  __syncthreads();
  // stage the fp32 partial tile in LDS, then atomics in contiguous 256-B wave segments
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int RS = BN + 4;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int i = 0; i < TT::TM; ++i)
#pragma unroll
    for (int j = 0; j < TT::TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r) * RS + wn * (BN / 2) + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int Ntot = g.KH * g.KW * g.C;
  static_assert((NT) % BN == 0, "epilogue column must be fixed per thread");
  const int c = threadIdx.x % BN, n = n0 + c;
  const long coff = wgrad_col(g, n);
  for (int e = threadIdx.x; e < BM * BN; e += NT) {
    const int row = e / BN, m = m0 + row;
    if (m < g.K && n < Ntot) wgrad_out(g, dw, split, (long)m * Ntot + coff, ct[row * RS + c]);
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

// Every conv weight of a model in one launch (training forward: the fp32 masters change every step):
// blockIdx.y = layer, blocks grid-stride over that layer's K*KH*KW*C elements (no channel padding).
struct WprepDesc {
  const float* w;
  void* wf;
  void* wt;
  int K, C, KH, KW;
};
// 32 (K) x 32 (C) x taps tiles through LDS: the OIHW rows are read contiguously (32 x 32 x taps floats) and both
// copies are written 32 consecutive elements at a time (OHWI along C, IHWO along K).  The elementwise form it
// replaces wrote the IHWO copy with a K-strided 2-byte scatter (1.59 ms per DMA-1536 step for 46 M weights).
// Kernels with more than 9 taps (the 6 x 6 stem) take the elementwise loop.
constexpr int kWpT = 9, kWpPitch = 32 * kWpT + 1;  // LDS row pitch (floats): odd, so the K-major reads are conflict-free
template <typename T>
__global__ void __launch_bounds__(256) wprep_multi_kernel(const WprepDesc* __restrict__ d) {
  const WprepDesc L = d[blockIdx.y];
  T* wf = reinterpret_cast<T*>(L.wf);
  T* wt = reinterpret_cast<T*>(L.wt);
  const int taps = L.KH * L.KW;
  if (taps > kWpT) {
    const long total = (long)L.K * L.C * taps;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
      const int c = (int)(i % L.C);
      const long t = i / L.C;
      const int tap = (int)(t % taps), k = (int)(t / taps);
      const float v = L.w[((long)k * L.C + c) * taps + tap];
      wf[i] = from_f<T>(v);
      if (wt) wt[((long)c * taps + tap) * L.K + k] = from_f<T>(v);
    }
    return;
  }
  __shared__ float s[32 * kWpPitch];  // [k][c * taps + tap]
  const int tc = (L.C + 31) / 32, nt = ((L.K + 31) / 32) * tc, row = 32 * taps;
  for (int tile = blockIdx.x; tile < nt; tile += gridDim.x) {
    const int k0 = (tile / tc) * 32, c0 = (tile % tc) * 32;
    const int nrow = min(32, L.C - c0) * taps;
    for (int e = threadIdx.x; e < 32 * row; e += 256) {
      const int kk = e / row, r = e - kk * row, k = k0 + kk;
      s[kk * kWpPitch + r] = (k < L.K && r < nrow) ? L.w[((long)k * L.C + c0) * taps + r] : 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * row; e += 256) {  // OHWI: (k, tap, c), c fastest
      const int cc = e & 31, t = e >> 5, tap = t % taps, kk = t / taps, k = k0 + kk, c = c0 + cc;
      if (k < L.K && c < L.C) wf[((long)k * taps + tap) * L.C + c] = from_f<T>(s[kk * kWpPitch + cc * taps + tap]);
    }
    if (wt) {
      for (int e = threadIdx.x; e < 32 * row; e += 256) {  // IHWO: (c, tap, k), k fastest
        const int kk = e & 31, t = e >> 5, tap = t % taps, cc = t / taps, k = k0 + kk, c = c0 + cc;
        if (k < L.K && c < L.C) wt[((long)c * taps + tap) * L.K + k] = from_f<T>(s[kk * kWpPitch + cc * taps + tap]);
      }
    }
    __syncthreads();
  }
}

// Stem k6 s2 p2 weights as the equivalent k3 s1 p1 conv over the space-to-depth image (dmy_image_s2d):
// ws[k][ky][kx][(dy * 2 + dx) * C + c] = w[k][c][2 ky + dy][2 kx + dx], channels [4C, Cs) zero
template <typename T>
__global__ void wprep_s2d_kernel(const float* __restrict__ w, T* __restrict__ ws, int K, int C, int Cs) {
  const long total = (long)K * 9 * Cs;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % Cs);
    const long t = i / Cs;
    const int tap = (int)(t % 9), k = (int)(t / 9);
    const int ky = tap / 3, kx = tap % 3;
    float v = 0.f;
    if (ch < 4 * C) {
      const int q = ch / C, c = ch - q * C;
      v = w[(((long)k * C + c) * 6 + 2 * ky + (q >> 1)) * 6 + 2 * kx + (q & 1)];
    }
    ws[i] = from_f<T>(v);
  }
}

// weight-grad of the s2d view [K][3][3][Cs] (GEMM order) -> the stem's OIHW [K][C][6][6] gradient
__global__ void wgrad_s2d_to_oihw_kernel(const float* __restrict__ src, float* __restrict__ dst, int K, int C, int Cs) {
  const long total = (long)K * C * 36;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int kw = (int)(i % 6), kh = (int)(i / 6 % 6), c = (int)(i / 36 % C), k = (int)(i / (36L * C));
    const int tap = (kh >> 1) * 3 + (kw >> 1), q = (kh & 1) * 2 + (kw & 1);
    dst[i] = src[((long)k * 9 + tap) * Cs + q * C + c];
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

// ---------------------------------------------------------------- v3 forward: LDS-DMA staged (bf16)
// BM x BN block tile of (BM/64) x (BN/64) waves, 64 x 64 per wave, BK = 64, a 3-stage LDS ring filled by
// global_load_lds_dwordx4 (no VGPR staging, no ds_write), counted vmcnt + raw s_barrier so the next
// stage's loads stay in flight across the barrier.  Operand rows are 128 B (64 bf16 of K) with the
// 16-B chunks XOR-swizzled by (row & 6): the LDS-DMA image is lane-linear (the swizzle is applied to
// each lane's SOURCE address) and the MFMA fragment reads (ds_read_b128) are conflict-free.
// Out-of-image taps / rows past M / channels past K read a zero page.
__device__ __attribute__((aligned(64))) uint4 g_zero_page[4] = {};

namespace v3 {
constexpr int BK = 64;
// WTR = output rows per wave (64: 64 x 64 wave tiles; 128: 128 x 64, the wide 256 x 256 block)
template <int BM, int BN, int NS = 3, int WTR = 64> struct Cfg3 {
  static constexpr int NSTAGE = NS;
  static constexpr int WM = BM / WTR, WN = BN / 64, NW = WM * WN, NTH = NW * 64;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  // 1-KiB LDS-DMA pieces of a stage (8 rows of 128 B) and per wave.  BM = 288 (the 288-row wide tile) has 36 A pieces
  // for 8 waves: waves take pieces j * NW + wid, the first PA % NW waves one more; only with NS = 2, whose main loop
  // waits for vmcnt(0), so the per-wave counts never enter a counted wait
  static constexpr int PA = A_BYTES / 1024, PB = B_BYTES / 1024;
  static constexpr int APW = (PA + NW - 1) / NW, BPW = PB / NW;
  static constexpr bool AEVEN = PA % NW == 0;
  static constexpr int CT = BM * (BN + 8) * 2;
  static constexpr int LDS = NSTAGE * STAGE > CT ? NSTAGE * STAGE : CT;
  static_assert(APW >= 1 && BPW >= 1 && PA * 1024 == A_BYTES && BPW * NW == PB && (AEVEN || NS == 2), "tile");
};

DEV void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// swizzled fragment read: rows of 64 bf16, lane gets X[r0 + (l&15)][k0 + 8(l>>4) .. +8)
DEV bf16x8 frag_sw(const bf16* X, int r0, int k0, int lane) {
  const int row = r0 + (lane & 15);
  const int chunk = (k0 >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(X + row * 64 + ((chunk ^ (row & 6)) << 3));
}

// Forward (DG = false): A row m = output pixel, K = (kh, kw, ci), source x[oh*S - P + kh][ow*S - P + kw].
// Data-grad, stride 1 (DG = true): A row m = input pixel, K = (kh, kw, co), source dy[ih + P - kh][iw + P - kw];
// B = the IHWO weight copy.  Both are the same gather with a sign on the tap.
template <int BM, int BN, int NS, bool P1, bool DG>
struct FwdLds {
  using C3_ = Cfg3<BM, BN, NS>;
  static_assert(C3_::AEVEN, "FwdLds: whole A pieces per wave");
  const bf16* x; const bf16* w; Geom g; int Ktot;
  int k, ci, kh, kw;  // this lane's K chunk for the next issue (advanced incrementally)
  long abase[C3_::APW]; int ih0[C3_::APW], iw0[C3_::APW]; bool aval[C3_::APW];
  long boff[C3_::BPW]; bool bval[C3_::BPW];
  // g here is the GEMM view: (H, W, C) = gathered tensor, (OH, OW) = rows, K = columns, xps = gather stride
  DEV FwdLds(const bf16* x_, const bf16* w_, const Geom& g_, long M, long m0, int n0, int wid, int lane)
      : x(x_), w(w_), g(g_) {
    Ktot = g.KH * g.KW * g.C;
    k = ((lane & 7) ^ ((lane >> 3) & 6)) * 8;  // swizzled source chunk (row & 6 == (lane >> 3) & 6)
    ci = k % g.C;
    const int t = k / g.C;
    kw = t % g.KW;
    kh = t / g.KW;
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const long m = m0 + (wid * C3_::APW + j) * 8 + (lane >> 3);
      aval[j] = m < M;
      const long mm = aval[j] ? m : 0;
      const int ow = (int)(mm % g.OW);
      const long tt = mm / g.OW;
      const int oh = (int)(tt % g.OH);
      const int b = (int)(tt / g.OH);
      if (P1) { abase[j] = mm * g.xps; ih0[j] = 0; iw0[j] = 0; }
      else if (DG) { abase[j] = (long)b * g.H * g.W * g.xps; ih0[j] = oh + g.P; iw0[j] = ow + g.P; }
      else { abase[j] = (long)b * g.H * g.W * g.xps; ih0[j] = oh * g.S - g.P; iw0[j] = ow * g.S - g.P; }
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j) {
      const int n = n0 + (wid * C3_::BPW + j) * 8 + (lane >> 3);
      bval[j] = n < g.K;
      boff[j] = (long)(bval[j] ? n : 0) * Ktot;
    }
  }
  // issue the LDS-DMA loads of the next K step into `stage`, then advance one K step
  DEV void issue(char* stage, int wid) {
    const bool kin = k < Ktot;
    const bf16* zero = reinterpret_cast<const bf16*>(g_zero_page);
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const bf16* src;
      if (P1) {
        src = (aval[j] && kin) ? x + abase[j] + k : zero;
      } else {
        const int ih = DG ? ih0[j] - kh : ih0[j] + kh, iw = DG ? iw0[j] - kw : iw0[j] + kw;
        const bool ok = aval[j] && kin && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        src = ok ? x + abase[j] + ((long)ih * g.W + iw) * g.xps + ci : zero;
      }
      glds16(src, stage + (wid * C3_::APW + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j) {
      const bf16* src = (bval[j] && kin) ? w + boff[j] + k : zero;
      glds16(src, stage + C3_::A_BYTES + (wid * C3_::BPW + j) * 1024);
    }
    k += BK;
    if (!P1) {
      ci += BK;
      while (ci >= g.C) {
        ci -= g.C;
        if (++kw == g.KW) { kw = 0; ++kh; }
      }
    }
  }
};

// Buffer-descriptor form of FwdLds for gathered tensors whose channel count is a multiple of BK
// (every K step then lies inside one tap, so the tap (kh, kw) and the channel base ci0 are uniform).
// Sources are 32-bit byte offsets against buffer descriptors: an out-of-image tap, a row past M or a
// column past K gets an offset beyond the descriptor's record count and the hardware's range check
// returns zeros (no zero page, no 64-bit address arithmetic).  Per K step a lane spends one add, two
// compares and a select per A piece and one add per B piece; the pixel bases are built once.
constexpr unsigned kBufOob = 0xFFFFFFF0u;  // >= every record count used (checked on the host)

DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
DEV void blds16(__amdgpu_buffer_rsrc_t r, unsigned off, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, off, 0, 0, 0);
}

// Stride-2 data-grad parity class (a, b) (S2): rows are the input pixels (2 i2 + a, 2 j2 + b); only the
// taps of matching parity (kh = a + P mod 2, kw = b + P mod 2, stepping by 2) reach them, from dy pixel
// (i2 + (a + P - kh) / 2, j2 + (b + P - kw) / 2).  The GEMM view g has (H, W, C) = dy, (OH, OW) = the
// class's rows, K = input channels; S2Cls carries the class and dx's spatial size for the epilogue.
struct S2Cls {
  int a, b, HX, WX;
};

// ES = operand element size in bytes: 2 (bf16, 64 elements per K step) or 1 (fp8 e4m3, 128 per K step; the
// LDS image is byte-identical: 128-B rows of 16-B chunks)
template <int BM, int BN, int NS, bool P1, bool DG, bool S2 = false, int ES = 2, int WTR = 64>
struct FwdLdsB {
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  static constexpr int BKE = 128 / ES;  // elements per K step
  __amdgpu_buffer_rsrc_t rx, rw;
  int H, W, C, KW, xps;
  int kh, kw, ci0, kpos;            // uniform cursor of the next K step
  int kw0, ca, cb, P;               // S2: first kw of the class's parity, class, pad
  int kl;                           // this lane's (swizzled) 16-B chunk within the step, in elements
  int pix[C3_::APW], ih0[C3_::APW], iw0[C3_::APW];
  bool aval[C3_::APW];
  unsigned boff[C3_::BPW];
  DEV FwdLdsB(const bf16* x, const bf16* w, const Geom& g, long M, long m0, int n0, int wid, int lane, unsigned xbytes,
              unsigned wbytes, S2Cls cls = S2Cls{0, 0, 0, 0})
      : H(g.H), W(g.W), C(g.C), KW(g.KW), xps((int)g.xps), kh(0), kw(0), ci0(0), kpos(0) {
    rx = make_rsrc(x, xbytes);
    rw = make_rsrc(w, wbytes);
    const int Ktot = g.KH * g.KW * g.C;
    P = g.P;
    ca = cls.a;
    cb = cls.b;
    kw0 = (cls.b + g.P) & 1;
    if (S2) { kh = (cls.a + g.P) & 1; kw = kw0; }
    kl = ((lane & 7) ^ ((lane >> 3) & 6)) * (16 / ES);
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const long m = m0 + apiece(wid, j) * 8 + (lane >> 3);
      aval[j] = m < M;
      const int mm = (int)(aval[j] ? m : 0);
      const int ow = mm % g.OW, t = mm / g.OW, oh = t % g.OH, b = t / g.OH;
      if (P1) { pix[j] = mm * xps; ih0[j] = 0; iw0[j] = 0; }
      else {
        ih0[j] = S2 ? oh : DG ? oh + g.P : oh * g.S - g.P;
        iw0[j] = S2 ? ow : DG ? ow + g.P : ow * g.S - g.P;
        pix[j] = ((b * g.H + ih0[j]) * g.W + iw0[j]) * xps;  // may be negative; valid taps land >= 0
      }
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j) {
      const int n = n0 + (wid * C3_::BPW + j) * 8 + (lane >> 3);
      boff[j] = n < g.K ? (unsigned)(n * Ktot + kl) * (unsigned)ES : kBufOob;
    }
  }
  // the A piece (8 rows) a wave's j-th load covers: consecutive per wave, or interleaved when the pieces do not split
  // evenly (BM = 288); a piece index >= PA is no load at all (wave-uniform)
  static DEV int apiece(int wid, int j) { return C3_::AEVEN ? wid * C3_::APW + j : j * C3_::NW + wid; }
  // advance the cursor by n K steps without loading (split-K: start at this split's first step)
  DEV void skip(int n) {
    kpos += n * BKE;
    if (!P1) {
      for (int i = 0; i < n; ++i) {
        ci0 += BKE;
        if (ci0 == C) {
          ci0 = 0;
          if (++kw == KW) {
            kw = 0;
            ++kh;
          }
        }
      }
    }
  }
  DEV void issue(char* stage, int wid) {
    const int dh = S2 ? (ca + P - kh) >> 1 : DG ? -kh : kh, dw = S2 ? (cb + P - kw) >> 1 : DG ? -kw : kw;
    const int delta = P1 ? kpos + kl : (dh * W + dw) * xps + ci0 + kl;
    const int bk = S2 ? (kh * KW + kw) * C + ci0 : kpos;  // this step's column of the (kh, kw, c) weight rows
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const int pc = apiece(wid, j);
      if (!C3_::AEVEN && pc >= C3_::PA) break;
      bool ok = aval[j];
      if (!P1) ok = ok && (unsigned)(ih0[j] + dh) < (unsigned)H && (unsigned)(iw0[j] + dw) < (unsigned)W;
      blds16(rx, ok ? (unsigned)(pix[j] + delta) * (unsigned)ES : kBufOob, stage + pc * 1024);
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j)
      blds16(rw, boff[j] == kBufOob ? kBufOob : boff[j] + (unsigned)bk * (unsigned)ES,
             stage + C3_::A_BYTES + (wid * C3_::BPW + j) * 1024);
    kpos += BKE;
    if (!P1) {
      ci0 += BKE;
      if (ci0 == C) {
        ci0 = 0;
        if (S2) {
          kw += 2;
          if (kw >= KW) { kw = kw0; kh += 2; }
        } else if (++kw == KW) {
          kw = 0;
          ++kh;
        }
      }
    }
  }
};

template <int N> DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// Main loop with the whole K step's fragments read up front (64 VGPRs), the next stage's LDS-DMA
// issued while those reads are in flight, then the step's 32 MFMAs back to back.
template <int BM, int BN, int NS, class LD>
DEV void mainloop4(LD& ld, int nk, char* smem, f32x4 (&acc)[4][4], int wid, int lane) {
  using C3_ = Cfg3<BM, BN, NS>;
  constexpr int PER = C3_::APW + C3_::BPW;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  ld.issue(smem, wid);
  if (NS == 3 && nk > 1) ld.issue(smem + C3_::STAGE, wid);
  for (int kt = 0; kt < nk; ++kt) {
    if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * C3_::STAGE);
    const bf16* Bs = As + BM * BK;
    bf16x8 a[2][4], b[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[h][i] = frag_sw(As, wm * 64 + i * 16, h * 32, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[h][j] = frag_sw(Bs, wn * 64 + j * 16, h * 32, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * C3_::STAGE, wid);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
  }
}

template <int BM, int BN, int NS, class LD>
DEV void mainloop3(LD& ld, int nk, char* smem, f32x4 (&acc)[4][4], int wid, int lane) {
  using C3_ = Cfg3<BM, BN, NS>;
  constexpr int PER = C3_::APW + C3_::BPW;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  ld.issue(smem, wid);
  if (NS == 3 && nk > 1) ld.issue(smem + C3_::STAGE, wid);
  for (int kt = 0; kt < nk; ++kt) {
    if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * C3_::STAGE, wid);
    const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * C3_::STAGE);
    const bf16* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag_sw(As, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag_sw(Bs, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
}

// Epilogue of the v3 GEMM kernels: (+bias) -> bf16 tile in LDS `ct` [BM][BN+8] + BN partials.  Partial rows
// follow the v2 numbering of dmy_conv_fwd_partial_rows: one per 64 rows of M when K > 64, one per 32 otherwise.
// Then 16-B stores (inference epilogue / accumulate / stride-2 class pixel mapping as configured).
template <int BM, int BN, int NS, bool DG, int BUF, int WTR = 64>
DEV void v3_epilogue(const f32x4 (&acc)[WTR / 16][4], bf16* ct, const float* __restrict__ bias, bf16* __restrict__ y,
                     float* __restrict__ psum, float* __restrict__ psq, int accumulate, const Geom& g, int tm,
                     long m0, int n0, const v3::S2Cls& cls, const Epi& ep) {
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  // 16-row fragments and 32-row groups per wave; PW: wave tiles of a row count that is no multiple of 32 (the 288-row
  // wide tile, 144 rows per wave) write ONE BN partial row per wave and tile, row tm * WM + wm (plan_v3's row count)
  constexpr int NI = WTR / 16;
  constexpr bool PW = WTR % 32 != 0;
  constexpr int NQ = PW ? 1 : NI / 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long M = (long)g.N * g.OH * g.OW;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  constexpr int RS = BN + 8;
  const bool half = g.K <= 64;
  const long nprow = half ? 2 * ((M + 63) / 64) : 2 * ((M + 127) / 128);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = wn * 64 + j * 16 + (lane & 15);
    const float bv = (bias != nullptr && n0 + c < g.K) ? bias[n0 + c] : 0.f;
    float s1[NQ], s2[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) s1[q] = s2[q] = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTR + i * 16 + 4 * (lane >> 4) + r;
        const float v = acc[i][j][r] + bv;
        ct[row * RS + c] = __float2bfloat16(v);
        if (m0 + row < M) {
          s1[PW ? 0 : i >> 1] += v;
          s2[PW ? 0 : i >> 1] += v * v;
        }
      }
    if (psum != nullptr) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        s1[q] += __shfl_xor(s1[q], 16, 64);
        s1[q] += __shfl_xor(s1[q], 32, 64);
        s2[q] += __shfl_xor(s2[q], 16, 64);
        s2[q] += __shfl_xor(s2[q], 32, 64);
      }
      const int n = n0 + c;
      if constexpr (PW) {
        if (lane < 16 && n < g.K) {
          const long wr = (long)tm * C3_::WM + wm;
          psum[wr * g.K + n] = s1[0];
          psq[wr * g.K + n] = s2[0];
        }
      } else if (lane < 16 && n < g.K) {
        const long b32 = (long)tm * (BM / 32) + wm * (WTR / 32);  // first 32-row block of this wave
        if (half) {
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            if (b32 + q < nprow) {
              psum[(b32 + q) * g.K + n] = s1[q];
              psq[(b32 + q) * g.K + n] = s2[q];
            }
        } else {
#pragma unroll
          for (int q = 0; q < NQ; q += 2) {
            const long wr = (b32 + q) / 2;  // 64-row block index
            if (wr < nprow) {
              psum[wr * g.K + n] = s1[q] + s1[q + 1];
              psq[wr * g.K + n] = s2[q] + s2[q + 1];
            }
          }
        }
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int e = threadIdx.x; e < BM * CPR; e += C3_::NTH) {
    const int row = e / CPR, cv = e % CPR;
    const long m = m0 + row;
    const int n = n0 + cv * 8;
    if (m >= M || n >= g.K) continue;
    uint4 v = *reinterpret_cast<const uint4*>(ct + row * RS + cv * 8);
    long pix = m;
    if (BUF == 3) {  // class row (b, i2, j2) -> dx pixel (b, 2 i2 + a, 2 j2 + b)
      const int j2 = (int)(m % g.OW);
      const long t = m / g.OW;
      const int i2 = (int)(t % g.OH), bb = (int)(t / g.OH);
      pix = ((long)bb * cls.HX + 2 * i2 + cls.a) * cls.WX + 2 * j2 + cls.b;
    }
    int nc = n;  // the output channel of column n
    if (BUF == 4 || BUF == 5) {  // 2 x 2 class GEMM (conv_dgrad_q2): row (b, i, j) -> dx pixel (2 i + a, 2 j + b) of
      // column cls * 64 + c (BUF 4), of column b * 128 + c at the tile's row class cls.a (BUF 5)
      const int j = (int)(m % g.OW);
      const long t = m / g.OW;
      const int i = (int)(t % g.OH), bb = (int)(t / g.OH);
      const int ca = BUF == 4 ? n / (BN / 2) : cls.a, cb = BUF == 4 ? (n / (BN / 4)) & 1 : n >> 7;
      if (2 * i + ca >= cls.HX || 2 * j + cb >= cls.WX) continue;
      pix = ((long)bb * cls.HX + 2 * i + ca) * cls.WX + 2 * j + cb;
      nc = BUF == 4 ? n % (BN / 4) : n & 127;
    }
    uint4* dst = reinterpret_cast<uint4*>(y + pix * g.yps + nc);
    if (!DG && ep.on) {
      epi_store<bf16, 8>(ep, ct + row * RS + cv * 8, y + pix * g.yps + n, n, g.K, pix, true);
      continue;
    }
    if (accumulate) {
      float a[8], b[8];
      unpack<bf16>(v, a);
      unpack<bf16>(*dst, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
      v = pack<bf16>(a);
    }
    *dst = v;
  }
}

// Persistent 1x1 GEMM with a register epilogue (stride-1 1x1 forward / data-grad, DMY_P1P).  The 1x1 layers are
// HBM-bound with 1..8 K steps per tile; on the one-tile blocks above every tile pays its load prologue and an
// LDS-staged epilogue (tile -> LDS -> barrier -> stores) with nothing else in flight, and they stream at 2.5-3.5 TB/s
// in the training step.  Here each block walks tiles t = b, b + G, ... (XCD-contiguous order) through ONE LDS-DMA
// ring that runs ahead across tile boundaries, and the epilogue never touches the ring: the MFMA runs transposed
// (D[channel][pixel] = W X^T, so a lane ends with 4 consecutive channels of one pixel), a permlane16 swap pairs two
// 16-channel tiles into 8 consecutive channels = one 16-B buffer store straight from registers, and the BN partials
// are reduced over the 16 pixel lanes with DPP and transposed through a 512-B per-wave LDS scratch.  Every memory
// operation of the epilogue is an unconditional buffer instruction (masked rows / columns get an out-of-range
// offset), so the counted vmcnt waits of the next tile's first steps know exactly how many stores are younger than
// the stage they wait for, and the stores drain under the next tile's MFMAs.
DEV float row_sum16(float v) {  // lane 15 of each 16-lane row ends with the row's total
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  return v;
}
DEV unsigned pk2_bf16(float a, float b) {
  const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (unsigned)*reinterpret_cast<const unsigned short*>(&x) |
         ((unsigned)*reinterpret_cast<const unsigned short*>(&y) << 16);
}

template <int BM, int BN, int NS, int WTR>
struct P1P {
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  static constexpr int NW = C3_::NW, NTH = C3_::NTH, PER = C3_::APW + C3_::BPW;
  static constexpr int NI = WTR / 16;      // 16-pixel blocks per wave
  static constexpr int NST = NI * 2;       // 16-B output stores per lane per tile (two 32-channel halves per block)
  static constexpr int LDS = NS * C3_::STAGE + NW * 512;
};

// LANE (forward, one column tile): the BN partials are NOT written per 32/64-pixel group; each lane keeps running Σz /
// Σz² of its 4 channels x its pixel lane over ALL tiles of the block (fp32, ~NI x tiles-per-wave terms), and each wave
// row writes ONE partial row at the end (row blockIdx.x * WM + wave row, its WN waves writing their 64-channel slices;
// dmy_conv_fwd_bn_rows reports G * WM rows).  For the
// <= 64-column layers the per-32-pixel rows cost 12.5 % extra write bytes plus their per-tile DPP reductions
// (64 -> 64 @384^2 bs32: 349 us with them vs 233 us without, round 4, gpurun_out r4/micro2_p1s.log).
template <int BM, int BN, int NS, int WTR, bool DG, bool LANE = false>
__global__ void __launch_bounds__((BM / WTR) * (BN / 64) * 64) conv_p1p(
    const bf16* __restrict__ x, const bf16* __restrict__ w, const float* __restrict__ bias, bf16* __restrict__ y,
    float* __restrict__ psum, float* __restrict__ psq, int /*accumulate: 0*/, Geom g, int gm, int gn, unsigned xbytes,
    unsigned wbytes, unsigned ybytes, int nprow, Epi ep, unsigned rbytes) {
  using PP = P1P<BM, BN, NS, WTR>;
  using C3_ = typename PP::C3_;
  constexpr int PER = PP::PER, NI = PP::NI;
  // epilogue VMEM instructions per lane (all unconditional): NST stores (+ NST loads when accumulating), and with BN
  // partials 2 stores per partial row the wave covers
  static_assert(NS == 2 || NS == 3, "ring depth");
  __shared__ __attribute__((aligned(1024))) char smem[PP::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  const int q = lane >> 4, pl = lane & 15;
  float* red = reinterpret_cast<float*>(smem + NS * C3_::STAGE) + wid * 128;
  const long M = (long)g.N * g.OH * g.OW;
  const int ntiles = gm * gn, nk = g.C / BK, G = gridDim.x;
  if ((int)blockIdx.x >= ntiles) return;
  const bool half = g.K <= 64;
  const int PR = half ? 32 : 64;                 // pixels per BN partial row (dmy_conv_fwd_partial_rows)
  const int ngrp = (psum != nullptr && !LANE) ? WTR / PR : 0;
  float ls1[4][4], ls2[4][4];  // LANE: this lane's running sums over the block's tiles, [16-channel group][4 channels]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) ls1[j][rr] = ls2[j][rr] = 0.f;
  // this wave's epilogue VMEM ops per tile (no accumulate: the host routes it away; the inference epilogue's residual
  // adds one 16-B load per store)
  const int nepi = PP::NST * (ep.on && ep.res != nullptr ? 2 : 1) + 2 * ngrp;
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(ep.res, ep.res != nullptr ? rbytes : 0u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, ybytes);
  const __amdgpu_buffer_rsrc_t rps = make_rsrc(psum, psum != nullptr ? (unsigned)((long)nprow * g.K * 4) : 0u);
  const __amdgpu_buffer_rsrc_t rpq = make_rsrc(psq, psq != nullptr ? (unsigned)((long)nprow * g.K * 4) : 0u);
  if (!LANE && psum != nullptr && BM < 2 * PR && blockIdx.x == 0) {
    // dmy_conv_fwd_partial_rows rounds the partial rows up to an even count; with 64-row tiles the last one can lie
    // past every tile: it holds no pixels and must still read as zero (plain stores, older than any stage load)
    for (long pr = (long)gm * BM / PR + threadIdx.x / 64; pr < nprow; pr += PP::NW)
      for (int c = lane; c < g.K; c += 64) {
        psum[pr * g.K + c] = 0.f;
        psq[pr * g.K + c] = 0.f;
      }
  }
  using LD = FwdLdsB<BM, BN, NS, true, DG, false, 2, WTR>;
  auto tile_of = [&](int L) { return xcd_remap(L, ntiles); };
  // issue cursor: (round, k step) of the next stage to load
  int lr = 0, lk = 0;
  int lt = tile_of(blockIdx.x);
  LD ld(x, w, g, M, (long)(lt / gn) * BM, (lt % gn) * BN, wid, lane, xbytes, wbytes);
  const int my_tiles = (ntiles - 1 - (int)blockIdx.x) / G + 1, total = my_tiles * nk;
  auto issue = [&](int st) {
    ld.issue(smem + (st % NS) * C3_::STAGE, wid);
    if (++lk == nk) {
      lk = 0;
      ++lr;
      const int L = lr * G + (int)blockIdx.x;
      if (L < ntiles) {
        lt = tile_of(L);
        ld = LD(x, w, g, M, (long)(lt / gn) * BM, (lt % gn) * BN, wid, lane, xbytes, wbytes);
      }
    }
  };
  issue(0);
  if (NS == 3 && total > 1) issue(1);
  int s = 0;
  for (int r = 0; r < my_tiles; ++r) {
    const int t = tile_of(r * G + (int)blockIdx.x);
    const int tm = t / gn, tn = t % gn;
    const long m0 = (long)tm * BM;
    const int n0 = tn * BN;
    f32x4 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt, ++s) {
      // stage s landed: younger VMEM ops allowed in flight = the next stage (NS = 3, if issued) + the previous tile's
      // epilogue when it was issued after stage s (kt < NS - 1 on every tile but the block's first)
      const bool nxt = NS == 3 && s + 1 < total;
      const bool epi = r > 0 && kt < NS - 1;
      if (!epi) {
        if (nxt) vm_wait<PER>();
        else vm_wait<0>();
      } else if (nepi == PP::NST) {
        if (nxt) vm_wait<PER + PP::NST>();
        else vm_wait<PP::NST>();
      } else if (nepi == PP::NST + 2 * (WTR / 64)) {
        if (nxt) vm_wait<PER + PP::NST + 2 * (WTR / 64)>();
        else vm_wait<PP::NST + 2 * (WTR / 64)>();
      } else if (nepi == PP::NST + 2 * (WTR / 32)) {
        if (nxt) vm_wait<PER + PP::NST + 2 * (WTR / 32)>();
        else vm_wait<PP::NST + 2 * (WTR / 32)>();
      } else if (nepi == 2 * PP::NST) {
        if (nxt) vm_wait<PER + 2 * PP::NST>();
        else vm_wait<2 * PP::NST>();
      } else {
        vm_wait<0>();  // other epilogue shapes (accumulate, 32-pixel partial rows): wait for everything
      }
      __builtin_amdgcn_s_barrier();
      if (s + NS - 1 < total) issue(s + NS - 1);
      const bf16* As = reinterpret_cast<const bf16*>(smem + (s % NS) * C3_::STAGE);
      const bf16* Bs = As + BM * BK;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 a[NI], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag_sw(Bs, wn * 64 + j * 16, h * 32, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) a[i] = frag_sw(As, wm * WTR + i * 16, h * 32, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
    }
    // ---- register epilogue: acc[i][j][r] = Y[pixel m0 + wm WTR + 16 i + pl][channel n0 + wn 64 + 16 j + 4 q + r]
    const long mw = m0 + wm * WTR;
    const int nw = n0 + wn * 64;
    if (bias != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int n = nw + 16 * j + 4 * q + rr;
          const float bv = n < g.K ? bias[n] : 0.f;
#pragma unroll
          for (int i = 0; i < NI; ++i) acc[i][j][rr] += bv;
        }
    }
    if (LANE && psum != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const float v = mw + 16 * i + pl < M ? acc[i][j][rr] : 0.f;
            ls1[j][rr] += v;
            ls2[j][rr] += v * v;
          }
    } else if (psum != nullptr) {
      for (int gi = 0; gi < ngrp; ++gi) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
              if (i * 16 / PR != gi) continue;
              const float v = mw + 16 * i + pl < M ? acc[i][j][rr] : 0.f;
              s1 += v;
              s2 += v * v;
            }
            s1 = row_sum16(s1);
            s2 = row_sum16(s2);
            if (pl == 15) {
              red[16 * j + 4 * q + rr] = s1;
              red[64 + 16 * j + 4 * q + rr] = s2;
            }
          }
        __builtin_amdgcn_wave_barrier();
        const float v1 = red[lane], v2 = red[64 + lane];
        __builtin_amdgcn_wave_barrier();
        const long prow = (mw + gi * PR) / PR;
        const bool ok = prow < nprow && nw + lane < g.K;
        const unsigned off = ok ? (unsigned)((prow * g.K + nw + lane) * 4) : kBufOob;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v1), rps, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v2), rpq, off, 0, 0);
      }
    }
    const int chq = (q & 1) * 16 + (q >> 1) * 8;
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const f32x4 &a = acc[i][2 * jp], &b = acc[i][2 * jp + 1];
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk2_bf16(a[0], a[1]), pk2_bf16(b[0], b[1]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk2_bf16(a[2], a[3]), pk2_bf16(b[2], b[3]), false, false);
        u4 v = {s0[0], s1[0], s0[1], s1[1]};
        const long m = mw + 16 * i + pl;
        const int n = nw + 32 * jp + chq;
        if (ep.on) {  // eval BN scale / shift + act (+ residual) on the bf16-rounded conv output, as epi_store
          u4 rv = {0u, 0u, 0u, 0u};
          if (ep.res != nullptr)
            rv = __builtin_amdgcn_raw_buffer_load_b128(rr, (m < M && n < g.K) ? (unsigned)((m * ep.rps + n) * 2) : kBufOob, 0, 0);
          float f[8], r8[8], sc[8], sh[8];
          unpack<bf16>(make_uint4(v[0], v[1], v[2], v[3]), f);
          unpack<bf16>(make_uint4(rv[0], rv[1], rv[2], rv[3]), r8);
          epi_coef8(ep, n < g.K ? n : 0, sc, sh);  // K % 8 == 0 here: a live vector has all 8 channels
          epi_apply8(ep.act, f, sc, sh, ep.res != nullptr ? r8 : nullptr);
          const uint4 o = pack<bf16>(f);
          v = u4{o.x, o.y, o.z, o.w};
        }
        const unsigned off = (m < M && n < g.K) ? (unsigned)((m * g.yps + n) * 2) : kBufOob;
        __builtin_amdgcn_raw_buffer_store_b128(v, ry, off, 0, 0);
      }
  }
  if (LANE && psum != nullptr) {  // one partial row per wave row: reduce the 16 pixel lanes, transpose through LDS
    const long prow = (long)blockIdx.x * C3_::WM + wm;  // the WN waves of wave row wm write its 64-channel slices
    const int nw = wn * 64;  // one column tile (gn == 1): n0 = 0
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float s1 = row_sum16(ls1[j][rr]), s2 = row_sum16(ls2[j][rr]);
        if (pl == 15) {
          red[16 * j + 4 * q + rr] = s1;
          red[64 + 16 * j + 4 * q + rr] = s2;
        }
      }
    __builtin_amdgcn_wave_barrier();
    const float v1 = red[lane], v2 = red[64 + lane];
    const bool ok = prow < nprow && nw + lane < g.K;
    const unsigned off = ok ? (unsigned)((prow * g.K + nw + lane) * 4) : kBufOob;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v1), rps, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v2), rpq, off, 0, 0);
  }
}

// Forward (DG = false) or stride-1 data-grad (DG = true; `g` is the GEMM view built by the host:
// rows = input pixels, columns = input channels, gather = dy) with the BN-partial / accumulate epilogue.
template <int BM, int BN, int NS, bool P1, bool DG, int BUF>
__global__ void __launch_bounds__(BM * BN / 64) conv_fwd_v3(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                            const float* __restrict__ bias, bf16* __restrict__ y,
                                                            float* __restrict__ psum, float* __restrict__ psq,
                                                            int accumulate, Geom g, int gm, int gn, unsigned xbytes,
                                                            unsigned wbytes, S2Cls cls, Epi ep) {
  using C3_ = Cfg3<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // BUF: 0 = FwdLds, 1 = buffer loader, 3 = buffer loader, stride-2 data-grad parity class `cls` (only the class's
  // taps: ceil((KH - kh0) / 2) x ceil((KW - kw0) / 2))
  const int nk = BUF == 3 ? ((g.KH - ((cls.a + g.P) & 1) + 1) / 2) * ((g.KW - ((cls.b + g.P) & 1) + 1) / 2) * (g.C / BK)
                          : (g.KH * g.KW * g.C + BK - 1) / BK;
  if constexpr (BUF == 3) {
    FwdLdsB<BM, BN, NS, false, true, true> ld(x, w, g, M, m0, n0, wid, lane, xbytes, wbytes, cls);
    mainloop4<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  } else if constexpr (BUF > 0) {
    FwdLdsB<BM, BN, NS, P1, DG> ld(x, w, g, M, m0, n0, wid, lane, xbytes, wbytes);
    mainloop4<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  } else {
    FwdLds<BM, BN, NS, P1, DG> ld(x, w, g, M, m0, n0, wid, lane);
    mainloop3<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  }
  __syncthreads();
  v3_epilogue<BM, BN, NS, DG, BUF>(acc, reinterpret_cast<bf16*>(smem), bias, y, psum, psq, accumulate, g, tm, m0, n0,
                                    cls, ep);
}

// All four output-parity classes of a stride-2 data-grad in ONE launch. Block u (XCD-contiguous order, xcd_remap) takes
// class u % 4 and tile u / 4, so the four classes' tiles over the same dy rows run together on one XCD and share its
// L2 (as four launches every class re-read dy: PMC traffic 1.35x the algorithmic bytes of the data-grad family), and
// the short 1-tap class-(0,0) tiles fill in behind the 4-tap ones instead of each launch draining separately.
// g = the layer's forward geometry; per class the GEMM view is the one launch_dgrad_s2_v3 builds on the host.
template <int BM, int BN, int NS>
__global__ void __launch_bounds__(BM * BN / 64) conv_dgrad_s2_v3(const bf16* __restrict__ dy, const bf16* __restrict__ wt,
                                                                 bf16* __restrict__ dx, int accumulate, Geom g, int gmax,
                                                                 int gn, unsigned xbytes, unsigned wbytes) {
  using C3_ = Cfg3<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int u = xcd_remap(blockIdx.x, 4 * gmax * gn);
  const int a = (u >> 1) & 1, b = u & 1, t = u >> 2, tm = t / gn, tn = t % gn;
  Geom gv = g;  // GEMM view of class (a, b): gather dy (OH x OW x K, stride yps), rows = the class's input pixels
  gv.H = g.OH; gv.W = g.OW; gv.C = g.K; gv.xps = g.yps; gv.K = g.C; gv.S = 2;
  gv.OH = (g.H - a + 1) / 2; gv.OW = (g.W - b + 1) / 2; gv.yps = g.xps;
  const long M = (long)gv.N * gv.OH * gv.OW;
  const long m0 = (long)tm * BM;
  if (gv.OH <= 0 || gv.OW <= 0 || m0 >= M) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = tn * BN;
  const S2Cls cls{a, b, g.H, g.W};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = ((gv.KH - ((a + gv.P) & 1) + 1) / 2) * ((gv.KW - ((b + gv.P) & 1) + 1) / 2) * (gv.C / BK);
  FwdLdsB<BM, BN, NS, false, true, true> ld(dy, wt, gv, M, m0, n0, wid, lane, xbytes, wbytes, cls);
  mainloop4<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  __syncthreads();
  v3_epilogue<BM, BN, NS, true, 3>(acc, reinterpret_cast<bf16*>(smem), nullptr, dx, nullptr, nullptr, accumulate, gv, tm,
                                    m0, n0, cls, Epi{});
}

// ---------------------------------------------------------------- wide tile: 256 x 256 block, 128 x 64 per wave
// Per K step a wave reads (128 + 64) x 64 bf16 from LDS for 64 MFMAs, against (64 + 64) x 64 for 32 in the
// 64 x 64 wave tile: the LDS array (256 B/clk/CU) stops pacing the MFMAs on the MFMA-bound layers.  2 LDS stages
// of 64 KiB (loads of step k + 1 in flight during step k), 8 waves (2 x 4), 128 accumulator registers per lane.
// Fragments first: the first half-step's 12 fragment reads are issued before the next stage's LDS-DMA, so the reads
// the MFMAs wait on are not queued behind the DMA's LDS writes.  Measured against DMA first (round 4,
// profiles/r04/wide_ff_ab.log, cold caches): 3x3 256 @96^2 fwd 430 -> 418 us, 512 @96^2 fwd 1201 -> 1171, dgrad 1156 ->
// 1114, 1024 @48^2 fwd 1254 -> 1211; DMA-1536 step 153.8 / 153.6 -> 154.8 / 154.4 img/s
template <int BM, int BN, int NS, int WTR, class LD>
DEV void mainloop_w(LD& ld, int nk, char* smem, f32x4 (&acc)[WTR / 16][4], int wid, int lane) {
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  constexpr int NI = WTR / 16;
  constexpr int PER = C3_::APW + C3_::BPW;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  ld.issue(smem, wid);
  if (NS == 3 && nk > 1) ld.issue(smem + C3_::STAGE, wid);
  for (int kt = 0; kt < nk; ++kt) {
    if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * C3_::STAGE);
    const bf16* Bs = As + BM * BK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 a[NI], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag_sw(Bs, wn * 64 + j * 16, h * 32, lane);
#pragma unroll
      for (int i = 0; i < NI; ++i) a[i] = frag_sw(As, wm * WTR + i * 16, h * 32, lane);
      if (h == 0) {
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * C3_::STAGE, wid);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
}

// BM x BN = 256 x 256 (2 x 4 waves of 128 x 64), 288 x 256 (2 x 4 waves of 144 x 64: the row count whose tile grid
// fills whole rounds of the chip on the DMA-YOLO / config-5 maps, see plan_v3) or 512 x 128 (4 x 2 waves, the
// 128-column layers; 2 x 80 KiB of LDS)
template <int BM, int BN, bool P1, bool DG>
__global__ void __launch_bounds__(512) conv_fwd_w(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                  const float* __restrict__ bias, bf16* __restrict__ y,
                                                  float* __restrict__ psum, float* __restrict__ psq, int accumulate,
                                                  Geom g, int gm, int gn, unsigned xbytes, unsigned wbytes, Epi ep) {
  constexpr int NS = 2, WN = BN / 64, WM = 8 / WN, WTR = BM / WM;
  static_assert(WM * WN == 8 && WTR % 16 == 0, "8 waves of WTR x 64");
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  f32x4 acc[WTR / 16][4];
#pragma unroll
  for (int i = 0; i < WTR / 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (g.KH * g.KW * g.C + BK - 1) / BK;
  FwdLdsB<BM, BN, NS, P1, DG, false, 2, WTR> ld(x, w, g, M, m0, n0, wid, lane, xbytes, wbytes);
  mainloop_w<BM, BN, NS, WTR>(ld, nk, smem, acc, wid, lane);
  __syncthreads();
  v3_epilogue<BM, BN, NS, DG, 1, WTR>(acc, reinterpret_cast<bf16*>(smem), bias, y, psum, psq, accumulate, g, tm, m0,
                                      n0, S2Cls{0, 0, 0, 0}, ep);
}

// ---------------------------------------------------------------- stride-2 data-grad classes on the wide / tall tiles
// One parity class (a, b) of a stride-2 data-grad (FwdLdsB S2 mode: the class's input pixels as rows, only the taps of
// matching parity) on conv_fwd_w's 128 x 64 wave tiles, 256 x 256 blocks, for >= 256 input channels -- the tile the
// stride-1 views of the same widths take (the 256 x 128 / 64 x 64-wave class tiles read (64 + 64) x 64 of LDS per 32
// MFMAs, these (128 + 64) x 64 per 64).
template <int BM, int BN>
__global__ void __launch_bounds__(512) conv_dgrad_s2_w(const bf16* __restrict__ dy, const bf16* __restrict__ wt,
                                                     bf16* __restrict__ dx, int accumulate, Geom gv, int gm, int gn,
                                                     unsigned xbytes, unsigned wbytes, S2Cls cls) {
  constexpr int NS = 2, WN = BN / 64, WM = 8 / WN, WTR = BM / WM;
  static_assert(WM * WN == 8 && WTR % 16 == 0, "8 waves of WTR x 64");
  using C3_ = Cfg3<BM, BN, NS, WTR>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)gv.N * gv.OH * gv.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  f32x4 acc[WTR / 16][4];
#pragma unroll
  for (int i = 0; i < WTR / 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = ((gv.KH - ((cls.a + gv.P) & 1) + 1) / 2) * ((gv.KW - ((cls.b + gv.P) & 1) + 1) / 2) * (gv.C / BK);
  FwdLdsB<BM, BN, NS, false, true, true, 2, WTR> ld(dy, wt, gv, M, m0, n0, wid, lane, xbytes, wbytes, cls);
  mainloop_w<BM, BN, NS, WTR>(ld, nk, smem, acc, wid, lane);
  __syncthreads();
  v3_epilogue<BM, BN, NS, true, 3, WTR>(acc, reinterpret_cast<bf16*>(smem), nullptr, dx, nullptr, nullptr, accumulate,
                                        gv, tm, m0, n0, cls, Epi{});
}

// ---------------------------------------------------------------- stride-2 data-grad of a 32 / 64 / 128-channel layer, one GEMM
// dx of a 3x3 stride-2 pad-1 conv at the four output parities (a, b) of the 2 x 2 block (2i .. 2i + 1, 2j .. 2j + 1)
// reads only dy[i .. i + 1][j .. j + 1] (class a = 0: tap kh = 1 from row i; a = 1: kh = 2 from row i, kh = 0 from row
// i + 1; the same for columns).  So the whole data-grad is ONE GEMM over dy pixels: rows (b, i, j), K = the 2 x 2 dy
// window x C_out (a stride-1 2 x 2 gather, zeros past the edge), columns = 4 classes x 64 input channels = 256 -- one
// 256 x 256 wide tile (conv_fwd_w's loop and epilogue) -- with the B operand gathered from the IHWO weights:
// B[cls * 64 + c][(dh, dw, co)] = W[c][a + 1 - 2 dh][b + 1 - 2 dw][co], zero where that tap does not exist.  It spends
// 16 / 9 of the useful MFMA work on those zeros, against the four class GEMMs' 2..8-step K loops over 256 x 64 tiles:
// 64 <- 128 @768^2 bs32 1936 -> 1711..1729 us, 64 <- 128 @160^2 bs64 170 -> 164 us (profiles/r06/q2_ab.log, cold caches).
// CI = 128 (128 input channels): 4 classes x 128 = 512 columns do not fit one tile, so a tile holds ONE row class a
// (columns = b x 128 + c) and walks only the dy rows that class reads: a = 0 the 1 x 2 window (K = 2 C_out, class
// (0, 0) wastes half), a = 1 the 2 x 2 window (class (1, 0) wastes half) -- 12 / 9 of the useful work, not 16 / 9.
// (The same split for 64 channels on 256 x 128 tiles measured slower at 768^2 / 960^2: profiles/r06/q2r_ab.log.)
// CI = 32: all four classes x 32 channels = 128 columns on 256 x 128 tiles (conv_fwd_v3's 3-stage loop, conv_dgrad_q2s).
template <int CI, int BN = 256>
struct LdsQ2 {
  static constexpr bool ALL = 4 * CI == BN;  // all four classes in one tile, else one row class a per tile
  static_assert((BN == 256 && (CI == 64 || CI == 128)) || (BN == 128 && CI == 32), "4 x 64 | 2 x 128 | 4 x 32 columns");
  using C3_ = Cfg3<256, BN, BN == 256 ? 2 : 3, BN == 256 ? 128 : 64>;
  __amdgpu_buffer_rsrc_t rx, rw;
  int H, W, xps, Cout;
  int dh, dw, ci0;  // uniform cursor: dy window tap, channel base
  int kl;
  int pix[C3_::APW], i0[C3_::APW], j0[C3_::APW];
  bool aval[C3_::APW];
  int wrow[C3_::BPW], ra[C3_::BPW], rb[C3_::BPW];  // B row: weight row base (c * 9 * Cout), the row's class (a, b)
  DEV LdsQ2(const bf16* dy, const bf16* wt, const Geom& g, long M, long m0, int wid, int lane, unsigned xbytes,
            unsigned wbytes, int a)
      : H(g.H), W(g.W), xps((int)g.xps), Cout(g.C), dh(0), dw(0), ci0(0) {
    rx = make_rsrc(dy, xbytes);
    rw = make_rsrc(wt, wbytes);
    kl = ((lane & 7) ^ ((lane >> 3) & 6)) * 8;
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const long m = m0 + (wid * C3_::APW + j) * 8 + (lane >> 3);
      aval[j] = m < M;
      const int mm = (int)(aval[j] ? m : 0);
      const int ow = mm % g.OW, t = mm / g.OW, oh = t % g.OH, b = t / g.OH;
      i0[j] = oh;
      j0[j] = ow;
      pix[j] = ((b * g.H + oh) * g.W + ow) * xps;
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j) {
      const int n = (wid * C3_::BPW + j) * 8 + (lane >> 3);
      wrow[j] = (n % CI) * 9 * Cout;
      ra[j] = ALL ? n / (2 * CI) : a;
      rb[j] = (n / CI) & 1;
    }
  }
  DEV void issue(char* stage, int wid) {
    const int delta = (dh * W + dw) * xps + ci0 + kl;
#pragma unroll
    for (int j = 0; j < C3_::APW; ++j) {
      const bool ok = aval[j] && i0[j] + dh < H && j0[j] + dw < W;
      blds16(rx, ok ? (unsigned)(pix[j] + delta) * 2u : kBufOob, stage + (wid * C3_::APW + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < C3_::BPW; ++j) {
      const int kh = ra[j] + 1 - 2 * dh, kw = rb[j] + 1 - 2 * dw;
      const bool ok = (unsigned)kh < 3u && (unsigned)kw < 3u;
      blds16(rw, ok ? (unsigned)(wrow[j] + (kh * 3 + kw) * Cout + ci0 + kl) * 2u : kBufOob,
             stage + C3_::A_BYTES + (wid * C3_::BPW + j) * 1024);
    }
    ci0 += BK;
    if (ci0 == Cout) {
      ci0 = 0;
      if (++dw == 2) { dw = 0; ++dh; }
    }
  }
};

// gq = the GEMM view: (H, W, C, xps) = dy, (OH, OW) = dy's map (rows), K = 256, yps = dx's pixel stride; cls carries
// dx's (HX, WX).  CI = 128: 2 gm blocks, the a = 1 tiles (twice the K loop) first
template <int CI>
__global__ void __launch_bounds__(512) conv_dgrad_q2(const bf16* __restrict__ dy, const bf16* __restrict__ wt,
                                                   bf16* __restrict__ dx, int accumulate, Geom gq, int gm,
                                                   unsigned xbytes, unsigned wbytes, S2Cls cls) {
  constexpr int NS = 2, WTR = 128;
  using C3_ = Cfg3<256, 256, NS, WTR>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int half = CI == 128 && (int)blockIdx.x >= gm;
  const int tm = xcd_remap((int)blockIdx.x - half * gm, gm);
  cls.a = CI == 128 ? 1 - half : 0;
  const long M = (long)gq.N * gq.OH * gq.OW;
  const long m0 = (long)tm * 256;
  f32x4 acc[WTR / 16][4];
#pragma unroll
  for (int i = 0; i < WTR / 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (CI == 64 || cls.a ? 4 : 2) * gq.C / BK;
  LdsQ2<CI> ld(dy, wt, gq, M, m0, wid, lane, xbytes, wbytes, cls.a);
  mainloop_w<256, 256, NS, WTR>(ld, nk, smem, acc, wid, lane);
  __syncthreads();
  v3_epilogue<256, 256, NS, true, CI == 64 ? 4 : 5, WTR>(acc, reinterpret_cast<bf16*>(smem), nullptr, dx, nullptr, nullptr,
                                          accumulate, gq, tm, m0, 0, cls, Epi{});
}

// CI = 32: the four classes x 32 channels = 128 columns, one 256 x 128 tile per 256 dy pixels (16 / 9 of the work)
__global__ void __launch_bounds__(512) conv_dgrad_q2s(const bf16* __restrict__ dy, const bf16* __restrict__ wt,
                                                    bf16* __restrict__ dx, int accumulate, Geom gq, int gm,
                                                    unsigned xbytes, unsigned wbytes, S2Cls cls) {
  constexpr int BM = 256, BN = 128, NS = 3;
  using C3_ = Cfg3<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tm = xcd_remap((int)blockIdx.x, gm);
  const long M = (long)gq.N * gq.OH * gq.OW;
  const long m0 = (long)tm * BM;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = 4 * gq.C / BK;
  LdsQ2<32, BN> ld(dy, wt, gq, M, m0, wid, lane, xbytes, wbytes, 0);
  mainloop4<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  __syncthreads();
  v3_epilogue<BM, BN, NS, true, 4>(acc, reinterpret_cast<bf16*>(smem), nullptr, dx, nullptr, nullptr, accumulate, gq, tm,
                                   m0, 0, cls, Epi{});
}

// ---------------------------------------------------------------- 256 x 256 half-tile pipeline (conv_fwd_8p, round 5)
// The wide tile above stages whole 64 KiB K steps in a 2-stage ring and drains the DMA queue (vmcnt(0)) before every
// barrier, so each step's loads have one step of MFMA time to land and the 8 waves run in lockstep: all read LDS, then
// all issue MFMAs.  This kernel is cdna_hip_programming.md §5's 256² phase template applied to the implicit-GEMM
// loaders:
//   * the staging unit is a HALF tile (128 rows x 64 k = 16 KiB = 2 LDS-DMA instructions per wave); A half-tiles are
//     triple-buffered and B half-tiles double-buffered (10 x 16 KiB = the whole 160 KiB of LDS);
//   * a K step is 4 phases; in each a wave reads one register subtile (p0: A rows 0-63 + B cols 0-31, p1: B cols
//     32-63, p2: A rows 64-127, p3: nothing -- every fragment it needs is still in registers), issues ONE half-tile of
//     a later K step (p0: B1(u+1), p1: A0(u+2), p2: A1(u+2), p3: B0(u+2)), barriers, and runs 16 MFMAs of one quadrant
//     of its 128 x 64 tile; the counted vmcnt(6) at p3 leaves 3 half-tiles in flight, never 0 inside the loop;
//   * the two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one barrier apart, so on every SIMD one wave's
//     LDS reads and DMA issue overlap the other wave's MFMAs.
// The RAW / WAR safety of exactly this schedule (every slot restaged >= 2 phases after its last read; every read one
// barrier after all waves' retiring vmcnt) is checked formally by tools/sched8p_check.py.  Same GEMM views, loaders'
// address arithmetic (FwdLdsB) and epilogue (v3_epilogue, 128 x 64 wave tiles) as conv_fwd_w.
namespace p8 {
constexpr int HALF = 16384;
constexpr int NA = 3, NB = 2;
constexpr int LDS = (2 * NA + 2 * NB) * HALF;  // 160 KiB
DEV char* slot_a(char* s, int h, int t) { return s + ((t % NA) * 2 + h) * HALF; }
DEV char* slot_b(char* s, int h, int t) { return s + (2 * NA + (t % NB) * 2 + h) * HALF; }
}  // namespace p8

template <bool P1, bool DG>
struct Lds8 {
  __amdgpu_buffer_rsrc_t rx, rw;
  int H, W, C, KW, xps;
  int kh, kw, ci0, kpos;  // A stream cursor
  int kposb;              // B stream cursor
  int kl;
  int pix[4], ih0[4], iw0[4];
  bool aval[4];
  unsigned boff[4];
  // piece J (half J >> 1, instruction J & 1) of wave wid covers rows (J >> 1) * 128 + wid * 16 + (J & 1) * 8 + lane / 8
  DEV Lds8(const bf16* x, const bf16* w, const Geom& g, long M, long m0, int n0, int wid, int lane, unsigned xbytes,
           unsigned wbytes)
      : H(g.H), W(g.W), C(g.C), KW(g.KW), xps((int)g.xps), kh(0), kw(0), ci0(0), kpos(0), kposb(0) {
    rx = make_rsrc(x, xbytes);
    rw = make_rsrc(w, wbytes);
    const int Ktot = g.KH * g.KW * g.C;
    kl = ((lane & 7) ^ ((lane >> 3) & 6)) * 8;
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      const int r = (J >> 1) * 128 + wid * 16 + (J & 1) * 8 + (lane >> 3);
      const long m = m0 + r;
      aval[J] = m < M;
      const int mm = (int)(aval[J] ? m : 0);
      const int ow = mm % g.OW, t = mm / g.OW, oh = t % g.OH, b = t / g.OH;
      if (P1) {
        pix[J] = mm * xps;
        ih0[J] = iw0[J] = 0;
      } else {
        ih0[J] = DG ? oh + g.P : oh * g.S - g.P;
        iw0[J] = DG ? ow + g.P : ow * g.S - g.P;
        pix[J] = ((b * g.H + ih0[J]) * g.W + iw0[J]) * xps;  // may be negative; valid taps land >= 0
      }
      const int n = n0 + r;
      boff[J] = n < g.K ? (unsigned)(n * Ktot + kl) * 2u : kBufOob;
    }
  }
  // half h of the A stream's next K step into `dst`; the cursor advances after half 1
  DEV void issue_a(char* dst, int h, int wid) {
    const int dh = DG ? -kh : kh, dw = DG ? -kw : kw;
    const int delta = P1 ? kpos + kl : (dh * W + dw) * xps + ci0 + kl;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int J = h * 2 + j;
      bool ok = aval[J];
      if (!P1) ok = ok && (unsigned)(ih0[J] + dh) < (unsigned)H && (unsigned)(iw0[J] + dw) < (unsigned)W;
      blds16(rx, ok ? (unsigned)(pix[J] + delta) * 2u : kBufOob, dst + (wid * 2 + j) * 1024);
    }
    if (h == 1) {
      kpos += BK;
      if (!P1) {
        ci0 += BK;
        if (ci0 == C) {
          ci0 = 0;
          if (++kw == KW) {
            kw = 0;
            ++kh;
          }
        }
      }
    }
  }
  DEV void issue_b(char* dst, int h, int wid) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int J = h * 2 + j;
      blds16(rw, boff[J] == kBufOob ? kBufOob : boff[J] + (unsigned)kposb * 2u, dst + (wid * 2 + j) * 1024);
    }
    if (h == 1) kposb += BK;
  }
};

#define P8_BAR()                          \
  do {                                    \
    __builtin_amdgcn_sched_barrier(0);    \
    __builtin_amdgcn_s_barrier();         \
    __builtin_amdgcn_sched_barrier(0);    \
  } while (0)

template <bool P1, bool DG>
__global__ void __launch_bounds__(512) conv_fwd_8p(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                   const float* __restrict__ bias, bf16* __restrict__ y,
                                                   float* __restrict__ psum, float* __restrict__ psq, int accumulate,
                                                   Geom g, int gm, int gn, unsigned xbytes, unsigned wbytes, Epi ep) {
  constexpr int BM = 256, BN = 256;
  __shared__ __attribute__((aligned(1024))) char smem[p8::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = wid >> 2, wm = wid & 1, wn = wid >> 1;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (g.KH * g.KW * g.C + BK - 1) / BK;
  Lds8<P1, DG> ld(x, w, g, M, m0, n0, wid, lane, xbytes, wbytes);
  // prologue: K step 0 whole, step 1's A0, A1, B0 (each operand's halves in stream order)
  ld.issue_a(p8::slot_a(smem, 0, 0), 0, wid);
  ld.issue_a(p8::slot_a(smem, 1, 0), 1, wid);
  ld.issue_b(p8::slot_b(smem, 0, 0), 0, wid);
  ld.issue_b(p8::slot_b(smem, 1, 0), 1, wid);
  if (nk > 1) {
    ld.issue_a(p8::slot_a(smem, 0, 1), 0, wid);
    ld.issue_a(p8::slot_a(smem, 1, 1), 1, wid);
    ld.issue_b(p8::slot_b(smem, 0, 1), 0, wid);
    vm_wait<6>();
  } else {
    vm_wait<0>();
  }
  P8_BAR();
  if (grp) P8_BAR();  // group 1 runs one barrier behind group 0
  const int rb = (wn & 1) * 64;  // this wave's first column (row of the B half-tile)
  bf16x8 a[2][4], b0[2][2], b1[2][2];
  for (int u = 0; u < nk; ++u) {
    const bf16* As = reinterpret_cast<const bf16*>(p8::slot_a(smem, wm, u));
    const bf16* Bs = reinterpret_cast<const bf16*>(p8::slot_b(smem, wn >> 1, u));
    // ---- p0: A rows 0-63, B cols 0-31; stage B1(u+1)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[h][i] = frag_sw(As, i * 16, h * 32, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[h][j] = frag_sw(Bs, rb + j * 16, h * 32, lane);
    }
    if (u + 1 < nk) ld.issue_b(p8::slot_b(smem, 1, u + 1), 1, wid);
    P8_BAR();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b0[h][j], acc[i][j], 0, 0, 0);
    P8_BAR();
    // ---- p1: B cols 32-63; stage A0(u+2)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[h][j] = frag_sw(Bs, rb + 32 + j * 16, h * 32, lane);
    if (u + 2 < nk) ld.issue_a(p8::slot_a(smem, 0, u + 2), 0, wid);
    P8_BAR();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b1[h][j], acc[i][2 + j], 0, 0, 0);
    P8_BAR();
    // ---- p2: A rows 64-127; stage A1(u+2)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[h][i] = frag_sw(As, 64 + i * 16, h * 32, lane);
    if (u + 2 < nk) ld.issue_a(p8::slot_a(smem, 1, u + 2), 1, wid);
    P8_BAR();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b1[h][j], acc[4 + i][2 + j], 0, 0, 0);
    P8_BAR();
    // ---- p3: no reads; stage B0(u+2); step u+1 must have landed before the next p0 (3 halves stay in flight)
    if (u + 2 < nk) {
      ld.issue_b(p8::slot_b(smem, 0, u + 2), 0, wid);
      vm_wait<6>();
    } else if (u + 1 < nk) {
      vm_wait<0>();
    }
    P8_BAR();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b0[h][j], acc[4 + i][j], 0, 0, 0);
    P8_BAR();
  }
  if (!grp) P8_BAR();  // group 0 catches up with group 1's extra barrier
  __syncthreads();
  v3_epilogue<BM, BN, 2, DG, 1, 128>(acc, reinterpret_cast<bf16*>(smem), bias, y, psum, psq, accumulate, g, tm, m0, n0,
                                     S2Cls{0, 0, 0, 0}, ep);
}
#undef P8_BAR

// ---------------------------------------------------------------- 1x1 streaming GEMM (p1s)
// Y[m][n] = sum_k X[m][k] W[n][k] for the stride-1 1x1 layers with a short reduction (KD = 64 / 128 / 256). Those
// GEMMs are HBM-bound, and on the LDS-DMA tiles above they ran at 25-50 % of the HBM rate: one block per CU walks
// 1..4 K steps, so a tile's time is its load prologue plus the LDS-staged epilogue with little else in flight.
// Here a block stages its column group of W in LDS once (rows padded by 16 B: conflict-free fragment reads), then
// each wave streams 64-pixel tiles with no block barrier: the X fragments come from HBM straight into registers
// (16-B buffer loads, zeros past M), the MFMA runs transposed (D[ch][px] = W X^T) so a lane ends with 4 consecutive
// channels of one pixel, and a permlane16 swap pairs two 16-channel tiles into 8 consecutive channels = one 16-B
// store. BN partials (one row per 64 pixels, per 32 when the layer has <= 64 columns: dmy_conv_fwd_partial_rows)
// are reduced over the 16 pixel lanes with DPP row shifts. Every X element is read once per column group.
// G3: the same streaming GEMM over a 3x3 stride-1 pad-1 gather of a 16-channel input (the space-to-depth stem of every
// yolov5 / DMA-YOLO model as a k3 conv): K index = tap * 16 + channel, KD = 160 (144 + a zero tap), each
// 16-B fragment is 8 channels of one tap of one pixel, out-of-image taps read zeros through the buffer range check.
// DG: the launch is a data-grad (the GEMM is the same; the argument only names the call family in a profile, so
// tools/pmc_traffic.py can attribute its dispatches)
template <int KD, int NTH, bool G3 = false, bool DG = false>
__global__ void __launch_bounds__(NTH, 1) conv_p1s(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                const float* __restrict__ bias, bf16* __restrict__ y,
                                                float* __restrict__ psum, float* __restrict__ psq, int accumulate,
                                                long M, int NC, int ng, long xps, long yps, unsigned xbytes,
                                                int ntiles, int kwrow, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) char p1s_smem[];
  constexpr int PITCH = KD + 8, KC = KD / 32, NW = NTH / 64;
  // 32-channel groups per column pass: 2 (64-column passes, whole 128-B output lines per pixel) up to 512 threads, 1 at
  // 768 / 1024 threads (3-4 waves per SIMD: no room for the second group's accumulators)
  constexpr int NG2 = NTH <= 512 ? 2 : 1, CP = 32 * NG2;
  bf16* ws = reinterpret_cast<bf16*>(p1s_smem);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* red = reinterpret_cast<float*>(p1s_smem + ng * PITCH * 2) + wid * 64;  // this wave's [2][32] partials
  const int c0 = blockIdx.y * ng;
  const int ncols = min(ng, NC - c0);  // a multiple of 32
  for (int e = threadIdx.x; e < ncols * (KD / 8); e += NTH) {
    const int r = e / (KD / 8), c8 = e % (KD / 8);
    *reinterpret_cast<uint4*>(ws + r * PITCH + c8 * 8) =
        c8 * 8 < kwrow ? *reinterpret_cast<const uint4*>(w + (long)(c0 + r) * kwrow + c8 * 8) : make_uint4(0, 0, 0, 0);
  }
  const bool half = NC <= 64;
  if (psum != nullptr && !half && (ntiles & 1) && blockIdx.x == 0) {  // the last 64-row partial row: no pixels
    for (int n = threadIdx.x; n < ncols; n += NTH) {
      psum[(long)ntiles * NC + c0 + n] = 0.f;
      psq[(long)ntiles * NC + c0 + n] = 0.f;
    }
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, xbytes);
  const int q = lane >> 4, pl = lane & 15;
  // this lane's 16-B output chunk of a 32-channel pair of 16-channel tiles (after the permlane16 swap)
  const int chq = (q & 1) * 16 + (q >> 1) * 8;
  // PF: the next tile's X fragments are loaded while this tile's column passes run (training variants, KD <= 128: 64
  // more VGPRs; DMY_P1S_PF = 0 turns it off at run time)
  constexpr bool PF = !G3 && KD <= 128;
  const int tstride = gridDim.x * NW;
  bf16x8 xf[4][KC];
  auto load_x = [&](bf16x8 (&dst)[4][KC], int tt) {
    const long p0 = (long)tt * 64;
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const long m = p0 + pb * 16 + pl;
      if constexpr (G3) {
        const int mm = m < M ? (int)m : 0, ow = mm % W, oh = (mm / W) % H, bi = mm / (W * H);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const int tap = 2 * kc + (q >> 1), kh = tap / 3, kw = tap - 3 * kh, ih = oh + kh - 1, iw = ow + kw - 1;
          const bool ok = m < M && tap < 9 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
          const unsigned off = ok ? (unsigned)(((bi * H + ih) * W + iw) * (int)xps + 8 * (q & 1)) * 2u : kBufOob;
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
          dst[pb][kc] = *reinterpret_cast<const bf16x8*>(&v);
        }
      } else {
        const unsigned base = m < M ? (unsigned)(m * xps + q * 8) * 2u : kBufOob;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const unsigned off = base == kBufOob ? kBufOob : base + kc * 64u;
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
          dst[pb][kc] = *reinterpret_cast<const bf16x8*>(&v);
        }
      }
    }
  };
  const int t0 = blockIdx.x * NW + wid;
  if (PF && t0 < ntiles) load_x(xf, t0);
  for (int t = t0; t < ntiles; t += tstride) {
    const long p0 = (long)t * 64;
    bf16x8 xn[4][KC];
    if (PF) {
      if (t + tstride < ntiles) load_x(xn, t + tstride);
    } else {
      load_x(xf, t);
    }
    // column passes of NG2 groups of 32 channels (CP = 32 * NG2 columns): the two 64-B halves of each 128-B output line
    // (64 channels of one pixel) leave in back-to-back stores.  Stored 32 channels per pass instead, a line's second
    // half followed a whole pass later and the write stream ran at 3.3-4.1 TB/s instead of 4.9-5.7 (round 4,
    // tools/gpu/store_lab.hip: 'halves' vs 'pairs')
    for (int ct = 0; ct < ncols; ct += CP) {
      const int ngr = min(NG2, (ncols - ct) / 32);  // 32-channel groups in this pass (ncols is a multiple of 32)
      f32x4 acc[2 * NG2][4];                       // [16-channel block][16-pixel block]
#pragma unroll
      for (int cb = 0; cb < 2 * NG2; ++cb)
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) acc[cb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int cb = 0; cb < 2 * NG2; ++cb) {
          if (cb >= 2 * ngr) break;
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(ws + (ct + cb * 16 + pl) * PITCH + kc * 32 + q * 8);
#pragma unroll
          for (int pb = 0; pb < 4; ++pb)
            acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf[pb][kc], acc[cb][pb], 0, 0, 0);
        }
      const int nb = c0 + ct;  // first column of this pass
      if (bias != nullptr) {
#pragma unroll
        for (int cb = 0; cb < 2 * NG2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float bv = cb < 2 * ngr ? bias[nb + cb * 16 + q * 4 + r] : 0.f;
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) acc[cb][pb][r] += bv;
          }
      }
      if (psum != nullptr) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if (!half && hh == 1) break;
#pragma unroll
          for (int gr = 0; gr < NG2; ++gr) {
            if (gr >= ngr) break;
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int cb = 2 * gr + c2;
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int pb = 0; pb < 4; ++pb) {
                  if (half && (pb >> 1) != hh) continue;
                  const float v = p0 + pb * 16 + pl < M ? acc[cb][pb][r] : 0.f;
                  s1 += v;
                  s2 += v * v;
                }
                s1 = row_sum16(s1);
                s2 = row_sum16(s2);
                if (pl == 15) {  // channel c2 * 16 + q * 4 + r of 32-channel group gr
                  red[c2 * 16 + q * 4 + r] = s1;
                  red[32 + c2 * 16 + q * 4 + r] = s2;
                }
              }
            // one 64-lane store per group: lanes 0..31 the 32 channel sums, lanes 32..63 the sums of squares (the
            // wave's own LDS rows: the lane-15 writes above are ordered before this read by the wave's lgkmcnt)
            __builtin_amdgcn_wave_barrier();
            const float v = red[lane];
            const long row = half ? 2L * t + hh : (long)t;
            (lane < 32 ? psum : psq)[row * NC + nb + gr * 32 + (lane & 31)] = v;
            __builtin_amdgcn_wave_barrier();
          }
        }
      }
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const long m = p0 + pb * 16 + pl;
#pragma unroll
        for (int gr = 0; gr < NG2; ++gr) {  // the groups of one pixel back to back: whole 128-B lines
          if (gr >= ngr) break;
          const f32x4 &a = acc[2 * gr][pb], &b = acc[2 * gr + 1][pb];
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk2_bf16(a[0], a[1]), pk2_bf16(b[0], b[1]), false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk2_bf16(a[2], a[3]), pk2_bf16(b[2], b[3]), false, false);
          uint4 v;
          v.x = s0[0];
          v.y = s1[0];
          v.z = s0[1];
          v.w = s1[1];
          if (m < M) {
            uint4* dst = reinterpret_cast<uint4*>(y + m * yps + nb + gr * 32 + chq);
            if (accumulate) {
              float f[8], o[8];
              unpack<bf16>(v, f);
              unpack<bf16>(*dst, o);
#pragma unroll
              for (int j = 0; j < 8; ++j) f[j] += o[j];
              v = pack<bf16>(f);
            }
            *dst = v;
          }
        }
      }
    }
    if (PF) {
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) xf[pb][kc] = xn[pb][kc];
    }
  }
}

// ---------------------------------------------------------------- split-K forward for small M (batch-1 inference)
// At batch 1 the stride-16 / -32 layers have 2304..9216 output pixels: 128-row tiles give 18..72 row tiles, a
// fraction of the 256 CUs, each walking the whole 9 * C reduction.  Split the K steps over blockIdx.y: every split
// writes its fp32 partial tile to a workspace slab, splitk_epi_kernel sums the slabs in split order and applies
// bias + the inference epilogue (eval BN, act, residual) to the bf16-rounded sum -- the same value contract as
// the one-launch path (deterministic; rounding order differs from the unsplit kernel).


template <int BM, int BN, int NS, bool P1>
__global__ void __launch_bounds__(BM * BN / 64) conv_fwd_split(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                               float* __restrict__ ws, Geom g, int gm, int gn, int per,
                                                               unsigned xbytes, unsigned wbytes) {
  using C3_ = Cfg3<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  const int nk = g.KH * g.KW * g.C / BK, split = blockIdx.y;
  const int k0 = split * per, steps = min(nk, k0 + per) - k0;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (steps > 0) {
    FwdLdsB<BM, BN, NS, P1, false> ld(x, w, g, M, m0, n0, wid, lane, xbytes, wbytes);
    ld.skip(k0);
    mainloop4<BM, BN, NS>(ld, steps, smem, acc, wid, lane);
  }
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  float* slab = ws + (long)split * M * g.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        if (m < M && n < g.K) slab[m * g.K + n] = acc[i][j][r];
      }
}

// ---------------------------------------------------------------- fp8 (e4m3) forward, MX-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 block scales (0x7f = 2^0): 2x the bf16 MFMA rate per clock
// (MI355X_MICROARCH.md, matrix-core table).  Operands are OCP e4m3fn: activations per tensor (x ~ x8 * amax / 448),
// weights per output channel (w ~ w8 * wscale[k]); the fp32 accumulator is dequantised by amax / 448 * wscale[n]
// before the shared v3 epilogue (bias, BN partials, inference BN / act / residual).  A K step is 128 fp8 = the
// same 128-B LDS rows as a bf16 step, so the loader (FwdLdsB<..., ES = 1>) and the swizzled image are unchanged.
// A 16x16x128 fragment is 32 bytes per lane; any k order used identically for A and B gives the same dot
// products, so lane group q takes 16-B chunks q and 4 + q of the row -- exactly the two conflict-free ds_read_b128
// of the bf16 kernel's h = 0 / 1 fragments (tools/gpu/probe_f8.hip checked the MFMA with exact integer data).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

DEV i32x8 frag_f8(const char* X, int r0, int lane) {
  const int row = r0 + (lane & 15), q = lane >> 4, sw = row & 6;
  const char* base = X + row * 128;
  const i32x4v lo = *reinterpret_cast<const i32x4v*>(base + ((q ^ sw) << 4));
  const i32x4v hi = *reinterpret_cast<const i32x4v*>(base + (((4 + q) ^ sw) << 4));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int BM, int BN, int NS, class LD>
DEV void mainloop_f8(LD& ld, int nk, char* smem, f32x4 (&acc)[4][4], int wid, int lane) {
  using C3_ = Cfg3<BM, BN, NS>;
  constexpr int PER = C3_::APW + C3_::BPW;
  const int wm = wid % C3_::WM, wn = wid / C3_::WM;
  ld.issue(smem, wid);
  if (NS == 3 && nk > 1) ld.issue(smem + C3_::STAGE, wid);
  for (int kt = 0; kt < nk; ++kt) {
    if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    const char* As = smem + (kt % NS) * C3_::STAGE;
    const char* Bs = As + C3_::A_BYTES;
    i32x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag_f8(As, wm * 64 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag_f8(Bs, wn * 64 + j * 16, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * C3_::STAGE, wid);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                     0x7f7f7f7f);
  }
}

template <int BM, int BN, int NS, bool P1>
__global__ void __launch_bounds__(BM * BN / 64) conv_fwd_f8(const unsigned char* __restrict__ x8,
                                                            const unsigned char* __restrict__ w8,
                                                            const float* __restrict__ xamax,
                                                            const float* __restrict__ wscale,
                                                            const float* __restrict__ bias, bf16* __restrict__ y,
                                                            float* __restrict__ psum, float* __restrict__ psq, Geom g,
                                                            int gm, int gn, unsigned xbytes, unsigned wbytes, Epi ep) {
  using C3_ = Cfg3<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[C3_::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int tile = xcd_remap(blockIdx.x, gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const long M = (long)g.N * g.OH * g.OW;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = g.KH * g.KW * g.C / 128;
  FwdLdsB<BM, BN, NS, P1, false, false, 1> ld(reinterpret_cast<const bf16*>(x8), reinterpret_cast<const bf16*>(w8), g,
                                              M, m0, n0, wid, lane, xbytes, wbytes);
  mainloop_f8<BM, BN, NS>(ld, nk, smem, acc, wid, lane);
  const float am = xamax[0];
  const float sx = am > 0.f ? am * (1.f / 448.f) : (am == 0.f ? 1.f : am);  // NaN amax propagates
  const int wn = wid / C3_::WM;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    const float f = sx * (n < g.K ? wscale[n] : 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] *= f;
  }
  __syncthreads();
  v3_epilogue<BM, BN, NS, false, 1>(acc, reinterpret_cast<bf16*>(smem), bias, y, psum, psq, 0, g, tm, m0, n0,
                                    S2Cls{0, 0, 0, 0}, ep);
}

// Weight-grad: rows m = output channel, columns n = (kh, kw, ci), reduction over pixels (split-K).
// Both operands are k-major ([64 pixels][128 channels], 256-B pixel rows) in the kmaj_off layout of
// the v2 kernel (16-B chunks XOR-swizzled per pixel row, read with ds_read_b64_tr_b16).  One 1-KiB
// LDS-DMA piece = 4 pixel rows; lane l fills pixel row 4i + (l >> 4), slot l & 15, i.e. logical chunk
// (l & 15) ^ key(row), key(row) = 2 ((row & 3) | ((row >> 3) & 1) << 2): two chunk values per lane.
template <int NS>
struct WgradLds {
  static constexpr int BM = 128, BN = 128, PPW = 4;  // pieces per wave per operand (4 waves)
  const bf16* x; const bf16* dy; Geom g; long NP; int Ntot, m0, n0;
  int cA[2], cB[2];                 // logical chunk for key bit 3 = 0 / 1
  bool bok[2]; int bkh[2], bkw[2], bci[2];
  long pix[PPW]; int pb[PPW], poh[PPW], pow_[PPW];  // this lane's pixel per piece (advanced by 64 per step)
  DEV WgradLds(const bf16* x_, const bf16* dy_, const Geom& g_, int m0_, int n0_, int kt0, int wid, int lane)
      : x(x_), dy(dy_), g(g_), m0(m0_), n0(n0_) {
    NP = (long)g.N * g.OH * g.OW;
    Ntot = g.KH * g.KW * g.C;
    const int q = lane >> 4, sl = lane & 15;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = sl ^ (2 * (q | (h << 2)));
      cA[h] = c;
      cB[h] = c;
      const int n = n0 + c * 8;
      bok[h] = n < Ntot;
      bci[h] = n % g.C;
      const int t = n / g.C;
      bkw[h] = t % g.KW;
      bkh[h] = t / g.KW;
    }
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      pix[j] = (long)kt0 * 64 + (wid * PPW + j) * 4 + q;
      const long pp = pix[j] < NP ? pix[j] : 0;
      pow_[j] = (int)(pp % g.OW);
      const long t = pp / g.OW;
      poh[j] = (int)(t % g.OH);
      pb[j] = (int)(t / g.OH);
    }
  }
  DEV void issue(char* stage, int wid) {
    const bf16* zero = reinterpret_cast<const bf16*>(g_zero_page);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int piece = wid * PPW + j;
      const int h = (piece >> 1) & 1;  // bit 3 of the pixel row (rows 4 piece .. 4 piece + 3)
      const bool pin = pix[j] < NP;
      const int co = m0 + cA[h] * 8;
      const bf16* sa = (pin && co < g.K) ? dy + pix[j] * g.yps + co : zero;
      glds16(sa, stage + piece * 1024);
      const int ih = poh[j] * g.S - g.P + bkh[h], iw = pow_[j] * g.S - g.P + bkw[h];
      const bool okb = pin && bok[h] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const bf16* sb = okb ? x + (((long)pb[j] * g.H + ih) * g.W + iw) * g.xps + bci[h] : zero;
      glds16(sb, stage + 16384 + piece * 1024);
      // advance this piece's pixel by one K step (64 pixels)
      pix[j] += 64;
      pow_[j] += 64;
      while (pow_[j] >= g.OW) {
        pow_[j] -= g.OW;
        if (++poh[j] == g.OH) { poh[j] = 0; ++pb[j]; }
      }
    }
  }
};

// Buffer-descriptor form of WgradLds: every address is a 32-bit element offset advanced by adds only
// (the per-pixel 64-bit products of WgradLds cost 32 quarter-rate v_mul_lo_u32 per K step).  Per
// piece the lane tracks its pixel (pix, oh, ow), ih/iw = oh*S - P / ow*S - P and the element bases
// dyb = pix * yps and xb = ((b H + ih) W + iw) xps; a 64-pixel step adds fixed deltas and walks the
// row / image wraps.  Invalid sources get kBufOob (range-checked to zero by the hardware).
struct WgradLdsB {
  static constexpr int PPW = 4;
  __amdgpu_buffer_rsrc_t rx, rdy;
  int NP, OW, OH, H, W, S;
  int dyStep, xStep, xWrapOW, xRow, xImg;   // uniform element deltas
  int co[2], tap[2], bkh[2], bkw[2];        // per lane half: dy column / x tap offset, tap
  bool cok[2], bok[2];
  int pix[PPW], oh[PPW], ow[PPW], ih[PPW], iw[PPW], dyb[PPW], xb[PPW];
  DEV WgradLdsB(const bf16* x, const bf16* dy, const Geom& g, int m0, int n0, int kt0, int wid, int lane,
                unsigned xbytes, unsigned dybytes)
      : OW(g.OW), OH(g.OH), H(g.H), W(g.W), S(g.S) {
    rx = make_rsrc(x, xbytes);
    rdy = make_rsrc(dy, dybytes);
    NP = g.N * g.OH * g.OW;
    const int Ntot = g.KH * g.KW * g.C, xps = (int)g.xps, yps = (int)g.yps;
    dyStep = 64 * yps;
    xStep = 64 * g.S * xps;
    xWrapOW = g.OW * g.S * xps;
    xRow = g.S * g.W * xps;
    xImg = (g.H - g.OH * g.S) * g.W * xps;
    const int q = lane >> 4, sl = lane & 15;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = sl ^ (2 * (q | (h << 2)));
      co[h] = m0 + c * 8;
      cok[h] = co[h] < g.K;
      const int n = n0 + c * 8;
      bok[h] = n < Ntot;
      const int nn = bok[h] ? n : 0;
      const int ci = nn % g.C, t = nn / g.C;
      bkw[h] = t % g.KW;
      bkh[h] = t / g.KW;
      tap[h] = (bkh[h] * g.W + bkw[h]) * xps + ci;
    }
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      pix[j] = kt0 * 64 + (wid * PPW + j) * 4 + q;
      const int pp = pix[j] < NP ? pix[j] : 0;
      ow[j] = pp % g.OW;
      const int t = pp / g.OW;
      oh[j] = t % g.OH;
      const int b = t / g.OH;
      ih[j] = oh[j] * g.S - g.P;
      iw[j] = ow[j] * g.S - g.P;
      dyb[j] = pix[j] * yps;
      xb[j] = ((b * g.H + ih[j]) * g.W + iw[j]) * xps;
    }
  }
  DEV void issue(char* stage, int wid) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int piece = wid * PPW + j;
      const int h = (j >> 1) & 1;  // bit 3 of the pixel row 4 piece + q (wid * PPW is a multiple of 4)
      const bool pin = pix[j] < NP;
      blds16(rdy, (pin && cok[h]) ? (unsigned)(dyb[j] + co[h]) * 2u : kBufOob, stage + piece * 1024);
      const bool okb = pin && bok[h] && (unsigned)(ih[j] + bkh[h]) < (unsigned)H && (unsigned)(iw[j] + bkw[h]) < (unsigned)W;
      blds16(rx, okb ? (unsigned)(xb[j] + tap[h]) * 2u : kBufOob, stage + 16384 + piece * 1024);
      pix[j] += 64;
      dyb[j] += dyStep;
      ow[j] += 64;
      iw[j] += 64 * S;
      xb[j] += xStep;
      while (ow[j] >= OW) {
        ow[j] -= OW;
        iw[j] -= OW * S;
        xb[j] += xRow - xWrapOW;
        ih[j] += S;
        if (++oh[j] == OH) {
          oh[j] = 0;
          ih[j] -= OH * S;
          xb[j] += xImg;
        }
      }
    }
  }
};

template <int NS, int BUF>
__global__ void __launch_bounds__(256) conv_wgrad_v3(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                     float* __restrict__ dw, int kt_per_split, Geom g, int gm, int gn,
                                                     unsigned xbytes, unsigned dybytes) {
  constexpr int BM = 128, BN = 128, STAGE = 32768;
  constexpr int LDS = NS * STAGE > BM * (BN + 4) * 4 ? NS * STAGE : BM * (BN + 4) * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // (tile, split) from the linear dispatch id: consecutive logical ids share an XCD, so all tiles of
  // a split (which read the same pixel chunk) run on one XCD and share its L2
  const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int tile = lin % (gm * gn), split = lin / (gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const int m0 = tm * BM, n0 = tn * BN;
  const long NP = (long)g.N * g.OH * g.OW;
  const int nk_all = (int)((NP + 63) / 64);
  const int kt0 = split * kt_per_split;
  const int nk = min(nk_all, kt0 + kt_per_split) - kt0;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0 && BUF > 0) {
    // fragments of the whole step first, then the next stage's DMA while they land, then 32 MFMAs
    WgradLdsB ld(x, dy, g, m0, n0, kt0, wid, lane, xbytes, dybytes);
    ld.issue(smem, wid);
    if (NS == 3 && nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (NS == 3 && kt + 1 < nk) vm_wait<8>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = As + 64 * BM;
      bf16x8 a[2][4], b[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[h][i] = frag_k<BM>(As, wm * 64 + i * 16, h * 32, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[h][j] = frag_k<BN>(Bs, wn * 64 + j * 16, h * 32, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (BUF == 1 && kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
    }
  } else if (nk > 0) {
    WgradLds<NS> ld(x, dy, g, m0, n0, kt0, wid, lane);
    ld.issue(smem, wid);
    if (NS == 3 && nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (NS == 3 && kt + 1 < nk) vm_wait<8>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = As + 64 * BM;
#pragma unroll
      for (int ks = 0; ks < 64; ks += 32) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = frag_k<BM>(As, wm * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag_k<BN>(Bs, wn * 64 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int RS = BN + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * RS + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int Ntot = g.KH * g.KW * g.C;
  static_assert((256) % BN == 0, "epilogue column must be fixed per thread");
  const int c = threadIdx.x % BN, n = n0 + c;
  const long coff = wgrad_col(g, n);
  for (int e = threadIdx.x; e < BM * BN; e += 256) {
    const int row = e / BN, m = m0 + row;
    if (m < g.K && n < Ntot) wgrad_out(g, dw, split, (long)m * Ntot + coff, ct[row * RS + c]);
  }
}
// Narrow-layer weight-grad (out channels <= 64): block tile BM (out channels, 32 or 64) x BN
// ((kh, kw, ci) columns, 128 or 256), NW = BN / 64 waves side by side, each BM x 64.  Same k-major
// swizzled LDS images as conv_wgrad_v3 (kmaj_off<BM> / kmaj_off<BN>), filled by LDS-DMA: a 1-KiB
// piece covers 1024 / rowbytes pixel rows, lane l writes row (l / slots), physical slot (l % slots),
// i.e. the logical chunk (slot ^ key(row)) & (slots - 1).
template <int ROW> DEV int kmaj_chunk(int row, int slot) {
  constexpr int RB = ROW * 2;
  int key;
  if constexpr (RB >= 256) key = 2 * ((row & 3) | (((row >> 3) & 1) << 2));
  else key = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
  return (slot ^ key) & (ROW / 8 - 1);
}

template <int BM, int BN>
struct WgradLdsN {
  static constexpr int NW = BN / 64;
  static constexpr int RA = BM * 2, RB = BN * 2;
  static constexpr int SA = RA / 16, SB = RB / 16;
  static constexpr int PAW = 64 * RA / 1024 / NW, PBW = 64 * RB / 1024 / NW;
  static constexpr int RPA = 1024 / RA, RPB = 1024 / RB;
  static constexpr int A_BYTES = 64 * RA, STAGE = 64 * (RA + RB);
  static_assert(PAW >= 1 && PBW >= 1 && PAW * NW * 1024 == A_BYTES, "tile");
  const bf16* x; const bf16* dy; Geom g; long NP;
  long apix[PAW]; int aco[PAW];
  long bpix[PBW]; int bb[PBW], boh[PBW], bow[PBW], bkh[PBW], bkw[PBW], bci[PBW]; bool bok[PBW];
  DEV WgradLdsN(const bf16* x_, const bf16* dy_, const Geom& g_, int m0, int n0, int kt0, int wid, int lane)
      : x(x_), dy(dy_), g(g_) {
    NP = (long)g.N * g.OH * g.OW;
    const int Ntot = g.KH * g.KW * g.C;
#pragma unroll
    for (int j = 0; j < PAW; ++j) {
      const int r = (wid * PAW + j) * RPA + lane / SA;
      apix[j] = (long)kt0 * 64 + r;
      const int co = m0 + 8 * kmaj_chunk<BM>(r, lane % SA);
      aco[j] = co < g.K ? co : -1;
    }
#pragma unroll
    for (int j = 0; j < PBW; ++j) {
      const int r = (wid * PBW + j) * RPB + lane / SB;
      bpix[j] = (long)kt0 * 64 + r;
      const long pp = bpix[j] < NP ? bpix[j] : 0;
      bow[j] = (int)(pp % g.OW);
      const long t = pp / g.OW;
      boh[j] = (int)(t % g.OH);
      bb[j] = (int)(t / g.OH);
      const int n = n0 + 8 * kmaj_chunk<BN>(r, lane % SB);
      bok[j] = n < Ntot;
      bci[j] = n % g.C;
      const int u = n / g.C;
      bkw[j] = u % g.KW;
      bkh[j] = u / g.KW;
    }
  }
  DEV void issue(char* stage, int wid) {
    const bf16* zero = reinterpret_cast<const bf16*>(g_zero_page);
#pragma unroll
    for (int j = 0; j < PAW; ++j) {
      const bf16* sa = (apix[j] < NP && aco[j] >= 0) ? dy + apix[j] * g.yps + aco[j] : zero;
      glds16(sa, stage + (wid * PAW + j) * 1024);
      apix[j] += 64;
    }
#pragma unroll
    for (int j = 0; j < PBW; ++j) {
      const int ih = boh[j] * g.S - g.P + bkh[j], iw = bow[j] * g.S - g.P + bkw[j];
      const bool ok = bpix[j] < NP && bok[j] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const bf16* sb = ok ? x + (((long)bb[j] * g.H + ih) * g.W + iw) * g.xps + bci[j] : zero;
      glds16(sb, stage + A_BYTES + (wid * PBW + j) * 1024);
      bpix[j] += 64;
      bow[j] += 64;
      while (bow[j] >= g.OW) {
        bow[j] -= g.OW;
        if (++boh[j] == g.OH) { boh[j] = 0; ++bb[j]; }
      }
    }
  }
};

// Buffer-descriptor form of WgradLdsN (same LDS images): 32-bit element offsets advanced by adds
// (see WgradLdsB).  A piece j: pixel row r, dy column co; B piece j: pixel row r, column n -> tap.
template <int BM, int BN, int NWV = BN / 64>
struct WgradLdsNB {
  using L = WgradLdsN<BM, BN>;  // LDS image layout (row bytes, slots, rows per piece); NWV waves share the pieces
  static constexpr int PAW = 64 * L::RA / 1024 / NWV, PBW = 64 * L::RB / 1024 / NWV, A_BYTES = L::A_BYTES;
  static_assert(PAW >= 1 && PBW >= 1 && PAW * NWV * 1024 == A_BYTES, "pieces");
  __amdgpu_buffer_rsrc_t rx, rdy;
  int NP, OW, OH, H, W, S, dyStep, xStep, xWrapOW, xRow, xImg;
  int apix[PAW], adyb[PAW];
  int bpix[PBW], boh[PBW], bow[PBW], bih[PBW], biw[PBW], bxb[PBW], bkh[PBW], bkw[PBW], btap[PBW];
  DEV WgradLdsNB(const bf16* x, const bf16* dy, const Geom& g, int m0, int n0, int kt0, int wid, int lane,
                 unsigned xbytes, unsigned dybytes)
      : OW(g.OW), OH(g.OH), H(g.H), W(g.W), S(g.S) {
    rx = make_rsrc(x, xbytes);
    rdy = make_rsrc(dy, dybytes);
    NP = g.N * g.OH * g.OW;
    const int Ntot = g.KH * g.KW * g.C, xps = (int)g.xps, yps = (int)g.yps;
    dyStep = 64 * yps;
    xStep = 64 * g.S * xps;
    xWrapOW = g.OW * g.S * xps;
    xRow = g.S * g.W * xps;
    xImg = (g.H - g.OH * g.S) * g.W * xps;
#pragma unroll
    for (int j = 0; j < PAW; ++j) {
      const int r = (wid * PAW + j) * L::RPA + lane / L::SA;
      apix[j] = kt0 * 64 + r;
      const int co = m0 + 8 * kmaj_chunk<BM>(r, lane % L::SA);
      // an out-of-range column never becomes valid: fold it into the pixel bound
      adyb[j] = apix[j] * yps + co;
      if (co >= g.K) apix[j] = 0x40000000;
    }
#pragma unroll
    for (int j = 0; j < PBW; ++j) {
      const int r = (wid * PBW + j) * L::RPB + lane / L::SB;
      bpix[j] = kt0 * 64 + r;
      const int pp = bpix[j] < NP ? bpix[j] : 0;
      bow[j] = pp % g.OW;
      const int t = pp / g.OW;
      boh[j] = t % g.OH;
      const int b = t / g.OH;
      bih[j] = boh[j] * g.S - g.P;
      biw[j] = bow[j] * g.S - g.P;
      bxb[j] = ((b * g.H + bih[j]) * g.W + biw[j]) * xps;
      const int n = n0 + 8 * kmaj_chunk<BN>(r, lane % L::SB);
      const int nn = n < Ntot ? n : 0;
      const int ci = nn % g.C, u = nn / g.C;
      bkw[j] = u % g.KW;
      bkh[j] = u / g.KW;
      btap[j] = (bkh[j] * g.W + bkw[j]) * xps + ci;
      if (n >= Ntot) bkh[j] = 0x40000000;  // never in-image
    }
  }
  DEV void issue(char* stage, int wid) {
#pragma unroll
    for (int j = 0; j < PAW; ++j) {
      blds16(rdy, apix[j] < NP ? (unsigned)adyb[j] * 2u : kBufOob, stage + (wid * PAW + j) * 1024);
      apix[j] += 64;
      adyb[j] += dyStep;
    }
#pragma unroll
    for (int j = 0; j < PBW; ++j) {
      const bool ok = bpix[j] < NP && (unsigned)(bih[j] + bkh[j]) < (unsigned)H && (unsigned)(biw[j] + bkw[j]) < (unsigned)W;
      blds16(rx, ok ? (unsigned)(bxb[j] + btap[j]) * 2u : kBufOob, stage + A_BYTES + (wid * PBW + j) * 1024);
      bpix[j] += 64;
      bow[j] += 64;
      biw[j] += 64 * S;
      bxb[j] += xStep;
      while (bow[j] >= OW) {
        bow[j] -= OW;
        biw[j] -= OW * S;
        bxb[j] += xRow - xWrapOW;
        bih[j] += S;
        if (++boh[j] == OH) {
          boh[j] = 0;
          bih[j] -= OH * S;
          bxb[j] += xImg;
        }
      }
    }
  }
};

template <int BM, int BN, int NS, bool BUF>
__global__ void __launch_bounds__(BN) conv_wgrad_v3n(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                    float* __restrict__ dw, int kt_per_split, Geom g, int gm, int gn,
                                                    unsigned xbytes, unsigned dybytes) {
  using LD = WgradLdsN<BM, BN>;
  constexpr int STAGE = LD::STAGE, TM = BM / 16, PER = LD::PAW + LD::PBW;
  constexpr int LDSB = NS * STAGE > BM * (BN + 4) * 4 ? NS * STAGE : BM * (BN + 4) * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // (tile, split) from the linear dispatch id: consecutive logical ids share an XCD, so all tiles of
  // a split (which read the same pixel chunk) run on one XCD and share its L2
  const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int tile = lin % (gm * gn), split = lin / (gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const int m0 = tm * BM, n0 = tn * BN;
  const long NP = (long)g.N * g.OH * g.OW;
  const int nk_all = (int)((NP + 63) / 64);
  const int kt0 = split * kt_per_split;
  const int nk = min(nk_all, kt0 + kt_per_split) - kt0;
  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0 && BUF) {
    WgradLdsNB<BM, BN> ld(x, dy, g, m0, n0, kt0, wid, lane, xbytes, dybytes);
    ld.issue(smem, wid);
    if (NS == 3 && nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE + LD::A_BYTES);
      bf16x8 a[2][TM], b[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < TM; ++i) a[h][i] = frag_k<BM>(As, i * 16, h * 32, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[h][j] = frag_k<BN>(Bs, wid * 64 + j * 16, h * 32, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
    }
  } else if (nk > 0) {
    LD ld(x, dy, g, m0, n0, kt0, wid, lane);
    ld.issue(smem, wid);
    if (NS == 3 && nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (NS == 3 && kt + 1 < nk) vm_wait<PER>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE + LD::A_BYTES);
#pragma unroll
      for (int ks = 0; ks < 64; ks += 32) {
        bf16x8 a[TM], b[4];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = frag_k<BM>(As, i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag_k<BN>(Bs, wid * 64 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int RS = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(i * 16 + 4 * (lane >> 4) + r) * RS + wid * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int Ntot = g.KH * g.KW * g.C;
  static_assert((BN) % BN == 0, "epilogue column must be fixed per thread");
  const int c = threadIdx.x % BN, n = n0 + c;
  const long coff = wgrad_col(g, n);
  for (int e = threadIdx.x; e < BM * BN; e += BN) {
    const int row = e / BN, m = m0 + row;
    if (m < g.K && n < Ntot) wgrad_out(g, dw, split, (long)m * Ntot + coff, ct[row * RS + c]);
  }
}
// Weight-grad v4: 8 waves (BM / 64 x BN / 64, each 64 x 64), BM x BN = 128 x 256 or 256 x 128, a
// 3-stage LDS-DMA ring (48 KiB stages, one block per CU, 2 waves per SIMD) with a counted
// vmcnt(pieces per wave) so one stage stays in flight across each barrier -- the forward kernel's
// structure; the narrow-tile buffer loader with the pieces shared by all 8 waves.
template <int BM, int BN>
__global__ void __launch_bounds__(512) conv_wgrad_v4(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                     float* __restrict__ dw, int kt_per_split, Geom g, int gm, int gn,
                                                     unsigned xbytes, unsigned dybytes) {
  constexpr int WM = BM / 64, NS = 3;
  static_assert(WM * (BN / 64) == 8, "8 waves");
  using LD = WgradLdsNB<BM, BN, 8>;
  constexpr int STAGE = WgradLdsN<BM, BN>::STAGE, PER = LD::PAW + LD::PBW;
  constexpr int CT = BM * (BN + 4) * 4;
  constexpr int LDSB = NS * STAGE > CT ? NS * STAGE : CT;
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int tile = lin % (gm * gn), split = lin / (gm * gn);
  const int tm = tile / gn, tn = tile % gn;
  const int m0 = tm * BM, n0 = tn * BN;
  const long NP = (long)g.N * g.OH * g.OW;
  const int nk_all = (int)((NP + 63) / 64);
  const int kt0 = split * kt_per_split;
  const int nk = min(nk_all, kt0 + kt_per_split) - kt0;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    LD ld(x, dy, g, m0, n0, kt0, wid, lane, xbytes, dybytes);
    ld.issue(smem, wid);
    if (nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) vm_wait<PER>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE + LD::A_BYTES);
      bf16x8 a[2][4], b[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[h][i] = frag_k<BM>(As, wm * 64 + i * 16, h * 32, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[h][j] = frag_k<BN>(Bs, wn * 64 + j * 16, h * 32, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
    }
  }
  vm_wait<0>();
  __syncthreads();
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int RS = BN + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * RS + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int Ntot = g.KH * g.KW * g.C;
  static_assert((512) % BN == 0, "epilogue column must be fixed per thread");
  const int c = threadIdx.x % BN, n = n0 + c;
  const long coff = wgrad_col(g, n);
  for (int e = threadIdx.x; e < BM * BN; e += 512) {
    const int row = e / BN, m = m0 + row;
    if (m < g.K && n < Ntot) wgrad_out(g, dw, split, (long)m * Ntot + coff, ct[row * RS + c]);
  }
}

// ---------------------------------------------------------------- tap-fused 3x3 stride-1 weight-grad
// C[m = out channel][n = (tap, ci)] = sum over output pixels p of dy[p][m] * x[p + tap shift][ci], for a block tile
// of 128 out channels x (all 9 taps x 32 input channels) = 288 columns.  The reduction walks 8 x 8 output-pixel
// patches (64 pixels per K step): the x operand is the patch's 10 x 10 halo (32 channels) loaded ONCE and read by
// all 9 taps through shifted LDS addresses, so x is fetched ~1.6x per (out-channel tile) and dy once per 32-channel
// group -- vs 9x / 18x for the (tap, channel)-column tiles of conv_wgrad_v3/v4.
//   A (dy): [64 pixel rows][BM ch] k-major, the kmaj_off<BM> swizzle, frag_k<BM> (as conv_wgrad_v3 / v3n);
//   BM = 128, or 64 for layers with <= 64 output channels.
//   B (x halo): 10 rows of pitch 12 pixels x 32 ch (64-B rows), chunk ^ 2 (halo row y & 1): the 8 rows one
//   ds_read_b64_tr_b16 group touches ((y, x .. x + 3), (y + 1, x .. x + 3)) then hit 64 distinct banks.
//   Stages: BM/8 KiB A + 8 KiB B (120 of 128 halo rows used), 3-stage LDS-DMA ring, a counted vmcnt keeps one
//   stage in flight across each barrier.  4 waves = 2 (m) x 2 (n), wave tile BM/2 x 144 (BM/32 x 9 MFMA frags).
// Valid for KH = KW = 3, S = 1, P = 1, OH = H, OW = W, C % 16 == 0 (host-checked; a
// 16-channel plane half loads zeros).  Split-K over patches; the
// (tile, split) -> linear id mapping keeps a split's tiles on one XCD (they read the same patches).
template <int BM, int NP = 1>  // NP halo planes of 32 input channels each (2: a block owns 64 input channels)
struct WgradTapLds {
  static constexpr int BC = 32, PH = 8, PW = 8, HP = 12;  // halo pitch 12 (10 used)
  static constexpr int A_BYTES = 64 * BM * 2, B_BYTES = NP * 8 * 1024, STAGE = A_BYTES + B_BYTES;
  static constexpr int APW = A_BYTES / 1024 / 4;           // dy pieces per wave (4 waves)
  static constexpr int SLOTS = BM / 8, RPP = 64 / SLOTS;   // 16-B slots per pixel row, pixel rows per piece
  __amdgpu_buffer_rsrc_t rx, rdy;
  int OH, OW, H, W, npw, nph;
  int pb, py, px;                    // patch cursor (uniform)
  int arel[APW], ar[APW], ac[APW];   // dy: per piece pixel (r, c) in the patch and element offset rel. to the patch
  int acol[APW];                     // dy column (element) this lane loads for the piece
  bool aok[APW];
  int brel[2], by[2], bx[2];         // x halo: per piece halo (y, x) and element offset rel. to the halo origin
  int bcol[2];
  bool bok[2];
  int yps, xps, cmax;
  DEV WgradTapLds(const bf16* x, const bf16* dy, const Geom& g, int m0, int c0, int kt0, int wid, int lane,
                  unsigned xbytes, unsigned dybytes)
      : OH(g.OH), OW(g.OW), H(g.H), W(g.W) {
    cmax = g.C;  // C % 32 == 16 (the 16-channel space-to-depth stem): the plane's chunks past C load zeros
    rx = make_rsrc(x, xbytes);
    rdy = make_rsrc(dy, dybytes);
    yps = (int)g.yps;
    xps = (int)g.xps;
    npw = (g.OW + PW - 1) / PW;
    nph = (g.OH + PH - 1) / PH;
    px = kt0 % npw;
    const int t = kt0 / npw;
    py = t % nph;
    pb = t / nph;
#pragma unroll
    for (int j = 0; j < APW; ++j) {  // piece wid * APW + j: pixel rows RPP * piece + lane / SLOTS
      const int row = (wid * APW + j) * RPP + lane / SLOTS;
      const int slot = lane % SLOTS;
      // physical slot -> logical chunk under the kmaj_off<BM> key of this pixel row
      const int key = (2 * BM >= 256) ? 2 * ((row & 3) | (((row >> 3) & 1) << 2))
                                      : 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
      const int chunk = (slot ^ key) & (SLOTS - 1);
      acol[j] = m0 + chunk * 8;
      aok[j] = acol[j] < g.K;
      ar[j] = row >> 3;
      ac[j] = row & 7;
      arel[j] = (ar[j] * g.OW + ac[j]) * yps;
    }
    // halo: 8 pieces x 16 rows of 64 B; this wave fills pieces wid * 2 + j; lane: row (lane >> 2), slot lane & 3
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (wid * 2 + j) * 16 + (lane >> 2);
      by[j] = row / HP;
      bx[j] = row % HP;
      const int chunk = (lane & 3) ^ (2 * (by[j] & 1));
      bok[j] = row < 10 * HP && bx[j] < 10;
      brel[j] = (by[j] * g.W + bx[j]) * xps;
      bcol[j] = c0 + chunk * 8;
    }
  }
  DEV void issue(char* stage, int wid) {
    const int oy0 = py * PH, ox0 = px * PW;
    const int abase = ((pb * OH + oy0) * OW + ox0) * yps;
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      const bool ok = aok[j] && oy0 + ar[j] < OH && ox0 + ac[j] < OW;
      blds16(rdy, ok ? (unsigned)(abase + arel[j] + acol[j]) * 2u : kBufOob, stage + (wid * APW + j) * 1024);
    }
    const int xbase = ((pb * H + oy0 - 1) * W + ox0 - 1) * xps;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ok = bok[j] && (unsigned)(oy0 - 1 + by[j]) < (unsigned)H && (unsigned)(ox0 - 1 + bx[j]) < (unsigned)W;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        blds16(rx, ok && bcol[j] + 32 * pl < cmax ? (unsigned)(xbase + brel[j] + bcol[j] + 32 * pl) * 2u : kBufOob,
               stage + A_BYTES + pl * 8192 + (wid * 2 + j) * 1024);
    }
    if (++px == npw) {
      px = 0;
      if (++py == nph) { py = 0; ++pb; }
    }
  }
};

// B fragment of tap (kh, kw), 16 channels from ch0, pixels k0 .. k0 + 31 of the patch (frag_k's lane mapping with
// pixel k -> halo row ((k >> 3) + kh, (k & 7) + kw))
DEV bf16x8 frag_halo(const bf16* Bs, int kh, int kw, int ch0, int k0, int lane) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3;
  const int ch = ch0 + 4 * p;
  const int y = (k0 >> 3) + g + kh;
  const int chunk = (ch >> 3) ^ (2 * (y & 1));
  const int off = (y * WgradTapLds<128>::HP + q + kw) * 32 + ((chunk & 3) << 3) + (ch & 7);
  s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(Bs + off));
  s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(Bs + off + 4 * 32));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// NP = 2 (layers with <= 64 output channels, BM = 64): a block owns 64 input channels (two halo planes) and its 4
// waves are 1 (m) x 4 (n), wave tile BM x 144 (4 A + 9 B fragments per 36 MFMAs instead of 2 + 9 per 18): the
// halo fragment reads, which bound the 64-channel layers on the LDS port, are amortised over twice the rows
template <int BM, int NP = 1>
__global__ void __launch_bounds__(256, 2) conv_wgrad_tap(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                         float* __restrict__ dw, int kt_per_split, Geom g, int gm,
                                                         int gn, int nk_all, unsigned xbytes, unsigned dybytes) {
  using LD = WgradTapLds<BM, NP>;
  constexpr int NS = 3, STAGE = LD::STAGE;
  constexpr int TM = NP == 2 ? BM / 16 : BM / 32;           // NP 1: 2 (m) x 2 (n) waves; NP 2: 1 x 4
  constexpr int NCOL = 288 * NP;                            // tile columns: NP planes x 9 taps x 32 channels
  constexpr int NPASS = (BM == 128 && NP == 2) ? 4 : 2;    // epilogue: the tile staged in NPASS row slices
  constexpr int CTR = BM / NPASS, CTS = NCOL + 4;
  constexpr int LDSB = NS * STAGE > CTR * CTS * 4 ? NS * STAGE : CTR * CTS * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = NP == 2 ? 0 : wid >> 1, wn = NP == 2 ? (wid & 1) : wid & 1, wpl = NP == 2 ? wid >> 1 : 0;
  const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int tile = lin % (gm * gn), split = lin / (gm * gn);
  const int tm = tile % gm, tc = tile / gm;  // out-channel tiles of one channel group adjacent (share the x halo)
  const int m0 = tm * BM, c0 = tc * LD::BC * NP;
  const int kt0 = split * kt_per_split;
  const int nk = min(nk_all, kt0 + kt_per_split) - kt0;
  f32x4 acc[TM][9];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    LD ld(x, dy, g, m0, c0, kt0, wid, lane, xbytes, dybytes);
    ld.issue(smem, wid);
    if (nk > 1) ld.issue(smem + STAGE, wid);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) vm_wait<LD::APW + 2 * NP>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + NS - 1 < nk) ld.issue(smem + ((kt + NS - 1) % NS) * STAGE, wid);
      const bf16* As = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE);
      const bf16* Bs = reinterpret_cast<const bf16*>(smem + (kt % NS) * STAGE + LD::A_BYTES + wpl * 8192);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 a[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = frag_k<BM>(As, wm * (BM / 2) + i * 16, h * 32, lane);
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const int f = wn * 9 + j, tap = f >> 1;
          const bf16x8 b = frag_halo(Bs, tap / 3, tap % 3, (f & 1) * 16, h * 32, lane);
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  vm_wait<0>();
  const int Ntot = 9 * g.C;
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int half = 0; half < NPASS; ++half) {
    __syncthreads();
    if (NP == 2 || wm == half) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = NP == 2 ? i * 16 - half * CTR : i * 16;  // row of the staged half
        if (NP == 2 && (row < 0 || row >= CTR)) continue;
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(row + 4 * (lane >> 4) + r) * CTS + wpl * 288 + (wn * 9 + j) * 16 + (lane & 15)] = acc[i][j][r];
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < CTR * NCOL; e += 256) {
      const int row = e / NCOL, col = e % NCOL, m = m0 + half * CTR + row;
      const int pl = col / 288, cc = col % 288;
      const int ci = c0 + pl * 32 + (cc & 31), n = (cc >> 5) * g.C + ci;  // cc = tap * 32 + ci
      if (m < g.K && ci < g.C) wgrad_out(g, dw, split, (long)m * Ntot + wgrad_col(g, n), ct[row * CTS + col]);
    }
  }
}

// ---------------------------------------------------------------- 3x3 stride-1 halo kernel, 64 -> 64 channels
// The 64-channel 3x3 layers (DMA-YOLO's C3 bottlenecks at 384^2, SCConv k3 at 768^2) ran at 20-26 % of the MFMA peak on
// the implicit-GEMM tiles: with 64 output columns every gathered A byte feeds only 128 flops, and the tap gather re-reads
// each input pixel 9 times from L2 (256 x 64 A rows per K step, 9 K steps per tile), so the tiles wait on L2 -> LDS
// traffic and on a 9-step pipeline's prologue / epilogue.  Here a block owns the whole layer's weights in LDS (9 taps
// x 64 x 64 bf16 = 72 KiB, loaded once: persistent grid, one block per CU) and walks output tiles of 8 image rows x
// 32 pixels: per tile ONE LDS-DMA load of the 10 x 34-pixel input halo (43 KiB, double-buffered so the next tile's
// halo streams in under this tile's MFMAs), then all 9 taps read the halo through shifted LDS addresses.  L2 -> LDS
// traffic per output pixel drops from 9 x 128 B to ~1.33 x 128 B.
//   MFMA v_mfma_f32_32x32x16_bf16, transposed (D[channel][pixel] = W X^T): 4 waves (one per SIMD), wave w computes
//   image rows 2w, 2w + 1 of the tile (32 pixels on the lanes each) x 64 channels = 2 x 2 accumulators, so per
//   (tap, 16-deep k step) 2 halo + 2 weight fragments feed 4 MFMAs (1 KiB of LDS reads per 32-cycle MFMA: half the
//   LDS array's 256 B/clk; a first version with 8 waves of one row each read 1.5 KiB per MFMA and ran at 34 % of the
//   MFMA peak).  A 16-B fragment is (row = l & 31, k chunk 2s + (l >> 5)) of a 128-B LDS row (a halo pixel, or a
//   (tap, channel) row of W), 16-B chunks XOR-swizzled by (row >> 1) & 7: for every 32-row window, aligned or not,
//   each ds_read_b128 lane group hits 16 distinct bank quads.
//   Epilogue from registers: bf16 pairs, v_permlane32_swap -> 8 consecutive channels per lane, 8 x 16-B buffer stores
//   per lane (they drain under the next tile's MFMAs: the next halo's wait counts exactly these 8 as younger).
//   BN partials: each lane accumulates sum z and sum z^2 of its pixel column over all tiles of the block in fp32;
//   after the last tile the block writes ONE partial row per wave (rows blockIdx.x * 4 + wave, fixed order, no
//   atomics): dmy_conv_fwd_bn_rows reports that row count to the host.
//   DG = true: stride-1 data-grad, same gather with the tap sign flipped (dy halo, IHWO weight copy); accumulate adds
//   the previous dx (loaded before the tile's MFMAs) as v3_epilogue does.
namespace halo {
constexpr int TH = 8, TW = 32;            // output tile: 8 image rows (two per wave) x 32 pixels
constexpr int HW = TW + 2;                // halo row width (34 pixels); 10 halo rows
constexpr int HPIX = (TH + 2) * HW;       // 340 pixels
constexpr int HPIECES = (HPIX + 7) / 8;   // 43 LDS-DMA pieces of 8 pixel rows (1 KiB)
constexpr int HBYTES = HPIECES * 1024;
constexpr int WBYTES = 9 * 64 * 128;      // [tap][n][64 channels]
constexpr int LDS = WBYTES + 2 * HBYTES;  // 161792 B
constexpr int NW = 4;
constexpr int NPC = (HPIECES + NW - 1) / NW;  // halo pieces per wave (waves >= HPIECES % NW issue one fewer)
}  // namespace halo
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
DEV int hsw(int row) { return (row >> 1) & 7; }
// accumulate epilogue: (bf16-rounded new value) + previous bf16 value, rounded once more -- the sum v3_epilogue forms
DEV u4 add_bf16x8(u4 a, u4 b) {
  float fa[8], fb[8];
  unpack<bf16>(make_uint4(a[0], a[1], a[2], a[3]), fa);
  unpack<bf16>(make_uint4(b[0], b[1], b[2], b[3]), fb);
#pragma unroll
  for (int e = 0; e < 8; ++e) fa[e] += fb[e];
  const uint4 o = pack<bf16>(fa);
  return u4{o.x, o.y, o.z, o.w};
}

template <bool DG, bool EP = false>
__global__ void __launch_bounds__(256, 1) conv3_halo64(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                        bf16* __restrict__ y, float* __restrict__ psum,
                                                        float* __restrict__ psq, Geom g, int twn, int thn, int ntiles,
                                                        int per, unsigned xbytes, unsigned wbytes, unsigned ybytes,
                                                        int accumulate, Epi ep, unsigned rbytes) {
  // the eval instantiation keeps the 64 channels' scale / shift after the ring (512 B, written before the first barrier)
  __shared__ __attribute__((aligned(1024))) char smem[halo::LDS + (EP ? 512 : 0)];
  if (EP && threadIdx.x < 128) {
    const int c = threadIdx.x & 63;
    const float* src = threadIdx.x < 64 ? ep.scale : ep.shift;
    reinterpret_cast<float*>(smem + halo::LDS)[threadIdx.x] = src != nullptr ? src[c] : (threadIdx.x < 64 ? 1.f : 0.f);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, px = lane & 31, hf = lane >> 5;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, xbytes), rw = make_rsrc(w, wbytes), ry = make_rsrc(y, ybytes);
  char* const wl = smem;
  const int u0 = blockIdx.x * per, u1 = min(u0 + per, ntiles);
  if (u0 >= u1) return;
  // weights: 72 pieces, 18 per wave; row r = tap * 64 + n holds chunk (lane & 7) ^ hsw(r) of its 64 channels
#pragma unroll
  for (int i = 0; i < 18; ++i) {
    const int pc = wid * 18 + i, r = pc * 8 + (lane >> 3), tap = r >> 6, n = r & 63;
    const int c = (lane & 7) ^ hsw(r);
    blds16(rw, (unsigned)((n * 576 + tap * 64 + c * 8) * 2), wl + pc * 1024);
  }
  // this lane's halo pieces: pixel slot p = 8 pc + (lane >> 3) -> halo (hr, hc), source chunk (lane & 7) ^ hsw(p)
  const int npc = wid < halo::HPIECES - halo::NW * (halo::NPC - 1) ? halo::NPC : halo::NPC - 1;
  int hr[halo::NPC], hc[halo::NPC], rel[halo::NPC];
#pragma unroll
  for (int i = 0; i < halo::NPC; ++i) {
    const int p = (wid + halo::NW * i) * 8 + (lane >> 3);
    const bool in = p < halo::HPIX;
    hr[i] = in ? p / halo::HW : -1000000;  // slots past the halo load zeros
    hc[i] = p % halo::HW;
    rel[i] = in ? (hr[i] * g.W + hc[i]) * (int)g.xps + (((lane & 7) ^ hsw(p)) << 3) : 0;
  }
  auto tile_pos = [&](int u, int& b, int& oh0, int& ow0) {
    const int th = u % thn, t2 = u / thn;
    oh0 = th * halo::TH;
    ow0 = (t2 % twn) * halo::TW;
    b = t2 / twn;
  };
  auto issue_halo = [&](int u, char* hl) {
    int b, oh0, ow0;
    tile_pos(u, b, oh0, ow0);
    const int base = ((b * g.H + oh0 - 1) * g.W + ow0 - 1) * (int)g.xps;
#pragma unroll
    for (int i = 0; i < halo::NPC; ++i) {
      if (i < npc) {
        const int ih = oh0 - 1 + hr[i], iw = ow0 - 1 + hc[i];
        const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        blds16(rx, ok ? (unsigned)(base + rel[i]) * 2u : kBufOob, hl + (wid + halo::NW * i) * 1024);
      }
    }
  };
  issue_halo(u0, smem + halo::WBYTES);
  vm_wait<0>();
  const bool stats = !EP && psum != nullptr;  // the eval instantiation never writes partials (launch_halo's caller)
  const bool resid = EP && ep.res != nullptr, pre = accumulate || resid;
  const long pstride = resid ? ep.rps : g.yps;
  const __amdgpu_buffer_rsrc_t rp = resid ? make_rsrc(ep.res, rbytes) : ry;
  // per channel block j: this lane's pixel column summed over both rows and every tile, in fp32.  A Kahan-compensated
  // fold every 16 tiles was built (round 4) and measured: 4 % slower at 768^2 / 384^2 (register pressure
  // in the MFMA loop) for no measurable gain -- batch variance at mean / std = 42 on the 768^2 bs32 layer within
  // 3.7e-5 compensated vs 4.5e-5 plain, both set by the fp32 conv outputs themselves
  // (tests/test_gpu_conv_bench_shapes.py::test_halo_bn_statistics_large_mean_at_bench_shape)
  f32x16 s1[2], s2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[j][r] = s2[j][r] = 0.f;
  for (int u = u0, it = 0; u < u1; ++u, ++it) {
    __builtin_amdgcn_s_barrier();  // halo(u) landed for every wave; every wave is done with the other buffer
    const char* const hl = smem + halo::WBYTES + (it & 1) * halo::HBYTES;
    if (u + 1 < u1) issue_halo(u + 1, smem + halo::WBYTES + ((it + 1) & 1) * halo::HBYTES);
    int b, oh0, ow0;
    tile_pos(u, b, oh0, ow0);
    unsigned mrow[2], prow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long pix = ((long)b * g.OH + oh0 + 2 * wid + i) * g.OW + ow0 + px;
      mrow[i] = (unsigned)(pix * g.yps);
      prow[i] = (unsigned)(pix * pstride);
    }
    // accumulate (data-grad): this lane's eight 16-B output vectors; inference epilogue with a residual: the residual
    // vectors at the same pixels / channels -- both loaded before the MFMAs
    u4 prev[2][2][2];
    if (pre) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int gq = 0; gq < 2; ++gq)
            prev[i][j][gq] = __builtin_amdgcn_raw_buffer_load_b128(
                rp, (prow[i] + (unsigned)(32 * j + 16 * gq + 8 * hf)) * 2u, 0, 0);
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // 18 half-taps (tap, k steps 2 hs .. 2 hs + 1), software-pipelined: the 8 fragment reads of half-tap h + 1 are
    // issued before the 8 MFMAs of half-tap h (one wave per SIMD: nothing else hides the LDS latency)
    bf16x8 fa[2][2][2], fb[2][2][2];  // [buffer][k step][row i / channel block j]
    auto load_half = [&](int h, bf16x8 (&a)[2][2], bf16x8 (&bw)[2][2]) {
      const int tap = h >> 1, kh = tap / 3, kw = tap % 3;
      const int dh = DG ? 1 - kh : kh - 1, dw = DG ? 1 - kw : kw - 1;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int c = 2 * (2 * (h & 1) + ss) + hf;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int p = (2 * wid + i + 1 + dh) * halo::HW + px + 1 + dw;
          a[ss][i] = *reinterpret_cast<const bf16x8*>(hl + p * 128 + ((c ^ hsw(p)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = 32 * j + px;
          bw[ss][j] = *reinterpret_cast<const bf16x8*>(wl + (tap * 64 + n) * 128 + ((c ^ hsw(n)) << 4));
        }
      }
    };
    load_half(0, fa[0], fb[0]);
#pragma unroll
    for (int h = 0; h < 18; ++h) {
      if (h + 1 < 18) load_half(h + 1, fa[(h + 1) & 1], fb[(h + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[h & 1][ss][j], fa[h & 1][ss][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: acc[i][j][r] = Y[pixel (row 2 wid + i, column px)][channel 32 j + (r & 3) + 8 (r >> 2) + 4 hf]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          v[r] = acc[i][j][r];
          if (stats) {
            s1[j][r] += v[r];
            s2[j][r] += v[r] * v[r];
          }
        }
#pragma unroll
        for (int gp = 0; gp < 4; gp += 2) {  // channel groups (gp, gp + 1) -> 8 consecutive channels per lane
          const unsigned a0 = pk2_bf16(v[4 * gp], v[4 * gp + 1]), a1 = pk2_bf16(v[4 * gp + 2], v[4 * gp + 3]);
          const unsigned b0 = pk2_bf16(v[4 * gp + 4], v[4 * gp + 5]), b1 = pk2_bf16(v[4 * gp + 6], v[4 * gp + 7]);
          const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
          u4 o = {r0[0], r1[0], r0[1], r1[1]};
          if (accumulate) o = add_bf16x8(o, prev[i][j][gp >> 1]);
          if (EP) {  // eval BN scale / shift + act (+ residual) on the bf16-rounded conv output (epi_store)
            const int n = 32 * j + 8 * gp + 8 * hf;
            float f[8], r8[8], sc[8], sh[8];
            unpack<bf16>(make_uint4(o[0], o[1], o[2], o[3]), f);
            if (resid) unpack<bf16>(make_uint4(prev[i][j][gp >> 1][0], prev[i][j][gp >> 1][1], prev[i][j][gp >> 1][2],
                                               prev[i][j][gp >> 1][3]), r8);
            const float4* cf = reinterpret_cast<const float4*>(smem + halo::LDS) + n / 4;  // [scale 64 | shift 64]
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float4 a = cf[h], b = cf[16 + h];
              sc[4 * h] = a.x; sc[4 * h + 1] = a.y; sc[4 * h + 2] = a.z; sc[4 * h + 3] = a.w;
              sh[4 * h] = b.x; sh[4 * h + 1] = b.y; sh[4 * h + 2] = b.z; sh[4 * h + 3] = b.w;
            }
            epi_apply8(ep.act, f, sc, sh, resid ? r8 : nullptr);
            const uint4 q4 = pack<bf16>(f);
            o = u4{q4.x, q4.y, q4.z, q4.w};
          }
          const unsigned off = (mrow[i] + (unsigned)(32 * j + 8 * gp + 8 * hf)) * 2u;
          __builtin_amdgcn_raw_buffer_store_b128(o, ry, off, 0, 0);
        }
      }
    if (u + 1 < u1) vm_wait<8>();  // the next halo landed (only this tile's 8 stores are younger)
  }
  if (!stats) return;
  // ---- one BN partial row per wave: sum the 32 pixel lanes of each channel in a fixed order (through LDS)
  vm_wait<0>();
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [2][4 waves][64 channels][33]
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ch = 32 * j + (r & 3) + 8 * (r >> 2) + 4 * hf;
      red[(wid * 64 + ch) * 33 + px] = s1[j][r];
      red[((halo::NW + wid) * 64 + ch) * 33 + px] = s2[j][r];
    }
  __syncthreads();
  float t1 = 0.f, t2 = 0.f;
  for (int q = 0; q < 32; ++q) {
    t1 += red[(wid * 64 + lane) * 33 + q];
    t2 += red[((halo::NW + wid) * 64 + lane) * 33 + q];
  }
  const long row = (long)blockIdx.x * halo::NW + wid;
  psum[row * 64 + lane] = t1;
  psq[row * 64 + lane] = t2;
}
}  // namespace v3

// ---------------------------------------------------------------- host dispatch
Geom make_geom(int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps) {
  Geom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.KH = KH; g.KW = KW; g.S = S; g.P = P;
  g.OH = OH; g.OW = OW; g.xps = xps; g.yps = yps;
  g.oihw = 0; g.zeroed = 0;
  g.dws = nullptr; g.dws_slab = 0; g.plan = nullptr;
  return g;
}

// dw[i] += sum over splits s = 0, 1, ... of ws[s][i], in that order (the deterministic split-K reduction)
__global__ void wgrad_split_reduce(const float* __restrict__ ws, float* __restrict__ dw, long slab, int splits) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < slab; i += (long)gridDim.x * blockDim.x) {
    float acc = ws[i];
    for (int k = 1; k < splits; ++k) acc += ws[(long)k * slab + i];
    dw[i] += acc;
  }
}

// Called by every weight-grad launcher once its split count is known.  Returns true when the caller must return
// right away (plan query).  Deterministic mode with one split keeps the single atomic per element (exact: it adds
// to a zero or to an earlier stream-ordered launch's value), so g.dws is dropped.
inline bool wgrad_begin(Geom& g, int splits) {
  if (g.plan != nullptr) {
    *g.plan = splits;
    return true;
  }
  if (g.dws != nullptr && splits <= 1) g.dws = nullptr;
  return false;
}
inline void wgrad_end(const Geom& g, float* dw, int splits, hipStream_t st) {
  if (g.dws != nullptr)
    wgrad_split_reduce<<<grid_cap(ceil_div(g.dws_slab, 256), 2048), 256, 0, st>>>(g.dws, dw, g.dws_slab, splits);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// tile choice shared by launch and partial-row query
// v2 (register-staged) tiles.  The BN partial-row numbering of every training forward (dmy_conv_fwd_partial_rows:
// one row per 64 output rows when 128-row tiles are taken, per 32 otherwise) follows big_tile_rows, so a launch that
// writes partials keeps that rule.  Launches without partials (inference, data-grads) take 128 x 128 tiles only when
// that grid still fills the chip: the batch-1 96^2 1x1 layers (9216 rows) run 64 x 64 tiles, 4x the blocks
// (profiles/r06/bigt_ab.log, graph-replayed: 256 -> 256 12.0 -> 8.0 us, 1024 -> 256 22.1 -> 16.9 us; batch-1 detect
// p50 DMA-1536 4.41 -> 4.30 ms, yolov5s 0.629 -> 0.608 ms)
inline bool big_tile_rows(long M, int N) { return M >= 4096 && N > 64; }
inline bool big_tile(long M, int N) { return big_tile_rows(M, N) && ceil_div(M, 128) * ceil_div(N, 128) >= 256; }

template <typename T, int BM, int BN>
int launch_fwd(const T* x, const T* w, const float* b, T* y, float* ps, float* pq, const Geom& g, hipStream_t st,
               const Epi& ep = Epi{}) {
  constexpr int VW = Traits<T>::VW;
  const long M = (long)g.N * g.OH * g.OW;
  const int gm = ceil_div(M, BM), gn = ceil_div(g.K, BN);
  const bool p1 = g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0;
  const bool vec = g.C % VW == 0 && g.xps % VW == 0 && aligned16(x);
  const unsigned grid = (unsigned)gm * gn;
  if (vec && p1) conv_fwd_kernel<T, BM, BN, true, true><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g, gm, gn, ep);
  else if (vec) conv_fwd_kernel<T, BM, BN, true, false><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g, gm, gn, ep);
  else if (p1) conv_fwd_kernel<T, BM, BN, false, true><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g, gm, gn, ep);
  else conv_fwd_kernel<T, BM, BN, false, false><<<grid, NT, 0, st>>>(x, w, b, y, ps, pq, g, gm, gn, ep);
  return (int)hipGetLastError();
}

template <typename T, int BM, int BN>
int launch_dgrad(const T* dy, const T* wt, T* dx, int acc, const Geom& g, hipStream_t st) {
  constexpr int VW = Traits<T>::VW;
  const bool p1 = g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0;
  const bool s2 = g.S == 2;
  const long M = s2 ? (long)g.N * ((g.H + 1) / 2) * ((g.W + 1) / 2) : (long)g.N * g.H * g.W;
  const int gm = ceil_div(M, BM), gn = ceil_div(g.C, BN);
  const bool vec = g.K % VW == 0 && g.yps % VW == 0 && aligned16(dy);
  const dim3 grid((unsigned)gm * gn, s2 ? 4 : 1);
  if (s2) {
    if (vec) conv_dgrad_kernel<T, BM, BN, true, false, true><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
    else conv_dgrad_kernel<T, BM, BN, false, false, true><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
  } else if (vec && p1) conv_dgrad_kernel<T, BM, BN, true, true, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
  else if (vec) conv_dgrad_kernel<T, BM, BN, true, false, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
  else if (p1) conv_dgrad_kernel<T, BM, BN, false, true, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
  else conv_dgrad_kernel<T, BM, BN, false, false, false><<<grid, NT, 0, st>>>(dy, wt, dx, acc, g, gm, gn);
  return (int)hipGetLastError();
}

template <typename T, int BM, int BN>
int launch_wgrad(const T* x, const T* dy, float* dw, Geom g, hipStream_t st) {
  constexpr int VW = Traits<T>::VW;
  constexpr int BK = Cfg<T>::BK;
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
  const int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  const dim3 grid((unsigned)gm * gn, splits);
  if (wgrad_begin(g, splits)) return 0;
  const bool va = g.K % VW == 0 && g.yps % VW == 0 && aligned16(dy);
  const bool vb = g.C % VW == 0 && g.xps % VW == 0 && aligned16(x);
  if (!g.zeroed) (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * Ntot, st);
  if (va && vb) conv_wgrad_kernel<T, BM, BN, true, true><<<grid, NT, 0, st>>>(x, dy, dw, per, g, gm, gn);
  else if (va) conv_wgrad_kernel<T, BM, BN, true, false><<<grid, NT, 0, st>>>(x, dy, dw, per, g, gm, gn);
  else if (vb) conv_wgrad_kernel<T, BM, BN, false, true><<<grid, NT, 0, st>>>(x, dy, dw, per, g, gm, gn);
  else conv_wgrad_kernel<T, BM, BN, false, false><<<grid, NT, 0, st>>>(x, dy, dw, per, g, gm, gn);
  wgrad_end(g, dw, splits, st);
  return (int)hipGetLastError();
}

// v3 (LDS-DMA) kernels apply to bf16 with 16-B vectors everywhere and enough rows to fill the chip
inline bool v3_ok(int C, long xps, int K, long yps, const void* x, const void* w, const void* y, long M) {
  return C % 8 == 0 && xps % 8 == 0 && K % 8 == 0 && yps % 8 == 0 && aligned16(x) && aligned16(w) && aligned16(y) &&
         M >= 16384 && K >= 32;
}

// gv = GEMM view (rows N*OH*OW, columns K, gather tensor H x W x C with stride xps); BN partials need
// 64-row wave rows, numbered 4 per 256-row tile (= dmy_conv_fwd_partial_rows when K > 64)
// Routing of the bf16 training / inference convolutions.  Round 6 removed the measured-and-rejected variants and their
// environment switches (DESIGN.md §3.1 keeps their numbers): the persistent 1x1 GEMM (conv_p1_persist: 15-40 % slower,
// profiles/r02/ab_p1_persist.log), the small-M GEMM (conv_sk, profiles/r03/det_sk_ab.log), small-grid LDS-DMA tiles
// (DMY_V3_FILL, profiles/r02/ab_fill.log), the persistent stride-2 class kernel (conv_s2p, gpurun_out/r5/ab_s2p.log),
// the wide 256 x 256 weight-grad tile (conv_wgrad_w, profiles/r04/wgrad_wide_ab.log), the two-plane 128-row tap
// weight-grad (profiles/r05/wgrad_tap_np128_ab.log), the in-launch split-K combine (profiles/r03/det_splitk_fused_ab.log),
// the half-tile pipeline on 3x3 tiles (gpurun_out/r5/ab_w8p.log), the streaming GEMM's 1x1 eval epilogue
// (profiles/r04/det_p1s_ep_ab.log) and the fragments-first orders of the halo / tap / persistent 1x1 loops
// (profiles/r04/halo_tap_ff_ab.log, p1p_ff_ab.log).  What is left has one path per shape class.
inline int num_cus();
// wide 256 x 256 tiles (v3::conv_fwd_w) for GEMM views with >= 256 columns and at least one block per CU: +9..21 % on
// every DMA-YOLO / yolov5s shape with >= 256 columns, 0.66-0.76x at 128 columns or below one block per CU
// (profiles/r02/ab_wide.log).  The 1x1 views among them run the half-tile pipeline (v3::conv_fwd_8p; round 5,
// gpurun_out/r5/ab_w8p.log: C1024 -> K1024 @48^2 bs32 fwd 200 -> 175 us, dgrad 186 -> 161, C4096 -> K1024 fwd 592 ->
// 526; every 3x3 shape within +-1.5 %, so those keep conv_fwd_w)
constexpr int kWideMinCols = 256;
// tall 512 x 128 tiles (v3::conv_fwd_w) for k > 1 GEMM views with 65..128 columns and >= 4 blocks per CU: +4..8 % on
// the 128-channel 3x3 layers of DMA-YOLO / config 5 (profiles/r02/ab_tall.log)
// 1x1 streaming GEMM (v3::conv_p1s) for the output-heavy stride-1 1x1 forwards (>= 2x as many columns as reduction):
// 1.05-1.38x the LDS-DMA tiles there (profiles/r02/ab_p1s.log); on the other 1x1 shapes those tiles already stream at
// 4.5-6 TB/s and stay faster
inline bool p1s_ok(const Geom& gv, const void* x, const void* w, const void* y) {
  if (gv.KH != 1 || gv.KW != 1 || gv.S != 1 || gv.P != 0) return false;
  if (gv.C != 64 && gv.C != 128 && gv.C != 256) return false;
  if (gv.K % 32 != 0 || gv.xps % 8 != 0 || gv.yps % 8 != 0 || !aligned16(x) || !aligned16(w) || !aligned16(y))
    return false;
  return 2.0 * ((double)gv.N * gv.OH * gv.OW * gv.xps) < (double)v3::kBufOob;
}
// threads per block of the training stem: 512 = 64-column passes that write whole 128-B output lines per pixel, for
// >= 64 output channels; 768 = 32-column passes otherwise.  Cold-cache (profiles/r04/stem_ab.log): DMA-1536 stem (64 ch
// @768^2 bs32) 1483 -> 1185 us, config 5 (64 @960^2 bs8) 585 -> 434 us, but yolov5s (32 ch @320^2 bs64: one 32-column
// pass either way) 213 -> 242 us with 512, so it keeps 768
inline int stem_nth(int K) { return K >= 64 ? 512 : 768; }
// the k3 s1 p1 view of the space-to-depth stem (16 input channels) on the streaming GEMM with its 3x3 gather
inline bool stem_s_ok(const Geom& gv, const void* x, const void* w, const void* y) {
  if (gv.C != 16 || gv.KH != 3 || gv.KW != 3 || gv.S != 1 || gv.P != 1 || gv.OH != gv.H || gv.OW != gv.W) return false;
  if (gv.K % 32 != 0 || gv.K > 256 || gv.xps % 8 != 0 || gv.yps % 8 != 0 || !aligned16(x) || !aligned16(w) || !aligned16(y))
    return false;
  return 2.0 * ((double)gv.N * gv.H * gv.W * gv.xps) < (double)v3::kBufOob && (long)gv.N * gv.H * gv.W < (1L << 31);
}
// column groups of a streaming-GEMM launch (conv_p1s, 512 threads, 160 KiB of LDS): each group holds ng columns of W
// in LDS and streams every X row again
inline int p1s_groups(int KD, int NC) {
  const int ng = ((160 * 1024 - 512 / 64 * 256) / ((KD + 8) * 2)) / 32 * 32;
  return ceil_div(NC, ng);
}
template <int KD, int NTH, bool G3 = false, bool DG = false>
int launch_p1s_kd(const bf16* x, const bf16* w, const float* b, bf16* y, float* ps, float* pq, int acc,
                  const Geom& gv, hipStream_t st, int lds_kib, int bpc) {
  constexpr int pitch_b = (KD + 8) * 2, scratch = NTH / 64 * 256;
  const long M = (long)gv.N * gv.OH * gv.OW;
  int ng = ((lds_kib * 1024 - scratch) / pitch_b) / 32 * 32;
  if (ng < 32) ng = 32;
  const int G = ceil_div(gv.K, ng);
  ng = ceil_div(ceil_div(gv.K, G), 32) * 32;
  const int lds = ng * pitch_b + scratch;
  static bool raised = false;
  if (!raised) {
    (void)hipFuncSetAttribute((const void*)v3::conv_p1s<KD, NTH, G3, DG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    raised = true;
  }
  const int ntiles = ceil_div(M, 64);
  int nbx = ceil_div(ceil_div((long)num_cus() * bpc, G), 8) * 8;
  const int maxb = ceil_div(ntiles, NTH / 64);
  if (nbx > maxb) nbx = maxb;
  const dim3 grid((unsigned)nbx, (unsigned)G);
  const double xb = 2.0 * ((double)gv.N * gv.H * gv.W * gv.xps);
  v3::conv_p1s<KD, NTH, G3, DG><<<grid, NTH, lds, st>>>(x, w, b, y, ps, pq, acc, M, gv.K, ng, gv.xps, gv.yps, (unsigned)xb,
                                               ntiles, gv.KH * gv.KW * gv.C, gv.H, gv.W);
  return (int)hipGetLastError();
}
// training forwards: 512 threads, the whole 160 KiB of LDS for the W column group, one block per CU
template <bool DG = false>
inline int launch_p1s(const bf16* x, const bf16* w, const float* b, bf16* y, float* ps, float* pq, int acc,
                      const Geom& gv, hipStream_t st) {
  if (gv.C == 64) return launch_p1s_kd<64, 512, false, DG>(x, w, b, y, ps, pq, acc, gv, st, 160, 1);
  if (gv.C == 128) return launch_p1s_kd<128, 512, false, DG>(x, w, b, y, ps, pq, acc, gv, st, 160, 1);
  return launch_p1s_kd<256, 512, false, DG>(x, w, b, y, ps, pq, acc, gv, st, 160, 1);
}

// persistent 1x1 GEMM with the register epilogue (v3::conv_p1p): 256 x 128 tiles (3 stages; 256 x 64 for <= 64
// columns) for GEMM views with <= 256 columns (cold-cache A/B on the DMA-YOLO 1x1 shapes, profiles/r03/ab_p1p.log: 256 ->
// 256 @96^2 fwd 118.7 -> 94.8 us, 128 -> 128 @384^2 636 -> 492 us, 4..23 % on every <= 256-column view; 7..15 % SLOWER on
// the 512..1280-column views, where the 256 x 256 wide tile reads each input row once).  Training forwards with one
// column tile keep per-lane BN partials (LANE).  Not for the inference epilogue, the fused producer-BN reduce or an
// accumulating data-grad.
constexpr int kP1pMaxCols = 256;
// conv_p1p's persistent grid: blocks per CU from the LDS footprint, capped at the tile count, a multiple of 8 (XCDs)
// BN partial rows written by the last training forward launched on this host thread (dmy_conv_fwd_last_rows).  The
// persistent kernels (halo, LANE conv_p1p) write one row per wave of their grid; every other kernel writes
// dmy_conv_fwd_partial_rows(M, K).  The host allocates dmy_conv_fwd_bound_rows rows and reads the count back, so no
// second copy of the routing decides it; a persistent launch whose rows would pass the bound declines.
thread_local long t_prow_last = 0;
inline long prow_persist_cap() { return 64L * num_cus(); }
inline int p1p_grid(int ntiles, int lds) {
  const int bpc = (160 * 1024) / lds;
  int G = num_cus() * (bpc < 1 ? 1 : bpc);
  return G > ntiles ? ntiles : G / 8 * 8;
}
// the tile configuration launch_p1p picks: f(BM, BN, NS, WTR) as integral constants; -1 when it declines
template <bool DG, class F>
int p1p_plan(const Geom& gv, int acc, const Epi& ep, F&& f) {
  const long M = (long)gv.N * gv.OH * gv.OW;
  const int nk = gv.C / v3::BK;
  const double yb = 2.0 * ((double)(M - 1) * gv.yps + gv.K);
  const double rb = ep.res != nullptr ? 2.0 * ((double)(M - 1) * ep.rps + gv.K) : 0.0;
  if (acc || gv.K % 8 != 0 || yb >= (double)v3::kBufOob || rb >= (double)v3::kBufOob || nk < 1 ||
      (ep.res != nullptr && (ep.rps % 8 != 0 || !aligned16(ep.res))) || gv.K > kP1pMaxCols)
    return -1;
  // 129..256 columns over a >= 1024-deep reduction: the 256 x 256 half-tile pipeline reads each input row once and
  // keeps its 16+ K steps in flight (profiles/r06/route_ab.log, cold caches: 1024 -> 256 @96^2 fwd 224 -> 201 us,
  // 1280 -> 256 fwd 288 -> 245, data-grad 256 <- 1024 208 -> 184; the 256-deep 256 -> 256 stays here, 86 vs 102 us)
  if (gv.K > 128 && gv.C >= 1024) return -1;
  using std::integral_constant;
#define P1P_CFG(BM, BN, NS, WTR) \
  return f(integral_constant<int, BM>{}, integral_constant<int, BN>{}, integral_constant<int, NS>{}, integral_constant<int, WTR>{})
  if (gv.K > 64) {
    if (nk >= 2) P1P_CFG(256, 128, 3, 64);
    P1P_CFG(256, 128, 2, 64);
  }
  P1P_CFG(256, 64, 2, 64);
#undef P1P_CFG
}
// BN partial rows of a LANE launch (one per wave row of the persistent grid), or 0 when launch_p1p would not use LANE
inline long p1p_lane_rows(const Geom& gv) {
  const long M = (long)gv.N * gv.OH * gv.OW;
  return p1p_plan<false>(gv, 0, Epi{}, [&](auto bm, auto bn, auto ns, auto wtr) -> int {
    using PP = v3::P1P<decltype(bm)::value, decltype(bn)::value, decltype(ns)::value, decltype(wtr)::value>;
    const int gm = ceil_div(M, decltype(bm)::value), gn = ceil_div(gv.K, decltype(bn)::value);
    const long r = gn == 1 ? (long)p1p_grid(gm * gn, PP::LDS) * PP::C3_::WM : 0;
    return r <= prow_persist_cap() ? (int)r : 0;
  });
}
template <bool DG>
int launch_p1p(const bf16* x, const bf16* w, const float* b, bf16* y, float* ps, float* pq, int acc, const Geom& gv,
               hipStream_t st, unsigned xbytes, unsigned wbytes, const Epi& ep, bool lane) {
  const long M = (long)gv.N * gv.OH * gv.OW;
  const double yb = 2.0 * ((double)(M - 1) * gv.yps + gv.K);
  const double rb = ep.res != nullptr ? 2.0 * ((double)(M - 1) * ep.rps + gv.K) : 0.0;
  return p1p_plan<DG>(gv, acc, ep, [&](auto bm, auto bn, auto ns, auto wtr) -> int {
    constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value, NS = decltype(ns)::value, WTR = decltype(wtr)::value;
    using PP = v3::P1P<BM, BN, NS, WTR>;
    const int gm = ceil_div(M, BM), gn = ceil_div(gv.K, BN), ntiles = gm * gn;
    const int G = p1p_grid(ntiles, PP::LDS);
    if constexpr (!DG) {
      if (lane) {  // one BN partial row per wave (plan_v3: p1p_lane_rows)
        v3::conv_p1p<BM, BN, NS, WTR, false, true><<<(unsigned)G, PP::NTH, 0, st>>>(
            x, w, b, y, ps, pq, acc, gv, gm, gn, xbytes, wbytes, (unsigned)yb, G * PP::C3_::WM, ep, (unsigned)rb);
        return (int)hipGetLastError();
      }
    }
    const int nprow = ps != nullptr ? dmy_conv_fwd_partial_rows(M, gv.K) : 0;
    v3::conv_p1p<BM, BN, NS, WTR, DG><<<(unsigned)G, PP::NTH, 0, st>>>(x, w, b, y, ps, pq, acc, gv, gm, gn, xbytes,
                                                                      wbytes, (unsigned)yb, nprow, ep, (unsigned)rb);
    return (int)hipGetLastError();
  });
}

// 3x3 stride-1 64 -> 64-channel layers on the persistent halo kernel (v3::conv3_halo64).  g = the GEMM view (gathered H x W x C with pixel stride xps, output OH x OW x K with stride yps); whole 8 x 32
// output tiles only, at least one tile per CU, no bias / inference epilogue (the callers check those).
inline long halo_units(const Geom& g) { return (long)g.N * (g.H / v3::halo::TH) * (g.W / v3::halo::TW); }
inline bool halo_ok(const Geom& g, const void* x, const void* w, const void* y) {
  if (g.KH != 3 || g.KW != 3 || g.S != 1 || g.P != 1 || g.C != 64 || g.K != 64 ||
      g.OH != g.H || g.OW != g.W || g.H % v3::halo::TH != 0 || g.W % v3::halo::TW != 0 || g.xps % 8 != 0 ||
      g.yps % 8 != 0 || !aligned16(x) || !aligned16(w) || !aligned16(y))
    return false;
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), yb = 2.0 * ((double)g.N * g.OH * g.OW * g.yps);
  return xb < (double)v3::kBufOob && yb < (double)v3::kBufOob && halo_units(g) >= num_cus();
}
// persistent grid: per = tiles per block, every block gets at least one (so every BN partial row is written)
inline int halo_blocks(const Geom& g, int* per_out = nullptr) {
  const long nt = halo_units(g);
  const int per = ceil_div(nt, num_cus());
  if (per_out) *per_out = per;
  return ceil_div(nt, per);
}
// BN partial rows the halo kernel writes: one per wave
inline int halo_rows(const Geom& g) { return v3::halo::NW * halo_blocks(g); }
template <bool DG>
int launch_halo(const bf16* x, const bf16* w, bf16* y, float* ps, float* pq, const Geom& g, hipStream_t st,
                int acc = 0, const Epi& ep = Epi{}) {
  const int thn = g.H / v3::halo::TH, twn = g.W / v3::halo::TW, nt = (int)halo_units(g);
  int per = 1;
  const int G = halo_blocks(g, &per);
  const unsigned xb = (unsigned)(2.0 * ((double)g.N * g.H * g.W * g.xps));
  const unsigned yb = (unsigned)(2.0 * ((double)g.N * g.OH * g.OW * g.yps));
  const unsigned rb = ep.res != nullptr ? (unsigned)(2.0 * ((double)g.N * g.OH * g.OW * ep.rps)) : 0u;
  if (!DG && ep.on)  // inference epilogue: its own instantiation, so the training kernel's registers are untouched
    v3::conv3_halo64<false, true><<<(unsigned)G, 64 * v3::halo::NW, 0, st>>>(x, w, y, ps, pq, g, twn, thn, nt, per,
                                                                           xb, 2u * 64 * 576, yb, acc, ep, rb);
  else
    v3::conv3_halo64<DG><<<(unsigned)G, 64 * v3::halo::NW, 0, st>>>(x, w, y, ps, pq, g, twn, thn, nt, per, xb,
                                                                    2u * 64 * 576, yb, acc, ep, rb);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- routing plans
// One function decides which kernel a bf16 implicit-GEMM launch takes; the launch executes that plan and
// dmy_conv_fwd_bn_rows reads the BN partial-row count off the same plan, so the two cannot drift.
enum class Kern { HALO, SPLITK, P1S, STEM, P1P, PIPE8, WIDE, WIDE288, TALL, V3, V2 };
struct Plan {
  Kern k;
  bool buf;   // buffer-descriptor loader (C % 64 == 0, byte offsets < 4 GiB)
  bool lane;  // P1P: per-lane BN partials, one row per wave of the persistent grid
  long rows;  // BN partial rows the launch writes (when it writes them)
};
// the v3 family for GEMM view gv (forward, or data-grad when DG)
template <bool DG>
Plan plan_v3(const Geom& gv, const void* x, const void* w, const void* y, int acc, const Epi& ep) {
  const long M = (long)gv.N * gv.OH * gv.OW;
  const bool p1 = gv.KH == 1 && gv.KW == 1 && gv.S == 1 && gv.P == 0;
  Plan pl{Kern::V3, false, false, dmy_conv_fwd_partial_rows(M, gv.K)};
  // output-heavy 1x1 data-grads (dx channels >= 2 x dy channels) on the streaming GEMM too, when W fits <= 4 column
  // groups (profiles/r06/p1sdg_ab.log, cold caches: 512 <- 128 @192^2 bs32 465 -> 355 us, 1024 <- 256 @96^2 269 -> 230;
  // 1280 <- 256 (5 groups, X streamed 5 times) 318 -> 450, kept on the LDS-DMA tiles)
  if (DG && !ep.on && p1s_ok(gv, x, w, y) && gv.K >= 2 * gv.C && p1s_groups(gv.C, gv.K) <= 4)
    return pl.k = Kern::P1S, pl;
  if (!DG && !ep.on) {
    if (p1s_ok(gv, x, w, y) && gv.K >= 2 * gv.C) return pl.k = Kern::P1S, pl;  // output-heavy 1x1: streaming GEMM
    if (stem_s_ok(gv, x, w, y)) return pl.k = Kern::STEM, pl;  // the 16-channel 3x3 stem view (p1s, G3 gather)
  }
  const double xb = 2.0 * ((double)gv.N * gv.H * gv.W * gv.xps), wb = 2.0 * gv.K * gv.KH * gv.KW * gv.C;
  pl.buf = gv.C % 64 == 0 && xb < (double)v3::kBufOob && wb < (double)v3::kBufOob;
  if (p1 && pl.buf && !ep.on && p1p_plan<DG>(gv, acc, ep, [](auto, auto, auto, auto) { return 0; }) >= 0) {
    pl.k = Kern::P1P;  // persistent 1x1 with the register epilogue
    if (!DG) {
      const long r = p1p_lane_rows(gv);
      if (r > 0) pl.lane = true, pl.rows = r;
    }
    return pl;
  }
  if (pl.buf && gv.K >= kWideMinCols && (long)ceil_div(M, 256) * ceil_div(gv.K, 256) >= num_cus()) {
    // 1x1 views: the half-tile pipeline (conv_fwd_8p); an inference launch with <= 2 K steps (<= 128 input channels)
    // keeps the 256 x 128 tiles, whose grid is twice as wide (batch-1 128 -> 512 @192^2 37.6 -> 31.7 us, detect p50
    // @1536 4.25 -> 4.19 ms, profiles/r06/ep8_ab.log)
    if (p1 && ep.on && gv.C <= 128) return pl;
    if (p1) return pl.k = Kern::PIPE8, pl;
    // k > 1: 256- or 288-row tiles, whichever grid ends in fewer row-weighted rounds of the chip.  A block per CU at a
    // time, so a grid of 4.5 rounds (3x3 256 @96^2 bs32: 1152 tiles of 256 rows) costs 5 and idles half the chip for
    // the last; 288 = 9 x 32 divides every DMA-YOLO @1536 / config-5 @1920 map (1536^2 and 1920^2 carry a factor 9):
    // 1024 tiles, 4 rounds of 288 rows = 1152 row-times against 1280.  (2.25 -> 2 rounds at 512 @48^2.)
    const long gn = ceil_div(gv.K, 256), NC = num_cus();
    const long t256 = ceil_div(ceil_div(M, 256) * gn, NC) * 256, t288 = ceil_div(ceil_div(M, 288) * gn, NC) * 288;
    if (t288 < t256) {
      pl.k = Kern::WIDE288;
      pl.rows = ceil_div(M, 288) * 2;  // one BN partial row per wave row (2) and row tile
      return pl;
    }
    return pl.k = Kern::WIDE, pl;
  }
  if (pl.buf && !p1 && gv.K > 64 && gv.K <= 128 && (long)ceil_div(M, 512) * ceil_div(gv.K, 128) >= 4L * num_cus())
    return pl.k = Kern::TALL, pl;
  return pl;
}
template <bool DG>
int launch_v3(const bf16* x, const bf16* w, const float* b, bf16* y, float* ps, float* pq, int acc, const Geom& gv,
              hipStream_t st, const Epi& ep, const Plan& pl) {
  const long M = (long)gv.N * gv.OH * gv.OW;
  const bool p1 = gv.KH == 1 && gv.KW == 1 && gv.S == 1 && gv.P == 0;
  const double xb = 2.0 * ((double)gv.N * gv.H * gv.W * gv.xps), wb = 2.0 * gv.K * gv.KH * gv.KW * gv.C;
  const unsigned xbytes = pl.buf ? (unsigned)xb : 0u, wbytes = pl.buf ? (unsigned)wb : 0u;
#define W_GO(BM, BN)                                                                                                 \
  {                                                                                                                  \
    const int gm = ceil_div(M, BM), gn = ceil_div(gv.K, BN);                                                         \
    if (p1) v3::conv_fwd_w<BM, BN, true, DG><<<(unsigned)gm * gn, 512, 0, st>>>(x, w, b, y, ps, pq, acc, gv, gm, gn, \
                                                                              xbytes, wbytes, ep);                  \
    else v3::conv_fwd_w<BM, BN, false, DG><<<(unsigned)gm * gn, 512, 0, st>>>(x, w, b, y, ps, pq, acc, gv, gm, gn,   \
                                                                               xbytes, wbytes, ep);                 \
    return (int)hipGetLastError();                                                                                   \
  }
#define V3_GO(BM, BN, NS, BUF_)                                                                               \
  {                                                                                                           \
    const int gm = ceil_div(M, BM), gn = ceil_div(gv.K, BN);                                                  \
    if (p1)                                                                                                   \
      v3::conv_fwd_v3<BM, BN, NS, true, DG, BUF_><<<(unsigned)gm * gn, BM * BN / 64, 0, st>>>(                \
          x, w, b, y, ps, pq, acc, gv, gm, gn, xbytes, wbytes, v3::S2Cls{0, 0, 0, 0}, ep);                    \
    else                                                                                                      \
      v3::conv_fwd_v3<BM, BN, NS, false, DG, BUF_><<<(unsigned)gm * gn, BM * BN / 64, 0, st>>>(               \
          x, w, b, y, ps, pq, acc, gv, gm, gn, xbytes, wbytes, v3::S2Cls{0, 0, 0, 0}, ep);                    \
    return (int)hipGetLastError();                                                                            \
  }
  switch (pl.k) {
    case Kern::P1S: return launch_p1s<DG>(x, w, b, y, ps, pq, acc, gv, st);
    case Kern::STEM:
      return stem_nth(gv.K) == 512 ? launch_p1s_kd<160, 512, true>(x, w, b, y, ps, pq, acc, gv, st, 160, 1)
                                   : launch_p1s_kd<160, 768, true>(x, w, b, y, ps, pq, acc, gv, st, 160, 1);
    case Kern::P1P: return launch_p1p<DG>(x, w, b, y, ps, pq, acc, gv, st, xbytes, wbytes, ep, pl.lane);
    case Kern::PIPE8: {
      const int gm = ceil_div(M, 256), gn = ceil_div(gv.K, 256);
      v3::conv_fwd_8p<true, DG><<<(unsigned)gm * gn, 512, 0, st>>>(x, w, b, y, ps, pq, acc, gv, gm, gn, xbytes, wbytes, ep);
      return (int)hipGetLastError();
    }
    case Kern::WIDE: W_GO(256, 256)
    case Kern::WIDE288: W_GO(288, 256)
    case Kern::TALL: W_GO(512, 128)
    default: break;
  }
  if (gv.K > 64) {
    if (pl.buf) V3_GO(256, 128, 3, 1)
    V3_GO(256, 128, 3, 0)
  }
  if (pl.buf) V3_GO(256, 64, 2, 1)
  V3_GO(256, 64, 2, 0)
#undef W_GO
#undef V3_GO
}

// sum the split slabs in order, + bias, round to bf16, inference epilogue (or plain store)
__global__ void __launch_bounds__(256) splitk_epi_kernel(const float* __restrict__ ws, int splits, long M, int K,
                                                         const float* __restrict__ bias, bf16* __restrict__ y, long yps,
                                                         Epi ep) {
  const int CV = K / 8;
  const long total = M * CV;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const long m = v / CV;
    const int c = (int)(v - m * CV) * 8;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float4* src = reinterpret_cast<const float4*>(ws + ((long)sp * M + m) * K + c);
      const float4 a = src[0], b = src[1];
      f[0] += a.x; f[1] += a.y; f[2] += a.z; f[3] += a.w;
      f[4] += b.x; f[5] += b.y; f[6] += b.z; f[7] += b.w;
    }
    bf16 t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = __float2bfloat16(f[j] + (bias != nullptr ? bias[c + j] : 0.f));
    if (ep.on) epi_store<bf16, 8>(ep, t, y + m * yps + c, c, K, m, true);
    else *reinterpret_cast<uint4*>(y + m * yps + c) = *reinterpret_cast<const uint4*>(t);
  }
}

// split-K plan of a small-M bf16 forward (no BN partials): splits > 1 when the tile grid is under two blocks per CU
// and the buffer loader applies; 0 = not split
inline int splitk_plan(const Geom& g, const void* x, const void* w, const void* y, int& gm, int& gn, int& per) {
  const long M = (long)g.N * g.OH * g.OW;
  if (M >= 16384 || M == 0 || g.C % 64 != 0 || g.xps % 8 != 0 || g.K % 8 != 0 || g.yps % 8 != 0 || g.K < 32 ||
      !aligned16(x) || !aligned16(w) || !aligned16(y))
    return 0;
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), wb = 2.0 * g.K * g.KH * g.KW * g.C;
  if (xb >= (double)v3::kBufOob || wb >= (double)v3::kBufOob) return 0;
  // detect-path A/B (profiles/r02/det_splitk.log): target 2 blocks per CU, at least 2 K steps per split; 1x1 layers
  // stay unsplit (their fp32 slabs + the reduce pass cost more than the split gains; bs1 detect DMA-1536 6.68 -> 6.45
  // ms, yolov5s 1.035 -> 0.968 ms)
  constexpr int pct = 200, mink = 2;
  if (g.KH == 1 && g.KW == 1) return 0;
  const int BN = g.K > 64 ? 128 : 64;
  gm = (int)ceil_div(M, 128);
  gn = ceil_div(g.K, BN);
  const int nk = g.KH * g.KW * g.C / v3::BK, tiles = gm * gn;
  int splits = ceil_div((long)pct * num_cus() / 100, tiles);
  if (splits > nk / mink) splits = nk / mink;
  if (splits < 2) return 0;
  per = ceil_div(nk, splits);
  return ceil_div(nk, per);
}

inline long splitk_elems(const Geom& g, const void* x, const void* w, const void* y) {
  int gm, gn, per;
  const int sp = splitk_plan(g, x, w, y, gm, gn, per);
  return sp ? (long)sp * g.N * g.OH * g.OW * g.K : 0;
}

inline int launch_splitk(const bf16* x, const bf16* w, const float* b, bf16* y, const Geom& g, float* ws, hipStream_t st,
                         const Epi& ep) {
  int gm, gn, per;
  const int sp = splitk_plan(g, x, w, y, gm, gn, per);
  const long M = (long)g.N * g.OH * g.OW;
  const unsigned xb = (unsigned)(2.0 * ((double)g.N * g.H * g.W * g.xps)), wb = (unsigned)(2.0 * g.K * g.KH * g.KW * g.C);
  const bool p1 = g.KH == 1 && g.KW == 1 && g.S == 1 && g.P == 0;
  const dim3 grid((unsigned)gm * gn, (unsigned)sp);
  if (g.K > 64) {
    if (p1) v3::conv_fwd_split<128, 128, 2, true><<<grid, 256, 0, st>>>(x, w, ws, g, gm, gn, per, xb, wb);
    else v3::conv_fwd_split<128, 128, 2, false><<<grid, 256, 0, st>>>(x, w, ws, g, gm, gn, per, xb, wb);
  } else {
    if (p1) v3::conv_fwd_split<128, 64, 2, true><<<grid, 128, 0, st>>>(x, w, ws, g, gm, gn, per, xb, wb);
    else v3::conv_fwd_split<128, 64, 2, false><<<grid, 128, 0, st>>>(x, w, ws, g, gm, gn, per, xb, wb);
  }
  splitk_epi_kernel<<<grid_cap(ceil_div(M * (g.K / 8), 256), 4096), 256, 0, st>>>(ws, sp, M, g.K, b, y, g.yps, ep);
  return (int)hipGetLastError();
}

// the bf16 forward's plan: bn = the launch writes BN partials (training); ws_elems = the split-K workspace it has
Plan plan_fwd(const Geom& g, const void* x, const void* w, const float* b, const void* y, bool bn, const Epi& ep,
              long ws_elems) {
  const long M = (long)g.N * g.OH * g.OW;
  const bool res_ok = !ep.res || (ep.rps % 8 == 0 && aligned16(ep.res));
  if (b == nullptr && halo_ok(g, x, w, y) && (!ep.on || !bn) && halo_rows(g) <= prow_persist_cap() &&
      (!ep.on || ep.res == nullptr ||
       (res_ok && 2.0 * ((double)g.N * g.OH * g.OW * ep.rps) < (double)v3::kBufOob)))
    return Plan{Kern::HALO, true, false, halo_rows(g)};  // one BN partial row per wave
  if (ws_elems > 0 && !bn && res_ok) {
    const long need = splitk_elems(g, x, w, y);
    if (need > 0 && need <= ws_elems) return Plan{Kern::SPLITK, true, false, 0};
  }
  if (v3_ok(g.C, g.xps, g.K, g.yps, x, w, y, M) && res_ok) return plan_v3<false>(g, x, w, y, 0, ep);
  return Plan{Kern::V2, false, false, dmy_conv_fwd_partial_rows(M, g.K)};
}

template <typename T>
int conv_fwd_t(const void* x, const void* w, const float* b, void* y, float* ps, float* pq, const Geom& g, hipStream_t st,
               const Epi& ep = Epi{}, float* ws = nullptr, long ws_elems = 0) {
  const long M = (long)g.N * g.OH * g.OW;
  Plan pl{Kern::V2, false, false, dmy_conv_fwd_partial_rows(M, g.K)};
  if constexpr (sizeof(T) == 2) pl = plan_fwd(g, x, w, b, y, ps != nullptr, ep, ws != nullptr ? ws_elems : 0);
  if (ps != nullptr) t_prow_last = pl.rows;
  if constexpr (sizeof(T) == 2) {
    switch (pl.k) {
      case Kern::HALO: return launch_halo<false>((const bf16*)x, (const bf16*)w, (bf16*)y, ps, pq, g, st, 0, ep);
      case Kern::SPLITK: return launch_splitk((const bf16*)x, (const bf16*)w, b, (bf16*)y, g, ws, st, ep);
      case Kern::V2: break;
      default: return launch_v3<false>((const bf16*)x, (const bf16*)w, b, (bf16*)y, ps, pq, 0, g, st, ep, pl);
    }
  }
  if (ps != nullptr ? big_tile_rows(M, g.K) : big_tile(M, g.K))
    return launch_fwd<T, 128, 128>((const T*)x, (const T*)w, b, (T*)y, ps, pq, g, st, ep);
  return launch_fwd<T, 64, 64>((const T*)x, (const T*)w, b, (T*)y, ps, pq, g, st, ep);
}
// stride-2 data-grad on the v3 buffer loader: one launch per output-parity class (a, b), each a GEMM
// over the class's input pixels and only the taps of matching parity (FwdLdsB S2 mode)
inline bool dgrad_s2_v3_ok(const Geom& g, const void* dy, const void* wt, const void* dx) {
  if (g.S != 2 || g.K % 64 != 0 || g.KH < 2 || g.KW < 2) return false;
  const long Mmin = (long)g.N * (g.H / 2) * (g.W / 2);
  const double xb = 2.0 * ((double)g.N * g.OH * g.OW * g.yps), wb = 2.0 * g.C * g.KH * g.KW * g.K;
  return v3_ok(g.K, g.yps, g.C, g.xps, dy, wt, dx, Mmin) && xb < (double)v3::kBufOob && wb < (double)v3::kBufOob;
}
// the one-GEMM form (v3::conv_dgrad_q2 / _q2s) for 32 / 64 / 128 input channels, 3x3 stride 2 pad 1, a grid of >= one
// 256-row tile per CU.  32 channels, against the merged four-class launch (profiles/r06/q2s_ab.log): 32 <- 64 @320^2
// bs64 (yolov5s) 462 -> 290 us, @384^2 bs32 318 -> 198, @640^2 bs16 436 -> 262; yolov5s step 16.60 -> 16.42 ms.  128 channels, against the four 256 x 128 class launches (profiles/r06/q2h_ab.log): 128 <- 256 @384^2 bs32
// 1318 -> 1207 us, @80^2 bs64 127 -> 103, @480^2 bs8 545 -> 460
inline bool dgrad_q2_ok(const Geom& g) {
  if (g.C != 32 && g.C != 64 && g.C != 128) return false;
  return g.KH == 3 && g.KW == 3 && g.P == 1 && g.S == 2 && g.K % 64 == 0 &&
         g.OH == (g.H + 1) / 2 && g.OW == (g.W + 1) / 2 && g.xps % 8 == 0 &&
         ceil_div((long)g.N * g.OH * g.OW, 256) >= num_cus();
}
inline int launch_dgrad_s2_v3(const bf16* dy, const bf16* wt, bf16* dx, int acc, const Geom& g, hipStream_t st) {
  const unsigned xbytes = (unsigned)(2.0 * ((double)g.N * g.OH * g.OW * g.yps));
  const unsigned wbytes = (unsigned)(2.0 * g.C * g.KH * g.KW * g.K);
  if (dgrad_q2_ok(g)) {
    const Geom gq = make_geom(g.N, g.OH, g.OW, g.K, g.yps, 256, 2, 2, 1, 0, g.OH, g.OW, g.xps);
    const int gm = (int)ceil_div((long)g.N * g.OH * g.OW, 256);
    if (g.C == 32) {
      const Geom gs = make_geom(g.N, g.OH, g.OW, g.K, g.yps, 128, 2, 2, 1, 0, g.OH, g.OW, g.xps);
      v3::conv_dgrad_q2s<<<(unsigned)gm, 512, 0, st>>>(dy, wt, dx, acc, gs, gm, xbytes, wbytes, v3::S2Cls{0, 0, g.H, g.W});
    } else if (g.C == 64)
      v3::conv_dgrad_q2<64><<<(unsigned)gm, 512, 0, st>>>(dy, wt, dx, acc, gq, gm, xbytes, wbytes, v3::S2Cls{0, 0, g.H, g.W});
    else
      v3::conv_dgrad_q2<128><<<(unsigned)(2 * gm), 512, 0, st>>>(dy, wt, dx, acc, gq, gm, xbytes, wbytes,
                                                                 v3::S2Cls{0, 0, g.H, g.W});
    return (int)hipGetLastError();
  }
  // one launch for the four classes of <= 64-channel data-grads, one per class above.  Measured
  // (profiles/r02/ab_s2_merge.log): +4..14 % at 32 / 64 channels, 16-33 % slower on the 1-block-per-CU 256 x 128 tiles
  // of the 128 / 256-channel layers, where the per-class launches stay.  The persistent class kernel (conv_s2p, round 5)
  // was slower on every DMA-1536 shape (gpurun_out/r5/ab_s2p.log) and is gone.
  if (g.C <= 64) {
    const long Mmax = (long)g.N * ((g.H + 1) / 2) * ((g.W + 1) / 2);  // class (0, 0) has the most rows
    const int gmax = ceil_div(Mmax, 256), gn = ceil_div(g.C, 64);
    v3::conv_dgrad_s2_v3<256, 64, 2><<<(unsigned)(4 * gmax * gn), 256, 0, st>>>(dy, wt, dx, acc, g, gmax, gn, xbytes,
                                                                              wbytes);
    return (int)hipGetLastError();
  }
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      const int H2 = (g.H - a + 1) / 2, W2 = (g.W - b + 1) / 2;
      if (H2 <= 0 || W2 <= 0) continue;
      // GEMM view: gather dy (OH x OW x K, stride yps), rows = the class's (N, H2, W2), columns = C
      const Geom gv = make_geom(g.N, g.OH, g.OW, g.K, g.yps, g.C, g.KH, g.KW, 2, g.P, H2, W2, g.xps);
      const long M = (long)g.N * H2 * W2;
      const v3::S2Cls cls{a, b, g.H, g.W};
      // >= 256 input channels: the class on the wide tile, 256 or 288 rows (profiles/r06/s2w_ab.log and s2w288_ab.log,
      // cold caches, against the 256 x 128 class tiles: 256 <- 256 @192^2 bs32 604 -> 519 (256 rows) -> 460 us (288),
      // 256 <- 512 919 -> 843 -> 784, 512 <- 1024 @96^2 834 -> 758 -> 600; the 512 x 128 tall tile for 128 channels
      // measured 1228 -> 1257 and is not used)
      if (g.C % 256 == 0 && (long)ceil_div(M, 256) * (g.C / 256) >= num_cus()) {
        const int gn = g.C / 256;
        const long NC = num_cus();
        // 288-row tiles when their grid ends in fewer row-weighted rounds of the chip (plan_v3's rule)
        if (ceil_div(ceil_div(M, 288) * gn, NC) * 288 < ceil_div(ceil_div(M, 256) * gn, NC) * 256) {
          const int gm = ceil_div(M, 288);
          v3::conv_dgrad_s2_w<288, 256><<<(unsigned)gm * gn, 512, 0, st>>>(dy, wt, dx, acc, gv, gm, gn, xbytes, wbytes,
                                                                            cls);
        } else {
          const int gm = ceil_div(M, 256);
          v3::conv_dgrad_s2_w<256, 256><<<(unsigned)gm * gn, 512, 0, st>>>(dy, wt, dx, acc, gv, gm, gn, xbytes, wbytes,
                                                                            cls);
        }
      } else if (g.C > 64) {
        const int gm = ceil_div(M, 256), gn = ceil_div(g.C, 128);
        v3::conv_fwd_v3<256, 128, 3, false, true, 3><<<(unsigned)gm * gn, 512, 0, st>>>(
            dy, wt, nullptr, dx, nullptr, nullptr, acc, gv, gm, gn, xbytes, wbytes, cls, Epi{});
      } else {
        const int gm = ceil_div(M, 256), gn = ceil_div(g.C, 64);
        v3::conv_fwd_v3<256, 64, 2, false, true, 3><<<(unsigned)gm * gn, 256, 0, st>>>(
            dy, wt, nullptr, dx, nullptr, nullptr, acc, gv, gm, gn, xbytes, wbytes, cls, Epi{});
      }
    }
  return (int)hipGetLastError();
}

template <typename T>
int conv_dgrad_t(const void* dy, const void* wt, void* dx, int acc, const Geom& g, hipStream_t st) {
  const long M = (long)g.N * g.H * g.W / (g.S == 2 ? 4 : 1);
  if constexpr (sizeof(T) == 2) {
    if (dgrad_s2_v3_ok(g, dy, wt, dx))
      return launch_dgrad_s2_v3((const bf16*)dy, (const bf16*)wt, (bf16*)dx, acc, g, st);
    if (g.S == 1 && g.OH == g.H + 2 * g.P - g.KH + 1 && g.OW == g.W + 2 * g.P - g.KW + 1 &&
        v3_ok(g.K, g.yps, g.C, g.xps, dy, wt, dx, M)) {
      // GEMM view: rows = input pixels (N, H, W), columns = C, gather dy (OH x OW x K, stride yps)
      Geom gv = make_geom(g.N, g.OH, g.OW, g.K, g.yps, g.C, g.KH, g.KW, 1, g.P, g.H, g.W, g.xps);
      if (halo_ok(gv, dy, wt, dx))
        return launch_halo<true>((const bf16*)dy, (const bf16*)wt, (bf16*)dx, nullptr, nullptr, gv, st, acc);
      return launch_v3<true>((const bf16*)dy, (const bf16*)wt, nullptr, (bf16*)dx, nullptr, nullptr, acc, gv, st,
                             Epi{}, plan_v3<true>(gv, dy, wt, dx, acc, Epi{}));
    }
  }
  if (big_tile(M, g.C)) return launch_dgrad<T, 128, 128>((const T*)dy, (const T*)wt, (T*)dx, acc, g, st);
  return launch_dgrad<T, 64, 64>((const T*)dy, (const T*)wt, (T*)dx, acc, g, st);
}
inline int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

inline int launch_wgrad_v3(const bf16* x, const bf16* dy, float* dw, Geom g, hipStream_t st) {
  const long NP = (long)g.N * g.OH * g.OW;
  const int Ntot = g.KH * g.KW * g.C;
  const int gm = ceil_div(g.K, 128), gn = ceil_div(Ntot, 128);
  const int nk = ceil_div(NP, 64);
  // split-K over pixels.  Cost model (calibrated on MI355X): resident blocks R = 2 per CU; time ~
  // rounds(tiles*s / R) * (K steps per split) * 1.9 us + tiles*s * 64 KiB of fp32 atomics at 1.3 TB/s.  It beat fixed
  // 512 / 768-block targets on DMA-1536 (152.15 vs 150.76 / 147.91 img/s, profiles/r04/wgrad_target_ab.log)
  const int tiles = gm * gn;
  int maxs = nk / 8;
  if (maxs < 1) maxs = 1;
  int splits = 1;
  {
    const double R = 2.0 * num_cus();
    double best = 1e300;
    for (int sp = 1; sp <= maxs; sp += (sp < 16 ? 1 : sp / 16)) {
      const double blocks = (double)tiles * sp;
      const double t = ceil(blocks / R) * ceil_div(nk, sp) * 1.9 + blocks * 0.0504;
      if (t < best) { best = t; splits = sp; }
    }
  }
  if (splits > maxs) splits = maxs;
  const int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  const dim3 grid((unsigned)gm * gn, splits);
  if (wgrad_begin(g, splits)) return 0;
  if (!g.zeroed) (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * Ntot, st);
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), db = 2.0 * ((double)NP * g.yps);
  const bool buf = xb < (double)v3::kBufOob && db < (double)v3::kBufOob;
  if (buf)
    v3::conv_wgrad_v3<2, 1><<<grid, 256, 0, st>>>(x, dy, dw, per, g, gm, gn, (unsigned)xb, (unsigned)db);
  else
    v3::conv_wgrad_v3<2, 0><<<grid, 256, 0, st>>>(x, dy, dw, per, g, gm, gn, 0u, 0u);
  wgrad_end(g, dw, splits, st);
  return (int)hipGetLastError();
}

// wgrad v4 tile 256 x 128 for K_out >= 256, else the v3 128 x 128 kernel (tools/gpu/ab_conv.sh,
// profiles/r01/ab_wgrad_v4.log: +7-11 % at K_out >= 256, the 256-row tile is half idle and a 128 x 256 one no faster at
// K_out = 128)
template <int BM, int BN>
int launch_wgrad_v4(const bf16* x, const bf16* dy, float* dw, Geom g, hipStream_t st) {
  const long NP = (long)g.N * g.OH * g.OW;
  const int Ntot = g.KH * g.KW * g.C;
  const int gm = ceil_div(g.K, BM), gn = ceil_div(Ntot, BN);
  const int nk = ceil_div(NP, 64);
  const int tiles = gm * gn;
  int maxs = nk / 8;
  if (maxs < 1) maxs = 1;
  int splits = 1;
  {
    // launch_wgrad_v3's model with one resident block per CU, twice the tile per K step and atomics
    const double R = num_cus(), sc = (double)BM * BN / (256.0 * 128.0);
    double best = 1e300;
    for (int sp = 1; sp <= maxs; sp += (sp < 16 ? 1 : sp / 16)) {
      const double blocks = (double)tiles * sp;
      const double t = ceil(blocks / R) * ceil_div(nk, sp) * 1.9 * 2 * 0.5 * sc + blocks * 0.0504 * 2 * sc;
      if (t < best) { best = t; splits = sp; }
    }
  }
  if (splits > maxs) splits = maxs;
  const int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  const dim3 grid((unsigned)tiles, splits);
  if (wgrad_begin(g, splits)) return 0;
  if (!g.zeroed) (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * Ntot, st);
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), db = 2.0 * ((double)NP * g.yps);
  v3::conv_wgrad_v4<BM, BN><<<grid, 512, 0, st>>>(x, dy, dw, per, g, gm, gn, (unsigned)xb, (unsigned)db);
  wgrad_end(g, dw, splits, st);
  return (int)hipGetLastError();
}
// tap-fused 3x3 s1 weight-grad (v3::conv_wgrad_tap) where it applies
inline bool wgrad_tap_ok(const Geom& g, const void* x, const void* dy) {
  if (g.KH != 3 || g.KW != 3 || g.S != 1 || g.P != 1 || g.OH != g.H || g.OW != g.W) return false;
  if (g.C % 16 != 0 || g.xps % 8 != 0 || g.yps % 8 != 0 || g.K % 8 != 0 || !aligned16(x) || !aligned16(dy)) return false;
  // C % 32 == 16 (the space-to-depth stem, 16 channels) included: the upper half of the halo plane loads zeros
  // (yolov5s 3845 -> 3876 img/s against the v3n column tiles, profiles/r05/wgrad_tap16_ab.log)
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), db = 2.0 * ((double)g.N * g.OH * g.OW * g.yps);
  if (xb >= (double)v3::kBufOob || db >= (double)v3::kBufOob) return false;
  // enough (patch, tile) work units that the per-block fp32 atomics of the 288-column tile stay a small share
  // (tools/gpu/tune_conv.py: 20^2 / 40^2 / 80^2 yolov5s layers are faster on the v3 / v4 column tiles)
  const long units = (long)g.N * ceil_div(g.OH, 8) * ceil_div(g.OW, 8) * ceil_div(g.K, 128) * ceil_div(g.C, 32);
  // 10000: the yolov5s 64-channel @80^2 layers (12800 units) measured 96 -> 79 us on the tap kernel, the 256-channel
  // @20^2 ones (9216) 70 -> 106 us (profiles/r02/ab_wgrad_v5s.log); lower thresholds were slower on yolov5s
  // (profiles/r05/wgrad_tap_units_ab.log)
  return units >= 10000;
}
// the <= 64-output-channel layers with C % 64 == 0 run the two-plane tile (a block owns 64 input channels: 13 fragment
// reads per 36 MFMAs instead of 11 per 18; DMA-1536 158.4 -> 159.1 img/s, profiles/r05/wgrad_tap_np2_ab.log); the
// same for the 128-row tile needs 288 accumulators, one block per CU, and measured 2 % slower
// (profiles/r05/wgrad_tap_np128_ab.log)
template <int BM, int NP = 1>
int launch_wgrad_tap(const bf16* x, const bf16* dy, float* dw, Geom g, hipStream_t st) {
  const int gm = ceil_div(g.K, BM), gn = ceil_div(g.C, 32 * NP);
  const int nk = g.N * ceil_div(g.OH, 8) * ceil_div(g.OW, 8);  // 8 x 8 patches
  const int tiles = gm * gn;
  int maxs = nk / 8;
  if (maxs < 1) maxs = 1;
  int splits = 1;
  {
    // two resident blocks per CU; ~1.1 us per patch step of the 128-row tile (288 MFMA per wave pair at ~45 %
    // of peak) and its 147 KiB fp32 tile of atomics per block at 1.3 TB/s (MI355X_MICROARCH.md §Global float
    // atomics); the 64-row tile halves both
    const double R = 2.0 * num_cus(), f = BM / 128.0 * NP;
    double best = 1e300;
    for (int sp = 1; sp <= maxs; sp += (sp < 16 ? 1 : sp / 16)) {
      const double blocks = (double)tiles * sp;
      const double t = ceil(blocks / R) * ceil_div(nk, sp) * 1.1 * f + blocks * 0.113 * f;
      if (t < best) { best = t; splits = sp; }
    }
  }
  if (splits > maxs) splits = maxs;
  const int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  const dim3 grid((unsigned)tiles, splits);
  if (wgrad_begin(g, splits)) return 0;
  if (!g.zeroed) (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * 9 * g.C, st);
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), db = 2.0 * ((double)g.N * g.OH * g.OW * g.yps);
  v3::conv_wgrad_tap<BM, NP><<<grid, 256, 0, st>>>(x, dy, dw, per, g, gm, gn, nk, (unsigned)xb, (unsigned)db);
  wgrad_end(g, dw, splits, st);
  return (int)hipGetLastError();
}

// narrow layers (K <= 64): BM = 32 / 64 out-channel tiles, BN = 128 / 256 column tiles
template <int BM, int BN>
int launch_wgrad_v3n(const bf16* x, const bf16* dy, float* dw, Geom g, hipStream_t st) {
  const long NP = (long)g.N * g.OH * g.OW;
  const int Ntot = g.KH * g.KW * g.C;
  const int gm = ceil_div(g.K, BM), gn = ceil_div(Ntot, BN);
  const int nk = ceil_div(NP, 64);
  const int tiles = gm * gn;
  int maxs = nk / 8;
  if (maxs < 1) maxs = 1;
  int splits = 1;
  {
    // same cost model as launch_wgrad_v3 with the tile's share of a 128 x 128 step and atomics
    const double R = 2.0 * num_cus() * (128.0 * 128.0) / (BM * BN) * 0.5;
    const double step = 1.9 * (BM * BN) / (128.0 * 128.0) + 0.25;
    double best = 1e300;
    for (int sp = 1; sp <= maxs; sp += (sp < 16 ? 1 : sp / 16)) {
      const double blocks = (double)tiles * sp;
      const double t = ceil(blocks / R) * ceil_div(nk, sp) * step + blocks * 0.0504 * (BM * BN) / (128.0 * 128.0);
      if (t < best) { best = t; splits = sp; }
    }
  }
  if (splits > maxs) splits = maxs;
  const int per = ceil_div(nk, splits);
  splits = ceil_div(nk, per);
  const dim3 grid((unsigned)tiles, splits);
  if (wgrad_begin(g, splits)) return 0;
  if (!g.zeroed) (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)g.K * Ntot, st);
  constexpr int NS = 3 * v3::WgradLdsN<BM, BN>::STAGE <= 80 * 1024 ? 3 : 2;  // keep 2 blocks per CU
  const double xb = 2.0 * ((double)g.N * g.H * g.W * g.xps), db = 2.0 * ((double)NP * g.yps);
  if (xb < (double)v3::kBufOob && db < (double)v3::kBufOob)
    v3::conv_wgrad_v3n<BM, BN, NS, true><<<grid, BN, 0, st>>>(x, dy, dw, per, g, gm, gn, (unsigned)xb, (unsigned)db);
  else
    v3::conv_wgrad_v3n<BM, BN, NS, false><<<grid, BN, 0, st>>>(x, dy, dw, per, g, gm, gn, 0u, 0u);
  wgrad_end(g, dw, splits, st);
  return (int)hipGetLastError();
}

// weight-grad of layers with <= 64 output channels: 1 = the narrow LDS-DMA tiles (BM 32/64) past 8 M pixels at
// K = 64, 2 = the 128 x 128 LDS-DMA tile (half its rows idle at K = 64) otherwise (tools/gpu/ab_conv.sh: 64 ch @768^2
// x 32 narrow 483 / 128-tile 394 / v2 257 TFLOP/s; @384^2 280 / 384 / 261; yolov5s layers 128-tile best)
inline int wgrad_narrow_for(const Geom& g, long NP) { return (g.K == 64 && NP >= 8L * 1024 * 1024) ? 1 : 2; }

template <typename T>
int conv_wgrad_t(const void* x, const void* dy, float* dw, const Geom& g, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    const long NP = (long)g.N * g.OH * g.OW;
    const int Ntot = g.KH * g.KW * g.C;
    const bool vec = g.C % 8 == 0 && g.xps % 8 == 0 && g.K % 8 == 0 && g.yps % 8 == 0 && aligned16(x) && aligned16(dy);
    const int nm = wgrad_narrow_for(g, NP);
    const double xb4 = 2.0 * ((double)g.N * g.H * g.W * g.xps), db4 = 2.0 * ((double)NP * g.yps);
    if (wgrad_tap_ok(g, x, dy))
      return g.K > 64 ? launch_wgrad_tap<128>((const bf16*)x, (const bf16*)dy, dw, g, st)
             : g.C % 64 == 0 ? launch_wgrad_tap<64, 2>((const bf16*)x, (const bf16*)dy, dw, g, st)
                             : launch_wgrad_tap<64>((const bf16*)x, (const bf16*)dy, dw, g, st);
    if (vec && g.K >= 256 && Ntot >= 128 && NP >= 16384 && xb4 < (double)v3::kBufOob && db4 < (double)v3::kBufOob)
      return launch_wgrad_v4<256, 128>((const bf16*)x, (const bf16*)dy, dw, g, st);
    if (vec && (g.K > 64 || nm == 2) && Ntot >= 64 && NP >= 16384)
      return launch_wgrad_v3((const bf16*)x, (const bf16*)dy, dw, g, st);
    if (vec && g.K <= 64 && Ntot >= 128 && NP >= 16384 && nm == 1) {
      // one 256-column tile also for 128 < Ntot < 256 (the 144-column space-to-depth stem view: on 128-column tiles
      // the second tile re-read every dy row for 16 columns of work; profiles/r04/stem_wgrad_ab.log 1638 -> 1276 us)
      const bool wide = Ntot >= 512 || Ntot % 256 == 0 || (Ntot > 128 && Ntot < 256);
      if (g.K <= 32) return wide ? launch_wgrad_v3n<32, 256>((const bf16*)x, (const bf16*)dy, dw, g, st)
                                 : launch_wgrad_v3n<32, 128>((const bf16*)x, (const bf16*)dy, dw, g, st);
      return wide ? launch_wgrad_v3n<64, 256>((const bf16*)x, (const bf16*)dy, dw, g, st)
                  : launch_wgrad_v3n<64, 128>((const bf16*)x, (const bf16*)dy, dw, g, st);
    }
  }
  if (g.K > 64 && g.KH * g.KW * g.C > 64) return launch_wgrad<T, 128, 128>((const T*)x, (const T*)dy, dw, g, st);
  return launch_wgrad<T, 64, 64>((const T*)x, (const T*)dy, dw, g, st);
}

}  // namespace

// ================================================================ C ABI (include/dmayolo.h)
#define DMY_WGRAD_OIHW 1
#define DMY_WGRAD_ZEROED 2
DMY_API int dmy_conv_wgrad_ex(int dtype, const void* x, const void* dy, float* dw, int N, int H, int W, int C,
                              long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, int flags,
                              void* stream);
// BN partial rows of the forward epilogue: 2 per 128 (big tile) or 64 rows of M.  The v3 kernel's
// 64-row wave rows number the same way (wave row wm of 256-row tile tm = row 4 tm + wm).
// ---------------------------------------------------------------- fp8 operand preparation
// Per-tensor activation scaling in two passes without atomics: fp8_blockmax_kernel writes one max per block
// (grid G <= kF8Blocks), fp8_quant_kernel reduces those G maxima in every block (G floats from L2), records the
// amax it used for the conv's dequantisation and writes x8[row][c] = e4m3(x * 448 / amax) densely.  A NaN
// anywhere makes amax NaN (and so the conv output), as an unquantised conv would propagate it.
constexpr int kF8Blocks = 1024;


DEV float block_nanmax(float m, float* red) {  // 256 threads
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = nanmax(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = nanmax(nanmax(red[0], red[1]), nanmax(red[2], red[3]));
  __syncthreads();
  return m;
}

__global__ void __launch_bounds__(256) fp8_blockmax_kernel(const bf16* __restrict__ x, unsigned nvec, int cv, long xps,
                                                           float* __restrict__ bmax) {
  __shared__ float red[4];
  float m = 0.f;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    const unsigned row = v / (unsigned)cv, c8 = v - row * (unsigned)cv;
    float f[8];
    unpack<bf16>(*reinterpret_cast<const uint4*>(x + (long)row * xps + c8 * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = nanmax(m, fabsf(f[j]));
  }
  m = block_nanmax(m, red);
  if (threadIdx.x == 0) bmax[blockIdx.x] = m;
}

__global__ void __launch_bounds__(256) fp8_quant_kernel(const bf16* __restrict__ x, unsigned nvec, int cv, long xps,
                                                        unsigned char* __restrict__ q, const float* __restrict__ bmax,
                                                        int nb, float* __restrict__ used) {
  __shared__ float red[4];
  float a = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) a = nanmax(a, bmax[i]);
  a = block_nanmax(a, red);
  if (blockIdx.x == 0 && threadIdx.x == 0) used[0] = a;
  const float inv = a > 0.f ? 448.f / a : 1.f;
  for (unsigned v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    const unsigned row = v / (unsigned)cv, c8 = v - row * (unsigned)cv;
    float f[8];
    unpack<bf16>(*reinterpret_cast<const uint4*>(x + (long)row * xps + c8 * 8), f);
    uint2 o;
    o.x = pack4_e4m3(f[0] * inv, f[1] * inv, f[2] * inv, f[3] * inv);
    o.y = pack4_e4m3(f[4] * inv, f[5] * inv, f[6] * inv, f[7] * inv);
    *reinterpret_cast<uint2*>(q + (size_t)v * 8) = o;
  }
}

// fp32 OIHW weight -> e4m3 OHWI [K][KH][KW][C] with a per-output-channel scale wscale[k] = amax_k / 448
__global__ void __launch_bounds__(256) wprep_fp8_kernel(const float* __restrict__ w, unsigned char* __restrict__ w8,
                                                        float* __restrict__ wscale, int C, int KH, int KW) {
  __shared__ float red[4];
  const int k = blockIdx.x, n = C * KH * KW;
  const float* src = w + (long)k * n;
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, fabsf(src[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float inv = m > 0.f ? 448.f / m : 1.f;
  for (int i = threadIdx.x * 4; i < n; i += 1024) {  // C % 128 == 0: 4 consecutive channels share (kh, kw)
    const int c = i % C, t = i / C, kw = t % KW, kh = t / KW;
    const float* s0 = src + ((long)c * KH + kh) * KW + kw;
    const long cs = (long)KH * KW;
    *reinterpret_cast<unsigned*>(w8 + (long)k * n + i) =
        pack4_e4m3(s0[0] * inv, s0[cs] * inv, s0[2 * cs] * inv, s0[3 * cs] * inv);
  }
  if (threadIdx.x == 0) wscale[k] = m > 0.f ? m / 448.f : 1.f;
}

inline bool fp8_fwd_ok(int C, int K, long yps, const void* x8, const void* w8, const void* y, double xbytes,
                       double wbytes) {
  return C % 128 == 0 && K % 8 == 0 && K >= 32 && yps % 8 == 0 && aligned16(x8) && aligned16(w8) && aligned16(y) &&
         xbytes < (double)v3::kBufOob && wbytes < (double)v3::kBufOob;
}

DMY_API int dmy_conv_fwd_partial_rows(long M, int K) { return 2 * ceil_div(M, big_tile_rows(M, K) ? 128 : 64); }

DMY_API long dmy_conv_fwd_bound_rows(long M, int K) {
  const long r = dmy_conv_fwd_partial_rows(M, K);
  return r > prow_persist_cap() ? r : prow_persist_cap();
}
DMY_API long dmy_conv_fwd_last_rows() { return t_prow_last; }

DMY_API int dmy_conv_fwd_bn_rows(int dtype, const void* x, const void* w, const float* bias, const void* y,
                                 int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P,
                                 int OH, int OW, long yps) {
  const Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if (!dtype) return dmy_conv_fwd_partial_rows((long)N * OH * OW, K);
  return (int)plan_fwd(g, x, w, bias, y, true, Epi{}, 0).rows;  // the training forward's own plan (conv_fwd_t)
}

DMY_API int dmy_conv_fwd(int dtype, const void* x, const void* w, const float* bias, void* y, float* psum, float* psq,
                         int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW,
                         long yps, void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * OH * OW == 0 || K == 0) return 0;
  return dtype ? conv_fwd_t<bf16>(x, w, bias, y, psum, psq, g, (hipStream_t)stream)
               : conv_fwd_t<float>(x, w, bias, y, psum, psq, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_fwd_act(int dtype, const void* x, const void* w, const float* bias, void* y, int N, int H, int W,
                             int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps,
                             const float* scale, const float* shift, int act, const void* res, long rps,
                             void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * OH * OW == 0 || K == 0) return 0;
  const Epi ep{scale, shift, res, rps, act, 1};
  return dtype ? conv_fwd_t<bf16>(x, w, bias, y, nullptr, nullptr, g, (hipStream_t)stream, ep)
               : conv_fwd_t<float>(x, w, bias, y, nullptr, nullptr, g, (hipStream_t)stream, ep);
}

// ws: at least dmy_fp8_quant_ws_elems() floats; ws[0] receives the amax the quantisation used
DMY_API long dmy_fp8_quant_ws_elems() { return 1 + kF8Blocks; }
DMY_API int dmy_fp8_quant(const void* x, long rows, int C, long xps, void* x8, float* ws, void* stream) {
  if (C % 8 != 0 || xps % 8 != 0 || !aligned16(x) || rows * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const unsigned nvec = (unsigned)(rows * (C / 8));
  if (nvec == 0) {
    (void)hipMemsetAsync(ws, 0, sizeof(float), st);
    return (int)hipGetLastError();
  }
  const int grid = grid_cap(ceil_div(nvec, 256), kF8Blocks);
  fp8_blockmax_kernel<<<grid, 256, 0, st>>>((const bf16*)x, nvec, C / 8, xps, ws + 1);
  fp8_quant_kernel<<<grid, 256, 0, st>>>((const bf16*)x, nvec, C / 8, xps, (unsigned char*)x8, ws + 1, grid, ws);
  return (int)hipGetLastError();
}

DMY_API int dmy_conv_wprep_fp8(const float* w_oihw, void* w8, float* wscale, int K, int C, int KH, int KW,
                               void* stream) {
  if (C % 4 != 0) return (int)hipErrorInvalidValue;
  wprep_fp8_kernel<<<K, 256, 0, (hipStream_t)stream>>>(w_oihw, (unsigned char*)w8, wscale, C, KH, KW);
  return (int)hipGetLastError();
}

// BN partial rows the fp8 kernel's epilogue writes (v3 numbering at every M: 2 per 128 rows when K > 64, else per 64)
DMY_API int dmy_conv_fwd_fp8_partial_rows(long M, int K) { return 2 * ceil_div(M, K > 64 ? 128 : 64); }

DMY_API int dmy_conv_fwd_fp8(const void* x8, const void* w8, const float* xamax, const float* wscale,
                             const float* bias, void* y, float* psum, float* psq, int N, int H, int W, int C, int K,
                             int KH, int KW, int S, int P, int OH, int OW, long yps, const float* scale,
                             const float* shift, int act, const void* res, long rps, void* stream) {
  const Geom g = make_geom(N, H, W, C, C, K, KH, KW, S, P, OH, OW, yps);
  const long M = (long)N * OH * OW;
  if (M == 0 || K == 0) return 0;
  const double xb = (double)N * H * W * C, wb = (double)K * KH * KW * C;
  if (!fp8_fwd_ok(C, K, yps, x8, w8, y, xb, wb) || (res && (rps % 8 != 0 || !aligned16(res))))
    return (int)hipErrorInvalidValue;
  const Epi ep{scale, shift, res, rps, act, scale != nullptr || res != nullptr || act != 0 ? 1 : 0};
  const bool p1 = KH == 1 && KW == 1 && S == 1 && P == 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned xbytes = (unsigned)xb, wbytes = (unsigned)wb;
  const unsigned char *a = (const unsigned char*)x8, *b = (const unsigned char*)w8;
#define F8_GO(BM, BN, NS)                                                                                          \
  {                                                                                                                \
    const int gm = ceil_div(M, BM), gn = ceil_div(K, BN);                                                          \
    if (p1)                                                                                                        \
      v3::conv_fwd_f8<BM, BN, NS, true><<<(unsigned)gm * gn, BM * BN / 64, 0, st>>>(                                \
          a, b, xamax, wscale, bias, (bf16*)y, psum, psq, g, gm, gn, xbytes, wbytes, ep);                          \
    else                                                                                                           \
      v3::conv_fwd_f8<BM, BN, NS, false><<<(unsigned)gm * gn, BM * BN / 64, 0, st>>>(                               \
          a, b, xamax, wscale, bias, (bf16*)y, psum, psq, g, gm, gn, xbytes, wbytes, ep);                          \
  }
  if (K > 64) F8_GO(256, 128, 3)
  else F8_GO(256, 64, 2)
#undef F8_GO
  return (int)hipGetLastError();
}

// Inference forward with a split-K workspace for small M (batch-1 detect): dmy_conv_fwd_act semantics; when
// dmy_conv_fwd_splitk_elems > 0 for the same arguments, a workspace of that many floats lets the small-M layers
// split their reduction over the chip (0: the call is dmy_conv_fwd_act).  scale == shift == res == nullptr and
// act == 0 is the plain forward (no BN partials).
DMY_API long dmy_conv_fwd_splitk_elems(int dtype, const void* x, const void* w, const void* y, int N, int H, int W,
                                       int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps) {
  if (!dtype) return 0;
  return splitk_elems(make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps), x, w, y);
}

DMY_API int dmy_conv_fwd_act_ws(int dtype, const void* x, const void* w, const float* bias, void* y, int N, int H,
                                int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps,
                                const float* scale, const float* shift, int act, const void* res, long rps, float* ws,
                                long ws_elems, void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * OH * OW == 0 || K == 0) return 0;
  const Epi ep{scale, shift, res, rps, act, scale != nullptr || res != nullptr || act != 0 ? 1 : 0};
  return dtype ? conv_fwd_t<bf16>(x, w, bias, y, nullptr, nullptr, g, (hipStream_t)stream, ep, ws, ws_elems)
               : conv_fwd_t<float>(x, w, bias, y, nullptr, nullptr, g, (hipStream_t)stream, ep);
}

DMY_API int dmy_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int accumulate, int N, int H, int W,
                           int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps,
                           void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  if ((long)N * H * W == 0 || C == 0) return 0;
  if (S > 2) return (int)hipErrorInvalidValue;
  return dtype ? conv_dgrad_t<bf16>(dy, wt, dx, accumulate, g, (hipStream_t)stream)
               : conv_dgrad_t<float>(dy, wt, dx, accumulate, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_wgrad(int dtype, const void* x, const void* dy, float* dw_ohwi, int N, int H, int W, int C,
                           long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, void* stream) {
  return dmy_conv_wgrad_ex(dtype, x, dy, dw_ohwi, N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps, 0, stream);
}

DMY_API int dmy_conv_wgrad_ex(int dtype, const void* x, const void* dy, float* dw, int N, int H, int W, int C,
                              long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, int flags,
                              void* stream) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  g.oihw = flags & DMY_WGRAD_OIHW ? 1 : 0;
  g.zeroed = flags & DMY_WGRAD_ZEROED ? 1 : 0;
  return dtype ? conv_wgrad_t<bf16>(x, dy, dw, g, (hipStream_t)stream)
               : conv_wgrad_t<float>(x, dy, dw, g, (hipStream_t)stream);
}

// deterministic weight-grad: fp32 workspace elements it needs (0 = the dispatch uses one split: no workspace)
DMY_API long dmy_conv_wgrad_ws_elems(int dtype, const void* x, const void* dy, int N, int H, int W, int C, long xps,
                                     int K, int KH, int KW, int S, int P, int OH, int OW, long yps, int flags) {
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  g.oihw = flags & DMY_WGRAD_OIHW ? 1 : 0;
  g.zeroed = flags & DMY_WGRAD_ZEROED ? 1 : 0;
  int splits = 1;
  g.plan = &splits;
  (void)(dtype ? conv_wgrad_t<bf16>(x, dy, nullptr, g, nullptr) : conv_wgrad_t<float>(x, dy, nullptr, g, nullptr));
  return splits > 1 ? (long)splits * K * KH * KW * C : 0;
}

DMY_API int dmy_conv_wgrad_det(int dtype, const void* x, const void* dy, float* dw, int N, int H, int W, int C,
                               long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, int flags,
                               float* ws, long ws_elems, void* stream) {
  const long need = dmy_conv_wgrad_ws_elems(dtype, x, dy, N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps, flags);
  if (need > 0 && (ws == nullptr || ws_elems < need)) return (int)hipErrorInvalidValue;
  Geom g = make_geom(N, H, W, C, xps, K, KH, KW, S, P, OH, OW, yps);
  g.oihw = flags & DMY_WGRAD_OIHW ? 1 : 0;
  g.zeroed = flags & DMY_WGRAD_ZEROED ? 1 : 0;
  if (need > 0) {
    g.dws = ws;
    g.dws_slab = (long)K * KH * KW * C;
  }
  return dtype ? conv_wgrad_t<bf16>(x, dy, dw, g, (hipStream_t)stream)
               : conv_wgrad_t<float>(x, dy, dw, g, (hipStream_t)stream);
}

DMY_API int dmy_conv_wprep(int dtype, const float* w_oihw, void* w_ohwi, void* w_ihwo, int K, int C, int Cp, int KH,
                           int KW, void* stream) {
  const long total = (long)K * Cp * KH * KW;
  const int grid = grid_cap(ceil_div(total, 256), 1024);
  if (dtype) wprep_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (bf16*)w_ohwi, (bf16*)w_ihwo, K, C, Cp, KH, KW);
  else wprep_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (float*)w_ohwi, (float*)w_ihwo, K, C, Cp, KH, KW);
  return (int)hipGetLastError();
}

// descs: device array of n WprepDesc {w, wf, wt (nullable), K, C, KH, KW} (40 bytes each, include/dmayolo.h)
DMY_API int dmy_conv_wprep_multi(int dtype, const void* descs, int n, void* stream) {
  if (n <= 0) return 0;
  static_assert(sizeof(WprepDesc) == 40, "WprepDesc layout is part of the C ABI");
  const dim3 grid(128, n);
  if (dtype) wprep_multi_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>((const WprepDesc*)descs);
  else wprep_multi_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>((const WprepDesc*)descs);
  return (int)hipGetLastError();
}

DMY_API int dmy_conv_wprep_s2d(int dtype, const float* w_oihw, void* w_s2d, int K, int C, int Cs, void* stream) {
  const int grid = grid_cap(ceil_div((long)K * 9 * Cs, 256), 1024);
  if (dtype) wprep_s2d_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (bf16*)w_s2d, K, C, Cs);
  else wprep_s2d_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>(w_oihw, (float*)w_s2d, K, C, Cs);
  return (int)hipGetLastError();
}

DMY_API int dmy_conv_wgrad_s2d_to_oihw(const float* dw_s2d, float* dw_oihw, int K, int C, int Cs, void* stream) {
  wgrad_s2d_to_oihw_kernel<<<grid_cap(ceil_div((long)K * C * 36, 256), 1024), 256, 0, (hipStream_t)stream>>>(
      dw_s2d, dw_oihw, K, C, Cs);
  return (int)hipGetLastError();
}

DMY_API int dmy_conv_wgrad_to_oihw(const float* dw_ohwi, float* dw_oihw, int K, int C, int Cp, int KH, int KW,
                                   void* stream) {
  const long total = (long)K * C * KH * KW;
  wgrad_to_oihw_kernel<<<grid_cap(ceil_div(total, 256), 1024), 256, 0, (hipStream_t)stream>>>(dw_ohwi, dw_oihw, K, C,
                                                                                               Cp, KH, KW);
  return (int)hipGetLastError();
}
