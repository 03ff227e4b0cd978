// Memory-bound NHWC kernels of the DMA-YOLO path (HBM roofline):
//   max-pool k5 s1 (SPPF models/common.py:243-258, SPPFCSPC :1257-1276), avg-pool r (SCConv k2 :1282),
//   nearest resize (nn.Upsample yaml:31/36, F.interpolate in SCConv :1311), channel-slice copy with
//   BiFPN weights (Concat :656-664, AdConcat2/3 :994-1026), SCConv gate (:1311-1314),
//   CoorAttention pooling / re-weighting (:1183-1207), input normalisation (train.py:402).
#include "common.h"
#include <initializer_list>
#include <type_traits>

namespace {

inline bool al16(const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; }

// NV = elements per thread: the 16-byte vector width (channels % VW == 0, 16-B aligned bases and
// pixel strides) or 1 (scalar fallback).  All math per element in fp32, identical in both forms.
template <typename T, int NV> DEV void ldv(const T* p, float* f) {
  if constexpr (NV == Traits<T>::VW) unpack<T>(*reinterpret_cast<const uint4*>(p), f);
  else
#pragma unroll
    for (int j = 0; j < NV; ++j) f[j] = to_f(p[j]);
}
template <typename T, int NV> DEV void stv(T* p, const float* f) {
  if constexpr (NV == Traits<T>::VW) *reinterpret_cast<uint4*>(p) = pack<T>(f);
  else
#pragma unroll
    for (int j = 0; j < NV; ++j) p[j] = from_f<T>(f[j]);
}
// i = q * d + r with a 32-bit unsigned division when i fits (see vidx)
DEV void divmod(long i, int d, long& q, int& r) {
  if ((unsigned long)i < 0xFFFFFFFFul) {
    const unsigned u = (unsigned)i, qq = u / (unsigned)d;
    q = qq;
    r = (int)(u - qq * (unsigned)d);
    return;
  }
  q = i / d;
  r = (int)(i % d);
}

// decompose a vector index over [N][H][W][C/NV] -> (b, h, w, c).  32-bit unsigned divisions whenever the index
// fits (every activation here): a 64-bit division is a long software sequence, and three of them per 16-B vector
// made the SCConv gate / pool / resize kernels VALU-bound at a third of the HBM rate.
DEV void vidx(long i, int H, int W, int CV, int NV, int& b, int& h, int& w, int& c) {
  if ((unsigned long)i < 0xFFFFFFFFul) {
    const unsigned u = (unsigned)i, t0 = u / (unsigned)CV, t1 = t0 / (unsigned)W;
    c = (int)(u - t0 * (unsigned)CV) * NV;
    w = (int)(t0 - t1 * (unsigned)W);
    h = (int)(t1 % (unsigned)H);
    b = (int)(t1 / (unsigned)H);
    return;
  }
  c = (int)(i % CV) * NV;
  long t = i / CV;
  w = (int)(t % W);
  t /= W;
  h = (int)(t % H);
  b = (int)(t / H);
}

// ---------------------------------------------------------------- max-pool (k odd, stride 1, pad k/2)
// ATen's max_pool2d rule (CPU and CUDA kernels alike): scan the window row-major, update when
// `v > best || isnan(v)`, start from -inf with the index of the first in-image tap.  The window
// offset of the winner (dh * k + dw) is written for the backward.  KS > 0: compile-time window,
// every tap is loaded branch-free (out-of-image taps read the centre pixel and are masked), so the
// loads of a window issue back to back; KS = 0: runtime window (k > 13).
template <typename T, int NV, int KS>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C, int kr) {
  const int k = KS > 0 ? KS : kr;
  const int CV = C / NV;
  const long total = (long)N * H * W * CV;
  const int p = k / 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, h, w, c;
    vidx(i, H, W, CV, NV, b, h, w, c);
    const int h0 = h - p, w0 = w - p;
    const int first = ((h0 < 0 ? 0 : h0) - h0) * k + ((w0 < 0 ? 0 : w0) - w0);
    float best[NV];
    int bi[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) { best[j] = -INFINITY; bi[j] = first; }
    const T* xb = x + (long)b * H * W * xps + c;
    if constexpr (KS > 0) {
      // one window row per batch: KS independent loads in flight, 32-bit offsets inside the image
      const int ixps = (int)xps;
#pragma unroll
      for (int dh = 0; dh < KS; ++dh) {
        const int hh = h0 + dh;
        const bool hok = (unsigned)hh < (unsigned)H;
        float v[KS][NV];
#pragma unroll
        for (int dw = 0; dw < KS; ++dw) {
          const int ww = w0 + dw;
          const bool ok = hok && (unsigned)ww < (unsigned)W;
          ldv<T, NV>(xb + ((ok ? hh : h) * W + (ok ? ww : w)) * ixps, v[dw]);
        }
#pragma unroll
        for (int dw = 0; dw < KS; ++dw) {
          const int ww = w0 + dw;
          const bool ok = hok && (unsigned)ww < (unsigned)W;
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            // bitwise (not short-circuit) so the selects stay branch-free
            const float vv = ok ? v[dw][j] : -INFINITY;
            const unsigned up = (unsigned)(vv > best[j]) | (unsigned)__builtin_isnan(vv);
            best[j] = up ? vv : best[j];
            bi[j] = up ? dh * KS + dw : bi[j];
          }
        }
      }
    }
    if constexpr (KS == 0) {
      for (int dh = 0; dh < k; ++dh) {
        const int hh = h0 + dh;
        if ((unsigned)hh >= (unsigned)H) continue;
        for (int dw = 0; dw < k; ++dw) {
          const int ww = w0 + dw;
          if ((unsigned)ww >= (unsigned)W) continue;
          float v[NV];
          ldv<T, NV>(xb + ((long)hh * W + ww) * xps, v);
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            const bool up = v[j] > best[j] || isnan(v[j]);
            best[j] = up ? v[j] : best[j];
            bi[j] = up ? dh * k + dw : bi[j];
          }
        }
      }
    }
    const long pix = ((long)b * H + h) * W + w;
    stv<T, NV>(y + pix * yps + c, best);
    // one packed store of the NV argmax bytes
    uint8_t a[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) a[j] = (uint8_t)bi[j];
    if constexpr (NV == 8) *reinterpret_cast<uint2*>(arg + pix * C + c) = *reinterpret_cast<const uint2*>(a);
    else if constexpr (NV == 4) *reinterpret_cast<uint32_t*>(arg + pix * C + c) = *reinterpret_cast<const uint32_t*>(a);
    else
#pragma unroll
      for (int j = 0; j < NV; ++j) arg[pix * C + c + j] = a[j];
  }
}

// dx[p] = sum of dy[q] over windows q whose argmax is p (gather: deterministic, no atomics); only the
// dy vectors that route to p are loaded.
template <typename T, int NV>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const T* __restrict__ dy, long dps, const uint8_t* __restrict__ arg,
                                                          T* __restrict__ dx, long dxps, int accumulate, int N, int H, int W,
                                                          int C, int kr) {
  const int k = kr;
  const int CV = C / NV;
  const long total = (long)N * H * W * CV;
  const int p = k / 2;
  using AW = typename std::conditional<NV == 8, uint2, typename std::conditional<NV == 4, uint32_t, uint8_t>::type>::type;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, h, w, c;
    vidx(i, H, W, CV, NV, b, h, w, c);
    float s[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] = 0.f;
    const long img = (long)b * H * W;
    for (int oh = h - p; oh <= h + p; ++oh) {
      if (oh < 0 || oh >= H) continue;
      for (int ow = w - p; ow <= w + p; ++ow) {
        if (ow < 0 || ow >= W) continue;
        const long q = img + (long)oh * W + ow;
        const int want = (h - oh + p) * k + (w - ow + p);
        uint8_t a[NV];
        *reinterpret_cast<AW*>(a) = *reinterpret_cast<const AW*>(arg + q * C + c);
        bool any = false;
#pragma unroll
        for (int j = 0; j < NV; ++j) any |= a[j] == want;
        if (!any) continue;
        float d[NV];
        ldv<T, NV>(dy + q * dps + c, d);
#pragma unroll
        for (int j = 0; j < NV; ++j)
          if (a[j] == want) s[j] += d[j];
      }
    }
    T* o = dx + (((long)b * H + h) * W + w) * dxps + c;
    if (accumulate) {
      float d[NV];
      ldv<T, NV>(o, d);
#pragma unroll
      for (int j = 0; j < NV; ++j) s[j] += d[j];
    }
    stv<T, NV>(o, s);
  }
}

// ---------------------------------------------------------------- max-pool, LDS-tiled (16-B channel vectors)
// One workgroup = a TH x TW tile of outputs x one 16-B channel vector of one image.  The input tile
// with its (K-1) halo is staged in LDS once; the window max is separable: a row pass (max over dw
// per (input row, output col), first-valid start, ATen update rule) then a column pass over dh
// (start = first valid row's row winner) gives exactly the row-major scan's winner (NaN: the last
// one, as in ATen).  Backward: the window arguments and dy of every output that can route into the
// tile are staged in LDS and each input pixel gathers its contributions (deterministic, no atomics).
constexpr int MP_TH = 16, MP_TW = 32;

// Block -> (image, tile, 16-B channel vector) of the LDS max-pool kernels: one 1-D grid in an XCD-contiguous logical
// order with the channel vector fastest, so the CV blocks that read the same pixel rows (one 16-B slice of each
// 128..2048-B pixel row per block) run together on one XCD and share its L2 instead of each re-reading the rows from
// HBM / the Infinity Cache (the 3-D grid it replaces put every image's tiles of one channel slice before the next).
struct MpTile {
  int b, c, h0, w0;
};
DEV MpTile mp_tile(int CV, int NV, int twn, int thn) {
  const int nwg = (int)gridDim.x, id = (int)blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = id % 8, loc = id / 8;
  int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  MpTile t;
  t.c = (L % CV) * NV;
  L /= CV;
  t.w0 = (L % twn) * MP_TW;
  L /= twn;
  t.h0 = (L % thn) * MP_TH;
  t.b = L / thn;
  return t;
}

template <typename T, int K>
__global__ void __launch_bounds__(256) maxpool_fwd_lds(const T* __restrict__ x, long xps, T* __restrict__ y, long yps,
                                                       uint8_t* __restrict__ arg, int H, int W, int C) {
  constexpr int NV = Traits<T>::VW, P = K / 2, IH = MP_TH + K - 1, IW = MP_TW + K - 1;
  __shared__ uint4 xin[IH * IW];
  __shared__ uint4 rm[IH * MP_TW];
  __shared__ uint2 ra[IH * MP_TW];
  const MpTile tl = mp_tile(C / NV, NV, (W + MP_TW - 1) / MP_TW, (H + MP_TH - 1) / MP_TH);
  const int b = tl.b, c = tl.c, h0 = tl.h0, w0 = tl.w0;
  const T* xb = x + (long)b * H * W * xps + c;
  for (int e = threadIdx.x; e < IH * IW; e += 256) {
    const int hh = h0 - P + e / IW, ww = w0 - P + e % IW;
    xin[e] = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                 ? *reinterpret_cast<const uint4*>(xb + ((long)hh * W + ww) * xps) : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  // row pass: rm[r][w] = max over dw of input (row r, col w + dw)
  const int wlo = w0 - P;  // image col of tile col 0 of xin
  for (int e = threadIdx.x; e < IH * MP_TW; e += 256) {
    const int r = e / MP_TW, w = e % MP_TW;
    const int c0 = wlo + w;  // image col of tap dw = 0
    const int first = c0 < 0 ? -c0 : 0;
    float best[NV];
    uint8_t bi[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) { best[j] = -INFINITY; bi[j] = (uint8_t)first; }
#pragma unroll
    for (int dw = 0; dw < K; ++dw) {
      const bool ok = (unsigned)(c0 + dw) < (unsigned)W;
      float v[NV];
      unpack<T>(xin[r * IW + w + dw], v);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float vv = ok ? v[j] : -INFINITY;
        const unsigned up = (unsigned)(vv > best[j]) | (unsigned)__builtin_isnan(vv);
        best[j] = up ? vv : best[j];
        bi[j] = up ? (uint8_t)dw : bi[j];
      }
    }
    rm[e] = pack<T>(best);
    ra[e] = *reinterpret_cast<const uint2*>(bi);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < MP_TH * MP_TW; e += 256) {
    const int h = e / MP_TW, w = e % MP_TW;
    const int oh = h0 + h, ow = w0 + w;
    if (oh >= H || ow >= W) continue;
    const int r0 = oh - P;  // image row of tap dh = 0 (= tile row h of xin / rm)
    const int first = r0 < 0 ? -r0 : 0;
    float best[NV];
    int bi[NV];
    {
      const uint8_t* fa = reinterpret_cast<const uint8_t*>(&ra[(h + first) * MP_TW + w]);
#pragma unroll
      for (int j = 0; j < NV; ++j) { best[j] = -INFINITY; bi[j] = first * K + fa[j]; }
    }
#pragma unroll
    for (int dh = 0; dh < K; ++dh) {
      const bool ok = (unsigned)(r0 + dh) < (unsigned)H;
      float v[NV];
      unpack<T>(rm[(h + dh) * MP_TW + w], v);
      const uint2 a2 = ra[(h + dh) * MP_TW + w];
      const uint8_t* a = reinterpret_cast<const uint8_t*>(&a2);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float vv = ok ? v[j] : -INFINITY;
        const unsigned up = (unsigned)(vv > best[j]) | (unsigned)__builtin_isnan(vv);
        best[j] = up ? vv : best[j];
        bi[j] = up ? dh * K + a[j] : bi[j];
      }
    }
    const long pix = ((long)b * H + oh) * W + ow;
    *reinterpret_cast<uint4*>(y + pix * yps + c) = pack<T>(best);
    uint8_t ab[8];
#pragma unroll
    for (int j = 0; j < NV; ++j) ab[j] = (uint8_t)bi[j];
    if constexpr (NV == 8) *reinterpret_cast<uint2*>(arg + pix * C + c) = *reinterpret_cast<const uint2*>(ab);
    else *reinterpret_cast<uint32_t*>(arg + pix * C + c) = *reinterpret_cast<const uint32_t*>(ab);
  }
}

// Backward, separable like the forward: an output q routes dy[q] to input (q_h + dh* - P, q_w + dw* - P) where dh* is
// its column-pass winner and dw* the row-pass winner at (that row, q_w) -- the same dw* for every output that picks
// that row position.  Stage A sums, for each (tile row, output column), the dy of the outputs whose column pass chose
// that row (K checks) and keeps their dw*; stage B sums, for each input pixel, the stage-A sums whose dw* points at it
// (K checks): 2K window checks per input instead of the K^2 of a direct gather (the k = 13 SPP pools of config 5 spent
// 5 ms per call there).  Sums over dh then dw, in fixed order (deterministic, no atomics).
template <typename T, int K>
__global__ void __launch_bounds__(256) maxpool_bwd_lds(const T* __restrict__ dy, long dps, const uint8_t* __restrict__ arg,
                                                       T* __restrict__ dx, long dxps, int accumulate, int H, int W, int C) {
  constexpr int NV = Traits<T>::VW, P = K / 2, IH = MP_TH + K - 1, IW = MP_TW + K - 1;
  using AW = typename std::conditional<NV == 8, uint2, uint32_t>::type;
  __shared__ uint4 gs[IH * IW];       // dy of every output that can route into the tile
  __shared__ AW as_[IH * IW];         // their window offsets dh* K + dw* (0xFF: out of image)
  __shared__ float dr[MP_TH * IW * NV];  // stage A: per (tile row, output column) the column-routed sums
  __shared__ AW rs[MP_TH * IW];       // ... and their row-pass winner dw* (0xFF: nothing routed)
  const MpTile tl = mp_tile(C / NV, NV, (W + MP_TW - 1) / MP_TW, (H + MP_TH - 1) / MP_TH);
  const int b = tl.b, c = tl.c, h0 = tl.h0, w0 = tl.w0;
  // outputs q in [h0 - P, h0 + TH - 1 + P] x [w0 - P, w0 + TW - 1 + P]; out-of-image ones never route
  for (int e = threadIdx.x; e < IH * IW; e += 256) {
    const int qh = h0 - P + e / IW, qw = w0 - P + e % IW;
    const bool ok = (unsigned)qh < (unsigned)H && (unsigned)qw < (unsigned)W;
    const long q = ((long)b * H + qh) * W + qw;
    gs[e] = ok ? *reinterpret_cast<const uint4*>(dy + q * dps + c) : make_uint4(0, 0, 0, 0);
    as_[e] = ok ? *reinterpret_cast<const AW*>(arg + q * C + c) : AW{0xFFFFFFFFu};
    if constexpr (NV == 8) { if (!ok) as_[e] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu); }
  }
  __syncthreads();
  // stage A: tile row h (input row h0 + h) x output column index ec; output row h0 + h + P - dh = gs row h + K - 1 - dh
  for (int e = threadIdx.x; e < MP_TH * IW; e += 256) {
    const int h = e / IW, ec = e % IW;
    float s[NV];
    uint8_t sel[sizeof(AW)];
#pragma unroll
    for (int j = 0; j < NV; ++j) { s[j] = 0.f; sel[j] = 0xFF; }
#pragma unroll
    for (int dh = 0; dh < K; ++dh) {
      const int slot = (h + K - 1 - dh) * IW + ec;
      const AW a2 = as_[slot];
      const uint8_t* a = reinterpret_cast<const uint8_t*>(&a2);
      bool any = false;
#pragma unroll
      for (int j = 0; j < NV; ++j) any |= a[j] != 0xFF && a[j] / K == dh;
      if (!any) continue;
      float d[NV];
      unpack<T>(gs[slot], d);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const bool m = a[j] != 0xFF && a[j] / K == dh;
        s[j] += m ? d[j] : 0.f;
        sel[j] = m ? (uint8_t)(a[j] % K) : sel[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) dr[e * NV + j] = s[j];
    rs[e] = *reinterpret_cast<const AW*>(sel);
  }
  __syncthreads();
  // stage B: input (h0 + h, w0 + w) gathers the stage-A sums at output column index w + K - 1 - dw whose dw* == dw
  for (int e = threadIdx.x; e < MP_TH * MP_TW; e += 256) {
    const int h = e / MP_TW, w = e % MP_TW;
    const int ih = h0 + h, iw = w0 + w;
    if (ih >= H || iw >= W) continue;
    float s[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] = 0.f;
#pragma unroll
    for (int dw = 0; dw < K; ++dw) {
      const int pos = h * IW + w + K - 1 - dw;
      const AW a2 = rs[pos];
      const uint8_t* a = reinterpret_cast<const uint8_t*>(&a2);
#pragma unroll
      for (int j = 0; j < NV; ++j) s[j] += a[j] == dw ? dr[pos * NV + j] : 0.f;
    }
    T* o = dx + (((long)b * H + ih) * W + iw) * dxps + c;
    if (accumulate) {
      float d[NV];
      unpack<T>(*reinterpret_cast<const uint4*>(o), d);
#pragma unroll
      for (int j = 0; j < NV; ++j) s[j] += d[j];
    }
    *reinterpret_cast<uint4*>(o) = pack<T>(s);
  }
}

// ---------------------------------------------------------------- avg-pool r x r, stride r, floor mode
template <typename T, int NV>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, int N, int H, int W, int C,
                                   int r) {
  const int OH = H / r, OW = W / r, CV = C / NV;
  const long total = (long)N * OH * OW * CV;
  const float inv = 1.0f / (r * r);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, oh, ow, c;
    vidx(i, OH, OW, CV, NV, b, oh, ow, c);
    float s[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] = 0.f;
    for (int dh = 0; dh < r; ++dh)
      for (int dw = 0; dw < r; ++dw) {
        float v[NV];
        ldv<T, NV>(x + (((long)b * H + oh * r + dh) * W + ow * r + dw) * xps + c, v);
#pragma unroll
        for (int j = 0; j < NV; ++j) s[j] += v[j];
      }
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] *= inv;
    stv<T, NV>(y + (((long)b * OH + oh) * OW + ow) * C + c, s);
  }
}

template <typename T, int NV>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, long dxps, int accumulate, int N,
                                   int H, int W, int C, int r) {
  const int OH = H / r, OW = W / r, CV = C / NV;
  const long total = (long)N * H * W * CV;
  const float inv = 1.0f / (r * r);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, h, w, c;
    vidx(i, H, W, CV, NV, b, h, w, c);
    const int oh = h / r, ow = w / r;
    float v[NV];
    if (oh < OH && ow < OW) {
      ldv<T, NV>(dy + (((long)b * OH + oh) * OW + ow) * C + c, v);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] *= inv;
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = 0.f;
    }
    T* o = dx + (((long)b * H + h) * W + w) * dxps + c;
    if (accumulate) {
      float d[NV];
      ldv<T, NV>(o, d);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] += d[j];
    }
    stv<T, NV>(o, v);
  }
}

// ---------------------------------------------------------------- nearest resize (ATen nearest_idx)
DEV int nearest_src(int d, int in, int out) {
  if (out == in) return d;
  if (out == 2 * in) return d >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf(__fmul_rn((float)d, scale));
  return s < in - 1 ? s : in - 1;
}

template <typename T, int NV>
__global__ void resize_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps, float yscale,
                                  int N, int IH, int IW, int OH, int OW, int C) {
  const int CV = C / NV;
  const long total = (long)N * OH * OW * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, oh, ow, c;
    vidx(i, OH, OW, CV, NV, b, oh, ow, c);
    const int ih = nearest_src(oh, IH, OH), iw = nearest_src(ow, IW, OW);
    float v[NV];
    ldv<T, NV>(x + (((long)b * IH + ih) * IW + iw) * xps + c, v);
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] *= yscale;
    stv<T, NV>(y + (((long)b * OH + oh) * OW + ow) * yps + c, v);
  }
}

// dx[ih,iw] = sum over dst (oh,ow) mapping to it; preimages are contiguous ranges
template <typename T, int NV>
__global__ void resize_bwd_kernel(const T* __restrict__ dy, long dps, T* __restrict__ dx, long dxps, int N, int IH,
                                  int IW, int OH, int OW, int C) {
  const int CV = C / NV;
  const long total = (long)N * IH * IW * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, ih, iw, c;
    vidx(i, IH, IW, CV, NV, b, ih, iw, c);
    int h0, h1, w0, w1;
    if (OH == 2 * IH) { h0 = 2 * ih; h1 = h0 + 1; }
    else { h0 = max(0, (int)((long)ih * OH / IH) - 2); h1 = min(OH - 1, (int)((long)(ih + 1) * OH / IH) + 2); }
    if (OW == 2 * IW) { w0 = 2 * iw; w1 = w0 + 1; }
    else { w0 = max(0, (int)((long)iw * OW / IW) - 2); w1 = min(OW - 1, (int)((long)(iw + 1) * OW / IW) + 2); }
    float s[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) s[j] = 0.f;
    for (int oh = h0; oh <= h1; ++oh) {
      if (nearest_src(oh, IH, OH) != ih) continue;
      for (int ow = w0; ow <= w1; ++ow)
        if (nearest_src(ow, IW, OW) == iw) {
          float v[NV];
          ldv<T, NV>(dy + (((long)b * OH + oh) * OW + ow) * dps + c, v);
#pragma unroll
          for (int j = 0; j < NV; ++j) s[j] += v[j];
        }
    }
    stv<T, NV>(dx + (((long)b * IH + ih) * IW + iw) * dxps + c, s);
  }
}

// ---------------------------------------------------------------- space_to_depth (models/common.py:1451-1458)
// y[b, h, w, q*C + c] = x[b, 2h + dy_q, 2w + dx_q, c], q = 0..3 <-> (dy, dx) = (0,0), (1,0), (0,1), (1,1)
// (the cat order x[::2, ::2], x[1::2, ::2], x[::2, 1::2], x[1::2, 1::2]); backward is the inverse copy.
template <typename T, int NV>
__global__ void s2d_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps, int N, int H, int W, int C,
                           int backward) {
  const int OH = H / 2, OW = W / 2, CV = C / NV;
  const long total = (long)N * OH * OW * 4 * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % CV) * NV;
    long t = i / CV;
    const int q = (int)(t % 4);
    t /= 4;
    const int w = (int)(t % OW);
    t /= OW;
    const int h = (int)(t % OH);
    const int b = (int)(t / OH);
    const int dy = q & 1, dx = q >> 1;
    const long xi = (((long)b * H + 2 * h + dy) * W + 2 * w + dx) * xps + c;
    const long yi = (((long)b * OH + h) * OW + w) * yps + q * C + c;
    float v[NV];
    if (backward) {
      ldv<T, NV>(y + yi, v);
      stv<T, NV>(const_cast<T*>(x) + xi, v);
    } else {
      ldv<T, NV>(x + xi, v);
      stv<T, NV>(y + yi, v);
    }
  }
}

// ---------------------------------------------------------------- CBAM (models/common.py:260-310)
// channel attention: [avg; max] global pools -> shared MLP (conv kernels) -> sigmoid(sum of halves);
// spatial attention: out1 = x * ca, s2 = [mean_c out1, max_c out1] -> 7x7 conv + sigmoid (conv kernels)
// -> out = out1 * sa.  Max-pool gradients go to the first maximum (torch's index semantics).
// Stage 1: grid (S pixel chunks, N, channel groups).  A workgroup is L lanes across NV-wide channel
// vectors x (256 / L) pixel parts; each lane scans its pixels in increasing order (first max wins),
// the parts merge in LDS (equal max -> smaller pixel), and the chunk's (sum, max, argmax) partials go
// to the fp32/int workspace [3][S][N][C].  Stage 2 folds the S chunks in order, so the result is
// deterministic and the argmax is the first maximum in pixel order (AdaptiveMaxPool2d's rule).
template <typename T, int NV>
__global__ void __launch_bounds__(256) gpool_part_kernel(const T* __restrict__ x, long xps, int N, int HW, int C, int L,
                                                         int chunk, float* __restrict__ ws) {
  const int S = gridDim.x, s = blockIdx.x, n = blockIdx.y;
  const int lane = threadIdx.x % L, part = threadIdx.x / L, parts = 256 / L;
  const int c = (blockIdx.z * L + lane) * NV;
  __shared__ float ss[256 * NV], sm[256 * NV];
  __shared__ int sa[256 * NV];
  float sum[NV], mx[NV];
  int am[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) { sum[j] = 0.f; mx[j] = -INFINITY; am[j] = 0x7fffffff; }
  const int p0 = s * chunk, p1 = min(HW, p0 + chunk);
  if (c < C) {
    const T* xb = x + (long)n * HW * xps + c;
    for (int p = p0 + part; p < p1; p += parts) {
      float v[NV];
      ldv<T, NV>(xb + (long)p * xps, v);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        sum[j] += v[j];
        const bool up = v[j] > mx[j];
        mx[j] = up ? v[j] : mx[j];
        am[j] = up ? p : am[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    ss[threadIdx.x * NV + j] = sum[j];
    sm[threadIdx.x * NV + j] = mx[j];
    sa[threadIdx.x * NV + j] = am[j];
  }
  __syncthreads();
  if (part == 0 && c < C) {
    const long plane = (long)S * N * C;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      float t = 0.f, m = -INFINITY;
      int a = 0x7fffffff;
      for (int q = 0; q < parts; ++q) {
        const int e = (q * L + lane) * NV + j;
        t += ss[e];
        if (sm[e] > m || (sm[e] == m && sa[e] < a)) { m = sm[e]; a = sa[e]; }
      }
      const long o = ((long)s * N + n) * C + c + j;
      ws[o] = t;
      ws[plane + o] = m;
      reinterpret_cast<int*>(ws)[2 * plane + o] = a;
    }
  }
}

template <typename T>
__global__ void gpool_final_kernel(const float* __restrict__ ws, int S, int N, int HW, int C, T* __restrict__ out,
                                   int* __restrict__ arg) {
  const long NC = (long)N * C, plane = (long)S * NC;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < NC; i += (long)gridDim.x * blockDim.x) {
    float t = 0.f, m = -INFINITY;
    int a = 0x7fffffff;
    for (int s = 0; s < S; ++s) {
      const long o = s * NC + i;
      t += ws[o];
      const float mm = ws[plane + o];
      const int aa = reinterpret_cast<const int*>(ws)[2 * plane + o];
      if (mm > m || (mm == m && aa < a)) { m = mm; a = aa; }
    }
    if (a == 0x7fffffff) a = 0;  // all -inf: the first pixel (ATen starts from index 0)
    const int n = (int)(i / C), c = (int)(i % C);
    out[(long)n * C + c] = from_f<T>(t / HW);
    out[(long)(N + n) * C + c] = from_f<T>(m);
    arg[i] = a;
  }
}

template <typename T, int NV>
__global__ void gpool_bwd_kernel(const T* __restrict__ dz, const int* __restrict__ arg, T* __restrict__ dx, long dxps,
                                 int accumulate, int N, int HW, int C) {
  const int CV = C / NV;
  const long total = (long)N * HW * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % CV) * NV;
    const long t = i / CV;
    const int p = (int)(t % HW), n = (int)(t / HW);
    float v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      v[j] = to_f(dz[(long)n * C + c + j]) / HW;
      if (arg[(long)n * C + c + j] == p) v[j] += to_f(dz[(long)(N + n) * C + c + j]);
    }
    T* o = dx + ((long)n * HW + p) * dxps + c;
    if (accumulate) {
      float d[NV];
      ldv<T, NV>(o, d);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] += d[j];
    }
    stv<T, NV>(o, v);
  }
}

// ca = sigmoid(z[:N] + z[N:]) (the two MLP branches); backward gives both halves the same gradient
template <typename T>
__global__ void halves_sigmoid_kernel(const T* __restrict__ z, int N, int C, T* __restrict__ ca, const T* __restrict__ dca,
                                      T* __restrict__ dz) {
  const long total = (long)N * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const float u = to_f(from_f<T>(to_f(z[i]) + to_f(z[i + total])));
    const float s = sigmoidf_(u);
    if (dca == nullptr) {
      ca[i] = from_f<T>(s);
    } else {
      const float g = to_f(dca[i]) * s * (1.f - s);
      dz[i] = from_f<T>(g);
      dz[i + total] = from_f<T>(g);
    }
  }
}

// one wave per pixel: out1 = x * ca, s2 = (mean_c out1, max_c out1), am = first argmax channel
template <typename T, int NV>
__global__ void __launch_bounds__(256) cbam_in_fwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ ca,
                                                          int N, int HW, int C, T* __restrict__ out1,
                                                          T* __restrict__ s2, int* __restrict__ am) {
  const int lane = threadIdx.x & 63;
  const long P = (long)N * HW;
  for (long pix = blockIdx.x * 4L + (threadIdx.x >> 6); pix < P; pix += gridDim.x * 4L) {
    const int n = (int)(pix / HW);
    float s = 0.f, mx = -INFINITY;
    int a = 0x7fffffff;
    for (int c0 = lane * NV; c0 < C; c0 += 64 * NV) {
      float xv[NV], cv[NV];
      ldv<T, NV>(x + pix * xps + c0, xv);
      ldv<T, NV>(ca + (long)n * C + c0, cv);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        xv[j] = to_f(from_f<T>(xv[j] * cv[j]));
        s += xv[j];
        if (xv[j] > mx) { mx = xv[j]; a = c0 + j; }
      }
      stv<T, NV>(out1 + pix * C + c0, xv);
    }
    s = wave_sum(s);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(mx, o, 64);
      const int a2 = __shfl_xor(a, o, 64);
      if (m2 > mx || (m2 == mx && a2 < a)) { mx = m2; a = a2; }
    }
    if (lane == 0) {
      s2[pix * 2] = from_f<T>(s / C);
      s2[pix * 2 + 1] = from_f<T>(mx);
      am[pix] = a;
    }
  }
}

// backward: d_out1 total = d_out1 + d_mean / C + [c == am] d_max;  dx = total * ca;
// wave w takes pixels [(w % wpi) * ppw, +ppw) of image w / wpi and writes its partial sum over them of total * x to
// part[w][c]; cbam_fold_kernel adds an image's wpi partials in wave order (deterministic, no float atomics)
template <typename T, int NV>
__global__ void __launch_bounds__(256) cbam_in_bwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ ca,
                                                          const T* __restrict__ dout1, long dps, const T* __restrict__ ds2,
                                                          const int* __restrict__ am, int N, int HW, int C, int ppw,
                                                          int wpi, T* __restrict__ dx, long dxps, int accumulate,
                                                          float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (w >= (long)N * wpi) return;
  const int n = (int)(w / wpi);
  const long p0 = (long)n * HW + (w % wpi) * (long)ppw;
  const long p1 = min((long)(n + 1) * HW, p0 + ppw);
  for (int c0 = lane * NV; c0 < C; c0 += 64 * NV) {
    float acc[NV], cv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = 0.f;
    ldv<T, NV>(ca + (long)n * C + c0, cv);
    for (long pix = p0; pix < p1; ++pix) {
      float xv[NV], gv[NV];
      ldv<T, NV>(x + pix * xps + c0, xv);
      ldv<T, NV>(dout1 + pix * dps + c0, gv);
      const float gm = to_f(ds2[pix * 2]) / C, gx = to_f(ds2[pix * 2 + 1]);
      const int a = am[pix];
      float o[NV];
      if (accumulate) ldv<T, NV>(dx + pix * dxps + c0, o);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const float t = gv[j] + gm + (c0 + j == a ? gx : 0.f);
        acc[j] += t * xv[j];
        o[j] = (accumulate ? o[j] : 0.f) + t * cv[j];
      }
      stv<T, NV>(dx + pix * dxps + c0, o);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) part[w * C + c0 + j] = acc[j];
  }
}

__global__ void cbam_fold_kernel(const float* __restrict__ part, int N, int C, int wpi, float* __restrict__ dca) {
  const long total = (long)N * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / C), c = (int)(i % C);
    const float* q = part + (long)n * wpi * C + c;
    float s = 0.f;
    for (int j = 0; j < wpi; ++j) s += q[(long)j * C];
    dca[i] = s;
  }
}

// out = out1 * sa (sa one value per pixel);  backward: d_out1 = d_out * sa, d_sa = sum_c d_out * out1
template <typename T, int NV>
__global__ void __launch_bounds__(256) pixscale_kernel(const T* __restrict__ out1, const T* __restrict__ sa, long sps,
                                                       int N, int HW, int C, T* __restrict__ out, long ops,
                                                       const T* __restrict__ dout, long dps, T* __restrict__ dout1,
                                                       T* __restrict__ dsa) {
  const int lane = threadIdx.x & 63;
  const long P = (long)N * HW;
  for (long pix = blockIdx.x * 4L + (threadIdx.x >> 6); pix < P; pix += gridDim.x * 4L) {
    const float sv = to_f(sa[pix * sps]);
    float s = 0.f;
    for (int c0 = lane * NV; c0 < C; c0 += 64 * NV) {
      float a[NV];
      ldv<T, NV>(out1 + pix * C + c0, a);
      if (dout == nullptr) {
#pragma unroll
        for (int j = 0; j < NV; ++j) a[j] *= sv;
        stv<T, NV>(out + pix * ops + c0, a);
      } else {
        float g[NV], d[NV];
        ldv<T, NV>(dout + pix * dps + c0, g);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          s += g[j] * a[j];
          d[j] = g[j] * sv;
        }
        stv<T, NV>(dout1 + pix * C + c0, d);
      }
    }
    if (dout != nullptr) {
      s = wave_sum(s);
      if (lane == 0) dsa[pix] = from_f<T>(s);
    }
  }
}

// ---------------------------------------------------------------- channel-slice copy with BiFPN weight
// scale = wvec ? wvec[idx] / (sum(wvec[0..nw)) + eps) : 1
DEV float bifpn_scale(const float* wv, int idx, int nw, float eps) {
  if (!wv) return 1.f;
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += wv[i];
  return wv[idx] / (s + eps);
}

template <typename T, bool VEC>
__global__ void slice_copy_kernel(const T* __restrict__ src, long sps, T* __restrict__ dst, long dps, long M, int C,
                                  const float* __restrict__ wv, int idx, int nw, float eps, int accumulate) {
  constexpr int VW = Traits<T>::VW;
  const float sc = bifpn_scale(wv, idx, nw, eps);
  const int cv = VEC ? C / VW : C;
  const long total = M * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long m;
    int c;
    divmod(i, cv, m, c);
    c *= VEC ? VW : 1;
    if (VEC) {
      float f[VW];
      unpack<T>(*reinterpret_cast<const uint4*>(src + m * sps + c), f);
      if (accumulate) {
        float g[VW];
        unpack<T>(*reinterpret_cast<const uint4*>(dst + m * dps + c), g);
#pragma unroll
        for (int j = 0; j < VW; ++j) f[j] = f[j] * sc + g[j];
      } else {
#pragma unroll
        for (int j = 0; j < VW; ++j) f[j] *= sc;
      }
      *reinterpret_cast<uint4*>(dst + m * dps + c) = pack<T>(f);
    } else {
      float v = to_f(src[m * sps + c]) * sc;
      if (accumulate) v += to_f(dst[m * dps + c]);
      dst[m * dps + c] = from_f<T>(v);
    }
  }
}

// per-block partial of sum(a*b) over a [M][C] slice pair
template <typename T, int NV>
__global__ void dot_partial_kernel(const T* __restrict__ a, long aps, const T* __restrict__ b, long bps, long M,
                                   int C, float* __restrict__ part) {
  const int CV = C / NV;
  const long total = M * CV;
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / CV;
    const int c = (int)(i % CV) * NV;
    float av[NV], bv[NV];
    ldv<T, NV>(a + m * aps + c, av);
    ldv<T, NV>(b + m * bps + c, bv);
#pragma unroll
    for (int j = 0; j < NV; ++j) s += av[j] * bv[j];
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// BiFPN weighted-concat backward of one input in one pass over its dy slice: g (+)= scale * dy (slice_copy_kernel's
// arithmetic) and the block partial of sum(dy * x) (dot_partial_kernel's, same grid-stride element order per thread),
// reading dy once instead of once per kernel
template <typename T>
__global__ void slice_copy_dot_kernel(const T* __restrict__ dy, long dps, T* __restrict__ g, long gps,
                                      const T* __restrict__ x, long xps, long M, int C, const float* __restrict__ wv,
                                      int idx, int nw, float eps, int accumulate, float* __restrict__ part) {
  constexpr int VW = Traits<T>::VW;
  const float sc = bifpn_scale(wv, idx, nw, eps);
  const int cv = C / VW;
  const long total = M * cv;
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long m;
    int c;
    divmod(i, cv, m, c);
    c *= VW;
    float f[VW], xv[VW];
    unpack<T>(*reinterpret_cast<const uint4*>(dy + m * dps + c), f);
    unpack<T>(*reinterpret_cast<const uint4*>(x + m * xps + c), xv);
#pragma unroll
    for (int j = 0; j < VW; ++j) s += f[j] * xv[j];
    if (accumulate) {
      float o[VW];
      unpack<T>(*reinterpret_cast<const uint4*>(g + m * gps + c), o);
#pragma unroll
      for (int j = 0; j < VW; ++j) f[j] = f[j] * sc + o[j];
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) f[j] *= sc;
    }
    *reinterpret_cast<uint4*>(g + m * gps + c) = pack<T>(f);
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// dw_j = sum_i g_i * d(scale_i)/d(w_j),  scale_i = w_i / S, S = sum(w) + eps
__global__ void bifpn_wgrad_kernel(const float* __restrict__ part, int nblk, int nw, const float* __restrict__ wv,
                                   float eps, float* __restrict__ dw) {
  __shared__ float g[4];
  if (threadIdx.x < (unsigned)nw) {
    float s = 0.f;
    for (int i = 0; i < nblk; ++i) s += part[threadIdx.x * nblk + i];
    g[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)nw) {
    float S = eps;
    for (int i = 0; i < nw; ++i) S += wv[i];
    const int j = threadIdx.x;
    float d = 0.f;
    for (int i = 0; i < nw; ++i) d += g[i] * ((i == j ? 1.f / S : 0.f) - wv[i] / (S * S));
    dw[j] = d;
  }
}

// ---------------------------------------------------------------- SCConv gate
// out = u3 * sigmoid(x + nearest(g))   with g the k2 branch at the pooled resolution
// torch computes sigmoid(add(identity, y_)) in storage precision, then mul: reproduced per element.
template <typename T, int NV>
__global__ void scgate_fwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ u3, const T* __restrict__ g,
                                  T* __restrict__ out, int N, int H, int W, int C, int GH, int GW) {
  const int CV = C / NV;
  const long total = (long)N * H * W * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, h, w, c;
    vidx(i, H, W, CV, NV, b, h, w, c);
    const long pix = ((long)b * H + h) * W + w;
    const int gh = nearest_src(h, GH, H), gw = nearest_src(w, GW, W);
    float xv[NV], gv[NV], uv[NV];
    ldv<T, NV>(x + pix * xps + c, xv);
    ldv<T, NV>(g + (((long)b * GH + gh) * GW + gw) * C + c, gv);
    ldv<T, NV>(u3 + pix * C + c, uv);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float sg = sigmoidf_(to_f(from_f<T>(xv[j] + gv[j])));
      uv[j] = uv[j] * to_f(from_f<T>(sg));
    }
    stv<T, NV>(out + pix * C + c, uv);
  }
}

// d u3 = dout * s ;  dpre = dout * u3 * s(1-s)  (-> dx contribution, written or accumulated into dpre)
template <typename T, int NV>
__global__ void scgate_bwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ u3, const T* __restrict__ g,
                                  const T* __restrict__ dout, T* __restrict__ du3, T* __restrict__ dpre, long dpps,
                                  int accumulate, int N, int H, int W, int C, int GH, int GW) {
  const int CV = C / NV;
  const long total = (long)N * H * W * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b, h, w, c;
    vidx(i, H, W, CV, NV, b, h, w, c);
    const long pix = ((long)b * H + h) * W + w;
    const int gh = nearest_src(h, GH, H), gw = nearest_src(w, GW, W);
    float xv[NV], gv[NV], uv[NV], dv[NV], pv[NV];
    ldv<T, NV>(x + pix * xps + c, xv);
    ldv<T, NV>(g + (((long)b * GH + gh) * GW + gw) * C + c, gv);
    ldv<T, NV>(u3 + pix * C + c, uv);
    ldv<T, NV>(dout + pix * C + c, dv);
    if (accumulate) ldv<T, NV>(dpre + pix * dpps + c, pv);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float sg = sigmoidf_(to_f(from_f<T>(xv[j] + gv[j])));
      const float dp = dv[j] * uv[j] * sg * (1.f - sg);
      pv[j] = accumulate ? pv[j] + dp : dp;
      uv[j] = dv[j] * sg;
    }
    stv<T, NV>(du3 + pix * C + c, uv);
    stv<T, NV>(dpre + pix * dpps + c, pv);
  }
}

// ---------------------------------------------------------------- CoorAttention
// y[b, h, c] = mean_w x ;  y[b, H + w, c] = mean_h x       (y is [N, H+W, C])
template <typename T>
__global__ void ca_pool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, int N, int H, int W, int C) {
  const long total = (long)N * (H + W) * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t;
    int c;
    divmod(i, C, t, c);
    const int r = (int)(t % (H + W));
    const int b = (int)(t / (H + W));
    float s = 0.f;
    if (r < H) {
      for (int w = 0; w < W; ++w) s += to_f(x[(((long)b * H + r) * W + w) * xps + c]);
      s /= (float)W;
    } else {
      const int w = r - H;
      for (int h = 0; h < H; ++h) s += to_f(x[(((long)b * H + h) * W + w) * xps + c]);
      s /= (float)H;
    }
    y[i] = from_f<T>(s);
  }
}

template <typename T>
__global__ void ca_pool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, long dxps, int accumulate, int N,
                                   int H, int W, int C) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t;
    int c;
    divmod(i, C, t, c);
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    float v = to_f(dy[((long)b * (H + W) + h) * C + c]) / (float)W +
              to_f(dy[((long)b * (H + W) + H + w) * C + c]) / (float)H;
    T* o = dx + (((long)b * H + h) * W + w) * dxps + c;
    if (accumulate) v += to_f(*o);
    *o = from_f<T>(v);
  }
}

// out = x * sigmoid(lw[b, H+w]) * sigmoid(lh[b, h])   (lh, lw: [N, H+W, C] logits of conv_h / conv_w)
template <typename T>
__global__ void ca_apply_fwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ lh,
                                    const T* __restrict__ lw, T* __restrict__ out, long ops, int N, int H, int W,
                                    int C) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t;
    int c;
    divmod(i, C, t, c);
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const long pix = ((long)b * H + h) * W + w;
    // x * a_w * a_h in fp32, rounded once to the storage type (round 6: the attention weights and x * a_w were rounded
    // to bf16 on the way, three extra roundings that put the bf16 output error at 1.8x the storage emulation's)
    const float ah = sigmoidf_(to_f(lh[((long)b * (H + W) + h) * C + c]));
    const float aw = sigmoidf_(to_f(lw[((long)b * (H + W) + H + w) * C + c]));
    const float xv = to_f(x[pix * xps + c]);
    out[pix * ops + c] = from_f<T>(xv * aw * ah);
  }
}

// dx = dout*aw*ah ; dlh[b,h] = sum_w dout*x*aw * ah(1-ah) ; dlw[b,H+w] = sum_h dout*x*ah * aw(1-aw)
template <typename T>
__global__ void ca_apply_bwd_dx_kernel(const T* __restrict__ x, long xps, const T* __restrict__ lh,
                                       const T* __restrict__ lw, const T* __restrict__ dout, long dps,
                                       T* __restrict__ dx, long dxps, int N, int H, int W, int C) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t;
    int c;
    divmod(i, C, t, c);
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const long pix = ((long)b * H + h) * W + w;
    const float ah = sigmoidf_(to_f(lh[((long)b * (H + W) + h) * C + c]));
    const float aw = sigmoidf_(to_f(lw[((long)b * (H + W) + H + w) * C + c]));
    dx[pix * dxps + c] = from_f<T>(to_f(dout[pix * dps + c]) * aw * ah);
  }
}

template <typename T>
__global__ void ca_apply_bwd_att_kernel(const T* __restrict__ x, long xps, const T* __restrict__ lh,
                                        const T* __restrict__ lw, const T* __restrict__ dout, long dps,
                                        T* __restrict__ dlh, T* __restrict__ dlw, int N, int H, int W, int C) {
  const long total = (long)N * (H + W) * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t;
    int c;
    divmod(i, C, t, c);
    const int r = (int)(t % (H + W));
    const int b = (int)(t / (H + W));
    float s = 0.f;
    if (r < H) {
      const float ah = sigmoidf_(to_f(lh[i]));
      for (int w = 0; w < W; ++w) {
        const long pix = ((long)b * H + r) * W + w;
        const float aw = sigmoidf_(to_f(lw[((long)b * (H + W) + H + w) * C + c]));
        s += to_f(dout[pix * dps + c]) * to_f(x[pix * xps + c]) * aw;
      }
      dlh[i] = from_f<T>(s * ah * (1.f - ah));
      dlw[i] = from_f<T>(0.f);
    } else {
      const int w = r - H;
      const float aw = sigmoidf_(to_f(lw[i]));
      for (int h = 0; h < H; ++h) {
        const long pix = ((long)b * H + h) * W + w;
        const float ah = sigmoidf_(to_f(lh[((long)b * (H + W) + h) * C + c]));
        s += to_f(dout[pix * dps + c]) * to_f(x[pix * xps + c]) * ah;
      }
      dlw[i] = from_f<T>(s * aw * (1.f - aw));
      dlh[i] = from_f<T>(0.f);
    }
  }
}

// ---------------------------------------------------------------- input normalisation / layout
// NCHW (uint8 or fp32) -> NHWC T, times `scale` (1/255 for uint8 images, train.py:402)
template <typename S, typename T>
__global__ void nchw_to_nhwc_kernel(const S* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W, int Cp,
                                    float scale) {
  // one thread per pixel: C plane reads (coalesced across threads along w), Cp contiguous writes
  // (16-B vectors when Cp*sizeof(T) is a multiple of 16); channels [C, Cp) are zero (stem padding)
  const long HW = (long)H * W, total = (long)N * HW;
  constexpr int VW = Traits<T>::VW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / HW, r = i % HW;
    const S* src = x + b * C * HW + r;
    T* dst = y + i * Cp;
    for (int c0 = 0; c0 < Cp; c0 += VW) {
      float f[VW];
#pragma unroll
      for (int j = 0; j < VW; ++j) f[j] = (c0 + j < C) ? (float)src[(long)(c0 + j) * HW] * scale : 0.f;
      if (c0 + VW <= Cp) {
        *reinterpret_cast<uint4*>(dst + c0) = pack<T>(f);
      } else {
        for (int j = 0; c0 + j < Cp; ++j) dst[c0 + j] = from_f<T>(f[j]);
      }
    }
  }
}

template <typename T, typename D>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ x, long xps, D* __restrict__ y, int N, int C, int H, int W) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    long t = i / W;
    const int h = (int)(t % H);
    t /= H;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    y[i] = (D)to_f(x[(((long)b * H + h) * W + w) * xps + c]);
  }
}

// ---------------------------------------------------------------- flat pointwise
// op: 0 y=a+b, 1 y=act(a), 2 y=dy*act'(a) (b=dy), 3 y=a*alpha, 4 y=a+alpha*b
template <typename T>
__global__ void pointwise_kernel(int op, int act, const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y,
                                 long n, float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float av = to_f(a[i]);
    float v;
    switch (op) {
      case 0: v = av + to_f(b[i]); break;
      case 1: v = act_fwd(act, av); break;
      case 2: v = to_f(b[i]) * act_grad(act, av); break;
      case 3: v = av * alpha; break;
      default: v = av + alpha * to_f(b[i]); break;
    }
    y[i] = from_f<T>(v);
  }
}

template <typename S, typename D>
__global__ void cast_kernel(const S* __restrict__ x, D* __restrict__ y, long n, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = from_f<D>(to_f(x[i]) * scale);
}

// grid of the grid-stride elementwise kernels: blocks of 256 threads, capped at 16384 (DMA-1536 step 157.61 / 157.98
// -> 158.13 / 158.32 img/s against 8192, alternating on one box, profiles/r05/elt_grid_ab.log)
inline int egrid(long n) { return grid_cap(ceil_div(n, 256), 16384); }

}  // namespace

#define DISPATCH_T(dtype, ...)         \
  if (dtype) {                         \
    using T = bf16;                    \
    __VA_ARGS__;                       \
  } else {                             \
    using T = float;                   \
    __VA_ARGS__;                       \
  }

// T = storage type; NV = 16-byte vector width when `vec` holds, else 1 (scalar)
#define DISPATCH_TV(dtype, vec, ...)                \
  if (dtype) {                                      \
    using T = bf16;                                 \
    if (vec) { constexpr int NV = 8; __VA_ARGS__; } \
    else { constexpr int NV = 1; __VA_ARGS__; }     \
  } else {                                          \
    using T = float;                                \
    if (vec) { constexpr int NV = 4; __VA_ARGS__; } \
    else { constexpr int NV = 1; __VA_ARGS__; }     \
  }

namespace {
// all channel counts / pixel strides multiples of the 16-B vector and all bases 16-B aligned
// Inference SPPF / SPPFCSPC pyramid (models/common.py:243-258, :1257-1276 under torch.no_grad): y1 = pool(x),
// y2 = pool(y1), y3 = pool(y2) with the same k x k stride-1 window, in ONE launch instead of three.  The tile is loaded
// with a 3P halo and the three pools run back to back in LDS, each over the region the next one needs, with
// out-of-image positions -inf at every stage, the row pass before the column pass, taps in increasing order and
// maxpool_fwd_lds's update rule (greater, or NaN): the bits of the three chained launches.  No argmax (no backward).
template <typename T, int K>
DEV void mp_stage(const uint4* src, int SW, uint4* rowb, uint4* dst, int DH, int DW, int gh0, int gw0, int H, int W) {
  // src: (DH + K - 1) x SW, SW = DW + K - 1, origin image (gh0 - P, gw0 - P); dst: DH x DW, origin (gh0, gw0)
  constexpr int NV = Traits<T>::VW, P = K / 2;
  const int SH = DH + K - 1;
  for (int e = threadIdx.x; e < SH * DW; e += 256) {
    const int r = e / DW, w = e % DW;
    float best[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) best[j] = -INFINITY;
#pragma unroll
    for (int dw = 0; dw < K; ++dw) {
      float v[NV];
      unpack<T>(src[r * SW + w + dw], v);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const unsigned up = (unsigned)(v[j] > best[j]) | (unsigned)__builtin_isnan(v[j]);
        best[j] = up ? v[j] : best[j];
      }
    }
    rowb[e] = pack<T>(best);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < DH * DW; e += 256) {
    const int h = e / DW, w = e % DW;
    float best[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) best[j] = -INFINITY;
    const int gh = gh0 + h, gw = gw0 + w;
    if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) {
#pragma unroll
      for (int dh = 0; dh < K; ++dh) {
        float v[NV];
        unpack<T>(rowb[(h + dh) * DW + w], v);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const unsigned up = (unsigned)(v[j] > best[j]) | (unsigned)__builtin_isnan(v[j]);
          best[j] = up ? v[j] : best[j];
        }
      }
    }
    dst[e] = pack<T>(best);  // -inf off the image: the next pool's padding
  }
  __syncthreads();
}

template <typename T, int K, int TH, int TW>
__global__ void __launch_bounds__(256) maxpool_chain3_lds(const T* __restrict__ x, long xps, T* __restrict__ y1,
                                                          T* __restrict__ y2, T* __restrict__ y3, long yps, int H, int W,
                                                          int C) {
  constexpr int NV = Traits<T>::VW, P = K / 2;
  constexpr int XH = TH + 6 * P, XW = TW + 6 * P;  // x with the 3P halo
  constexpr int AH = TH + 4 * P, AW = TW + 4 * P;  // y1 region (2P halo)
  __shared__ uint4 bufx[XH * XW];       // x, later y2
  __shared__ uint4 bufr[XH * AW];       // row-pass scratch (largest: stage 1)
  __shared__ uint4 bufa[AH * AW];       // y1
  // block -> (image, tile, channel vector), channel vector fastest (mp_tile's order, without its XCD grouping: these
  // grids are small)
  const int CV = C / NV, twn = (W + TW - 1) / TW, thn = (H + TH - 1) / TH;
  int L = (int)blockIdx.x;
  const int c = (L % CV) * NV;
  L /= CV;
  const int w0 = (L % twn) * TW;
  L /= twn;
  const int h0 = (L % thn) * TH, b = L / thn;
  const T* xb = x + (long)b * H * W * xps + c;
  float ninf[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) ninf[j] = -INFINITY;
  const uint4 pad = pack<T>(ninf);
  for (int e = threadIdx.x; e < XH * XW; e += 256) {
    const int hh = h0 - 3 * P + e / XW, ww = w0 - 3 * P + e % XW;
    bufx[e] = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                  ? *reinterpret_cast<const uint4*>(xb + ((long)hh * W + ww) * xps) : pad;
  }
  __syncthreads();
  mp_stage<T, K>(bufx, XW, bufr, bufa, AH, AW, h0 - 2 * P, w0 - 2 * P, H, W);   // y1 over the 2P halo
  constexpr int BH = TH + 2 * P, BW = TW + 2 * P;
  mp_stage<T, K>(bufa, AW, bufr, bufx, BH, BW, h0 - P, w0 - P, H, W);           // y2 over the P halo (into bufx)
  // y3 over the tile: into bufa (y1 is still needed for its store: stored first)
  for (int e = threadIdx.x; e < TH * TW; e += 256) {
    const int h = e / TW, w = e % TW, oh = h0 + h, ow = w0 + w;
    if (oh >= H || ow >= W) continue;
    const long pix = ((long)b * H + oh) * W + ow;
    *reinterpret_cast<uint4*>(y1 + pix * yps + c) = bufa[(h + 2 * P) * AW + w + 2 * P];
    *reinterpret_cast<uint4*>(y2 + pix * yps + c) = bufx[(h + P) * BW + w + P];
  }
  __syncthreads();
  mp_stage<T, K>(bufx, BW, bufr, bufa, TH, TW, h0, w0, H, W);
  for (int e = threadIdx.x; e < TH * TW; e += 256) {
    const int h = e / TW, w = e % TW, oh = h0 + h, ow = w0 + w;
    if (oh >= H || ow >= W) continue;
    *reinterpret_cast<uint4*>(y3 + (((long)b * H + oh) * W + ow) * yps + c) = bufa[e];
  }
}

inline bool vec_ok(int dtype, std::initializer_list<long> ns, std::initializer_list<const void*> ps) {
  const long VW = dtype ? 8 : 4;
  for (long n : ns)
    if (n % VW) return false;
  for (const void* p : ps)
    if (!al16(p)) return false;
  return true;
}
inline long vw_of(int dtype, bool vec) { return vec ? (dtype ? 8 : 4) : 1; }
}  // namespace

DMY_API int dmy_maxpool_fwd(int dtype, const void* x, long xps, void* y, long yps, unsigned char* arg, int N, int H,
                            int W, int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps, yps}, {x, y});
  if (k < 1 || k > 15 || (k & 1) == 0) return (int)hipErrorInvalidValue;  // uint8 window offsets
  if (v && N * (C / (dtype ? 8 : 4)) < 65536 && k >= 3 && k <= 13) {
    const unsigned gl = (unsigned)ceil_div(W, MP_TW) * ceil_div(H, MP_TH) * N * (C / (dtype ? 8 : 4));  // mp_tile order
#define MP_LDS(KS) if (dtype) maxpool_fwd_lds<bf16, KS><<<gl, 256, 0, st>>>((const bf16*)x, xps, (bf16*)y, yps, arg, H, W, C); \
                   else maxpool_fwd_lds<float, KS><<<gl, 256, 0, st>>>((const float*)x, xps, (float*)y, yps, arg, H, W, C)
    switch (k) {
      case 3: MP_LDS(3); break;
      case 5: MP_LDS(5); break;
      case 7: MP_LDS(7); break;
      case 9: MP_LDS(9); break;
      case 11: MP_LDS(11); break;
      default: MP_LDS(13); break;
    }
#undef MP_LDS
    return (int)hipGetLastError();
  }
  const int g = egrid((long)N * H * W * C / (v ? (dtype ? 8 : 4) : 1));
#define MP_FWD(KS) DISPATCH_TV(dtype, v, maxpool_fwd_kernel<T, NV, KS><<<g, 256, 0, st>>>((const T*)x, xps, (T*)y, yps, arg, N, H, W, C, k))
  switch ((long)H * W * xps < (1L << 31) ? k : 0) {  // compile-time windows use 32-bit in-image offsets
    case 3: MP_FWD(3); break;
    case 5: MP_FWD(5); break;
    case 7: MP_FWD(7); break;
    case 9: MP_FWD(9); break;
    case 11: MP_FWD(11); break;
    case 13: MP_FWD(13); break;
    default: MP_FWD(0); break;
  }
#undef MP_FWD
  return (int)hipGetLastError();
}
// y1 = pool(x), y2 = pool(y1), y3 = pool(y2) (k x k, stride 1, pad k / 2) in one launch, no argmax (inference); the
// three outputs share the pixel stride yps (three channel slices of one concat buffer, or three tensors)
DMY_API int dmy_maxpool_chain3_fwd(int dtype, const void* x, long xps, void* y1, void* y2, void* y3, long yps, int N,
                                   int H, int W, int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!vec_ok(dtype, {C, xps, yps}, {x, y1, y2, y3}) || (k != 3 && k != 5) || N * (C / (dtype ? 8 : 4)) >= 65536)
    return (int)hipErrorInvalidValue;
  // 16 x 32 tiles, or 8 x 16 when those leave most CUs idle (the 20^2 / 40^2 maps of batch-1 detect)
  const long cv = N * (C / (dtype ? 8 : 4));
  const bool small = cv * ceil_div(W, 32) * ceil_div(H, 16) < 256;
  const unsigned gl = (unsigned)(cv * (small ? ceil_div(W, 16) * ceil_div(H, 8) : ceil_div(W, 32) * ceil_div(H, 16)));
#define MP3(KS, TH, TW) if (dtype) maxpool_chain3_lds<bf16, KS, TH, TW><<<gl, 256, 0, st>>>((const bf16*)x, xps, (bf16*)y1, (bf16*)y2, (bf16*)y3, yps, H, W, C); \
                        else maxpool_chain3_lds<float, KS, TH, TW><<<gl, 256, 0, st>>>((const float*)x, xps, (float*)y1, (float*)y2, (float*)y3, yps, H, W, C)
  if (k == 5) {
    if (small) MP3(5, 8, 16);
    else MP3(5, 16, 32);
  } else {
    if (small) MP3(3, 8, 16);
    else MP3(3, 16, 32);
  }
#undef MP3
  return (int)hipGetLastError();
}
DMY_API int dmy_maxpool_bwd(int dtype, const void* dy, long dps, const unsigned char* arg, void* dx, long dxps,
                            int accumulate, int N, int H, int W, int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, dps, dxps}, {dy, dx});
  if (k < 1 || k > 15 || (k & 1) == 0) return (int)hipErrorInvalidValue;
  if (v && N * (C / (dtype ? 8 : 4)) < 65536 && k >= 3 && k <= 13) {
    const unsigned gl = (unsigned)ceil_div(W, MP_TW) * ceil_div(H, MP_TH) * N * (C / (dtype ? 8 : 4));  // mp_tile order
#define MP_LDS(KS) if (dtype) maxpool_bwd_lds<bf16, KS><<<gl, 256, 0, st>>>((const bf16*)dy, dps, arg, (bf16*)dx, dxps, accumulate, H, W, C); \
                   else maxpool_bwd_lds<float, KS><<<gl, 256, 0, st>>>((const float*)dy, dps, arg, (float*)dx, dxps, accumulate, H, W, C)
    switch (k) {
      case 3: MP_LDS(3); break;
      case 5: MP_LDS(5); break;
      case 7: MP_LDS(7); break;
      case 9: MP_LDS(9); break;
      case 11: MP_LDS(11); break;
      default: MP_LDS(13); break;
    }
#undef MP_LDS
    return (int)hipGetLastError();
  }
  DISPATCH_TV(dtype, v, maxpool_bwd_kernel<T, NV><<<egrid((long)N * H * W * C / NV), 256, 0, st>>>((const T*)dy, dps, arg, (T*)dx, dxps, accumulate, N, H, W, C, k));
  return (int)hipGetLastError();
}
DMY_API int dmy_avgpool_fwd(int dtype, const void* x, long xps, void* y, int N, int H, int W, int C, int r,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps}, {x, y});
  DISPATCH_TV(dtype, v, avgpool_fwd_kernel<T, NV><<<egrid((long)N * (H / r) * (W / r) * C / NV), 256, 0, st>>>((const T*)x, xps, (T*)y, N, H, W, C, r));
  return (int)hipGetLastError();
}
DMY_API int dmy_avgpool_bwd(int dtype, const void* dy, void* dx, long dxps, int accumulate, int N, int H, int W, int C,
                            int r, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, dxps}, {dy, dx});
  DISPATCH_TV(dtype, v, avgpool_bwd_kernel<T, NV><<<egrid((long)N * H * W * C / NV), 256, 0, st>>>((const T*)dy, (T*)dx, dxps, accumulate, N, H, W, C, r));
  return (int)hipGetLastError();
}
DMY_API int dmy_resize_fwd(int dtype, const void* x, long xps, void* y, long yps, float yscale, int N, int IH, int IW,
                           int OH, int OW, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps, yps}, {x, y});
  DISPATCH_TV(dtype, v, resize_fwd_kernel<T, NV><<<egrid((long)N * OH * OW * C / NV), 256, 0, st>>>((const T*)x, xps, (T*)y, yps, yscale, N, IH, IW, OH, OW, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_resize_bwd(int dtype, const void* dy, long dps, void* dx, long dxps, int N, int IH, int IW, int OH,
                           int OW, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, dps, dxps}, {dy, dx});
  DISPATCH_TV(dtype, v, resize_bwd_kernel<T, NV><<<egrid((long)N * IH * IW * C / NV), 256, 0, st>>>((const T*)dy, dps, (T*)dx, dxps, N, IH, IW, OH, OW, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_space_to_depth(int dtype, const void* x, long xps, void* y, long yps, int N, int H, int W, int C,
                               int backward, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if ((H | W) & 1) return (int)hipErrorInvalidValue;  // the reference's cat needs even sizes
  const bool v = vec_ok(dtype, {C, xps, yps}, {x, y});
  DISPATCH_TV(dtype, v, s2d_kernel<T, NV><<<egrid((long)N * H * W * C / NV), 256, 0, st>>>((const T*)x, xps, (T*)y, yps, N, H, W, C, backward));
  return (int)hipGetLastError();
}
namespace {
// pixel chunks of the global pool: about 2048 workgroups over (chunks x N x channel groups), >= 64
// pixels per chunk
struct GPoolPlan {
  int L, groups, S, chunk;
  GPoolPlan(int N, int HW, int C, int NV) {
    const int CV = ceil_div(C, NV);
    L = 1;
    while (L < CV && L < 256) L <<= 1;
    groups = ceil_div(CV, L);
    const long per = (long)N * groups;
    const long by_work = ceil_div((long)HW, 64L), by_grid = 2048L / (per > 0 ? per : 1L);
    S = (int)(by_work < by_grid ? by_work : by_grid);
    if (S < 1) S = 1;
    chunk = ceil_div(HW, S);
    S = ceil_div(HW, chunk);
  }
};
}  // namespace

DMY_API long dmy_gpool_ws_bytes(int dtype, int N, int HW, int C) {
  const GPoolPlan pl(N, HW, C, dtype ? 8 : 4);  // the vector plan has at least as many chunks as the scalar one
  const GPoolPlan ps(N, HW, C, 1);
  return 3L * (pl.S > ps.S ? pl.S : ps.S) * N * C * 4;
}
DMY_API int dmy_gpool_fwd(int dtype, const void* x, long xps, int N, int HW, int C, void* out, int* arg, float* ws,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps}, {x});
  const GPoolPlan pl(N, HW, C, (int)vw_of(dtype, v));
  const dim3 grid(pl.S, N, pl.groups);
  DISPATCH_TV(dtype, v, gpool_part_kernel<T, NV><<<grid, 256, 0, st>>>((const T*)x, xps, N, HW, C, pl.L, pl.chunk, ws));
  DISPATCH_T(dtype, gpool_final_kernel<T><<<egrid((long)N * C), 256, 0, st>>>(ws, pl.S, N, HW, C, (T*)out, arg));
  return (int)hipGetLastError();
}
DMY_API int dmy_gpool_bwd(int dtype, const void* dz, const int* arg, void* dx, long dxps, int accumulate, int N, int HW,
                          int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, dxps}, {dx});
  DISPATCH_TV(dtype, v, gpool_bwd_kernel<T, NV><<<egrid((long)N * HW * C / NV), 256, 0, st>>>((const T*)dz, arg, (T*)dx, dxps, accumulate, N, HW, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_halves_sigmoid(int dtype, const void* z, int N, int C, void* ca, const void* dca, void* dz, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, halves_sigmoid_kernel<T><<<egrid((long)N * C), 256, 0, st>>>((const T*)z, N, C, (T*)ca, (const T*)dca, (T*)dz));
  return (int)hipGetLastError();
}
DMY_API int dmy_cbam_in_fwd(int dtype, const void* x, long xps, const void* ca, int N, int HW, int C, void* out1, void* s2,
                            int* am, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps}, {x, ca, out1});
  DISPATCH_TV(dtype, v, cbam_in_fwd_kernel<T, NV><<<grid_cap(ceil_div((long)N * HW, 4), 8192), 256, 0, st>>>((const T*)x, xps, (const T*)ca, N, HW, C, (T*)out1, (T*)s2, am));
  return (int)hipGetLastError();
}
static const int kCbamPpw = 64;  // pixels per wave of cbam_in_bwd_kernel
DMY_API long dmy_cbam_in_bwd_ws_elems(int N, int HW, int C) {
  return (long)N * ceil_div((long)HW, kCbamPpw) * C;
}
DMY_API int dmy_cbam_in_bwd(int dtype, const void* x, long xps, const void* ca, const void* dout1, long dps,
                            const void* ds2, const int* am, int N, int HW, int C, void* dx, long dxps, int accumulate,
                            float* dca, float* ws, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps, dps, dxps}, {x, ca, dout1, dx});
  const int wpi = (int)ceil_div((long)HW, kCbamPpw);
  const long waves = (long)N * wpi;
  DISPATCH_TV(dtype, v, cbam_in_bwd_kernel<T, NV><<<(unsigned)ceil_div(waves, 4), 256, 0, st>>>((const T*)x, xps, (const T*)ca, (const T*)dout1, dps, (const T*)ds2, am, N, HW, C, kCbamPpw, wpi, (T*)dx, dxps, accumulate, ws));
  cbam_fold_kernel<<<grid_cap(ceil_div((long)N * C, 256)), 256, 0, st>>>(ws, N, C, wpi, dca);
  return (int)hipGetLastError();
}
DMY_API int dmy_pixscale(int dtype, const void* out1, const void* sa, long sps, int N, int HW, int C, void* out, long ops,
                         const void* dout, long dps, void* dout1, void* dsa, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, ops, dout ? dps : 0}, {out1, out, dout, dout1});
  DISPATCH_TV(dtype, v, pixscale_kernel<T, NV><<<grid_cap(ceil_div((long)N * HW, 4), 8192), 256, 0, st>>>((const T*)out1, (const T*)sa, sps, N, HW, C, (T*)out, ops, (const T*)dout, dps, (T*)dout1, (T*)dsa));
  return (int)hipGetLastError();
}
DMY_API int dmy_slice_copy(int dtype, const void* src, long sps, void* dst, long dps, long M, int C, const float* wv,
                           int idx, int nw, float eps, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int VW = dtype ? 8 : 4;
  const bool vec = C % VW == 0 && sps % VW == 0 && dps % VW == 0 && al16(src) && al16(dst);
  const long work = M * (vec ? C / VW : C);
  if (vec) {
    DISPATCH_T(dtype, slice_copy_kernel<T, true><<<egrid(work), 256, 0, st>>>((const T*)src, sps, (T*)dst, dps, M, C, wv, idx, nw, eps, accumulate));
  } else {
    DISPATCH_T(dtype, slice_copy_kernel<T, false><<<egrid(work), 256, 0, st>>>((const T*)src, sps, (T*)dst, dps, M, C, wv, idx, nw, eps, accumulate));
  }
  return (int)hipGetLastError();
}
DMY_API int dmy_dot_partial_blocks(long M, int C) { return grid_cap(ceil_div(M * C, 256 * 64), 2048); }
DMY_API int dmy_dot_partial(int dtype, const void* a, long aps, const void* b, long bps, long M, int C, float* part,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int nb = dmy_dot_partial_blocks(M, C);
  const bool v = vec_ok(dtype, {C, aps, bps}, {a, b});
  DISPATCH_TV(dtype, v, dot_partial_kernel<T, NV><<<nb, 256, 0, st>>>((const T*)a, aps, (const T*)b, bps, M, C, part));
  return (int)hipGetLastError();
}
// dmy_slice_copy (accumulate as given) + dmy_dot_partial(dy, x) in one launch; part gets dmy_dot_partial_blocks(M, C)
// partials.  16-B vectors only (returns hipErrorInvalidValue otherwise: use the two calls)
DMY_API int dmy_slice_copy_dot(int dtype, const void* dy, long dps, void* g, long gps, const void* x, long xps, long M,
                               int C, const float* wv, int idx, int nw, float eps, int accumulate, float* part,
                               void* stream) {
  if (!vec_ok(dtype, {C, dps, gps, xps}, {dy, g, x})) return (int)hipErrorInvalidValue;
  const int nb = dmy_dot_partial_blocks(M, C);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, slice_copy_dot_kernel<T><<<nb, 256, 0, st>>>((const T*)dy, dps, (T*)g, gps, (const T*)x, xps, M, C,
                                                                  wv, idx, nw, eps, accumulate, part));
  return (int)hipGetLastError();
}
DMY_API int dmy_bifpn_wgrad(const float* part, int nblk, int nw, const float* wv, float eps, float* dw, void* stream) {
  bifpn_wgrad_kernel<<<1, 64, 0, (hipStream_t)stream>>>(part, nblk, nw, wv, eps, dw);
  return (int)hipGetLastError();
}
DMY_API int dmy_scgate_fwd(int dtype, const void* x, long xps, const void* u3, const void* g, void* out, int N, int H,
                           int W, int C, int GH, int GW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps}, {x, u3, g, out});
  DISPATCH_TV(dtype, v, scgate_fwd_kernel<T, NV><<<egrid((long)N * H * W * C / NV), 256, 0, st>>>((const T*)x, xps, (const T*)u3, (const T*)g, (T*)out, N, H, W, C, GH, GW));
  return (int)hipGetLastError();
}
DMY_API int dmy_scgate_bwd(int dtype, const void* x, long xps, const void* u3, const void* g, const void* dout,
                           void* du3, void* dpre, long dpps, int accumulate, int N, int H, int W, int C, int GH, int GW,
                           void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(dtype, {C, xps, dpps}, {x, u3, g, dout, du3, dpre});
  DISPATCH_TV(dtype, v, scgate_bwd_kernel<T, NV><<<egrid((long)N * H * W * C / NV), 256, 0, st>>>((const T*)x, xps, (const T*)u3, (const T*)g, (const T*)dout, (T*)du3, (T*)dpre, dpps, accumulate, N, H, W, C, GH, GW));
  return (int)hipGetLastError();
}
DMY_API int dmy_ca_pool_fwd(int dtype, const void* x, long xps, void* y, int N, int H, int W, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, ca_pool_fwd_kernel<T><<<egrid((long)N * (H + W) * C), 256, 0, st>>>((const T*)x, xps, (T*)y, N, H, W, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_ca_pool_bwd(int dtype, const void* dy, void* dx, long dxps, int accumulate, int N, int H, int W, int C,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, ca_pool_bwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)dy, (T*)dx, dxps, accumulate, N, H, W, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_ca_apply_fwd(int dtype, const void* x, long xps, const void* lh, const void* lw, void* out, long ops,
                             int N, int H, int W, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, ca_apply_fwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)x, xps, (const T*)lh, (const T*)lw, (T*)out, ops, N, H, W, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_ca_apply_bwd(int dtype, const void* x, long xps, const void* lh, const void* lw, const void* dout,
                             long dps, void* dx, long dxps, void* dlh, void* dlw, int N, int H, int W, int C,
                             void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, ca_apply_bwd_dx_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)x, xps, (const T*)lh, (const T*)lw, (const T*)dout, dps, (T*)dx, dxps, N, H, W, C));
  DISPATCH_T(dtype, ca_apply_bwd_att_kernel<T><<<egrid((long)N * (H + W) * C), 256, 0, st>>>((const T*)x, xps, (const T*)lh, (const T*)lw, (const T*)dout, dps, (T*)dlh, (T*)dlw, N, H, W, C));
  return (int)hipGetLastError();
}
// NCHW image (uint8 or fp32, H and W even) -> space-to-depth NHWC [N][H/2][W/2][Cs] T, channel
// (dy * 2 + dx) * C + c = x[c][2 oy + dy][2 ox + dx] * scale, channels [4C, Cs) zero.  The k6 s2 p2 stem
// conv (models/common.py:50-77 with yolov5*.yaml layer 0 args [64, 6, 2, 2]) over x equals a k3 s1 p1
// conv over this tensor (DESIGN.md §3.1 "stem"): half the stem's input bytes of the 8-channel padded
// layout and a dense 3x3 contraction instead of a stride-2 6x6 gather.
template <typename S, typename T>
__global__ void image_s2d_kernel(const S* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W, int Cs,
                                 float scale) {
  constexpr int VW = Traits<T>::VW;
  const int H2 = H >> 1, W2 = W >> 1;
  const long HW = (long)H * W, total = (long)N * H2 * W2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % W2);
    const long t = i / W2;
    const int oy = (int)(t % H2);
    const long b = t / H2;
    const S* src = x + b * C * HW + (long)(2 * oy) * W + 2 * ox;
    T* dst = y + i * Cs;
    for (int c0 = 0; c0 < Cs; c0 += VW) {
      float f[VW];
#pragma unroll
      for (int j = 0; j < VW; ++j) {
        const int ch = c0 + j;
        if (ch < 4 * C) {
          const int q = ch / C, c = ch - q * C;  // q = dy * 2 + dx
          f[j] = (float)src[(long)c * HW + (q >> 1) * W + (q & 1)] * scale;
        } else {
          f[j] = 0.f;
        }
      }
      *reinterpret_cast<uint4*>(dst + c0) = pack<T>(f);
    }
  }
}

DMY_API int dmy_image_s2d(int dtype, int src_kind, const void* x, void* y, int N, int C, int H, int W, int Cs,
                          float scale, void* stream) {
  const int VW = dtype ? 8 : 4;
  if ((H | W) & 1 || Cs % VW || Cs < 4 * C || (((uintptr_t)y) & 15)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)N * (H / 2) * (W / 2);
  if (src_kind == 0) {
    DISPATCH_T(dtype, image_s2d_kernel<uint8_t, T><<<egrid(n), 256, 0, st>>>((const uint8_t*)x, (T*)y, N, C, H, W, Cs, scale));
  } else {
    DISPATCH_T(dtype, image_s2d_kernel<float, T><<<egrid(n), 256, 0, st>>>((const float*)x, (T*)y, N, C, H, W, Cs, scale));
  }
  return (int)hipGetLastError();
}
// src_kind: 0 = uint8, 1 = fp32; output NHWC with pixel stride Cp >= C (zero-filled tail channels)
DMY_API int dmy_nchw_to_nhwc(int dtype, int src_kind, const void* x, void* y, int N, int C, int H, int W, int Cp,
                             float scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)N * H * W;
  if (src_kind == 0) {
    DISPATCH_T(dtype, nchw_to_nhwc_kernel<uint8_t, T><<<egrid(n), 256, 0, st>>>((const uint8_t*)x, (T*)y, N, C, H, W, Cp, scale));
  } else {
    DISPATCH_T(dtype, nchw_to_nhwc_kernel<float, T><<<egrid(n), 256, 0, st>>>((const float*)x, (T*)y, N, C, H, W, Cp, scale));
  }
  return (int)hipGetLastError();
}
DMY_API int dmy_nhwc_to_nchw_f32(int dtype, const void* x, long xps, float* y, int N, int C, int H, int W,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, nhwc_to_nchw_kernel<T, float><<<egrid((long)N * C * H * W), 256, 0, st>>>((const T*)x, xps, y, N, C, H, W));
  return (int)hipGetLastError();
}
DMY_API int dmy_pointwise(int dtype, int op, int act, const void* a, const void* b, void* y, long n, float alpha,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, pointwise_kernel<T><<<egrid(n), 256, 0, st>>>(op, act, (const T*)a, (const T*)b, (T*)y, n, alpha));
  return (int)hipGetLastError();
}
// kinds: 0 f32, 1 bf16
DMY_API int dmy_cast(int src_kind, int dst_kind, const void* x, void* y, long n, float scale, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int g = egrid(n);
  if (src_kind == 0 && dst_kind == 1) cast_kernel<float, bf16><<<g, 256, 0, st>>>((const float*)x, (bf16*)y, n, scale);
  else if (src_kind == 1 && dst_kind == 0) cast_kernel<bf16, float><<<g, 256, 0, st>>>((const bf16*)x, (float*)y, n, scale);
  else if (src_kind == 0) cast_kernel<float, float><<<g, 256, 0, st>>>((const float*)x, (float*)y, n, scale);
  else cast_kernel<bf16, bf16><<<g, 256, 0, st>>>((const bf16*)x, (bf16*)y, n, scale);
  return (int)hipGetLastError();
}
