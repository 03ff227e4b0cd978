// Memory-bound NHWC kernels of the DMA-YOLO path (HBM roofline):
//   max-pool k5 s1 (SPPF models/common.py:243-258, SPPFCSPC :1257-1276), avg-pool r (SCConv k2 :1282),
//   nearest resize (nn.Upsample yaml:31/36, F.interpolate in SCConv :1311), channel-slice copy with
//   BiFPN weights (Concat :656-664, AdConcat2/3 :994-1026), SCConv gate (:1311-1314),
//   CoorAttention pooling / re-weighting (:1183-1207), input normalisation (train.py:402).
#include "common.h"

namespace {

inline bool al16(const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; }

// ---------------------------------------------------------------- max-pool (k odd, stride 1, pad k/2)
// Writes the first-max window offset (row-major scan, like ATen's CPU kernel) for the backward.
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps,
                                   uint8_t* __restrict__ arg, int N, int H, int W, int C, int k) {
  const long total = (long)N * H * W * C;
  const int p = k / 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    float best = -INFINITY;
    int bi = 0;
    for (int dh = 0; dh < k; ++dh) {
      const int hh = h - p + dh;
      if (hh < 0 || hh >= H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int ww = w - p + dw;
        if (ww < 0 || ww >= W) continue;
        const float v = to_f(x[(((long)b * H + hh) * W + ww) * xps + c]);
        if (v > best || isnan(v)) {
          best = v;
          bi = dh * k + dw;
          if (isnan(v)) { dh = k; break; }
        }
      }
    }
    const long pix = ((long)b * H + h) * W + w;
    y[pix * yps + c] = from_f<T>(best);
    arg[pix * C + c] = (uint8_t)bi;
  }
}

// dx[p] = sum of dy[q] over windows q whose argmax is p (gather: deterministic, no atomics)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, long dps, const uint8_t* __restrict__ arg,
                                   T* __restrict__ dx, long dxps, int accumulate, int N, int H, int W, int C, int k) {
  const long total = (long)N * H * W * C;
  const int p = k / 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    float s = 0.f;
    for (int oh = h - p; oh <= h + p; ++oh) {
      if (oh < 0 || oh >= H) continue;
      for (int ow = w - p; ow <= w + p; ++ow) {
        if (ow < 0 || ow >= W) continue;
        const long q = ((long)b * H + oh) * W + ow;
        const int a = arg[q * C + c];
        if (a == (h - oh + p) * k + (w - ow + p)) s += to_f(dy[q * dps + c]);
      }
    }
    T* o = dx + (((long)b * H + h) * W + w) * dxps + c;
    if (accumulate) s += to_f(*o);
    *o = from_f<T>(s);
  }
}

// ---------------------------------------------------------------- avg-pool r x r, stride r, floor mode
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, int N, int H, int W, int C,
                                   int r) {
  const int OH = H / r, OW = W / r;
  const long total = (long)N * OH * OW * C;
  const float inv = 1.0f / (r * r);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int b = (int)(t / OH);
    float s = 0.f;
    for (int dh = 0; dh < r; ++dh)
      for (int dw = 0; dw < r; ++dw) s += to_f(x[(((long)b * H + oh * r + dh) * W + ow * r + dw) * xps + c]);
    y[i] = from_f<T>(s * inv);
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, long dxps, int accumulate, int N,
                                   int H, int W, int C, int r) {
  const int OH = H / r, OW = W / r;
  const long total = (long)N * H * W * C;
  const float inv = 1.0f / (r * r);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const int oh = h / r, ow = w / r;
    float v = (oh < OH && ow < OW) ? to_f(dy[(((long)b * OH + oh) * OW + ow) * C + c]) * inv : 0.f;
    T* o = dx + (((long)b * H + h) * W + w) * dxps + c;
    if (accumulate) v += to_f(*o);
    *o = from_f<T>(v);
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

template <typename T>
__global__ void resize_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, long yps, float yscale,
                                  int N, int IH, int IW, int OH, int OW, int C) {
  const long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int b = (int)(t / OH);
    const int ih = nearest_src(oh, IH, OH), iw = nearest_src(ow, IW, OW);
    y[(((long)b * OH + oh) * OW + ow) * yps + c] = from_f<T>(yscale * to_f(x[(((long)b * IH + ih) * IW + iw) * xps + c]));
  }
}

// dx[ih,iw] = sum over dst (oh,ow) mapping to it; preimages are contiguous ranges
template <typename T>
__global__ void resize_bwd_kernel(const T* __restrict__ dy, long dps, T* __restrict__ dx, long dxps, int N, int IH,
                                  int IW, int OH, int OW, int C) {
  const long total = (long)N * IH * IW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int iw = (int)(t % IW);
    t /= IW;
    const int ih = (int)(t % IH);
    const int b = (int)(t / IH);
    const int h0 = max(0, (int)((long)ih * OH / IH) - 2), h1 = min(OH - 1, (int)((long)(ih + 1) * OH / IH) + 2);
    const int w0 = max(0, (int)((long)iw * OW / IW) - 2), w1 = min(OW - 1, (int)((long)(iw + 1) * OW / IW) + 2);
    float s = 0.f;
    for (int oh = h0; oh <= h1; ++oh) {
      if (nearest_src(oh, IH, OH) != ih) continue;
      for (int ow = w0; ow <= w1; ++ow)
        if (nearest_src(ow, IW, OW) == iw) s += to_f(dy[(((long)b * OH + oh) * OW + ow) * dps + c]);
    }
    dx[(((long)b * IH + ih) * IW + iw) * dxps + c] = from_f<T>(s);
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
    const long m = i / cv;
    const int c = (int)(i % cv) * (VEC ? VW : 1);
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
template <typename T>
__global__ void dot_partial_kernel(const T* __restrict__ a, long aps, const T* __restrict__ b, long bps, long M,
                                   int C, float* __restrict__ part) {
  const long total = M * C;
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / C;
    const int c = (int)(i % C);
    s += to_f(a[m * aps + c]) * to_f(b[m * bps + c]);
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
template <typename T>
__global__ void scgate_fwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ u3, const T* __restrict__ g,
                                  T* __restrict__ out, int N, int H, int W, int C, int GH, int GW) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const long pix = ((long)b * H + h) * W + w;
    const int gh = nearest_src(h, GH, H), gw = nearest_src(w, GW, W);
    const float gv = to_f(g[(((long)b * GH + gh) * GW + gw) * C + c]);
    // torch: sigmoid(add(identity, y_)) computed in storage precision, then mul
    const float s = sigmoidf_(to_f(from_f<T>(to_f(x[pix * xps + c]) + gv)));
    out[pix * C + c] = from_f<T>(to_f(u3[pix * C + c]) * to_f(from_f<T>(s)));
  }
}

// d u3 = dout * s ;  dpre = dout * u3 * s(1-s)  (-> dx contribution, written to dpre)
template <typename T>
__global__ void scgate_bwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ u3, const T* __restrict__ g,
                                  const T* __restrict__ dout, T* __restrict__ du3, T* __restrict__ dpre, int N, int H,
                                  int W, int C, int GH, int GW) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const long pix = ((long)b * H + h) * W + w;
    const int gh = nearest_src(h, GH, H), gw = nearest_src(w, GW, W);
    const float gv = to_f(g[(((long)b * GH + gh) * GW + gw) * C + c]);
    const float s = sigmoidf_(to_f(from_f<T>(to_f(x[pix * xps + c]) + gv)));
    const float d = to_f(dout[pix * C + c]);
    du3[pix * C + c] = from_f<T>(d * s);
    dpre[pix * C + c] = from_f<T>(d * to_f(u3[pix * C + c]) * s * (1.f - s));
  }
}

// ---------------------------------------------------------------- CoorAttention
// y[b, h, c] = mean_w x ;  y[b, H + w, c] = mean_h x       (y is [N, H+W, C])
template <typename T>
__global__ void ca_pool_fwd_kernel(const T* __restrict__ x, long xps, T* __restrict__ y, int N, int H, int W, int C) {
  const long total = (long)N * (H + W) * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
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
    const int c = (int)(i % C);
    long t = i / C;
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
    const int c = (int)(i % C);
    long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int b = (int)(t / H);
    const long pix = ((long)b * H + h) * W + w;
    const float ah = to_f(from_f<T>(sigmoidf_(to_f(lh[((long)b * (H + W) + h) * C + c]))));
    const float aw = to_f(from_f<T>(sigmoidf_(to_f(lw[((long)b * (H + W) + H + w) * C + c]))));
    const float xv = to_f(x[pix * xps + c]);
    out[pix * ops + c] = from_f<T>(to_f(from_f<T>(xv * aw)) * ah);
  }
}

// dx = dout*aw*ah ; dlh[b,h] = sum_w dout*x*aw * ah(1-ah) ; dlw[b,H+w] = sum_h dout*x*ah * aw(1-aw)
template <typename T>
__global__ void ca_apply_bwd_dx_kernel(const T* __restrict__ x, long xps, const T* __restrict__ lh,
                                       const T* __restrict__ lw, const T* __restrict__ dout, long dps,
                                       T* __restrict__ dx, long dxps, int N, int H, int W, int C) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
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
    const int c = (int)(i % C);
    long t = i / C;
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

inline int egrid(long n) { return grid_cap(ceil_div(n, 256), 8192); }

}  // namespace

#define DISPATCH_T(dtype, ...)         \
  if (dtype) {                         \
    using T = bf16;                    \
    __VA_ARGS__;                       \
  } else {                             \
    using T = float;                   \
    __VA_ARGS__;                       \
  }

DMY_API int dmy_maxpool_fwd(int dtype, const void* x, long xps, void* y, long yps, unsigned char* arg, int N, int H,
                            int W, int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, maxpool_fwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)x, xps, (T*)y, yps, arg, N, H, W, C, k));
  return (int)hipGetLastError();
}
DMY_API int dmy_maxpool_bwd(int dtype, const void* dy, long dps, const unsigned char* arg, void* dx, long dxps,
                            int accumulate, int N, int H, int W, int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, maxpool_bwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)dy, dps, arg, (T*)dx, dxps, accumulate, N, H, W, C, k));
  return (int)hipGetLastError();
}
DMY_API int dmy_avgpool_fwd(int dtype, const void* x, long xps, void* y, int N, int H, int W, int C, int r,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, avgpool_fwd_kernel<T><<<egrid((long)N * (H / r) * (W / r) * C), 256, 0, st>>>((const T*)x, xps, (T*)y, N, H, W, C, r));
  return (int)hipGetLastError();
}
DMY_API int dmy_avgpool_bwd(int dtype, const void* dy, void* dx, long dxps, int accumulate, int N, int H, int W, int C,
                            int r, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, avgpool_bwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)dy, (T*)dx, dxps, accumulate, N, H, W, C, r));
  return (int)hipGetLastError();
}
DMY_API int dmy_resize_fwd(int dtype, const void* x, long xps, void* y, long yps, float yscale, int N, int IH, int IW,
                           int OH, int OW, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, resize_fwd_kernel<T><<<egrid((long)N * OH * OW * C), 256, 0, st>>>((const T*)x, xps, (T*)y, yps, yscale, N, IH, IW, OH, OW, C));
  return (int)hipGetLastError();
}
DMY_API int dmy_resize_bwd(int dtype, const void* dy, long dps, void* dx, long dxps, int N, int IH, int IW, int OH,
                           int OW, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, resize_bwd_kernel<T><<<egrid((long)N * IH * IW * C), 256, 0, st>>>((const T*)dy, dps, (T*)dx, dxps, N, IH, IW, OH, OW, C));
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
DMY_API int dmy_dot_partial_blocks(long M, int C) { return grid_cap(ceil_div(M * C, 256 * 8), 512); }
DMY_API int dmy_dot_partial(int dtype, const void* a, long aps, const void* b, long bps, long M, int C, float* part,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int nb = dmy_dot_partial_blocks(M, C);
  DISPATCH_T(dtype, dot_partial_kernel<T><<<nb, 256, 0, st>>>((const T*)a, aps, (const T*)b, bps, M, C, part));
  return (int)hipGetLastError();
}
DMY_API int dmy_bifpn_wgrad(const float* part, int nblk, int nw, const float* wv, float eps, float* dw, void* stream) {
  bifpn_wgrad_kernel<<<1, 64, 0, (hipStream_t)stream>>>(part, nblk, nw, wv, eps, dw);
  return (int)hipGetLastError();
}
DMY_API int dmy_scgate_fwd(int dtype, const void* x, long xps, const void* u3, const void* g, void* out, int N, int H,
                           int W, int C, int GH, int GW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, scgate_fwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)x, xps, (const T*)u3, (const T*)g, (T*)out, N, H, W, C, GH, GW));
  return (int)hipGetLastError();
}
DMY_API int dmy_scgate_bwd(int dtype, const void* x, long xps, const void* u3, const void* g, const void* dout,
                           void* du3, void* dpre, int N, int H, int W, int C, int GH, int GW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, scgate_bwd_kernel<T><<<egrid((long)N * H * W * C), 256, 0, st>>>((const T*)x, xps, (const T*)u3, (const T*)g, (const T*)dout, (T*)du3, (T*)dpre, N, H, W, C, GH, GW));
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
