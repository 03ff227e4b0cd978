// Detect-head decode and the anchor-based YOLO loss on gfx950.
//
//  * detect_decode: models/yolo.py:78-101 (inference branch): sigmoid, (2s-0.5+grid)*stride, (2s)^2*anchor_grid.
//  * build_targets: utils/loss.py:220-276, candidate order offset-major -> anchor -> target (the
//    reference's repeat/mask order), stream-compacted by ONE block per level with a block scan;
//    gij is clamped before tbox (the reference's in-place clamp_).
//  * loss: utils/loss.py:167-218 with utils/metrics.py:192-235 (SIoU).  Gradients of SIoU come from
//    forward-mode dual numbers (4 partials: px, py, pw, ph), so they follow the same expression as
//    the reference autograd graph; torch.minimum/maximum ties split the gradient in half, abs'(0)=0.
//    tobj keeps the max clamped IoU per cell (sort_obj_iou forced on, loss.py:191-194) via an
//    integer atomicMax on non-negative float bits -> deterministic.  Per-target gradients are summed per cell in
//    ascending target order (the reference's index_put_ accumulate order) and the loss sums go through per-block
//    partials reduced in a fixed order: no float atomics, the loss and dL/dp are run-to-run bit-identical.
// Everything stays on device: target counts are read by the kernels, never by the host.
#include "common.h"
#include "dual.h"

namespace {

// ---------------------------------------------------------------- decode
template <typename T>
__global__ void decode_kernel(const T* __restrict__ y, long sb, long sh, long sw, int N, int H, int W, int na, int no,
                              float stride, const float* __restrict__ anchors, float* __restrict__ z, long zoff,
                              long ztotal) {
  const long total = (long)N * na * H * W * no;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % no);
    long t = i / no;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    t /= H;
    const int a = (int)(t % na);
    const int b = (int)(t / na);
    const float v = to_f(y[b * sb + h * sh + w * sw + a * no + c]);
    float s = 1.0f / (1.0f + expf(-v));
    float o;
    if (c < 2) {
      const float g = (float)(c == 0 ? w : h);
      o = (s * 2.0f - 0.5f + g) * stride;
    } else if (c < 4) {
      const float ag = anchors[a * 2 + (c - 2)] * stride;
      const float q = s * 2.0f;
      o = (q * q) * ag;
    } else {
      o = s;
    }
    z[((long)b * ztotal + zoff + ((long)a * H + h) * W + w) * no + c] = o;
  }
}

// all levels of one Detect forward in one launch: the level of a flat element index from the cumulative element
// counts, then decode_kernel's arithmetic (the same bits)
constexpr int kDecLevels = 4;
struct DecTab {
  const void* y[kDecLevels];
  long sb[kDecLevels], sh[kDecLevels], sw[kDecLevels], zoff[kDecLevels], cum[kDecLevels + 1];
  int H[kDecLevels], W[kDecLevels];
  float stride[kDecLevels];
  int nl;
};

template <typename T>
__global__ void decode_levels_kernel(DecTab tab, int N, int na, int no, const float* __restrict__ anchors,
                                     float* __restrict__ z, long ztotal) {
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < tab.cum[tab.nl]; g += (long)gridDim.x * blockDim.x) {
    int L = 0;
#pragma unroll
    for (int l = 1; l < kDecLevels; ++l)
      if (l < tab.nl && g >= tab.cum[l]) L = l;
    const long i = g - tab.cum[L];
    const int H = tab.H[L], W = tab.W[L];
    const int c = (int)(i % no);
    long t = i / no;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    t /= H;
    const int a = (int)(t % na);
    const int b = (int)(t / na);
    const T* y = static_cast<const T*>(tab.y[L]);
    const float v = to_f(y[b * tab.sb[L] + h * tab.sh[L] + w * tab.sw[L] + a * no + c]);
    const float stride = tab.stride[L];
    float s = 1.0f / (1.0f + expf(-v));
    float o;
    if (c < 2) {
      const float gg = (float)(c == 0 ? w : h);
      o = (s * 2.0f - 0.5f + gg) * stride;
    } else if (c < 4) {
      const float ag = anchors[(L * na + a) * 2 + (c - 2)] * stride;
      const float q = s * 2.0f;
      o = (q * q) * ag;
    } else {
      o = s;
    }
    z[((long)b * ztotal + tab.zoff[L] + ((long)a * H + h) * W + w) * no + c] = o;
  }
}

// ---------------------------------------------------------------- build_targets
struct TgtOut {
  int* b; int* a; int* gj; int* gi; int* tcls; float* tbox; float* anch; int* count;
};

__global__ void __launch_bounds__(1024) build_targets_kernel(const float* __restrict__ tg, int nt, const float* __restrict__ anchors,
                                                             int na, int H, int W, float anchor_t, TgtOut o) {
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const long ncand = 5L * na * nt;
  const float gw_ = (float)W, gh_ = (float)H;
  for (long c0 = 0; c0 < ncand; c0 += blockDim.x) {
    const long idx = c0 + threadIdx.x;
    bool valid = false;
    int oo = 0, a = 0, t = 0;
    float gx = 0, gy = 0, tw = 0, th = 0;
    if (idx < ncand) {
      oo = (int)(idx / ((long)na * nt));
      const int rem = (int)(idx % ((long)na * nt));
      a = rem / nt;
      t = rem % nt;
      const float* r = tg + (long)t * 6;
      gx = r[2] * gw_;
      gy = r[3] * gh_;
      tw = r[4] * gw_;
      th = r[5] * gh_;
      const float rw = tw / anchors[a * 2], rh = th / anchors[a * 2 + 1];
      const float m = fmaxf(fmaxf(rw, 1.0f / rw), fmaxf(rh, 1.0f / rh));
      valid = m < anchor_t;
      if (valid && oo > 0) {
        const float v = (oo == 1) ? gx : (oo == 2) ? gy : (oo == 3) ? (gw_ - gx) : (gh_ - gy);
        valid = (fmodf(v, 1.0f) < 0.5f) && (v > 1.0f);
      }
    }
    // block-wide exclusive scan of `valid`
    const unsigned long long bal = __ballot(valid);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int pre = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int woff = 0;
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < wid; ++k) woff += wsum[k];
    int tot = 0;
    for (int k = 0; k < nw; ++k) tot += wsum[k];
    if (valid) {
      const int j = base + woff + pre;
      const float ox = (oo == 1) ? 0.5f : (oo == 3) ? -0.5f : 0.f;
      const float oy = (oo == 2) ? 0.5f : (oo == 4) ? -0.5f : 0.f;
      int gi = (int)(gx - ox), gj = (int)(gy - oy);  // .long(): truncation toward zero
      gi = min(max(gi, 0), W - 1);
      gj = min(max(gj, 0), H - 1);
      const float* r = tg + (long)t * 6;
      o.b[j] = (int)r[0];
      o.tcls[j] = (int)r[1];
      o.a[j] = a;
      o.gj[j] = gj;
      o.gi[j] = gi;
      o.tbox[j * 4 + 0] = gx - (float)gi;
      o.tbox[j * 4 + 1] = gy - (float)gj;
      o.tbox[j * 4 + 2] = tw;
      o.tbox[j * 4 + 3] = th;
      o.anch[j * 2 + 0] = anchors[a * 2];
      o.anch[j * 2 + 1] = anchors[a * 2 + 1];
    }
    __syncthreads();
    if (threadIdx.x == 0) base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *o.count = base;
}

// SIoU(b1, b2) for xywh boxes, utils/metrics.py:192-235; b1 carries the derivatives
DEV D4 siou(D4 x1, D4 y1, D4 w1_, D4 h1_, float x2, float y2, float w2_, float h2_) {
  const float eps = 1e-7f;
  D4 b1x1 = x1 - scal(w1_, 0.5f), b1x2 = x1 + scal(w1_, 0.5f);
  D4 b1y1 = y1 - scal(h1_, 0.5f), b1y2 = y1 + scal(h1_, 0.5f);
  D4 b2x1 = dc(x2 - w2_ / 2), b2x2 = dc(x2 + w2_ / 2);
  D4 b2y1 = dc(y2 - h2_ / 2), b2y2 = dc(y2 + h2_ / 2);
  D4 inter = dclamp0(dmin(b1x2, b2x2) - dmax(b1x1, b2x1)) * dclamp0(dmin(b1y2, b2y2) - dmax(b1y1, b2y1));
  D4 w1 = b1x2 - b1x1, h1 = b1y2 - b1y1 + dc(eps);
  D4 w2 = b2x2 - b2x1, h2 = b2y2 - b2y1 + dc(eps);
  D4 uni = w1 * h1 + w2 * h2 - inter + dc(eps);
  D4 iou = inter / uni;
  D4 cw = dmax(b1x2, b2x2) - dmin(b1x1, b2x1);
  D4 ch = dmax(b1y2, b2y2) - dmin(b1y1, b2y1);
  D4 scw = scal(b2x1 + b2x2 - b1x1 - b1x2, 0.5f);
  D4 sch = scal(b2y1 + b2y2 - b1y1 - b1y2, 0.5f);
  D4 sigma = dsqrt(dsq(scw) + dsq(sch));
  D4 sa1 = dabs(scw) / sigma, sa2 = dabs(sch) / sigma;
  const float thr = 0.70710678118654757f;  // pow(2, 0.5) / 2 (python double -> fp32 compare)
  D4 sa = sa1.v > thr ? sa2 : sa1;
  D4 ang = dcos(scal(dasin(sa), 2.f) - dc(1.5707963267948966f));
  D4 rx = dsq(scw / cw), ry = dsq(sch / ch);
  D4 gam = ang - dc(2.f);
  D4 dist = dc(2.f) - dexp(gam * rx) - dexp(gam * ry);
  D4 ow = dabs(w1 - w2) / dmax(w1, w2);
  D4 oh = dabs(h1 - h2) / dmax(h1, h2);
  D4 shape = dpow4(dc(1.f) - dexp(scal(ow, -1.f))) + dpow4(dc(1.f) - dexp(scal(oh, -1.f)));
  return iou - scal(dist + shape, 0.5f);
}

// BCEWithLogits(pos_weight) element and its derivative (ATen formulation)
DEV float bce(float x, float t, float pw, float* g) {
  const float lw = 1.f + (pw - 1.f) * t;
  const float mx = fmaxf(-x, 0.f);
  const float l = (1.f - t) * x + lw * (log1pf(expf(-fabsf(x))) + mx);
  *g = (1.f - t) - lw / (1.f + expf(x));  // (1-t) - lw*sigmoid(-x)
  return l;
}

struct LossCfg {
  float box_gain, obj_gain, cls_gain, cls_pw, obj_pw, cp, cn, balance, bs;
  int nc, na, no, N, H, W;
  long sb, sa, sh, sw;  // element strides of p (batch, anchor, row, col); channel stride = 1
};

// Loss partial sums: every block writes its own slot of part[3][LOSS_PMAX] (row 0 lbox, 1 lobj, 2 lcls; per level),
// reduced in a fixed order by loss_finalize_kernel -- no float atomics, so the loss is run-to-run bit-identical.
constexpr int LOSS_PMAX = 2048;

// per selected target j: SIoU box loss + cls BCE + tobj scatter-max.  The target's gradient contribution to its
// cell's box / cls channels goes to tgrad[j][4 + nc] (no atomics), and j is pushed on its cell's list (head / nxt);
// loss_combine_kernel then sums each cell's contributions in ascending j -- the order of the reference's
// index_put_(accumulate=True) backward of pi[b, a, gj, gi] (utils/loss.py:179).
template <typename T>
__global__ void loss_targets_kernel(const T* __restrict__ p, LossCfg cfg, const int* __restrict__ tb,
                                    const int* __restrict__ ta, const int* __restrict__ tgj, const int* __restrict__ tgi,
                                    const int* __restrict__ tcls, const float* __restrict__ tbox,
                                    const float* __restrict__ anch, const int* __restrict__ count,
                                    float* __restrict__ tgrad, int* __restrict__ head, int* __restrict__ nxt,
                                    float* __restrict__ tobj, float* __restrict__ part) {
  const int M = *count;
  const int ng = 4 + (cfg.nc > 1 ? cfg.nc : 0);
  float lbox = 0.f, lcls = 0.f;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < M; j += gridDim.x * blockDim.x) {
    const int b = tb[j], a = ta[j], gj = tgj[j], gi = tgi[j];
    const long off = b * cfg.sb + gj * cfg.sh + gi * cfg.sw + (long)a * cfg.sa;
    const T* ps = p + off;
    float sg[4];
    for (int k = 0; k < 4; ++k) sg[k] = 1.f / (1.f + expf(-to_f(ps[k])));
    // pxy = 2s - 0.5, pwh = (2s)^2 * anchor; seed derivatives w.r.t. (pxy, pwh)
    D4 px = dc(sg[0] * 2.f - 0.5f), py = dc(sg[1] * 2.f - 0.5f);
    const float q2 = sg[2] * 2.f, q3 = sg[3] * 2.f;
    D4 pw = dc((q2 * q2) * anch[j * 2]), ph = dc((q3 * q3) * anch[j * 2 + 1]);
    px.d[0] = 1.f; py.d[1] = 1.f; pw.d[2] = 1.f; ph.d[3] = 1.f;
    D4 iou = siou(px, py, pw, ph, tbox[j * 4], tbox[j * 4 + 1], tbox[j * 4 + 2], tbox[j * 4 + 3]);
    lbox += 1.f - iou.v;
    // d(mean(1-iou))/d p_k  scaled by box gain * bs
    const float gs = -cfg.box_gain * cfg.bs / (float)M;
    float* g = tgrad + (long)j * ng;
    g[0] = gs * iou.d[0] * 2.f * sg[0] * (1.f - sg[0]);
    g[1] = gs * iou.d[1] * 2.f * sg[1] * (1.f - sg[1]);
    g[2] = gs * iou.d[2] * 2.f * q2 * 2.f * sg[2] * (1.f - sg[2]) * anch[j * 2];
    g[3] = gs * iou.d[3] * 2.f * q3 * 2.f * sg[3] * (1.f - sg[3]) * anch[j * 2 + 1];
    // tobj[b,a,gj,gi] = max(clamp(iou,0))
    const long cell = (((long)b * cfg.na + a) * cfg.H + gj) * cfg.W + gi;
    const float sc = fmaxf(iou.v, 0.f);
    atomicMax(reinterpret_cast<int*>(tobj) + cell, __float_as_int(sc));
    if (cfg.nc > 1) {
      const float cg = cfg.cls_gain * cfg.bs / ((float)M * cfg.nc);
      const int tc = tcls[j];
      for (int c = 0; c < cfg.nc; ++c) {
        float d;
        lcls += bce(to_f(ps[5 + c]), c == tc ? cfg.cp : cfg.cn, cfg.cls_pw, &d);
        g[4 + c] = cg * d;
      }
    }
    nxt[j] = atomicExch(head + cell, j);  // list order is arbitrary; the combine sorts it
  }
  __shared__ float r1[16], r2[16];
  lbox = wave_sum(lbox);
  lcls = wave_sum(lcls);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { r1[wid] = lbox; r2[wid] = lcls; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s1 = 0.f, s2 = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { s1 += r1[w]; s2 += r2[w]; }
    if (M > 0) {
      part[blockIdx.x] = s1 / (float)M;
      if (cfg.nc > 1) part[2 * LOSS_PMAX + blockIdx.x] = s2 / ((float)M * cfg.nc);
    }
  }
}

// one thread per target: the smallest j on a cell's list owns the cell and writes G's box / cls channels there as
// 0 + c_j0 + c_j1 + ... in ascending j (lists hold the few targets sharing a (b, a, gj, gi) cell)
__global__ void loss_combine_kernel(LossCfg cfg, const int* __restrict__ tb, const int* __restrict__ ta,
                                    const int* __restrict__ tgj, const int* __restrict__ tgi,
                                    const int* __restrict__ count, const float* __restrict__ tgrad,
                                    const int* __restrict__ head, const int* __restrict__ nxt, float* __restrict__ G) {
  const int M = *count;
  const int ng = 4 + (cfg.nc > 1 ? cfg.nc : 0);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < M; j += gridDim.x * blockDim.x) {
    const int b = tb[j], a = ta[j], gj = tgj[j], gi = tgi[j];
    const long cell = (((long)b * cfg.na + a) * cfg.H + gj) * cfg.W + gi;
    int mn = j;
    for (int k = head[cell]; k >= 0; k = nxt[k]) mn = min(mn, k);
    if (mn != j) continue;
    float* g = G + b * cfg.sb + gj * cfg.sh + gi * cfg.sw + (long)a * cfg.sa;
    // the cell's targets in ascending index order, collected once (insertion sort of the short list) and then summed
    // channel by channel in that order; a cell with more than LMAX targets walks the list per channel instead
    constexpr int LMAX = 32;
    int ord[LMAX];
    int L = 0;
    for (int k = head[cell]; k >= 0; k = nxt[k]) {
      if (L < LMAX) {
        int q = L;
        while (q > 0 && ord[q - 1] > k) { ord[q] = ord[q - 1]; --q; }
        ord[q] = k;
      }
      ++L;
    }
    for (int c = 0; c < ng; ++c) {
      float acc = 0.f;
      if (L <= LMAX) {
        for (int q = 0; q < L; ++q) acc += tgrad[(long)ord[q] * ng + c];
      } else {
        int last = -1;
        while (true) {  // next target of the cell in ascending index order
          int nj = 0x7fffffff;
          for (int k = head[cell]; k >= 0; k = nxt[k])
            if (k > last && k < nj) nj = k;
          if (nj == 0x7fffffff) break;
          acc += tgrad[(long)nj * ng + c];
          last = nj;
        }
      }
      g[c < 4 ? c : c + 1] = acc;  // channels 0-3 box, 5.. cls (4 is objectness, written by loss_obj_kernel)
    }
  }
}

// dense objectness BCE over every (b, a, h, w); writes the obj-channel gradient
template <typename T>
__global__ void loss_obj_kernel(const T* __restrict__ p, LossCfg cfg, const float* __restrict__ tobj,
                                float* __restrict__ G, float* __restrict__ part) {
  const long total = (long)cfg.N * cfg.na * cfg.H * cfg.W;
  const float gs = cfg.balance * cfg.obj_gain * cfg.bs / (float)total;
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % cfg.W);
    long t = i / cfg.W;
    const int h = (int)(t % cfg.H);
    t /= cfg.H;
    const int a = (int)(t % cfg.na);
    const int b = (int)(t / cfg.na);
    const long off = b * cfg.sb + h * cfg.sh + w * cfg.sw + (long)a * cfg.sa + 4;
    float d;
    s += bce(to_f(p[off]), tobj[i], cfg.obj_pw, &d);
    G[off] = gs * d;
  }
  __shared__ float r[16];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float q = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) q += r[k];
    part[LOSS_PMAX + blockIdx.x] = q * cfg.balance / (float)total;
  }
}

// part per level: [3][LOSS_PMAX] block partials (lbox mean, lobj balanced, lcls mean); one 256-thread block reduces
// every row in a fixed order (strided serial sums, then a fixed tree) -> loss[1], items[3]
__global__ void __launch_bounds__(256) loss_finalize_kernel(const float* __restrict__ part, int nl, float box, float obj,
                                                            float cls, float bs, float* __restrict__ loss,
                                                            float* __restrict__ items) {
  __shared__ float red[256];
  __shared__ float row[3];
  float tot[3] = {0.f, 0.f, 0.f};
  for (int lvl = 0; lvl < nl; ++lvl)
    for (int r = 0; r < 3; ++r) {
      const float* pr = part + ((long)lvl * 3 + r) * LOSS_PMAX;
      float v = 0.f;
      for (int k = threadIdx.x; k < LOSS_PMAX; k += 256) v += pr[k];
      red[threadIdx.x] = v;
      __syncthreads();
      for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
      }
      if (threadIdx.x == 0) row[r] = red[0];
      __syncthreads();
      tot[r] += row[r];
      __syncthreads();
    }
  if (threadIdx.x == 0) {
    const float lb = tot[0] * box, lo = tot[1] * obj, lc = tot[2] * cls;
    items[0] = lb;
    items[1] = lo;
    items[2] = lc;
    loss[0] = (lb + lo + lc) * bs;
  }
}

// dp = G * upstream  (G fp32 p-shaped with strides; output T with the same strides)
template <typename T>
__global__ void loss_grad_kernel(const float* __restrict__ G, const float* __restrict__ up, T* __restrict__ dp,
                                 long n) {
  const float u = *up;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dp[i] = from_f<T>(G[i] * u);
}

}  // namespace

DMY_API int dmy_detect_decode(int dtype, const void* y, long sb, long sh, long sw, int N, int H, int W, int na, int no,
                              float stride, const float* anchors, float* z, long zoff, long ztotal, void* stream) {
  const long total = (long)N * na * H * W * no;
  const int g = grid_cap(ceil_div(total, 256), 8192);
  if (dtype) decode_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)y, sb, sh, sw, N, H, W, na, no, stride, anchors, z, zoff, ztotal);
  else decode_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)y, sb, sh, sw, N, H, W, na, no, stride, anchors, z, zoff, ztotal);
  return (int)hipGetLastError();
}

DMY_API int dmy_detect_decode_levels(int dtype, int nl, const void* const* ys, const long* strides, const int* hw,
                                     const float* lvl_stride, int N, int na, int no, const float* anchors, float* z,
                                     long ztotal, void* stream) {
  if (nl < 1 || nl > kDecLevels) return (int)hipErrorInvalidValue;
  DecTab tab{};
  tab.nl = nl;
  long zoff = 0;
  tab.cum[0] = 0;
  for (int l = 0; l < nl; ++l) {
    tab.y[l] = ys[l];
    tab.sb[l] = strides[3 * l];
    tab.sh[l] = strides[3 * l + 1];
    tab.sw[l] = strides[3 * l + 2];
    tab.H[l] = hw[2 * l];
    tab.W[l] = hw[2 * l + 1];
    tab.stride[l] = lvl_stride[l];
    tab.zoff[l] = zoff;
    zoff += (long)na * tab.H[l] * tab.W[l];
    tab.cum[l + 1] = tab.cum[l] + (long)N * na * tab.H[l] * tab.W[l] * no;
  }
  if (zoff != ztotal) return (int)hipErrorInvalidValue;
  const int g = grid_cap(ceil_div(tab.cum[nl], 256), 8192);
  if (dtype) decode_levels_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>(tab, N, na, no, anchors, z, ztotal);
  else decode_levels_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>(tab, N, na, no, anchors, z, ztotal);
  return (int)hipGetLastError();
}

DMY_API int dmy_build_targets(const float* targets, int nt, const float* anchors, int na, int H, int W, float anchor_t,
                              int* b, int* a, int* gj, int* gi, int* tcls, float* tbox, float* anch, int* count,
                              void* stream) {
  TgtOut o{b, a, gj, gi, tcls, tbox, anch, count};
  build_targets_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(targets, nt, anchors, na, H, W, anchor_t, o);
  return (int)hipGetLastError();
}

DMY_API int dmy_yolo_loss_part_rows() { return 3 * LOSS_PMAX; }

// One level of the loss.  part = this level's dmy_yolo_loss_part_rows() fp32 block partials (zeroed by the caller),
// G zeroed (p-shaped fp32), tobj zeroed (N*na*H*W).  Workspaces (contents on entry do not matter): tgrad
// cap * (4 + nc) fp32, links N*na*H*W + cap int32.
DMY_API int dmy_yolo_loss_level(int dtype, const void* p, long sb, long sa, long sh, long sw, int N, int na, int H, int W,
                                int no, int nc, float box_gain, float obj_gain, float cls_gain, float cls_pw,
                                float obj_pw, float cp, float cn, float balance, float bs, const int* tb,
                                const int* ta, const int* tgj, const int* tgi, const int* tcls, const float* tbox,
                                const float* anch, const int* count, int cap, float* G, float* tobj, float* part,
                                float* tgrad, int* links, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  LossCfg cfg{box_gain, obj_gain, cls_gain, cls_pw, obj_pw, cp, cn, balance, bs, nc, na, no, N, H, W, sb, sa, sh, sw};
  const int gt = grid_cap(ceil_div(cap, 256), 1024);
  const long cells = (long)N * na * H * W;
  const int go = grid_cap(ceil_div(cells, 256), LOSS_PMAX);
  int* head = links;
  int* nxt = links + cells;
  (void)hipMemsetAsync(head, 0xff, sizeof(int) * (size_t)cells, st);  // empty lists (-1)
  if (dtype)
    loss_targets_kernel<bf16><<<gt, 256, 0, st>>>((const bf16*)p, cfg, tb, ta, tgj, tgi, tcls, tbox, anch, count,
                                                  tgrad, head, nxt, tobj, part);
  else
    loss_targets_kernel<float><<<gt, 256, 0, st>>>((const float*)p, cfg, tb, ta, tgj, tgi, tcls, tbox, anch, count,
                                                   tgrad, head, nxt, tobj, part);
  loss_combine_kernel<<<gt, 256, 0, st>>>(cfg, tb, ta, tgj, tgi, count, tgrad, head, nxt, G);
  if (dtype) loss_obj_kernel<bf16><<<go, 256, 0, st>>>((const bf16*)p, cfg, tobj, G, part);
  else loss_obj_kernel<float><<<go, 256, 0, st>>>((const float*)p, cfg, tobj, G, part);
  return (int)hipGetLastError();
}

DMY_API int dmy_yolo_loss_finalize(const float* part, int nl, float box, float obj, float cls, float bs, float* loss,
                                   float* items, void* stream) {
  loss_finalize_kernel<<<1, 256, 0, (hipStream_t)stream>>>(part, nl, box, obj, cls, bs, loss, items);
  return (int)hipGetLastError();
}

DMY_API int dmy_loss_grad(int dtype, const float* G, const float* up, void* dp, long n, void* stream) {
  const int g = grid_cap(ceil_div(n, 256), 4096);
  if (dtype) loss_grad_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>(G, up, (bf16*)dp, n);
  else loss_grad_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>(G, up, (float*)dp, n);
  return (int)hipGetLastError();
}

// SIoU of n xywh box pairs through the loss kernel's own siou(): value and d(iou)/d(b1) (test entry)
__global__ void siou_eval_kernel(const float* __restrict__ b1, const float* __restrict__ b2, float* __restrict__ iou,
                                 float* __restrict__ grad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  D4 x = dc(b1[i * 4]), y = dc(b1[i * 4 + 1]), w = dc(b1[i * 4 + 2]), h = dc(b1[i * 4 + 3]);
  x.d[0] = 1.f; y.d[1] = 1.f; w.d[2] = 1.f; h.d[3] = 1.f;
  const D4 r = siou(x, y, w, h, b2[i * 4], b2[i * 4 + 1], b2[i * 4 + 2], b2[i * 4 + 3]);
  iou[i] = r.v;
  for (int k = 0; k < 4; ++k) grad[i * 4 + k] = r.d[k];
}

DMY_API int dmy_siou_eval(const float* b1, const float* b2, float* iou, float* grad, int n, void* stream) {
  if (n <= 0) return 0;
  siou_eval_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(b1, b2, iou, grad, n);
  return (int)hipGetLastError();
}
