// Anchor-free TAL path on gfx950: TDetect head flatten / decode, TaskAlignedAssigner and
// ComputeLoss_TAL (CIoU box loss, DFL, BCE with pos_weight), gradients written in the forward.
//
// Replaces utils/tal.py:81-221 (ComputeLoss_TAL, BboxLoss, bbox2dist, dist2bbox, make_anchors),
// utils/tal_assign.py:54-189 (TaskAlignedAssigner) and models/detect_t.py:38-90 (TDetect train /
// eval outputs, DFL).  Layout: the head outputs of all levels flattened anchor-major,
// F[b][a][64 + nc] (64 = 4 sides x 16 DFL bins), read through generic (batch, channel, anchor)
// strides so the reference's [B, C, A] tensors work as well.
//
// Assigner (per image b, gt j in original target order):
//   metric(j, a) = sigmoid(cls[b, label_j, a])^alpha * max(CIoU(gt_j, pbox_a), 0)^beta
//   candidates: the top-10 anchors by metric among anchors whose centre lies strictly inside gt_j
//     and whose metric is > 0.  (The reference's torch.topk also returns zero-metric anchors when a gt
//     has fewer than 10 positive ones; those carry zero target score and weight, so they never change
//     the loss -- only which zero-weight anchors count as foreground, which depends on topk's
//     implementation-defined tie order.)
//   an anchor claimed by several gts goes to argmax_j CIoU(gt_j, pbox_a) over all gts (first max);
//   norm(a) = metric(j*, a) * max_{a' of j*} CIoU / (max_{a' of j*} metric + 1e-9).
// Losses (sums over anchors, divided by tss = sum of norms):
//   cls: BCEWithLogits(cls, t, pos_weight) with t = norm on the assigned label, box: (1 - CIoU)*norm,
//   dfl: per side CE(bins, floor(t)) * (floor(t) + 1 - t) + CE(bins, floor(t) + 1) * (t - floor(t)),
//   mean over sides, * norm;  loss = (7.5 box + 0.5 cls + 1.5 dfl) * B.
#include "common.h"
#include "dual.h"

namespace {

constexpr int RM = 16;   // DFL bins (reg_max)
constexpr int TOPK = 10;

struct LevelTab {        // anchor index -> level geometry (up to 8 levels)
  int nl;
  int a0[9];             // first anchor of each level (a0[nl] = A)
  int W[8];
  float stride[8];
};

DEV void anchor_of(const LevelTab& lt, int a, float& ax, float& ay, float& st) {
  int l = 0;
  while (l + 1 < lt.nl && a >= lt.a0[l + 1]) ++l;
  const int r = a - lt.a0[l];
  ax = (float)(r % lt.W[l]) + 0.5f;
  ay = (float)(r / lt.W[l]) + 0.5f;
  st = lt.stride[l];
}

// CIoU of xyxy boxes (bbox_iou(xywh=False, CIoU=True)), plain value
DEV float ciou_v(float ax1, float ay1, float ax2, float ay2, float bx1, float by1, float bx2, float by2) {
  const float eps = 1e-7f;
  const float w1 = ax2 - ax1, h1 = ay2 - ay1 + eps, w2 = bx2 - bx1, h2 = by2 - by1 + eps;
  const float inter = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f) * fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float uni = w1 * h1 + w2 * h2 - inter + eps;
  const float iou = inter / uni;
  const float cw = fmaxf(ax2, bx2) - fminf(ax1, bx1), ch = fmaxf(ay2, by2) - fminf(ay1, by1);
  const float c2 = cw * cw + ch * ch + eps;
  const float dx = bx1 + bx2 - ax1 - ax2, dy = by1 + by2 - ay1 - ay2;
  const float rho2 = (dx * dx + dy * dy) / 4.f;
  const float t = atanf(w2 / h2) - atanf(w1 / h1);
  const float v = (4.f / (float)(M_PI * M_PI)) * t * t;
  const float alpha = v / (v - iou + (1.f + eps));
  return iou - (rho2 / c2 + v * alpha);
}

// CIoU with the first box carrying derivatives; alpha is a constant (no_grad in the reference)
DEV D4 ciou_d(D4 ax1, D4 ay1, D4 ax2, D4 ay2, float bx1, float by1, float bx2, float by2) {
  const float eps = 1e-7f;
  D4 w1 = ax2 - ax1, h1 = ay2 - ay1 + dc(eps);
  const float w2 = bx2 - bx1, h2 = by2 - by1 + eps;
  D4 inter = dclamp0(dmin(ax2, dc(bx2)) - dmax(ax1, dc(bx1))) * dclamp0(dmin(ay2, dc(by2)) - dmax(ay1, dc(by1)));
  D4 uni = w1 * h1 + dc(w2 * h2) - inter + dc(eps);
  D4 iou = inter / uni;
  D4 cw = dmax(ax2, dc(bx2)) - dmin(ax1, dc(bx1));
  D4 ch = dmax(ay2, dc(by2)) - dmin(ay1, dc(by1));
  D4 c2 = cw * cw + ch * ch + dc(eps);
  D4 dx = dc(bx1 + bx2) - ax1 - ax2, dy = dc(by1 + by2) - ay1 - ay2;
  D4 rho2 = scal(dx * dx + dy * dy, 0.25f);
  D4 t = dc(atanf(w2 / h2)) - datan(w1 / h1);
  D4 v = scal(t * t, 4.f / (float)(M_PI * M_PI));
  const float alpha = v.v / (v.v - iou.v + (1.f + eps));
  return iou - (rho2 / c2 + scal(v, alpha));
}

template <typename T> DEV float ldf(const T* p, long i) { return to_f(p[i]); }

// softmax over 16 bins of one side; returns expectation and fills probabilities
template <typename T>
DEV float side_softmax(const T* box, long sb_c, int side, float* p) {
  float mx = -3.0e38f;
#pragma unroll
  for (int k = 0; k < RM; ++k) {
    p[k] = ldf(box, (long)(side * RM + k) * sb_c);
    mx = fmaxf(mx, p[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < RM; ++k) {
    p[k] = expf(p[k] - mx);
    s += p[k];
  }
  const float inv = 1.f / s;
  float e = 0.f;
#pragma unroll
  for (int k = 0; k < RM; ++k) {
    p[k] *= inv;
    e += p[k] * (float)k;
  }
  return e;
}

// ---------------------------------------------------------------- targets -> per-image gt lists
// gt[b][j] = (cls, x1, y1, x2, y2) in pixels, j in original row order; cnt[b]
__global__ void tal_targets_kernel(const float* __restrict__ tg, int nt, int B, float iw, float ih, int cap,
                                   float* __restrict__ gt, int* __restrict__ cnt) {
  __shared__ int scan[256];
  for (int b = 0; b < B; ++b) {
    int base = 0;
    for (int i0 = 0; i0 < nt; i0 += blockDim.x) {
      const int i = i0 + threadIdx.x;
      const int f = (i < nt && (int)tg[i * 6] == b) ? 1 : 0;
      scan[threadIdx.x] = f;
      __syncthreads();
      for (int o = 1; o < (int)blockDim.x; o <<= 1) {
        const int v = threadIdx.x >= (unsigned)o ? scan[threadIdx.x - o] : 0;
        __syncthreads();
        scan[threadIdx.x] += v;
        __syncthreads();
      }
      if (f) {
        const int j = base + scan[threadIdx.x] - 1;
        const float* r = tg + i * 6;
        float* o = gt + ((long)b * cap + j) * 5;
        const float x = r[2] * iw, y = r[3] * ih, w = r[4] * iw, h = r[5] * ih;
        o[0] = r[1];
        o[1] = x - w / 2;
        o[2] = y - h / 2;
        o[3] = x + w / 2;
        o[4] = y + h / 2;
      }
      base += scan[blockDim.x - 1];
      __syncthreads();
    }
    if (threadIdx.x == 0) cnt[b] = base;
  }
}

// ---------------------------------------------------------------- decode: pbox (grid units, xyxy)
template <typename T>
__global__ void tal_decode_kernel(const T* __restrict__ box, long sbb, long sbc, long sba, int B, int A, LevelTab lt,
                                  float* __restrict__ pbox) {
  const long n = (long)B * A;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / A), a = (int)(i % A);
    const T* bp = box + b * sbb + a * sba;
    float ax, ay, st, p[RM], d[4];
    anchor_of(lt, a, ax, ay, st);
#pragma unroll
    for (int s = 0; s < 4; ++s) d[s] = side_softmax(bp, sbc, s, p);
    float* o = pbox + i * 4;
    o[0] = ax - d[0];
    o[1] = ay - d[1];
    o[2] = ax + d[2];
    o[3] = ay + d[3];
  }
}

template <typename T>
DEV float align_metric(const T* cls, long scb, long scc, long sca, int b, int a, int label, const float* gt5,
                       const float* pbox, long ia, float st, float alpha, float beta, float* ov_out) {
  const float* pb = pbox + ia * 4;
  float ov = ciou_v(gt5[1], gt5[2], gt5[3], gt5[4], pb[0] * st, pb[1] * st, pb[2] * st, pb[3] * st);
  ov = fmaxf(ov, 0.f);
  *ov_out = ov;
  const float s = 1.f / (1.f + expf(-ldf(cls, b * scb + (long)label * scc + a * sca)));
  return powf(s, alpha) * powf(ov, beta);
}

// ---------------------------------------------------------------- top-10 candidates per (image, gt)
template <typename T>
__global__ void __launch_bounds__(256) tal_topk_kernel(const T* __restrict__ cls, long scb, long scc, long sca,
                                                       const float* __restrict__ pbox, const float* __restrict__ gt,
                                                       const int* __restrict__ cnt, int B, int A, int cap, LevelTab lt,
                                                       float alpha, float beta, int* __restrict__ cand) {
  const int b = blockIdx.y, j = blockIdx.x;
  int* out = cand + ((long)b * cap + j) * TOPK;
  if (j >= cnt[b]) return;
  const float* g5 = gt + ((long)b * cap + j) * 5;
  const int label = (int)g5[0];
  float tv[TOPK];
  int ti[TOPK];
#pragma unroll
  for (int k = 0; k < TOPK; ++k) { tv[k] = 0.f; ti[k] = -1; }
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    float ax, ay, st;
    anchor_of(lt, a, ax, ay, st);
    const float px = ax * st, py = ay * st;
    const float dmin = fminf(fminf(px - g5[1], py - g5[2]), fminf(g5[3] - px, g5[4] - py));
    if (!(dmin > 1e-9f)) continue;
    float ov;
    const float m = align_metric(cls, scb, scc, sca, b, a, label, g5, pbox, (long)b * A + a, st, alpha, beta, &ov);
    if (!(m > tv[TOPK - 1])) continue;
    int k = TOPK - 1;
    while (k > 0 && m > tv[k - 1]) {
      tv[k] = tv[k - 1];
      ti[k] = ti[k - 1];
      --k;
    }
    tv[k] = m;
    ti[k] = a;
  }
  // merge: TOPK rounds of block-wide argmax over the threads' current heads
  __shared__ float sv[256];
  __shared__ int si[256], st_[256];
  int head = 0;
  for (int r = 0; r < TOPK; ++r) {
    sv[threadIdx.x] = head < TOPK ? tv[head] : 0.f;
    si[threadIdx.x] = head < TOPK ? ti[head] : -1;
    st_[threadIdx.x] = threadIdx.x;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if (threadIdx.x < (unsigned)o) {
        const float v2 = sv[threadIdx.x + o];
        const int i2 = si[threadIdx.x + o];
        if (v2 > sv[threadIdx.x] || (v2 == sv[threadIdx.x] && i2 >= 0 && (si[threadIdx.x] < 0 || i2 < si[threadIdx.x]))) {
          sv[threadIdx.x] = v2;
          si[threadIdx.x] = i2;
          st_[threadIdx.x] = st_[threadIdx.x + o];
        }
      }
      __syncthreads();
    }
    const int win = st_[0];
    const int widx = sv[0] > 0.f ? si[0] : -1;
    if (threadIdx.x == 0) out[r] = widx;
    __syncthreads();
    if ((int)threadIdx.x == win) ++head;
  }
}

// ---------------------------------------------------------------- claims per anchor
__global__ void tal_claim_kernel(const int* __restrict__ cand, const int* __restrict__ cnt, int B, int A, int cap,
                                 int* __restrict__ nclaim, int* __restrict__ owner) {
  const long n = (long)B * cap * TOPK;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / ((long)cap * TOPK));
    const int j = (int)((i / TOPK) % cap);
    if (j >= cnt[b]) continue;
    const int a = cand[i];
    if (a < 0) continue;
    atomicAdd(nclaim + (long)b * A + a, 1);
    atomicMax(owner + (long)b * A + a, j);
  }
}

// resolve one gt per anchor, per-gt maxima of metric / overlap over its anchors
template <typename T>
__global__ void tal_resolve_kernel(const T* __restrict__ cls, long scb, long scc, long sca,
                                   const float* __restrict__ pbox, const float* __restrict__ gt,
                                   const int* __restrict__ cnt, const int* __restrict__ nclaim, int* __restrict__ owner,
                                   int B, int A, int cap, LevelTab lt, float alpha, float beta,
                                   float* __restrict__ metric, int* __restrict__ amax_m, int* __restrict__ amax_o) {
  const long n = (long)B * A;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / A), a = (int)(i % A);
    const int c = nclaim[i];
    if (c == 0) { owner[i] = -1; continue; }
    float ax, ay, st;
    anchor_of(lt, a, ax, ay, st);
    int j = owner[i];
    if (c > 1) {  // argmax over all gts of the clamped CIoU, first max
      const float* pb = pbox + i * 4;
      float best = -1.f;
      for (int g = 0; g < cnt[b]; ++g) {
        const float* g5 = gt + ((long)b * cap + g) * 5;
        const float ov = fmaxf(ciou_v(g5[1], g5[2], g5[3], g5[4], pb[0] * st, pb[1] * st, pb[2] * st, pb[3] * st), 0.f);
        if (ov > best) { best = ov; j = g; }
      }
      owner[i] = j;
    }
    const float* g5 = gt + ((long)b * cap + j) * 5;
    float ov;
    const float m = align_metric(cls, scb, scc, sca, b, a, (int)g5[0], g5, pbox, i, st, alpha, beta, &ov);
    metric[i] = m;
    atomicMax(amax_m + (long)b * cap + j, __float_as_int(m));   // non-negative floats order as ints
    atomicMax(amax_o + (long)b * cap + j, __float_as_int(ov));
  }
}

// a 256-thread block's sums of V values, written to part[blockIdx.x * V + v]: waves combined in wave order
template <int V>
__device__ void block_partials(float* v, float* __restrict__ part) {
  __shared__ float red[4][V];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const float t = wave_sum(v[k]);
    if ((threadIdx.x & 63) == 0) red[wv][k] = t;
  }
  __syncthreads();
  if (threadIdx.x < V) {
    const int k = threadIdx.x;
    part[(long)blockIdx.x * V + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
  }
}

// norm per anchor + tss
__global__ void tal_norm_kernel(const int* __restrict__ owner, const float* __restrict__ metric,
                                const int* __restrict__ amax_m, const int* __restrict__ amax_o, int B, int A, int cap,
                                float* __restrict__ norm, float* __restrict__ part) {
  const long n = (long)B * A;
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int j = owner[i];
    float v = 0.f;
    if (j >= 0) {
      const int b = (int)(i / A);
      v = metric[i] * __int_as_float(amax_o[(long)b * cap + j]) / (__int_as_float(amax_m[(long)b * cap + j]) + 1e-9f);
    }
    norm[i] = v;
    s += v;
  }
  block_partials<1>(&s, part);
}

// acc[a0 + v] = sum over blocks b < nb of part[b * V + v], in block order (one 256-thread block; fixed tree)
template <int V>
__global__ void tal_fold_kernel(const float* __restrict__ part, int nb, float* __restrict__ acc, int a0) {
  __shared__ float red[256];
  for (int k = 0; k < V; ++k) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += 256) s += part[(long)b * V + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) acc[a0 + k] = red[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- losses + gradients
// acc[0] = sum (1 - CIoU) w, acc[1] = sum BCE, acc[2] = sum dfl w, acc[3] = tss
// G layout: [b][a][64 + nc] fp32 (d loss_total / d logit, before the upstream gradient)
template <typename T>
__global__ void tal_loss_kernel(const T* __restrict__ box, long sbb, long sbc, long sba, const T* __restrict__ cls,
                                long scb, long scc, long sca, const float* __restrict__ gt, const int* __restrict__ owner,
                                const float* __restrict__ norm, int B, int A, int nc, int cap, LevelTab lt, float pw,
                                const float* __restrict__ acc, float* __restrict__ part, float* __restrict__ G) {
  const long n = (long)B * A;
  const float tss = acc[3];
  const float kb = 7.5f * B / tss, kc = 0.5f * B / tss, kd = 1.5f * B / tss;
  float lb = 0.f, lc = 0.f, ld = 0.f;
  const int no = 4 * RM + nc;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / A), a = (int)(i % A);
    const int j = owner[i];
    const float w = norm[i];
    float* g = G + i * no;
    const T* cp = cls + b * scb + a * sca;
    const int label = j >= 0 ? (int)gt[((long)b * cap + j) * 5] : -1;
    for (int c = 0; c < nc; ++c) {
      const float x = ldf(cp, (long)c * scc);
      const float t = c == label ? w : 0.f;
      // BCEWithLogits(pos_weight): (1-t) x + (1 + (pw-1) t) (log(1 + e^-|x|) + max(-x, 0))
      const float lw = 1.f + (pw - 1.f) * t;
      lc += (1.f - t) * x + lw * (log1pf(expf(-fabsf(x))) + fmaxf(-x, 0.f));
      g[4 * RM + c] = kc * ((1.f - t) - lw / (1.f + expf(x)));
    }
    const T* bp = box + b * sbb + a * sba;
    if (j < 0) {
      for (int k = 0; k < 4 * RM; ++k) g[k] = 0.f;
      continue;
    }
    float ax, ay, st;
    anchor_of(lt, a, ax, ay, st);
    const float* g5 = gt + ((long)b * cap + j) * 5;
    const float tx1 = g5[1] / st, ty1 = g5[2] / st, tx2 = g5[3] / st, ty2 = g5[4] / st;
    float p[4][RM], d[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) d[s] = side_softmax(bp, sbc, s, p[s]);
    // CIoU on the decoded box; seeds = the 4 side distances
    D4 dl = dc(d[0]), dt = dc(d[1]), dr = dc(d[2]), db = dc(d[3]);
    dl.d[0] = 1.f; dt.d[1] = 1.f; dr.d[2] = 1.f; db.d[3] = 1.f;
    D4 ci = ciou_d(dc(ax) - dl, dc(ay) - dt, dc(ax) + dr, dc(ay) + db, tx1, ty1, tx2, ty2);
    lb += (1.f - ci.v) * w;
    // DFL targets (bbox2dist, clamp to reg_max - 1 - 0.01)
    const float tgt[4] = {fminf(fmaxf(ax - tx1, 0.f), RM - 1 - 0.01f), fminf(fmaxf(ay - ty1, 0.f), RM - 1 - 0.01f),
                          fminf(fmaxf(tx2 - ax, 0.f), RM - 1 - 0.01f), fminf(fmaxf(ty2 - ay, 0.f), RM - 1 - 0.01f)};
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int tl = (int)tgt[s];
      const float wl = (float)(tl + 1) - tgt[s], wr = 1.f - wl;
      dsum += -logf(p[s][tl]) * wl - logf(p[s][tl + 1]) * wr;
      // d/d logit_k: box term through the expectation, dfl term through the softmax
      const float dbox = -w * ci.d[s];  // d (1 - CIoU) w / d dist_s
#pragma unroll
      for (int k = 0; k < RM; ++k) {
        const float de = p[s][k] * ((float)k - d[s]);
        const float ddfl = (p[s][k] - (k == tl ? wl : 0.f) - (k == tl + 1 ? wr : 0.f)) * 0.25f * w;
        g[s * RM + k] = kb * dbox * de + kd * ddfl;
      }
    }
    ld += dsum * 0.25f * w;
  }
  float v[3] = {lb, lc, ld};
  block_partials<3>(v, part);
}

__global__ void tal_finalize_kernel(const float* __restrict__ acc, float bs, float* __restrict__ loss,
                                    float* __restrict__ items) {
  const float tss = acc[3];
  const float lbox = acc[0] / tss * 7.5f, lcls = acc[1] / tss * 0.5f, ldfl = acc[2] / tss * 1.5f;
  items[0] = lbox;
  items[1] = lcls;
  items[2] = ldfl;
  loss[0] = (lbox + lcls + ldfl) * bs;
}

// flatten per-level NHWC head outputs [B, H_l, W_l, no] (pixel stride ps_l) into F[b][a][no]
template <typename T>
__global__ void tal_flatten_kernel(const T* __restrict__ x, long xps, int B, int HW, int A, int a0, int no,
                                   T* __restrict__ F, int backward) {
  const long n = (long)B * HW * no;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % no);
    const long t = i / no;
    const int p = (int)(t % HW), b = (int)(t / HW);
    const long fi = ((long)b * A + a0 + p) * no + c;
    const long xi = ((long)b * HW + p) * xps + c;
    if (backward) const_cast<T*>(x)[xi] = F[fi];
    else F[fi] = x[xi];
  }
}

// TDetect inference output y[b][4 + nc][a]: xywh (pixels) from the DFL expectation, sigmoid scores
template <typename T>
__global__ void tal_detect_out_kernel(const T* __restrict__ F, int B, int A, int nc, LevelTab lt, float* __restrict__ y) {
  const long n = (long)B * A;
  const int no = 4 * RM + nc;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / A), a = (int)(i % A);
    const T* fp = F + i * no;
    float ax, ay, st, p[RM], d[4];
    anchor_of(lt, a, ax, ay, st);
#pragma unroll
    for (int s = 0; s < 4; ++s) d[s] = side_softmax(fp, 1, s, p);
    const float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
    float* yb = y + (long)b * (4 + nc) * A + a;
    yb[0] = (x1 + x2) / 2 * st;
    yb[(long)A] = (y1 + y2) / 2 * st;
    yb[2L * A] = (x2 - x1) * st;
    yb[3L * A] = (y2 - y1) * st;
    for (int c = 0; c < nc; ++c) yb[(long)(4 + c) * A] = 1.f / (1.f + expf(-to_f(fp[4 * RM + c])));
  }
}

LevelTab make_levels(int nl, const int* H, const int* W, const float* stride) {
  LevelTab lt;
  lt.nl = nl;
  int a = 0;
  for (int l = 0; l < nl; ++l) {
    lt.a0[l] = a;
    lt.W[l] = W[l];
    lt.stride[l] = stride[l];
    a += H[l] * W[l];
  }
  lt.a0[nl] = a;
  return lt;
}

inline int egrid(long n) { return grid_cap(ceil_div(n, 256), 8192); }

}  // namespace

#define TAL_T(dtype, ...)    \
  if (dtype) {               \
    using T = bf16;          \
    __VA_ARGS__;             \
  } else {                   \
    using T = float;         \
    __VA_ARGS__;             \
  }

DMY_API long dmy_tal_workspace_bytes(int B, int A, int cap) {
  // gt[B][cap][5] f32, cnt[B] i32, cand[B][cap][10] i32, nclaim/owner [B][A] i32, metric/norm [B][A] f32,
  // amax_m/amax_o [B][cap] i32, pbox [B][A][4] f32, acc[4] f32, per-block loss partials [8192][4] f32
  const long b = 4L * ((long)B * cap * 5 + B + (long)B * cap * TOPK + 2L * B * A + 2L * B * A + 2L * B * cap +
                       4L * B * A + 4 + 4L * 8192) + 16 * 256;  // + per-buffer 256-B alignment
  return b > 0x7fffffffL ? -1 : (int)b;
}

// targets [nt, 6] (img, cls, x, y, w, h normalised); box / cls = head outputs through (batch, channel,
// anchor) strides; levels (H, W, stride) per level; G = [B][A][64 + nc] fp32 gradient (see above)
DMY_API int dmy_tal_loss(int dtype, const void* box, long sbb, long sbc, long sba, const void* cls, long scb, long scc,
                         long sca, int B, int nc, int nl, const int* H, const int* W, const float* stride,
                         const float* targets, int nt, float alpha, float beta, float pos_weight, void* workspace,
                         float* G, float* loss, float* items, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (nl < 1 || nl > 8) return (int)hipErrorInvalidValue;
  LevelTab lt = make_levels(nl, H, W, stride);
  const int A = lt.a0[nl];
  const int cap = nt > 0 ? nt : 1;
  char* w = (char*)workspace;
  auto take = [&](long bytes) { char* p = w; w += (bytes + 255) / 256 * 256; return p; };
  float* gt = (float*)take(4L * B * cap * 5);
  int* cnt = (int*)take(4L * B);
  int* cand = (int*)take(4L * B * cap * TOPK);
  int* nclaim = (int*)take(4L * B * A);
  int* owner = (int*)take(4L * B * A);
  float* metric = (float*)take(4L * B * A);
  float* norm = (float*)take(4L * B * A);
  int* amax_m = (int*)take(4L * B * cap);
  int* amax_o = (int*)take(4L * B * cap);
  float* pbox = (float*)take(16L * B * A);
  float* acc = (float*)take(16);
  float* part = (float*)take(16L * 8192);  // egrid() caps the grid at 8192 blocks
  (void)hipMemsetAsync(nclaim, 0, 4L * B * A, st);
  (void)hipMemsetAsync(owner, 0xff, 4L * B * A, st);
  (void)hipMemsetAsync(amax_m, 0, 4L * B * cap, st);
  (void)hipMemsetAsync(amax_o, 0, 4L * B * cap, st);
  (void)hipMemsetAsync(acc, 0, 16, st);
  const float iw = (float)W[0] * stride[0], ih = (float)H[0] * stride[0];
  if (nt > 0) tal_targets_kernel<<<1, 256, 0, st>>>(targets, nt, B, iw, ih, cap, gt, cnt);
  else (void)hipMemsetAsync(cnt, 0, 4L * B, st);
  TAL_T(dtype, {
    const T* bx = (const T*)box;
    const T* cl = (const T*)cls;
    tal_decode_kernel<T><<<egrid((long)B * A), 256, 0, st>>>(bx, sbb, sbc, sba, B, A, lt, pbox);
    tal_topk_kernel<T><<<dim3(cap, B), 256, 0, st>>>(cl, scb, scc, sca, pbox, gt, cnt, B, A, cap, lt, alpha, beta, cand);
    tal_claim_kernel<<<egrid((long)B * cap * TOPK), 256, 0, st>>>(cand, cnt, B, A, cap, nclaim, owner);
    tal_resolve_kernel<T><<<egrid((long)B * A), 256, 0, st>>>(cl, scb, scc, sca, pbox, gt, cnt, nclaim, owner, B, A, cap,
                                                              lt, alpha, beta, metric, amax_m, amax_o);
    // loss sums: per-block partials folded in block order (deterministic, no float atomics)
    const int nb = egrid((long)B * A);
    tal_norm_kernel<<<nb, 256, 0, st>>>(owner, metric, amax_m, amax_o, B, A, cap, norm, part);
    tal_fold_kernel<1><<<1, 256, 0, st>>>(part, nb, acc, 3);
    tal_loss_kernel<T><<<nb, 256, 0, st>>>(bx, sbb, sbc, sba, cl, scb, scc, sca, gt, owner, norm, B, A, nc, cap, lt,
                                           pos_weight, acc, part, G);
    tal_fold_kernel<3><<<1, 256, 0, st>>>(part, nb, acc, 0);
  });
  tal_finalize_kernel<<<1, 1, 0, st>>>(acc, (float)B, loss, items);
  return (int)hipGetLastError();
}

DMY_API int dmy_tal_flatten(int dtype, const void* x, long xps, int B, int H, int W, int A, int a0, int no, void* F,
                            int backward, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TAL_T(dtype, tal_flatten_kernel<T><<<egrid((long)B * H * W * no), 256, 0, st>>>((const T*)x, xps, B, H * W, A, a0, no,
                                                                                   (T*)F, backward));
  return (int)hipGetLastError();
}

DMY_API int dmy_tal_detect_out(int dtype, const void* F, int B, int nc, int nl, const int* H, const int* W,
                               const float* stride, float* y, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (nl < 1 || nl > 8) return (int)hipErrorInvalidValue;
  LevelTab lt = make_levels(nl, H, W, stride);
  const int A = lt.a0[nl];
  TAL_T(dtype, tal_detect_out_kernel<T><<<egrid((long)B * A), 256, 0, st>>>((const T*)F, B, A, nc, lt, y));
  return (int)hipGetLastError();
}
