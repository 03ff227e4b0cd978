// Batched non_max_suppression on gfx950 (utils/general.py:633-725 + torchvision.ops.nms).
//
// Bit-exact contract with the reference CPU path:
//   * candidates: obj > conf; cls' = cls * obj (fp32); multi-label rows (r, j) with cls' > conf in
//     row-major order, or best class = FIRST max; optional class filter.
//   * order: stable descending score == ascending 64-bit key (~score_bits << 32 | r*nc + j); the
//     max_nms cut and torchvision's own stable sort both reduce to this one total order.
//   * suppression: greedy over that order, IoU(i, j) = inter / (area_i + area_j - inter) with
//     boxes offset by cls * 4096 (fp32 adds), suppress iff IoU > thr; every product/sum uses
//     explicit round-to-nearest intrinsics so no FMA contraction changes a bit.
//   * lazy IoU rows: only rows that are KEPT compute IoU against the rest, and the scan stops at
//     max_det kept rows, so work is O(n * kept) instead of the O(n^2) mask.
#include "common.h"

namespace {

constexpr unsigned long long PADKEY = 0xFFFFFFFFFFFFFFFFull;

struct NmsCfg {
  int A, no, nc;          // anchors per image, row width, classes
  float conf, iou;
  int multi, agnostic, max_det, max_nms;
  const unsigned char* cls_ok;  // nullable [nc] class filter
};

// score recomputation shared by candidate and gather kernels (identical fp32 ops)
DEV float cand_score(const float* row, int j) { return __fmul_rn(row[5 + j], row[4]); }

DEV int best_class(const float* row, int nc, float* sc) {
  int bj = 0;
  float bv = cand_score(row, 0);
  for (int j = 1; j < nc; ++j) {
    const float v = cand_score(row, j);
    if (v > bv) { bv = v; bj = j; }
  }
  *sc = bv;
  return bj;
}

__global__ void nms_candidates_kernel(const float* __restrict__ pred, NmsCfg cfg, unsigned long long* __restrict__ keys,
                                      long cap, int* __restrict__ counts) {
  const int b = blockIdx.y;
  const float* P = pred + (long)b * cfg.A * cfg.no;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < cfg.A; r += gridDim.x * blockDim.x) {
    const float* row = P + (long)r * cfg.no;
    if (!(row[4] > cfg.conf)) continue;
    if (cfg.multi) {
      for (int j = 0; j < cfg.nc; ++j) {
        const float s = cand_score(row, j);
        if (s > cfg.conf && (!cfg.cls_ok || cfg.cls_ok[j])) {
          const int slot = atomicAdd(counts + b, 1);
          if (slot < cap)
            keys[(long)b * cap + slot] = ((unsigned long long)(~__float_as_uint(s)) << 32) | (unsigned)(r * cfg.nc + j);
        }
      }
    } else {
      float s;
      const int j = best_class(row, cfg.nc, &s);
      if (s > cfg.conf && (!cfg.cls_ok || cfg.cls_ok[j])) {
        const int slot = atomicAdd(counts + b, 1);
        if (slot < cap)
          keys[(long)b * cap + slot] = ((unsigned long long)(~__float_as_uint(s)) << 32) | (unsigned)(r * cfg.nc + j);
      }
    }
  }
}

__global__ void pad_keys_kernel(unsigned long long* keys, long cap, const int* counts, int nimg) {
  const int b = blockIdx.y;
  const int n = min((long)counts[b], cap);
  for (long i = n + blockIdx.x * (long)blockDim.x + threadIdx.x; i < cap; i += (long)gridDim.x * blockDim.x)
    keys[(long)b * cap + i] = PADKEY;
}

// ---- bitonic sort of each image's segment (length cap = power of two)
__global__ void bitonic_global_kernel(unsigned long long* keys, long cap, long k, long j) {
  const int b = blockIdx.y;
  unsigned long long* K = keys + (long)b * cap;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < cap; i += (long)gridDim.x * blockDim.x) {
    const long l = i ^ j;
    if (l > i) {
      const unsigned long long a = K[i], c = K[l];
      const bool up = (i & k) == 0;
      if ((a > c) == up) { K[i] = c; K[l] = a; }
    }
  }
}

// all passes with j < 1024 for a 2048-element tile in LDS.  In the first call (k_begin 2: no global pass has moved a key
// between tiles yet) a tile wholly past the image's candidate count holds only pad keys (pad_keys_kernel), sorted in
// either direction: it is skipped -- later calls may not skip, a descending merge carries real keys to a block's end.
// When the whole segment is one tile (cap 2048), only the first P = pow2 >= count keys are sorted: the rest are pad
// keys (written here as the tile is loaded), so the network over the prefix leaves the segment ascending (batch-1 detect at random init:
// ~0 candidates, 27 us -> a few)
__global__ void __launch_bounds__(1024) bitonic_local_kernel(unsigned long long* keys, long cap, long k_begin, long k_end,
                                                             const int* counts) {
  __shared__ unsigned long long s[2048];
  const int b = blockIdx.y;
  unsigned long long* K = keys + (long)b * cap + (long)blockIdx.x * 2048;
  const long g0 = (long)blockIdx.x * 2048;
  const long n = min((long)counts[b], cap);
  if (k_begin == 2 && g0 >= n && cap > 2048) return;  // (one tile: still writes its pads)
  int P = 2048;
  const bool one = cap == 2048 && k_begin == 2;
  if (one) {
    P = 2;
    while (P < n) P <<= 1;
    k_end = P;
  }
  // one tile: the pad keys past the count are made here (dmy_nms_sort launches no pad_keys_kernel for cap 2048)
  s[threadIdx.x] = one && threadIdx.x >= n ? PADKEY : K[threadIdx.x];
  s[threadIdx.x + 1024] = one && threadIdx.x + 1024 >= n ? PADKEY : K[threadIdx.x + 1024];
  __syncthreads();
  for (long k = k_begin; k <= k_end; k <<= 1) {
    for (long j = (k >> 1) < 1024 ? (k >> 1) : 1024; j > 0; j >>= 1) {
      if (j >= 2048) continue;
      for (int t = threadIdx.x; t < P; t += 1024) {
        const int l = t ^ (int)j;
        if (l > t) {
          const unsigned long long a = s[t], c = s[l];
          const bool up = ((g0 + t) & k) == 0;
          if ((a > c) == up) { s[t] = c; s[l] = a; }
        }
      }
      __syncthreads();
    }
  }
  K[threadIdx.x] = s[threadIdx.x];
  K[threadIdx.x + 1024] = s[threadIdx.x + 1024];
}

// ---- greedy NMS, one block per image, lazy IoU rows
DEV void cand_box(const float* pred, const NmsCfg& cfg, int b, unsigned long long key, float* bx, float* score,
                  float* cls) {
  const unsigned rj = (unsigned)(key & 0xFFFFFFFFull);
  const int r = rj / cfg.nc, j = rj % cfg.nc;
  const float* row = pred + ((long)b * cfg.A + r) * cfg.no;
  // xywh2xyxy (general.py:539-546)
  const float hw = row[2] / 2.f, hh = row[3] / 2.f;
  bx[0] = __fsub_rn(row[0], hw);
  bx[1] = __fsub_rn(row[1], hh);
  bx[2] = __fadd_rn(row[0], hw);
  bx[3] = __fadd_rn(row[1], hh);
  *score = __uint_as_float(~(unsigned)(key >> 32));
  *cls = (float)j;
}

__global__ void __launch_bounds__(1024) nms_greedy_kernel(const float* __restrict__ pred, NmsCfg cfg,
                                                         const unsigned long long* __restrict__ keys, long cap,
                                                         int* __restrict__ counts, float* __restrict__ boxes,
                                                         float* __restrict__ out, int* __restrict__ nkeep,
                                                         int* __restrict__ ncand) {
  extern __shared__ unsigned long long dead[];  // ceil(n/64) words
  const int b = blockIdx.x;
  const int n = min(min(counts[b], (int)cap), cfg.max_nms);
  const int nw = (n + 63) / 64;
  float* B = boxes + (long)b * cfg.max_nms * 5;  // offset boxes + area, sorted order
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float bx[4], sc, cl;
    cand_box(pred, cfg, b, keys[(long)b * cap + i], bx, &sc, &cl);
    const float off = cfg.agnostic ? 0.f : __fmul_rn(cl, 4096.f);
    for (int q = 0; q < 4; ++q) B[i * 5 + q] = __fadd_rn(bx[q], off);
    B[i * 5 + 4] = __fmul_rn(__fsub_rn(B[i * 5 + 2], B[i * 5 + 0]), __fsub_rn(B[i * 5 + 3], B[i * 5 + 1]));
  }
  for (int w = threadIdx.x; w < nw; w += blockDim.x) dead[w] = 0ull;
  __syncthreads();
  __shared__ int kept;
  if (threadIdx.x == 0) kept = 0;
  __syncthreads();
  for (int w = 0; w < nw && kept < cfg.max_det; ++w) {
    while (true) {
      __syncthreads();
      const unsigned long long valid = (w == nw - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
      const unsigned long long alive = ~dead[w] & valid;
      if (alive == 0ull || kept >= cfg.max_det) break;
      const int i = w * 64 + __ffsll((long long)alive) - 1;
      __syncthreads();
      if (threadIdx.x == 0) {
        float bx[4], sc, cl;
        cand_box(pred, cfg, b, keys[(long)b * cap + i], bx, &sc, &cl);
        float* o = out + ((long)b * cfg.max_det + kept) * 6;
        o[0] = bx[0]; o[1] = bx[1]; o[2] = bx[2]; o[3] = bx[3]; o[4] = sc; o[5] = cl;
        atomicOr(&dead[w], 1ull << (i & 63));
        kept = kept + 1;
      }
      const float x1 = B[i * 5], y1 = B[i * 5 + 1], x2 = B[i * 5 + 2], y2 = B[i * 5 + 3], ai = B[i * 5 + 4];
      for (int jj = i + 1 + threadIdx.x; jj < n; jj += blockDim.x) {
        const float* c = B + jj * 5;
        const float iw = fmaxf(__fsub_rn(fminf(x2, c[2]), fmaxf(x1, c[0])), 0.f);
        const float ih = fmaxf(__fsub_rn(fminf(y2, c[3]), fmaxf(y1, c[1])), 0.f);
        const float inter = __fmul_rn(iw, ih);
        const float iou = __fdiv_rn(inter, __fsub_rn(__fadd_rn(ai, c[4]), inter));
        if (iou > cfg.iou) atomicOr(&dead[jj >> 6], 1ull << (jj & 63));
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    nkeep[b] = kept;
    if (ncand != nullptr) {  // the count leaves through ncand; the counter is zero again for the next call
      ncand[b] = counts[b];
      counts[b] = 0;
    }
  }
}


// ---- bitmask NMS for capacities <= kMaskCap (one IoU bitmask row per sorted candidate, then a one-wave scan).
// The lazy kernel above walks kept boxes one at a time with block barriers and global box reads per step (~3 us each:
// ~1 ms for 2,000 candidates). Here nms_mask_kernel computes every IoU(i, j > i) > thr bit in parallel with the lazy
// kernel's exact fp32 operations (IoU is symmetric in its rounding: the adds / min / max commute), and nms_scan_kernel
// resolves the greedy order per 64-row block: the diagonal word sequentially in scalar registers, then the kept rows'
// mask words ORed into the later blocks' removed words in parallel (one word per lane). Same keep set and order.
constexpr int kMaskCap = 4096;

// the offset box + area of sorted candidate i (nms_boxes_kernel's arithmetic)
DEV void offset_box(const float* pred, const NmsCfg& cfg, int b, unsigned long long key, float* o) {
  float bx[4], sc, cl;
  cand_box(pred, cfg, b, key, bx, &sc, &cl);
  const float off = cfg.agnostic ? 0.f : __fmul_rn(cl, 4096.f);
  for (int q = 0; q < 4; ++q) o[q] = __fadd_rn(bx[q], off);
  o[4] = __fmul_rn(__fsub_rn(o[2], o[0]), __fsub_rn(o[3], o[1]));
}

// grid (cap/64 row blocks, cap/64 column blocks, nimg), 64 threads: mask[b][i][cb] bit c = IoU(i, 64 cb + c) > thr, j > i.
// The boxes come straight from the sorted keys (offset_box): no separate boxes launch
__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ pred, NmsCfg cfg,
                                                      const unsigned long long* __restrict__ keys, long cap,
                                                      const int* __restrict__ counts,
                                                      unsigned long long* __restrict__ mask) {
  const int rb = blockIdx.x, cb = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  if (cb < rb) return;
  const int n = min(min(counts[b], (int)cap), cfg.max_nms);
  if (rb * 64 >= n) return;
  __shared__ float cbx[64][5];
  const int j0 = cb * 64;
  if (j0 + t < n) offset_box(pred, cfg, b, keys[(long)b * cap + j0 + t], cbx[t]);
  __syncthreads();
  const int i = rb * 64 + t;
  if (i >= n) return;
  float rbx[5];
  offset_box(pred, cfg, b, keys[(long)b * cap + i], rbx);
  const float x1 = rbx[0], y1 = rbx[1], x2 = rbx[2], y2 = rbx[3], ai = rbx[4];
  unsigned long long bits = 0ull;
  const int cend = min(64, n - j0);
  for (int c = 0; c < cend; ++c) {
    if (j0 + c <= i) continue;
    const float* q = cbx[c];
    const float iw = fmaxf(__fsub_rn(fminf(x2, q[2]), fmaxf(x1, q[0])), 0.f);
    const float ih = fmaxf(__fsub_rn(fminf(y2, q[3]), fmaxf(y1, q[1])), 0.f);
    const float inter = __fmul_rn(iw, ih);
    const float iou = __fdiv_rn(inter, __fsub_rn(__fadd_rn(ai, q[4]), inter));
    if (iou > cfg.iou) bits |= 1ull << c;
  }
  mask[((long)b * cap + i) * (cap / 64) + cb] = bits;
}

DEV unsigned long long readlane64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, l), hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}

// one wave per image; lane w holds the removed-bits word of candidates [64 w, 64 w + 64)
__global__ void __launch_bounds__(64) nms_scan_kernel(const float* __restrict__ pred, NmsCfg cfg,
                                                      const unsigned long long* __restrict__ keys, long cap,
                                                      int* __restrict__ counts,
                                                      const unsigned long long* __restrict__ mask,
                                                      float* __restrict__ out, int* __restrict__ nkeep,
                                                      int* __restrict__ ncand) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = min(min(counts[b], (int)cap), cfg.max_nms);
  const int nw = (n + 63) / 64, W = (int)(cap / 64);
  const unsigned long long* Mb = mask + (long)b * cap * W;
  unsigned long long removed = 0ull;
  int kept = 0;
  for (int rb = 0; rb < nw && kept < cfg.max_det; ++rb) {
    const int i = rb * 64 + lane;
    const unsigned long long diag = i < n ? Mb[(long)i * W + rb] : 0ull;
    const unsigned long long valid = (rb == nw - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
    unsigned long long alive = ~readlane64(removed, rb) & valid;
    unsigned long long keepm = 0ull;
    const int kbase = kept;
    while (alive != 0ull && kept < cfg.max_det) {
      const int t = __builtin_amdgcn_readfirstlane(__ffsll((long long)alive) - 1);
      keepm |= 1ull << t;
      ++kept;
      alive &= ~(readlane64(diag, t) | (1ull << t));
    }
    if ((keepm >> lane) & 1ull) {
      float bx[4], sc, cl;
      cand_box(pred, cfg, b, keys[(long)b * cap + i], bx, &sc, &cl);
      const int idx = kbase + __popcll(keepm & ((1ull << lane) - 1ull));
      float* o = out + ((long)b * cfg.max_det + idx) * 6;
      o[0] = bx[0]; o[1] = bx[1]; o[2] = bx[2]; o[3] = bx[3]; o[4] = sc; o[5] = cl;
    }
    if (lane > rb && lane < nw) {
      unsigned long long km = keepm;
      while (km != 0ull) {
        const int t = __ffsll((long long)km) - 1;
        km &= km - 1ull;
        removed |= Mb[(long)(rb * 64 + t) * W + lane];
      }
    }
  }
  if (lane == 0) {
    nkeep[b] = kept;
    if (ncand != nullptr) {  // the count leaves through ncand; the counter is zero again for the next call
      ncand[b] = counts[b];
      counts[b] = 0;
    }
  }
}

}  // namespace

DMY_API int dmy_nms_candidates(const float* pred, int nimg, int A, int no, float conf, int multi,
                               const unsigned char* cls_ok, unsigned long long* keys, long cap, int* counts,
                               void* stream) {
  NmsCfg cfg{A, no, no - 5, conf, 0.f, multi, 0, 0, 0, cls_ok};
  dim3 grid(grid_cap(ceil_div(A, 256), 256), nimg);
  nms_candidates_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(pred, cfg, keys, cap, counts);
  return (int)hipGetLastError();
}

// cap must be a power of two >= 2048; sorts each image's [0, cap) key segment ascending
DMY_API int dmy_nms_sort(unsigned long long* keys, long cap, const int* counts, int nimg, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 gp(grid_cap(ceil_div(cap, 256), 1024), nimg);
  if (cap > 2048) pad_keys_kernel<<<gp, 256, 0, st>>>(keys, cap, counts, nimg);  // cap 2048: bitonic_local pads
  dim3 gl((unsigned)(cap / 2048), nimg);
  bitonic_local_kernel<<<gl, 1024, 0, st>>>(keys, cap, 2, 2048, counts);
  for (long k = 4096; k <= cap; k <<= 1) {
    for (long j = k >> 1; j >= 2048; j >>= 1) bitonic_global_kernel<<<gp, 256, 0, st>>>(keys, cap, k, j);
    bitonic_local_kernel<<<gl, 1024, 0, st>>>(keys, cap, k, k, counts);
  }
  return (int)hipGetLastError();
}

DMY_API int dmy_nms_greedy(const float* pred, int nimg, int A, int no, float iou, int agnostic, int max_det,
                           int max_nms, const unsigned long long* keys, long cap, int* counts, float* boxes,
                           float* out, int* nkeep, int* ncand, void* stream) {
  NmsCfg cfg{A, no, no - 5, 0.f, iou, 0, agnostic, max_det, max_nms, nullptr};
  const size_t lds = sizeof(unsigned long long) * (size_t)((max_nms + 63) / 64);
  nms_greedy_kernel<<<nimg, 1024, lds, (hipStream_t)stream>>>(pred, cfg, keys, cap, counts, boxes, out, nkeep,
                                                                ncand);
  return (int)hipGetLastError();
}

DMY_API int dmy_nms_mask_rows() { return kMaskCap; }

// the bitmask path: cap (the sort capacity) <= dmy_nms_mask_rows(); mask holds nimg * cap * cap / 64 words
DMY_API int dmy_nms_greedy_mask(const float* pred, int nimg, int A, int no, float iou, int agnostic, int max_det,
                                int max_nms, const unsigned long long* keys, long cap, int* counts, float* boxes,
                                unsigned long long* mask, float* out, int* nkeep, int* ncand, void* stream) {
  if (cap > kMaskCap || cap % 64 != 0) return (int)hipErrorInvalidValue;
  NmsCfg cfg{A, no, no - 5, 0.f, iou, 0, agnostic, max_det, max_nms, nullptr};
  hipStream_t st = (hipStream_t)stream;
  (void)boxes;  // the mask kernel makes its boxes from the keys (the lazy path's scratch; kept in the ABI)
  nms_mask_kernel<<<dim3((unsigned)(cap / 64), (unsigned)(cap / 64), nimg), 64, 0, st>>>(pred, cfg, keys, cap, counts,
                                                                                          mask);
  nms_scan_kernel<<<nimg, 64, 0, st>>>(pred, cfg, keys, cap, counts, mask, out, nkeep, ncand);
  return (int)hipGetLastError();
}
