// Training augmentation tail on the GPU ("GPU-side uint8 normalise"): for a batch of
// mosaic / letterbox canvases, one kernel does what datasets.py:552-622 does per image on the host after the
// random draws -- random_perspective's warp (cv2.warpAffine / warpPerspective, INTER_LINEAR, border 114), mixup,
// augment_hsv (BGR -> HSV, LUTs, HSV -> BGR), the up-down / left-right flips, BGR -> RGB and HWC -> CHW -- and
// writes the uint8 [B, 3, H, W] batch that Model.to_input consumes.  The arithmetic is the host restatement's
// (dmayolo/augment.py) operation for operation: the 1/32-pixel fixed-point inverse map from double products with
// round-half-even, the 15-bit bilinear weights ((32 - fx)(32 - fy) * 32 ... , exact), (v + 2^14) >> 15, OpenCV's
// integer BGR2HSV (tables built on the host with the same double formula), the float32 HSV2BGR sector formula with
// every product / difference rounded separately (no contraction), and mixup's float64 blend truncated to uint8 --
// so the batch equals the host path bit for bit (tests/test_gpu_augment.py).  One thread per output pixel; the
// canvases are read through L2 (4 taps x 3 bytes), the output planes are written coalesced.
#include "common.h"

// Every float / double operation here must round exactly as the host restatement's numpy ops do: this file is
// built with -ffp-contract=off (__graft_entry__ FILE_FLAGS) -- with the library's -ffp-contract=fast, 1 - s * h
// became one FMA and moved values on a rounding boundary by one level (234 of the 2^24 colours through HSV).
#pragma clang fp contract(off)

namespace {

// Host-built descriptor, one per image (C ABI: 8-byte fields first; sizeof checked by dmy_aug_desc_bytes).
struct AugDesc {
  const unsigned char* src;   // canvas, HWC BGR uint8, rows of W * 3 bytes
  const unsigned char* src2;  // mixup canvas (nullptr: no mixup)
  double m[9];                // inverse map: affine [A11, A12, B1, A21, A22, B2, -, -, -]; perspective: 3 x 3 inverse
  double m2[9];
  double mix_r;               // mixup ratio r: out = trunc(a * r + b * (1 - r))
  int H, W, H2, W2;
  int persp, persp2, copy, copy2;  // copy: the canvas IS the output (no warp: same size, identity)
  int flipud, fliplr, use_lut, pad_;
  unsigned char lut[3][256];  // hue / sat / val LUTs of augment_hsv
};
static_assert(sizeof(AugDesc) == 984, "AugDesc layout is part of the C ABI");

__constant__ int c_sdiv[256];
__constant__ int c_hdiv[256];

__device__ __forceinline__ long long rne(double v) { return (long long)rint(v); }

// source coordinates in 1/32 pixel (cv2 warpAffine / warpPerspective with INTER_LINEAR, imgwarp.cpp)
__device__ __forceinline__ void map_xy(const double* m, int persp, int x, int y, long long& X, long long& Y) {
  const double xd = (double)x, yd = (double)y;
  if (!persp) {
    const long long adelta = rne(__dmul_rn(__dmul_rn(m[0], xd), 1024.0));
    const long long bdelta = rne(__dmul_rn(__dmul_rn(m[3], xd), 1024.0));
    const long long X0 = rne(__dmul_rn(__dadd_rn(__dmul_rn(m[1], yd), m[2]), 1024.0)) + 16;
    const long long Y0 = rne(__dmul_rn(__dadd_rn(__dmul_rn(m[4], yd), m[5]), 1024.0)) + 16;
    X = (X0 + adelta) >> 5;
    Y = (Y0 + bdelta) >> 5;
  } else {
    double w = __dadd_rn(__dadd_rn(__dmul_rn(m[6], xd), __dmul_rn(m[7], yd)), m[8]);
    w = w != 0.0 ? __ddiv_rn(32.0, w) : 0.0;
    double fx = __dmul_rn(__dadd_rn(__dadd_rn(__dmul_rn(m[0], xd), __dmul_rn(m[1], yd)), m[2]), w);
    double fy = __dmul_rn(__dadd_rn(__dadd_rn(__dmul_rn(m[3], xd), __dmul_rn(m[4], yd)), m[5]), w);
    fx = fmin(fmax(fx, -2147483648.0), 2147483647.0);
    fy = fmin(fmax(fy, -2147483648.0), 2147483647.0);
    X = rne(fx);
    Y = rne(fy);
  }
}

// bilinear tap of remap (BORDER_CONSTANT 114): bgr[3]
__device__ __forceinline__ void sample(const unsigned char* src, int H, int W, long long X, long long Y, int* bgr) {
  const long long sx = X >> 5, sy = Y >> 5;
  const int fx = (int)(X & 31), fy = (int)(Y & 31);
  if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
    bgr[0] = bgr[1] = bgr[2] = 114;
    return;
  }
  const int w[4] = {(32 - fx) * (32 - fy) * 32, fx * (32 - fy) * 32, (32 - fx) * fy * 32, fx * fy * 32};
  int acc[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long xx = sx + (k & 1), yy = sy + (k >> 1);
    const bool in = xx >= 0 && xx < W && yy >= 0 && yy < H;
    const unsigned char* p = src + (in ? (yy * W + xx) * 3 : 0);
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += (in ? (int)p[c] : 114) * w[k];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int v = (acc[c] + (1 << 14)) >> 15;
    bgr[c] = v < 0 ? 0 : (v > 255 ? 255 : v);
  }
}

__device__ __forceinline__ void fetch(const unsigned char* src, int H, int W, const double* m, int persp, int copy,
                                      int x, int y, int* bgr) {
  if (copy) {
    const unsigned char* p = src + ((long long)y * W + x) * 3;
    bgr[0] = p[0];
    bgr[1] = p[1];
    bgr[2] = p[2];
    return;
  }
  long long X, Y;
  map_xy(m, persp, x, y, X, Y);
  sample(src, H, W, X, Y, bgr);
}

__device__ __forceinline__ unsigned char to_u8(float v) {  // saturate_cast<uchar>(v * 255.f), round half to even
  const float r = rintf(__fmul_rn(v, 255.f));
  return (unsigned char)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
}

__global__ void __launch_bounds__(256) augment_batch_kernel(const AugDesc* __restrict__ descs, unsigned char* out,
                                                            int OH, int OW) {
  const AugDesc& d = descs[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= OH * OW) return;
  const int y = i / OW, x = i - y * OW;
  const int xs = d.fliplr ? OW - 1 - x : x, ys = d.flipud ? OH - 1 - y : y;
  int bgr[3];
  fetch(d.src, d.H, d.W, d.m, d.persp, d.copy, xs, ys, bgr);
  if (d.src2 != nullptr) {
    int b2[3];
    fetch(d.src2, d.H2, d.W2, d.m2, d.persp2, d.copy2, xs, ys, b2);
    const double r = d.mix_r, q = __dsub_rn(1.0, r);
#pragma unroll
    for (int c = 0; c < 3; ++c) bgr[c] = (int)__dadd_rn(__dmul_rn((double)bgr[c], r), __dmul_rn((double)b2[c], q));
  }
  if (d.use_lut) {
    // cvtColor BGR2HSV, 8U, hrange 180 (integer)
    const int b = bgr[0], g = bgr[1], r = bgr[2];
    const int v = max(max(b, g), r), vmin = min(min(b, g), r), diff = v - vmin;
    const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    const int s = (diff * c_sdiv[v] + (1 << 11)) >> 12;
    int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + (~vg & (r - g + 4 * diff))));
    h = (h * c_hdiv[diff] + (1 << 11)) >> 12;
    h += h < 0 ? 180 : 0;
    const int H_ = d.lut[0][h & 255], S_ = d.lut[1][s], V_ = d.lut[2][v];
    // cvtColor HSV2BGR, 8U (float32 sector formula)
    float hf = __fmul_rn((float)H_, (float)(6.0 / 180));
    const float sf = __fmul_rn((float)S_, (float)(1.0 / 255)), vf = __fmul_rn((float)V_, (float)(1.0 / 255));
    if (hf < 0.f) hf = __fadd_rn(hf, 6.f);
    else if (hf >= 6.f) hf = __fsub_rn(hf, 6.f);
    int sector = (int)floorf(hf);
    hf = __fsub_rn(hf, (float)sector);
    if (sector < 0 || sector >= 6) {
      sector = 0;
      hf = 0.f;
    }
    float tab[4];
    tab[0] = vf;
    tab[1] = __fmul_rn(vf, __fsub_rn(1.f, sf));
    tab[2] = __fmul_rn(vf, __fsub_rn(1.f, __fmul_rn(sf, hf)));
    tab[3] = __fmul_rn(vf, __fsub_rn(1.f, __fmul_rn(sf, __fsub_rn(1.f, hf))));
    const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
#pragma unroll
    for (int c = 0; c < 3; ++c) bgr[c] = to_u8(sf == 0.f ? vf : tab[sd[sector][c]]);
  }
  const long long plane = (long long)OH * OW;
  unsigned char* o = out + (long long)blockIdx.y * 3 * plane + i;
  o[0] = (unsigned char)bgr[2];  // R
  o[plane] = (unsigned char)bgr[1];
  o[2 * plane] = (unsigned char)bgr[0];
}

// ---- mosaic composition (datasets.py:680-724, load_image :659-675): the 2s x 2s canvas of a 4-image mosaic, built
// on the GPU from the DECODED images (the workers only decode and draw).  Each quadrant is a rectangle
// [y1a, y2a) x [x1a, x2a) of the canvas filled from the image resized to (h, w) by cv2 INTER_LINEAR (resize_linear:
// 11-bit fixed-point coefficients, built on the host per axis exactly as data._linear_coeffs does), offset by
// (y1b - y1a, x1b - x1a); the four rectangles are disjoint; everything else is 114.  Integer arithmetic only, so the
// canvas equals the host restatement's bit for bit (tests/test_gpu_augment.py).
struct MosaicQuad {
  const unsigned char* src;  // decoded image, HWC BGR uint8, H0 x W0
  const int* xt;             // [4][w]: x0, x1, a0, a1 of the resized columns
  const int* yt;             // [4][h]: y0, y1, b0, b1 of the resized rows
  int H0, W0, h, w;
  int x1a, y1a, x2a, y2a, x1b, y1b;
  int rgb;  // 1: the decoded image is RGB (load_image_raw), the canvas BGR
  int pad1;
};
struct MosaicDesc {
  unsigned char* dst;  // canvas, HWC BGR uint8, S2 x S2
  int S2, pad;
  MosaicQuad q[4];
};
static_assert(sizeof(MosaicQuad) == 72 && sizeof(MosaicDesc) == 304, "MosaicDesc layout is part of the C ABI");

__global__ void __launch_bounds__(256) mosaic_compose_kernel(const MosaicDesc* __restrict__ descs) {
  const MosaicDesc& d = descs[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= d.S2 * d.S2) return;
  const int y = i / d.S2, x = i - y * d.S2;
  int bgr[3] = {114, 114, 114};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const MosaicQuad& q = d.q[k];
    if (x < q.x1a || x >= q.x2a || y < q.y1a || y >= q.y2a) continue;
    const int xr = x - q.x1a + q.x1b, yr = y - q.y1a + q.y1b;  // pixel of the resized image
    const int x0 = q.xt[xr], x1 = q.xt[q.w + xr], a0 = q.xt[2 * q.w + xr], a1 = q.xt[3 * q.w + xr];
    const int y0 = q.yt[yr], y1 = q.yt[q.h + yr], b0 = q.yt[2 * q.h + yr], b1 = q.yt[3 * q.h + yr];
    const unsigned char* r0 = q.src + (long long)y0 * q.W0 * 3;
    const unsigned char* r1 = q.src + (long long)y1 * q.W0 * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int cs = q.rgb ? 2 - c : c;  // source channel of canvas channel c (BGR)
      const long long h0 = (long long)r0[x0 * 3 + cs] * a0 + (long long)r0[x1 * 3 + cs] * a1;
      const long long h1 = (long long)r1[x0 * 3 + cs] * a0 + (long long)r1[x1 * 3 + cs] * a1;
      const long long v = (h0 * b0 + h1 * b1 + (1LL << 21)) >> 22;
      bgr[c] = v < 0 ? 0 : (v > 255 ? 255 : (int)v);
    }
  }
  unsigned char* o = d.dst + (long long)i * 3;
  o[0] = (unsigned char)bgr[0];
  o[1] = (unsigned char)bgr[1];
  o[2] = (unsigned char)bgr[2];
}

bool tables_ready = false;

}  // namespace

DMY_API long dmy_mosaic_desc_bytes() { return (long)sizeof(MosaicDesc); }

// descs: device array of n MosaicDesc (S2 = the largest canvas side); each canvas written into its dst
DMY_API int dmy_mosaic_compose(const void* descs, int n, int S2, void* stream) {
  if (n <= 0 || S2 <= 0) return 0;
  const dim3 grid((unsigned)(((long)S2 * S2 + 255) / 256), (unsigned)n);
  mosaic_compose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const MosaicDesc*)descs);
  return (int)hipGetLastError();
}

DMY_API long dmy_aug_desc_bytes() { return (long)sizeof(AugDesc); }

// descs: device array of n AugDesc; out: uint8 [n, 3, OH, OW]
DMY_API int dmy_augment_batch(const void* descs, int n, void* out, int OH, int OW, void* stream) {
  if (n <= 0 || OH <= 0 || OW <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (!tables_ready) {  // OpenCV RGB2HSV_b tables: saturate_cast<int>((255 << 12) / (1. * i)), (180 << 12) / (6. * i)
    int sdiv[256], hdiv[256];
    sdiv[0] = hdiv[0] = 0;
    for (int i = 1; i < 256; ++i) {
      sdiv[i] = (int)rint((255 << 12) / (1.0 * i));
      hdiv[i] = (int)rint((180 << 12) / (6.0 * i));
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_sdiv), sdiv, sizeof(sdiv)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_hdiv), hdiv, sizeof(hdiv)) != hipSuccess)
      return (int)hipErrorInvalidValue;
    tables_ready = true;
  }
  const dim3 grid((unsigned)((OH * OW + 255) / 256), (unsigned)n);
  augment_batch_kernel<<<grid, 256, 0, st>>>((const AugDesc*)descs, (unsigned char*)out, OH, OW);
  return (int)hipGetLastError();
}
