// Fused backward of a train-mode 1x1 stride-1 Conv -> BatchNorm -> activation layer, gfx950.
//
// Replaces, for the 1x1 `Conv` modules (models/common.py:67-73 with k = 1: act(bn(conv(x))), reached from every C3 /
// Bottleneck / SPPFCSPC / CoorAttention 1x1 projection, :159-182, :1257-1276), the last three of the four passes the
// reference's autograd runs per layer:
//   bn_bwd_apply (reads dy, z, writes dz) -> data-grad dx (+)= dz W (reads dz) -> weight-grad dW += dz^T x (reads dz, x)
// as ONE persistent launch that computes dz in registers from (dy, z) with dmy_bn_bwd_apply's expression, stages the
// bf16 dz tile in LDS and feeds both GEMMs from it: dz never reaches HBM.  Per layer that removes 3 passes of M x K
// bf16 (dz written once, read twice) and two launches; the reduce pass (Sum du, Sum du * xhat) stays in front of it,
// because the apply needs the whole layer's sums.
//
// Block = 4 waves (one per SIMD), persistent over TP-pixel tiles, 1 block per CU:
//   * Wt (the IHWO weight copy, [C][K]) is loaded into LDS once per block (16-B chunks XOR-swizzled by row).
//   * Per tile: the (dy, z, x) loads of the NEXT tile are in flight in registers while this tile computes.  dz is
//     computed by the thread that loaded it (its 8-channel chunk is fixed for the launch, so the BN / act coefficients
//     stay in registers) and written with x into k-major LDS tiles ([pixel][channel], conv.hip's kmaj swizzle).
//   * Data-grad: D^T[c][px] = sum_k Wt[c][k] dz[px][k] (v_mfma_f32_16x16x32_bf16, W from LDS, dz row fragments from
//     LDS), in units of 32 pixels x 64 channels per wave; a permlane16 swap gives each lane 8 consecutive channels of one
//     pixel, so a pixel's 128-B line leaves in two back-to-back 16-B stores (the store order round 4 measured fastest).
//     An accumulating data-grad (functional.GradSink) adds the bf16-rounded result to the stored dx, as conv.hip does.
//   * Weight-grad: dW[k][c] += sum_px dz[px][k] x[px][c], both operands read transposed from LDS
//     (ds_read_b64_tr_b16); each wave owns a (K/2) x (C/2) block of fp32 accumulators for the whole launch and adds it
//     to dw with fp32 atomics at the end (dw is the caller-zeroed arena slice, OIHW = [K][C] for a 1x1).
// Shapes: the (K, C) pairs of plan() (K in {64, 128, 256}, C <= 512; Wt + the two tiles fit the LDS and the
// weight-grad accumulators fit the registers, with the dx channels split over 2 blocks per tile where one block's would
// not), 16-B aligned pixel strides; the host query dmy_conv1x1_bwd_bn_ok says which, everything else keeps the
// three-pass path.
#include "common.h"

namespace {
namespace b1 {

constexpr unsigned kOob = 0xFFFFFFF0u;  // a buffer offset past every record count: the load returns zeros

DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
DEV uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return *reinterpret_cast<const uint4*>(&v);
}

// k-major tile [k = pixel][ROW = channels], 16-B chunks XOR-swizzled per pixel row so the transposed reads of 8
// consecutive pixels are bank-conflict free (the kmaj layout of conv.hip's weight-grad tiles)
template <int ROW> DEV int ksw(int k, int row) {
  constexpr int RB = ROW * 2;
  const int c = row >> 3, w = row & 7;
  int key;
  if constexpr (RB >= 256) key = 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else key = 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  return k * ROW + (((c ^ key) & (ROW / 8 - 1)) << 3) + w;
}
// Wt rows ([C][K], K contiguous): chunk index XOR-ed with the row so 16 rows' same chunk hit 16 distinct bank groups
template <int K> DEV int wsw(int r, int ch) {
  if constexpr (K * 2 >= 256) return (ch ^ (r & 15)) & (K / 8 - 1);
  else return (ch ^ ((r >> 1) & 7)) & (K / 8 - 1);
}
// transposed fragment of a k-major tile: lane (g, il) gets T[k0 + 8g .. +8][r0 + il] (MFMA A / B layout, 8 consecutive
// reduction elements of row r0 + il)
template <int ROW> DEV bf16x8 frag_t(const bf16* base, int r0, int k0, int lane) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3;
  const bf16* a0 = base + ksw<ROW>(k0 + 8 * g + q, r0 + 4 * p);
  const bf16* a1 = base + ksw<ROW>(k0 + 8 * g + 4 + q, r0 + 4 * p);
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
DEV unsigned pk2(float a, float b) {
  const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (unsigned)*reinterpret_cast<const unsigned short*>(&x) |
         ((unsigned)*reinterpret_cast<const unsigned short*>(&y) << 16);
}

// K = dz channels, CB = the block's slice of dx channels (C / nsplit), TP = pixels per tile, PX = 16-pixel tiles per
// data-grad unit (a unit = 16 PX pixels x 64 channels)
template <int K, int CB, int TP, int PX>
struct Shape {
  static constexpr int NT = 256, KCH = K / 8, CCH = CB / 8;
  static constexpr int NDZ = TP * KCH / NT, NX = TP * CCH / NT;  // 16-B chunks per thread and tile (dy / z, x)
  static constexpr int RDZ = NT / KCH, RXS = NT / CCH;            // pixel rows between a thread's chunks
  static constexpr int KW = K / 2, CW = CB / 2, MI = KW / 16, NJ = CW / 16;  // weight-grad block of a wave (2 x 2)
  static constexpr int PGN = TP / (16 * PX), U = PGN * (CB / 64), UPW = (U + 3) / 4;  // data-grad units
  static constexpr int LDS = (CB * K + TP * K + TP * CB) * 2;
  static_assert(K % 64 == 0 && CB % 64 == 0 && NT % KCH == 0 && NT % CCH == 0, "channels");
  static_assert(NDZ >= 1 && NX >= 1 && TP % 32 == 0 && TP % (16 * PX) == 0 && U >= 1, "tile");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// nsplit > 1 (layers whose Wt or weight-grad accumulators do not fit one block): the dx channels are split over nsplit
// blocks, each with its own slice of Wt, x, dx and dw, all computing the tile's whole dz (the transform runs nsplit
// times, dy / z are read once from HBM and nsplit - 1 times from L2).  Blocks b and b + 8 share an XCD (dispatch is
// round-robin over the 8 XCDs), so the nsplit blocks of one tile group are placed 8 apart and walk the same tiles.
template <int K, int CB, int TP, int PX>
__global__ void __launch_bounds__(256, 1) conv1x1_bwd_bn(
    const bf16* __restrict__ dy, long dps, const bf16* __restrict__ z, const bf16* __restrict__ x, long xps,
    const bf16* __restrict__ wt, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, int act, const float* __restrict__ ca,
    const float* __restrict__ cb, const float* __restrict__ cc, bf16* __restrict__ dx, long bps, int accumulate,
    float* __restrict__ dw, float* __restrict__ dws, long M, int ntiles, int C, int nsplit, unsigned dyb, unsigned zb,
    unsigned xb) {
  using S = Shape<K, CB, TP, PX>;
  extern __shared__ __attribute__((aligned(16))) char b1_smem[];
  bf16* ws = reinterpret_cast<bf16*>(b1_smem);  // the block's Wt rows [CB][K]
  bf16* dzs = ws + CB * K;                       // dz tile [TP][K]
  bf16* xs = dzs + TP * K;                       // x tile [TP][CB]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, il = lane & 15;
  const int slot = blockIdx.x >> 3, cs = slot % nsplit;
  const int grp = (blockIdx.x & 7) + 8 * (slot / nsplit), ngrp = gridDim.x / nsplit;
  const int cbase = cs * CB;  // first dx channel of this block
  x += cbase;
  dx += cbase;
  dw += cbase;

  for (int e = tid; e < CB * S::KCH; e += S::NT) {
    const int r = e / S::KCH, ch = e % S::KCH;
    *reinterpret_cast<uint4*>(ws + r * K + (wsw<K>(r, ch) << 3)) =
        *reinterpret_cast<const uint4*>(wt + (long)(cbase + r) * K + ch * 8);
  }

  // this thread's fixed 8-channel chunk of dz, and dmy_bn_bwd_apply's coefficients for it:
  // dz = ca * (dy * act'(z * scale + shift)) + (cb - cc * invstd * mean) + cc * invstd * z
  const int kc8 = (tid % S::KCH) * 8, xc8 = (tid % S::CCH) * 8;
  float sc[8], sh[8], k1[8], k0[8], k2[8];
  {
    float t0[8], t1[8];
    ldf<8>(scale + kc8, sc);
    ldf<8>(shift + kc8, sh);
    ldf<8>(ca + kc8, k1);
    ldf<8>(cc + kc8, k2);
    ldf<8>(invstd + kc8, t0);
    ldf<8>(cb + kc8, k0);
    ldf<8>(mean + kc8, t1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k2[j] = k2[j] * t0[j];
      k0[j] = k0[j] - k2[j] * t1[j];
    }
  }

  // x's descriptor starts at the block's channel slice: the record count shrinks by the same bytes
  const __amdgpu_buffer_rsrc_t rdy = rsrc(dy, dyb), rz = rsrc(z, zb), rx = rsrc(x, xb - 2u * cbase);
  uint4 pg[S::NDZ], pz[S::NDZ], pxv[S::NX];
  auto issue = [&](int t) {
    const long m0 = (long)t * TP;
#pragma unroll
    for (int j = 0; j < S::NDZ; ++j) {
      const long m = m0 + tid / S::KCH + j * S::RDZ;
      const bool ok = m < M;
      pg[j] = bload(rdy, ok ? (unsigned)((m * dps + kc8) * 2) : kOob);
      pz[j] = bload(rz, ok ? (unsigned)((m * K + kc8) * 2) : kOob);
    }
#pragma unroll
    for (int j = 0; j < S::NX; ++j) {
      const long m = m0 + tid / S::CCH + j * S::RXS;
      pxv[j] = bload(rx, m < M ? (unsigned)((m * xps + xc8) * 2) : kOob);
    }
  };

  f32x4 wacc[S::MI][S::NJ];
#pragma unroll
  for (int i = 0; i < S::MI; ++i)
#pragma unroll
    for (int j = 0; j < S::NJ; ++j) wacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wk = wid >> 1, wc = wid & 1;
  const int chq = (g & 1) * 16 + (g >> 1) * 8;  // this lane's 8 channels of a 32-channel pair after the permlane swap

  int t = grp;
  if (t < ntiles) issue(t);
  __syncthreads();  // Wt in LDS
  for (; t < ntiles; t += ngrp) {
    const long m0 = (long)t * TP;
#pragma unroll
    for (int j = 0; j < S::NDZ; ++j) {
      float zf[8], gf[8], o[8];
      unpack<bf16>(pz[j], zf);
      unpack<bf16>(pg[j], gf);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = zf[e] * sc[e] + sh[e];
      act_grad_n<8>(act, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = k1[e] * (gf[e] * o[e]) + k0[e] + k2[e] * zf[e];
      pg[j] = pack<bf16>(o);
    }
    __syncthreads();  // the previous tile's readers of dzs / xs are done
#pragma unroll
    for (int j = 0; j < S::NDZ; ++j)
      *reinterpret_cast<uint4*>(dzs + ksw<K>(tid / S::KCH + j * S::RDZ, kc8)) = pg[j];
#pragma unroll
    for (int j = 0; j < S::NX; ++j)
      *reinterpret_cast<uint4*>(xs + ksw<CB>(tid / S::CCH + j * S::RXS, xc8)) = pxv[j];
    __syncthreads();

    // the stored dx of an accumulating data-grad: loaded before the next tile's prefetch so waiting for them does not
    // wait for the prefetch (one in-order vmcnt)
    uint4 old[S::UPW][PX][2];
    if (accumulate) {
#pragma unroll
      for (int s = 0; s < S::UPW; ++s) {
        const int u = wid + 4 * s, p0 = (u % S::PGN) * 16 * PX, c0 = (u / S::PGN) * 64;
        if (u >= S::U) break;
#pragma unroll
        for (int pt = 0; pt < PX; ++pt) {
          const long m = m0 + p0 + pt * 16 + il;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            old[s][pt][h] = m < M ? *reinterpret_cast<const uint4*>(dx + m * bps + c0 + h * 32 + chq)
                                  : make_uint4(0, 0, 0, 0);
        }
      }
    }
    if (t + ngrp < ntiles) issue(t + ngrp);

    // data-grad units
#pragma unroll
    for (int s = 0; s < S::UPW; ++s) {
      const int u = wid + 4 * s, p0 = (u % S::PGN) * 16 * PX, c0 = (u / S::PGN) * 64;
      if (u >= S::U) break;  // fewer units than waves (narrow column slices): the idle waves go on to the weight-grad
      f32x4 acc[4][PX];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int pt = 0; pt < PX; ++pt) acc[ct][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int kc = 0; kc < K / 32; ++kc) {
        bf16x8 b[PX];
#pragma unroll
        for (int pt = 0; pt < PX; ++pt)
          b[pt] = *reinterpret_cast<const bf16x8*>(dzs + ksw<K>(p0 + pt * 16 + il, kc * 32 + 8 * g));
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int r = c0 + ct * 16 + il;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(ws + r * K + (wsw<K>(r, kc * 4 + g) << 3));
#pragma unroll
          for (int pt = 0; pt < PX; ++pt)
            acc[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[pt], acc[ct][pt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int pt = 0; pt < PX; ++pt) {
        const long m = m0 + p0 + pt * 16 + il;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // channels c0 + 32 h .. + 32: the two halves of the pixel's 128-B line
          const f32x4 &a = acc[2 * h][pt], &b = acc[2 * h + 1][pt];
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk2(a[0], a[1]), pk2(b[0], b[1]), false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk2(a[2], a[3]), pk2(b[2], b[3]), false, false);
          uint4 v;
          v.x = s0[0];
          v.y = s1[0];
          v.z = s0[1];
          v.w = s1[1];
          if (accumulate) {
            float f[8], o[8];
            unpack<bf16>(v, f);
            unpack<bf16>(old[s][pt][h], o);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += o[j];
            v = pack<bf16>(f);
          }
          if (m < M) *reinterpret_cast<uint4*>(dx + m * bps + c0 + h * 32 + chq) = v;
        }
      }
    }

    // weight-grad: this wave's (K / 2) x (CB / 2) block over the tile's pixels (rows past M are zero in xs)
#pragma unroll
    for (int ps = 0; ps < TP / 32; ++ps) {
      bf16x8 a[S::MI];
#pragma unroll
      for (int i = 0; i < S::MI; ++i) a[i] = frag_t<K>(dzs, wk * S::KW + i * 16, ps * 32, lane);
#pragma unroll
      for (int j = 0; j < S::NJ; ++j) {
        const bf16x8 b = frag_t<CB>(xs, wc * S::CW + j * 16, ps * 32, lane);
#pragma unroll
        for (int i = 0; i < S::MI; ++i)
          wacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, wacc[i][j], 0, 0, 0);
      }
    }
  }
  // lane (g, il) holds dW[k = .. + 4 g + r][c = .. + il]: 16 consecutive floats per (g, r).  fp32 atomics into dw, or
  // (deterministic mode, dws != null) the block's partial [K][CB] in its own workspace slot, summed in block order by
  // wgrad_slots_reduce: the tiles a block walks are fixed by its id, so every partial is run-to-run identical
  float* part = dws != nullptr ? dws + (long)blockIdx.x * K * CB : nullptr;
#pragma unroll
  for (int i = 0; i < S::MI; ++i)
#pragma unroll
    for (int j = 0; j < S::NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = wk * S::KW + i * 16 + 4 * g + r, c = wc * S::CW + j * 16 + il;
        if (part != nullptr) part[kk * CB + c] = wacc[i][j][r];
        else atomicAdd(dw + (long)kk * C + c, wacc[i][j][r]);
      }
}

// deterministic mode: dw[k][c] += sum over the blocks b holding channel slice c / CB, in increasing b, of their slots
__global__ void __launch_bounds__(256) wgrad_slots_reduce(const float* __restrict__ dws, float* __restrict__ dw, int K,
                                                          int C, int CB, int nblocks, int nsplit) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)K * C) return;
  const int k = (int)(e / C), c = (int)(e % C), cs = c / CB, cl = c % CB;
  float s = 0.f;
  for (int b = 0; b < nblocks; ++b)
    if (((b >> 3) % nsplit) == cs) s += dws[((long)b * K + k) * CB + cl];
  dw[e] += s;
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// the configurations built, (K, C) -> (dx channels per block CB, pixels per tile TP, 16-px tiles per data-grad unit
// PX).  CB = C: one block per tile; CB < C: C / CB blocks per tile (column split).  K = 256 on one block per tile (C =
// 128 / 256: 128-256 weight-grad accumulator registers per lane) was measured at 0.42-0.68x the three launches with
// 49 / 106 spilled VGPRs (profiles/r05/bwd1x1_ab_v1.log).  K = 512 x C = 128 split over 2 blocks (CB 64, TP 32, no
// spills) measured 0.86x (1733 vs 1491 us @192^2 bs32, profiles/r05/bwd1x1_ab_v3.log): its dz transform, ~20 VALU
// issue cycles per element run twice for 512 channels, is worth ~0.6 ms of VALU on its own, so it is not built
// A second register set of prefetched (dy, z, x) chunks (tile t + 2 in flight while t computes; the sets rotated at
// the prefetch point) measured 1-11 % SLOWER on every shape (profiles/r05/bwd1x1_depth2_ab.log): the PMC passes show
// these launches issue-bound (~50 % of wave cycles issuing, 25-39 % waiting, profiles/r05/pmc_bwd1x1.txt), not
// starved for loads in flight
// 64-pixel tiles for the K = 256 column-split shapes (PX 1 or 2) spill 29-32 VGPRs at 256 VGPRs + 256 AGPRs and
// measured slower: C256 -> K256 @96^2 bs32 266 -> 307..326 us, @192^2 911 -> 1071..1147 us (round 6,
// profiles/r06/bwd1x1_tp_ab.log)
// An 8-wave single block per tile for the K = 256 layers (no column split, the transform once; 4 x 2 or 2 x 4 wave grid)
// does not fit: 2 waves per SIMD leave 256 registers per wave, and the kernel's working set besides the weight-grad
// accumulators is ~290 (63-80 VGPRs spilled at 256 x 256 / 256 x 128), so it was not built
struct Plan {
  int cb, tp, px;
};
constexpr Plan plan(int K, int C) {
  return (K == 64 && C == 64) ? Plan{64, 128, 2} : (K == 128 && C == 64) ? Plan{64, 128, 2}
       : (K == 64 && C == 128) ? Plan{128, 64, 2} : (K == 128 && C == 128) ? Plan{128, 64, 2}
       : (K == 128 && C == 256) ? Plan{256, 64, 2} : (K == 128 && C == 512) ? Plan{256, 64, 2}
       : (K == 256 && C == 256) ? Plan{128, 32, 1} : (K == 256 && C == 128) ? Plan{128, 32, 1}
       : (K == 64 && C == 256) ? Plan{256, 64, 2} : Plan{0, 0, 0};
}

// blocks of a launch: whole XCD groups of nsplit blocks (one per CU), no more groups than tiles
inline int grid_blocks(long M, int K, int C) {
  const Plan pl = plan(K, C);
  const int ns = C / pl.cb, ntiles = ceil_div(M, pl.tp);
  int ngrp = num_cus() / ns;
  if (ngrp > ntiles) ngrp = (ntiles + 7) / 8 * 8;
  return ngrp * ns;
}

template <int K, int C>
int launch(const bf16* dy, long dps, const bf16* z, const bf16* x, long xps, const bf16* wt, const float* scale,
           const float* shift, const float* mean, const float* invstd, int act, const float* ca, const float* cb,
           const float* cc, bf16* dx, long bps, int acc, float* dw, float* ws, long M, hipStream_t st) {
  constexpr Plan pl = plan(K, C);
  constexpr int CB = pl.cb, TP = pl.tp, PX = pl.px, NS = C / CB;
  using S = Shape<K, CB, TP, PX>;
  static bool raised = false;
  if (!raised) {
    (void)hipFuncSetAttribute((const void*)conv1x1_bwd_bn<K, CB, TP, PX>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS);
    raised = true;
  }
  const int nb = grid_blocks(M, K, C);
  conv1x1_bwd_bn<K, CB, TP, PX><<<nb, 256, S::LDS, st>>>(
      dy, dps, z, x, xps, wt, scale, shift, mean, invstd, act, ca, cb, cc, dx, bps, acc, dw, ws, M, ceil_div(M, TP), C,
      NS, (unsigned)(2.0 * (double)M * dps), (unsigned)(2.0 * (double)M * K), (unsigned)(2.0 * (double)M * xps));
  if (ws != nullptr)
    wgrad_slots_reduce<<<ceil_div((long)K * C, 256), 256, 0, st>>>(ws, dw, K, C, CB, nb, NS);
  return (int)hipGetLastError();
}
}  // namespace b1
}  // namespace

DMY_API int dmy_conv1x1_bwd_bn_ok(long M, int K, int C, long dps, long xps, long bps, const void* dy, const void* z,
                                  const void* x, const void* dx) {
  if (b1::plan(K, C).cb == 0 || M <= 0) return 0;
  if (dps % 8 || xps % 8 || bps % 8 || dps < K || xps < C || bps < C) return 0;
  for (const void* p : {dy, z, x, dx})
    if (((uintptr_t)p & 15) != 0) return 0;
  // 32-bit buffer offsets (the out-of-range offset kOob must stay past every record)
  const double lim = (double)b1::kOob - 64.0;
  if (2.0 * (double)M * dps >= lim || 2.0 * (double)M * K >= lim || 2.0 * (double)M * xps >= lim) return 0;
  return 1;
}

DMY_API long dmy_conv1x1_bwd_bn_ws_elems(long M, int K, int C) {
  if (b1::plan(K, C).cb == 0 || M <= 0) return 0;
  return (long)b1::grid_blocks(M, K, C) * K * b1::plan(K, C).cb;
}

DMY_API int dmy_conv1x1_bwd_bn(const void* dy, long dps, const void* z, const void* x, long xps, const void* wt,
                               const float* scale, const float* shift, const float* mean, const float* invstd, int act,
                               const float* ca, const float* cb, const float* cc, void* dx, long bps, int accumulate,
                               float* dw, float* ws, long ws_elems, long M, int K, int C, void* stream) {
  if (!dmy_conv1x1_bwd_bn_ok(M, K, C, dps, xps, bps, dy, z, x, dx)) return -1;
  if (ws != nullptr && ws_elems < dmy_conv1x1_bwd_bn_ws_elems(M, K, C)) return -1;
  hipStream_t st = (hipStream_t)stream;
#define B1_GO(K_, C_)                                                                                                 \
  if (K == K_ && C == C_)                                                                                            \
    return b1::launch<K_, C_>((const bf16*)dy, dps, (const bf16*)z, (const bf16*)x, xps, (const bf16*)wt, scale,     \
                              shift, mean, invstd, act, ca, cb, cc, (bf16*)dx, bps, accumulate, dw, ws, M, st);
  B1_GO(64, 64)
  B1_GO(128, 64)
  B1_GO(64, 128)
  B1_GO(128, 128)
  B1_GO(128, 256)
  B1_GO(128, 512)
  B1_GO(256, 128)
  B1_GO(256, 256)
  B1_GO(64, 256)
#undef B1_GO
  return -1;
}
