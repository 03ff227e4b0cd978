// Swin window attention for C3STR (models/common.py:452-654) on gfx950.
//
// The reference layer works on x.permute(0,3,2,1) = [B, W, H, C] (common.py:596-597), i.e. its
// "rows" are the image W axis.  Tokens stay in our NHWC buffers; the kernels map window
// coordinates -> pixels on the fly, folding pad (F.pad after norm1 -> zero tokens), roll(-s,-s),
// window_partition/reverse and the crop into address arithmetic:
//   shifted (rs, cs) -> unshifted padded (r0 = (rs+s) % Rp, c0 = (cs+s) % Cp) -> pixel (h = c0, w = r0)
// The shifted-window mask reproduces the reference's create_mask, including the h_slices[0]
// tuple-indexing bug: labels are computed in shifted window space.
//   label(r, c) = r >= Rp-s ? 6+cg : r >= Rp-ws ? 3+cg : r == 0 ? cg : 0,
//   cg(c)       = c < Cp-ws ? 0 : c < Cp-s ? 1 : 2;   mask = -100 where labels differ.
// One workgroup per (window, head); head_dim 32, window 8 (64 tokens); fp32 math in LDS.
// Backward recomputes P (flash-style: nothing N x N is stored) and accumulates the
// relative-position-bias gradient per workgroup in LDS, then once per workgroup to a slab.
#include "common.h"

namespace {

constexpr int WS = 8, NTOK = 64, HD = 32;

struct SwinGeom {
  int B, H, W, C, nh;     // image H, W (NHWC); C = channels, nh heads (C = nh * 32)
  int Rp, Cp, shift;      // padded Swin-space rows (image W) / cols (image H), shift
  float scale;
};

DEV int win_label(int r, int c, int Rp, int Cp, int s) {
  const int cg = c < Cp - WS ? 0 : (c < Cp - s ? 1 : 2);
  if (r >= Rp - s) return 6 + cg;
  if (r >= Rp - WS) return 3 + cg;
  if (r == 0) return cg;
  return 0;
}

// token t of window (wr, wc) -> pixel index in [B*H*W) or -1 for padding
DEV long tok_pixel(const SwinGeom& g, int b, int wr, int wc, int t) {
  const int rs = wr * WS + (t >> 3), cs = wc * WS + (t & 7);
  const int r0 = (rs + g.shift) % g.Rp, c0 = (cs + g.shift) % g.Cp;
  if (r0 >= g.W || c0 >= g.H) return -1;
  return ((long)b * g.H + c0) * g.W + r0;  // h = c0, w = r0
}

// ---------------------------------------------------------------- LayerNorm over channels (eps from module)
template <typename T>
__global__ void ln_fwd_kernel(const T* __restrict__ x, long xps, const float* __restrict__ w, const float* __restrict__ b,
                              T* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd, long M, int C,
                              float eps) {
  const int lane = threadIdx.x & 63;
  for (long m = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); m < M; m += (long)gridDim.x * (blockDim.x >> 6)) {
    const T* xr = x + m * xps;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += to_f(xr[c]);
    const float mu = wave_sum(s) / C;
    float v = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = to_f(xr[c]) - mu;
      v += d * d;
    }
    const float rs = rsqrtf(wave_sum(v) / C + eps);
    for (int c = lane; c < C; c += 64) y[m * C + c] = from_f<T>((to_f(xr[c]) - mu) * rs * w[c] + b[c]);
    if (lane == 0) {
      mean[m] = mu;
      rstd[m] = rs;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w; per-block partials of dw, db.
// Deterministic: each wave accumulates its rows into its own LDS row pair [wave][2][C], where lane l owns channels
// l, l + 64, ... (no two lanes touch one slot), and the block partial is the sum over waves in wave order.
template <typename T>
__global__ void ln_bwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ dy, long dps,
                              const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
                              T* __restrict__ dx, long dxps, int accumulate, long M, int C, int rows_per_block,
                              float* __restrict__ pdw, float* __restrict__ pdb) {
  extern __shared__ float sh[];  // [waves][2][C]
  const int nwv = blockDim.x >> 6, wv = threadIdx.x >> 6;
  for (int c = threadIdx.x; c < 2 * C * nwv; c += blockDim.x) sh[c] = 0.f;
  __syncthreads();
  float* sdw = sh + (long)wv * 2 * C;
  float* sdb = sdw + C;
  const int lane = threadIdx.x & 63;
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (long m = r0 + wv; m < r1; m += nwv) {
    const float mu = mean[m], rs = rstd[m];
    float a1 = 0.f, a2 = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float xh = (to_f(x[m * xps + c]) - mu) * rs;
      const float gy = to_f(dy[m * dps + c]);
      const float g = gy * w[c];
      a1 += g;
      a2 += g * xh;
      sdw[c] += gy * xh;
      sdb[c] += gy;
    }
    a1 = wave_sum(a1) / C;
    a2 = wave_sum(a2) / C;
    for (int c = lane; c < C; c += 64) {
      const float xh = (to_f(x[m * xps + c]) - mu) * rs;
      const float g = to_f(dy[m * dps + c]) * w[c];
      const float v = rs * (g - a1 - xh * a2);
      dx[m * dxps + c] = from_f<T>(accumulate ? v + to_f(dx[m * dxps + c]) : v);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < nwv; ++k) {
      a += sh[(long)k * 2 * C + c];
      b += sh[(long)k * 2 * C + C + c];
    }
    pdw[(long)blockIdx.x * C + c] = a;
    pdb[(long)blockIdx.x * C + c] = b;
  }
}

// Vectorised LayerNorm: a row of C channels is held by L lanes (16-B vectors, L = pow2 >= C/VW),
// 64/L rows per wave, one global read per element; backward keeps the per-channel dw/db partials
// in registers (a thread's channels are fixed) and reduces them once per workgroup.
template <typename T, int L>
__global__ void __launch_bounds__(256) ln_fwd_vec(const T* __restrict__ x, long xps, const float* __restrict__ w,
                                                  const float* __restrict__ b, T* __restrict__ y,
                                                  float* __restrict__ mean, float* __restrict__ rstd, long M, int C,
                                                  float eps) {
  constexpr int VW = Traits<T>::VW, RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane % L, rw = lane / L;
  const int c0 = sub * VW;
  const bool on = c0 < C;
  // gamma / beta of this lane's VW channels: 16-B loads (the scalar form was 2 x VW loads per wave, a wave's whole
  // VMEM stream at batch-1 sizes where it handles one row: 19.4 us for 18.9 MB, 3.5 us for a copy of it)
  float wv[VW], bv[VW];
  if (((((uintptr_t)w) | ((uintptr_t)b)) & 15) == 0) {
#pragma unroll
    for (int j = 0; j < VW; j += 4) {
      const float4 a = on ? *reinterpret_cast<const float4*>(w + c0 + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 e = on ? *reinterpret_cast<const float4*>(b + c0 + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      wv[j] = a.x; wv[j + 1] = a.y; wv[j + 2] = a.z; wv[j + 3] = a.w;
      bv[j] = e.x; bv[j + 1] = e.y; bv[j + 2] = e.z; bv[j + 3] = e.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      wv[j] = on ? w[c0 + j] : 0.f;
      bv[j] = on ? b[c0 + j] : 0.f;
    }
  }
  const long rpb = (long)(blockDim.x >> 6) * RPW;
  for (long mb = (long)blockIdx.x * rpb; mb < M; mb += (long)gridDim.x * rpb) {
    const long m = mb + (threadIdx.x >> 6) * RPW + rw;
    const bool ok = on && m < M;
    float v[VW];
    if (ok) unpack<T>(*reinterpret_cast<const uint4*>(x + m * xps + c0), v);
    else
#pragma unroll
      for (int j = 0; j < VW; ++j) v[j] = 0.f;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VW; ++j) s += v[j];
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mu = s / C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      v[j] -= mu;
      q += ok ? v[j] * v[j] : 0.f;
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rs = rsqrtf(q / C + eps);
    if (ok) {
      float o_[VW];
#pragma unroll
      for (int j = 0; j < VW; ++j) o_[j] = v[j] * rs * wv[j] + bv[j];
      *reinterpret_cast<uint4*>(y + m * C + c0) = pack<T>(o_);
    }
    if (sub == 0 && m < M) {
      mean[m] = mu;
      rstd[m] = rs;
    }
  }
}

template <typename T, int L>
__global__ void __launch_bounds__(256) ln_bwd_vec(const T* __restrict__ x, long xps, const T* __restrict__ dy, long dps,
                                                  const float* __restrict__ w, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, T* __restrict__ dx, long dxps,
                                                  int accumulate, long M, int C, float* __restrict__ pdw,
                                                  float* __restrict__ pdb) {
  constexpr int VW = Traits<T>::VW, RPW = 64 / L;
  extern __shared__ float sh[];  // [waves][2][C]
  const int lane = threadIdx.x & 63, sub = lane % L, rw = lane / L;
  const int c0 = sub * VW;
  const bool on = c0 < C;
  float wv[VW], aw[VW], ab[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) {
    wv[j] = 0.f;
    aw[j] = 0.f;
    ab[j] = 0.f;
  }
  if (on) ldf<VW>(w + c0, wv);
  const long rpb = (long)(blockDim.x >> 6) * RPW;
  for (long mb = (long)blockIdx.x * rpb; mb < M; mb += (long)gridDim.x * rpb) {
    const long m = mb + (threadIdx.x >> 6) * RPW + rw;
    const bool ok = on && m < M;
    float xv[VW], gv[VW];
    float mu = 0.f, rs = 0.f;
    if (ok) {
      unpack<T>(*reinterpret_cast<const uint4*>(x + m * xps + c0), xv);
      unpack<T>(*reinterpret_cast<const uint4*>(dy + m * dps + c0), gv);
      mu = mean[m];
      rs = rstd[m];
    } else {
#pragma unroll
      for (int j = 0; j < VW; ++j) xv[j] = gv[j] = 0.f;
    }
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      xv[j] = (xv[j] - mu) * rs;  // xhat
      aw[j] += gv[j] * xv[j];
      ab[j] += gv[j];
      gv[j] *= wv[j];
      a1 += gv[j];
      a2 += gv[j] * xv[j];
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) {
      a1 += __shfl_xor(a1, o, 64);
      a2 += __shfl_xor(a2, o, 64);
    }
    a1 /= C;
    a2 /= C;
    if (ok) {
      float o_[VW], p_[VW];
      if (accumulate) unpack<T>(*reinterpret_cast<const uint4*>(dx + m * dxps + c0), p_);
#pragma unroll
      for (int j = 0; j < VW; ++j) o_[j] = rs * (gv[j] - a1 - xv[j] * a2) + (accumulate ? p_[j] : 0.f);
      *reinterpret_cast<uint4*>(dx + m * dxps + c0) = pack<T>(o_);
    }
  }
  // deterministic block partial: the RPW row slots of a wave that share channels are folded by a fixed xor tree, the
  // wave's row goes to LDS [wave][2][C], and the waves are summed in order (no LDS atomics)
#pragma unroll
  for (int o = L; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      aw[j] += __shfl_xor(aw[j], o, 64);
      ab[j] += __shfl_xor(ab[j], o, 64);
    }
  const int wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  if (on && rw == 0) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      sh[(long)wid * 2 * C + c0 + j] = aw[j];
      sh[(long)wid * 2 * C + C + c0 + j] = ab[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < nwv; ++k) {
      a += sh[(long)k * 2 * C + c];
      b += sh[(long)k * 2 * C + C + c];
    }
    pdw[(long)blockIdx.x * C + c] = a;
    pdb[(long)blockIdx.x * C + c] = b;
  }
}

// L = lanes per row (pow2 >= C / VW); 0 if the vector kernels do not apply
template <typename T> int ln_lanes(int C, long xps, long yps, const void* x, const void* y) {
  constexpr int VW = Traits<T>::VW;
  if (C % VW || xps % VW || yps % VW || (((uintptr_t)x | (uintptr_t)y) & 15)) return 0;
  const int n = C / VW;
  int L = 4;
  while (L < n) L <<= 1;
  return L <= 64 ? L : 0;
}

// ---------------------------------------------------------------- window attention
// LDS layout (floats): Q[64][33] K[64][33] V[64][33] P[64][65]
constexpr int QS = HD + 1, PS = NTOK + 1;

template <typename T>
DEV void load_qkv(const T* qkv, const SwinGeom& g, int b, int wr, int wc, int head, float* Q, float* K, float* V,
                  long* pix) {
  const int C3 = 3 * g.C;
  for (int e = threadIdx.x; e < NTOK * HD; e += blockDim.x) {
    const int t = e / HD, d = e % HD;
    const long p = tok_pixel(g, b, wr, wc, t);
    if (d == 0) pix[t] = p;
    float q = 0.f, k = 0.f, v = 0.f;
    if (p >= 0) {
      const T* row = qkv + p * C3 + head * HD + d;
      q = to_f(row[0]);
      k = to_f(row[g.C]);
      v = to_f(row[2 * g.C]);
    }
    Q[t * QS + d] = q * g.scale;  // q = q * self.scale (common.py:520)
    K[t * QS + d] = k;
    V[t * QS + d] = v;
  }
}

// P = softmax(Q K^T + bias + mask): thread (row = tid/4, 16 cols)
DEV void scores_softmax(const SwinGeom& g, int wr, int wc, int head, const float* __restrict__ table, const float* Q,
                        const float* K, float* P) {
  const int i = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;
  float s[16];
  const int ri = i >> 3, ci = i & 7;
  const int lab_i = g.shift > 0 ? win_label(wr * WS + ri, wc * WS + ci, g.Rp, g.Cp, g.shift) : 0;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    const int j = j0 + jj;
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) a += Q[i * QS + d] * K[j * QS + d];
    const int rj = j >> 3, cj = j & 7;
    const int idx = (ri - rj + WS - 1) * (2 * WS - 1) + (ci - cj + WS - 1);
    a += table[idx * g.nh + head];
    if (g.shift > 0 && win_label(wr * WS + rj, wc * WS + cj, g.Rp, g.Cp, g.shift) != lab_i) a += -100.0f;
    s[jj] = a;
  }
  float mx = s[0];
#pragma unroll
  for (int jj = 1; jj < 16; ++jj) mx = fmaxf(mx, s[jj]);
  mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
  float sum = 0.f;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    s[jj] = expf(s[jj] - mx);
    sum += s[jj];
  }
  sum += __shfl_xor(sum, 1, 64);
  sum += __shfl_xor(sum, 2, 64);
  const float inv = 1.f / sum;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) P[i * PS + j0 + jj] = s[jj] * inv;
}

// bias-table bin e = (dr + 7) * 15 + (dc + 7) of a [64][ld] dS matrix (row = query, col = key): the sum over every
// (q, k) with ri - rj = dr, ci - cj = dc, in ascending q (fixed order: deterministic)
DEV float bin_dtab(const float* S, int ld, int e) {
  const int dr = e / (2 * WS - 1) - (WS - 1), dc = e % (2 * WS - 1) - (WS - 1);
  float a = 0.f;
  for (int ri = max(0, dr); ri < min(WS, WS + dr); ++ri)
    for (int ci = max(0, dc); ci < min(WS, WS + dc); ++ci) a += S[(ri * WS + ci) * ld + (ri - dr) * WS + (ci - dc)];
  return a;
}

template <typename T>
__global__ void __launch_bounds__(256) winattn_fwd_kernel(const T* __restrict__ qkv, const float* __restrict__ table,
                                                          T* __restrict__ out, SwinGeom g) {
  __shared__ float Q[NTOK * QS], K[NTOK * QS], V[NTOK * QS], P[NTOK * PS];
  __shared__ long pix[NTOK];
  const int nwr = g.Rp / WS, nwc = g.Cp / WS;
  const int head = blockIdx.y;
  const int wid = blockIdx.x;
  const int b = wid / (nwr * nwc), wr = (wid / nwc) % nwr, wc = wid % nwc;
  load_qkv(qkv, g, b, wr, wc, head, Q, K, V, pix);
  __syncthreads();
  scores_softmax(g, wr, wc, head, table, Q, K, P);
  __syncthreads();
  // O[i][d0..d0+8) = sum_j P[i][j] V[j][d]
  const int i = threadIdx.x >> 2, d0 = (threadIdx.x & 3) * 8;
  float o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < NTOK; ++j) {
    const float p = P[i * PS + j];
#pragma unroll
    for (int d = 0; d < 8; ++d) o[d] += p * V[j * QS + d0 + d];
  }
  const long px = pix[i];
  if (px >= 0) {
#pragma unroll
    for (int d = 0; d < 8; ++d) out[px * g.C + head * HD + d0 + d] = from_f<T>(o[d]);
  }
}

// grid: (window groups, heads); each block walks `wpb` windows of one head
template <typename T>
__global__ void __launch_bounds__(256) winattn_bwd_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                          const float* __restrict__ table, T* __restrict__ dqkv,
                                                          float* __restrict__ dtab_part, int nwin_total, int wpb,
                                                          SwinGeom g) {
  __shared__ float Q[NTOK * QS], K[NTOK * QS], V[NTOK * QS], P[NTOK * PS], D[NTOK * QS];
  __shared__ long pix[NTOK];
  const int ntab = (2 * WS - 1) * (2 * WS - 1);
  float dsacc[16];
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) dsacc[jj] = 0.f;
  const int nwr = g.Rp / WS, nwc = g.Cp / WS;
  const int head = blockIdx.y;
  for (int wid = blockIdx.x * wpb; wid < min(nwin_total, (blockIdx.x + 1) * wpb); ++wid) {
    const int b = wid / (nwr * nwc), wr = (wid / nwc) % nwr, wc = wid % nwc;
    __syncthreads();
    load_qkv(qkv, g, b, wr, wc, head, Q, K, V, pix);
    __syncthreads();
    for (int e = threadIdx.x; e < NTOK * HD; e += blockDim.x) {
      const int t = e / HD, d = e % HD;
      const long p = pix[t];
      D[t * QS + d] = p >= 0 ? to_f(dout[p * g.C + head * HD + d]) : 0.f;  // dO
    }
    scores_softmax(g, wr, wc, head, table, Q, K, P);
    __syncthreads();
    // dV[j][d] = sum_i P[i][j] dO[i][d]    thread: j = tid/4, 8 dims
    {
      const int j = threadIdx.x >> 2, d0 = (threadIdx.x & 3) * 8;
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int i = 0; i < NTOK; ++i) {
        const float p = P[i * PS + j];
#pragma unroll
        for (int d = 0; d < 8; ++d) a[d] += p * D[i * QS + d0 + d];
      }
      const long px = pix[j];
      if (px >= 0) {
#pragma unroll
        for (int d = 0; d < 8; ++d) dqkv[px * 3 * g.C + 2 * g.C + head * HD + d0 + d] = from_f<T>(a[d]);
      }
    }
    // dP[i][j] = dO[i] . V[j];  dS = P * (dP - sum_j P dP)   (row i = tid/4, 16 cols)
    {
      const int i = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;
      float dp[16];
      float rs = 0.f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        float a = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) a += D[i * QS + d] * V[(j0 + jj) * QS + d];
        dp[jj] = a;
        rs += a * P[i * PS + j0 + jj];
      }
      rs += __shfl_xor(rs, 1, 64);
      rs += __shfl_xor(rs, 2, 64);
      __syncthreads();  // everyone done reading P for dV / dP
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = j0 + jj;
        const float ds = P[i * PS + j] * (dp[jj] - rs);
        P[i * PS + j] = ds;  // P now holds dS
        dsacc[jj] += ds;     // this thread's (i, j) positions, summed over the block's windows in window order
      }
    }
    __syncthreads();
    // dQ[i][d] = scale * sum_j dS[i][j] K[j][d];  dK[j][d] = sum_i dS[i][j] Qs[i][d]
    {
      const int r = threadIdx.x >> 2, d0 = (threadIdx.x & 3) * 8;
      float aq[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ak[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int j = 0; j < NTOK; ++j) {
        const float s1 = P[r * PS + j], s2 = P[j * PS + r];
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          aq[d] += s1 * K[j * QS + d0 + d];
          ak[d] += s2 * Q[j * QS + d0 + d];
        }
      }
      const long px = pix[r];
      if (px >= 0) {
        T* row = dqkv + px * 3 * g.C + head * HD + d0;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          row[d] = from_f<T>(aq[d] * g.scale);
          row[g.C + d] = from_f<T>(ak[d]);
        }
      }
    }
  }
  // bias-table bins, deterministic: the summed dS matrix goes to LDS (P), then bin (dr, dc) adds its (q, k) positions
  // in ascending q order
  __syncthreads();
  {
    const int i = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) P[i * PS + j0 + jj] = dsacc[jj];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < ntab; e += blockDim.x)
    dtab_part[((long)blockIdx.x * g.nh + head) * ntab + e] = bin_dtab(P, PS, e);
}

// table grad [225][nh] = sum over window groups
// one workgroup per table entry: 256 lanes stride over the groups, fixed-order fp64 tree in LDS
__global__ void __launch_bounds__(256) dtab_reduce_kernel(const float* __restrict__ part, int ngroups, int nh,
                                                          float* __restrict__ dtab) {
  const int ntab = (2 * WS - 1) * (2 * WS - 1);
  const int e = blockIdx.x;
  const int idx = e / nh, h = e % nh;
  __shared__ double red[256];
  double s = 0.0;
  for (int gi = threadIdx.x; gi < ngroups; gi += 256) s += part[((long)gi * nh + h) * ntab + idx];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) dtab[e] = (float)red[0];
}

// per-sample scale (DropPath, common.py:386-403): y = x * sc[b]  (sc = floor(keep + u) / keep)
template <typename T>
__global__ void sample_scale_kernel(const T* __restrict__ x, const float* __restrict__ sc, T* __restrict__ y, long per,
                                    long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = from_f<T>(to_f(x[i]) * sc[i / per]);
}

// DropPath fused with the residual add it feeds (an active SwinTransformerLayer drop_path, common.py:621-627):
// y = x + f * s[b], s[b] = floor(keep + u[b]) / keep -- torch's (keep + rand).floor_().div_(keep) on the drawn u, in
// fp32, one rounding of the sum (the unfused pair rounded f * s first).  grad: df = dy * s[b] (dx = dy needs no pass).
// Samples are contiguous blocks of `per` elements (NHWC); 8-element vectors when per % 8 == 0 and 16-B aligned.
DEV float dp_scale(const float* u, long b, float keep) { return floorf(keep + u[b]) / keep; }
template <typename T>
__global__ void droppath_add_kernel(const T* __restrict__ x, const T* __restrict__ f, const float* __restrict__ u,
                                    float keep, T* __restrict__ y, long per, long n, int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  if (vec) {
    for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n / 8; v += stride) {
      const long i = v * 8;
      const float sc = dp_scale(u, i / per, keep);
      float a[8], b[8];
      unpack<T>(*reinterpret_cast<const uint4*>(x + i), a);
      unpack<T>(*reinterpret_cast<const uint4*>(f + i), b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j] * sc;
      *reinterpret_cast<uint4*>(y + i) = pack<T>(a);
    }
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = from_f<T>(to_f(x[i]) + to_f(f[i]) * dp_scale(u, i / per, keep));
}
template <typename T>
__global__ void droppath_grad_kernel(const T* __restrict__ dy, const float* __restrict__ u, float keep,
                                     T* __restrict__ df, long per, long n, int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  if (vec) {
    for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n / 8; v += stride) {
      const long i = v * 8;
      const float sc = dp_scale(u, i / per, keep);
      float a[8];
      unpack<T>(*reinterpret_cast<const uint4*>(dy + i), a);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] *= sc;
      *reinterpret_cast<uint4*>(df + i) = pack<T>(a);
    }
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
    df[i] = from_f<T>(to_f(dy[i]) * dp_scale(u, i / per, keep));
}

// ---------------------------------------------------------------- bf16 window attention on MFMA
// Throughput mode: one wave per (window, head), NW waves per workgroup sharing one head (the
// bias-table column is staged once per workgroup).  All six products are 16x16x32 bf16 MFMAs
// over LDS-staged [64][32] / [64][64] bf16 tiles:
//   fwd: S^T = K Q^T (lane holds 4 consecutive keys of one query row), softmax in registers,
//        P -> LDS, O^T = V^T P^T;
//   bwd: recompute P; dP^T = V dO^T; dS = P (dP - rowsum(P dP)); dV^T = dO^T P; dQ^T = K^T dS^T;
//        dK^T = Q^T dS (scale folded into the fp32 epilogue); dS also feeds the bias-table grad.
// Operand fragments: fr_row = 16-B row read, fr_col = transposed read (ds_read_b64_tr_b16).
constexpr int LQ = HD + 8;      // [64][32] bf16 row stride (80 B)
constexpr int LP = NTOK + 8;    // [64][64] bf16 row stride (144 B)
constexpr int MATQ = NTOK * LQ;
constexpr int MATP = NTOK * LP;
constexpr int NTAB = (2 * WS - 1) * (2 * WS - 1);

typedef short s4v __attribute__((ext_vector_type(4)));

// lane gets X[r0 + (lane&15)][k0 + 8g .. +8)   (g = lane >> 4)
DEV bf16x8 fr_row(const bf16* X, int ld, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(X + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4));
}
// lane gets X[k0 + 8g + e][r0 + (lane&15)], e = 0..7
DEV bf16x8 fr_col(const bf16* X, int ld, int r0, int k0, int lane) {
  const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3;
  const bf16* a0 = X + (k0 + 8 * g + q) * ld + r0 + 4 * p;
  const bf16* a1 = X + (k0 + 8 * g + 4 + q) * ld + r0 + 4 * p;
  s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a0));
  s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
DEV f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// 4 fp32 -> 4 bf16 as one 8-byte LDS store
DEV void st4(bf16* dst, float a, float b, float c, float d) {
  union { bf16 h[4]; uint2 u; } v;
  v.h[0] = __float2bfloat16(a); v.h[1] = __float2bfloat16(b);
  v.h[2] = __float2bfloat16(c); v.h[3] = __float2bfloat16(d);
  *reinterpret_cast<uint2*>(dst) = v.u;
}

// S^T tiles (lane: query q = 16bq + il, keys 16bk + 4g + r) -> scaled, biased, masked -> softmax.
// P[bq][bk][r] in fp32 on return.
// qf[bq] / kf[bk]: the row fragments of queries / keys 16 b + (lane & 15), dims 8 (lane >> 4) .. + 8
DEV void softmax_f(const bf16x8 (&qf)[4], const bf16x8 (&kf)[4], const float* tab, const SwinGeom& g, int wr, int wc,
                   int lane, float (&P)[4][4][4]) {
  const int il = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int bq = 0; bq < 4; ++bq) {
    const int q = 16 * bq + il, ri = q >> 3, ci = q & 7;
    const int lq = g.shift > 0 ? win_label(wr * WS + ri, wc * WS + ci, g.Rp, g.Cp, g.shift) : 0;
    float mx = -3.0e38f;
#pragma unroll
    for (int bk = 0; bk < 4; ++bk) {
      f32x4 acc = mma(kf[bk], qf[bq], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * bk + 4 * gq + r, rj = k >> 3, cj = k & 7;
        float v = acc[r] * g.scale + tab[(ri - rj + WS - 1) * (2 * WS - 1) + (ci - cj + WS - 1)];
        if (g.shift > 0 && win_label(wr * WS + rj, wc * WS + cj, g.Rp, g.Cp, g.shift) != lq) v += -100.0f;
        P[bq][bk][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int bk = 0; bk < 4; ++bk)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        P[bq][bk][r] = __expf(P[bq][bk][r] - mx);
        sum += P[bq][bk][r];
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
#pragma unroll
    for (int bk = 0; bk < 4; ++bk)
#pragma unroll
      for (int r = 0; r < 4; ++r) P[bq][bk][r] *= inv;
  }
}

DEV void softmax_t(const bf16* Qs, const bf16* Ks, const float* tab, const SwinGeom& g, int wr, int wc, int lane,
                   float (&P)[4][4][4]) {
  bf16x8 qf[4], kf[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    qf[b] = fr_row(Qs, LQ, 16 * b, 0, lane);
    kf[b] = fr_row(Ks, LQ, 16 * b, 0, lane);
  }
  softmax_f(qf, kf, tab, g, wr, wc, lane, P);
}

// P (registers, S^T layout) -> Ps[q][k] bf16
DEV void store_p(bf16* Ps, const float (&P)[4][4][4], int lane) {
  const int il = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int bq = 0; bq < 4; ++bq)
#pragma unroll
    for (int bk = 0; bk < 4; ++bk)
      st4(Ps + (16 * bq + il) * LP + 16 * bk + 4 * gq, P[bq][bk][0], P[bq][bk][1], P[bq][bk][2], P[bq][bk][3]);
}

// 1-D grid of (window group, head) blocks in XCD-aware order: block id i runs on XCD i % 8 (round-robin dispatch), and
// the nh heads of one window group are ids 8 h + (group % 8) (+ 8 nh per 8 groups), so they share an XCD and arrive
// together: each head reads 64 B of every token's 128-B qkv lines, the other heads the rest of those lines, from L2
// instead of HBM. Group counts are padded to a multiple of 8 (empty groups do nothing). Speed only: any order is correct.
DEV int xhead(int nh) { return (int)(blockIdx.x >> 3) % nh; }
DEV int xgroup(int nh) { return (int)(blockIdx.x & 7) + 8 * (int)(blockIdx.x / (8u * nh)); }

// X^T accumulator tiles (lane: d = 16 dt + 4 (lane >> 4) + r, token 16 bt + (lane & 15)) -> 16-B stores straight from
// registers: a permlane16 swap pairs the two 16-dim tiles so each lane holds 8 consecutive dims of one token
DEV unsigned pk2(float a, float b) {
  const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (unsigned)*reinterpret_cast<const unsigned short*>(&x) | ((unsigned)*reinterpret_cast<const unsigned short*>(&y) << 16);
}
DEV void store_direct(bf16* dst, long dps, const f32x4 (&A)[2][4], float scale, const long (&px)[4], int lane) {
  const int gq = lane >> 4, chq = (gq & 1) * 16 + (gq >> 1) * 8;
#pragma unroll
  for (int bt = 0; bt < 4; ++bt) {
    const f32x4 &a = A[0][bt], &b = A[1][bt];
    const auto s0 = __builtin_amdgcn_permlane16_swap(pk2(a[0] * scale, a[1] * scale), pk2(b[0] * scale, b[1] * scale),
                                                     false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(pk2(a[2] * scale, a[3] * scale), pk2(b[2] * scale, b[3] * scale),
                                                     false, false);
    uint4 v;
    v.x = s0[0];
    v.y = s1[0];
    v.z = s0[1];
    v.w = s1[1];
    if (px[bt] >= 0) *reinterpret_cast<uint4*>(dst + px[bt] * dps + chq) = v;
  }
}

template <int NW>
__global__ void __launch_bounds__(64 * NW, 2) winattn_fwd_mfma(const bf16* __restrict__ qkv,
                                                            const float* __restrict__ table, bf16* __restrict__ out,
                                                            SwinGeom g, int nwin, int wpb) {
  __shared__ __attribute__((aligned(16))) bf16 sm[NW * (MATQ + MATP)];
  __shared__ float tab[NTAB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int head = xhead(g.nh), grp = xgroup(g.nh);
  const int il = lane & 15, gq = lane >> 4;
  const int nwr = g.Rp / WS, nwc = g.Cp / WS;
  bf16* Vs = sm + w * (MATQ + MATP);
  bf16* Ps = Vs + MATQ;
  const int w0 = grp * wpb, w1 = min(nwin, w0 + wpb);
  const long offq = (long)head * HD;
  uint4 pre[3][4];  // [Q, K, V][token block i]: 16 B of token 16 i + il at dims 8 gq
  long ppre[4], px[4];
  auto fetch = [&](int wn) {
    const int bn = wn / (nwr * nwc), wrn = (wn / nwc) % nwr, wcn = wn % nwc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ppre[i] = tok_pixel(g, bn, wrn, wcn, 16 * i + il);
      const uint4* src = reinterpret_cast<const uint4*>(qkv + (ppre[i] >= 0 ? ppre[i] : 0) * 3L * g.C + offq + gq * 8);
#pragma unroll
      for (int m = 0; m < 3; ++m) pre[m][i] = ppre[i] >= 0 ? src[m * (g.C / 8)] : make_uint4(0, 0, 0, 0);
    }
  };
  // the first window's Q / K / V loads go out before the bias-table gather, so the two share one memory round trip
  // (at batch 1 a block runs one or two windows and this prologue is most of its time)
  if (w0 + w < w1) fetch(w0 + w);
  for (int e = threadIdx.x; e < NTAB; e += blockDim.x) tab[e] = table[e * g.nh + head];
  __syncthreads();  // tab staged; the per-wave buffers below need no block barrier
  for (int wid = w0 + w; wid < w1; wid += NW) {
    const int wr = (wid / nwc) % nwr, wc = wid % nwc;
    bf16x8 qf[4], kf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      px[i] = ppre[i];
      qf[i] = *reinterpret_cast<const bf16x8*>(&pre[0][i]);
      kf[i] = *reinterpret_cast<const bf16x8*>(&pre[1][i]);
      *reinterpret_cast<uint4*>(Vs + (16 * i + il) * LQ + gq * 8) = pre[2][i];
    }
    if (wid + NW < w1) fetch(wid + NW);
    float P[4][4][4];
    softmax_f(qf, kf, tab, g, wr, wc, lane, P);
    store_p(Ps, P, lane);
    // O^T[d][q] = sum_k V[k][d] P[q][k]
    f32x4 O[2][4];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int bq = 0; bq < 4; ++bq) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c) acc = mma(fr_col(Vs, LQ, 16 * dt, 32 * c, lane), fr_row(Ps, LP, 16 * bq, 32 * c, lane), acc);
        O[dt][bq] = acc;
      }
    store_direct(out + offq, g.C, O, 1.f, px, lane);
  }
}

// Backward, one wave per (window, head), walking every NW-th window of its group. Q, K, V, dO row fragments come straight
// from the token rows (fragment pattern, fetched behind the current window's dV / dK / dQ); Q, K and dO are also written to LDS for the transposed
// reads, V never is (it is only read by rows). dQ, dK, dV leave through store_direct, so LDS holds Q / K / dO / P-dS
// (24 KiB per wave, was 29.7 with V and the output staging) and no block barrier is needed inside the loop.
template <int NW>
__global__ void __launch_bounds__(64 * NW) winattn_bwd_mfma(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                               const float* __restrict__ table, bf16* __restrict__ dqkv,
                                                               float* __restrict__ dtab_part, int nwin, int wpb,
                                                               SwinGeom g) {
  __shared__ __attribute__((aligned(16))) bf16 sm[NW * (3 * MATQ + MATP)];
  __shared__ float tab[NTAB];
  static_assert((3 * MATQ + MATP) * 2 >= NTOK * NTOK * 4, "a wave's buffers hold its fp32 [64][64] dS sum");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int head = xhead(g.nh), grp = xgroup(g.nh);
  const int il = lane & 15, gq = lane >> 4;
  for (int e = threadIdx.x; e < NTAB; e += blockDim.x) tab[e] = table[e * g.nh + head];
  const int nwr = g.Rp / WS, nwc = g.Cp / WS;
  bf16* Qs = sm + w * (3 * MATQ + MATP);
  bf16* Ks = Qs + MATQ;
  bf16* Ds = Ks + MATQ;  // dO
  bf16* Ps = Ds + MATQ;  // P, then dS
  const int w0 = grp * wpb, w1 = min(nwin, w0 + wpb);
  const long offq = (long)head * HD;
  // dS summed per (q, k) position over this wave's windows in registers; binned into the bias-table
  // gradient once per workgroup (the bin depends on (q, k) only, not on the window)
  float dsacc[4][4][4];
#pragma unroll
  for (int bq = 0; bq < 4; ++bq)
#pragma unroll
    for (int bk = 0; bk < 4; ++bk)
#pragma unroll
      for (int r = 0; r < 4; ++r) dsacc[bq][bk][r] = 0.f;
  uint4 pre[4][4];  // [Q, K, V, dO][token block i]: 16 B of token 16 i + il at dims 8 gq
  long ppre[4], px[4];
  auto fetch = [&](int wn) {
    const int bn = wn / (nwr * nwc), wrn = (wn / nwc) % nwr, wcn = wn % nwc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ppre[i] = tok_pixel(g, bn, wrn, wcn, 16 * i + il);
      const long pp = ppre[i] >= 0 ? ppre[i] : 0;
      const uint4* src = reinterpret_cast<const uint4*>(qkv + pp * 3L * g.C + offq + gq * 8);
#pragma unroll
      for (int m = 0; m < 3; ++m) pre[m][i] = ppre[i] >= 0 ? src[m * (g.C / 8)] : make_uint4(0, 0, 0, 0);
      pre[3][i] = ppre[i] >= 0 ? *reinterpret_cast<const uint4*>(dout + pp * g.C + offq + gq * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  __syncthreads();  // tab / dtab staged; the per-wave buffers below need no block barrier
  if (w0 + w < w1) fetch(w0 + w);
  for (int wid = w0 + w; wid < w1; wid += NW) {
    const int wr = (wid / nwc) % nwr, wc = wid % nwc;
    bf16x8 qf[4], kf[4], vf[4], df[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      px[i] = ppre[i];
      qf[i] = *reinterpret_cast<const bf16x8*>(&pre[0][i]);
      kf[i] = *reinterpret_cast<const bf16x8*>(&pre[1][i]);
      vf[i] = *reinterpret_cast<const bf16x8*>(&pre[2][i]);
      df[i] = *reinterpret_cast<const bf16x8*>(&pre[3][i]);
      *reinterpret_cast<uint4*>(Qs + (16 * i + il) * LQ + gq * 8) = pre[0][i];
      *reinterpret_cast<uint4*>(Ks + (16 * i + il) * LQ + gq * 8) = pre[1][i];
      *reinterpret_cast<uint4*>(Ds + (16 * i + il) * LQ + gq * 8) = pre[3][i];
    }
    float P[4][4][4];
    softmax_f(qf, kf, tab, g, wr, wc, lane, P);
    store_p(Ps, P, lane);
    // dP^T[k][q] = V[k] . dO[q]  (same layout as P);  dS = P (dP - sum_k P dP), P -> dS in registers
#pragma unroll
    for (int bq = 0; bq < 4; ++bq) {
      float dp[4][4];
      float rs = 0.f;
#pragma unroll
      for (int bk = 0; bk < 4; ++bk) {
        f32x4 acc = mma(vf[bk], df[bq], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dp[bk][r] = acc[r];
          rs += acc[r] * P[bq][bk][r];
        }
      }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
#pragma unroll
      for (int bk = 0; bk < 4; ++bk)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ds = P[bq][bk][r] * (dp[bk][r] - rs);
          P[bq][bk][r] = ds;
          dsacc[bq][bk][r] += ds;
        }
    }
    // the row fragments are dead from here on: prefetch the next window behind dV / dK / dQ
    if (wid + NW < w1) fetch(wid + NW);
    {
      // dV^T[d][k] = sum_q dO[q][d] P[q][k]  (Ps still holds P)
      f32x4 A[2][4];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int bk = 0; bk < 4; ++bk) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 2; ++c) acc = mma(fr_col(Ds, LQ, 16 * dt, 32 * c, lane), fr_col(Ps, LP, 16 * bk, 32 * c, lane), acc);
          A[dt][bk] = acc;
        }
      store_direct(dqkv + 2L * g.C + offq, 3L * g.C, A, 1.f, px, lane);
    }
    store_p(Ps, P, lane);  // dS (after every read of P above: one wave's LDS accesses complete in order)
    {
      // dK^T[d][k] = sum_q Q[q][d] dS[q][k]
      f32x4 A[2][4];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 2; ++c) acc = mma(fr_col(Qs, LQ, 16 * dt, 32 * c, lane), fr_col(Ps, LP, 16 * bt, 32 * c, lane), acc);
          A[dt][bt] = acc;
        }
      store_direct(dqkv + g.C + offq, 3L * g.C, A, g.scale, px, lane);
    }
    {
      // dQ^T[d][q] = sum_k K[k][d] dS[q][k]
      f32x4 A[2][4];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 2; ++c) acc = mma(fr_col(Ks, LQ, 16 * dt, 32 * c, lane), fr_row(Ps, LP, 16 * bt, 32 * c, lane), acc);
          A[dt][bt] = acc;
        }
      store_direct(dqkv + offq, 3L * g.C, A, g.scale, px, lane);
    }
  }
  // bias-table gradient, deterministic: each wave stores its dS sums as fp32 [q][k] over its own (now dead) buffers,
  // then bin e sums its (q, k) positions per wave and the waves in order
  __syncthreads();
  float* S = reinterpret_cast<float*>(Qs);
#pragma unroll
  for (int bq = 0; bq < 4; ++bq)
#pragma unroll
    for (int bk = 0; bk < 4; ++bk)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(16 * bq + il) * NTOK + 16 * bk + 4 * gq + r] = dsacc[bq][bk][r];
  __syncthreads();
  for (int e = threadIdx.x; e < NTAB; e += blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < NW; ++k) a += bin_dtab(reinterpret_cast<const float*>(sm + k * (3 * MATQ + MATP)), NTOK, e);
    dtab_part[((long)grp * g.nh + head) * NTAB + e] = a;
  }
}

SwinGeom make(int B, int H, int W, int C, int nh, int shift, float scale) {
  SwinGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C; g.nh = nh; g.shift = shift; g.scale = scale;
  g.Rp = (W + WS - 1) / WS * WS;  // Swin rows = image W axis
  g.Cp = (H + WS - 1) / WS * WS;
  return g;
}

}  // namespace

template <typename T>
int ln_fwd_t(const T* x, long xps, const float* w, const float* b, T* y, float* mean, float* rstd, long M, int C,
             float eps, hipStream_t st) {
  const int L = ln_lanes<T>(C, xps, C, x, y);
  if (L) {
    const int g = grid_cap(ceil_div(M, 4L * (64 / L)), 8192);
    switch (L) {
      case 4: ln_fwd_vec<T, 4><<<g, 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps); break;
      case 8: ln_fwd_vec<T, 8><<<g, 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps); break;
      case 16: ln_fwd_vec<T, 16><<<g, 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps); break;
      case 32: ln_fwd_vec<T, 32><<<g, 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps); break;
      default: ln_fwd_vec<T, 64><<<g, 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps); break;
    }
  } else {
    ln_fwd_kernel<T><<<grid_cap(ceil_div(M, 4), 4096), 256, 0, st>>>(x, xps, w, b, y, mean, rstd, M, C, eps);
  }
  return (int)hipGetLastError();
}

DMY_API int dmy_layernorm_fwd(int dtype, const void* x, long xps, const float* w, const float* b, void* y, float* mean,
                              float* rstd, long M, int C, float eps, void* stream) {
  if (dtype) return ln_fwd_t<bf16>((const bf16*)x, xps, w, b, (bf16*)y, mean, rstd, M, C, eps, (hipStream_t)stream);
  return ln_fwd_t<float>((const float*)x, xps, w, b, (float*)y, mean, rstd, M, C, eps, (hipStream_t)stream);
}

DMY_API int dmy_layernorm_bwd_blocks(long M) { return grid_cap(ceil_div(M, 64), 1024); }

template <typename T>
int ln_bwd_t(const T* x, long xps, const T* dy, long dps, const float* w, const float* mean, const float* rstd, T* dx,
             long dxps, int acc, long M, int C, float* pdw, float* pdb, hipStream_t st) {
  const int P = dmy_layernorm_bwd_blocks(M);
  const size_t lds = 4 * 2 * sizeof(float) * C;  // [4 waves][2][C]
  int L = ln_lanes<T>(C, xps, dxps, x, dx);
  if (L && (dps % Traits<T>::VW || ((uintptr_t)dy & 15))) L = 0;
  switch (L) {
    case 4: ln_bwd_vec<T, 4><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, pdw, pdb); break;
    case 8: ln_bwd_vec<T, 8><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, pdw, pdb); break;
    case 16: ln_bwd_vec<T, 16><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, pdw, pdb); break;
    case 32: ln_bwd_vec<T, 32><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, pdw, pdb); break;
    case 64: ln_bwd_vec<T, 64><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, pdw, pdb); break;
    default: {
      const int rpb = (int)((M + P - 1) / P);
      ln_bwd_kernel<T><<<P, 256, lds, st>>>(x, xps, dy, dps, w, mean, rstd, dx, dxps, acc, M, C, rpb, pdw, pdb);
    }
  }
  return (int)hipGetLastError();
}

DMY_API int dmy_layernorm_bwd(int dtype, const void* x, long xps, const void* dy, long dps, const float* w,
                              const float* mean, const float* rstd, void* dx, long dxps, int accumulate, long M, int C,
                              float* pdw, float* pdb, void* stream) {
  if (dtype)
    return ln_bwd_t<bf16>((const bf16*)x, xps, (const bf16*)dy, dps, w, mean, rstd, (bf16*)dx, dxps, accumulate, M, C,
                          pdw, pdb, (hipStream_t)stream);
  return ln_bwd_t<float>((const float*)x, xps, (const float*)dy, dps, w, mean, rstd, (float*)dx, dxps, accumulate, M,
                         C, pdw, pdb, (hipStream_t)stream);
}

DMY_API int dmy_winattn_fwd(int dtype, const void* qkv, const float* table, void* out, int B, int H, int W, int C,
                            int nh, int shift, float scale, void* stream) {
  if (C != nh * HD) return (int)hipErrorInvalidValue;
  SwinGeom g = make(B, H, W, C, nh, shift, scale);
  const int nwin = B * (g.Rp / WS) * (g.Cp / WS);
  dim3 grid(nwin, nh);
  if (dtype) {
    constexpr int NW = 2;
    long groups = 4096 / (nh > 0 ? nh : 1);  // ~4096 blocks: every window group keeps a prefetch chain of a few windows
    if (groups > ceil_div(nwin, NW)) groups = ceil_div(nwin, NW);
    const int wpb = ceil_div(nwin, groups);
    const int g8 = ceil_div(ceil_div(nwin, wpb), 8) * 8;  // xgroup / xhead order
    winattn_fwd_mfma<NW><<<g8 * nh, 64 * NW, 0, (hipStream_t)stream>>>((const bf16*)qkv, table, (bf16*)out, g, nwin, wpb);
  } else winattn_fwd_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>((const float*)qkv, table, (float*)out, g);
  return (int)hipGetLastError();
}

DMY_API int dmy_winattn_bwd_groups(int B, int H, int W, int nh) {
  const long nwin = (long)B * ((W + WS - 1) / WS) * ((H + WS - 1) / WS);
  long groups = 2048 / (nh > 0 ? nh : 1);
  if (groups < 1) groups = 1;
  if (groups > nwin) groups = nwin;
  return (int)((groups + 7) / 8 * 8);  // padded for the bf16 kernel's xgroup / xhead order (empty groups write zeros)
}

// every real pixel lies in exactly one window, so dqkv is fully written (padding tokens have no storage)
DMY_API int dmy_winattn_bwd(int dtype, const void* qkv, const void* dout, const float* table, void* dqkv,
                            float* dtab_part, float* dtab, int B, int H, int W, int C, int nh, int shift, float scale,
                            void* stream) {
  if (C != nh * HD) return (int)hipErrorInvalidValue;
  SwinGeom g = make(B, H, W, C, nh, shift, scale);
  const int nwin = B * (g.Rp / WS) * (g.Cp / WS);
  const int groups = dmy_winattn_bwd_groups(B, H, W, nh);
  const int wpb = (nwin + groups - 1) / groups;
  dim3 grid(groups, nh);
  hipStream_t st = (hipStream_t)stream;
  if (dtype) winattn_bwd_mfma<2><<<groups * nh, 128, 0, st>>>((const bf16*)qkv, (const bf16*)dout, table, (bf16*)dqkv, dtab_part, nwin, wpb, g);
  else winattn_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)qkv, (const float*)dout, table, (float*)dqkv, dtab_part, nwin, wpb, g);
  const int ntab = (2 * WS - 1) * (2 * WS - 1) * nh;
  dtab_reduce_kernel<<<ntab, 256, 0, st>>>(dtab_part, groups, nh, dtab);
  return (int)hipGetLastError();
}

DMY_API int dmy_droppath_add(int dtype, const void* x, const void* f, const float* u, float keep, void* y, long per,
                             long n, void* stream) {
  if (n == 0) return 0;
  const int vec = dtype && per % 8 == 0 && (((uintptr_t)x | (uintptr_t)f | (uintptr_t)y) & 15) == 0;
  const int g = grid_cap(ceil_div(vec ? n / 8 : n, 256), 16384);
  if (dtype) droppath_add_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)x, (const bf16*)f, u, keep, (bf16*)y, per, n, vec);
  else droppath_add_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)x, (const float*)f, u, keep, (float*)y, per, n, 0);
  return (int)hipGetLastError();
}
DMY_API int dmy_droppath_grad(int dtype, const void* dy, const float* u, float keep, void* df, long per, long n,
                              void* stream) {
  if (n == 0) return 0;
  const int vec = dtype && per % 8 == 0 && (((uintptr_t)dy | (uintptr_t)df) & 15) == 0;
  const int g = grid_cap(ceil_div(vec ? n / 8 : n, 256), 16384);
  if (dtype) droppath_grad_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)dy, u, keep, (bf16*)df, per, n, vec);
  else droppath_grad_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)dy, u, keep, (float*)df, per, n, 0);
  return (int)hipGetLastError();
}

DMY_API int dmy_sample_scale(int dtype, const void* x, const float* sc, void* y, long per, long n, void* stream) {
  const int g = grid_cap(ceil_div(n, 256), 8192);
  if (dtype) sample_scale_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)x, sc, (bf16*)y, per, n);
  else sample_scale_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)x, sc, (float*)y, per, n);
  return (int)hipGetLastError();
}
