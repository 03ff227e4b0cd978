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

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w; per-block partials of dw, db
template <typename T>
__global__ void ln_bwd_kernel(const T* __restrict__ x, long xps, const T* __restrict__ dy, long dps,
                              const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
                              T* __restrict__ dx, long dxps, long M, int C, int rows_per_block, float* __restrict__ pdw,
                              float* __restrict__ pdb) {
  extern __shared__ float sh[];  // [2][C]
  float* sdw = sh;
  float* sdb = sh + C;
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) sh[c] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (long m = r0 + (threadIdx.x >> 6); m < r1; m += (blockDim.x >> 6)) {
    const float mu = mean[m], rs = rstd[m];
    float a1 = 0.f, a2 = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float xh = (to_f(x[m * xps + c]) - mu) * rs;
      const float gy = to_f(dy[m * dps + c]);
      const float g = gy * w[c];
      a1 += g;
      a2 += g * xh;
      atomicAdd(&sdw[c], gy * xh);
      atomicAdd(&sdb[c], gy);
    }
    a1 = wave_sum(a1) / C;
    a2 = wave_sum(a2) / C;
    for (int c = lane; c < C; c += 64) {
      const float xh = (to_f(x[m * xps + c]) - mu) * rs;
      const float g = to_f(dy[m * dps + c]) * w[c];
      dx[m * dxps + c] = from_f<T>(rs * (g - a1 - xh * a2));
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    pdw[(long)blockIdx.x * C + c] = sdw[c];
    pdb[(long)blockIdx.x * C + c] = sdb[c];
  }
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
  __shared__ float dtab[(2 * WS - 1) * (2 * WS - 1)];
  const int ntab = (2 * WS - 1) * (2 * WS - 1);
  for (int e = threadIdx.x; e < ntab; e += blockDim.x) dtab[e] = 0.f;
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
        const int idx = ((i >> 3) - (j >> 3) + WS - 1) * (2 * WS - 1) + ((i & 7) - (j & 7) + WS - 1);
        atomicAdd(&dtab[idx], ds);
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
  __syncthreads();
  for (int e = threadIdx.x; e < ntab; e += blockDim.x)
    dtab_part[((long)blockIdx.x * g.nh + head) * ntab + e] = dtab[e];
}

// table grad [225][nh] = sum over window groups
__global__ void dtab_reduce_kernel(const float* __restrict__ part, int ngroups, int nh, float* __restrict__ dtab) {
  const int ntab = (2 * WS - 1) * (2 * WS - 1);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ntab * nh) return;
  const int idx = e / nh, h = e % nh;
  double s = 0.0;
  for (int gi = 0; gi < ngroups; ++gi) s += part[((long)gi * nh + h) * ntab + idx];
  dtab[e] = (float)s;
}

// per-sample scale (DropPath, common.py:386-403): y = x * sc[b]  (sc = floor(keep + u) / keep)
template <typename T>
__global__ void sample_scale_kernel(const T* __restrict__ x, const float* __restrict__ sc, T* __restrict__ y, long per,
                                    long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = from_f<T>(to_f(x[i]) * sc[i / per]);
}

SwinGeom make(int B, int H, int W, int C, int nh, int shift, float scale) {
  SwinGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C; g.nh = nh; g.shift = shift; g.scale = scale;
  g.Rp = (W + WS - 1) / WS * WS;  // Swin rows = image W axis
  g.Cp = (H + WS - 1) / WS * WS;
  return g;
}

}  // namespace

DMY_API int dmy_layernorm_fwd(int dtype, const void* x, long xps, const float* w, const float* b, void* y, float* mean,
                              float* rstd, long M, int C, float eps, void* stream) {
  const int g = grid_cap(ceil_div(M, 4), 4096);
  if (dtype) ln_fwd_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)x, xps, w, b, (bf16*)y, mean, rstd, M, C, eps);
  else ln_fwd_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)x, xps, w, b, (float*)y, mean, rstd, M, C, eps);
  return (int)hipGetLastError();
}

DMY_API int dmy_layernorm_bwd_blocks(long M) { return grid_cap(ceil_div(M, 64), 1024); }

DMY_API int dmy_layernorm_bwd(int dtype, const void* x, long xps, const void* dy, long dps, const float* w,
                              const float* mean, const float* rstd, void* dx, long dxps, long M, int C, float* pdw,
                              float* pdb, void* stream) {
  const int P = dmy_layernorm_bwd_blocks(M);
  const int rpb = (int)((M + P - 1) / P);
  const size_t lds = 2 * sizeof(float) * C;
  if (dtype) ln_bwd_kernel<bf16><<<P, 256, lds, (hipStream_t)stream>>>((const bf16*)x, xps, (const bf16*)dy, dps, w, mean, rstd, (bf16*)dx, dxps, M, C, rpb, pdw, pdb);
  else ln_bwd_kernel<float><<<P, 256, lds, (hipStream_t)stream>>>((const float*)x, xps, (const float*)dy, dps, w, mean, rstd, (float*)dx, dxps, M, C, rpb, pdw, pdb);
  return (int)hipGetLastError();
}

DMY_API int dmy_winattn_fwd(int dtype, const void* qkv, const float* table, void* out, int B, int H, int W, int C,
                            int nh, int shift, float scale, void* stream) {
  if (C != nh * HD) return (int)hipErrorInvalidValue;
  SwinGeom g = make(B, H, W, C, nh, shift, scale);
  dim3 grid(B * (g.Rp / WS) * (g.Cp / WS), nh);
  if (dtype) winattn_fwd_kernel<bf16><<<grid, 256, 0, (hipStream_t)stream>>>((const bf16*)qkv, table, (bf16*)out, g);
  else winattn_fwd_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>((const float*)qkv, table, (float*)out, g);
  return (int)hipGetLastError();
}

DMY_API int dmy_winattn_bwd_groups(int B, int H, int W, int nh) {
  const long nwin = (long)B * ((W + WS - 1) / WS) * ((H + WS - 1) / WS);
  long groups = 2048 / (nh > 0 ? nh : 1);
  if (groups < 1) groups = 1;
  if (groups > nwin) groups = nwin;
  return (int)groups;
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
  if (dtype) winattn_bwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)qkv, (const bf16*)dout, table, (bf16*)dqkv, dtab_part, nwin, wpb, g);
  else winattn_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)qkv, (const float*)dout, table, (float*)dqkv, dtab_part, nwin, wpb, g);
  const int ntab = (2 * WS - 1) * (2 * WS - 1) * nh;
  dtab_reduce_kernel<<<ceil_div(ntab, 256), 256, 0, st>>>(dtab_part, groups, nh, dtab);
  return (int)hipGetLastError();
}

DMY_API int dmy_sample_scale(int dtype, const void* x, const float* sc, void* y, long per, long n, void* stream) {
  const int g = grid_cap(ceil_div(n, 256), 8192);
  if (dtype) sample_scale_kernel<bf16><<<g, 256, 0, (hipStream_t)stream>>>((const bf16*)x, sc, (bf16*)y, per, n);
  else sample_scale_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)x, sc, (float*)y, per, n);
  return (int)hipGetLastError();
}
