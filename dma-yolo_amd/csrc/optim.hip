// Multi-tensor optimizer / EMA kernels (HBM-bound).  Replaces torch.optim.SGD(nesterov) / Adam as
// configured by train.py:197-222 and ModelEMA.update (utils/torch_utils.py:329-339).
// One launch per parameter group: blocks walk a (tensor, chunk) table built on the host.
#include "common.h"

namespace {

constexpr int CHUNK = 8192;

struct TList {
  float* const* p;        // params (or EMA tensors)
  const float* const* g;  // grads (or model tensors)
  float* const* m;        // momentum / exp_avg
  float* const* v;        // exp_avg_sq
  const long* n;          // numel per tensor
  const int* tid;         // chunk table: tensor index
  const long* off;        // chunk table: element offset
};

__global__ void sgd_kernel(TList L, float lr, float mom, float wd, int nesterov, int first) {
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* p = L.p[t];
  const float* g = L.g[t];
  float* b = L.m[t];
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) {
    float d = g[i];
    if (wd != 0.f) d += wd * p[i];
    float bv;
    if (first) bv = d;
    else bv = mom * b[i] + d;
    b[i] = bv;
    if (nesterov) d = d + mom * bv;
    else d = bv;
    p[i] -= lr * d;
  }
}

__global__ void adam_kernel(TList L, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2s) {
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* p = L.p[t];
  const float* g = L.g[t];
  float* m = L.m[t];
  float* v = L.v[t];
  const float step = lr / bc1;
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) {
    float d = g[i];
    if (wd != 0.f) d += wd * p[i];
    const float mv = m[i] + (1.f - b1) * (d - m[i]);  // torch: exp_avg.lerp_(grad, 1 - beta1)
    const float vv = v[i] * b2 + (1.f - b2) * d * d;
    m[i] = mv;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2s + eps;
    p[i] -= step * (mv / denom);
  }
}

__global__ void ema_kernel(TList L, float d) {
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* e = L.p[t];
  const float* s = L.g[t];
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) e[i] = e[i] * d + (1.f - d) * s[i];
}

}  // namespace

DMY_API int dmy_chunk_size() { return CHUNK; }

DMY_API int dmy_sgd(float* const* p, const float* const* g, float* const* m, const long* n, const int* tid,
                    const long* off, int nchunks, float lr, float mom, float wd, int nesterov, int first,
                    void* stream) {
  if (nchunks == 0) return 0;
  TList L{p, g, m, nullptr, n, tid, off};
  sgd_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, lr, mom, wd, nesterov, first);
  return (int)hipGetLastError();
}

DMY_API int dmy_adam(float* const* p, const float* const* g, float* const* m, float* const* v, const long* n,
                     const int* tid, const long* off, int nchunks, float lr, float b1, float b2, float eps, float wd,
                     float bc1, float bc2s, void* stream) {
  if (nchunks == 0) return 0;
  TList L{p, g, m, v, n, tid, off};
  adam_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, lr, b1, b2, eps, wd, bc1, bc2s);
  return (int)hipGetLastError();
}

DMY_API int dmy_ema(float* const* e, const float* const* s, const long* n, const int* tid, const long* off,
                    int nchunks, float d, void* stream) {
  if (nchunks == 0) return 0;
  TList L{e, s, nullptr, nullptr, n, tid, off};
  ema_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, d);
  return (int)hipGetLastError();
}
