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

// GradScaler (train.py:354, 445-450; torch.amp.GradScaler defaults) kept on the device: `scale` is the loss
// scale, `found` the non-finite flag of this step's gradients.  Both null = scaler disabled.  The optimizer
// kernels unscale on the fly (g * (1 / scale), exact: the scale is a power of two) and skip the update when
// `found` is set, as scaler.step() skips optimizer.step(); no host synchronisation anywhere.
DEV bool amp_skip(const float* found) { return found != nullptr && *found != 0.f; }
DEV float amp_inv(const float* scale) { return scale != nullptr ? (float)(1.0 / (double)*scale) : 1.f; }

__global__ void sgd_kernel(TList L, float lr, float mom, float wd, int nesterov, const float* scale,
                           const float* found) {
  if (amp_skip(found)) return;
  const float inv = amp_inv(scale);
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* p = L.p[t];
  const float* g = L.g[t];
  float* b = L.m[t];
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) {
    float d = g[i] * inv;
    if (wd != 0.f) d += wd * p[i];
    // momentum buffers start zeroed: mom * 0 + d == d is torch.optim.SGD's clone-on-first-step exactly
    const float bv = mom * b[i] + d;
    b[i] = bv;
    if (nesterov) d = d + mom * bv;
    else d = bv;
    p[i] -= lr * d;
  }
}

// dstep (nullable): the group's step count on the device, the count BEFORE this step.  When given, the bias
// corrections come from it (bc1 = 1 - b1^t, bc2s = sqrt(1 - b2^t), t = *dstep + 1, in double as torch.optim.Adam
// computes them on the host) and adam_step_kernel advances it afterwards only if the step was not skipped: a step
// the GradScaler skips does not advance Adam's t, as torch, where scaler.step() never calls optimizer.step().
__global__ void adam_kernel(TList L, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2s,
                            const float* scale, const float* found, const int* dstep) {
  if (amp_skip(found)) return;
  if (dstep != nullptr) {
    const double t = (double)(*dstep + 1);
    bc1 = (float)(1.0 - pow((double)b1, t));
    bc2s = (float)sqrt(1.0 - pow((double)b2, t));
  }
  const float inv = amp_inv(scale);
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* p = L.p[t];
  const float* g = L.g[t];
  float* m = L.m[t];
  float* v = L.v[t];
  const float step = lr / bc1;
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) {
    float d = g[i] * inv;
    if (wd != 0.f) d += wd * p[i];
    const float mv = m[i] + (1.f - b1) * (d - m[i]);  // torch: exp_avg.lerp_(grad, 1 - beta1)
    const float vv = v[i] * b2 + (1.f - b2) * d * d;
    m[i] = mv;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2s + eps;
    p[i] -= step * (mv / denom);
  }
}

__global__ void adam_step_kernel(int* dstep, const float* found) {
  if (threadIdx.x == 0 && !amp_skip(found)) *dstep += 1;
}

__global__ void ema_kernel(TList L, float d) {
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  float* e = L.p[t];
  const float* s = L.g[t];
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) e[i] = e[i] * d + (1.f - d) * s[i];
}

// scaler.unscale_'s non-finite check over every gradient of the step (the g list of the table)
__global__ void amp_check_kernel(TList L, const float* __restrict__ scale, float* __restrict__ found) {
  const int t = L.tid[blockIdx.x];
  const long o = L.off[blockIdx.x];
  const long end = min(L.n[t], o + CHUNK);
  const float inv = amp_inv(scale);
  const float* g = L.g[t];
  bool bad = false;
  for (long i = o + threadIdx.x; i < end; i += blockDim.x) bad |= !isfinite(g[i] * inv);
  if (__any(bad) && (threadIdx.x & 63) == 0) *found = 1.f;  // every writer stores the same value
}

// scaler.update(): backoff on a non-finite step, growth after `interval` clean steps; gup = scale * world is the
// loss's upstream gradient (scaler.scale(loss * WORLD_SIZE).backward(), train.py:440-445); found is re-armed
__global__ void amp_update_kernel(float* scale, float* gup, int* tracker, float* found, float world, float growth,
                                  float backoff, int interval) {
  if (threadIdx.x != 0) return;
  float s = *scale;
  if (*found != 0.f) {
    s *= backoff;
    *tracker = 0;
  } else {
    const int n = *tracker + 1;
    if (n == interval) {
      s *= growth;
      *tracker = 0;
    } else {
      *tracker = n;
    }
  }
  *scale = s;
  *gup = s * world;
  *found = 0.f;
}

}  // namespace

DMY_API int dmy_chunk_size() { return CHUNK; }

DMY_API int dmy_amp_check(const float* const* g, const long* n, const int* tid, const long* off, int nchunks,
                          const float* scale, float* found, void* stream) {
  if (nchunks == 0) return 0;
  TList L{nullptr, g, nullptr, nullptr, n, tid, off};
  amp_check_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, scale, found);
  return (int)hipGetLastError();
}

DMY_API int dmy_amp_update(float* scale, float* gup, int* tracker, float* found, float world, float growth,
                           float backoff, int interval, void* stream) {
  amp_update_kernel<<<1, 64, 0, (hipStream_t)stream>>>(scale, gup, tracker, found, world, growth, backoff, interval);
  return (int)hipGetLastError();
}

DMY_API int dmy_sgd(float* const* p, const float* const* g, float* const* m, const long* n, const int* tid,
                    const long* off, int nchunks, float lr, float mom, float wd, int nesterov, const float* scale,
                    const float* found, void* stream) {
  if (nchunks == 0) return 0;
  TList L{p, g, m, nullptr, n, tid, off};
  sgd_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, lr, mom, wd, nesterov, scale, found);
  return (int)hipGetLastError();
}

DMY_API int dmy_adam(float* const* p, const float* const* g, float* const* m, float* const* v, const long* n,
                     const int* tid, const long* off, int nchunks, float lr, float b1, float b2, float eps, float wd,
                     float bc1, float bc2s, const float* scale, const float* found, int* dstep, void* stream) {
  if (nchunks == 0) return 0;
  TList L{p, g, m, v, n, tid, off};
  adam_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, lr, b1, b2, eps, wd, bc1, bc2s, scale, found, dstep);
  if (dstep != nullptr) adam_step_kernel<<<1, 64, 0, (hipStream_t)stream>>>(dstep, found);
  return (int)hipGetLastError();
}

DMY_API int dmy_ema(float* const* e, const float* const* s, const long* n, const int* tid, const long* off,
                    int nchunks, float d, void* stream) {
  if (nchunks == 0) return 0;
  TList L{e, s, nullptr, nullptr, n, tid, off};
  ema_kernel<<<nchunks, 256, 0, (hipStream_t)stream>>>(L, d);
  return (int)hipGetLastError();
}
