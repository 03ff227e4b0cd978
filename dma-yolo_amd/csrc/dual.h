// Forward-mode dual numbers over 4 seed variables (a predicted box): value + 4 partials.  Used for
// the IoU-family losses (SIoU in detect_loss.hip, CIoU in tal.hip) so their gradients come out of the
// same evaluation as the loss (no autograd tape).  Tie rules follow torch (minimum / maximum split
// the gradient on ties, clamp(min=0) passes it at 0).
#pragma once
#include "common.h"

struct D4 {
  float v, d[4];
};
DEV D4 dc(float v) { D4 r; r.v = v; r.d[0] = r.d[1] = r.d[2] = r.d[3] = 0.f; return r; }
DEV D4 operator+(D4 a, D4 b) { D4 r; r.v = a.v + b.v; for (int i = 0; i < 4; ++i) r.d[i] = a.d[i] + b.d[i]; return r; }
DEV D4 operator-(D4 a, D4 b) { D4 r; r.v = a.v - b.v; for (int i = 0; i < 4; ++i) r.d[i] = a.d[i] - b.d[i]; return r; }
DEV D4 operator*(D4 a, D4 b) { D4 r; r.v = a.v * b.v; for (int i = 0; i < 4; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i]; return r; }
DEV D4 operator/(D4 a, D4 b) {
  D4 r; r.v = a.v / b.v;
  for (int i = 0; i < 4; ++i) r.d[i] = (a.d[i] * b.v - a.v * b.d[i]) / (b.v * b.v);
  return r;
}
DEV D4 scal(D4 a, float s) { D4 r; r.v = a.v * s; for (int i = 0; i < 4; ++i) r.d[i] = a.d[i] * s; return r; }
DEV D4 dmin(D4 a, D4 b) {  // torch.minimum: ties split the gradient
  if (a.v < b.v) return a;
  if (b.v < a.v) return b;
  D4 r; r.v = a.v; for (int i = 0; i < 4; ++i) r.d[i] = 0.5f * (a.d[i] + b.d[i]); return r;
}
DEV D4 dmax(D4 a, D4 b) {
  if (a.v > b.v) return a;
  if (b.v > a.v) return b;
  D4 r; r.v = a.v; for (int i = 0; i < 4; ++i) r.d[i] = 0.5f * (a.d[i] + b.d[i]); return r;
}
DEV D4 dclamp0(D4 a) {  // clamp(min=0): gradient passes where a >= 0
  if (a.v >= 0.f) return a;
  return dc(0.f);
}
DEV D4 dabs(D4 a) {
  const float s = a.v > 0.f ? 1.f : (a.v < 0.f ? -1.f : 0.f);
  D4 r; r.v = fabsf(a.v); for (int i = 0; i < 4; ++i) r.d[i] = s * a.d[i]; return r;
}
DEV D4 dfun(D4 a, float v, float dv) { D4 r; r.v = v; for (int i = 0; i < 4; ++i) r.d[i] = dv * a.d[i]; return r; }
DEV D4 dexp(D4 a) { const float e = expf(a.v); return dfun(a, e, e); }
DEV D4 dsqrt(D4 a) { const float s = powf(a.v, 0.5f); return dfun(a, s, 0.5f * powf(a.v, -0.5f)); }
DEV D4 dcos(D4 a) { return dfun(a, cosf(a.v), -sinf(a.v)); }
DEV D4 dasin(D4 a) { return dfun(a, asinf(a.v), 1.0f / sqrtf(1.0f - a.v * a.v)); }
DEV D4 dsq(D4 a) { return dfun(a, a.v * a.v, 2.f * a.v); }
DEV D4 dpow4(D4 a) { const float s = a.v * a.v; return dfun(a, s * s, 4.f * s * a.v); }

DEV D4 datan(D4 a) { return dfun(a, atanf(a.v), 1.0f / (1.0f + a.v * a.v)); }
