// Validation matching on gfx950: the reference's process_batch (val.py:62-83) for a whole batch of
// images in one launch, one workgroup per image.  box_iou follows utils/metrics.py:254-276 (labels are
// box1, detections box2; no eps), in fp32 with products kept unfused so every IoU is the bit pattern
// the reference computes.
//
// The reference's matching (val.py:70-81), restated per image:
//   candidates (l, d): iou(l, d) >= iouv[0] and class(l) == class(d)
//   1. for every detection keep its highest-IoU candidate (argsort(iou)[::-1] then np.unique over the
//      detection column keeps the first occurrence); on an exact IoU tie the later label wins (numpy's
//      insertion sort for <= 16 candidates is stable, reversed: the larger where-index first; beyond 16
//      candidates numpy's introsort leaves exact ties unspecified -- ties need duplicate label boxes)
//   2. np.unique orders the survivors by detection index; np.unique over the label column then keeps,
//      for every label, the survivor with the SMALLEST detection index (not the highest IoU: the
//      re-sort is commented out at val.py:78)
//   3. correct[d][t] = matched_iou(d) >= iouv[t]
#include "common.h"

namespace {

DEV float box_iou_ref(const float* a, const float* b) {  // a = label xyxy, b = detection xyxy
  const float w = fmaxf(fminf(a[2], b[2]) - fmaxf(a[0], b[0]), 0.f);
  const float h = fmaxf(fminf(a[3], b[3]) - fmaxf(a[1], b[1]), 0.f);
  const float inter = __fmul_rn(w, h);
  const float area_a = __fmul_rn(a[2] - a[0], a[3] - a[1]);
  const float area_b = __fmul_rn(b[2] - b[0], b[3] - b[1]);
  return inter / (area_a + area_b - inter);
}

// det [ND][6] (x1 y1 x2 y2 conf cls), lab [NL][5] (cls x1 y1 x2 y2); doff / loff [B + 1] row offsets
__global__ void __launch_bounds__(256) process_batch_kernel(const float* __restrict__ det, const int* __restrict__ doff,
                                                            const float* __restrict__ lab, const int* __restrict__ loff,
                                                            const float* __restrict__ iouv, int T,
                                                            int* __restrict__ best_lab, float* __restrict__ best_iou,
                                                            int* __restrict__ win, unsigned char* __restrict__ correct) {
  const int b = blockIdx.x;
  const int d0 = doff[b], d1 = doff[b + 1], l0 = loff[b], l1 = loff[b + 1];
  const float thr = iouv[0];
  // 1. best label per detection
  for (int d = d0 + (int)threadIdx.x; d < d1; d += blockDim.x) {
    const float* db = det + (long)d * 6;
    int bl = -1;
    float bi = 0.f;
    for (int l = l0; l < l1; ++l) {
      const float* lb = lab + (long)l * 5;
      if (lb[0] != db[5]) continue;
      const float iou = box_iou_ref(lb + 1, db);
      if (iou >= thr && (bl < 0 || iou >= bi)) {  // >=: the later label wins an exact tie
        bl = l;
        bi = iou;
      }
    }
    best_lab[d] = bl;
    best_iou[d] = bi;
    win[d] = 0;
  }
  __syncthreads();
  // 2. every label keeps its smallest-index surviving detection
  for (int l = l0 + (int)threadIdx.x; l < l1; l += blockDim.x)
    for (int d = d0; d < d1; ++d)
      if (best_lab[d] == l) {
        win[d] = 1;
        break;
      }
  __syncthreads();
  // 3. correct flags per IoU level
  for (long e = (long)d0 * T + threadIdx.x; e < (long)d1 * T; e += blockDim.x) {
    const int d = (int)(e / T), t = (int)(e % T);
    correct[e] = (win[d] && best_iou[d] >= iouv[t]) ? 1 : 0;
  }
}

}  // namespace

DMY_API int dmy_process_batch(const float* det, const int* det_off, const float* lab, const int* lab_off, int B,
                              const float* iouv, int T, int* ws_lab, float* ws_iou, int* ws_win,
                              unsigned char* correct, void* stream) {
  if (B <= 0) return 0;
  process_batch_kernel<<<B, 256, 0, (hipStream_t)stream>>>(det, det_off, lab, lab_off, iouv, T, ws_lab, ws_iou, ws_win,
                                                           correct);
  return (int)hipGetLastError();
}
