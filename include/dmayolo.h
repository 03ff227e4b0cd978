/* dmayolo.h — C ABI of the MI355X-native (gfx950) DMA-YOLO detection path.
 *
 * The reference (Yaling-Li/DMA-YOLO) is pure Python: its plugin boundary is the YAML module
 * namespace that models/yolo.py:377 resolves with eval(name), plus ComputeLoss
 * (utils/loss.py:135-218) and non_max_suppression (utils/general.py:633-725).  Every ATen kernel
 * those Python entry points reach is replaced by one entry point below; the Python host side
 * (dma-yolo_amd/dmayolo) binds them with ctypes.
 *
 * Conventions
 *   dtype      0 = float32 storage (parity mode), 1 = bfloat16 storage (throughput mode)
 *   layout     activations are NHWC; `*ps` is the pixel stride in elements (>= C), so a channel
 *              slice of a concatenation buffer is (base + c0, ps = Ctot)
 *   weights    fp32 master weights are OIHW (torch layout); conv kernels consume OHWI / IHWO copies
 *   stream     hipStream_t passed as void*; every call is stream-ordered and never synchronises
 *   return     0 on success, else the hipError_t of the launch.  *_partial_rows / *_blocks return sizes.
 */
#ifndef DMAYOLO_H
#define DMAYOLO_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- convolution: replaces nn.Conv2d in models/cspcm.py:15 (YAML Conv), models/common.py:67 (Conv),
 *      :1283-1304 (SCConv k2/k3/k4), :1172-1178 (CoorAttention conv1/conv_h/conv_w), models/yolo.py:63
 *      (Detect.m), and nn.Linear (common.py:105-108, 483-484) as a 1x1 conv over tokens. */
int dmy_conv_fwd_partial_rows(long M, int K);
/* BN partial rows dmy_conv_fwd writes for exactly these arguments (psum / psq must hold that many rows of K floats):
 * the per-tile count of dmy_conv_fwd_partial_rows, or one row per wave of the persistent halo kernel
 * (3x3 stride-1 64 -> 64-channel layers, csrc/conv.hip conv3_halo64) */
/* BN partial rows: an upper bound for any route of a training forward with these M / K (allocate this many rows of
 * psum / psq), and the rows the last training forward launched on this host thread actually wrote (pass that count
 * to dmy_colsum2 / dmy_bn_finalize).  Replaces the host-side prediction dmy_conv_fwd_bn_rows for allocation: the
 * count comes from the routing that launched.  BatchNorm2d.forward's batch statistics,
 * torch/nn/modules/batchnorm.py via models/common.py:72 */
long dmy_conv_fwd_bound_rows(long M, int K);
long dmy_conv_fwd_last_rows(void);
int dmy_conv_fwd_bn_rows(int dtype, const void* x, const void* w_ohwi, const float* bias, const void* y, int N,
                                int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW,
                                long yps);
int dmy_conv_fwd(int dtype, const void* x, const void* w_ohwi, const float* bias, void* y, float* psum, float* psq,
                 int N, int H, int W, int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps,
                 void* stream);
/* Inference form (eval BN / fused-model Conv), in one launch:
 * y = act(T(conv(x) + bias) * scale + shift) (+ res), the value dmy_conv_fwd + dmy_bn_act_fwd produce, in one
 * launch (models/common.py:69-77 forward / forward_fuse with BN in eval mode).  scale/shift may be NULL. */
int dmy_conv_fwd_act(int dtype, const void* x, const void* w_ohwi, const float* bias, void* y, int N, int H, int W,
                     int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, const float* scale,
                     const float* shift, int act, const void* res, long rps, void* stream);
/* inference forward with a split-K workspace for small M (batch-1 detect, csrc conv_fwd_split + splitk_epi):
 * dmy_conv_fwd_act semantics; ws of dmy_conv_fwd_splitk_elems floats (0 = no split for these arguments). */
long dmy_conv_fwd_splitk_elems(int dtype, const void* x, const void* w_ohwi, const void* y, int N, int H, int W, int C,
                               long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps);
int dmy_conv_fwd_act_ws(int dtype, const void* x, const void* w_ohwi, const float* bias, void* y, int N, int H, int W,
                        int C, long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, const float* scale,
                        const float* shift, int act, const void* res, long rps, float* ws, long ws_elems, void* stream);
int dmy_conv_dgrad(int dtype, const void* dy, const void* w_ihwo, void* dx, int accumulate, int N, int H, int W, int C,
                   long xps, int K, int KH, int KW, int S, int P, int OH, int OW, long yps, void* stream);
int dmy_conv_wgrad(int dtype, const void* x, const void* dy, float* dw_ohwi, int N, int H, int W, int C, long xps,
                   int K, int KH, int KW, int S, int P, int OH, int OW, long yps, void* stream);
/* bwd1x1.hip: fused backward of a train-mode 1x1 stride-1 Conv -> BatchNorm -> act (models/common.py:67-73, k = 1),
 * bf16: dz = dmy_bn_bwd_apply's value on (dy, z) in registers (never stored), then dx (+)= dz Wt and dw += dz^T x in
 * one persistent launch.  Replaces dmy_bn_bwd_apply + dmy_conv_dgrad + dmy_conv_wgrad_ex(OIHW) of such a layer; the
 * reduce / finalize that produce ca, cb, cc run before it as before.  x / dx / dy: [M][C] / [M][C] / [M][K] rows of
 * pixel stride xps / bps / dps; z dense [M][K]; wt = the IHWO copy [C][K]; dw fp32 [K][C], ACCUMULATED (the caller
 * zeroes it).  _ok: 1 when this shape / alignment is supported (else the call returns -1 and launches nothing).
 * ws (nullable): deterministic mode -- the per-block weight-grad partials go to ws (ws_elems >= _ws_elems) and are
 * summed in block order (run-to-run bit-identical dw), instead of fp32 atomics. */
int dmy_conv1x1_bwd_bn_ok(long M, int K, int C, long dps, long xps, long bps, const void* dy, const void* z,
                          const void* x, const void* dx);
int dmy_conv1x1_bwd_bn(const void* dy, long dps, const void* z, const void* x, long xps, const void* wt,
                       const float* scale, const float* shift, const float* mean, const float* invstd, int act,
                       const float* ca, const float* cb, const float* cc, void* dx, long bps, int accumulate,
                       float* dw, float* ws, long ws_elems, long M, int K, int C, void* stream);
long dmy_conv1x1_bwd_bn_ws_elems(long M, int K, int C);
/* flags: 1 = write dw in torch OIHW order (the parameter's .grad layout, no wgrad_to_oihw pass; needs Cp == C),
 *        2 = dw is already zero (a per-step gradient arena cleared once), skip the memset.  Same sums as above. */
int dmy_conv_wgrad_ex(int dtype, const void* x, const void* dy, float* dw, int N, int H, int W, int C, long xps, int K,
                      int KH, int KW, int S, int P, int OH, int OW, long yps, int flags, void* stream);
/* Deterministic weight-grad (same sums, run-to-run bit-identical): the split-K partials go to the fp32 workspace
 * ws (no atomics) and are reduced in split order.  dmy_conv_wgrad_ws_elems: workspace elements the same call needs
 * (0 = one split, ws may be NULL). */
long dmy_conv_wgrad_ws_elems(int dtype, const void* x, const void* dy, int N, int H, int W, int C, long xps, int K,
                             int KH, int KW, int S, int P, int OH, int OW, long yps, int flags);
int dmy_conv_wgrad_det(int dtype, const void* x, const void* dy, float* dw, int N, int H, int W, int C, long xps,
                       int K, int KH, int KW, int S, int P, int OH, int OW, long yps, int flags, float* ws,
                       long ws_elems, void* stream);
/* Cp >= C: input channels zero-padded to a full 16-byte vector (the 3-channel stem, yaml:15) */
int dmy_conv_wprep(int dtype, const float* w_oihw, void* w_ohwi, void* w_ihwo, int K, int C, int Cp, int KH, int KW,
                   void* stream);
/* All conv weights of a model in one launch: descs is a DEVICE array of n records
 * { const float* w_oihw; void* w_ohwi; void* w_ihwo (nullable); int K, C, KH, KW; } (40 bytes, 8-byte aligned),
 * each as dmy_conv_wprep with Cp == C. */
int dmy_conv_wprep_multi(int dtype, const void* descs, int n, void* stream);
/* Stem as space-to-depth (yolov5*.yaml / DMA-YOLO yaml layer 0: Conv(3, c2, 6, 2, 2), models/common.py:50-77):
 * the k6 s2 p2 conv over x == a k3 s1 p1 conv over dmy_image_s2d(x) with these weights (Cs >= 4C channels). */
int dmy_conv_wprep_s2d(int dtype, const float* w_oihw, void* w_s2d, int K, int C, int Cs, void* stream);
int dmy_conv_wgrad_s2d_to_oihw(const float* dw_s2d, float* dw_oihw, int K, int C, int Cs, void* stream);
int dmy_conv_wgrad_to_oihw(const float* dw_ohwi, float* dw_oihw, int K, int C, int Cp, int KH, int KW, void* stream);

/* ---- fp8 (OCP e4m3fn) forward conv for config 5 (BASELINE configs[4], "fp8 MFMA conv"): replaces the forward of
 *      Conv.conv (models/common.py:61-74) when enabled; backward stays bf16.  Activations are quantised per
 *      tensor with the current amax (x ~ x8 * amax / 448), weights per output channel (w ~ w8 * wscale[k]);
 *      the MX-scaled 16x16x128 MFMA runs with unit block scales and the accumulator is dequantised in the
 *      epilogue.  Requirements: C % 128 == 0, K % 8 == 0, x8 dense [N*H*W][C]. */
long dmy_fp8_quant_ws_elems(void);  /* float workspace of dmy_fp8_quant; ws[0] = the amax used */
int dmy_fp8_quant(const void* x_bf16, long rows, int C, long xps, void* x8, float* ws, void* stream);
int dmy_conv_wprep_fp8(const float* w_oihw, void* w8_ohwi, float* wscale, int K, int C, int KH, int KW, void* stream);
int dmy_conv_fwd_fp8_partial_rows(long M, int K); /* BN partial rows of dmy_conv_fwd_fp8's epilogue */
int dmy_conv_fwd_fp8(const void* x8, const void* w8_ohwi, const float* xamax, const float* wscale, const float* bias,
                     void* y, float* psum, float* psq, int N, int H, int W, int C, int K, int KH, int KW, int S, int P,
                     int OH, int OW, long yps, const float* scale, const float* shift, int act, const void* res,
                     long rps, void* stream);

/* ---- BatchNorm2d + activation: replaces nn.BatchNorm2d/nn.SiLU/nn.Hardswish in models/common.py:68-73,
 *      1176-1180, 1284-1306 with utils/torch_utils.py:161-170 eps/momentum. act: 0 none 1 silu 2 hardswish
 *      3 sigmoid 4 gelu(erf). */
int dmy_bn_partial_rows(long M);
int dmy_bn_stats(int dtype, const void* z, long zps, long M, int C, float* psum, float* psq, void* stream);
int dmy_bn_finalize(const float* psum, const float* psq, int P, int C, double count, const float* gamma,
                    const float* beta, float* running_mean, float* running_var, long long* num_batches_tracked,
                    float momentum, float eps, int update, float* mean, float* invstd, float* scale, float* shift,
                    void* stream);
int dmy_bn_eval_coef(const float* gamma, const float* beta, const float* running_mean, const float* running_var,
                     float eps, int C, float* scale, float* shift, void* stream);
int dmy_bn_act_fwd(int dtype, const void* z, long zps, const float* scale, const float* shift, int act,
                   const void* res, long rps, void* y, long yps, long M, int C, void* stream);
/* config-5 fp8 with delayed scaling: dmy_bn_act_fwd (bf16) that also writes the e4m3 copy y8 [M][C] (dense) of its
 * output for an e4m3 conv consumer (dmy_conv_fwd_fp8), quantised with the PREVIOUS step's amax -- the max over the
 * dmy_bn_act_f8_blocks() floats pmax that the previous call left in its nmax; used[0] receives that amax (the conv's
 * xamax) -- and leaves this step's block maxima in nmax (same size).  Replaces dmy_fp8_quant's two passes.
 * headroom (>= 1) multiplies that amax (Transformer-Engine-style margin against a growing range); nsat (nullable, same
 * size as nmax) receives per block the count of elements that saturated at +-448. */
int dmy_bn_act_f8_blocks(void);
int dmy_bn_act_fwd_f8(const void* z, long zps, const float* scale, const float* shift, int act, const void* res,
                      long rps, void* y, long yps, long M, int C, void* y8, const float* pmax, float* nmax, float* used,
                      float headroom, float* nsat, void* stream);
int dmy_bn_bwd_reduce(int dtype, const void* z, long zps, const void* dy, long dps, const float* scale,
                      const float* shift, const float* mean, const float* invstd, int act, long M, int C, float* pdb,
                      float* pdg, void* stream);
int dmy_bn_bwd_finalize(const float* pdb, const float* pdg, int P, int C, double count, const float* gamma,
                        const float* invstd, float* dgamma, float* dbeta, float* ca, float* cb, float* cc,
                        void* stream);
int dmy_bn_bwd_apply(int dtype, const void* z, long zps, const void* dy, long dps, const float* scale,
                     const float* shift, const float* mean, const float* invstd, int act, const float* ca,
                     const float* cb, const float* cc, void* dz, long dzps, long M, int C, void* stream);
int dmy_reduce_rows(const float* part, int P, int C, float* out, int accumulate, void* stream);
int dmy_bn_reduce_rows(int dtype, const void* z, long zps, const void* dy, long dps, long M, int C);
int dmy_colsum2_rows(long P);
int dmy_colsum2(const float* a, const float* b, long P, int C, float* oa, float* ob, void* stream);

/* ---- memory-bound NHWC ops */
/* nn.MaxPool2d(k, 1, k//2): SPPF common.py:250-258, SPPFCSPC :1266-1274 */
int dmy_maxpool_fwd(int dtype, const void* x, long xps, void* y, long yps, unsigned char* argmax, int N, int H, int W,
                    int C, int k, void* stream);
int dmy_maxpool_bwd(int dtype, const void* dy, long dps, const unsigned char* argmax, void* dx, long dxps,
                    int accumulate, int N, int H, int W, int C, int k, void* stream);
/* inference SPPF / SPPFCSPC pyramid (common.py:250-258, :1266-1274 under no_grad): y1 = pool(x), y2 = pool(y1),
   y3 = pool(y2) in one launch, bit-identical to three dmy_maxpool_fwd calls; k 3 or 5, 16-B vectors, no argmax */
int dmy_maxpool_chain3_fwd(int dtype, const void* x, long xps, void* y1, void* y2, void* y3, long yps, int N, int H,
                           int W, int C, int k, void* stream);
/* nn.AvgPool2d(r, r): SCConv.k2[0] common.py:1282 */
int dmy_avgpool_fwd(int dtype, const void* x, long xps, void* y, int N, int H, int W, int C, int r, void* stream);
int dmy_avgpool_bwd(int dtype, const void* dy, void* dx, long dxps, int accumulate, int N, int H, int W, int C, int r,
                    void* stream);
/* nearest resize: nn.Upsample (yaml head), F.interpolate in SCConv common.py:1311 */
int dmy_resize_fwd(int dtype, const void* x, long xps, void* y, long yps, float yscale, int N, int IH, int IW, int OH,
                   int OW, int C, void* stream);
int dmy_resize_bwd(int dtype, const void* dy, long dps, void* dx, long dxps, int N, int IH, int IW, int OH, int OW,
                   int C, void* stream);
/* torch.cat / AdConcat2/3 fast-normalised weights: common.py:656-664, 994-1026 */
int dmy_slice_copy(int dtype, const void* src, long sps, void* dst, long dps, long M, int C, const float* w, int idx,
                   int nw, float eps, int accumulate, void* stream);
int dmy_dot_partial_blocks(long M, int C);
int dmy_dot_partial(int dtype, const void* a, long aps, const void* b, long bps, long M, int C, float* part,
                    void* stream);
/* BiFPN weighted-concat backward of one input in one pass: dmy_slice_copy(dy -> g, scale, accumulate) and
   dmy_dot_partial(dy, x -> part) reading dy once (16-B vectors; else hipErrorInvalidValue) */
int dmy_slice_copy_dot(int dtype, const void* dy, long dps, void* g, long gps, const void* x, long xps, long M, int C,
                       const float* wv, int idx, int nw, float eps, int accumulate, float* part, void* stream);
int dmy_bifpn_wgrad(const float* part, int nblk, int nw, const float* w, float eps, float* dw, void* stream);
/* SCConv gate k3(x) * sigmoid(x + up(k2(x))): common.py:1311-1314 */
int dmy_scgate_fwd(int dtype, const void* x, long xps, const void* u3, const void* g, void* out, int N, int H, int W,
                   int C, int GH, int GW, void* stream);
int dmy_scgate_bwd(int dtype, const void* x, long xps, const void* u3, const void* g, const void* dout, void* du3,
                   void* dpre, long dpps, int accumulate, int N, int H, int W, int C, int GH, int GW, void* stream);
/* the same gate with k3's BatchNorm (common.py:1296-1300) folded in (bf16): the forward reads k3's pre-BN conv output z
   and applies scale / shift; the backward also writes k3's BN backward-reduce partials, one row per block
   (dmy_scgate_bn_rows rows of C floats each) */
int dmy_scgate_bn_rows(int N, int H, int W, int C);
int dmy_scgate_bn_fwd(const void* x, long xps, const void* z, const float* scale, const float* shift, const void* g,
                      void* out, int N, int H, int W, int C, int GH, int GW, void* stream);
int dmy_scgate_bn_bwd(const void* x, long xps, const void* z, const float* scale, const float* shift,
                      const float* mean, const float* invstd, const void* g, const void* dout, void* du3, void* dpre,
                      int N, int H, int W, int C, int GH, int GW, float* pdb, float* pdg, void* stream);
/* CoorAttention pooling + re-weighting: common.py:1183-1207 */
int dmy_ca_pool_fwd(int dtype, const void* x, long xps, void* y, int N, int H, int W, int C, void* stream);
int dmy_ca_pool_bwd(int dtype, const void* dy, void* dx, long dxps, int accumulate, int N, int H, int W, int C,
                    void* stream);
int dmy_ca_apply_fwd(int dtype, const void* x, long xps, const void* lh, const void* lw, void* out, long ops, int N,
                     int H, int W, int C, void* stream);
int dmy_ca_apply_bwd(int dtype, const void* x, long xps, const void* lh, const void* lw, const void* dout, long dps,
                     void* dx, long dxps, void* dlh, void* dlw, int N, int H, int W, int C, void* stream);
/* input normalisation imgs.float()/255 (train.py:402) + layout changes */
/* NCHW image (uint8 / fp32, even H, W) -> space-to-depth NHWC [N][H/2][W/2][Cs], channel (dy*2+dx)*C+c,
 * times scale (train.py:402 `/255`); the stem conv's input in its k3 s1 form */
int dmy_image_s2d(int dtype, int src_kind, const void* x, void* y, int N, int C, int H, int W, int Cs, float scale,
                  void* stream);
int dmy_nchw_to_nhwc(int dtype, int src_kind, const void* x, void* y, int N, int C, int H, int W, int Cp, float scale,
                     void* stream);
int dmy_nhwc_to_nchw_f32(int dtype, const void* x, long xps, float* y, int N, int C, int H, int W, void* stream);
int dmy_pointwise(int dtype, int op, int act, const void* a, const void* b, void* y, long n, float alpha,
                  void* stream);
int dmy_cast(int src_kind, int dst_kind, const void* x, void* y, long n, float scale, void* stream);

/* ---- Detect decode (models/yolo.py:78-101) and ComputeLoss (utils/loss.py:167-276, metrics.py:192-235) */
int dmy_detect_decode(int dtype, const void* y, long sb, long sh, long sw, int N, int H, int W, int na, int no,
                      float stride, const float* anchors, float* z, long zoff, long ztotal, void* stream);
/* every level of one Detect forward in one launch (yolo.py:63-76 under eval): level l's NHWC head output ys[l] with
   element strides strides[3l .. 3l+2] = (batch, row, col), hw[2l], hw[2l+1] = its H, W, lvl_stride[l] its stride,
   anchors [nl][na][2] (device); z rows of level l start at the sum of the earlier levels' na*H*W.  The bits of one
   dmy_detect_decode per level */
int dmy_detect_decode_levels(int dtype, int nl, const void* const* ys, const long* strides, const int* hw,
                             const float* lvl_stride, int N, int na, int no, const float* anchors, float* z, long ztotal,
                             void* stream);
int dmy_build_targets(const float* targets, int nt, const float* anchors, int na, int H, int W, float anchor_t,
                      int* b, int* a, int* gj, int* gi, int* tcls, float* tbox, float* anch, int* count,
                      void* stream);
/* per level: part = dmy_yolo_loss_part_rows() fp32 block partials (caller-zeroed), G / tobj caller-zeroed;
 * workspaces tgrad [cap][4 + nc] fp32 and links [N*na*H*W + cap] int32 (no float atomics: deterministic) */
int dmy_yolo_loss_part_rows(void);
int dmy_yolo_loss_level(int dtype, const void* p, long sb, long sa, long sh, long sw, int N, int na, int H, int W,
                        int no, int nc, float box_gain, float obj_gain, float cls_gain, float cls_pw, float obj_pw,
                        float cp, float cn, float balance, float bs, const int* b, const int* a, const int* gj,
                        const int* gi, const int* tcls, const float* tbox, const float* anch, const int* count,
                        int cap, float* grad, float* tobj, float* part, float* tgrad, int* links, void* stream);
int dmy_yolo_loss_finalize(const float* part, int nl, float box, float obj, float cls, float bs, float* loss,
                           float* items, void* stream);
int dmy_loss_grad(int dtype, const float* grad, const float* upstream, void* dp, long n, void* stream);
/* SIoU (utils/metrics.py:192-235, bbox_iou(..., x1y1x2y2=False, SIoU=True)) of n xywh pairs through the
 * loss kernel's device function: iou [n] and d iou / d b1 [n][4] (forward-mode duals). */
int dmy_siou_eval(const float* b1, const float* b2, float* iou, float* grad_b1, int n, void* stream);

/* ---- non_max_suppression (utils/general.py:633-725 -> torchvision.ops.nms at :708) */
int dmy_nms_candidates(const float* pred, int nimg, int A, int no, float conf, int multi_label,
                       const unsigned char* class_ok, unsigned long long* keys, long cap, int* counts, void* stream);
int dmy_nms_sort(unsigned long long* keys, long cap, const int* counts, int nimg, void* stream);
/* ncand (nullable): the greedy launch also writes each image's candidate count there and re-zeroes counts[b], so a
   persistent counts buffer is zero for the next dmy_nms_candidates without a fill launch */
int dmy_nms_greedy(const float* pred, int nimg, int A, int no, float iou, int agnostic, int max_det, int max_nms,
                   const unsigned long long* keys, long cap, int* counts, float* boxes, float* out, int* nkeep,
                   int* ncand, void* stream);
/* the same greedy keep set / order through an IoU bitmask (cap <= dmy_nms_mask_rows(); mask: nimg * cap * cap / 64 words;
   boxes is not used: the mask kernel makes each box from its key) */
int dmy_nms_mask_rows(void);
int dmy_nms_greedy_mask(const float* pred, int nimg, int A, int no, float iou, int agnostic, int max_det, int max_nms,
                        const unsigned long long* keys, long cap, int* counts, float* boxes,
                        unsigned long long* mask, float* out, int* nkeep, int* ncand, void* stream);

/* ---- Swin / C3STR (models/common.py:452-654): LayerNorm, shifted-window attention core with the
 *      reference's mask semantics, per-sample DropPath scale (common.py:386-403) */
int dmy_layernorm_fwd(int dtype, const void* x, long xps, const float* w, const float* b, void* y, float* mean,
                      float* rstd, long M, int C, float eps, void* stream);
int dmy_layernorm_bwd_blocks(long M);
int dmy_layernorm_bwd(int dtype, const void* x, long xps, const void* dy, long dps, const float* w, const float* mean,
                      const float* rstd, void* dx, long dxps, int accumulate, long M, int C, float* pdw, float* pdb,
                      void* stream);
int dmy_winattn_fwd(int dtype, const void* qkv, const float* table, void* out, int B, int H, int W, int C, int nh,
                    int shift, float scale, void* stream);
int dmy_winattn_bwd_groups(int B, int H, int W, int nh);
int dmy_winattn_bwd(int dtype, const void* qkv, const void* dout, const float* table, void* dqkv, float* dtab_part,
                    float* dtab, int B, int H, int W, int C, int nh, int shift, float scale, void* stream);
int dmy_sample_scale(int dtype, const void* x, const float* scale, void* y, long per, long n, void* stream);
/* DropPath fused with the residual add of an active SwinTransformerLayer drop_path (common.py:386-403, 621-627): y = x +
 * f * s[b], s[b] = floor(keep + u[b]) / keep on torch's drawn uniforms u [N] (samples = contiguous blocks of `per`
 * elements); _grad: df = dy * s[b]. */
int dmy_droppath_add(int dtype, const void* x, const void* f, const float* u, float keep, void* y, long per, long n,
                     void* stream);
int dmy_droppath_grad(int dtype, const void* dy, const float* u, float keep, void* df, long per, long n, void* stream);

/* ---- optimizer step / EMA (train.py:216-222, 449-454; utils/torch_utils.py:329-339) and the GradScaler
 *      (train.py:354, 445-450).  scale / found: device [1] fp32 loss scale and non-finite flag, or both NULL
 *      (scaler disabled); the update is skipped on the device when *found != 0 (scaler.step). */
int dmy_chunk_size(void);
int dmy_sgd(float* const* p, const float* const* g, float* const* m, const long* n, const int* tid, const long* off,
            int nchunks, float lr, float momentum, float weight_decay, int nesterov, const float* scale,
            const float* found, void* stream);
/* dstep: NULL (bias corrections from the two floats) or the group's device step count before this step: the kernel
 * derives the bias corrections from it and advances it unless the GradScaler skipped the step (as torch's Adam t). */
int dmy_adam(float* const* p, const float* const* g, float* const* m, float* const* v, const long* n, const int* tid,
             const long* off, int nchunks, float lr, float beta1, float beta2, float eps, float weight_decay,
             float bias_corr1, float bias_corr2_sqrt, const float* scale, const float* found, int* dstep,
             void* stream);
/* scaler.unscale_ check: *found = 1 if any g * (1 / *scale) is non-finite (found is not cleared here) */
int dmy_amp_check(const float* const* g, const long* n, const int* tid, const long* off, int nchunks,
                  const float* scale, float* found, void* stream);
/* scaler.update(): backoff / growth of *scale, *gup = *scale * world (the loss's upstream gradient), re-arms found */
int dmy_amp_update(float* scale, float* gup, int* tracker, float* found, float world, float growth, float backoff,
                   int interval, void* stream);
int dmy_ema(float* const* ema, const float* const* src, const long* n, const int* tid, const long* off, int nchunks,
            float decay, void* stream);


/* ---- anchor-free TAL path: replaces models/detect_t.py:38-101 (TDetect outputs, DFL decode),
 *      utils/tal.py:81-221 (ComputeLoss_TAL, BboxLoss, bbox2dist) and utils/tal_assign.py:54-189
 *      (TaskAlignedAssigner); models/common.py:1451-1458 (space_to_depth).  H, W, stride are HOST
 *      arrays of nl entries; box / cls are read through (batch, channel, anchor) element strides. */
long dmy_tal_workspace_bytes(int B, int A, int cap);
int dmy_tal_loss(int dtype, const void* box, long sbb, long sbc, long sba, const void* cls, long scb, long scc, long sca,
                 int B, int nc, int nl, const int* H, const int* W, const float* stride, const float* targets, int nt,
                 float alpha, float beta, float pos_weight, void* workspace, float* G, float* loss, float* items,
                 void* stream);
int dmy_tal_flatten(int dtype, const void* x, long xps, int B, int H, int W, int A, int a0, int no, void* F, int backward,
                    void* stream);
int dmy_tal_detect_out(int dtype, const void* F, int B, int nc, int nl, const int* H, const int* W, const float* stride,
                       float* y, void* stream);
int dmy_space_to_depth(int dtype, const void* x, long xps, void* y, long yps, int N, int H, int W, int C, int backward,
                       void* stream);


/* ---- config-5 modules: CBAM (models/common.py:260-310) channel / spatial attention pieces; SPP
 *      (common.py:212-227) reuses dmy_maxpool_* with k = 3..13. */
/* global avg + max pool (CBAM ChannelAttentionModule avg_pool / max_pool, common.py:266-267):
 * out [2N][C] = (means; maxima), arg [N][C] = first argmax pixel.  ws: dmy_gpool_ws_bytes() of fp32 scratch. */
long dmy_gpool_ws_bytes(int dtype, int N, int HW, int C);
int dmy_gpool_fwd(int dtype, const void* x, long xps, int N, int HW, int C, void* out, int* arg, float* ws,
                  void* stream);
int dmy_gpool_bwd(int dtype, const void* dz, const int* arg, void* dx, long dxps, int accumulate, int N, int HW, int C,
                  void* stream);
int dmy_halves_sigmoid(int dtype, const void* z, int N, int C, void* ca, const void* dca, void* dz, void* stream);
int dmy_cbam_in_fwd(int dtype, const void* x, long xps, const void* ca, int N, int HW, int C, void* out1, void* s2,
                    int* am, void* stream);
long dmy_cbam_in_bwd_ws_elems(int N, int HW, int C);
int dmy_cbam_in_bwd(int dtype, const void* x, long xps, const void* ca, const void* dout1, long dps, const void* ds2,
                    const int* am, int N, int HW, int C, void* dx, long dxps, int accumulate, float* dca, float* ws,
                    void* stream);
int dmy_pixscale(int dtype, const void* out1, const void* sa, long sps, int N, int HW, int C, void* out, long ops,
                 const void* dout, long dps, void* dout1, void* dsa, void* stream);

/* ---- config-5 C3TR (models/common.py:184-189, 312-355): the attention core of the
 *      nn.MultiheadAttention (common.py:323; torch multi_head_attention_forward: softmax(q k^T / sqrt(d)) v
 *      per head, after the in-projection) over the H*W tokens of each image, and the TransformerLayer
 *      nn.Dropout(0.1) (common.py:328).  q/k/v/o are NHWC token rows [B*L][ps], head h = columns
 *      [h d, h d + d); lse2 = fp32 [B][nh][L] (log2-domain log-sum-exp, saved for the backward);
 *      Dq = fp32 workspace [B][nh][L]; dq/dk/dv use the token stride `ops`.  d <= 128; bf16 with
 *      d in {32, 64, 128} runs on MFMA, everything else on the fp32-math generic kernels.
 *      dmy_mha_fwd_ref always runs the generic kernel (test reference for the MFMA path). */
int dmy_mha_fwd(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps, void* o, long ops,
                float* lse2, int B, int L, int nh, int d, float scale, void* stream);
int dmy_mha_fwd_ref(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps, void* o,
                    long ops, float* lse2, int B, int L, int nh, int d, float scale, void* stream);
int dmy_mha_bwd(int dtype, const void* q, long qps, const void* k, long kps, const void* v, long vps, const void* o,
                const void* dout, long ops, const float* lse2, float* Dq, void* dq, void* dk, void* dv, int B, int L,
                int nh, int d, float scale, void* stream);
/* y[m][c] = x[m][c] * (u(*seed, m * C + c) >= p) / (1 - p); the same call with the same seed on dy is the backward.
 * seed is device memory (graph-replay safe); dmy_dropout_seed advances a device generator state and writes a
 * fresh seed (nn.Dropout's per-call RNG draw, common.py:328). */
int dmy_dropout_seed(unsigned long long* state, unsigned long long* seed, void* stream);
int dmy_dropout(int dtype, const void* x, long xps, void* y, long yps, long M, int C, float p,
                const unsigned long long* seed, void* stream);

/* ---- validation matching: replaces process_batch (val.py:62-83) with box_iou (utils/metrics.py:254-276) for
 *      a batch of images in one launch.  det [ND][6] (x1 y1 x2 y2 conf cls), lab [NL][5] (cls x1 y1 x2 y2),
 *      det_off / lab_off [B + 1] per-image row offsets, iouv [T]; workspaces ws_* of ND entries;
 *      correct [ND][T] (0/1).  Matching rules: csrc/metrics.hip header. */
int dmy_process_batch(const float* det, const int* det_off, const float* lab, const int* lab_off, int B,
                      const float* iouv, int T, int* ws_lab, float* ws_iou, int* ws_win, unsigned char* correct,
                      void* stream);

/* ---- training augmentation tail (augment.hip): utils/datasets.py:552-622 after the random draws -- warp
 *      (cv2.warpAffine / warpPerspective INTER_LINEAR, border 114), mixup, augment_hsv, flips, BGR->RGB, HWC->CHW --
 *      for n host-built descriptors (984-byte AugDesc: canvas pointers, inverse maps, mixup ratio, HSV LUTs,
 *      flips; layout in dmayolo/augment.py AUG_DESC) into uint8 out [n, 3, OH, OW]. */
long dmy_aug_desc_bytes(void);
int dmy_augment_batch(const void* descs, int n, void* out, int OH, int OW, void* stream);
/* mosaic canvas composition (utils/datasets.py:680-724 with load_image :659-675's INTER_LINEAR resize): n MosaicDesc
 * (4 decoded images, their host-built resize tables and canvas rectangles; layout in dmayolo/augment.py MOSAIC_DESC,
 * sizeof = dmy_mosaic_desc_bytes) -> each desc's uint8 HWC BGR canvas of S2 x S2 (114 outside the four images). */
long dmy_mosaic_desc_bytes(void);
int dmy_mosaic_compose(const void* descs, int n, int S2, void* stream);

#ifdef __cplusplus
}
#endif
#endif
