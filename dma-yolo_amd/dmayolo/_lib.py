"""ctypes binding of the gfx950 C-ABI library (include/dmayolo.h).

The product path has NO fallback: if libdmayolo_hip.so is missing or a symbol is absent the
import fails loudly.  All tensors are passed as raw device pointers + sizes + strides and every
launch is stream-ordered on torch's current HIP stream.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libdmayolo_hip.so')
if os.environ.get('DMY_LIB_AB'):  # kernel A/B tooling only: another in-tree build of the same C ABI, by file name
    LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ['DMY_LIB_AB']))

P, I, L, F, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_double

# name -> argtypes, exactly the header's parameter list (tests/test_abi.py derives both from include/dmayolo.h and
# compares them); the return type is the header's: long for the *_bytes / *_elems queries and the *_bound_rows /
# *_last_rows queries, else int (a hipError_t, or a size for the *_rows / *_blocks / *_groups queries)
SIGNATURES = {
    # conv.hip
    'dmy_conv_fwd_partial_rows': [L, I],
    'dmy_conv_fwd_bound_rows': [L, I],
    'dmy_conv_fwd_last_rows': [],
    'dmy_conv_fwd_bn_rows': [I, P, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L],
    'dmy_conv_fwd': [I, P, P, P, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, P],
    'dmy_conv_dgrad': [I, P, P, P, I, I, I, I, I, L, I, I, I, I, I, I, I, L, P],
    'dmy_conv_wgrad': [I, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, P],
    'dmy_conv_wprep_multi': [I, P, I, P],
    'dmy_conv_wprep_s2d': [I, P, P, I, I, I, P],
    'dmy_conv_wgrad_s2d_to_oihw': [P, P, I, I, I, P],
    'dmy_image_s2d': [I, I, P, P, I, I, I, I, I, F, P],
    'dmy_conv_fwd_act': [I, P, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, P, P, I, P, L, P],
    'dmy_conv_fwd_splitk_elems': [I, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L],
    'dmy_conv_fwd_act_ws': [I, P, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, P, P, I, P, L, P, L, P],
    'dmy_conv_wgrad_ex': [I, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, I, P],
    'dmy_conv_wgrad_ws_elems': [I, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, I],
    'dmy_conv_wgrad_det': [I, P, P, P, I, I, I, I, L, I, I, I, I, I, I, I, L, I, P, L, P],
    'dmy_conv_wprep': [I, P, P, P, I, I, I, I, I, P],
    # bwd1x1.hip
    'dmy_conv1x1_bwd_bn_ok': [L, I, I, L, L, L, P, P, P, P],
    'dmy_conv1x1_bwd_bn': [P, L, P, P, L, P, P, P, P, P, I, P, P, P, P, L, I, P, P, L, L, I, I, P],
    'dmy_conv1x1_bwd_bn_ws_elems': [L, I, I],
    # augment.hip
    'dmy_aug_desc_bytes': [],
    'dmy_augment_batch': [P, I, P, I, I, P],
    'dmy_mosaic_desc_bytes': [],
    'dmy_mosaic_compose': [P, I, I, P],
    'dmy_fp8_quant_ws_elems': [],
    'dmy_fp8_quant': [P, L, I, L, P, P, P],
    'dmy_conv_wprep_fp8': [P, P, P, I, I, I, I, P],
    'dmy_conv_fwd_fp8_partial_rows': [L, I],
    'dmy_conv_fwd_fp8': [P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, L, P, P, I, P, L, P],
    'dmy_conv_wgrad_to_oihw': [P, P, I, I, I, I, I, P],
    # bn.hip
    'dmy_bn_partial_rows': [L],
    'dmy_bn_stats': [I, P, L, L, I, P, P, P],
    'dmy_bn_finalize': [P, P, I, I, D, P, P, P, P, P, F, F, I, P, P, P, P, P],
    'dmy_bn_eval_coef': [P, P, P, P, F, I, P, P, P],
    'dmy_bn_act_fwd': [I, P, L, P, P, I, P, L, P, L, L, I, P],
    'dmy_bn_act_f8_blocks': [],
    'dmy_bn_act_fwd_f8': [P, L, P, P, I, P, L, P, L, L, I, P, P, P, P, F, P, P],
    'dmy_bn_bwd_reduce': [I, P, L, P, L, P, P, P, P, I, L, I, P, P, P],
    'dmy_bn_bwd_finalize': [P, P, I, I, D, P, P, P, P, P, P, P, P],
    'dmy_bn_bwd_apply': [I, P, L, P, L, P, P, P, P, I, P, P, P, P, L, L, I, P],
    'dmy_reduce_rows': [P, I, I, P, I, P],
    'dmy_bn_reduce_rows': [I, P, L, P, L, L, I],
    'dmy_colsum2_rows': [L],
    'dmy_colsum2': [P, P, L, I, P, P, P],
    # eltwise.hip
    'dmy_maxpool_fwd': [I, P, L, P, L, P, I, I, I, I, I, P],
    'dmy_maxpool_chain3_fwd': [I, P, L, P, P, P, L, I, I, I, I, I, P],
    'dmy_maxpool_bwd': [I, P, L, P, P, L, I, I, I, I, I, I, P],
    'dmy_avgpool_fwd': [I, P, L, P, I, I, I, I, I, P],
    'dmy_avgpool_bwd': [I, P, P, L, I, I, I, I, I, I, P],
    'dmy_resize_fwd': [I, P, L, P, L, F, I, I, I, I, I, I, P],
    'dmy_resize_bwd': [I, P, L, P, L, I, I, I, I, I, I, P],
    'dmy_slice_copy': [I, P, L, P, L, L, I, P, I, I, F, I, P],
    'dmy_slice_copy_dot': [I, P, L, P, L, P, L, L, I, P, I, I, F, I, P, P],
    'dmy_dot_partial_blocks': [L, I],
    'dmy_dot_partial': [I, P, L, P, L, L, I, P, P],
    'dmy_bifpn_wgrad': [P, I, I, P, F, P, P],
    'dmy_scgate_fwd': [I, P, L, P, P, P, I, I, I, I, I, I, P],
    'dmy_scgate_bwd': [I, P, L, P, P, P, P, P, L, I, I, I, I, I, I, I, P],
    'dmy_scgate_bn_rows': [I, I, I, I],
    'dmy_scgate_bn_fwd': [P, L, P, P, P, P, P, I, I, I, I, I, I, P],
    'dmy_scgate_bn_bwd': [P, L, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P],
    'dmy_ca_pool_fwd': [I, P, L, P, I, I, I, I, P],
    'dmy_ca_pool_bwd': [I, P, P, L, I, I, I, I, I, P],
    'dmy_ca_apply_fwd': [I, P, L, P, P, P, L, I, I, I, I, P],
    'dmy_ca_apply_bwd': [I, P, L, P, P, P, L, P, L, P, P, I, I, I, I, P],
    'dmy_nchw_to_nhwc': [I, I, P, P, I, I, I, I, I, F, P],
    'dmy_nhwc_to_nchw_f32': [I, P, L, P, I, I, I, I, P],
    'dmy_pointwise': [I, I, I, P, P, P, L, F, P],
    'dmy_cast': [I, I, P, P, L, F, P],
    # detect_loss.hip
    'dmy_detect_decode': [I, P, L, L, L, I, I, I, I, I, F, P, P, L, L, P],
    'dmy_detect_decode_levels': [I, I, P, P, P, P, I, I, I, P, P, L, P],
    'dmy_build_targets': [P, I, P, I, I, I, F, P, P, P, P, P, P, P, P, P],
    'dmy_yolo_loss_part_rows': [],
    'dmy_yolo_loss_level': [I, P, L, L, L, L, I, I, I, I, I, I, F, F, F, F, F, F, F, F, F, P, P, P, P, P, P, P, P,
                            I, P, P, P, P, P, P],
    'dmy_yolo_loss_finalize': [P, I, F, F, F, F, P, P, P],
    'dmy_loss_grad': [I, P, P, P, L, P],
    'dmy_siou_eval': [P, P, P, P, I, P],
    # tal.hip
    'dmy_tal_workspace_bytes': [I, I, I],
    'dmy_tal_loss': [I, P, L, L, L, P, L, L, L, I, I, I, P, P, P, P, I, F, F, F, P, P, P, P, P],
    'dmy_tal_flatten': [I, P, L, I, I, I, I, I, I, P, I, P],
    'dmy_tal_detect_out': [I, P, I, I, I, P, P, P, P, P],
    'dmy_space_to_depth': [I, P, L, P, L, I, I, I, I, I, P],
    'dmy_gpool_ws_bytes': [I, I, I, I],
    'dmy_gpool_fwd': [I, P, L, I, I, I, P, P, P, P],
    'dmy_gpool_bwd': [I, P, P, P, L, I, I, I, I, P],
    'dmy_halves_sigmoid': [I, P, I, I, P, P, P, P],
    'dmy_cbam_in_fwd': [I, P, L, P, I, I, I, P, P, P, P],
    'dmy_cbam_in_bwd_ws_elems': [I, I, I],
    'dmy_cbam_in_bwd': [I, P, L, P, P, L, P, P, I, I, I, P, L, I, P, P, P],
    'dmy_pixscale': [I, P, P, L, I, I, I, P, L, P, L, P, P, P],
    # mha.hip
    'dmy_mha_fwd': [I, P, L, P, L, P, L, P, L, P, I, I, I, I, F, P],
    'dmy_mha_fwd_ref': [I, P, L, P, L, P, L, P, L, P, I, I, I, I, F, P],
    'dmy_mha_bwd': [I, P, L, P, L, P, L, P, P, L, P, P, P, P, P, I, I, I, I, F, P],
    'dmy_dropout_seed': [P, P, P],
    'dmy_dropout': [I, P, L, P, L, L, I, F, P, P],
    # nms.hip
    'dmy_nms_candidates': [P, I, I, I, F, I, P, P, L, P, P],
    'dmy_nms_sort': [P, L, P, I, P],
    'dmy_nms_greedy': [P, I, I, I, F, I, I, I, P, L, P, P, P, P, P, P],
    'dmy_nms_mask_rows': [],
    'dmy_nms_greedy_mask': [P, I, I, I, F, I, I, I, P, L, P, P, P, P, P, P, P],
    # metrics.hip
    'dmy_process_batch': [P, P, P, P, I, P, I, P, P, P, P, P],
    # swin.hip
    'dmy_layernorm_fwd': [I, P, L, P, P, P, P, P, L, I, F, P],
    'dmy_layernorm_bwd_blocks': [L],
    'dmy_layernorm_bwd': [I, P, L, P, L, P, P, P, P, L, I, L, I, P, P, P],
    'dmy_winattn_fwd': [I, P, P, P, I, I, I, I, I, I, F, P],
    'dmy_winattn_bwd_groups': [I, I, I, I],
    'dmy_winattn_bwd': [I, P, P, P, P, P, P, I, I, I, I, I, I, F, P],
    'dmy_sample_scale': [I, P, P, P, L, L, P],
    'dmy_droppath_add': [I, P, P, P, F, P, L, L, P],
    'dmy_droppath_grad': [I, P, P, F, P, L, L, P],
}


# symbols whose argtypes dmayolo/optim.py sets itself (multi-tensor optimizer / GradScaler / EMA kernels)
SELF_BOUND = {'dmy_chunk_size', 'dmy_sgd', 'dmy_adam', 'dmy_ema', 'dmy_amp_check', 'dmy_amp_update'}
LONG_RET = {'dmy_conv_fwd_bound_rows', 'dmy_conv_fwd_last_rows'}


def restype(name):
    return ctypes.c_long if name.endswith(('_bytes', '_elems')) or name in LONG_RET else ctypes.c_int


class LibraryMissing(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(f'{LIB_PATH} not built: run `python -c "import __graft_entry__ as g; g.build()"` '
                             '(the DMA-YOLO HIP path has no CPU fallback)')
    lib = ctypes.CDLL(LIB_PATH)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = stale build: fail loudly
        fn.argtypes = argt
        fn.restype = restype(name)
    return lib


lib = _load()


def call(name, *args):
    rc = getattr(lib, name)(*args)
    if name.endswith(('_rows', '_blocks', '_groups', '_bytes', '_elems', '_ok')):
        return rc
    if rc != 0:
        raise RuntimeError(f'{name} failed with hipError {rc}')
    return rc


_raw_stream = getattr(torch._C, '_cuda_getCurrentRawStream', None)


def stream():
    """torch's current HIP stream on the current device (the raw-pointer query skips the Stream
    object construction, ~10 us of host time per launch)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(torch.cuda.current_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


ACT_NONE, ACT_SILU, ACT_HARDSWISH, ACT_SIGMOID, ACT_GELU, ACT_RELU = 0, 1, 2, 3, 4, 5
