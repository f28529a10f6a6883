"""Locating and loading the in-tree native artefacts (vgpu/_lib).

The kernels library must be loaded AFTER torch so that its NEEDED
libamdhip64.so.7 binds to the HIP runtime PyTorch already loaded (same SONAME)
instead of pulling in a second runtime.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parents[1] / "_lib"
FAKES_DIR = LIB_DIR / "fakes"


class NativeMissing(RuntimeError):
    pass


def lib_path(name: str) -> Path:
    return LIB_DIR / name


def shim_path() -> Path:
    return lib_path("libvgpu.so")


def ensure_built(kernels: bool = True) -> None:
    """Build whatever is missing (hipcc/g++ are in the image on the GPU box too)."""
    need = not shim_path().exists() or (kernels and not lib_path("libvgpu_kernels.so").exists())
    if need:
        from . import build
        build.build_all(kernels=kernels)


_kernels = None
_capi = None


def load_kernels() -> ctypes.CDLL:
    """Load libvgpu_kernels.so; raises NativeMissing (never falls back)."""
    global _kernels
    if _kernels is not None:
        return _kernels
    import torch  # noqa: F401  (must precede: bind to torch's HIP runtime)
    p = lib_path("libvgpu_kernels.so")
    if not p.exists():
        raise NativeMissing(f"{p} not built: run `python -m vgpu.native.build kernels`")
    lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    vp, u32, u64, i64p = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
    lib.vgpu_census.argtypes = [vp, u32, u64, vp, vp]
    lib.vgpu_busy.argtypes = [vp, u32, u32, vp]
    lib.vgpu_busy_via.argtypes = [vp, u32, u32, vp, ctypes.c_int]
    lib.vgpu_gather_pages.argtypes = [vp, vp, i64p, u64, u64, vp]
    lib.vgpu_scatter_pages.argtypes = [vp, vp, i64p, u64, u64, vp]
    lib.vgpu_fill_pattern.argtypes = [vp, u64, u32, vp]
    lib.vgpu_verify_pattern.argtypes = [vp, u64, u32, vp, vp]
    lib.vgpu_bias_act_nhwc.argtypes = [vp, vp, u64, u32, ctypes.c_int, vp]
    lib.vgpu_scale_shift_act_nhwc.argtypes = [vp, vp, vp, vp, u64, u32, ctypes.c_int, vp]
    lib.vgpu_add_scale_shift_act_nhwc.argtypes = [vp, vp, vp, vp, vp, vp, u64, u32, ctypes.c_int, vp]
    lib.vgpu_relu_bias_grad_workspace.argtypes = [u64, u32]
    lib.vgpu_relu_bias_grad_workspace.restype = ctypes.c_int64
    lib.vgpu_relu_bias_grad_nhwc.argtypes = [vp, vp, vp, vp, vp, u64, u32, ctypes.c_int, vp]
    lib.vgpu_relu_bias_grad_nhwc.restype = ctypes.c_int
    lib.vgpu_pool_relu_bias_grad_nhwc.argtypes = [vp] * 6 + [ctypes.c_int] * 3 + [u32, ctypes.c_int, ctypes.c_int, vp]
    lib.vgpu_pool_relu_bias_grad_nhwc.restype = ctypes.c_int
    lib.vgpu_relu_bias_grad_partial_nhwc.argtypes = [vp] * 5 + [ctypes.c_int] * 3 + [u32, ctypes.c_int, vp, vp]
    lib.vgpu_relu_bias_grad_partial_nhwc.restype = ctypes.c_int
    lib.vgpu_conv_wgrad_db_nhwc.argtypes = [vp] * 4 + [ctypes.c_int64] + [ctypes.c_int] * 8 + [vp] + \
        [ctypes.c_int] * 2 + [vp, ctypes.c_int, ctypes.c_int, vp]
    lib.vgpu_conv_wgrad_db_nhwc.restype = ctypes.c_int
    lib.vgpu_bias_grad_reduce.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, vp]
    lib.vgpu_conv2d_masked_splitk.argtypes = [vp] * 3 + [ctypes.c_int] * 7 + [vp, vp, ctypes.c_int64, vp,
                                                                            ctypes.c_int64, vp, vp]
    lib.vgpu_conv2d_masked_splitk.restype = ctypes.c_int
    lib.vgpu_conv2d_masked_pool_splitk.argtypes = [vp, vp] + [ctypes.c_int] * 7 + [vp, ctypes.c_int, vp, vp, vp,
                                                                                  ctypes.c_int64, vp, ctypes.c_int64,
                                                                                  vp, vp]
    lib.vgpu_conv2d_masked_pool_splitk.restype = ctypes.c_int
    lib.vgpu_bias_grad_reduce.restype = ctypes.c_int
    lib.vgpu_pad_channels.argtypes = [vp, vp, u64, u32, u32, vp]
    lib.vgpu_pad_channels.restype = ctypes.c_int
    ci = ctypes.c_int
    lib.vgpu_conv2d_nhwc.argtypes = [vp, vp, vp, vp, vp, vp, vp] + [ci] * 9 + [vp]
    lib.vgpu_conv2d_nhwc_ws.argtypes = [vp, vp, vp, vp, vp, vp, vp] + [ci] * 9 + [vp, ctypes.c_int64, vp]
    lib.vgpu_conv2d_nhwc_ws.restype = ci
    lib.vgpu_conv2d_workspace.argtypes = [ci] * 9
    lib.vgpu_conv2d_workspace.restype = ctypes.c_int64
    lib.vgpu_conv_set_splitk.argtypes = [ci]
    lib.vgpu_maxpool_nhwc.argtypes = [vp, vp] + [ci] * 7 + [vp]
    lib.vgpu_stem_pool_nhwc.argtypes = [vp, vp, vp] + [ci] * 3 + [vp]
    lib.vgpu_conv_set_big.argtypes = [ci]
    lib.vgpu_conv_set_halo.argtypes = [ci]
    lib.vgpu_conv_halo_launches.restype = ctypes.c_ulonglong
    lib.vgpu_lstm_recurrence.argtypes = [vp, vp, vp, vp, ci, ci, ci, vp]
    lib.vgpu_lstm_recurrence.restype = ci
    lib.vgpu_lstm_forward_train.argtypes = [vp] * 5 + [ci, ci, ci, vp]
    lib.vgpu_lstm_forward_train.restype = ci
    lib.vgpu_lstm_backward.argtypes = [vp] * 5 + [ci, ci, ci, vp]
    lib.vgpu_lstm_backward.restype = ci
    i64 = ctypes.c_int64
    lib.vgpu_lstm_recurrence_window.argtypes = [vp, vp, vp, i64, i64, vp, vp, ci, vp, vp, ci, ci, ci, vp, vp]
    lib.vgpu_lstm_recurrence_window.restype = ci
    lib.vgpu_lstm_backward_window.argtypes = [vp, vp, vp, i64, i64, vp, vp, vp, vp, ci, ci, ci, ci, vp]
    lib.vgpu_lstm_backward_window.restype = ci
    lib.vgpu_lstm2_forward.argtypes = [vp] * 14 + [ci, ci, ci, vp]
    lib.vgpu_lstm2_forward.restype = ci
    lib.vgpu_lstm2_backward.argtypes = [vp] * 12 + [ci, ci, ci, vp]
    lib.vgpu_lstm2_backward.restype = ci
    lib.vgpu_lstm2_flags_error.argtypes = [vp, ci]
    lib.vgpu_lstm2_flags_error.restype = ci
    lib.vgpu_scale_shift_relu_mean_nhwc.argtypes = [vp, vp, vp, vp, ci, ci, ci, vp]
    i64, cf = ctypes.c_int64, ctypes.c_float
    lib.vgpu_bn_workspace.argtypes = [i64, ci]
    lib.vgpu_bn_workspace.restype = i64
    lib.vgpu_bn_act_fwd_train.argtypes = [vp] * 9 + [i64, ci, cf, cf, ci, ci, vp]
    lib.vgpu_bn_act_fwd_train_add.argtypes = [vp] * 9 + [i64, ci, cf, cf, ci, ci, vp, vp]
    lib.vgpu_bn_act_bwd.argtypes = [vp] * 10 + [i64, ci, ci, ci, vp]
    lib.vgpu_bn_act_bwd_add.argtypes = [vp] * 10 + [i64, ci, ci, ci, vp, vp]
    lib.vgpu_bn_act_bwd_add.restype = ci
    lib.vgpu_bn_set_tuning.argtypes = [ci, ci]
    lib.vgpu_bn_set_fuse_small.argtypes = [ci]
    lib.vgpu_maxpool_fwd_idx_nhwc.argtypes = [vp, vp, vp] + [ci] * 7 + [vp]
    lib.vgpu_maxpool_fwd_idx_nhwc.restype = ci
    lib.vgpu_maxpool_fwd_idx_nchw_out.argtypes = [vp, vp, vp] + [ci] * 7 + [vp]
    lib.vgpu_maxpool_fwd_idx_nchw_out.restype = ci
    lib.vgpu_relu_bias_grad_partial2.argtypes = [vp] * 5 + [ci] * 3 + [u32, ci, ci, vp, vp]
    lib.vgpu_relu_bias_grad_partial2.restype = ci
    lib.vgpu_maxpool_bwd_nhwc.argtypes = [vp, vp, vp] + [ci] * 7 + [vp]
    lib.vgpu_maxpool_bwd_nhwc.restype = ci
    # BatchNorm statistics from the conv epilogue (vgpu.ops.bnconv)
    lib.vgpu_conv2d_nhwc_bn.argtypes = [vp] * 4 + [ci] * 8 + [vp, vp, vp, ci, ci, vp]
    lib.vgpu_conv2d_nhwc_bn.restype = ci
    lib.vgpu_bn_act_fwd_partials.argtypes = [vp, i64] + [vp] * 7 + [i64, ci, cf, cf, ci, ci, vp]
    lib.vgpu_bn_act_fwd_partials.restype = ci
    lib.vgpu_bn_act_fwd_train_coef.argtypes = [vp] * 8 + [i64, ci, cf, cf, ci, ci, vp]
    lib.vgpu_bn_act_fwd_train_coef.restype = ci
    lib.vgpu_bn_bwd_partials.argtypes = [vp, i64] + [vp] * 10 + [i64, ci, ci, vp, vp]
    lib.vgpu_bn_bwd_partials.restype = ci
    lib.vgpu_conv_wgrad_workspace.argtypes = [ci] * 8
    lib.vgpu_conv_wgrad_workspace.restype = i64
    lib.vgpu_conv_wgrad_nhwc.argtypes = [vp] * 4 + [i64] + [ci] * 8 + [vp]
    lib.vgpu_conv_wgrad_nhwc.restype = ci
    lib.vgpu_wt_flip_tiles.argtypes = [ci, ci, ci]
    lib.vgpu_wt_flip_tiles.restype = ci
    lib.vgpu_wt_flip_batched.argtypes = [vp, ci, ci, vp]
    lib.vgpu_wt_flip_batched.restype = ci
    lib.vgpu_wt_desc_size.restype = ci
    for f in ("vgpu_bn_act_fwd_train", "vgpu_bn_act_bwd","vgpu_census", "vgpu_busy", "vgpu_busy_via", "vgpu_gather_pages", "vgpu_scatter_pages",
              "vgpu_fill_pattern", "vgpu_verify_pattern", "vgpu_kernels_abi_version",
              "vgpu_bias_act_nhwc", "vgpu_scale_shift_act_nhwc", "vgpu_add_scale_shift_act_nhwc",
              "vgpu_conv2d_nhwc", "vgpu_maxpool_nhwc", "vgpu_stem_pool_nhwc",
              "vgpu_scale_shift_relu_mean_nhwc"):
        getattr(lib, f).restype = ctypes.c_int
    _kernels = lib
    return lib


class RegionLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "region_size", "proc_slot_size", "dev_usage_size", "device_cfg_size", "off_lock",
        "off_num_devices", "off_recent_kernel", "off_dev", "off_procs", "mutex_size")]


def load_capi() -> ctypes.CDLL:
    """libvgpu.so's C ABI (region attach/lock/feedback) for the node monitor and tests.
    Loading it into a process without HIP is harmless: hooks stay dormant."""
    global _capi
    if _capi is not None:
        return _capi
    p = shim_path()
    if not p.exists():
        raise NativeMissing(f"{p} not built: run `python -m vgpu.native.build shim`")
    lib = ctypes.CDLL(str(p))
    vp, ci, cu64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
    lib.vgpu_region_layout.argtypes = [ctypes.POINTER(RegionLayout)]
    lib.vgpu_region_create.argtypes = [ctypes.c_char_p]
    lib.vgpu_region_create.restype = vp
    lib.vgpu_region_attach.argtypes = [ctypes.c_char_p]
    lib.vgpu_region_attach.restype = vp
    lib.vgpu_region_detach.argtypes = [vp]
    lib.vgpu_region_lock.argtypes = [vp]
    lib.vgpu_region_unlock.argtypes = [vp]
    lib.vgpu_region_purge.argtypes = [vp, ci]
    lib.vgpu_region_claim.argtypes = [vp, ci, ci, ci]
    lib.vgpu_region_release.argtypes = [vp, ci]
    lib.vgpu_region_device_used.argtypes = [vp, ci]
    lib.vgpu_region_device_used.restype = cu64
    lib.vgpu_region_set_feedback.argtypes = [vp, ci, ci, ci]
    lib.vgpu_region_decay_recent.argtypes = [vp]
    lib.vgpu_region_set_cu_mask.argtypes = [vp, ci, ctypes.POINTER(ctypes.c_uint64)]
    lib.vgpu_region_signal_all.argtypes = [vp, ci, ci]
    lib.vgpu_region_set_host_pid.argtypes = [vp, ci, ci, ci, ci]
    lib.vgpu_parse_mem.argtypes = [ctypes.c_char_p]
    lib.vgpu_parse_mem.restype = cu64
    lib.vgpu_parse_cu_mask.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64), ci]
    _capi = lib
    return lib


def region_layout() -> dict[str, int]:
    lib = load_capi()
    lay = RegionLayout()
    lib.vgpu_region_layout(ctypes.byref(lay))
    return {n: getattr(lay, n) for n, _ in RegionLayout._fields_}


def preload_env(base: dict[str, str] | None = None) -> dict[str, str]:
    """Environment for a child process running under the enforcement library."""
    env = dict(os.environ if base is None else base)
    cur = env.get("LD_PRELOAD", "")
    sp = str(shim_path())
    if sp not in cur.split():
        env["LD_PRELOAD"] = (sp + " " + cur).strip()
    return env
