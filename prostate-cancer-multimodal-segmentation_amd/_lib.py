"""ctypes binding of libpcms_hip.so (the C ABI declared in include/pcms_hip.h).

There is no fallback: if the library is missing or a call fails, this raises.  Tensors are
passed as raw device pointers; every call is enqueued on the current torch stream.
"""
from __future__ import annotations

import ctypes
import os

import torch

LIB_PATH = os.environ.get("PCMS_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpcms_hip.so")

F32, BF16, F32X3 = 0, 1, 2  # F32X3: conv3 entry points only (fp32 data, bf16x3 arithmetic)

# name -> argument codes: i int32, l int64, d double, f float, p pointer, s hipStream_t
SIGNATURES = {
    "pcms_pack_input": "ippiilis",
    "pcms_conv3_chunk": "i",
    "pcms_conv3_pack_elems": "iii",
    "pcms_conv3_mblocks": "iiii",
    "pcms_conv3_fwd_rows": "iiiiiiii",
    "pcms_conv3_big_min_boxes": "i",
    "pcms_conv3_big_max_wgs": "i",
    "pcms_conv3_fwd_box_vol": "i",
    "pcms_conv3_small_box_mtw2": "i",
    "pcms_conv3_pack": "ippiiis",
    "pcms_conv3_pack2": "ipppiis",
    "pcms_conv3_splits": "iii",
    "pcms_conv3_fwd": "ipipippppippiiiiiiis",
    "pcms_conv3_fwd_bnin": "ipi" + "p" * 6 + "iiiii" + "s",
    "pcms_conv3_wgrad_bnin": "ipi" + "p" * 5 + "i" * 8 + "s",
    "pcms_conv3_bnin_ok": "iiiiiii",
    "pcms_conv3_wgrad_ws_floats": "iiiiiiiii",
    "pcms_conv3_wgrad": "ipipipppiiiiiiiis",
    "pcms_conv3_wgrad_tg_maxbox": "i",
    "pcms_conv3_wgrad_k16": "i",
    "pcms_conv3_wgrad_x6_dma": "i",
    "pcms_conv3_wgrad_reduce_fused": "i",
    "pcms_conv3_big16_ok": "iiiiiii",
    "pcms_conv3_fwd16_rows": "iiiiiii",
    "pcms_conv3_b16_nt8": "i",
    "pcms_conv3_fwd16_split_ok": "iiiiiii",
    "pcms_conv3_fwd16_split": "pipippiiiiiis",
    "pcms_conv3_pack16_elems": "ii",
    "pcms_conv3_pack16": "piis",
    "pcms_conv3_fwd16": "pipippppppipiiiiiis",
    "pcms_stem_pack_elems": "",
    "pcms_stem_wgrad_dense": "i",
    "pcms_stem_pack": "ppis",
    "pcms_stem_supported": "iiii",
    "pcms_stem_fwd_rows": "iiii",
    "pcms_stem_fwd": "pppppiiiiis",
    "pcms_stem_wgrad_ws_floats": "iiiii",
    "pcms_stem_wgrad": "ppppiiiiis",
    "pcms_stem_wgrad_bn": "ppppppppppiiiiis",
    "pcms_split_epilogue_rows": "l",
    "pcms_split_epilogue": "ipipppipilis",
    "pcms_bn_ws_doubles": "i",
    "pcms_bn_finalize": "piidpppppffppppps",
    "pcms_bn_eval_coeffs": "ppppfipps",
    "pcms_bn_fold": "ppppppfilpps",
    "pcms_bn_relu": "ippppils",
    "pcms_bn_bwd_rows": "iil",
    "pcms_bn_relu_bwd": "i" + "p" * 12 + "ilps",
    "pcms_maxpool_fwd": "ippiiiiis",
    "pcms_maxpool_bwd": "ipppiiiiis",
    "pcms_bn_relu_pool": "ipppppiiiiis",
    "pcms_maxpool_bwd_bn_rows": "iiiiii",
    "pcms_maxpool_bwd_bn": "ippppppppiiiiis",
    "pcms_maxpool_bwd_bn_sums": "ippppppppiiiiis",
    "pcms_maxpool_bn_apply": "ipppppppppiiiiis",
    "pcms_bn_relu_bwd_finish": "i" + "p" * 8 + "ippppilps",
    "pcms_convt_pack": "ippiiis",
    "pcms_convt_pack_elems": "iii",
    "pcms_convt_fwd_stream": "i",
    "pcms_convt_fwd": "ippppiiiiiiiiis",
    "pcms_convt_fwd_ws_floats": "iiiiii",
    "pcms_convt_fwd_ws": "ipppppiiiiiiiiis",
    "pcms_convt_dgrad": "ipppiiiiiiiiis",
    "pcms_convt_dgrad_ws_floats": "iiiiii",
    "pcms_convt_dgrad_ws": "ippppiiiiiiiiis",
    "pcms_convt_wgrad_ws_floats": "iiiiiii",
    "pcms_convt_wgrad_taps": "i",
    "pcms_convt_reduce_fused": "i",
    "pcms_bn_bwd_rows_cap": "i",
    "pcms_convt_wgrad": "ippppiiiiiiiiiis",
    "pcms_convt_wgrad_bias_ws_floats": "iiiiiiii",
    "pcms_convt_wgrad_bias": "ippppppiiiiiiiiiis",
    "pcms_box_channel_sum_ws_floats": "iiiiii",
    "pcms_box_channel_sum": "ipppiiiiiiiiiiis",
    "pcms_head_fwd": "ippppliiifs",
    "pcms_head_bwd_ws_floats": "lii",
    "pcms_head_bwd": "ipppppppliis",
    "pcms_head_bn_fwd": "ippppppliiifs",
    "pcms_head_bn_bwd_rows": "li",
    "pcms_head_bn_bwd": "i" + "p" * 16 + "liips",
    "pcms_loss_rows": "l",
    "pcms_loss_fwd": "pplfffppps",
    "pcms_loss_bwd": "pplpfffpps",
    "pcms_adam": "pppplfffffffps",
    "pcms_adam_pack_conv3": "pppppiifffffffps",
    "pcms_adam_pack_convt": "pppppiifffffffps",
    "pcms_adam_pack_conv3_x6": "pppppiifffffffps",
    "pcms_adam_pack_convt_x6": "pppppiifffffffps",
    "pcms_adam_ranges": "pppppilfffffffps",
    "pcms_grad_clip_ws_doubles": "",
    "pcms_fill_ranges": "ppilfs",
    "pcms_grad_clip": "plffippps",
    "pcms_add": "ippls",
    "pcms_unpack_output": "ippiiils",
    "pcms_clock_probe": "pis",
    "pcms_clock_spin": "pils",
}

_CT = {"i": ctypes.c_int, "l": ctypes.c_long, "d": ctypes.c_double, "f": ctypes.c_float,
       "p": ctypes.c_void_p, "s": ctypes.c_void_p}

_lib = None


class HipError(RuntimeError):
    pass


def load():
    """Load the HIP library; raises (never falls back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). pcms_amd has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, sig in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = [_CT[c] for c in sig]
        fn.restype = ctypes.c_int
    _lib = lib
    return lib


def exported_symbols():
    return list(SIGNATURES)


def ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def call(name: str, *args):
    """Call ``name`` with tensors/None/ints/floats; appends the current stream."""
    lib = load()
    conv = []
    sig = SIGNATURES[name]
    for code, a in zip(sig, args):
        if code == "p":
            conv.append(ptr(a))
        else:
            conv.append(a)
    if sig.endswith("s"):
        conv.append(stream())
    rc = getattr(lib, name)(*conv)
    if rc != 0 and sig.endswith("s"):
        raise HipError(f"{name} failed with status {rc}")
    return rc


def query(name: str, *args) -> int:
    """Host-only helpers (no stream): sizes / counts."""
    return getattr(load(), name)(*args)
