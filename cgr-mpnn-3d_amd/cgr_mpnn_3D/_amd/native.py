"""ctypes binding of ``libcgr_mpnn3d.so`` (the C ABI declared in ``include/cgr_mpnn3d.h``).

There is deliberately no fallback: if the shared library is missing or fails to load, every
model call raises.  The library is built in-tree by ``__graft_entry__.build()`` /
``make -C cgr-mpnn-3d_amd/csrc`` into ``cgr_mpnn_3D/_amd/lib/``.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_uint64, c_void_p

_LIB_NAME = "libcgr_mpnn3d.so"
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CGR_MPNN3D_LIB", os.path.join(_HERE, "lib", _LIB_NAME))

ABI_VERSION = 6
TRAIN_DROPOUT, TRAIN_FOR_BACKWARD = 1, 2  # cgr_gnn_forward / _backward `training` bits
MAX_DEPTH = 32
ACT_RELU, ACT_SILU, ACT_GELU = 0, 1, 2
ACT_TANH, ACT_SIGMOID, ACT_ELU, ACT_LEAKY_RELU, ACT_SOFTPLUS, ACT_MISH, ACT_SELU = 3, 4, 5, 6, 7, 8, 9
ACT_NAMES = ("relu", "silu", "gelu", "tanh", "sigmoid", "elu", "leaky_relu", "softplus", "mish",
             "selu")  # index = cgr_activation code (include/cgr_mpnn3d.h)


class CgrGnnConfig(ctypes.Structure):
    _fields_ = [
        ("num_node_features", c_int32),
        ("num_edge_features", c_int32),
        ("hidden", c_int32),
        ("depth", c_int32),
        ("activation", c_int32),
        ("learnable_skip", c_int32),
        ("aggregation", c_int32),
        ("pooling", c_int32),
    ]


class CgrBatch(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p),
        ("edge_index", c_void_p),
        ("edge_attr", c_void_p),
        ("batch", c_void_p),
        ("graph_ptr", c_void_p),
        ("num_nodes", c_int64),
        ("num_edges", c_int64),
        ("num_graphs", c_int64),
    ]


ADAM_GROUP = 32


class CgrAdamTensor(ctypes.Structure):
    _fields_ = [
        ("param", c_void_p),
        ("grad", c_void_p),
        ("exp_avg", c_void_p),
        ("exp_avg_sq", c_void_p),
        ("max_exp_avg_sq", c_void_p),
        ("step", c_void_p),
        ("numel", c_int64),
    ]


# (name, restype, argtypes) of every symbol in include/cgr_mpnn3d.h
SIGNATURES = [
    ("cgr_abi_version", c_int32, []),
    ("cgr_last_error", c_char_p, []),
    ("cgr_gnn_num_params", c_int32, [POINTER(CgrGnnConfig)]),
    ("cgr_gnn_arena_bytes", c_int64, [POINTER(CgrGnnConfig), c_int64, c_int64, c_int64]),
    ("cgr_gnn_workspace_bytes", c_int64, [POINTER(CgrGnnConfig), c_int64, c_int64, c_int64]),
    ("cgr_gnn_arena_offset", c_int64,
     [POINTER(CgrGnnConfig), c_int64, c_int64, c_int64, c_char_p, c_int32]),
    ("cgr_graph_prep", c_int32, [POINTER(CgrGnnConfig), POINTER(CgrBatch), c_void_p, c_void_p]),
    ("cgr_gnn_forward", c_int32,
     [POINTER(CgrGnnConfig), POINTER(c_void_p), POINTER(CgrBatch), POINTER(c_float), c_uint64,
      c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    ("cgr_gnn_backward", c_int32,
     [POINTER(CgrGnnConfig), POINTER(c_void_p), POINTER(CgrBatch), POINTER(c_float), c_uint64,
      c_int32, c_void_p, c_void_p, POINTER(c_void_p), c_void_p, POINTER(c_void_p), c_void_p]),
    ("cgr_gnn_input_grads", c_int32,
     [POINTER(CgrGnnConfig), POINTER(c_void_p), POINTER(CgrBatch), c_void_p, c_void_p, c_void_p,
      c_void_p, c_void_p, c_void_p]),
    ("cgr_gnn_image_bytes", c_int64, [POINTER(CgrGnnConfig)]),
    ("cgr_gnn_pack_images", c_int32, [POINTER(CgrGnnConfig), POINTER(c_void_p), c_void_p,
                                      c_void_p]),
    ("cgr_gnn_predict_arena_bytes", c_int64,
     [POINTER(CgrGnnConfig), c_int64, c_int64, c_int64]),
    ("cgr_gnn_predict", c_int32,
     [POINTER(CgrGnnConfig), POINTER(c_void_p), POINTER(CgrBatch), POINTER(c_float), c_uint64,
      c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("cgr_segment_sum", c_int32,
     [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p]),
    ("cgr_dmpnn_conv_scratch_bytes", c_int64, [c_int64, c_int64, c_int64]),
    ("cgr_dmpnn_conv_forward", c_int32,
     [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
      c_void_p, c_int32, c_void_p]),
    ("cgr_dmpnn_conv_backward", c_int32,
     [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
      c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    ("cgr_adam_step", c_int32,
     [POINTER(CgrAdamTensor), c_int32, c_double, c_double, c_double, c_double, c_double, c_int32,
      c_int32, c_void_p]),
    ("cgr_collate", c_int32,
     [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
      c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
      c_void_p]),
    ("cgr_mse_loss_forward", c_int32,
     [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    ("cgr_mse_loss_backward", c_int32,
     [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    ("cgr_profile_enable", c_int32, [c_int32]),
    ("cgr_profile_collect", c_int32, []),
    ("cgr_profile_reset", None, []),
    ("cgr_profile_report", c_int64, [c_char_p, c_int64]),
    ("cgr_debug_stamps", c_int32, [c_void_p, c_int64]),
    ("cgr_device_errors", c_int32, [c_int32, c_int32]),
    ("cgr_debug_abort_backtrace", c_int32, [c_int32]),
]

DEVERR_UNPAIRED_SEEN, DEVERR_UNPAIRED_TIMEOUT = 4, 16  # cgr_device_errors bits

_lib = None
_load_error: Exception | None = None


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raise RuntimeError if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    try:
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    except OSError as e:  # no silent fallback: the product path needs the HIP library
        _load_error = e
        raise RuntimeError(
            f"cgr_mpnn_3D: native HIP library not loadable ({p}): {e}. Build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` or "
            f"`make -C cgr-mpnn-3d_amd/csrc`.") from e
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.cgr_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"cgr_mpnn_3D: ABI version mismatch (lib {v}, python {ABI_VERSION})")
    _lib = lib
    return lib


def check(rc: int):
    if rc != 0:
        msg = load().cgr_last_error()
        raise RuntimeError(msg.decode() if msg else f"cgr_mpnn_3D native call failed ({rc})")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


_raw_stream = None


def stream_ptr(device) -> int:
    """hipStream_t of ``device``'s current stream.  Read through torch's raw-stream accessor
    (the pointer alone, no Stream object: ~0.3 us instead of ~4 us, three times per training
    step); torch.cuda.current_stream() where that accessor is absent."""
    global _raw_stream
    import torch

    if _raw_stream is None:
        _raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", False)
    idx = getattr(device, "index", device)
    if idx is None:
        idx = torch.cuda.current_device()
    if _raw_stream:
        return _raw_stream(idx)
    return torch.cuda.current_stream(idx).cuda_stream


def device_guard(device):
    """Context making ``device`` the current HIP device around a native call: the C ABI enqueues
    on the stream it is given, but side streams, events and allocations follow the current
    device, so a model on cuda:1 driven while cuda:0 is current must switch first.  A no-op
    context when ``device`` is already current (the common case: no device switch per call)."""
    import contextlib

    import torch

    idx = device.index if isinstance(device, torch.device) else device
    if idx is None or idx == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(device)


def profile_report() -> dict:
    """{kernel class: (launches, total_ms)} accumulated since the last cgr_profile_reset()."""
    lib = load()
    check(lib.cgr_profile_collect())
    n = lib.cgr_profile_report(None, 0)
    buf = ctypes.create_string_buffer(int(n))
    lib.cgr_profile_report(buf, n)
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out


def raise_device_errors(device, clear: bool = True):
    """Raise if a kernel of `device` reported an error condition (cgr_device_errors: pinned host
    memory, no device sync).  Conditions surface once their kernel has run -- at the next native
    call of the model, or right away after a synchronize.  Returns the informational bits."""
    import torch

    idx = device.index if getattr(device, "index", None) is not None else \
        torch.cuda.current_device()
    bits = int(load().cgr_device_errors(int(idx), 1 if clear else 0))
    if bits & DEVERR_UNPAIRED_TIMEOUT:
        raise RuntimeError(
            "cgr_mpnn_3D: the unpaired-edge backward's completion timed out on "
            f"cuda:{idx}; the gradients of that backward are NaN-poisoned (ep_bwd.hpp)")
    return bits
