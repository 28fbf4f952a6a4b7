"""ctypes binding of libpn2.so (the C ABI declared in include/pn2.h).

The library is built in-tree for gfx950 (``make -C pointnet-like-pose-estimation_amd/csrc`` or
``__graft_entry__.build()``) and shares torch's HIP runtime: torch is imported first, so the
dynamic loader resolves libpn2's ``libamdhip64.so.7`` to the copy torch already loaded (one
HIP context, torch streams valid in both).

There is no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before libpn2.so: shared HIP runtime)

from . import tuning

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpn2.so")

_i64 = ctypes.c_int64
_int = ctypes.c_int
_vp = ctypes.c_void_p
_dbl = ctypes.c_double


class Pn2Error(RuntimeError):
    """A libpn2 entry point returned an error code (message from pn2_last_error)."""


class MlpLayer(ctypes.Structure):
    _fields_ = [("wt", _vp), ("alpha", _vp), ("beta", _vp), ("cin", _i64), ("cout", _i64),
                ("wt_split", _vp), ("flags", _i64)]


class FpsSide(ctypes.Structure):
    _fields_ = [("pts", _vp), ("B", _i64), ("N", _i64), ("C", _i64), ("sb", _i64), ("sn", _i64), ("sc", _i64),
                ("start_host", _vp), ("S", _i64),
                ("out_idx", _vp), ("out_pts", _vp), ("out_packed", _vp), ("pts_packed", _vp)]


class SaSrc(ctypes.Structure):
    _fields_ = [
        ("mode", _int),
        ("pts", _vp), ("pb", _i64), ("pn", _i64), ("pc", _i64),
        ("feat", _vp), ("fb", _i64), ("fn", _i64),
        ("ctr", _vp),
        ("idx", _vp),
        ("rows", _vp), ("rs", _i64),
        ("B", _i64), ("N", _i64), ("C", _i64), ("D", _i64), ("S", _i64), ("K", _i64),
        ("cnt", _vp),
        ("zero_out", _vp), ("zero_count", _i64),
        ("idx32", _vp),
        ("fps_side", _vp),
    ]


SRC_GROUP_XYZ_FIRST = 0
SRC_GROUP_FEAT_FIRST = 1
SRC_GROUP_ALL = 2
SRC_ROWS = 3
PATH_F32 = 1
PATH_SPLIT_BF16 = 2
PATH_BF16 = 3
LAYER_NO_RELU = 1
LINEAR_RELU = 1
TAIL_LOGSOFTMAX = 1
DEVERR_NO_NEIGHBOUR = 1
DEVERR_INDEX = 2

# name -> (restype, argtypes); every symbol include/pn2.h declares
SIGNATURES = {
    "pn2_abi_version": (_int, []),
    "pn2_last_error": (ctypes.c_char_p, []),
    "pn2_packed_stride": (_i64, [_i64]),
    "pn2_fps_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "pn2_fps_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64]),
    "pn2_fps_ws_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                              _i64, _vp]),
    "pn2_fps_host_ws_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp,
                                   _vp, _i64, _vp]),
    "pn2_pack_points_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp]),
    "pn2_ball_query_f32": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _dbl, _i64, _vp, _vp]),
    "pn2_ball_query_cnt_f32": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _dbl, _i64, _vp, _vp, _vp]),
    "pn2_ball_query_i32": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _dbl, _i64, _vp, _vp, _vp]),
    "pn2_ball_query_multi_i32": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp, _vp]),
    "pn2_square_distance_f32": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "pn2_index_points_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp]),
    "pn2_group_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64,
                             _vp, _i64, _vp, _i64, _int, _vp, _vp]),
    "pn2_layer_cin_pad": (_i64, [_i64]),
    "pn2_pack_layer_f32": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _dbl, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "pn2_layer_split_kblocks": (_i64, [_i64, _i64]),
    "pn2_layer_split_bytes": (_i64, [_i64, _i64, _i64]),
    "pn2_sa_mlp_last_path": (_int, []),
    "pn2_sa_mlp_last_planes": (_int, []),
    "pn2_sa_mlp_last_fps_side": (_int, []),
    "pn2_device_cu_count": (_int, [_int, ctypes.POINTER(_int)]),
    "pn2_stream_create_cu_masked": (_int, [_int, ctypes.POINTER(ctypes.c_uint32), _int, ctypes.POINTER(_vp)]),
    "pn2_stream_destroy": (_int, [_vp]),
    "pn2_bn_train_workspace_bytes": (_i64, [_i64, _i64]),
    "pn2_bn_train_stats_f32": (_int, [_vp, _i64, _i64, _i64, ctypes.c_double, ctypes.c_double, _vp,
                                      _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "pn2_bn_relu_apply_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _int,
                                     _vp]),
    "pn2_bn_train_forward_f32": (_int, [_vp, _i64, _i64, _i64, ctypes.c_double, ctypes.c_double, _vp,
                                        _vp, _vp, _vp, _vp, _i64, _int, _vp, _vp, _vp, _i64, _vp]),
    "pn2_linear_rows_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _int, _vp]),
    "pn2_group_max_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp]),
    "pn2_bn_relu_backward_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                        _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64,
                                        _int, _vp]),
    "pn2_prepare_points_f64": (_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i64, _int, _vp, _i64,
                                      _vp, _vp, _vp]),
    "pn2_pack_layer_split_bf16": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _vp]),
    "pn2_sa_mlp_workspace_bytes": (_i64, [ctypes.POINTER(SaSrc), ctypes.POINTER(MlpLayer), _int]),
    "pn2_sa_mlp_max_f32": (_int, [ctypes.POINTER(SaSrc), ctypes.POINTER(MlpLayer), _int, _int, _vp,
                                  _i64, _vp, _i64, _vp]),
    "pn2_sa_mlp_workspace_bytes_bf16": (_i64, [ctypes.POINTER(SaSrc), ctypes.POINTER(MlpLayer), _int]),
    "pn2_sa_mlp_max_bf16": (_int, [ctypes.POINTER(SaSrc), ctypes.POINTER(MlpLayer), _int, _int, _vp,
                                   _i64, _vp, _i64, _vp]),
    "pn2_tuning_get": (_int, [ctypes.c_char_p, ctypes.POINTER(_i64)]),
    "pn2_tuning_set": (_int, [ctypes.c_char_p, _i64]),
    "pn2_tuning_keys": (ctypes.c_char_p, []),
    "pn2_tuning_local": (_int, [_int]),
    "pn2_device_errors": (_int, [_int, ctypes.POINTER(ctypes.c_uint32)]),
    "pn2_error_slot_set": (_int, [_vp]),
    "pn2_error_slot_take": (_int, [_int, ctypes.POINTER(ctypes.c_uint32), _vp]),
    "pn2_tuning_default": (_int, [ctypes.c_char_p, ctypes.POINTER(_i64)]),
    "pn2_fc_tail_workspace_bytes": (_i64, [_i64, _i64, _i64]),
    "pn2_fc_tail_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64,
                               _int, _vp, _i64, _vp, _vp, _i64, _vp]),
}

ABI_VERSION = 17
_lib = None


def load():
    """Load libpn2.so (once).  Raises if it is missing or incompatible -- no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "pn2: %s is not built; run `make -C pointnet-like-pose-estimation_amd/csrc` "
            "(or __graft_entry__.build())" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.pn2_abi_version() != ABI_VERSION:
        raise ImportError("pn2: libpn2.so ABI %d != expected %d" % (L.pn2_abi_version(), ABI_VERSION))
    tuning.apply_env(L)
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = load().pn2_last_error().decode(errors="replace")
        raise Pn2Error("%s failed (code %d): %s" % (what, rc, msg))


# ------------------------------------------------------------------ device error slots
# Each (host thread, device) pair gets its own two-word slot (include/pn2.h pn2_error_slot_set),
# so a thread's check_device_errors() sees, and clears, only the bits its own launches raised
# (the reference's mutilthreading/predict_test.py:44-63 runs heads on four threads at once).
# Slots are never freed: a captured graph keeps raising into its capturing thread's slot.
_slots_tls = threading.local()
_slots_keep = []
_slots_lock = threading.Lock()


def bind_error_slot(device):
    """Make `device`'s launches from this thread raise into this thread's own slot (idempotent:
    a dict lookup after the first call).  While a stream capture is running no slot can be
    allocated: the thread then keeps the process-wide default slot until its next call."""
    idx = device.index if isinstance(device, torch.device) else int(device)
    if idx is None:
        idx = torch.cuda.current_device()
    bound = getattr(_slots_tls, "slots", None)
    if bound is None:
        bound = _slots_tls.slots = {}
    slot = bound.get(idx)
    if slot is not None:
        return slot
    if torch.cuda.is_current_stream_capturing():
        return None
    slot = torch.zeros(2, dtype=torch.int32, device="cuda:%d" % idx)
    torch.cuda.current_stream(idx).synchronize()  # zeroed before any kernel may raise into it
    with _slots_lock:
        _slots_keep.append(slot)
    with torch.cuda.device(idx):
        check(load().pn2_error_slot_set(slot.data_ptr()), "pn2_error_slot_set")
    bound[idx] = slot
    return slot


def device_errors(device=None, clear=True):
    """This thread's device error bits (DEVERR_*) on `device` after the device's queued work,
    cleared unless clear=False (include/pn2.h pn2_error_slot_take)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    bind_error_slot(dev)
    torch.cuda.synchronize(dev)  # every stream: this thread's launches may be on any of them
    bits = ctypes.c_uint32(0)
    with torch.cuda.device(dev):
        check(load().pn2_error_slot_take(1 if clear else 0, ctypes.byref(bits),
                                         torch.cuda.current_stream(dev).cuda_stream),
              "pn2_error_slot_take")
    return bits.value


def check_device_errors(device=None):
    """Raise IndexError -- what the reference raises -- when a kernel met an index the reference
    would have rejected since the last check (a ball-query centroid with no neighbour in its
    radius, or an out-of-range index_points / grouping index); clears the word."""
    bits = device_errors(device)
    if bits & DEVERR_NO_NEIGHBOUR:
        raise IndexError("pn2: a query_ball_point centroid had no point within its radius; its "
                         "group is padded with index N, which the reference's index_points "
                         "rejects (pointnet2_utils.py:85-89, 44)")
    if bits & DEVERR_INDEX:
        raise IndexError("pn2: index_points / grouping index out of range [-N, N)")


def stream_ptr(device):
    """hipStream_t of torch's current stream on `device`, as an int for ctypes (and this
    thread's device error slot bound first: every launch goes through here or ops._stream)."""
    bind_error_slot(device)
    return torch.cuda.current_stream(device).cuda_stream
