"""ctypes binding of the C ABI declared in include/rae.h (librae_hip.so).

The product path has no CPU fallback: if the HIP library is missing or a call fails, an
exception is raised.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "librae_hip.so"
LIB_PATH = os.path.join(_HERE, LIB_NAME)
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "rae.h")
# hipcc flags of the in-tree build (__graft_entry__.build); part of the build id
BUILD_FLAGS = ("-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared", "-Wall",
               "-Wno-unused-parameter", "-Wno-unused-variable")


def source_files():
    """The sources librae_hip.so is built from: csrc/*.hip, csrc/*.hpp and include/rae.h."""
    if not os.path.isdir(CSRC):
        return []
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
            if f.endswith((".hip", ".hpp"))] + [HEADER]


def source_build_id():
    """sha256 (16 hex digits) over the build flags and the sources' names and bytes; None
    when the sources are not next to the package.  build() compiles it into the library
    (rae_build_id()) and load() refuses a library whose id differs."""
    files = source_files()
    if not files or not all(os.path.exists(f) for f in files):
        return None
    h = hashlib.sha256(" ".join(BUILD_FLAGS).encode())
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def library_build_id(path=LIB_PATH):
    """The build id compiled into a built library, read from the file's bytes (a marker
    string rae.hip embeds) rather than by dlopen: a library already loaded in this process
    would shadow a rebuilt file of the same path.  None if absent."""
    try:
        with open(path, "rb") as fh:
            blob = fh.read()
    except OSError:
        return None
    i = blob.find(b"RAE_BUILD_ID:")
    if i < 0:
        return None
    j = blob.find(b"\0", i)
    return blob[i + len(b"RAE_BUILD_ID:"):j].decode(errors="replace")

RAE_OK = 0
RAE_DEC = {"sp": 0, "rescal": 1, "rescal+sp": 2}
RAE_OPT = {"adagrad": 0, "sgd": 1}
RAE_NEG_PER_CALL = 0
RAE_NEG_PER_EPOCH = 1

# Every symbol include/rae.h declares (checked by tests/test_abi.py against the header).
EXPORTS = (
    "rae_plan_create", "rae_plan_destroy", "rae_last_error", "rae_version", "rae_build_id",
    "rae_exchange_record_floats", "rae_exchange_floats", "rae_set_negatives",
    "rae_set_cursor", "rae_advance_cursor", "rae_cursor_moves", "rae_step_forward",
    "rae_step_update", "rae_step_forward_at", "rae_step_update_at",
    "rae_train_step", "rae_check", "rae_check_on", "rae_label", "rae_build_index", "rae_index_window",
    "rae_neg_sample", "rae_neg_sample_philox",
    "rae_time_next", "rae_event_create", "rae_event_destroy", "rae_event_elapsed_ms",
    "rae_stream_copy", "rae_mfma_probe", "rae_plan_forms",
    "rae_dp_block_floats", "rae_set_dp_buffers", "rae_dp_list_max", "rae_dp_pack",
    "rae_dp_unpack", "rae_dp_pack_at", "rae_dp_unpack_at",
    "rae_ipc_export", "rae_ipc_open", "rae_ipc_close", "rae_p2p_signals", "rae_set_peer",
    "rae_set_p2p_timeout", "rae_p2p_prologue",
)
RAE_IPC_HANDLE_BYTES = 64


class RaeConfig(C.Structure):
    _fields_ = [
        ("decoder", C.c_int32), ("optimizer", C.c_int32),
        ("n_examples", C.c_int64), ("n_features", C.c_int64), ("n_entities", C.c_int64),
        ("relations", C.c_int32), ("embed", C.c_int32), ("neg_samples", C.c_int32),
        ("batch_size", C.c_int32), ("world_size", C.c_int32), ("rank", C.c_int32),
        ("learning_rate", C.c_float), ("alpha", C.c_float), ("lambda1", C.c_float),
        ("lambda2", C.c_float), ("ext_reg", C.c_int32), ("max_batch_nnz", C.c_int32),
        ("max_row_nnz", C.c_int32), ("neg_mode", C.c_int32), ("neg_stride", C.c_int64),
        ("index_window", C.c_int64), ("mfma_bf16", C.c_int32),
        ("sp_forward", C.c_int32), ("bil_dp", C.c_int32), ("bil_prep", C.c_int32),
        ("dp_update", C.c_int32), ("priv_rows", C.c_int32), ("dp_dense", C.c_int32),
        ("heavy_chunk", C.c_int32), ("dp_xchg", C.c_int32),
    ]


# kernel forms (include/rae.h RAE_SPFWD_* / RAE_BILDP_* / RAE_BILPREP_* / RAE_DPUPD_*)
KERNEL_FORMS = {
    "sp_forward": {"auto": 0, "fused": 1, "split": 2},
    "bil_dp": {"auto": 0, "strided": 1, "staged": 2, "mtile": 3},
    "bil_prep": {"auto": 0, "kernel": 1},
    "dp_update": {"replicated": 0, "partitioned": 1},
    "priv_rows": {"auto": 0, "off": 1, "on": 2},
    "dp_dense": {"auto": 0, "records": 1, "partials": 2},
    "heavy_chunk": {"auto": 0, "off": 1, "on": 2},
    "dp_xchg": {"collective": 0, "p2p": 1, "p2p_pipe": 2},
}


_P = C.c_void_p


class RaeBuffers(C.Structure):
    _fields_ = [
        ("W", _P), ("Wb", _P), ("A", _P), ("Ab", _P), ("C1", _P), ("C2", _P), ("R3", _P),
        ("acc_W", _P), ("acc_Wb", _P), ("acc_A", _P), ("acc_Ab", _P), ("acc_C1", _P),
        ("acc_C2", _P), ("acc_R3", _P),
        ("indptr", _P), ("indices", _P), ("values", _P), ("args1", _P), ("args2", _P),
        ("neg1", _P), ("neg2", _P), ("exchange", _P), ("costs", _P),
    ]


class RaeError(RuntimeError):
    pass


_lib = None


def load(path: str | None = None):
    """Load librae_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("RAE_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RaeError(f"{p} not found: build the HIP extension first "
                       "(python __graft_entry__.py build)")
    lib = C.CDLL(p)
    lib.rae_build_id.restype = C.c_char_p
    if path is None and "RAE_LIB" not in os.environ:     # RAE_LIB: explicit variant builds
        want = source_build_id()
        got = lib.rae_build_id().decode()
        if want is not None and got != want:
            raise RaeError(f"{p} was built from other sources (build id {got}, sources {want}): "
                           "rebuild it (python __graft_entry__.py build)")
    lib.rae_last_error.restype = C.c_char_p
    lib.rae_version.restype = C.c_int
    lib.rae_exchange_record_floats.restype = C.c_int64
    lib.rae_exchange_record_floats.argtypes = [C.POINTER(RaeConfig)]
    lib.rae_exchange_floats.restype = C.c_int64
    lib.rae_exchange_floats.argtypes = [C.POINTER(RaeConfig)]
    lib.rae_plan_create.argtypes = [C.POINTER(RaeConfig), C.POINTER(RaeBuffers), C.POINTER(_P)]
    lib.rae_plan_destroy.argtypes = [_P]
    lib.rae_plan_forms.argtypes = [_P, C.POINTER(RaeConfig)]
    lib.rae_dp_block_floats.argtypes = [C.POINTER(RaeConfig), C.c_int32, C.c_int32]
    lib.rae_dp_block_floats.restype = C.c_int64
    lib.rae_set_dp_buffers.argtypes = [_P, _P, _P, C.c_int32, C.c_int32]
    lib.rae_dp_list_max.argtypes = [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    for fn in ("rae_dp_pack", "rae_dp_unpack", "rae_dp_pack_at", "rae_dp_unpack_at"):
        getattr(lib, fn).argtypes = [_P, C.c_int64, _P]
        getattr(lib, fn).restype = C.c_int
    for fn in ("rae_set_dp_buffers", "rae_dp_list_max"):
        getattr(lib, fn).restype = C.c_int
    lib.rae_ipc_export.argtypes = [_P, _P, C.POINTER(C.c_int64)]
    lib.rae_ipc_open.argtypes = [_P, C.POINTER(_P)]
    lib.rae_ipc_close.argtypes = [_P]
    lib.rae_p2p_signals.argtypes = [_P]
    lib.rae_p2p_signals.restype = _P
    lib.rae_set_peer.argtypes = [_P, C.c_int32, _P, _P, _P, _P, _P]
    lib.rae_set_p2p_timeout.argtypes = [_P, C.c_double]
    lib.rae_p2p_prologue.argtypes = [_P, C.c_int64, C.c_int32, _P]
    for fn in ("rae_ipc_export", "rae_ipc_open", "rae_ipc_close", "rae_set_peer",
               "rae_set_p2p_timeout", "rae_p2p_prologue"):
        getattr(lib, fn).restype = C.c_int
    lib.rae_set_negatives.argtypes = [_P, _P, _P, C.c_int32, C.c_int64]
    lib.rae_set_cursor.argtypes = [_P, C.c_int64, _P]
    lib.rae_advance_cursor.argtypes = [_P, C.c_int64, _P]
    lib.rae_cursor_moves.argtypes = [_P]
    lib.rae_cursor_moves.restype = C.c_int64
    lib.rae_step_forward.argtypes = [_P, C.c_int64, _P]
    lib.rae_step_update.argtypes = [_P, C.c_int64, _P]
    lib.rae_step_forward_at.argtypes = [_P, C.c_int64, _P]
    lib.rae_step_update_at.argtypes = [_P, C.c_int64, _P]
    lib.rae_train_step.argtypes = [_P, C.c_int64, _P, _P, _P]
    lib.rae_check.argtypes = [_P]
    lib.rae_check_on.argtypes = [_P, _P]
    lib.rae_build_index.argtypes = [_P, C.c_int64, C.c_int64, _P]
    lib.rae_index_window.argtypes = [_P]
    lib.rae_index_window.restype = C.c_int64
    lib.rae_label.argtypes = [_P, _P, _P, _P, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P, _P]
    lib.rae_neg_sample.argtypes = [_P, C.c_int64, _P, C.c_int64, _P, _P]
    lib.rae_neg_sample_philox.argtypes = [_P, C.c_int64, C.c_uint64, C.c_uint64, C.c_int64, _P, _P]
    lib.rae_time_next.argtypes = [_P, _P, _P]
    lib.rae_stream_copy.argtypes = [_P, _P, C.c_int64, _P]
    lib.rae_mfma_probe.argtypes = [C.c_int64, C.c_int32, _P, _P]
    lib.rae_event_create.argtypes = [C.POINTER(_P)]
    lib.rae_event_destroy.argtypes = [_P]
    lib.rae_event_elapsed_ms.argtypes = [_P, _P, C.POINTER(C.c_float)]
    for fn in ("rae_stream_copy", "rae_mfma_probe", "rae_time_next", "rae_event_create", "rae_event_destroy", "rae_event_elapsed_ms",
               "rae_neg_sample", "rae_neg_sample_philox", "rae_plan_create", "rae_plan_destroy", "rae_plan_forms", "rae_set_negatives", "rae_set_cursor",
               "rae_advance_cursor", "rae_step_forward", "rae_step_update", "rae_train_step",
               "rae_step_forward_at", "rae_step_update_at",
               "rae_check", "rae_check_on", "rae_label", "rae_build_index"):
        getattr(lib, fn).restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = "rae call"):
    if rc != RAE_OK:
        msg = load().rae_last_error()
        raise RaeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()
