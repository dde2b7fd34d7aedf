"""ctypes binding of libptgpu.so (include/ptgpu.h).

The product path: there is no fallback.  If the HIP library is missing or a
call fails, a PtgError is raised.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PTGPU_LIB selects an alternative build of the same ABI (A/B experiments only)
LIB_PATH = os.environ.get("PTGPU_LIB") or os.path.join(PKG_DIR, "libptgpu.so")
ABI_VERSION = 2  # include/ptgpu.h PTG_ABI_VERSION

# every symbol include/ptgpu.h declares
EXPORTS = (
    "ptg_abi_version", "ptg_last_error", "ptg_device_count", "ptg_render",
    "ptg_context_create", "ptg_context_destroy", "ptg_shard_rows", "ptg_render_device",
    "ptg_unshard_device", "ptg_tonemap_device", "ptg_trace_samples_device",
    "ptg_reset_accumulation_device", "ptg_accumulate_device", "ptg_resolve_device", "ptg_scene_layout",
    "ptg_render_multi", "ptg_multi_create", "ptg_multi_destroy", "ptg_multi_render",
    "ptg_multi_reset_accumulation", "ptg_multi_accumulate", "ptg_multi_resolve", "ptg_multi_frame_device",
    "ptg_multi_frame_timing", "ptg_multi_image", "ptg_math_probe_device", "ptg_multi_comm_info",
    "ptg_device_pci_bus_id", "ptg_launch_info",
)


class PtgError(RuntimeError):
    pass


class Params(C.Structure):  # ptg_params
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("samples", C.c_int32),
                ("num_subpixels", C.c_int32), ("seed", C.c_uint64), ("band_rows", C.c_int32),
                ("shard_rank", C.c_int32), ("shard_count", C.c_int32), ("chunk_samples", C.c_int32),
                ("flags", C.c_int32)]


assert C.sizeof(Params) == 48

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PtgError(f"{LIB_PATH} not built: run `make -C cpu-path-tracing_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        I = C.c_int
        sig = {
            "ptg_abi_version": (I, []),
            "ptg_last_error": (C.c_char_p, []),
            "ptg_device_count": (I, [C.POINTER(C.c_int)]),
            "ptg_render": (I, [P, C.c_size_t, P, C.POINTER(Params), I, P]),
            "ptg_context_create": (I, [P, C.c_size_t, P, I, C.POINTER(C.c_void_p)]),
            "ptg_context_destroy": (I, [P]),
            "ptg_shard_rows": (I, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
            "ptg_render_device": (I, [P, C.POINTER(Params), P, P, P]),
            "ptg_unshard_device": (I, [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P]),
            "ptg_tonemap_device": (I, [P, P, C.c_size_t, P]),
            "ptg_trace_samples_device": (I, [P, C.POINTER(Params), P, C.c_size_t, P, P, P]),
            "ptg_math_probe_device": (I, [P, C.c_int32, C.c_int32, P, P, C.c_size_t, P]),
            "ptg_reset_accumulation_device": (I, [P, C.POINTER(Params), P]),
            "ptg_accumulate_device": (I, [P, C.POINTER(Params), C.c_int32, C.c_int32, P, P]),
            "ptg_resolve_device": (I, [P, C.POINTER(Params), C.c_int32, P, P]),
            "ptg_scene_layout": (I, [P, C.c_size_t, P, P, P]),
            "ptg_render_multi": (I, [P, C.c_size_t, P, C.POINTER(Params), C.POINTER(C.c_int), I, P]),
            "ptg_multi_create": (I, [P, C.c_size_t, P, C.POINTER(C.c_int), I, C.POINTER(C.c_void_p)]),
            "ptg_multi_destroy": (I, [P]),
            "ptg_multi_render": (I, [P, C.POINTER(Params), P]),
            "ptg_multi_reset_accumulation": (I, [P, C.POINTER(Params)]),
            "ptg_multi_accumulate": (I, [P, C.POINTER(Params), C.c_int32, C.c_int32]),
            "ptg_multi_resolve": (I, [P, C.POINTER(Params), C.c_int32, P]),
            "ptg_multi_frame_device": (I, [P, C.POINTER(Params), P]),
            "ptg_multi_frame_timing": (I, [P, P, I, P]),
            "ptg_multi_image": (I, [P, C.POINTER(Params), P]),
            "ptg_multi_comm_info": (I, [P, P, P, P, I]),
            "ptg_device_pci_bus_id": (I, [I, C.c_char_p, I]),
            "ptg_launch_info": (I, [P, C.POINTER(Params), P, I]),
            "ptg_multi_inject_gather_fault_": (I, [P, I]),
            # internal (tests): n shards on one device, gathered by device copies
            "ptg_multi_create_local_": (I, [P, C.c_size_t, P, I, I, C.POINTER(C.c_void_p)]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("PTGPU_LIB") and not hasattr(L, name):
                continue  # A/B builds of older commits: entry points added since are absent
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.ptg_abi_version() != ABI_VERSION:
            raise PtgError("libptgpu.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ptg_last_error().decode(errors="replace")
        raise PtgError(f"{what} failed ({rc}): {msg}")
