"""ctypes binding of the engine's C ABI (include/mdl_engine.h -> marl_gpu/libmdl.so).

torch is imported first on purpose: torch bundles a HIP runtime whose SONAME
(libamdhip64.so.7) equals the system one, so once torch is loaded the dynamic
linker resolves libmdl.so's HIP imports to torch's runtime and device pointers
and stream handles are shared between the two.

There is no fallback: if the shared library is missing or fails to load, the
import raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede loading libmdl.so, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# MDL_LIB_PATH loads another build of the library (same-box A/B of profiling builds): honoured only
# with MDL_PROFILING=1, so no product run can pick up a profiling build by accident
_PROFILING = os.environ.get("MDL_PROFILING") == "1"
if os.environ.get("MDL_LIB_PATH") and not _PROFILING:
    raise ImportError("marl_gpu: MDL_LIB_PATH is set without MDL_PROFILING=1; it selects a profiling build of "
                      "libmdl.so and is refused otherwise")
LIB_PATH = (os.environ.get("MDL_LIB_PATH") if _PROFILING else None) or os.path.join(HERE, "libmdl.so")

MDL_TRACKER_FRESH = 0
MDL_TRACKER_MAPPO_STALE = 1
MDL_ACTION_TRAINER_INT = 0
MDL_ACTION_CODES = 1
MDL_MAX_ROBOTS = 64
MDL_MAX_PACKAGES = 1024
MDL_OBS_BUILDER_AUTO = 0
MDL_OBS_BUILDER_GENERIC = 1
MDL_STEP_LAYOUT_AUTO = 0
MDL_STEP_LAYOUT_WAVE = 1
MDL_STEP_LAYOUT_ROWS = 2
MDL_STEP_LAYOUT_HALVES = 3


class MdlConfig(C.Structure):
    _fields_ = [
        ("n_envs", C.c_int32),
        ("n_robots", C.c_int32),
        ("n_packages", C.c_int32),
        ("max_time_steps", C.c_int32),
        ("move_cost", C.c_double),
        ("delivery_reward", C.c_double),
        ("delay_reward", C.c_double),
        ("tracker_mode", C.c_int32),
        ("shaping", C.c_double * 9),
        ("obs_max_time_steps", C.c_int32),
        ("max_other_robots", C.c_int32),
        ("max_packages_obs", C.c_int32),
        ("max_robots_state", C.c_int32),
        ("max_packages_state", C.c_int32),
        ("obs_builder", C.c_int32),
        ("step_layout", C.c_int32),
    ]


MDL_RTERM_MOVE, MDL_RTERM_ONTIME, MDL_RTERM_LATE = 1, 2, 4


class MdlMailbox(C.Structure):
    """include/mdl_engine.h MdlMailbox: host-mapped sections of the dict-API mailbox."""
    _fields_ = [(n, C.c_void_p) for n in ("seq", "codes", "ids", "r_env", "r_shaped", "done", "robots", "pkgs", "t",
                                          "total_reward", "rterms")]


# name -> (restype, argtypes); every symbol include/mdl_engine.h declares
_vp, _i32, _i64p = C.c_void_p, C.c_int32, C.c_void_p
SIGNATURES = {
    "mdl_create": (C.c_int, [C.POINTER(MdlConfig), _vp, _vp, _i32, _vp, _i32, C.POINTER(C.c_void_p)]),
    "mdl_destroy": (C.c_int, [_vp]),
    "mdl_seed": (C.c_int, [_vp, _vp, _vp]),
    "mdl_reset": (C.c_int, [_vp, _vp, _i32, _vp]),
    "mdl_tracker_clear": (C.c_int, [_vp, _vp, _i32, _vp]),
    "mdl_step": (C.c_int, [_vp, _vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp]),
    "mdl_step_obs": (C.c_int, [_vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mdl_step_fused": (C.c_int, [_vp, _vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "mdl_step_floor": (C.c_int, [_vp, _i32, _vp]),
    "mdl_build_obs": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mdl_build_obs_alt": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _i32, _i32, _vp]),
    "mdl_views_alt_features": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp]),
    "mdl_views_idq_reward": (C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp]),
    "mdl_greedy_init": (C.c_int, [_vp, _vp, _i32, _vp]),
    "mdl_greedy_actions": (C.c_int, [_vp, _vp, _i32, _vp, _vp]),
    "mdl_mailbox": (C.c_int, [_vp, C.POINTER(MdlMailbox)]),
    "mdl_mail_step": (C.c_int, [_vp, _i32, _i32, _i32, _vp]),
    "mdl_mail_reset": (C.c_int, [_vp, _i32, _i32, _vp]),
    "mdl_mail_export": (C.c_int, [_vp, _i32, _i32, _vp]),
    "mdl_host_arena": (C.c_int, [_vp, C.c_int64, C.POINTER(C.c_void_p)]),
    "mdl_host_wait": (C.c_int, [_vp, _vp]),
    "mdl_state_bytes": (C.c_int, [_vp, C.POINTER(C.c_int64)]),
    "mdl_save_state": (C.c_int, [_vp, _vp, C.c_int64, _vp]),
    "mdl_load_state": (C.c_int, [_vp, _vp, C.c_int64, _vp]),
    "mdl_sample_actions": (C.c_int, [_vp, C.c_int64, _i32, C.c_uint64, C.c_uint64, _vp, _vp, _vp]),
    "mdl_sample_actions_dev": (C.c_int, [_vp, C.c_int64, _i32, C.c_uint64, _vp, C.c_uint64, _vp, _vp, _vp]),
    "mdl_counter_add": (C.c_int, [_vp, C.c_uint64, _vp]),
    "mdl_gae": (C.c_int, [_vp, _vp, _vp, _vp, _i32, C.c_int64, C.c_float, C.c_float, _vp, _vp, _vp]),
    "mdl_read_state": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mdl_views_features": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32,
                                     _vp, _vp, _vp, _vp, _vp]),
    "mdl_views_shaped_reward": (C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "mdl_host_views_features": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32,
                                          _vp, _vp, _vp, _vp, _vp]),
    "mdl_host_views_shaped_reward": (C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "mdl_host_view_features": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                                         _vp]),
    "mdl_host_view_shaped_reward": (C.c_int, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, C.c_double, _vp, _vp, _vp]),
    "mdl_rank_table": (C.c_int, [_i32, _i32, _vp]),
    "mdl_get_config": (C.c_int, [_vp, C.POINTER(MdlConfig)]),
    "mdl_obs_dims": (C.c_int, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "mdl_step_layout": (C.c_int, [_vp, _i32, _i32, C.POINTER(C.c_int32)]),
    "mdl_last_step_layout": (C.c_int, [_vp, C.POINTER(C.c_int32)]),
    "mdl_step_kernel_name": (C.c_int, [_vp, _i32, _i32, C.c_char_p, _i32]),
    "mdl_last_error": (C.c_char_p, []),
    "mdl_version": (C.c_char_p, []),
}

_lib = None


class MdlError(RuntimeError):
    pass


def lib():
    """Load libmdl.so (raises if it is missing: the engine has no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"marl_gpu: {LIB_PATH} not built; run `make -C marl-delivery_amd` "
                              "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if _PROFILING and LIB_PATH != os.path.join(HERE, "libmdl.so") and not hasattr(L, name):
                continue   # an older profiling build (same-box A/B): entry points it lacks stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_pack_bound = None


def pack():
    """The C extension of the per-call dict paths (_mdl_pack), bound once to libmdl.so's
    entries it calls directly (helpers: mdl_host_view*_*; errors: mdl_last_error / MdlError)."""
    global _pack_bound
    if _pack_bound is None:
        from . import _mdl_pack
        L = lib()
        addr = lambda f: C.cast(f, C.c_void_p).value  # noqa: E731
        _mdl_pack.bind(addr(L.mdl_host_views_features), addr(L.mdl_host_views_shaped_reward),
                       addr(L.mdl_host_view_features), addr(L.mdl_host_view_shaped_reward),
                       addr(L.mdl_last_error), MdlError)
        _pack_bound = _mdl_pack
    return _pack_bound


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().mdl_last_error().decode(errors="replace")
        raise MdlError(f"{what}: {msg}" if what else msg)


def ptr(t) -> int | None:
    """Device (or host) address of a tensor / None."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


_raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def raw_stream(index: int) -> int:
    """hipStream_t of torch's current stream on device ``index`` (the fast accessor
    when this torch build has it: no Stream object per call)."""
    if _raw is not None:
        return _raw(index)
    return torch.cuda.current_stream(index).cuda_stream
