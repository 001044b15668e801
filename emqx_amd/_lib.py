"""ctypes binding of libemqx_gpu_match.so (include/emqx_gpu_match.h + emqx_gm_ext.h).

The HIP library is the only compute path: if it is missing, or no device is
visible, every compute call raises :class:`GpuMatchError` — there is no CPU
fallback.
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EMQX_GM_LIB") or os.path.join(_HERE, "libemqx_gpu_match.so")

OK, EINVAL, ENOMEM, EDEVICE, EOVERFLOW, EUNSUPPORTED = 0, -1, -2, -3, -4, -5
WITH_EXACT = 0x1
DEVICE_IO = 0x2
NO_TIMING = 0x4
OPEN_MIRROR_EAGER = 0x1
OPEN_MIRROR_LAZY = 0x2
IMAGE_NO_BLOB = 0x1

ERRNAMES = {EINVAL: "EINVAL", ENOMEM: "ENOMEM", EDEVICE: "EDEVICE", EOVERFLOW: "EOVERFLOW",
            EUNSUPPORTED: "EUNSUPPORTED"}


class GpuMatchError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{ERRNAMES.get(code, code)}: {msg}")


MAX_DEVICES = 8


class Opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32), ("n_devices", C.c_uint32),
                ("devices", C.c_int32 * MAX_DEVICES), ("reserved0", C.c_uint32), ("reserved", C.c_uint64 * 2)]


class Csr(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("nnz", C.c_uint64), ("row_off", C.POINTER(C.c_uint64)),
                ("ids", C.POINTER(C.c_uint32)), ("on_device", C.c_int32), ("reserved0", C.c_int32),
                ("priv", C.c_void_p)]


class IndexInfo(C.Structure):
    _fields_ = [("n_filters", C.c_uint64), ("n_wildcard", C.c_uint64), ("n_nodes", C.c_uint64),
                ("n_edges", C.c_uint64), ("n_words", C.c_uint64), ("n_subs", C.c_uint64),
                ("device_bytes", C.c_uint64), ("max_depth", C.c_uint32), ("trie_empty", C.c_int32)]


class MatchStats(C.Structure):
    _fields_ = [("n_topics", C.c_uint64), ("nnz", C.c_uint64), ("n_overflow", C.c_uint64),
                ("n_wildcard_topics", C.c_uint64), ("match_kernel_ms", C.c_double),
                ("total_device_ms", C.c_double), ("algo_bytes", C.c_uint64), ("probes", C.c_uint64)]


class UpdateStats(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("replica_mode", C.c_uint32), ("replicas", C.c_uint32),
                ("mirror_loaded", C.c_int32), ("mirror_bytes", C.c_uint64), ("mirror_ms", C.c_double),
                ("device_ms", C.c_double), ("replicate_ms", C.c_double), ("total_ms", C.c_double),
                ("blobs_reused", C.c_uint32), ("blobs_fresh", C.c_uint32)]


UPD_KINDS = {0: "none", 1: "patch", 2: "overlay", 3: "rebuild", 4: "subs_only", 5: "build", 6: "import"}
REP_MODES = {0: "none", 1: "patched", 2: "copied", 3: "shared"}


# Every symbol declared in include/emqx_gpu_match.h and include/emqx_gm_ext.h.
_vp, _u64, _i32, _u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
SIGNATURES = {
    # emqx_gpu_match.h
    "emqx_gm_open": (_i32, [C.POINTER(Opts), C.POINTER(_vp)]),
    "emqx_gm_close": (_i32, [_vp]),
    "emqx_gm_last_error": (C.c_char_p, [_vp]),
    "emqx_gm_abi_version": (_i32, []),
    "emqx_gm_set_stream": (_i32, [_vp, _vp]),
    "emqx_gm_synchronize": (_i32, [_vp]),
    "emqx_gm_index_build": (_i32, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, C.POINTER(_vp)]),
    "emqx_gm_index_update": (_i32, [_vp, _vp, _vp, _vp, _vp, _u64, C.POINTER(_vp)]),
    "emqx_gm_index_update_subs": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u64, C.POINTER(_vp)]),
    "emqx_gm_index_export": (_i32, [_vp, _vp, _u32, _vp, C.POINTER(_u64)]),
    "emqx_gm_index_device_blob": (_i32, [_vp, C.POINTER(_vp), C.POINTER(_u64)]),
    "emqx_gm_index_import": (_i32, [_vp, _vp, _u64, _vp, C.POINTER(_vp)]),
    "emqx_gm_index_retain": (_i32, [_vp]),
    "emqx_gm_index_release": (_i32, [_vp]),
    "emqx_gm_index_info": (_i32, [_vp, C.POINTER(IndexInfo)]),
    "emqx_gm_index_filter": (_i32, [_vp, _u32, C.POINTER(_vp), C.POINTER(_u64)]),
    "emqx_gm_index_subscriber_count": (_i32, [_vp, _u32, C.POINTER(_u64)]),
    "emqx_gm_match": (_i32, [_vp, _vp, _vp, _vp, _u64, _u32, C.POINTER(Csr)]),
    "emqx_gm_match_submit": (_i32, [_vp, _vp, _vp, _vp, _u64, _u32, C.POINTER(_vp)]),
    "emqx_gm_match_wait": (_i32, [_vp, _vp, C.POINTER(Csr)]),
    "emqx_gm_host_alloc": (_i32, [_vp, _u64, C.POINTER(_vp)]),
    "emqx_gm_host_free": (_i32, [_vp, _vp]),
    "emqx_gm_devices": (_i32, [_vp, _vp, C.POINTER(_u32)]),
    "emqx_gm_fanout": (_i32, [_vp, _vp, C.POINTER(Csr), _u32, C.POINTER(Csr)]),
    "emqx_gm_match_fanout": (_i32, [_vp, _vp, _vp, _vp, _u64, _u32, C.POINTER(Csr), C.POINTER(Csr)]),
    "emqx_gm_csr_free": (_i32, [_vp, C.POINTER(Csr)]),
    "emqx_gm_last_stats": (_i32, [_vp, C.POINTER(MatchStats)]),
    "emqx_gm_filter_ranks": (_i32, [_vp, _vp, _u64, _vp, C.POINTER(_u64)]),
    "emqx_gm_shard_of": (_i32, [_vp, _vp, _u64, _u32, _vp]),
    "emqx_gm_index_build_shard": (_i32, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, _vp, C.POINTER(_vp)]),
    "emqx_gm_index_build_sharded": (_i32, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, C.POINTER(_vp)]),
    "emqx_gm_csr_row_lengths": (_i32, [_vp, C.POINTER(Csr), _vp]),
    "emqx_gm_merge_rows": (_i32, [_vp, _u64, _u64, _u32, _vp, _vp, _u32, C.POINTER(Csr)]),
    "emqx_gm_prefix_plan": (_i32, [_vp, _vp, _u64, _u32, _vp, C.POINTER(_vp)]),
    "emqx_gm_route_topics_host": (_i32, [_vp, _vp, _vp, _u64, _vp]),
    "emqx_gm_route_topics": (_i32, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "emqx_gm_route_release": (_i32, [_vp]),
    "emqx_gm_route_partition": (_i32, [_vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "emqx_gm_permute_topics": (_i32, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "emqx_gm_unpermute_rows": (_i32, [_vp, _u64, _vp, _vp, _vp, _u32, C.POINTER(Csr)]),
    # emqx_gm_ext.h
    "emqx_gm_gen_filter_codes": (_i32, [_u64, _u64, _i32, _vp]),
    "emqx_gm_render_codes": (_u64, [_vp, _u64, _vp, _vp]),
    "emqx_gm_gen_topics": (_i32, [_vp, _vp, _u64, _u64, _u64, _u64, C.POINTER(_vp), C.POINTER(_vp),
                                  C.POINTER(_u64)]),
    "emqx_gm_dev_alloc": (_i32, [_vp, _u64, C.POINTER(_vp)]),
    "emqx_gm_dev_free": (_i32, [_vp, _vp]),
    "emqx_gm_memcpy": (_i32, [_vp, _vp, _vp, _u64, _i32]),
    "emqx_gm_pool_trim": (_i32, [_vp]),
    "emqx_gm_index_compile_host": (_i32, [_vp, _vp, _u64, _vp, _vp, _vp, C.POINTER(IndexInfo)]),
    "emqx_gm_matched_filter_bytes": (_i32, [_vp, _vp, C.POINTER(Csr), C.POINTER(_u64)]),
    "emqx_gm_fanout_part": (_i32, [_vp, _vp, C.POINTER(Csr), _u32, _u32, _u32, C.POINTER(Csr), C.POINTER(_u64)]),
    "emqx_gm_select_filters": (_i32, [_vp, _vp, _u64, _vp, _u32, _vp, _vp, C.POINTER(_u64), C.POINTER(_u64)]),
    "emqx_gm_last_update_stats": (_i32, [_vp, C.POINTER(UpdateStats)]),
    "emqx_gm_index_replica_digest": (_i32, [_vp, _vp, _u32, C.POINTER(_u64), C.POINTER(_u64)]),
}

_LIB = None


def _one_hip_runtime():
    """torch-ROCm ships its own HIP / HSA runtime (torch/lib/libamdhip64.so,
    SONAME libamdhip64.so.7, the same as /opt/rocm's).  Loaded before it, the
    library would pull /opt/rocm's copy in and torch would still load its own
    by path: two HSA runtimes in one process, and whichever initialises second
    finds no device (round 5: a host-only call such as gen_filter_codes before
    the first Context, then torch.cuda, then emqx_gm_open -> EDEVICE;
    scripts/smoke_order_diag.py).  Importing torch first makes the library
    bind to torch's runtime by SONAME: one runtime.  A process without torch
    loads /opt/rocm's."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load the HIP library; raise loudly if it is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise GpuMatchError(EUNSUPPORTED, f"{LIB_PATH} is not built (run __graft_entry__.build() "
                                              f"or `make -C emqx_amd/csrc`)")
        _one_hip_runtime()
        L = C.CDLL(LIB_PATH)
        # an older build loaded for a same-box A/B (EMQX_GM_LIB) may lack the newest
        # entry points: those stay unbound there; the shipped library must have them all
        ab = bool(os.environ.get("EMQX_GM_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if ab and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def check(rc: int, ctx=None, what: str = ""):
    if rc != OK:
        msg = ""
        if ctx:
            m = lib().emqx_gm_last_error(ctx)
            msg = m.decode(errors="replace") if m else ""
        raise GpuMatchError(rc, f"{what}: {msg}")
    return rc
