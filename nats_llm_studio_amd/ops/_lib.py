"""ctypes binding of the in-tree HIP kernel library (`_kernels.so`, built for gfx950
by `nats_llm_studio_amd/build.py`). On a GPU tensor every op goes through this
library; if it is missing we raise -- there is no silent eager fallback."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NLS_KERNELS_SO") or os.path.join(os.path.dirname(_HERE), "_kernels.so")

_lib = None

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float


class SampleParams(ctypes.Structure):
    _fields_ = [("temperature", c_float), ("top_p", c_float), ("min_p", c_float), ("repeat_penalty", c_float),
                ("presence_penalty", c_float), ("frequency_penalty", c_float), ("u", c_float),
                ("top_k", c_int), ("n_hist", c_int), ("pad", c_int)]


class NlsSeg(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("xmap", c_void_p), ("ymap", c_void_p), ("mcount", c_void_p),
                ("type", c_int), ("rows", c_int), ("K", c_int), ("ycol", c_int)]


class NlsFuse(ctypes.Structure):
    """Optional fused operands of one GEMV launch (csrc/kernels/qgemv.hip NlsFuse)."""
    _fields_ = [("xf", c_void_p), ("ldxf", c_long), ("nw", c_void_p), ("eps", c_float),
                ("pos", c_void_p), ("slot", c_void_p), ("cs", c_void_p), ("bias", c_void_p),
                ("q_out", c_void_p), ("ldq", c_long), ("kc", c_void_p), ("vc", c_void_p),
                ("Hq", c_int), ("Hkv", c_int), ("D", c_int), ("pad0", c_int),
                ("hout", c_void_p), ("ldh", c_long), ("onw", c_void_p), ("cnt", c_void_p),
                ("ssq_out", c_void_p), ("ssq_in", c_void_p), ("ldss", c_int), ("nss_in", c_int),
                ("sel", c_void_p), ("sel_slots", c_int), ("sel_base", c_int), ("pad1", c_int),
                ("wr", c_void_p), ("E", c_int), ("topk", c_int), ("renorm", c_int), ("rcap", c_int),
                ("rlogits", c_void_p), ("topw", c_void_p), ("counts", c_void_p), ("xrows", c_void_p),
                ("yrows", c_void_p), ("rsel", c_void_p)]


_SIGS = {
    "nls_qgemv": [ctypes.POINTER(NlsSeg), c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_float, c_int,
                  c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "nls_qgemv_ex": [ctypes.POINTER(NlsSeg), c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_float, c_int,
                     c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, ctypes.POINTER(NlsFuse)],
    "nls_fuse_size": [],
    "nls_qgemv_norm": [ctypes.POINTER(NlsSeg), c_int, c_void_p, c_long, c_void_p, c_float, c_void_p, c_long, c_int,
                       c_float, c_int, c_void_p, c_int, c_int, c_void_p],
    "nls_prefetch": [c_void_p, c_long, c_int, c_void_p],
    "nls_graph_kernel_names": [c_void_p, c_void_p, c_long],
    "nls_epx_bytes": [c_int, c_int],
    "nls_epx_wgs": [],
    "nls_epx_init": [c_void_p, c_int, c_int, c_void_p],
    "nls_epx_run": [c_void_p, c_long, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                    c_long, c_int, c_void_p],
    "nls_epx_err_clear": [c_void_p, c_int, c_int, c_void_p],
    "nls_epx_err_fetch": [c_void_p, c_int, c_int, c_void_p, c_void_p],
    "nls_rmsnorm": [c_void_p, c_long, c_void_p, c_void_p, c_long, c_int, c_int, c_float, c_int, c_void_p],
    "nls_splitk_add_rmsnorm": [c_void_p, c_int, c_int, c_float, c_void_p, c_long, c_void_p, c_void_p, c_long, c_int,
                               c_float, c_void_p],
    "nls_rope_kv": [c_void_p, c_long, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                    c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nls_rope_kv8": [c_void_p, c_long, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                    c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nls_embed": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_float, c_void_p],
    "nls_embed_prev": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_float,
                       c_void_p],
    "nls_dequant": [c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_void_p],
    "nls_swiglu16": [c_void_p, c_long, c_int, c_int, c_float, c_void_p, c_long, c_void_p],
    "nls_argmax": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p],
    "nls_argmax_unpack": [c_void_p, c_int, c_void_p, c_void_p],
    "nls_argmax_unpack_rearm": [c_void_p, c_int, c_void_p, c_void_p],
    "nls_moe_route": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                      c_void_p, c_void_p],
    "nls_moe_norm_route": [c_void_p, c_long, c_void_p, c_float, c_int, c_void_p, c_void_p, c_long, c_void_p, c_int,
                           c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "nls_router_logits": [c_void_p, c_long, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p],
    "nls_moe_combine": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_long, c_int, c_float, c_int, c_void_p],
    "nls_moe_combine_norm": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_long, c_int, c_float, c_void_p, c_float,
                             c_void_p, c_long, c_void_p],
    "nls_attn_decode": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                        c_int, c_int, c_int, c_float, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    "nls_attn_decode8": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                        c_int, c_int, c_int, c_float, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    "nls_attn_prefill": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                         c_int, c_int, c_float, c_void_p, c_long, c_void_p],
    "nls_attn_prefill8": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                         c_int, c_int, c_float, c_void_p, c_long, c_void_p],
    "nls_attn_prefill_v1": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                            c_int, c_int, c_float, c_void_p, c_long, c_void_p],
    "nls_attn_prefill_v18": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                             c_int, c_int, c_float, c_void_p, c_long, c_void_p],
    "nls_sample": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "nls_sample_params_size": [],
    "nls_topc": [c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "nls_sample_decode": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                          c_void_p, c_void_p],
    "nls_sample_decode_cand": [c_void_p, c_long, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "nls_ar_alloc": [c_long, c_int, c_void_p, c_void_p],
    "nls_ar_open": [c_void_p, c_void_p],
    "nls_ar_close": [c_void_p],
    "nls_ar_free": [c_void_p],
    "nls_ar_handle_size": [],
    "nls_ar_blocks": [],
    "nls_ar_addnorm": [c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_long, c_int, c_int, c_float,
                       c_void_p, c_int, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p],
    "nls_ar_addnorm_sim": [c_void_p, c_long, c_void_p, c_long, c_void_p, c_void_p, c_long, c_int, c_int, c_float,
                           c_void_p, c_int, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                           c_int, c_long, c_long, c_long, c_long, c_long, c_long],
    "nls_ar_row_blocks": [c_int],
    "nls_ar_epoch_slots": [c_long],
    "nls_ag_epoch_slots": [c_long],
    "nls_ar_err_fetch": [c_void_p, c_long, c_int, c_void_p, c_void_p],
    "nls_ar_err_clear": [c_void_p, c_long, c_int, c_void_p],
    "nls_ar_err_words": [c_void_p, c_long, c_int, c_void_p, c_int, c_void_p],
    "nls_ar_peek": [c_void_p, c_long, c_int, c_void_p, c_void_p],
    "nls_ar_probe_hist": [c_int, c_void_p],
    "nls_ar_probe_depth": [],
    "nls_ar_set_norm_wgs": [c_int],
    "nls_ar_get_norm_wgs": [],
    "nls_epx_set_wgs": [c_int],
    "nls_ar_buffer_bytes": [c_long, c_int],
    "nls_ag_blocks": [],
    "nls_ag_run": [c_void_p, c_long, c_void_p, c_int, c_long, c_void_p, c_int, c_int, c_long, c_void_p, c_void_p,
                   c_long, c_void_p],
    "nls_ag_argmax": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_long, c_void_p, c_void_p, c_long,
                      c_void_p],
    "nls_ar_reinit": [c_void_p, c_long, c_int, c_void_p],
    "nls_ar_run": [c_void_p, c_long, c_void_p, c_int, c_int, c_long, c_void_p, c_void_p, c_long, c_void_p],
}


def load(path: str):
    """Load (and type) a kernel library without installing it (A/B of kernel variants in one process)."""
    L = ctypes.CDLL(path)
    for name, args in _SIGS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = c_int
    return L


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP kernel library missing: {LIB_PATH} (run `python -m nats_llm_studio_amd.build`)")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = c_int
        if L.nls_fuse_size() != ctypes.sizeof(NlsFuse):
            raise RuntimeError("stale _kernels.so: NlsFuse layout mismatch (rebuild the kernels)")
        if LIB_PATH.endswith(os.path.join("nats_llm_studio_amd", "_kernels.so")) and not built_from_sources():
            # the library's content stamp (build.py) does not match the kernel sources of this tree
            import warnings
            warnings.warn(f"{LIB_PATH} was not built from the current csrc/kernels sources "
                          "(run `python -m nats_llm_studio_amd.build`)", RuntimeWarning)
        _lib = L
    return _lib


_OP_TIMING = os.environ.get("NLS_OP_TIMING", "0") == "1"
_op_events = None


def check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")
    if _OP_TIMING:
        _op_mark(name)


def _op_mark(name: str):
    """NLS_OP_TIMING=1 (diagnostics): an event on the current stream after every launch that is not being captured,
    kept for the last 4096 launches (op_timing)."""
    global _op_events
    import collections
    import torch
    if not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        return
    if _op_events is None:
        _op_events = collections.deque(maxlen=4096)
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    _op_events.append((name, ev))


def op_timing(min_ms: float = 0.0):
    """(launch name, ms since the previous marked launch completed) of the marked launches, oldest first, after a
    device sync; only gaps >= min_ms are listed (with their index)."""
    import torch
    if not _op_events:
        return []
    torch.cuda.synchronize()
    evs = list(_op_events)
    out = []
    for i in range(1, len(evs)):
        ms = evs[i - 1][1].elapsed_time(evs[i][1])
        if ms >= min_ms:
            out.append((i - len(evs), evs[i][0], round(ms, 3)))
    return out


def available() -> bool:
    return os.path.exists(LIB_PATH)


def built_from_sources() -> bool:
    """True when `_kernels.so` carries the content hash of this tree's kernel sources (build.py stamp)."""
    from .. import build
    return build.kernels_current(LIB_PATH)
