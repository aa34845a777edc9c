"""ctypes binding of libdvcp_hip.so (the C ABI declared in include/dvcp.h).

The library is built in-tree (``make`` in deepvcp-pointcloud-registration_amd/, or
``__graft_entry__.build()``) and loaded after ``import torch`` so that it binds to the same
HIP runtime (SONAME libamdhip64.so.7) that owns torch's device memory and streams.  There is
no fallback: if the library is missing or no GPU is present, every op raises.
"""
import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DVCP_LIB_PATH: load another build of the library (the A/B scripts' variants) without touching
# the in-tree one; it must report this package's ABI version like any other
LIB_PATH = os.environ.get("DVCP_LIB_PATH") or os.path.join(_HERE, "libdvcp_hip.so")

F32, F64 = 0, 1
ABI_VERSION = 4   # include/dvcp.h DVCP_ABI_VERSION
_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_D = ctypes.c_double

# name -> argtypes (every entry point returns int, 0 on success)
SIGNATURES = {
    "dvcp_fps": [_I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P],
    "dvcp_fps_ws": [_I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "dvcp_fps_parts": [_I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _L, _P, _I, _P],
    "dvcp_fps_step_floor": [_I, _I, _P, _P],
    "dvcp_fps_pair": [_I, _P, _L, _L, _L, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    "dvcp_fps_split_probe": [_I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P, ctypes.c_uint32, _I, _P],
    "dvcp_ball_query": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _D, _I, _P, _P, _P, _P],
    "dvcp_ball_query_ws": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _D, _I, _P, _P, _P, _P, _P],
    "dvcp_square_distance": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _P, _P],
    "dvcp_sa_group_mlp": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                          _P, _P, _I, _I, _P, _P, _P, _P],
    "dvcp_sa_group_mlp_ws": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                             _P, _P, _I, _I, _P, _P, _P, _P, _P],
    "dvcp_sa_group_mlp_rows_ws": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _P, _L, _L, _I, _I, _P,
                                  _P, _P, _I, _I, _P, _P, _P, _P, _P],
    "dvcp_fe_head": [_P, _I, _P, _P, _P, _P],
    "dvcp_fe_head_rows": [_P, _P, _I, _I, _I, _P, _P, _P, _P],
    "dvcp_weighting": [_P, _I, _P, _P, _P],
    "dvcp_topk": [_P, _I, _I, _I, _P, _P],
    "dvcp_src_keypoints": [_I, _P, _P, _I, _P, _I, _I, _P, _D, _I, _P, _L, _P, _P, _P, _P],
    "dvcp_voxelize": [_I, _P, _L, _L, _L, _I, _I, _D, _D, _I, _P, _P, _P],
    "dvcp_knn": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P],
    "dvcp_knn_grid": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P],
    "dvcp_knn_tiled": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P],
    "dvcp_knn_tiled_insert": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P],
    "dvcp_dfe": [_I, _P, _L, _P, _P, _P],
    "dvcp_dfe_tgt": [_I, _P, _L, _L, _L, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P],
    "dvcp_points_pack4": [_P, _L, _L, _L, _I, _I, _P, _P],
    "dvcp_dfe_tgt_f16": [_I, _P, _L, _L, _L, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P],
    "dvcp_dfe_tgt_literal": [_I, _P, _L, _L, _L, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P],
    "dvcp_cpg": [_P, _P, _L, _L, _L, _P, _I, _I, _P, _P, _P, _P],
    "dvcp_rigid_transform": [_P, _P, _I, _I, _P, _P, _P],
    "dvcp_paper_pose": [_P, _P, _P, _I, _I, _I, _D, _P, _P, _P, _P, _P, _P],
    "dvcp_paper_pose_backward": [_P, _P, _P, _I, _I, _I, _D, _P, _P, _D, _P, _P, _P, _P],
    "dvcp_feature_propagation": [_P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _P, _L, _L, _L, _I, _P, _L, _L, _I,
                                 _I, _P, _P, _P, _P, _P],
    "dvcp_group_rows": [_P, _L, _L, _L, _I, _P, _L, _L, _L, _P, _L, _L, _I, _P, _P, _I, _I, _D, _I, _P, _P],
    "dvcp_cpg1d": [_P, _P, _P, _I, _I, _P, _P, _P, _P],
    "dvcp_svd_optimization": [_P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P],
    "dvcp_deepvcp_loss": [_P, _P, _P, _P, _I, _I, _D, _P, _P, _P, _P, _P],
    "dvcp_registration_error": [_P, _P, _P, _L, _P, _L, _I, _P, _P, _P],
    "dvcp_rigid_apply": [_I, _P, _L, _L, _L, _I, _I, _I, _P, _P, _L, _P, _P],
    "dvcp_svd_optimization_backward": [_P, _P, _P, _P, _I, _I, _P, _P, _D, _P, _P],
    "dvcp_dfe_backward": [_I, _P, _L, _P, _P, _P, _P, _P, _P],
    "dvcp_dfe_tgt_backward": [_I, _P, _L, _L, _L, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P],
    "dvcp_src_keypoints_backward": [_I, _P, _I, _P, _I, _I, _P, _D, _I, _P, _P, _P],
    "dvcp_cpg_backward": [_P, _P, _L, _L, _L, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "dvcp_sa_group_mlp_backward": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                                   _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    "dvcp_fe_head_backward": [_P, _I, _P, _P, _P, _P, _P, _P],
    "dvcp_sa_bn_stats": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                         _P, _P, _I, _I, _P, _P, _I, _P, _P, _P, _P],
    "dvcp_sa_bn_backward": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                            _P, _P, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P],
    "dvcp_sa_bn_zrows": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _I, _P, _L, _L, _L, _I,
                         _P, _P, _I, _I, _P, _P, _P, _P],
    "dvcp_sa_bnm_pre": [_P, _L, _L, _I, _I, _I, _P, _P, _P, _P],
    "dvcp_sa_bnm_pass": [_I, _P, _L, _L, _L, _I, _P, _L, _L, _L, _I, _I, _P, _L, _L, _L, _I, _P, _P, _I, _I, _P,
                         _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
}

_lib = None


def load():
    """Load the HIP library (once) and declare its prototypes."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"dvcp: HIP library not built ({LIB_PATH} missing). Run `make -j16` in "
            "deepvcp-pointcloud-registration_amd/ or __graft_entry__.build().")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    lib.dvcp_last_error.restype = ctypes.c_char_p
    lib.dvcp_last_error.argtypes = []
    lib.dvcp_abi_version.restype = ctypes.c_int
    lib.dvcp_abi_version.argtypes = []
    if lib.dvcp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"dvcp: {LIB_PATH} has ABI version {lib.dvcp_abi_version()}, this package expects "
                           f"{ABI_VERSION}: rebuild it (make -j16 in deepvcp-pointcloud-registration_amd/)")
    lib.dvcp_knn_grid_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_knn_grid_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.dvcp_knn_tiled_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_knn_tiled_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.dvcp_fps_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_fps_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.dvcp_fps_pair_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_fps_pair_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.dvcp_ball_query_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_ball_query_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.dvcp_sa_group_mlp_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_sa_group_mlp_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_void_p]
    lib.dvcp_dfe_backward_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_dfe_backward_workspace_bytes.argtypes = [ctypes.c_int64]
    lib.dvcp_dfe_tgt_backward_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_dfe_tgt_backward_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.dvcp_cpg_backward_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_cpg_backward_workspace_bytes.argtypes = [ctypes.c_int]
    lib.dvcp_sa_group_mlp_backward_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_sa_group_mlp_backward_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                               ctypes.c_void_p]
    lib.dvcp_fe_head_backward_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_fe_head_backward_workspace_bytes.argtypes = [ctypes.c_int]
    lib.dvcp_sa_bn_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_sa_bn_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.dvcp_sa_bn_rows_floats.restype = ctypes.c_int64
    lib.dvcp_sa_bn_feat_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_sa_bn_feat_workspace_bytes.argtypes = [ctypes.c_int] * 5
    lib.dvcp_sa_bn_rows_floats.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.dvcp_sa_bn_zrows_floats.restype = ctypes.c_int64
    lib.dvcp_sa_bn_zrows_floats.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.dvcp_cpg1d_nparams.restype = ctypes.c_int
    lib.dvcp_cpg1d_nparams.argtypes = []
    lib.dvcp_sa_bn_pack_floats.restype = ctypes.c_int64
    lib.dvcp_sa_bn_pack_floats.argtypes = [ctypes.c_int, ctypes.c_void_p]
    lib.dvcp_sa_bnm_supported.restype = ctypes.c_int
    lib.dvcp_sa_bnm_supported.argtypes = [ctypes.c_int, ctypes.c_void_p]
    lib.dvcp_sa_bnm_workspace_bytes.restype = ctypes.c_int64
    lib.dvcp_sa_bnm_workspace_bytes.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int]
    for name, args in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            raise RuntimeError(f"dvcp: {LIB_PATH} does not export {name} (a stale build of ABI {ABI_VERSION}): "
                               "rebuild it (make -j16 in deepvcp-pointcloud-registration_amd/)") from None
        fn.restype = ctypes.c_int
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return ["dvcp_last_error", "dvcp_abi_version", "dvcp_knn_grid_workspace_bytes",
            "dvcp_knn_tiled_workspace_bytes", "dvcp_ball_query_workspace_bytes",
            "dvcp_sa_group_mlp_workspace_bytes", "dvcp_dfe_backward_workspace_bytes",
            "dvcp_dfe_tgt_backward_workspace_bytes",
            "dvcp_cpg_backward_workspace_bytes", "dvcp_sa_group_mlp_backward_workspace_bytes",
            "dvcp_fe_head_backward_workspace_bytes", "dvcp_sa_bn_workspace_bytes",
            "dvcp_sa_bn_pack_floats", "dvcp_sa_bn_rows_floats", "dvcp_sa_bn_feat_workspace_bytes", "dvcp_sa_bn_zrows_floats",
            "dvcp_cpg1d_nparams", "dvcp_sa_bnm_supported", "dvcp_sa_bnm_workspace_bytes",
            "dvcp_fps_pair_workspace_bytes", "dvcp_fps_workspace_bytes"] + list(SIGNATURES)


# When a list, every entry-point call appends (name, start_event, end_event, work) recorded on
# torch's current stream (the stream the kernel is launched on) -- bench.py's live per-kernel
# HIP-event timing.  `work` = (algorithmic flops, algorithmic bytes[, executed[, workgroups,
# serial steps]]) of that launch: flops and bytes on the reference's op graph (DESIGN.md section
# 6); `executed` = (flops the kernels execute, of which on MFMA) where known -- a tuple, or a
# callable returning one that the bench evaluates after its timed region (the SA tables count
# their real ball-query hits) -- None when not counted; and for the latency-bound FPS chain its
# workgroup count and dependent steps.  None (the default) costs nothing.
EVENT_LOG = None


# Diagnostic (bench marginal-cost probes): DVCP_DUP=<entry> issues that entry point twice per call
# (same arguments, idempotent outputs), so the throughput drop is that kernel's marginal cost.
_DUP = os.environ.get("DVCP_DUP", "")


def call(name, *args, work=None):
    """Call an entry point; raise RuntimeError with the library's message on failure."""
    lib = load()
    if _DUP and name == _DUP:
        getattr(lib, name)(*args)
    if EVENT_LOG is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib, name)(*args)
        e1.record()
        EVENT_LOG.append((name, e0, e1, work))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {lib.dvcp_last_error().decode()}")


# Device error words (split-FPS guard, voxel grid length) checked without stalling the stream:
# each is copied to pinned host memory behind an event; ``check_device_flags`` raises for any
# whose event has completed with a nonzero word (block=True waits for all of them).
_PENDING_FLAGS = []
# While a step is captured into a graph (dvcp/graphs.py) the error words are collected here
# instead (a host copy and an event query cannot run inside a capture); the graph's owner checks
# them after each replay.
_CAPTURED_FLAGS = None


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


# Inside a step (``deferred_flags``, DeepVCP.forward) the words wait for the step's end: they are
# gathered per stream and copied once (one cat, one host copy) when the step closes, instead of
# one copy behind each flagged launch on the step's serial chain (the split-select FPS launches).
_STEP_FLAGS = None  # {stream handle: (stream, [(what, flag)])} while a step is open


def _queue_host_copy(items):
    """One pinned host copy of the error words ``items`` [(what, flag)] on the current stream."""
    words = items[0][1].reshape(-1) if len(items) == 1 else torch.cat([f.reshape(-1) for _, f in items])
    host = torch.empty(words.shape, dtype=words.dtype, pin_memory=True)
    host.copy_(words, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    off = 0
    for what, f in items:
        _PENDING_FLAGS.append((what, ev, host[off:off + f.numel()]))
        off += f.numel()


@contextlib.contextmanager
def deferred_flags():
    """Defer the error-word copies of the launches issued inside to the end of the block."""
    global _STEP_FLAGS
    if _STEP_FLAGS is not None or _capturing():  # nested, or captured (the graph collects them)
        yield
        return
    _STEP_FLAGS = {}
    try:
        yield
    finally:
        pending, _STEP_FLAGS = _STEP_FLAGS, None
        for s, items in pending.values():
            with torch.cuda.stream(s):  # the stream the flagged launches ran on
                _queue_host_copy(items)


def defer_flag_check(what, flag):
    if _CAPTURED_FLAGS is not None and _capturing():
        _CAPTURED_FLAGS.append((what, flag))
        return
    if _STEP_FLAGS is not None:
        s = torch.cuda.current_stream(flag.device)
        _STEP_FLAGS.setdefault(s.cuda_stream, (s, []))[1].append((what, flag))
        return
    _queue_host_copy([(what, flag)])


def check_device_flags(block=False):
    """Raise RuntimeError for a completed launch whose error word is set (see defer_flag_check)."""
    global _PENDING_FLAGS
    if _capturing():
        return
    keep, failed = [], None
    for what, ev, host in _PENDING_FLAGS:
        if block:
            ev.synchronize()
        if block or ev.query():
            if failed is None and bool((host != 0).any()):
                failed = what
        else:
            keep.append((what, ev, host))
    _PENDING_FLAGS = keep
    if failed is not None:
        raise RuntimeError(f"dvcp: {failed}")


def ptr(t):
    """Device pointer of a tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.float64:
        return F64
    raise TypeError(f"dvcp: coordinates must be float32 or float64, got {t.dtype}")


def require_gpu(*tensors):
    """The product path has no CPU fallback: every operand must already live on a GPU."""
    if not torch.cuda.is_available():
        raise RuntimeError("dvcp: no GPU available -- the HIP path has no CPU fallback")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("dvcp: expected a GPU tensor, got one on " + str(t.device))


def point_strides(t, point_dim, coord_dim):
    """Element strides (batch, coord, point) of a 3-D point tensor."""
    st = t.stride()
    return st[0], st[coord_dim], st[point_dim]
