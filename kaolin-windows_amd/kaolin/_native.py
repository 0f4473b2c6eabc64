"""Loader for libkaolin_hip.so, the gfx950 C-ABI library (include/kaolin_hip.h).

There is no fallback: if the library is missing or no HIP device is present, every
hot-path op raises.  The library is loaded from this package's ``_lib`` directory
(built in-tree by ``__graft_entry__.build()`` / ``make -C kaolin-windows_amd/csrc``).
"""
import ctypes
import os

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib')
# KAOLIN_HIP_LIB points at another build of the same library (development builds, e.g.
# `make STAMPS=1 OUT=...`); the default is the in-tree build
LIB_PATH = os.environ.get('KAOLIN_HIP_LIB') or os.path.join(_LIB_DIR, 'libkaolin_hip.so')

ABI_VERSION = 4  # include/kaolin_hip.h KL_ABI_VERSION: the signatures below

KL_F32, KL_F64, KL_F16, KL_U8, KL_I8, KL_I16, KL_I32, KL_I64 = range(8)
_DTYPES = {
    torch.float32: KL_F32, torch.float64: KL_F64, torch.float16: KL_F16, torch.uint8: KL_U8,
    torch.int8: KL_I8, torch.int16: KL_I16, torch.int32: KL_I32, torch.int64: KL_I64,
}

ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float
_SZ = ctypes.c_size_t
_PP = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    'kl_last_error': (ctypes.c_char_p, []),
    'kl_abi_version': (_I, []),
    'kl_stream_is_capturing': (_I, [_P]),
    'kl_loss_dot2_workspace_bytes': (ctypes.c_size_t, []),
    'kl_loss_dot2': (_I, [_P, _P, _I64, _P, _P, _I64, _P, _P, _P]),
    'kl_rasterize_workspace_bytes': (_SZ, [_I, _I, _I, _I64]),
    'kl_packed_rasterize_forward': (_I, [_I, _I, _I, _I, _I64, _I, _I64, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P,
                                         _SZ, _P]),
    'kl_rasterize_backward_workspace_bytes': (_SZ, [_I, _I, _I]),
    'kl_rasterize_backward': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _P, _P, _P, _SZ, _P]),
    'kl_dibr_rasterize_bwd_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'kl_soft_mask_backward_workspace_bytes': (_SZ, [_I, _I]),
    'kl_dibr_rasterize_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'kl_dibr_rasterize_forward': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _SZ,
                                       _P]),
    'kl_dibr_rasterize_backward': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P,
                                        _P, _P, _SZ, _P]),
    'kl_soft_mask_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'kl_dibr_soft_mask_forward_fused': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _F, ctypes.c_double, _F, _P, _P, _P,
                                             _P, _P, _P, _SZ, _P]),
    'kl_dibr_soft_mask_backward_fused': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P,
                                              _P, _SZ, _P]),
    'kl_soft_mask_compact_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'kl_soft_mask_compact_records': (_SZ, [_I, _I, _I, _I]),
    'kl_soft_mask_compact_segments': (_SZ, [_I, _I, _I]),
    'kl_soft_mask_compact_bwd_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'kl_dibr_soft_mask_forward_compact': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _F, ctypes.c_double, _F, _P, _P, _P,
                                               _P, _P, _P, _P, _SZ, _P]),
    'kl_dibr_soft_mask_backward_compact': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P, _I,
                                                _P, _P, _SZ, _P]),
    'kl_dibr_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'kl_dibr_bwd_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'kl_dibr_state_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'kl_dibr_soft_acc_bytes': (_SZ, [_I, _I]),
    'kl_dibr_forward': (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _F, ctypes.c_double, _F, _F, _P, _P, _P,
                             _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_dibr_backward': (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F,
                              _F, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_dibr_soft_mask_forward': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_dibr_soft_mask_backward': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _SZ,
                                        _P]),
    'kl_prepare_vertices_forward': (_I, [_I, _I, _I, _I, _I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    'kl_prepare_vertices_bwd_workspace_bytes': (_SZ, [_I, _I64]),
    'kl_prepare_vertices_backward': (_I, [_I, _I, _I, _I, _I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                          _P, _P, _P, _SZ, _P]),
    'kl_unbatched_triangle_distance_workspace_bytes': (_SZ, [_I64, _I64]),
    'kl_unbatched_triangle_distance_forward': (_I, [_I, _I64, _I64, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_unbatched_triangle_distance_bwd_workspace_bytes': (_SZ, [_I64]),
    'kl_unbatched_triangle_distance_backward': (_I, [_I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_unbatched_triangle_distance_backward_sums': (_I, [_I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    'kl_sided_distance_forward': (_I, [_I, _I, _I64, _I64, _P, _P, _P, _P, _P]),
    'kl_sided_distance_backward': (_I, [_I, _I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P]),
    'kl_sided_distance_backward_sums': (_I, [_I, _I, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    'kl_mesh_to_spc': (_I, [_I64, _P, ctypes.c_uint32, ALLOC_FN, _P, _PP, ctypes.POINTER(_I64), _PP, _PP,
                            ctypes.POINTER(_I64), _P]),
    'kl_mesh_to_spc_level_counts': (_I, [_P, _I]),
    'kl_mesh_to_spc_fixed_workspace_bytes': (_SZ, [_I64]),
    'kl_mesh_to_spc_fixed': (_I, [_I64, _P, ctypes.c_uint32, _I64, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_morton_to_octree': (_I, [_I64, _P, ctypes.c_uint32, ALLOC_FN, _P, _PP, ctypes.POINTER(_I64), _P]),
    'kl_scan_octrees': (_I, [_I, _P, _P, _P, _P, ctypes.POINTER(_I), _P]),
    'kl_generate_points': (_I, [_I, _I, _P, _P, _P, _P, _P]),
    'kl_points_to_morton': (_I, [_I64, _P, _P, _P]),
    'kl_morton_to_points': (_I, [_I64, _P, _P, _P]),
    'kl_raytrace_fixed_workspace_bytes': (_SZ, [_I64, _I64, _I]),
    'kl_raytrace_fixed': (_I, [_P, _P, _P, _P, _P, _I64, ctypes.c_uint32, _I, _I, _I64, _P, _P, _P, _P, _SZ, _P]),
    'kl_generate_primary_rays': (_I, [ctypes.c_uint32, ctypes.c_uint32, _P, _P, _P, _F, _P, _P, _P, _P]),
    'kl_generate_shadow_rays_workspace_bytes': (_SZ, [_I64]),
    'kl_generate_shadow_rays': (_I, [_I64, _P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(_I64), _P, _SZ, _P]),
    'kl_raytrace': (_I, [_P, _I64, _P, _I64, _P, _I, _P, _P, _I64, ctypes.c_uint32, _I, _I, ALLOC_FN, _P, _PP, _PP,
                         ctypes.POINTER(_I64), _P]),
    'kl_mark_pack_boundaries': (_I, [_I, _I64, _P, _P, _P]),
    'kl_pack_diff': (_I, [_I, _I64, _I64, _P, _P, _I64, _P, _P]),
    'kl_pack_cumsum': (_I, [_I, _I64, _I64, _P, _P, _I64, _I, _I, _P, _P]),
    'kl_pack_cumprod': (_I, [_I, _I64, _I64, _P, _P, _I64, _I, _I, _P, _P]),
    'kl_inclusive_sum_workspace_bytes': (_SZ, [_I64]),
    'kl_inclusive_sum_i32': (_I, [_I64, _P, _P, _P, _SZ, _P]),
    'kl_sum_reduce': (_I, [_I, _I64, _I64, _P, _P, _I64, _P, _P]),
    'kl_deftet_workspace_bytes': (_SZ, [_I64, _I64]),
    'kl_deftet_sparse_render_forward': (_I, [_I, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P,
                                             _P, _SZ, ALLOC_FN, _P, _P]),
    'kl_deftet_sparse_render_resolve': (_I, [_I, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                                             _P]),
    'kl_deftet_bwd_workspace_bytes': (_SZ, [_I64, _I64, _I64, _I64]),
    'kl_deftet_sparse_render_backward': (_I, [_I, _I64, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _F, _P, _P,
                                              _P, _SZ, _P]),
    'kl_unbatched_mesh_intersection': (_I, [_I, _I64, _I64, _P, _P, _P, _P, _P, _P, _SZ, ALLOC_FN, _P, _P]),
    'kl_check_sign_workspace_bytes': (_SZ, [_I, _I64, _I64, _I64]),
    'kl_check_sign': (_I, [_I, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _SZ, ALLOC_FN, _P, _P]),
    'kl_voxelgrid_mark': (_I, [_I64, _P, _I64, _P, _I, _I, _P, ALLOC_FN, _P, _P]),
    'kl_voxelgrid_bounds_workspace_bytes': (_SZ, [_I]),
    'kl_voxelgrid_bounds': (_I, [_I, _I, _I64, _P, _P, _P, _P, _SZ, _P]),
    'kl_voxelgrid_mark_f64': (_I, [_I64, _P, _I64, _P, _I, _I, _P, ALLOC_FN, _P, _P]),
    'kl_voxelgrid_mark_async_workspace_bytes': (_SZ, [_I, _I64]),
    'kl_voxelgrid_mark_async': (_I, [_I, _I64, _P, _I64, _P, _I, _I, _P, _I64, _P, _P, _SZ, _P]),
    'kl_voxelgrid_async': (_I, [_I, _I64, _P, _P, _P, _I64, _P, _I, _I, _P, _I64, _P, _P, _SZ, _P]),
    'kl_texture_mapping_forward': (_I, [_I, _I, _I, _I64, _I, _I, _I, _P, _P, _P, _P]),
    'kl_texture_mapping_bwd_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'kl_texture_mapping_backward': (_I, [_I, _I, _I, _I64, _I, _I, _I, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_mask_iou_workspace_bytes': (_SZ, [_I, _I64]),
    'kl_mask_iou_forward': (_I, [_I, _I, _I64, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'kl_mask_iou_backward': (_I, [_I, _I, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
}


def lib():
    """Load (once) and return the ctypes handle.  Raises if the library is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f'kaolin HIP library not found at {LIB_PATH}; build it with '
                '`make -C kaolin-windows_amd/csrc` (hipcc --offload-arch=gfx950)')
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        got = handle.kl_abi_version()
        if got != ABI_VERSION:
            raise RuntimeError(f'kaolin HIP library at {LIB_PATH} has ABI version {got}, this package expects '
                               f'{ABI_VERSION}; rebuild it with `make -C kaolin-windows_amd/csrc`')
        _lib = handle
    return _lib


def exported_symbols():
    return list(_SIGS)


def dtype_code(dtype):
    try:
        return _DTYPES[dtype]
    except KeyError:
        raise RuntimeError(f'dtype {dtype} is not supported by the kaolin HIP library') from None


def check(rc, func):
    if rc != 0:
        msg = lib().kl_last_error().decode(errors='replace')
        raise RuntimeError(f'{func}: {msg} (kaolin HIP error {rc})')


def ptr(t):
    """Device pointer of a tensor for a c_void_p argument (a plain int: ctypes converts it)."""
    return t.data_ptr() if t is not None else None


_raw_stream = torch._C._cuda_getCurrentRawStream


def stream_of(device):
    """The current HIP stream of `device` as a pointer-sized int (the raw handle: no Stream object)."""
    idx = device.index
    return _raw_stream(torch.cuda.current_device() if idx is None else idx)


def capturing(device):
    """True while `device`'s current stream is being captured into a graph: the entries that
    size outputs or lists on the host then take their capturable form (no allocator, nothing
    read back)."""
    return device.type == 'cuda' and torch.cuda.is_current_stream_capturing()


_SIZES = {}


def size(name, *args):
    """A `kl_*_bytes` / `kl_*_records` size query, memoised by its arguments (pure functions of the
    shapes: the eager step asks the same ones every call)."""
    key = (name,) + args
    v = _SIZES.get(key)
    if v is None:
        v = _SIZES[key] = int(getattr(lib(), name)(*args))
    return v


_WS = {}


def workspace(nbytes, device):
    """Scratch for one library call, reused across calls on the same (device, stream): every entry
    point treats its workspace as uninitialised and is done with it when the stream reaches the
    call's end, so stream order makes reuse safe.  Grows to the largest request; the current
    stream is part of the key (graph capture has its own stream, hence its own buffer)."""
    nbytes = max(int(nbytes), 16)
    if capturing(device):
        # a captured call gets its own buffer from the graph's private memory pool, which the graph
        # keeps for its replays: graphs captured on one stream do not share scratch (concurrent
        # replays), and a later, larger request cannot free memory an earlier graph points at
        return torch.empty(nbytes, dtype=torch.uint8, device=device)
    key = (device.index, stream_of(device))
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _WS[key] = t
    return t


_ZK = {}


def zero_kept(nbytes, device):
    """A buffer that is zero whenever the stream reaches a call that uses it, and that the call
    leaves zero (kl_dibr_backward's soft accumulator): zeroed once when allocated, one per
    (device, stream), grown to the largest request.  A call being captured into a graph gets its
    own buffer from the graph's pool, zeroed by a fill recorded in the graph."""
    nbytes = max(int(nbytes), 16)
    if capturing(device):
        return torch.zeros(nbytes, dtype=torch.uint8, device=device)
    key = (device.index, stream_of(device))
    t = _ZK.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        _ZK[key] = t
    return t


def require_gpu(func, *tensors):
    """The HIP path is the only path: CPU tensors or a missing device raise."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f'In {func}: kaolin-mi355x runs only on GPU tensors '
                               f'(got a {t.device} tensor); there is no CPU fallback')
    lib()


class Arena:
    """Device allocator handed to the C ABI for data-dependent outputs: every request
    becomes a torch uint8 tensor (caching allocator, current stream)."""

    def __init__(self, device):
        self.device = device
        self.by_ptr = {}
        self._cb = ALLOC_FN(self._alloc)

    def _alloc(self, ctx, nbytes):
        try:
            t = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)
        except Exception:  # pragma: no cover - OOM inside a C callback
            return None
        p = t.data_ptr()
        self.by_ptr[p] = t
        return p

    @property
    def fn(self):
        return self._cb

    def tensor(self, p, numel, dtype, shape):
        """View of an arena allocation as a typed tensor of `shape` (numel elements); p may point inside
        an allocation (several outputs carved from one request, r06)."""
        if numel == 0:
            return torch.empty(shape, dtype=dtype, device=self.device)
        esize = torch.empty((), dtype=dtype).element_size()
        base = self.by_ptr.get(p)
        if base is None:
            for q, t in self.by_ptr.items():
                if q <= p < q + t.numel():
                    base = t[p - q:]
                    break
        return base[:numel * esize].view(dtype).reshape(shape)


# ----------------------------------------------------------------- op timing
class OpTimer:
    """HIP-event timing of every native op call on the stream it is launched on
    (enabled by bench.py over its timed region)."""

    def __init__(self):
        self.records = {}

    def add(self, name, start, end):
        self.records.setdefault(name, []).append((start, end))

    def summary_ms(self):
        torch.cuda.synchronize()
        return {k: sum(s.elapsed_time(e) for s, e in v) / len(v) for k, v in self.records.items()}

    def counts(self):
        return {k: len(v) for k, v in self.records.items()}


_TIMER = None


def set_timer(timer):
    global _TIMER
    _TIMER = timer


class _NullCtx:
    __slots__ = ()

    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL = _NullCtx()


class _Timed:
    __slots__ = ('name', 'st', 'e')

    def __init__(self, name, device):
        self.name, self.st = name, torch.cuda.current_stream(device)

    def __enter__(self):
        s = torch.cuda.Event(enable_timing=True)
        self.e = (s, torch.cuda.Event(enable_timing=True))
        s.record(self.st)

    def __exit__(self, *exc):
        self.e[1].record(self.st)
        _TIMER.add(self.name, *self.e)
        return False


def timed(name, device):
    """HIP-event timing of the op on its stream while bench.py's timer is set; a shared no-op
    context otherwise (the per-call cost of the eager path)."""
    return _NULL if _TIMER is None else _Timed(name, device)


def on_device(device):
    """torch.cuda.device(device), skipped when it is already the current device."""
    idx = device.index
    if idx is None or idx == torch.cuda.current_device():
        return _NULL
    return torch.cuda.device(device)
