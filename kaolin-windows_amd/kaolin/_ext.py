"""The compiled autograd nodes (csrc/torch_ops.cpp), built in-tree as a torch C++ extension over
the C ABI library.  Plumbing for the eager host path only: the same kl_* entry points as the
ctypes route (kaolin/_fused.py), with at::empty allocations and no Python in the backward.

build() compiles it (g++ via torch.utils.cpp_extension, no GPU needed); get() imports it, or
returns None when it is absent -- the front-ends then take the ctypes route, which calls the same
HIP library (there is no CPU fallback either way).
"""
import importlib.util
import os

from . import _native as N

NAME = 'kaolin_mi355x_ops'
_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_HERE, '_lib', 'ext')
_CSRC = os.path.join(os.path.dirname(_HERE), 'csrc')
_INCLUDE = os.path.join(os.path.dirname(os.path.dirname(_HERE)), 'include')

_mod = False  # not yet looked up


def build(verbose=False):
    from torch.utils.cpp_extension import load
    os.makedirs(BUILD_DIR, exist_ok=True)
    lib_dir = os.path.dirname(N.LIB_PATH)
    return load(name=NAME, sources=[os.path.join(_CSRC, 'torch_ops.cpp')], extra_include_paths=[_INCLUDE],
                extra_cflags=['-O2'], extra_ldflags=[f'-L{lib_dir}', '-lkaolin_hip', f'-Wl,-rpath,{lib_dir}'],
                build_directory=BUILD_DIR, verbose=verbose)


def get():
    """The extension module, or None (not built / not loadable here)."""
    global _mod
    if _mod is False:
        _mod = None
        path = os.path.join(BUILD_DIR, NAME + '.so')
        if os.path.exists(path) and os.environ.get('KAOLIN_NO_EXT') != '1':
            N.lib()  # the ABI check first
            try:
                spec = importlib.util.spec_from_file_location(NAME, path)
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                if mod.abi_version() == N.ABI_VERSION:
                    _mod = mod
            except ImportError:
                _mod = None
    return _mod
