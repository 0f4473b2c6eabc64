"""Argument checks with the reference's messages.

The reference validates in C++ with ATen's TensorUtils (``at::checkSize``,
``at::checkAllContiguous``, ``at::checkSameType``, ``at::checkAllSameGPU``) keyed by
``TensorArg{tensor, "name", position}`` and the ``__func__`` of the binding
(e.g. rasterization.cpp:60-85, sided_distance.cpp:68-80).  Tests match these
messages verbatim (tests/python/kaolin/metrics/test_pointcloud.py:124-152), so they
are reproduced here.
"""
import torch


class Arg:
    __slots__ = ('t', 'name', 'pos')

    def __init__(self, t, name, pos):
        self.t, self.name, self.pos = t, name, pos

    def __str__(self):
        return f"argument #{self.pos} '{self.name}'"


def _shape(t):
    return '[' + ', '.join(str(s) for s in t.shape) + ']'


def check_dim(func, a, dim):
    if a.t.dim() != dim:
        raise RuntimeError(f'Expected {dim}-dimensional tensor, but got {a.t.dim()}-dimensional tensor for {a} '
                           f'(while checking arguments for {func})')


def check_size(func, a, sizes):
    check_dim(func, a, len(sizes))
    if list(a.t.shape) != [int(s) for s in sizes]:
        exp = '[' + ', '.join(str(int(s)) for s in sizes) + ']'
        raise RuntimeError(f'Expected tensor of size {exp}, but got tensor of size {_shape(a.t)} for {a} '
                           f'(while checking arguments for {func})')


def check_size_dim(func, a, dim, size):
    if a.t.shape[dim] != size:
        raise RuntimeError(f'Expected tensor to have size {size} at dimension {dim}, but got size '
                           f'{a.t.shape[dim]} for {a} (while checking arguments for {func})')


def check_contiguous(func, args):
    for a in args:
        if not a.t.is_contiguous():
            raise RuntimeError(f'Expected contiguous tensor, but got non-contiguous tensor for {a} '
                               f'(while checking arguments for {func})')


def check_same_type(func, a, b):
    if a.t.dtype != b.t.dtype:
        raise RuntimeError(f'Expected tensor for {a} to have the same type as tensor for {b}; but type '
                           f'{a.t.dtype} does not equal {b.t.dtype} (while checking arguments for {func})')


def check_same_size(func, a, b):
    if a.t.shape != b.t.shape:
        raise RuntimeError(f'Expected tensor for {a} to have same size as tensor for {b}; but {_shape(a.t)} '
                           f'does not equal {_shape(b.t)} (while checking arguments for {func})')


def check_all_same_gpu(func, args):
    for a in args:
        if not a.t.is_cuda:
            raise RuntimeError(f'Tensor for {a} is on CPU, but expected it to be on GPU '
                               f'(while checking arguments for {func})')
    if args:
        d0 = args[0].t.device
        for a in args[1:]:
            if a.t.device != d0:
                raise RuntimeError(f'Expected tensor for {args[0]} to have the same device as tensor for {a}; '
                                   f'but device {d0.index} does not equal {a.t.device.index} '
                                   f'(while checking arguments for {func})')


def check_dtype(func, name, t, allowed):
    if t.dtype not in allowed:
        raise RuntimeError(f'"{func}" not implemented for \'{str(t.dtype).replace("torch.", "").capitalize()}\'')


def device_guard(t):
    return torch.cuda.device(t.device)
