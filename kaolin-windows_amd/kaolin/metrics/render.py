"""mask_iou (kaolin/metrics/render.py:18-40): the silhouette loss used with dibr_soft_mask.

GPU f32 / f64 masks take the fused HIP path (csrc/maskiou.hip: one pass for both per-mask sums,
one for both gradients); other inputs run the reference's torch ops."""
import torch
from torch.autograd import Function

from .. import _ext, _native as N


class MaskIouHip(Function):
    """mask_iou forward and backward as one HIP pass each (kl_mask_iou_forward / _backward): the
    sums in double, rounded once; the gradients autograd's through the reference's ops."""

    @staticmethod
    def forward(ctx, lhs_mask, rhs_mask):
        B = lhs_mask.shape[0]
        lhs, rhs = lhs_mask.contiguous(), rhs_mask.contiguous()
        n = lhs.numel() // B
        dev = lhs.device
        up = torch.empty((B,), dtype=lhs.dtype, device=dev)
        down = torch.empty((B,), dtype=lhs.dtype, device=dev)
        loss = torch.empty((), dtype=lhs.dtype, device=dev)
        nbytes = N.size('kl_mask_iou_workspace_bytes', B, n)
        ws = N.workspace(nbytes, dev)
        with N.on_device(dev), N.timed('mask_iou', dev):
            N.check(N.lib().kl_mask_iou_forward(N.dtype_code(lhs.dtype), B, n, N.ptr(lhs), N.ptr(rhs), N.ptr(up),
                                                N.ptr(down), N.ptr(loss), N.ptr(ws), nbytes, N.stream_of(dev)),
                    'mask_iou')
        ctx.save_for_backward(lhs_mask, rhs_mask, up, down)  # the inputs themselves (double backward)
        return loss

    @staticmethod
    def backward(ctx, grad):
        lhs, rhs, up, down = ctx.saved_tensors
        if torch.is_grad_enabled():  # create_graph: the reference's torch gradient, differentiable
            from .._double_backward import mask_iou as dd
            return tuple(dd(lhs, rhs, grad))
        lhs, rhs = lhs.contiguous(), rhs.contiguous()
        need_l, need_r = ctx.needs_input_grad
        gl = torch.empty_like(lhs) if need_l else None
        gr = torch.empty_like(rhs) if need_r else None
        if gl is None and gr is None:
            return None, None
        B = lhs.shape[0]
        dev = lhs.device
        with N.on_device(dev):
            N.check(N.lib().kl_mask_iou_backward(N.dtype_code(lhs.dtype), B, lhs.numel() // B,
                                                 N.ptr(grad.contiguous()), N.ptr(lhs), N.ptr(rhs), N.ptr(up),
                                                 N.ptr(down), N.ptr(gl), N.ptr(gr), N.stream_of(dev)),
                    'mask_iou backward')
        return gl, gr


def mask_iou(lhs_mask, rhs_mask):
    r"""Intersection over union loss of two (B, H, W) masks: 1 - mean over the batch of
    sum(lhs * rhs) / (sum(lhs + rhs - lhs * rhs) + 1e-10)."""
    batch_size, height, width = lhs_mask.shape
    assert rhs_mask.shape == lhs_mask.shape
    if (lhs_mask.is_cuda and rhs_mask.device == lhs_mask.device and lhs_mask.dtype == rhs_mask.dtype
            and lhs_mask.dtype in (torch.float32, torch.float64) and lhs_mask.numel() > 0):
        ext = _ext.get()
        if ext is not None and N._TIMER is None and lhs_mask.device.index == torch.cuda.current_device():
            return ext.mask_iou(lhs_mask, rhs_mask, N.stream_of(lhs_mask.device))  # the node compiled
        return MaskIouHip.apply(lhs_mask, rhs_mask)
    return _mask_iou_torch(lhs_mask, rhs_mask)


def _mask_iou_torch(lhs_mask, rhs_mask):
    """The reference's torch ops (render.py:34-37)."""
    batch_size = lhs_mask.shape[0]
    sil_mul = lhs_mask * rhs_mask
    sil_add = lhs_mask + rhs_mask
    iou_up = torch.sum(sil_mul.reshape(batch_size, -1), dim=1)
    iou_down = torch.sum((sil_add - sil_mul).reshape(batch_size, -1), dim=1)
    iou_neg = iou_up / (iou_down + 1e-10)
    return 1.0 - torch.mean(iou_neg)
