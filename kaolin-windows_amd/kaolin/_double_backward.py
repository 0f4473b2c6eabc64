"""Second-order gradients of the HIP nodes whose reference is plain torch.

The reference computes mask_iou (metrics/render.py:34-37), prepare_vertices (render/mesh/utils.py:
160-175) and texture_mapping (render/mesh/utils.py:64-75) with torch ops, so its gradients can be
differentiated again (``backward(create_graph=True)``: gradient penalties, Hessian-vector
products).  The HIP nodes' backward is one opaque call each; when the autograd engine runs it
with grad mode on (create_graph), the nodes call these functions instead, which take the first
derivative of the reference's own torch chain with ``create_graph=True`` -- the reference's
gradient, itself differentiable.  The plain backward (create_graph=False) never comes here.
"""
import torch

__all__ = ['mask_iou', 'prepare_vertices', 'texture_mapping']


def _grads(out, inputs, grad_outputs):
    """d out / d inputs (None where an input needs none), with the graph kept."""
    live = [x for x in inputs if x is not None and x.requires_grad]
    if not live:
        return [None] * len(inputs)
    got = iter(torch.autograd.grad(out, live, grad_outputs, create_graph=True, allow_unused=True))
    return [next(got) if x is not None and x.requires_grad else None for x in inputs]


def mask_iou(lhs, rhs, grad):
    from .metrics.render import _mask_iou_torch
    return _grads([_mask_iou_torch(lhs, rhs)], [lhs, rhs], [grad])


def prepare_vertices(vertices, faces, proj, rot, trans, xf, g_fvc, g_fvi, g_fn):
    from .render.mesh.utils import _prepare_vertices_torch
    outs = _prepare_vertices_torch(vertices, faces, proj, rot, trans, xf)
    keep = [(o, g) for o, g in zip(outs, (g_fvc, g_fvi, g_fn)) if g is not None]
    if not keep:
        return [None] * 6
    return _grads([o for o, _ in keep], [vertices, None, proj, rot, trans, xf], [g for _, g in keep])


def texture_mapping(coords, tex, mode, grad):
    from .render.mesh.utils import _texture_mapping_torch
    out = _texture_mapping_torch(coords, tex, 'bilinear' if mode == 1 else 'nearest')
    return _grads([out], [coords, tex], [grad.reshape(out.shape)])
