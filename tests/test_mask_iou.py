"""mask_iou (kaolin/metrics/render.py:18-40) -- the DIB-R tutorial's silhouette loss.

GPU f32 / f64 masks run csrc/maskiou.hip.  The oracle is the reference's own torch ops: the loss
against them in float64 (the HIP sums are exact-in-double and rounded once, torch's float sums
round per partial), and the gradients bit for bit against autograd's formula through the
reference's ops evaluated on the HIP path's own per-mask sums.
"""
import pytest
import torch

DEV = 'cuda'


def _ref(lhs, rhs):
    b = lhs.shape[0]
    sil_mul = lhs * rhs
    sil_add = lhs + rhs
    up = torch.sum(sil_mul.reshape(b, -1), dim=1)
    down = torch.sum((sil_add - sil_mul).reshape(b, -1), dim=1)
    return 1.0 - torch.mean(up / (down + 1e-10))


def _inputs(dtype, dev, B=4, H=67, W=91, seed=0):
    g = torch.Generator().manual_seed(seed)
    lhs = torch.rand((B, H, W), generator=g, dtype=torch.float64)
    lhs[0, :3] = 0.
    lhs[1, 5:9] = 1.
    rhs = (torch.rand((B, H, W), generator=g) > 0.5).double()
    return lhs.to(dtype).to(dev), rhs.to(dtype).to(dev)


def test_cpu_tensors_take_the_reference_ops():
    import kaolin as kal
    lhs, rhs = _inputs(torch.float32, 'cpu')
    assert torch.equal(kal.metrics.render.mask_iou(lhs, rhs), _ref(lhs, rhs))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_forward_and_grads(dtype, monkeypatch):
    import kaolin as kal
    from kaolin import _ext
    # the Python node (its saved sums are read below); the compiled node (csrc/torch_ops.cpp) is
    # tested bit-equal to it in test_gpu_parity.py::test_compiled_tutorial_nodes_equal_python_nodes
    monkeypatch.setattr(_ext, '_mod', None)
    lhs, rhs = _inputs(dtype, DEV)
    a, b = lhs.clone().requires_grad_(True), rhs.clone().requires_grad_(True)
    loss = kal.metrics.render.mask_iou(a, b)
    assert loss.grad_fn is not None and 'MaskIouHip' in type(loss.grad_fn).__name__
    ref64 = _ref(lhs.double(), rhs.double())
    tol = 2e-7 if dtype == torch.float32 else 1e-14
    assert abs(float(loss.detach()) - float(ref64)) <= tol * max(1.0, abs(float(ref64)))
    assert abs(float(_ref(lhs, rhs)) - float(ref64)) <= 4 * tol * max(1.0, abs(float(ref64)))  # torch's own
    _, _, hup, hdown = [t.clone() for t in loss.grad_fn.saved_tensors]
    g = torch.tensor(0.731, dtype=dtype, device=DEV)
    loss.backward(g)
    # autograd's formula through the reference's ops, on the HIP path's own sums
    B = lhs.shape[0]
    up = torch.sum((lhs * rhs).double().reshape(B, -1), 1)
    gin = (-g) / B
    den = hdown + 1e-10
    gup = gin / den
    gden = -gin * ((hup / den) / den)
    assert torch.equal(a.grad, (gup - gden)[:, None, None] * rhs + gden[:, None, None])
    assert torch.equal(b.grad, (gup - gden)[:, None, None] * lhs + gden[:, None, None])
    # the sums: the dtype's products summed in double, rounded once
    torch.testing.assert_close(hup, up.to(dtype), rtol=1.2e-7 if dtype == torch.float32 else 1e-15, atol=0)
    # and the gradients agree with torch's autograd through its own float sums
    a2, b2 = lhs.clone().requires_grad_(True), rhs.clone().requires_grad_(True)
    _ref(a2, b2).backward(g)
    torch.testing.assert_close(a.grad, a2.grad, rtol=1e-5 if dtype == torch.float32 else 1e-12, atol=1e-9)
    torch.testing.assert_close(b.grad, b2.grad, rtol=1e-5 if dtype == torch.float32 else 1e-12, atol=1e-9)


@pytest.mark.gpu
def test_only_lhs_requires_grad_and_graph_capture():
    """The tutorial's call: the soft mask requires grad, the target does not; capturable."""
    import kaolin as kal
    lhs, rhs = _inputs(torch.float32, DEV, B=2, H=64, W=48, seed=3)
    a = lhs.clone().requires_grad_(True)
    kal.metrics.render.mask_iou(a, rhs).backward()
    g1 = a.grad.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    static_a = lhs.clone().requires_grad_(True)
    with torch.cuda.stream(s):
        kal.metrics.render.mask_iou(static_a, rhs).backward()
    torch.cuda.current_stream().wait_stream(s)
    static_a.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = kal.metrics.render.mask_iou(static_a, rhs)
        out.backward()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(static_a.grad, g1)
