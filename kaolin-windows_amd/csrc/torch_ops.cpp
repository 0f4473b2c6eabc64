// torch_ops.cpp -- the eager host path of dibr_rasterization (and of the tutorial loop's other
// library ops: prepare_vertices, mask_iou, texture_mapping) as compiled autograd nodes.
//
// The reference's native layer is a compiled extension (kaolin/csrc/bindings.cpp); its Python
// front-end (render/mesh/dibr.py:119-209) pays one autograd Function per op.  The ctypes route of
// kaolin/_fused.py costs ~45 us of Python per direction at cfg3 (13 output allocations, ~30
// ctypes arguments, the autograd Function's Python forward and backward) -- as much as the GPU
// work on a slow host.  This file is the same DibrRasterizationCuda node in C++: at::empty for the
// outputs and the compact soft-mask state, the C ABI (include/kaolin_hip.h) called directly, the
// backward run by the autograd engine without re-entering Python.  Results are those of
// kl_dibr_forward / kl_dibr_backward, i.e. bit-identical to the Python path
// (tests/test_gpu_parity.py::test_compiled_node_equals_python_node).
//
// Plumbing only: no torch types cross the C ABI; the stream is the caller's current HIP stream,
// passed in as a handle (torch._C._cuda_getCurrentRawStream) and kept for the backward, which the
// autograd engine runs on the forward's stream.
#include <torch/extension.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "kaolin_hip.h"

namespace {

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

void check(int rc, const char *func) {
  if (rc != 0) throw std::runtime_error(std::string(func) + ": " + kl_last_error() + " (kaolin HIP error " +
                                        std::to_string(rc) + ")");
}

kl_dtype dtype_code(at::ScalarType t) {
  if (t == at::kFloat) return KL_F32;
  if (t == at::kDouble) return KL_F64;
  throw std::runtime_error("kaolin compiled node: f32 / f64 only");
}

// scratch reused across calls on one (device, stream), grown to the largest request: every entry
// point treats its workspace as uninitialised and is done with it when the stream reaches the
// call's end (the Python path's _native.workspace).  A call being captured into a graph gets its
// own buffer from the graph's memory pool instead (graphs replayed concurrently do not share it,
// and a later, larger request cannot free what a graph points at).
at::Tensor workspace(size_t bytes, const at::Device &dev, int64_t stream) {
  if (kl_stream_is_capturing((kl_stream)stream))
    return at::empty({(int64_t)std::max<size_t>(bytes, 16)}, at::TensorOptions().dtype(at::kByte).device(dev));
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, at::Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  at::Tensor &t = cache[{dev.index(), stream}];
  const int64_t need = (int64_t)std::max<size_t>(bytes, 16);
  if (!t.defined() || t.numel() < need) t = at::empty({need}, at::TensorOptions().dtype(at::kByte).device(dev));
  return t;
}

// a buffer that is zero whenever the stream reaches a call that uses it, and that the call leaves
// zero (kl_dibr_backward's soft accumulator): zeroed once when allocated, per (device, stream);
// a captured call gets its own, zeroed by a fill recorded in the graph (_native.zero_kept)
at::Tensor zero_kept(size_t bytes, const at::Device &dev, int64_t stream) {
  const int64_t need = (int64_t)std::max<size_t>(bytes, 16);
  if (kl_stream_is_capturing((kl_stream)stream)) return at::zeros({need}, at::TensorOptions().dtype(at::kByte).device(dev));
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, at::Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  at::Tensor &t = cache[{dev.index(), stream}];
  if (!t.defined() || t.numel() < need) t = at::zeros({need}, at::TensorOptions().dtype(at::kByte).device(dev));
  return t;
}

void *ptr(const at::Tensor &t) { return t.defined() ? t.data_ptr() : nullptr; }

// Each node's backward is one opaque HIP call, so its gradients cannot be differentiated again.
// dibr_rasterization (whose reference backward is a CUDA kernel too) raises under create_graph
// (grad mode on inside the backward) rather than hand back gradients that silently drop its
// second-order term.  The nodes whose reference is plain torch (mask_iou, prepare_vertices,
// texture_mapping) instead take the reference chain's own differentiable gradient then
// (the *_chain functions below), as the reference would give.
void no_double_backward(const char *op) {
  TORCH_CHECK(!at::GradMode::is_enabled(), op,
              ": backward with create_graph=True is not supported (the backward is one HIP call and is not "
              "differentiable)");
}

// The reference's torch chains (kaolin/_double_backward.py restates them for the Python nodes), in
// ATen ops: the same kernels the Python front-ends' torch fallbacks dispatch to, so the gradients
// taken through them are the reference's.  No Python here: the backward runs on the autograd
// engine's device thread.
// Every op is its own statement, in the order Python evaluates the reference's expressions: the
// autograd engine orders the adds of a tensor's gradients by node creation order, and C++ leaves
// the order of a call's argument expressions unspecified.
at::Tensor mask_iou_chain(const at::Tensor &lhs, const at::Tensor &rhs) {  // metrics/render.py:34-37
  const int64_t B = lhs.size(0);
  const at::Tensor sil_mul = lhs * rhs;
  const at::Tensor sil_add = lhs + rhs;
  const at::Tensor up = at::sum(sil_mul.reshape({B, -1}), 1);
  const at::Tensor diff = sil_add - sil_mul;
  const at::Tensor down = at::sum(diff.reshape({B, -1}), 1);
  const at::Tensor den = down + 1e-10;
  const at::Tensor iou = up / den;
  return at::rsub(at::mean(iou), 1.0);
}

at::Tensor by_faces(const at::Tensor &x, const at::Tensor &faces) {  // index_vertices_by_faces
  const at::Tensor inp = x.unsqueeze(2).expand({-1, -1, faces.size(-1), -1});
  const at::Tensor idx = faces.unsqueeze(0).unsqueeze(-1).expand({x.size(0), -1, -1, x.size(-1)});
  return at::gather(inp, 1, idx);
}

// render/mesh/utils.py:160-175 (rotate_translate_points / pad @ transform, perspective_camera,
// index_vertices_by_faces, face_normals(unit=True))
std::vector<at::Tensor> prepare_chain(const at::Tensor &v, const at::Tensor &faces, const at::Tensor &proj,
                                      const at::Tensor &rot, const at::Tensor &trans, const at::Tensor &xf) {
  at::Tensor vc;
  if (xf.defined()) {
    const at::Tensor padded = at::constant_pad_nd(v, {0, 1}, 1.0);
    vc = at::matmul(padded, xf);
  } else {
    const at::Tensor tv = trans.view({-1, 1, 3});
    const at::Tensor translated = v - tv;
    const at::Tensor rt = rot.permute({0, 2, 1});
    vc = at::matmul(translated, rt);
  }
  const at::Tensor pv = proj.view({-1, 1, 3});
  const at::Tensor pp = vc * pv;
  const at::Tensor pxy = pp.slice(2, 0, 2);
  const at::Tensor pz = pp.slice(2, 2, 3);
  const at::Tensor vi = pxy / pz;
  const at::Tensor fvc = by_faces(vc, faces);
  const at::Tensor fvi = by_faces(vi, faces);
  const at::Tensor c1 = fvc.select(2, 1);
  const at::Tensor c0 = fvc.select(2, 0);
  const at::Tensor e0 = c1 - c0;
  const at::Tensor c2 = fvc.select(2, 2);
  const at::Tensor c0b = fvc.select(2, 0);
  const at::Tensor e1 = c2 - c0b;
  const at::Tensor n = at::cross(e0, e1, 2);
  const at::Tensor len = at::linalg_vector_norm(n, 2, at::IntArrayRef{2}, true);
  const at::Tensor den = len + 1e-10;
  return {fvc, fvi, n / den};
}

at::Tensor texture_chain(const at::Tensor &coords, const at::Tensor &tex, int64_t mode) {  // utils.py:64-75
  const int64_t B = coords.size(0);
  const at::Tensor cl = at::clamp(coords.reshape({B, -1, 1, 2}), 0., 1.);
  const at::Tensor c2 = cl * 2;
  at::Tensor c = c2 - 1;
  const at::Tensor ny = -c.select(3, 1);
  c.select(3, 1).copy_(ny);
  const at::Tensor out = at::grid_sampler(tex, c, mode == 1 ? 0 : 1, /*border*/ 1, false);
  return out.permute({0, 2, 3, 1}).reshape({B, -1, tex.size(1)});
}

// d outputs / d inputs with the graph kept (create_graph): undefined where an input needs none
variable_list chain_grads(const variable_list &outs, const variable_list &gouts, const variable_list &inputs) {
  variable_list live, o, g;
  for (const auto &x : inputs)
    if (x.defined() && x.requires_grad()) live.push_back(x);
  for (size_t k = 0; k < outs.size(); k++)
    if (gouts[k].defined()) {
      o.push_back(outs[k]);
      g.push_back(gouts[k]);
    }
  variable_list res(inputs.size());
  if (live.empty() || o.empty()) return res;
  const variable_list got = torch::autograd::grad(o, live, g, /*retain_graph=*/true, /*create_graph=*/true,
                                                  /*allow_unused=*/true);
  size_t j = 0;
  for (size_t k = 0; k < inputs.size(); k++)
    if (inputs[k].defined() && inputs[k].requires_grad()) res[k] = got[j++];
  return res;
}

struct DibrRasterization : public torch::autograd::Function<DibrRasterization> {
  static variable_list forward(AutogradContext *ctx, int64_t height, int64_t width, at::Tensor fvz, at::Tensor fvi,
                               at::Tensor feat, at::Tensor fnz, double sigmainv, double boxlen, int64_t knum,
                               double multiplier, double eps, int64_t stream) {
    fvz = fvz.contiguous();
    fvi = fvi.contiguous();
    feat = feat.contiguous();
    fnz = fnz.detach().contiguous();
    // one dtype for every float input: the kernels read all of them as fvi's type
    TORCH_CHECK(fvz.scalar_type() == fvi.scalar_type() && feat.scalar_type() == fvi.scalar_type() &&
                    fnz.scalar_type() == fvi.scalar_type(),
                "dibr_rasterization: face_vertices_z, face_vertices_image, face_features and face_normals_z must "
                "share one dtype");
    const int64_t B = fvz.size(0), F = fvz.size(1), D = feat.size(-1);
    const int H = (int)height, W = (int)width, K = (int)knum;
    const auto opt = fvi.options();
    const auto dev = fvi.device();
    const kl_dtype dt = dtype_code(fvi.scalar_type());
    at::Tensor feats = at::empty({B, H, W, D}, opt);
    at::Tensor idx = at::empty({B, H, W}, opt.dtype(at::kLong));
    at::Tensor w = at::empty({B, H, W, 3}, opt);
    at::Tensor mask = at::empty({B, H, W}, opt);
    at::Tensor hits = at::empty({B, H, W}, opt.dtype(at::kByte));
    const int64_t nrec = std::max<int64_t>((int64_t)kl_soft_mask_compact_records((int)B, H, W, K), 1);
    at::Tensor rec_face = at::empty({nrec}, opt.dtype(at::kInt));
    at::Tensor rec_prob = at::empty({nrec}, opt);
    at::Tensor seg_tot =
        at::empty({std::max<int64_t>((int64_t)kl_soft_mask_compact_segments((int)B, H, W), 1)}, opt.dtype(at::kInt));
    // the backward's soft-mask work items (written by the forward)
    at::Tensor scratch = at::empty({(int64_t)kl_dibr_state_bytes((int)B, H, W, (int)F, K)}, opt.dtype(at::kByte));
    at::Tensor ranges = at::empty({B, F, 2}, opt.dtype(at::kInt));
    const size_t nbytes = kl_dibr_workspace_bytes((int)B, H, W, (int)F);
    at::Tensor ws = workspace(nbytes, dev, stream);
    check(kl_dibr_forward(dt, (int)B, H, W, (int)F, (int)D, K, ptr(fvz), ptr(fvi), ptr(feat), ptr(fnz), (float)sigmainv,
                          boxlen * multiplier, (float)multiplier, (float)eps, ptr(feats), idx.data_ptr<int64_t>(),
                          ptr(w), ptr(mask), hits.data_ptr<uint8_t>(), (uint32_t *)rec_face.data_ptr(), ptr(rec_prob),
                          seg_tot.data_ptr<int>(), scratch.data_ptr(),
                          F > 0 ? (uint32_t *)ranges.data_ptr() : nullptr, ws.data_ptr(), nbytes,
                          (kl_stream)stream),
          "dibr_rasterization");
    ctx->mark_non_differentiable({idx});
    ctx->set_materialize_grads(false);
    ctx->saved_data["sigmainv"] = sigmainv;
    ctx->saved_data["multiplier"] = multiplier;
    ctx->saved_data["eps"] = eps;
    ctx->saved_data["knum"] = knum;
    ctx->saved_data["stream"] = stream;
    ctx->saved_data["has_ranges"] = F > 0;
    ctx->save_for_backward({idx, w, fvi, feat, fnz, mask, ranges, hits, rec_face, rec_prob, seg_tot, scratch});
    return {feats, mask, idx};
  }

  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const at::Tensor &idx = saved[0], &w = saved[1], &fvi = saved[2], &feat = saved[3], &fnz = saved[4],
                     &mask = saved[5], &ranges = saved[6], &hits = saved[7], &rec_face = saved[8],
                     &rec_prob = saved[9], &seg_tot = saved[10], &scratch = saved[11];
    no_double_backward("dibr_rasterization");
    at::Tensor gf = grads[0], gm = grads[1];
    variable_list out(12);
    if (!gf.defined() && !gm.defined()) return out;
    if (!gf.defined()) gf = at::zeros({idx.size(0), idx.size(1), idx.size(2), feat.size(-1)}, feat.options());
    gf = gf.contiguous();
    if (gm.defined()) gm = gm.contiguous();
    const int64_t B = fvi.size(0), F = fvi.size(1), D = feat.size(-1);
    const int H = (int)idx.size(1), W = (int)idx.size(2), K = (int)ctx->saved_data["knum"].toInt();
    const int64_t stream = ctx->saved_data["stream"].toInt();
    at::Tensor g_img = at::empty_like(fvi);
    at::Tensor g_feat = at::empty_like(feat);
    const size_t nbytes = kl_dibr_bwd_workspace_bytes((int)B, H, W, (int)F, K);
    at::Tensor ws = workspace(nbytes, fvi.device(), stream);
    at::Tensor acc = gm.defined() ? zero_kept(kl_dibr_soft_acc_bytes((int)B, (int)F), fvi.device(), stream) : at::Tensor();
    check(kl_dibr_backward(dtype_code(fvi.scalar_type()), (int)B, H, W, (int)F, (int)D, K, ptr(gf), ptr(gm),
                           idx.data_ptr<int64_t>(), ptr(w), ptr(fvi), ptr(feat), ptr(fnz), ptr(mask),
                           hits.data_ptr<uint8_t>(), (const uint32_t *)rec_face.data_ptr(), ptr(rec_prob),
                           seg_tot.data_ptr<int>(), (float)ctx->saved_data["sigmainv"].toDouble(),
                           (float)ctx->saved_data["multiplier"].toDouble(), (float)ctx->saved_data["eps"].toDouble(),
                           ptr(g_img), ptr(g_feat), scratch.data_ptr(),
                           ctx->saved_data["has_ranges"].toBool() ? (const uint32_t *)ranges.data_ptr() : nullptr,
                           ptr(acc), ws.data_ptr(), nbytes, (kl_stream)stream),
          "dibr_rasterization backward");
    out[3] = g_img;
    out[4] = g_feat;
    return out;
  }
};

// mask_iou (metrics/render.py MaskIouHip): kl_mask_iou_forward / _backward
struct MaskIou : public torch::autograd::Function<MaskIou> {
  static variable_list forward(AutogradContext *ctx, at::Tensor lhs_in, at::Tensor rhs_in, int64_t stream) {
    const at::Tensor lhs = lhs_in.contiguous(), rhs = rhs_in.contiguous();
    const int64_t B = lhs.size(0), n = lhs.numel() / B;
    const auto opt = lhs.options();
    at::Tensor up = at::empty({B}, opt), down = at::empty({B}, opt), loss = at::empty({}, opt);
    const size_t nbytes = kl_mask_iou_workspace_bytes((int)B, n);
    at::Tensor ws = workspace(nbytes, lhs.device(), stream);
    check(kl_mask_iou_forward(dtype_code(lhs.scalar_type()), (int)B, n, ptr(lhs), ptr(rhs), ptr(up), ptr(down),
                              ptr(loss), ws.data_ptr(), nbytes, (kl_stream)stream),
          "mask_iou");
    ctx->saved_data["stream"] = stream;
    ctx->save_for_backward({lhs_in, rhs_in, up, down});  // the inputs themselves (double backward)
    return {loss};
  }
  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const at::Tensor &up = saved[2], &down = saved[3];
    const bool need_l = ctx->needs_input_grad(0), need_r = ctx->needs_input_grad(1);
    variable_list out(3);
    if (!need_l && !need_r) return out;
    at::Tensor g = grads[0].defined() ? grads[0].contiguous() : at::ones({}, saved[0].options());
    if (at::GradMode::is_enabled()) {  // create_graph: the reference's torch gradient
      const auto r = chain_grads({mask_iou_chain(saved[0], saved[1])}, {g}, {saved[0], saved[1]});
      out[0] = r[0];
      out[1] = r[1];
      return out;
    }
    const at::Tensor lhs = saved[0].contiguous(), rhs = saved[1].contiguous();
    at::Tensor gl = need_l ? at::empty_like(lhs) : at::Tensor(), gr = need_r ? at::empty_like(rhs) : at::Tensor();
    const int64_t B = lhs.size(0);
    check(kl_mask_iou_backward(dtype_code(lhs.scalar_type()), (int)B, lhs.numel() / B, ptr(g), ptr(lhs), ptr(rhs),
                               ptr(up), ptr(down), ptr(gl), ptr(gr), (kl_stream)ctx->saved_data["stream"].toInt()),
          "mask_iou backward");
    out[0] = gl;
    out[1] = gr;
    return out;
  }
};

at::Tensor mask_iou(at::Tensor lhs, at::Tensor rhs, int64_t stream) { return MaskIou::apply(lhs, rhs, stream)[0]; }

// prepare_vertices (render/mesh/utils.py PrepareVerticesHip): kl_prepare_vertices_forward / _backward.
// cam_a, cam_b = rot, trans; or xf (camera_transform) twice (has_xf; the second slot gets no
// gradient) -- autograd's apply takes no undefined tensors.  batches (B, Bv, Bc, Bp) as the Python
// front-end computes them.
struct PrepareVertices : public torch::autograd::Function<PrepareVertices> {
  static variable_list forward(AutogradContext *ctx, at::Tensor vertices, at::Tensor faces, at::Tensor proj,
                               at::Tensor cam_a, at::Tensor cam_b, bool has_xf, std::vector<int64_t> batches,
                               int64_t stream) {
    const int64_t B = batches[0], Bv = batches[1], Bc = batches[2], Bp = batches[3];
    at::Tensor verts = vertices.contiguous(), fc = faces.contiguous(), pj = proj.contiguous();
    at::Tensor r = has_xf ? at::Tensor() : cam_a.contiguous(), t = has_xf ? at::Tensor() : cam_b.contiguous();
    at::Tensor x = has_xf ? cam_a.contiguous() : at::Tensor();
    const int64_t V = verts.size(1), F = fc.size(0);
    const auto opt = verts.options();
    at::Tensor fvc = at::empty({B, F, 3, 3}, opt), fvi = at::empty({B, F, 3, 2}, opt), fn = at::empty({B, F, 3}, opt);
    check(kl_prepare_vertices_forward(dtype_code(verts.scalar_type()), (int)B, (int)Bv, (int)Bc, (int)Bp, V, F,
                                      ptr(verts), fc.data_ptr<int64_t>(), ptr(r), ptr(t), ptr(x), ptr(pj), ptr(fvc),
                                      ptr(fvi), ptr(fn), (kl_stream)stream),
          "prepare_vertices");
    ctx->saved_data["batches"] = batches;
    ctx->saved_data["stream"] = stream;
    ctx->saved_data["proj_shape"] = proj.sizes().vec();
    ctx->saved_data["trans_shape"] = has_xf ? std::vector<int64_t>{} : cam_b.sizes().vec();
    ctx->saved_data["has_xf"] = has_xf;
    ctx->set_materialize_grads(false);
    // the inputs themselves (a double backward differentiates the reference's chain of them)
    ctx->save_for_backward({vertices, faces, proj, has_xf ? at::Tensor() : cam_a, has_xf ? at::Tensor() : cam_b,
                            has_xf ? cam_a : at::Tensor()});
    return {fvc, fvi, fn};
  }
  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    variable_list out(8);
    if (!grads[0].defined() && !grads[1].defined() && !grads[2].defined()) return out;
    const bool has_xf = ctx->saved_data["has_xf"].toBool();
    if (at::GradMode::is_enabled()) {  // create_graph: the reference's torch gradient
      const auto g = chain_grads(prepare_chain(saved[0], saved[1], saved[2], saved[3], saved[4], saved[5]),
                                 {grads[0], grads[1], grads[2]}, {saved[0], saved[2], saved[3], saved[4], saved[5]});
      out[0] = g[0];
      out[2] = g[1];
      out[3] = has_xf ? g[4] : g[2];
      if (!has_xf) out[4] = g[3];
      return out;
    }
    const at::Tensor verts = saved[0].contiguous(), fc = saved[1].contiguous(), pj = saved[2].contiguous();
    const at::Tensor r = saved[3].defined() ? saved[3].contiguous() : at::Tensor();
    const at::Tensor t = saved[4].defined() ? saved[4].contiguous() : at::Tensor();
    const at::Tensor x = saved[5].defined() ? saved[5].contiguous() : at::Tensor();
    const auto b = ctx->saved_data["batches"].toIntVector();
    const int64_t B = b[0], Bv = b[1], Bc = b[2], Bp = b[3];
    const bool need_v = ctx->needs_input_grad(0), need_p = ctx->needs_input_grad(2),
               need_r = !has_xf && ctx->needs_input_grad(3), need_t = !has_xf && ctx->needs_input_grad(4),
               need_x = has_xf && ctx->needs_input_grad(3);
    const auto opt = verts.options();
    at::Tensor g_v = need_v ? at::empty_like(verts) : at::Tensor();
    at::Tensor g_cam = (need_r || need_t || need_x) ? at::empty({Bc, 12}, opt) : at::Tensor();
    at::Tensor g_proj = need_p ? at::empty({Bp, 3}, opt) : at::Tensor();
    const int64_t V = verts.size(1), F = fc.size(0);
    const int64_t stream = ctx->saved_data["stream"].toInt();
    const size_t nbytes = kl_prepare_vertices_bwd_workspace_bytes((int)B, V);
    at::Tensor ws = workspace(nbytes, verts.device(), stream);
    at::Tensor g0 = grads[0].defined() ? grads[0].contiguous() : at::Tensor();
    at::Tensor g1 = grads[1].defined() ? grads[1].contiguous() : at::Tensor();
    at::Tensor g2 = grads[2].defined() ? grads[2].contiguous() : at::Tensor();
    check(kl_prepare_vertices_backward(dtype_code(verts.scalar_type()), (int)B, (int)Bv, (int)Bc, (int)Bp, V, F,
                                       ptr(verts), fc.data_ptr<int64_t>(), ptr(r), ptr(t), ptr(x), ptr(pj), ptr(g0),
                                       ptr(g1), ptr(g2), ptr(g_v), ptr(g_cam), ptr(g_proj), ws.data_ptr(), nbytes,
                                       (kl_stream)stream),
          "prepare_vertices backward");
    out[0] = g_v;
    if (need_p) out[2] = g_proj.reshape(ctx->saved_data["proj_shape"].toIntVector());
    if (need_r) out[3] = g_cam.narrow(1, 0, 9).reshape({Bc, 3, 3});
    if (need_t) out[4] = g_cam.narrow(1, 9, 3).reshape(ctx->saved_data["trans_shape"].toIntVector());
    if (need_x) out[3] = g_cam.reshape({Bc, 4, 3});
    return out;
  }
};

std::tuple<at::Tensor, at::Tensor, at::Tensor> prepare_vertices(at::Tensor vertices, at::Tensor faces, at::Tensor proj,
                                                                c10::optional<at::Tensor> rot,
                                                                c10::optional<at::Tensor> trans,
                                                                c10::optional<at::Tensor> xf,
                                                                std::vector<int64_t> batches, int64_t stream) {
  const bool has_xf = xf.has_value() && xf->defined();
  TORCH_CHECK(has_xf || (rot.has_value() && trans.has_value()), "prepare_vertices: camera_rot and camera_trans, or "
              "camera_transform");
  auto r = has_xf ? PrepareVertices::apply(vertices, faces, proj, *xf, *xf, true, batches, stream)
                  : PrepareVertices::apply(vertices, faces, proj, *rot, *trans, false, batches, stream);
  return {r[0], r[1], r[2]};
}

// texture_mapping (render/mesh/utils.py TextureMappingHip): kl_texture_mapping_forward / _backward
struct TextureMapping : public torch::autograd::Function<TextureMapping> {
  static variable_list forward(AutogradContext *ctx, at::Tensor coords, at::Tensor tex, int64_t mode, int64_t stream) {
    at::Tensor c = coords.contiguous(), t = tex.contiguous();
    const int64_t B = t.size(0), C = t.size(1), TH = t.size(2), TW = t.size(3);
    const int64_t n = B ? c.numel() / (2 * B) : 0;
    at::Tensor out = at::empty({B, n, C}, t.options());
    check(kl_texture_mapping_forward(dtype_code(t.scalar_type()), (int)mode, (int)B, n, (int)C, (int)TH, (int)TW,
                                     ptr(c), ptr(t), ptr(out), (kl_stream)stream),
          "texture_mapping");
    ctx->saved_data["mode"] = mode;
    ctx->saved_data["n"] = n;
    ctx->saved_data["stream"] = stream;
    ctx->save_for_backward({coords, tex});  // the inputs themselves (double backward)
    return {out};
  }
  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const bool need_c = ctx->needs_input_grad(0), need_t = ctx->needs_input_grad(1);
    variable_list out(4);
    if ((!need_c && !need_t) || !grads[0].defined()) return out;
    if (at::GradMode::is_enabled()) {  // create_graph: the reference's torch gradient
      const at::Tensor o = texture_chain(saved[0], saved[1], ctx->saved_data["mode"].toInt());
      const auto g = chain_grads({o}, {grads[0].reshape(o.sizes())}, {saved[0], saved[1]});
      out[0] = g[0];
      out[1] = g[1];
      return out;
    }
    const at::Tensor c = saved[0].contiguous(), t = saved[1].contiguous();
    const int64_t B = t.size(0), C = t.size(1), TH = t.size(2), TW = t.size(3);
    const int64_t stream = ctx->saved_data["stream"].toInt();
    at::Tensor gc = need_c ? at::empty_like(c) : at::Tensor(), gt = need_t ? at::empty_like(t) : at::Tensor();
    const size_t nbytes = need_t ? kl_texture_mapping_bwd_workspace_bytes((int)B, (int)C, (int)TH, (int)TW) : 0;
    at::Tensor ws = need_t ? workspace(nbytes, t.device(), stream) : at::Tensor();
    check(kl_texture_mapping_backward(dtype_code(t.scalar_type()), (int)ctx->saved_data["mode"].toInt(), (int)B,
                                      ctx->saved_data["n"].toInt(), (int)C, (int)TH, (int)TW,
                                      ptr(grads[0].contiguous()), ptr(c), ptr(t), ptr(gc), ptr(gt), ptr(ws), nbytes,
                                      (kl_stream)stream),
          "texture_mapping backward");
    out[0] = gc;
    out[1] = gt;
    return out;
  }
};

at::Tensor texture_mapping(at::Tensor coords, at::Tensor tex, int64_t mode, int64_t stream) {
  return TextureMapping::apply(coords, tex, mode, stream)[0];
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> dibr_rasterization(int64_t height, int64_t width, at::Tensor fvz,
                                                                   at::Tensor fvi, at::Tensor feat, at::Tensor fnz,
                                                                   double sigmainv, double boxlen, int64_t knum,
                                                                   double multiplier, double eps, int64_t stream) {
  auto r = DibrRasterization::apply(height, width, fvz, fvi, feat, fnz, sigmainv, boxlen, knum, multiplier, eps,
                                    stream);
  return {r[0], r[1], r[2]};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "kaolin-mi355x compiled autograd nodes over the C ABI (include/kaolin_hip.h)";
  m.def("abi_version", []() { return kl_abi_version(); });
  m.def("dibr_rasterization", &dibr_rasterization,
        "dibr_rasterization's fused node: (features, soft_mask, face_idx); see kaolin/render/mesh/dibr.py");
  m.def("mask_iou", &mask_iou, "mask_iou's fused node; see kaolin/metrics/render.py");
  m.def("prepare_vertices", &prepare_vertices, "prepare_vertices' node; see kaolin/render/mesh/utils.py");
  m.def("texture_mapping", &texture_mapping, "texture_mapping's node; see kaolin/render/mesh/utils.py");
  // the double-backward reference chains, exposed for tests (tests/test_cpu_paths.py)
  m.def("_mask_iou_chain", &mask_iou_chain);
  m.def("_prepare_chain", [](at::Tensor v, at::Tensor faces, at::Tensor proj, c10::optional<at::Tensor> rot,
                             c10::optional<at::Tensor> trans, c10::optional<at::Tensor> xf) {
    return prepare_chain(v, faces, proj, rot.value_or(at::Tensor()), trans.value_or(at::Tensor()),
                         xf.value_or(at::Tensor()));
  });
  m.def("_texture_chain", &texture_chain);
}
