// torch_ops.cpp -- the eager host path of dibr_rasterization as a compiled autograd node.
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
  throw std::runtime_error("dibr_rasterization: f32 / f64 only");
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

void *ptr(const at::Tensor &t) { return t.defined() ? t.data_ptr() : nullptr; }

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
    // the backward's soft-mask work items and its zeroed accumulator (written by the forward)
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
    check(kl_dibr_backward(dtype_code(fvi.scalar_type()), (int)B, H, W, (int)F, (int)D, K, ptr(gf), ptr(gm),
                           idx.data_ptr<int64_t>(), ptr(w), ptr(fvi), ptr(feat), ptr(fnz), ptr(mask),
                           hits.data_ptr<uint8_t>(), (const uint32_t *)rec_face.data_ptr(), ptr(rec_prob),
                           seg_tot.data_ptr<int>(), (float)ctx->saved_data["sigmainv"].toDouble(),
                           (float)ctx->saved_data["multiplier"].toDouble(), (float)ctx->saved_data["eps"].toDouble(),
                           ptr(g_img), ptr(g_feat), scratch.data_ptr(),
                           ctx->saved_data["has_ranges"].toBool() ? (const uint32_t *)ranges.data_ptr() : nullptr,
                           ws.data_ptr(), nbytes, (kl_stream)stream),
          "dibr_rasterization backward");
    out[3] = g_img;
    out[4] = g_feat;
    return out;
  }
};

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
}
