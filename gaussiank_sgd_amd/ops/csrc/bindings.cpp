// Torch op registrations for the gfx950 kernel library and the RCCL engine.
//
// Ops are registered under the `gksgd` namespace (torch.ops.gksgd.*) and run
// asynchronously on the current HIP stream of the tensors' device.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <cstring>
#include <vector>

#include "comm/rccl_engine.h"
#include "kernels/gk_kernels.h"

namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_f32(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}

// ---------------------------------------------------------------------------
// compressor pipeline
// ---------------------------------------------------------------------------
int64_t ctrl_bytes() { return (int64_t)sizeof(gk::GkCtrl); }
int64_t workspace_bytes() { return (int64_t)gk::compress_workspace_bytes(0); }

void compress(at::Tensor g, at::Tensor r, at::Tensor ctrl, at::Tensor ws, at::Tensor record, int64_t mode, bool ec,
              bool zero_g, int64_t loops, double z, double fixed_thr, double sample_p, int64_t k, int64_t k_cap,
              int64_t seed, int64_t n_stats, c10::optional<at::Tensor> stats_out, c10::optional<at::Tensor> valid,
              c10::optional<at::Tensor> u, c10::optional<at::Tensor> w, c10::optional<at::Tensor> chunks,
              int64_t chunk_begin, int64_t chunk_count, int64_t chunk_base, std::vector<double> mc_mu,
              std::vector<double> mc_wd, c10::optional<at::Tensor> seed_dev, int64_t handoff) {
  check_f32(g, "g");
  check_f32(r, "r");
  check_dev(ctrl, "ctrl");
  check_dev(ws, "ws");
  check_dev(record, "record");
  TORCH_CHECK(g.numel() == r.numel(), "g and r must have the same numel");
  TORCH_CHECK(ctrl.nbytes() >= sizeof(gk::GkCtrl), "ctrl buffer too small");
  TORCH_CHECK(ws.nbytes() >= gk::compress_workspace_bytes(g.numel()), "workspace too small");
  TORCH_CHECK(record.scalar_type() == at::kInt, "record must be int32");
  TORCH_CHECK(k_cap >= 1 && record.numel() >= 4 + 2 * k_cap, "record must hold 4 + 2*k_cap int32");
  TORCH_CHECK(g.numel() < (int64_t)0x7fffffff, "bucket too large for int32 indices");
  TORCH_CHECK(mode >= 0 && mode <= 7, "bad mode");
  TORCH_CHECK(loops >= 1 && loops * (loops + 1) / 2 <= gk::kMaxCand, "loops out of range");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(ctrl.data_ptr()) & 7) == 0, "ctrl must be 8-byte aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(ws.data_ptr()) & 255) == 0, "ws must be 256-byte aligned");
  c10::DeviceGuard guard(g.device());
  gk::CompressArgs a;
  a.g = g.data_ptr<float>();
  a.r = r.data_ptr<float>();
  a.n = g.numel();
  a.n_stats = n_stats;
  a.mode = (int)mode;
  a.ec = ec ? 1 : 0;
  a.zero_g = zero_g ? 1 : 0;
  a.loops = (int)loops;
  a.z = z;
  a.fixed_thr = fixed_thr;
  a.sample_p = sample_p;
  a.k = k < 1 ? 1 : k;
  a.k_cap = k_cap;
  a.seed = (uint32_t)(seed & 0xffffffff);
  if (seed_dev.has_value() && seed_dev->defined()) {
    // graph replays: the seed word is refreshed in device memory before each replay
    check_dev(*seed_dev, "seed_dev");
    TORCH_CHECK(seed_dev->scalar_type() == at::kInt && seed_dev->numel() >= 1, "seed_dev must be int32[>=1]");
    a.seed_dev = reinterpret_cast<const uint32_t*>(seed_dev->data_ptr<int32_t>());
  }
  a.ctrl = ctrl.data_ptr();
  a.ws = ws.data_ptr();
  a.record = record.data_ptr<int32_t>();
  a.stats_out = nullptr;
  if (stats_out.has_value()) {
    check_f32(*stats_out, "stats_out");
    TORCH_CHECK(stats_out->numel() >= 4, "stats_out needs 4 floats");
    a.stats_out = stats_out->data_ptr<float>();
  }
  if (valid.has_value() && valid->defined()) {
    check_dev(*valid, "valid");
    TORCH_CHECK(valid->scalar_type() == at::kInt && valid->numel() * 32 >= g.numel(),
                "valid must be an int32 bitmask of >= n bits");
    a.valid = reinterpret_cast<const uint32_t*>(valid->data_ptr<int32_t>());
  }
  if (u.has_value() && u->defined()) {
    TORCH_CHECK(w.has_value() && w->defined() && chunks.has_value() && chunks->defined(),
                "momentum-corrected compress needs u, w and the chunk table");
    check_f32(*u, "u");
    check_f32(*w, "w");
    check_dev(*chunks, "chunks");
    TORCH_CHECK(chunks->scalar_type() == at::kLong, "chunks must be int64");
    TORCH_CHECK(u->numel() == g.numel() && w->numel() == g.numel(), "u / w must be bucket slices like g");
    TORCH_CHECK(zero_g, "momentum-corrected compress always zeroes g");
    TORCH_CHECK(chunk_begin >= 0 && chunk_count >= 1 && (chunk_begin + chunk_count) * 2 <= chunks->numel(),
                "chunk range out of bounds");
    TORCH_CHECK(mc_mu.size() >= 1 && mc_mu.size() <= 8 && mc_wd.size() == mc_mu.size(), "1..8 param groups");
    TORCH_CHECK(((reinterpret_cast<uintptr_t>(u->data_ptr()) | reinterpret_cast<uintptr_t>(w->data_ptr()) |
                  reinterpret_cast<uintptr_t>(g.data_ptr()) | reinterpret_cast<uintptr_t>(r.data_ptr())) & 15) == 0,
                "u / w / g / r must be 16-byte aligned");
    a.u = u->data_ptr<float>();
    a.w = w->data_ptr<float>();
    a.chunks = reinterpret_cast<const gk::Chunk*>(chunks->data_ptr<int64_t>());
    a.chunk_begin = (int)chunk_begin;
    a.chunk_count = (int)chunk_count;
    a.chunk_base = chunk_base;
    for (size_t i = 0; i < mc_mu.size(); ++i) {
      a.mc_mu[i] = (float)mc_mu[i];
      a.mc_wd[i] = (float)mc_wd[i];
    }
  }
  a.handoff = (int)handoff;
  gk::compress(a, cur_stream(g));
}

void apply_records_sgd(at::Tensor w, c10::optional<at::Tensor> w_bf16, at::Tensor records, int64_t P, int64_t k_cap,
                       double scale, double lr, c10::optional<at::Tensor> lr_mult) {
  check_f32(w, "w");
  check_dev(records, "records");
  TORCH_CHECK(records.scalar_type() == at::kInt, "records must be int32");
  TORCH_CHECK(P >= 1 && records.numel() >= P * (4 + 2 * k_cap), "records too small for P x (4 + 2 k_cap)");
  uint16_t* sh = nullptr;
  if (w_bf16.has_value() && w_bf16->defined()) {
    TORCH_CHECK(w_bf16->scalar_type() == at::kBFloat16 && w_bf16->numel() == w.numel() && w_bf16->is_contiguous(),
                "w_bf16 must be a contiguous bf16 tensor of w's size");
    sh = reinterpret_cast<uint16_t*>(w_bf16->data_ptr());
  }
  const float* lm = nullptr;
  if (lr_mult.has_value() && lr_mult->defined()) {
    check_f32(*lr_mult, "lr_mult");
    lm = lr_mult->data_ptr<float>();
  }
  c10::DeviceGuard guard(w.device());
  gk::apply_records_sgd(w.data_ptr<float>(), sh, w.numel(), records.data_ptr<int32_t>(), (int)P, k_cap, (float)scale,
                        (float)lr, lm, cur_stream(w));
}

void arena_digest(at::Tensor x, at::Tensor out, at::Tensor ws) {
  check_f32(x, "x");
  check_dev(out, "out");
  check_dev(ws, "ws");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() >= 2, "out must be int64[2]");
  TORCH_CHECK(ws.scalar_type() == at::kLong && ws.numel() >= 2048, "ws must be int64[>=2048]");
  c10::DeviceGuard guard(x.device());
  gk::arena_digest(x.data_ptr<float>(), x.numel(), reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()),
                   reinterpret_cast<uint64_t*>(ws.data_ptr<int64_t>()), cur_stream(x));
}

void tensor_stats(at::Tensor x, at::Tensor ctrl, at::Tensor ws) {
  check_f32(x, "x");
  check_dev(ctrl, "ctrl");
  check_dev(ws, "ws");
  TORCH_CHECK(ctrl.nbytes() >= sizeof(gk::GkCtrl), "ctrl buffer too small");
  c10::DeviceGuard guard(x.device());
  gk::tensor_stats(x.data_ptr<float>(), x.numel(), ctrl.data_ptr(), ws.data_ptr(), cur_stream(x));
}

// ---------------------------------------------------------------------------
// aggregation / bucket compressor
// ---------------------------------------------------------------------------
void scatter_add_records(at::Tensor dst, at::Tensor records, int64_t P, int64_t k_cap, double scale,
                         bool deterministic) {
  check_f32(dst, "dst");
  check_dev(records, "records");
  TORCH_CHECK(records.scalar_type() == at::kInt, "records must be int32");
  TORCH_CHECK(records.numel() >= P * (4 + 2 * k_cap), "records too small for P x (4 + 2 k_cap)");
  c10::DeviceGuard guard(dst.device());
  gk::scatter_add_records(dst.data_ptr<float>(), dst.numel(), records.data_ptr<int32_t>(), (int)P, k_cap,
                          (float)scale, deterministic ? 1 : 0, cur_stream(dst));
}

void fill_zero(at::Tensor dst) {
  check_f32(dst, "dst");
  c10::DeviceGuard guard(dst.device());
  gk::fill_zero(dst.data_ptr<float>(), dst.numel(), cur_stream(dst));
}

int64_t sign_bucket_workspace_bytes() { return (int64_t)gk::sign_bucket_workspace_bytes(0); }

void sign_bucket_compress(at::Tensor x, at::Tensor mask, at::Tensor means, at::Tensor ws) {
  check_f32(x, "x");
  check_dev(mask, "mask");
  check_f32(means, "means");
  check_dev(ws, "ws");
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() >= x.numel(), "mask must be uint8[n]");
  TORCH_CHECK(means.numel() >= 2, "means needs 2 floats");
  c10::DeviceGuard guard(x.device());
  gk::sign_bucket_compress(x.data_ptr<float>(), x.numel(), mask.data_ptr<uint8_t>(), means.data_ptr<float>(),
                           ws.data_ptr(), cur_stream(x));
}

void sign_bucket_decompress(at::Tensor x, at::Tensor mask, at::Tensor means) {
  check_f32(x, "x");
  check_dev(mask, "mask");
  check_f32(means, "means");
  c10::DeviceGuard guard(x.device());
  gk::sign_bucket_decompress(x.data_ptr<float>(), x.numel(), mask.data_ptr<uint8_t>(), means.data_ptr<float>(),
                             cur_stream(x));
}

// ---------------------------------------------------------------------------
// fused optimizers
// ---------------------------------------------------------------------------
void check_chunks(const at::Tensor& chunks) {
  check_dev(chunks, "chunks");
  TORCH_CHECK(chunks.scalar_type() == at::kLong && chunks.numel() % 2 == 0,
              "chunks must be int64[nchunks*2] (start, len|group<<32|seg<<48)");
}

void fused_sgd(at::Tensor w, c10::optional<at::Tensor> m, at::Tensor g, at::Tensor chunks, std::vector<double> lr,
               std::vector<double> momentum, std::vector<double> dampening, std::vector<double> weight_decay,
               std::vector<int64_t> nesterov, std::vector<int64_t> first_step, bool zero_grad,
               c10::optional<at::Tensor> grad_scale, c10::optional<at::Tensor> w_bf16,
               c10::optional<at::Tensor> lr_mult) {
  check_f32(w, "w");
  check_f32(g, "g");
  check_chunks(chunks);
  const size_t ng = lr.size();
  TORCH_CHECK(ng >= 1 && ng <= (size_t)gk::kMaxGroups, "1..8 param groups supported");
  TORCH_CHECK(momentum.size() == ng && dampening.size() == ng && weight_decay.size() == ng && nesterov.size() == ng &&
                  first_step.size() == ng,
              "hyper-parameter lists must have one entry per group");
  TORCH_CHECK(w.numel() == g.numel(), "w/g size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0,
              "arenas must be 16-byte aligned");
  gk::SgdArgs a;
  a.w = w.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.m = nullptr;
  if (m.has_value() && m->defined()) {
    check_f32(*m, "m");
    TORCH_CHECK(m->numel() == w.numel(), "momentum arena size mismatch");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(m->data_ptr()) & 15) == 0, "momentum arena must be 16-byte aligned");
    a.m = m->data_ptr<float>();
  }
  for (size_t i = 0; i < ng; ++i) {
    a.groups[i].lr = (float)lr[i];
    a.groups[i].momentum = (float)momentum[i];
    a.groups[i].dampening = (float)dampening[i];
    a.groups[i].weight_decay = (float)weight_decay[i];
    a.groups[i].nesterov = (int)nesterov[i];
    a.groups[i].first_step = (int)first_step[i];
    TORCH_CHECK(a.groups[i].momentum == 0.f || a.m != nullptr, "momentum arena required");
  }
  a.ngroups = (int)ng;
  a.chunks = reinterpret_cast<const gk::Chunk*>(chunks.data_ptr<int64_t>());
  a.nchunks = (int)(chunks.numel() / 2);
  a.zero_grad = zero_grad ? 1 : 0;
  a.grad_scale = nullptr;
  if (grad_scale.has_value() && grad_scale->defined()) {
    check_f32(*grad_scale, "grad_scale");
    a.grad_scale = grad_scale->data_ptr<float>();
  }
  if (w_bf16.has_value() && w_bf16->defined()) {
    TORCH_CHECK(w_bf16->scalar_type() == at::kBFloat16 && w_bf16->numel() == w.numel() && w_bf16->is_contiguous() &&
                    (reinterpret_cast<uintptr_t>(w_bf16->data_ptr()) & 15) == 0,
                "w_bf16 must be a 16-byte aligned contiguous bf16 arena of w's size");
    a.w_bf16 = reinterpret_cast<uint16_t*>(w_bf16->data_ptr());
  }
  if (lr_mult.has_value() && lr_mult->defined()) {
    check_f32(*lr_mult, "lr_mult");
    a.lr_mult = lr_mult->data_ptr<float>();
  }
  c10::DeviceGuard guard(w.device());
  gk::fused_sgd(a, cur_stream(w));
}

void segmented_sumsq(at::Tensor w, at::Tensor g, at::Tensor chunks, at::Tensor out) {
  check_f32(w, "w");
  check_f32(g, "g");
  check_chunks(chunks);
  check_dev(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kDouble, "out must be float64[2*nseg]");
  c10::DeviceGuard guard(w.device());
  gk::segmented_sumsq(w.data_ptr<float>(), g.data_ptr<float>(),
                      reinterpret_cast<const gk::Chunk*>(chunks.data_ptr<int64_t>()), (int)(chunks.numel() / 2),
                      out.data_ptr<double>(), cur_stream(w));
}

void fused_lars(at::Tensor w, at::Tensor m, at::Tensor g, at::Tensor chunks, at::Tensor seg_sumsq,
                std::vector<double> lr, std::vector<double> momentum, std::vector<double> weight_decay,
                std::vector<double> eeta, std::vector<double> epsilon) {
  check_f32(w, "w");
  check_f32(m, "m");
  check_f32(g, "g");
  check_chunks(chunks);
  check_dev(seg_sumsq, "seg_sumsq");
  const size_t ng = lr.size();
  TORCH_CHECK(ng >= 1 && ng <= (size_t)gk::kMaxGroups, "1..8 param groups supported");
  gk::LarsArgs a;
  a.w = w.data_ptr<float>();
  a.m = m.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.chunks = reinterpret_cast<const gk::Chunk*>(chunks.data_ptr<int64_t>());
  a.nchunks = (int)(chunks.numel() / 2);
  a.seg_sumsq = seg_sumsq.data_ptr<double>();
  for (size_t i = 0; i < ng; ++i) {
    a.lr[i] = (float)lr[i];
    a.momentum[i] = (float)momentum[i];
    a.weight_decay[i] = (float)weight_decay[i];
    a.eeta[i] = (float)eeta[i];
    a.epsilon[i] = (float)epsilon[i];
  }
  a.ngroups = (int)ng;
  c10::DeviceGuard guard(w.device());
  gk::fused_lars(a, cur_stream(w));
}

void clip_grad_norm(at::Tensor g, double max_norm, at::Tensor ws, at::Tensor coef, at::Tensor norm) {
  check_f32(g, "g");
  check_dev(ws, "ws");
  check_f32(coef, "coef");
  check_f32(norm, "norm");
  TORCH_CHECK(ws.scalar_type() == at::kDouble && ws.numel() >= 1024, "ws must be float64[>=1024]");
  c10::DeviceGuard guard(g.device());
  gk::clip_grad_norm(g.data_ptr<float>(), g.numel(), (float)max_norm, ws.data_ptr<double>(), coef.data_ptr<float>(),
                     norm.data_ptr<float>(), cur_stream(g));
}

// ---------------------------------------------------------------------------
// fused batch norm + add + relu (channels-last)
// ---------------------------------------------------------------------------
int64_t channels_of(const at::Tensor& x) { return x.dim() == 4 ? x.size(1) : x.size(-1); }

void check_cl(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last contiguous");
  } else {
    TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), name, " must be 4-D channels_last or 2-D [M, C]");
  }
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name, " must be bf16 or fp32");
}

const float* opt_f32(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->is_cuda(), "expected fp32 GPU tensor");
  return t->data_ptr<float>();
}

float* opt_f32_mut(const c10::optional<at::Tensor>& t) { return const_cast<float*>(opt_f32(t)); }

// optional tensor that must have `ref`'s dtype, shape and channels-last layout
const void* opt_like(const c10::optional<at::Tensor>& t, const at::Tensor& ref, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cl(*t, name);
  TORCH_CHECK(t->scalar_type() == ref.scalar_type() && t->sizes() == ref.sizes(), name, " must match dy");
  return t->data_ptr();
}

int64_t* opt_i64(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() == 1 && t->is_cuda(), "expected int64[1] GPU tensor");
  return t->data_ptr<int64_t>();
}

int64_t bn_workspace_floats(int64_t M, int64_t C, int64_t elem_bytes) {
  return (int64_t)gk::bn_workspace_floats(M, (int)C, (int)elem_bytes);
}

bool bn_supported(int64_t C, int64_t elem_bytes) { return gk::bn_supported((int)C, (int)elem_bytes); }

int64_t bn_mask_bytes(int64_t M, int64_t C, int64_t elem_bytes) {
  return (int64_t)gk::bn_mask_bytes(M, (int)C, (int)elem_bytes);
}

// per-layer in-launch finalize state (bn_act.hip FinSync): a zero-initialised
// uint8 GPU tensor of at least bn_fin_state_bytes(C), kept by the layer
void* fin_state(const c10::optional<at::Tensor>& fin, int64_t C) {
  if (!fin.has_value() || !fin->defined()) return nullptr;
  TORCH_CHECK(fin->is_cuda() && fin->is_contiguous() && fin->nbytes() >= gk::bn_fin_state_bytes((int)C) &&
                  reinterpret_cast<uintptr_t>(fin->data_ptr()) % 16 == 0,
              "fin: a contiguous, 16-byte aligned GPU tensor of bn_fin_state_bytes(C) bytes");
  return fin->data_ptr();
}

int64_t bn_fin_state_bytes(int64_t C) { return (int64_t)gk::bn_fin_state_bytes((int)C); }

void bn_act_forward(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, c10::optional<at::Tensor> mask,
                    c10::optional<at::Tensor> w,
                    c10::optional<at::Tensor> b, c10::optional<at::Tensor> run_mean,
                    c10::optional<at::Tensor> run_var, at::Tensor save_mean, at::Tensor save_invstd,
                    at::Tensor scale, at::Tensor shift, at::Tensor ws, double eps, double momentum, bool relu,
                    c10::optional<at::Tensor> nbt, c10::optional<at::Tensor> pre, int64_t pre_rows,
                    c10::optional<at::Tensor> fin, c10::optional<at::Tensor> rscale,
                    c10::optional<at::Tensor> rshift) {
  check_cl(x, "x");
  check_cl(y, "y");
  const int64_t C = channels_of(x);
  void* fs = fin_state(fin, C);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  TORCH_CHECK(y.scalar_type() == x.scalar_type() && y.numel() == x.numel(), "y must match x");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_cl(*res, "residual");
    TORCH_CHECK(res->scalar_type() == x.scalar_type() && res->numel() == x.numel(), "residual must match x");
    rp = res->data_ptr();
  }
  // deferred residual BN: res * rscale + rshift (ops/bn.py _BNDeferFn)
  const float* rsc = opt_f32(rscale);
  const float* rsh = opt_f32(rshift);
  TORCH_CHECK((rsc == nullptr) == (rsh == nullptr), "rscale and rshift go together");
  if (rsc) {
    TORCH_CHECK(rp != nullptr, "rscale / rshift need a residual");
    for (const at::Tensor* t : {&*rscale, &*rshift})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= C && t->is_cuda() && t->is_contiguous(),
                  "rscale / rshift: fp32[C]");
  }
  for (const at::Tensor* t : {&save_mean, &save_invstd, &scale, &shift})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= C && t->is_cuda(), "stat buffers: fp32[C]");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  uint8_t* mp = nullptr;
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->scalar_type() == at::kByte && mask->is_cuda() &&
                    mask->numel() >= (int64_t)gk::bn_mask_bytes(M, (int)C, eb),
                "relu needs a uint8 mask of bn_mask_bytes");
    mp = mask->data_ptr<uint8_t>();
  }
  c10::DeviceGuard guard(x.device());
  if (pre.has_value() && pre->defined()) {   // statistics pre-reduced by the producer (conv epilogue)
    TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kFloat && pre->is_contiguous() && pre->dim() == 3 &&
                    pre->size(0) == 2 && pre->size(2) == C && pre_rows > 0 && pre_rows <= pre->size(1),
                "pre must be fp32 [2, rows, C] partials with 0 < pre_rows <= rows");
    // the finalize reads rows [0, pre_rows) of each half
    const float* ps = pre->data_ptr<float>();
    gk::bn_act_forward_pre(x.data_ptr(), rp, y.data_ptr(), mp, M, (int)C, eb, ps, ps + pre->size(1) * C,
                           (int)pre_rows, opt_f32(w), opt_f32(b), (float)eps, (float)momentum, opt_f32_mut(run_mean),
                           opt_f32_mut(run_var), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                           scale.data_ptr<float>(), shift.data_ptr<float>(), relu ? 1 : 0, opt_i64(nbt),
                           cur_stream(x), fs, rsc, rsh);
    return;
  }
  gk::bn_act_forward(x.data_ptr(), rp, y.data_ptr(), mp, M, (int)C, eb, opt_f32(w), opt_f32(b), (float)eps,
                     (float)momentum, opt_f32_mut(run_mean), opt_f32_mut(run_var), save_mean.data_ptr<float>(),
                     save_invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                     ws.data_ptr<float>(), relu ? 1 : 0, opt_i64(nbt), cur_stream(x), fs, rsc, rsh);
}

// statistics + finalize of a BN whose apply is deferred into its consumer
void bn_act_finalize(at::Tensor x, c10::optional<at::Tensor> w, c10::optional<at::Tensor> b,
                     c10::optional<at::Tensor> run_mean, c10::optional<at::Tensor> run_var, at::Tensor save_mean,
                     at::Tensor save_invstd, at::Tensor scale, at::Tensor shift, at::Tensor ws, double eps,
                     double momentum, c10::optional<at::Tensor> nbt, c10::optional<at::Tensor> pre, int64_t pre_rows) {
  check_cl(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  for (const at::Tensor* t : {&save_mean, &save_invstd, &scale, &shift})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= C && t->is_cuda(), "stat buffers: fp32[C]");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  const float* ps = nullptr;
  const float* pq = nullptr;
  if (pre.has_value() && pre->defined()) {
    TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kFloat && pre->is_contiguous() && pre->dim() == 3 &&
                    pre->size(0) == 2 && pre->size(2) == C && pre_rows > 0 && pre_rows <= pre->size(1),
                "pre must be fp32 [2, rows, C] partials with 0 < pre_rows <= rows");
    ps = pre->data_ptr<float>();
    pq = ps + pre->size(1) * C;
  }
  c10::DeviceGuard guard(x.device());
  gk::bn_act_finalize(x.data_ptr(), M, (int)C, eb, ps, pq, (int)pre_rows, opt_f32(w), opt_f32(b), (float)eps,
                      (float)momentum, opt_f32_mut(run_mean), opt_f32_mut(run_var), save_mean.data_ptr<float>(),
                      save_invstd.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                      ws.data_ptr<float>(), opt_i64(nbt), cur_stream(x));
}

void bn_act_backward(at::Tensor dy, c10::optional<at::Tensor> mask, at::Tensor x, at::Tensor dx,
                     c10::optional<at::Tensor> dres, c10::optional<at::Tensor> w, at::Tensor mean, at::Tensor invstd,
                     at::Tensor dgamma, at::Tensor dbeta, at::Tensor ws, bool relu,
                     c10::optional<at::Tensor> gw_acc, c10::optional<at::Tensor> gb_acc,
                     c10::optional<at::Tensor> dy2, c10::optional<at::Tensor> fin) {
  check_cl(dy, "dy");
  check_cl(x, "x");
  check_cl(dx, "dx");
  const int64_t C = channels_of(x);
  void* fs = fin_state(fin, C);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dx.scalar_type() == x.scalar_type(), "dtype mismatch");
  const uint8_t* mp = nullptr;
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->scalar_type() == at::kByte &&
                    mask->numel() >= (int64_t)gk::bn_mask_bytes(M, (int)C, eb),
                "relu backward needs the forward's mask");
    mp = mask->data_ptr<uint8_t>();
  }
  void* rp = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_cl(*dres, "dres");
    rp = dres->data_ptr();
  }
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  c10::DeviceGuard guard(x.device());
  const void* d2 = opt_like(dy2, dy, "dy2");
  gk::bn_act_backward(dy.data_ptr(), d2, mp, x.data_ptr(), dx.data_ptr(), rp, M, (int)C, eb, opt_f32(w),
                      mean.data_ptr<float>(), invstd.data_ptr<float>(), dgamma.data_ptr<float>(),
                      dbeta.data_ptr<float>(), ws.data_ptr<float>(), relu ? 1 : 0, opt_f32_mut(gw_acc),
                      opt_f32_mut(gb_acc), cur_stream(x), fs);
}

void bn_act_backward_pre(at::Tensor dz, at::Tensor x, at::Tensor dx, c10::optional<at::Tensor> w, at::Tensor mean,
                         at::Tensor invstd, at::Tensor dgamma, at::Tensor dbeta, at::Tensor part, int64_t rows,
                         c10::optional<at::Tensor> gw_acc, c10::optional<at::Tensor> gb_acc,
                         c10::optional<at::Tensor> fin) {
  check_cl(dz, "dz");
  check_cl(x, "x");
  check_cl(dx, "dx");
  const int64_t C = channels_of(x);
  void* fs = fin_state(fin, C);
  const int64_t M = x.numel() / C;
  TORCH_CHECK((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) &&
                  dz.scalar_type() == x.scalar_type() && dx.scalar_type() == x.scalar_type() &&
                  dz.numel() == x.numel() && dx.numel() == x.numel(),
              "bn_act_backward_pre: dz / x / dx of one shape and dtype (bf16 or fp32)");
  const int eb = (int)x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 &&
                  part.size(0) == 2 && part.size(2) == C && rows > 0 && rows <= part.size(1),
              "part must be fp32 [2, rows, C] partials with 0 < rows <= part.size(1)");
  for (const at::Tensor* t : {&mean, &invstd, &dgamma, &dbeta})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= C, "per-channel buffers: fp32[C]");
  c10::DeviceGuard guard(x.device());
  const float* ps = part.data_ptr<float>();
  gk::bn_act_backward_pre(dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C, eb, opt_f32(w), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), ps,
                          ps + part.size(1) * C, (int)rows, opt_f32_mut(gw_acc), opt_f32_mut(gb_acc), cur_stream(x),
                          fs);
}

// bn_act_backward_pre + the deferred residual BN of x2 (dx2 from the same apply pass)
void bn_act_backward_pre_dual(at::Tensor dz, at::Tensor x, at::Tensor dx, c10::optional<at::Tensor> w, at::Tensor mean,
                              at::Tensor invstd, at::Tensor dgamma, at::Tensor dbeta, at::Tensor part, int64_t rows,
                              c10::optional<at::Tensor> gw_acc, c10::optional<at::Tensor> gb_acc, at::Tensor x2,
                              at::Tensor dx2, c10::optional<at::Tensor> w2, at::Tensor mean2, at::Tensor invstd2,
                              at::Tensor dgamma2, at::Tensor dbeta2, at::Tensor ws2,
                              c10::optional<at::Tensor> gw2_acc, c10::optional<at::Tensor> gb2_acc) {
  for (const at::Tensor* t : {&dz, &x, &dx, &x2, &dx2}) check_cl(*t, "dz / x / dx / x2 / dx2");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  for (const at::Tensor* t : {&dz, &dx, &x2, &dx2})
    TORCH_CHECK(t->scalar_type() == x.scalar_type() && t->numel() == x.numel(),
                "bn_act_backward_pre_dual: dz / x / dx / x2 / dx2 of one shape and dtype");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "bf16 or fp32");
  const int eb = (int)x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 &&
                  part.size(0) == 2 && part.size(2) == C && rows > 0 && rows <= part.size(1),
              "part must be fp32 [2, rows, C] partials with 0 < rows <= part.size(1)");
  for (const at::Tensor* t : {&mean, &invstd, &dgamma, &dbeta, &mean2, &invstd2, &dgamma2, &dbeta2})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= C, "per-channel buffers: fp32[C]");
  TORCH_CHECK(ws2.scalar_type() == at::kFloat && ws2.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  c10::DeviceGuard guard(x.device());
  const float* ps = part.data_ptr<float>();
  gk::bn_act_backward_pre_dual(dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C, eb, opt_f32(w),
                               mean.data_ptr<float>(), invstd.data_ptr<float>(), dgamma.data_ptr<float>(),
                               dbeta.data_ptr<float>(), ps, ps + part.size(1) * C, (int)rows, opt_f32_mut(gw_acc),
                               opt_f32_mut(gb_acc), x2.data_ptr(), dx2.data_ptr(), opt_f32(w2), mean2.data_ptr<float>(),
                               invstd2.data_ptr<float>(), dgamma2.data_ptr<float>(), dbeta2.data_ptr<float>(),
                               ws2.data_ptr<float>(), opt_f32_mut(gw2_acc), opt_f32_mut(gb2_acc), cur_stream(x));
}

// ---- lazy BN backward (bn_act.hip bn_bwd_finalize_lazy): no apply pass ----
void check_lazy_out(const at::Tensor& x, int64_t C, const at::Tensor& coef, const at::Tensor& padz,
                    const at::Tensor& padx) {
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() >= 4 * C,
              "coef must be a contiguous fp32 [C, 4] GPU tensor");
  for (const at::Tensor* t : {&padz, &padx})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == x.scalar_type() && t->is_contiguous() && t->numel() >= C,
                "padz / padx must be contiguous [C] GPU tensors of x's dtype");
}

void bn_bwd_lazy_pre(at::Tensor x, at::Tensor part, int64_t rows, c10::optional<at::Tensor> w, at::Tensor mean,
                     at::Tensor invstd, at::Tensor dgamma, at::Tensor dbeta, at::Tensor coef, at::Tensor padz,
                     at::Tensor padx, c10::optional<at::Tensor> gw_acc, c10::optional<at::Tensor> gb_acc) {
  check_cl(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 &&
                  part.size(0) == 2 && part.size(2) == C && rows > 0 && rows <= part.size(1),
              "part must be fp32 [2, rows, C] partials with 0 < rows <= part.size(1)");
  for (const at::Tensor* t : {&mean, &invstd, &dgamma, &dbeta})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= C, "per-channel buffers: fp32[C]");
  check_lazy_out(x, C, coef, padz, padx);
  c10::DeviceGuard guard(x.device());
  const float* ps = part.data_ptr<float>();
  gk::bn_bwd_finalize_lazy(ps, ps + part.size(1) * C, (int)rows, M, (int)C, (int)x.element_size(), 1, opt_f32(w),
                           mean.data_ptr<float>(), invstd.data_ptr<float>(), dgamma.data_ptr<float>(),
                           dbeta.data_ptr<float>(), opt_f32_mut(gw_acc), opt_f32_mut(gb_acc), coef.data_ptr<float>(),
                           padz.data_ptr(), padx.data_ptr(), cur_stream(x));
}

void bn_act_backward_lazy(at::Tensor dy, c10::optional<at::Tensor> dy2, c10::optional<at::Tensor> mask, at::Tensor x,
                          at::Tensor dz, c10::optional<at::Tensor> w, at::Tensor mean, at::Tensor invstd,
                          at::Tensor dgamma, at::Tensor dbeta, at::Tensor ws, bool relu, at::Tensor coef,
                          at::Tensor padz, at::Tensor padx, c10::optional<at::Tensor> gw_acc,
                          c10::optional<at::Tensor> gb_acc) {
  check_cl(dy, "dy");
  check_cl(x, "x");
  check_cl(dz, "dz");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dz.scalar_type() == x.scalar_type() && dz.numel() == x.numel(),
              "dtype / shape mismatch");
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  const uint8_t* mp = nullptr;
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->scalar_type() == at::kByte &&
                    mask->numel() >= (int64_t)gk::bn_mask_bytes(M, (int)C, eb),
                "relu backward needs the forward's mask");
    mp = mask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  check_lazy_out(x, C, coef, padz, padx);
  c10::DeviceGuard guard(x.device());
  const void* d2 = opt_like(dy2, dy, "dy2");
  gk::bn_act_backward_lazy(dy.data_ptr(), d2, mp, x.data_ptr(), dz.data_ptr(), M, (int)C, eb, opt_f32(w),
                           mean.data_ptr<float>(), invstd.data_ptr<float>(), dgamma.data_ptr<float>(),
                           dbeta.data_ptr<float>(), ws.data_ptr<float>(), relu ? 1 : 0, opt_f32_mut(gw_acc),
                           opt_f32_mut(gb_acc), coef.data_ptr<float>(), padz.data_ptr(), padx.data_ptr(),
                           cur_stream(x));
}

void bn_stats_partials(at::Tensor x, at::Tensor ws) {
  check_cl(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  const int eb = (int)x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  c10::DeviceGuard guard(x.device());
  gk::bn_stats_partials(x.data_ptr(), M, (int)C, eb, ws.data_ptr<float>(), cur_stream(x));
}

void bn_lazy_apply(at::Tensor dz, at::Tensor x, at::Tensor dx, at::Tensor coef) {
  check_cl(dz, "dz");
  check_cl(x, "x");
  check_cl(dx, "dx");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(dz.scalar_type() == x.scalar_type() && dx.scalar_type() == x.scalar_type() &&
                  dz.numel() == x.numel() && dx.numel() == x.numel(), "dz / x / dx of one shape and dtype");
  TORCH_CHECK(gk::bn_supported((int)C, (int)x.element_size()), "channel count not supported by the fused kernel");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.numel() >= 4 * C, "coef: fp32 [C, 4]");
  c10::DeviceGuard guard(x.device());
  gk::bn_lazy_apply(dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C, (int)x.element_size(),
                    coef.data_ptr<float>(), cur_stream(x));
}

gk::PoolGeo pool_geo(const at::Tensor& x, const at::Tensor& y, int64_t k, int64_t st, int64_t pad) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(1) == y.size(1), "pool shapes");
  gk::PoolGeo pg;
  pg.H = (int)x.size(2);
  pg.W = (int)x.size(3);
  pg.OH = (int)y.size(2);
  pg.OW = (int)y.size(3);
  pg.k = (int)k;
  pg.s = (int)st;
  pg.p = (int)pad;
  TORCH_CHECK(k >= 1 && k <= 15 && st >= 1 && pad >= 0 && 2 * pad <= k, "unsupported pool window");
  TORCH_CHECK(pg.OH == (pg.H + 2 * pg.p - pg.k) / pg.s + 1 && pg.OW == (pg.W + 2 * pg.p - pg.k) / pg.s + 1,
              "pool output shape mismatch (ceil_mode unsupported)");
  TORCH_CHECK(x.numel() / x.size(1) < (int64_t(1) << 32), "N*H*W must be < 2^32");
  return pg;
}

void bn_relu_pool_forward(at::Tensor x, at::Tensor y, at::Tensor amax, c10::optional<at::Tensor> w,
                          c10::optional<at::Tensor> b, c10::optional<at::Tensor> run_mean,
                          c10::optional<at::Tensor> run_var, at::Tensor save_mean, at::Tensor save_invstd,
                          at::Tensor scale, at::Tensor shift, at::Tensor ws, double eps, double momentum, int64_t k,
                          int64_t st, int64_t pad, c10::optional<at::Tensor> nbt, c10::optional<at::Tensor> pre,
                          int64_t pre_rows) {
  check_cl(x, "x");
  check_cl(y, "y");
  TORCH_CHECK(x.dim() == 4 && y.scalar_type() == x.scalar_type(), "y must be 4-D with x's dtype");
  const gk::PoolGeo pg = pool_geo(x, y, k, st, pad);
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(gk::bn_supported((int)C, eb), "channel count not supported by the fused kernel");
  TORCH_CHECK(amax.scalar_type() == at::kByte && amax.is_cuda() && amax.numel() >= y.numel(), "amax: uint8[y.numel]");
  for (const at::Tensor* t : {&save_mean, &save_invstd, &scale, &shift})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= C && t->is_cuda(), "stat buffers: fp32[C]");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  c10::DeviceGuard guard(x.device());
  if (pre.has_value() && pre->defined()) {   // statistics pre-reduced by the producer (stem conv epilogue)
    TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kFloat && pre->is_contiguous() && pre->dim() == 3 &&
                    pre->size(0) == 2 && pre->size(2) == C && pre_rows > 0 && pre_rows <= pre->size(1),
                "pre must be fp32 [2, rows, C] partials with 0 < pre_rows <= rows");
    const float* ps = pre->data_ptr<float>();
    gk::bn_relu_pool_forward_pre(x.data_ptr(), y.data_ptr(), amax.data_ptr<uint8_t>(), x.size(0), (int)C, pg, eb, ps,
                                 ps + pre->size(1) * C, (int)pre_rows, opt_f32(w), opt_f32(b), (float)eps,
                                 (float)momentum, opt_f32_mut(run_mean), opt_f32_mut(run_var),
                                 save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), scale.data_ptr<float>(),
                                 shift.data_ptr<float>(), opt_i64(nbt), cur_stream(x));
    return;
  }
  gk::bn_relu_pool_forward(x.data_ptr(), y.data_ptr(), amax.data_ptr<uint8_t>(), x.size(0), (int)C, pg, eb,
                           opt_f32(w), opt_f32(b), (float)eps, (float)momentum, opt_f32_mut(run_mean),
                           opt_f32_mut(run_var), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                           scale.data_ptr<float>(), shift.data_ptr<float>(), ws.data_ptr<float>(), opt_i64(nbt),
                           cur_stream(x));
}

void bn_relu_pool_backward(at::Tensor dy, at::Tensor amax, at::Tensor x, at::Tensor dx, c10::optional<at::Tensor> w,
                           at::Tensor mean, at::Tensor invstd, at::Tensor dgamma, at::Tensor dbeta, at::Tensor ws,
                           int64_t k, int64_t st, int64_t pad, c10::optional<at::Tensor> gw_acc,
                           c10::optional<at::Tensor> gb_acc, c10::optional<at::Tensor> dy2) {
  check_cl(dy, "dy");
  check_cl(x, "x");
  check_cl(dx, "dx");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dx.scalar_type() == x.scalar_type(), "dtype mismatch");
  TORCH_CHECK(dx.sizes() == x.sizes(), "dx must match x");
  const gk::PoolGeo pg = pool_geo(x, dy, k, st, pad);
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  const int eb = x.element_size();
  TORCH_CHECK(amax.scalar_type() == at::kByte && amax.numel() >= dy.numel(), "amax: uint8[dy.numel]");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (int64_t)gk::bn_workspace_floats(M, (int)C, eb),
              "workspace too small");
  c10::DeviceGuard guard(x.device());
  const void* d2 = opt_like(dy2, dy, "dy2");
  gk::bn_relu_pool_backward(dy.data_ptr(), d2, amax.data_ptr<uint8_t>(), x.data_ptr(), dx.data_ptr(), x.size(0), (int)C,
                            pg, eb, opt_f32(w), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                            dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), ws.data_ptr<float>(),
                            opt_f32_mut(gw_acc), opt_f32_mut(gb_acc), cur_stream(x));
}

// ---------------------------------------------------------------------------
// DGC momentum correction + momentum factor masking
// ---------------------------------------------------------------------------
void momentum_correct(at::Tensor u, at::Tensor g, at::Tensor w, at::Tensor chunks, int64_t begin, int64_t count,
                      std::vector<double> momentum, std::vector<double> weight_decay) {
  check_f32(u, "u");
  check_f32(g, "g");
  check_f32(w, "w");
  check_chunks(chunks);
  TORCH_CHECK(u.numel() == g.numel() && w.numel() == g.numel(), "arena size mismatch");
  for (const at::Tensor* t : {&u, &g, &w})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "arenas must be 16-byte aligned");
  TORCH_CHECK(begin >= 0 && count >= 0 && (begin + count) * 2 <= chunks.numel(), "chunk range out of bounds");
  const size_t ng = momentum.size();
  TORCH_CHECK(ng >= 1 && ng <= (size_t)gk::kMaxGroups && weight_decay.size() == ng, "1..8 param groups");
  gk::McArgs a;
  a.u = u.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.w = w.data_ptr<float>();
  a.chunks = reinterpret_cast<const gk::Chunk*>(chunks.data_ptr<int64_t>()) + begin;
  a.nchunks = (int)count;
  for (size_t i = 0; i < ng; ++i) {
    a.momentum[i] = (float)momentum[i];
    a.weight_decay[i] = (float)weight_decay[i];
  }
  c10::DeviceGuard guard(u.device());
  gk::momentum_correct(a, cur_stream(u));
}

void mask_records(at::Tensor u, at::Tensor record, int64_t k_cap) {
  check_f32(u, "u");
  TORCH_CHECK(record.scalar_type() == at::kInt && record.is_contiguous() && record.is_cuda() &&
                  record.numel() >= gk::kRecHdr + 2 * k_cap,
              "record: int32[4 + 2*k_cap]");
  c10::DeviceGuard guard(u.device());
  gk::mask_records(u.data_ptr<float>(), record.data_ptr<int32_t>(), k_cap, cur_stream(u));
}

// ---------------------------------------------------------------------------
// direct-to-arena gradient accumulation / bf16 shadow weights
// ---------------------------------------------------------------------------
void accum_grad(at::Tensor dst, at::Tensor src) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda(), "GPU tensors required");
  TORCH_CHECK(dst.scalar_type() == at::kFloat, "dst must be fp32");
  TORCH_CHECK(src.scalar_type() == at::kBFloat16 || src.scalar_type() == at::kFloat, "src must be bf16 or fp32");
  TORCH_CHECK(dst.sizes() == src.sizes(), "shape mismatch");
  bool same = true;  // identical element order: strides agree on every dim of size > 1
  for (int64_t d = 0; d < dst.dim(); ++d)
    if (dst.size(d) > 1 && dst.stride(d) != src.stride(d)) same = false;
  TORCH_CHECK(same && dst.is_non_overlapping_and_dense() && src.is_non_overlapping_and_dense(),
              "dst/src must be dense with the same element order");
  c10::DeviceGuard guard(dst.device());
  gk::accum_grad(dst.data_ptr<float>(), src.data_ptr(), dst.numel(), (int)src.element_size(), cur_stream(dst));
}

void cast_bf16(at::Tensor dst, at::Tensor src) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda() && dst.scalar_type() == at::kBFloat16 &&
                  src.scalar_type() == at::kFloat && dst.numel() == src.numel() && dst.is_contiguous() &&
                  src.is_contiguous(),
              "cast_bf16: contiguous bf16 dst, fp32 src");
  c10::DeviceGuard guard(dst.device());
  gk::cast_bf16(reinterpret_cast<uint16_t*>(dst.data_ptr()), src.data_ptr<float>(), dst.numel(), cur_stream(dst));
}

// ---------------------------------------------------------------------------
// RCCL engine (torch custom class)
// ---------------------------------------------------------------------------
ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL");
  }
  return ncclFloat32;
}

struct RcclEngine : torch::CustomClassHolder {
  gk::RcclComm comm;

  static at::Tensor unique_id() {
    std::vector<uint8_t> id = gk::RcclComm::make_unique_id();
    at::Tensor t = at::empty({(int64_t)id.size()}, at::TensorOptions().dtype(at::kByte));
    std::memcpy(t.data_ptr<uint8_t>(), id.data(), id.size());
    return t;
  }

  void init(at::Tensor uid, int64_t rank, int64_t world, int64_t device) {
    TORCH_CHECK(!uid.is_cuda() && uid.scalar_type() == at::kByte, "uid must be a CPU uint8 tensor");
    at::Tensor c = uid.contiguous();
    std::vector<uint8_t> v(c.data_ptr<uint8_t>(), c.data_ptr<uint8_t>() + c.numel());
    comm.init(v, (int)rank, (int)world, (int)device);
  }

  // non-blocking bootstrap (parallel/comm.py _bootstrap_native)
  void init_async(at::Tensor uid, int64_t rank, int64_t world, int64_t device) {
    TORCH_CHECK(!uid.is_cuda() && uid.scalar_type() == at::kByte, "uid must be a CPU uint8 tensor");
    at::Tensor c = uid.contiguous();
    std::vector<uint8_t> v(c.data_ptr<uint8_t>(), c.data_ptr<uint8_t>() + c.numel());
    comm.init_async(v, (int)rank, (int)world, (int)device);
  }
  int64_t init_poll() { return comm.init_poll(); }
  void init_wait(double timeout_s) { comm.init_wait(timeout_s); }
  void abort() { comm.abort(); }
  void set_op_timeout(double s) { comm.set_op_timeout(s); }

  void allgather(at::Tensor send, at::Tensor recv) {
    check_dev(send, "send");
    check_dev(recv, "recv");
    TORCH_CHECK(recv.nbytes() == send.nbytes() * (size_t)comm.world(), "recv must be world x send bytes");
    c10::DeviceGuard guard(send.device());
    comm.allgather_bytes(send.data_ptr(), recv.data_ptr(), send.nbytes(), cur_stream(send));
  }

  void allreduce(at::Tensor t, int64_t op) {
    check_dev(t, "t");
    c10::DeviceGuard guard(t.device());
    ncclRedOp_t o = op == 0 ? ncclSum : (op == 1 ? ncclAvg : (op == 2 ? ncclMax : ncclMin));
    comm.allreduce(t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), o, cur_stream(t));
  }

  void broadcast(at::Tensor t, int64_t root) {
    check_dev(t, "t");
    c10::DeviceGuard guard(t.device());
    comm.broadcast(t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), (int)root, cur_stream(t));
  }

  void allgather_many(std::vector<at::Tensor> sends, std::vector<at::Tensor> recvs) {
    TORCH_CHECK(sends.size() == recvs.size() && !sends.empty(), "allgather_many: matching non-empty lists");
    std::vector<const void*> sp;
    std::vector<void*> rp;
    std::vector<size_t> nb;
    for (size_t i = 0; i < sends.size(); ++i) {
      check_dev(sends[i], "send");
      check_dev(recvs[i], "recv");
      TORCH_CHECK(sends[i].device() == sends[0].device() && recvs[i].device() == sends[0].device(),
                  "allgather_many: one device");
      TORCH_CHECK(recvs[i].nbytes() == sends[i].nbytes() * (size_t)comm.world(), "recv must be world x send bytes");
      sp.push_back(sends[i].data_ptr());
      rp.push_back(recvs[i].data_ptr());
      nb.push_back(sends[i].nbytes());
    }
    c10::DeviceGuard guard(sends[0].device());
    comm.allgather_many(sp, rp, nb, cur_stream(sends[0]));
  }

  void inject_failure(std::string why) { comm.inject_failure(why); }
  void destroy() { comm.destroy(); }
  int64_t rank() const { return comm.rank(); }
  int64_t world() const { return comm.world(); }

  void set_tracking(bool on) { comm.set_tracking(on); }
  void start_watchdog(double timeout_s, double poll_ms) { comm.start_watchdog(timeout_s, poll_ms); }
  void stop_watchdog() { comm.stop_watchdog(); }
  int64_t poll() { return comm.poll(); }
  bool failed() const { return comm.failed(); }
  std::string error() const { return comm.error(); }
  void check() const { comm.check(); }
  int64_t in_flight() const { return comm.in_flight(); }
  void reset_stats() { comm.reset_stats(); }
  // [calls, bytes, ms_total, ms_max] of op 0 all-gather, 1 all-reduce, 2 broadcast, 3 grouped all-gather
  std::vector<double> stats(int64_t op) const {
    gk::OpStats st = comm.stats((int)op);
    return {(double)st.calls, (double)st.bytes, st.ms_total, st.ms_max};
  }
};

// ---------------------------------------------------------------------------
// 1x1-convolution GEMMs (gemm.hip)
// ---------------------------------------------------------------------------
bool gemm_supported(int64_t N, int64_t K) { return gk::gemm_supported(N, K); }

// GEMM operand: 2-D bf16 or fp32 rows (one dtype per call: `like`)
bool is_gemm_dtype(const at::Tensor& t) { return t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat; }

void check_rows(const at::Tensor& t, const char* name, const at::Tensor& like) {
  TORCH_CHECK(t.is_cuda() && is_gemm_dtype(t) && t.scalar_type() == like.scalar_type() && t.dim() == 2, name,
              " must be a 2-D bf16 or fp32 GPU tensor (all operands one dtype)");
  TORCH_CHECK(t.stride(1) == 1 && (t.stride(0) * t.element_size()) % 16 == 0, name,
              " rows must be contiguous, 16-byte aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

// stats (optional): fp32 [2, rows, N] BatchNorm partials of C; returns the rows written
float* stats_ptr(const c10::optional<at::Tensor>& st, int64_t N, int* rows) {
  if (!st.has_value()) {
    *rows = 0;
    return nullptr;
  }
  const at::Tensor& t = *st;
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 3 && t.size(0) == 2 &&
                  t.size(2) == N && t.size(1) > 0,
              "stats must be a contiguous fp32 [2, rows, N] GPU tensor");
  *rows = (int)t.size(1);
  return t.data_ptr<float>();
}

// ---- ResNet stem (stem.hip) ----
void check_stem_x(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) == 3 &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: x must be a channels-last fp32 / bf16 [N, 3, H, W] GPU tensor");
  TORCH_CHECK(gk::stem_supported((int)x.size(2), (int)x.size(3)), "stem: unsupported image size");
  TORCH_CHECK(x.size(0) * x.size(2) * x.size(3) < (int64_t(1) << 31), "stem: batch too large");
}

void stem_pack(at::Tensor w, at::Tensor wp) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 &&
                  w.size(2) == 7 && w.size(3) == 7,
              "stem_pack: w must be fp32 [64, 3, 7, 7]");
  TORCH_CHECK(wp.is_cuda() && wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == 64 * 224,
              "stem_pack: wp must be contiguous bf16 [64, 224]");
  c10::DeviceGuard guard(w.device());
  gk::stem_pack_weight(w.data_ptr<float>(), w.stride(0), w.stride(1), w.stride(2), w.stride(3),
                       static_cast<uint16_t*>(wp.data_ptr()), cur_stream(w));
}

int64_t stem_fwd(at::Tensor x, at::Tensor wp, at::Tensor y, c10::optional<at::Tensor> stats) {
  check_stem_x(x);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(wp.is_cuda() && wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == 64 * 224,
              "stem_fwd: wp must be the packed bf16 [64, 224] weights");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 && y.size(0) == N && y.size(1) == 64 &&
                  y.size(2) == OH && y.size(3) == OW && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_fwd: y must be channels-last bf16 [N, 64, OH, OW]");
  int rows = 0;
  float* sp = stats_ptr(stats, 64, &rows);
  c10::DeviceGuard guard(x.device());
  return gk::stem_forward(x.data_ptr(), x.scalar_type() == at::kFloat, (int)N, (int)H, (int)W,
                          static_cast<const uint16_t*>(wp.data_ptr()), static_cast<uint16_t*>(y.data_ptr()), sp, rows,
                          cur_stream(x));
}

int64_t stem_wgrad_ws(int64_t N, int64_t H, int64_t W) {
  return (int64_t)gk::stem_wgrad_blocks((int)N, (int)H, (int)W) * 64 * 224;
}

void stem_wgrad(at::Tensor x, at::Tensor dy, at::Tensor out, at::Tensor part) {
  check_stem_x(x);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N &&
                  dy.size(1) == 64 && dy.size(2) == OH && dy.size(3) == OW &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_wgrad: dy must be channels-last bf16 [N, 64, OH, OW]");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(0) == 64 &&
                  out.size(1) == 3 && out.size(2) == 7 && out.size(3) == 7,
              "stem_wgrad: out must be fp32 [64, 3, 7, 7]");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= stem_wgrad_ws(N, H, W),
              "stem_wgrad: part must hold stem_wgrad_ws(N, H, W) floats");
  c10::DeviceGuard guard(x.device());
  gk::stem_wgrad(x.data_ptr(), x.scalar_type() == at::kFloat, (int)N, (int)H, (int)W,
                 static_cast<const uint16_t*>(dy.data_ptr()), part.data_ptr<float>(), out.data_ptr<float>(),
                 out.stride(0), out.stride(1), out.stride(2), out.stride(3), cur_stream(x));
}

// fp32 stem (stem_f32.hip): x [N, 3, 224, 224] channels-last fp32, w [64, 3, 7, 7] fp32,
// y [N, 64, 112, 112] channels-last fp32
int64_t stem_f32_fwd(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> stats) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && gk::stem_f32_supported((int)x.size(2), (int)x.size(3)) &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "stem_f32_fwd: x must be a channels-last fp32 [N, 3, 224, 224] GPU tensor (16-byte aligned)");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 &&
                  w.size(2) == 7 && w.size(3) == 7, "stem_f32_fwd: w must be fp32 [64, 3, 7, 7]");
  const int64_t N = x.size(0);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kFloat && y.dim() == 4 && y.size(0) == N && y.size(1) == 64 &&
                  y.size(2) == 112 && y.size(3) == 112 && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_f32_fwd: y must be a channels-last fp32 [N, 64, 112, 112] GPU tensor");
  int rows = 0;
  float* sp = stats_ptr(stats, 64, &rows);
  c10::DeviceGuard guard(x.device());
  return gk::stem_f32_forward(x.data_ptr<float>(), (int)N, (int)x.size(2), (int)x.size(3), w.data_ptr<float>(),
                              w.stride(0), w.stride(1), w.stride(2), w.stride(3), y.data_ptr<float>(), sp, rows,
                              cur_stream(x));
}

// bf16x6 stem forward: as stem_f32_fwd, plus wp3 = bf16 workspace of
// stem_f32x6_wplanes() elements for the split weight planes
int64_t stem_f32x6_wplanes() { return gk::stem_f32x6_wplanes(); }

int64_t stem_f32x6_fwd(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> stats, at::Tensor wp3) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && gk::stem_f32_supported((int)x.size(2), (int)x.size(3)) &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "stem_f32x6_fwd: x must be a channels-last fp32 [N, 3, 224, 224] GPU tensor (16-byte aligned)");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 &&
                  w.size(2) == 7 && w.size(3) == 7, "stem_f32x6_fwd: w must be fp32 [64, 3, 7, 7]");
  const int64_t N = x.size(0);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kFloat && y.dim() == 4 && y.size(0) == N && y.size(1) == 64 &&
                  y.size(2) == 112 && y.size(3) == 112 && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_f32x6_fwd: y must be a channels-last fp32 [N, 64, 112, 112] GPU tensor");
  TORCH_CHECK(wp3.is_cuda() && wp3.scalar_type() == at::kBFloat16 && wp3.is_contiguous() &&
                  wp3.numel() >= gk::stem_f32x6_wplanes() && reinterpret_cast<uintptr_t>(wp3.data_ptr()) % 16 == 0,
              "stem_f32x6_fwd: wp3 must be a contiguous bf16 GPU tensor of stem_f32x6_wplanes() elements");
  int rows = 0;
  float* sp = stats_ptr(stats, 64, &rows);
  c10::DeviceGuard guard(x.device());
  return gk::stem_f32x6_forward(x.data_ptr<float>(), (int)N, (int)x.size(2), (int)x.size(3), w.data_ptr<float>(),
                                w.stride(0), w.stride(1), w.stride(2), w.stride(3),
                                static_cast<uint16_t*>(wp3.data_ptr()), y.data_ptr<float>(), sp, rows, cur_stream(x));
}

int64_t stem_f32_wgrad_ws(int64_t N) { return (int64_t)gk::stem_f32_wgrad_blocks((int)N) * 64 * 148; }

void stem_f32_wgrad(at::Tensor x, at::Tensor dy, at::Tensor out, at::Tensor part, bool x6) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && gk::stem_f32_supported((int)x.size(2), (int)x.size(3)) &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "stem_f32_wgrad: x must be a channels-last fp32 [N, 3, 224, 224] GPU tensor (16-byte aligned)");
  const int64_t N = x.size(0);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kFloat && dy.dim() == 4 && dy.size(0) == N &&
                  dy.size(1) == 64 && dy.size(2) == 112 && dy.size(3) == 112 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_f32_wgrad: dy must be a channels-last fp32 [N, 64, 112, 112] GPU tensor");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(0) == 64 &&
                  out.size(1) == 3 && out.size(2) == 7 && out.size(3) == 7, "stem_f32_wgrad: out must be fp32 [64, 3, 7, 7]");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= stem_f32_wgrad_ws(N), "stem_f32_wgrad: part must hold stem_f32_wgrad_ws(N) floats");
  c10::DeviceGuard guard(x.device());
  gk::stem_f32_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), (int)N, (int)x.size(2), (int)x.size(3),
                     part.data_ptr<float>(), out.data_ptr<float>(), out.stride(0), out.stride(1), out.stride(2),
                     out.stride(3), x6, cur_stream(x));
}

// optional device seed word (graph replays): int32[>=1] on the GPU
const uint32_t* seed_word(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "seed_dev must be a GPU int32[>=1]");
  return reinterpret_cast<const uint32_t*>(t->data_ptr<int32_t>());
}

// C[M, N] = A[M, K] . B[N, K]^T
const float* bias_ptr(const c10::optional<at::Tensor>& b, int64_t N) {
  if (!b.has_value() || !b->defined()) return nullptr;
  TORCH_CHECK(b->is_cuda() && b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == N,
              "bias must be a contiguous fp32 [N] GPU tensor");
  return b->data_ptr<float>();
}

// BatchNorm-backward epilogue operands (gemm.hip BnBwd): all-or-nothing on h
bool bn_bwd_args(const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& dy2,
                 const c10::optional<at::Tensor>& mask, int64_t M, int64_t N,
                 int64_t ldc, bool has_stats, at::ScalarType dt, gk::BnBwdArgs* out) {
  if (!h.has_value() || !h->defined()) return false;
  TORCH_CHECK(has_stats, "BN-backward epilogue needs the stats partials buffer");
  auto rows_ok = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.numel() == M * N &&
                    (t.dim() == 2 ? t.stride(0) == ldc && t.stride(1) == 1
                                  : t.is_contiguous(at::MemoryFormat::ChannelsLast) && ldc == N),
                what, " must have C's dtype, shape and row stride");
  };
  rows_ok(*h, "bn h");
  out->h = h->data_ptr();
  out->dy2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    rows_ok(*dy2, "bn dy2");
    out->dy2 = dy2->data_ptr();
  }
  out->mask = nullptr;
  if (mask.has_value() && mask->defined()) {
    const int64_t V = dt == at::kFloat ? 4 : 8;   // channels per mask byte (bn_act.hip)
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->numel() >= M * (N / V),
                "bn mask must hold M * N / V bytes");
    out->mask = mask->data_ptr<uint8_t>();
  }
  return true;
}

// lazy BN-backward operand (gemm.hip LazyA): x like dz (the operand), fp32
// coef [C][4], padz / padx [C]; all four or none
bool lazy_args(const c10::optional<at::Tensor>& x, const c10::optional<at::Tensor>& coef,
               const c10::optional<at::Tensor>& padz, const c10::optional<at::Tensor>& padx, const at::Tensor& dz,
               int64_t C, gk::LazyArgs* out) {
  if (!x.has_value() || !x->defined()) return false;
  TORCH_CHECK(dz.scalar_type() == at::kFloat, "lazy BN operand: fp32 kernels only");
  TORCH_CHECK(x->is_cuda() && x->scalar_type() == dz.scalar_type() && x->sizes() == dz.sizes() &&
                  x->strides() == dz.strides(),
              "lz_x must match the dz operand's dtype, shape and strides");
  TORCH_CHECK(coef.has_value() && coef->defined() && coef->is_cuda() && coef->scalar_type() == at::kFloat &&
                  coef->is_contiguous() && coef->numel() >= 4 * C,
              "lz_coef must be a contiguous fp32 [C, 4] GPU tensor");
  for (const c10::optional<at::Tensor>* t : {&padz, &padx})
    TORCH_CHECK(t->has_value() && (*t)->defined() && (*t)->is_cuda() && (*t)->scalar_type() == dz.scalar_type() &&
                    (*t)->is_contiguous() && (*t)->numel() >= C,
                "lz_padz / lz_padx must be contiguous [C] GPU tensors of dz's dtype");
  TORCH_CHECK(C > 0 && C % 64 == 0, "lazy BN operand: channels must be a multiple of 64");
  out->x = x->data_ptr();
  out->coef = coef->data_ptr<float>();
  out->padz = padz->data_ptr();
  out->padx = padx->data_ptr();
  out->C = (int)C;
  return true;
}

int64_t gemm_nt(at::Tensor A, at::Tensor B, at::Tensor C, int64_t cfg, int64_t max_blocks,
                c10::optional<at::Tensor> stats, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> bn_h,
                c10::optional<at::Tensor> bn_dy2, c10::optional<at::Tensor> bn_mask, c10::optional<at::Tensor> lz_x, c10::optional<at::Tensor> lz_coef,
                c10::optional<at::Tensor> lz_padz, c10::optional<at::Tensor> lz_padx) {
  check_rows(A, "A", A);
  check_rows(B, "B", A);
  check_rows(C, "C", A);
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && C.size(0) == M && C.size(1) == N, "gemm_nt: shape mismatch");
  TORCH_CHECK(gk::gemm_supported(N, K), "gemm_nt: N and K must be multiples of 64");
  TORCH_CHECK(M > 0, "gemm_nt: empty M");
  int rows = 0;
  float* sp = stats_ptr(stats, N, &rows);
  gk::BnBwdArgs bn{};
  const bool has_bn = bn_bwd_args(bn_h, bn_dy2, bn_mask, M, N, C.stride(0), sp != nullptr, C.scalar_type(), &bn);
  TORCH_CHECK(!has_bn || !bias.has_value() || !bias->defined(), "gemm_nt: bias and BN epilogue are exclusive");
  gk::LazyArgs lz{};
  const bool has_lz = lazy_args(lz_x, lz_coef, lz_padz, lz_padx, A, K, &lz);
  c10::DeviceGuard guard(A.device());
  // cfg digit 10000: split-K over S = (cfg / 10000) % 10 fp32 partial planes (gemm.hip nt_splitk_reduce_kernel);
  // digit 100000: fp32 operands multiplied as bf16x6 products (gemm_kern.h X6)
  const int64_t S = (cfg / 10000) % 10;
  at::Tensor ws;
  if (S > 1) {
    TORCH_CHECK(A.scalar_type() == at::kFloat && !has_lz && S <= 16 && K % (64 * S) == 0,
                "gemm_nt split-K: fp32, no lazy operand, S <= 16 and K % (64 S) == 0");
    ws = at::empty({S, M, N}, A.options().dtype(at::kFloat));
  }
  // digit 300000: register-staged bf16x6 with B split into bf16 planes here, once per call
  at::Tensor b3;
  if ((cfg / 100000) % 10 == 3) {
    TORCH_CHECK(B.scalar_type() == at::kFloat && K % 32 == 0, "gemm_nt: cfg family 3 takes fp32 operands");
    b3 = at::empty({N, 3 * K}, B.options().dtype(at::kBFloat16));
    gk::split3_rows(B.data_ptr<float>(), B.stride(0), b3.data_ptr(), N, (int)K, cur_stream(A));
  }
  const int r = gk::gemm_nt(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0), M, (int)N,
                            (int)K, A.scalar_type() == at::kFloat, (int)cfg, (int)max_blocks, sp, rows,
                            bias_ptr(bias, N), has_bn ? &bn : nullptr, has_lz ? &lz : nullptr, cur_stream(A),
                            S > 1 ? ws.data_ptr<float>() : nullptr, b3.defined() ? b3.data_ptr() : nullptr);
  TORCH_CHECK(r != -2, "gemm_nt: the register-staged bf16x6 kernels (cfg digit 200000/300000) take plain row GEMMs only");
  TORCH_CHECK(r >= 0, "gemm_nt: the lazy operand's coefficient table does not fit this tile configuration");
  return r;
}

// W[N, K] += G[M, N]^T . X[M, K]   (fp32 W, float atomics)
void gemm_tn_acc(at::Tensor G, at::Tensor X, at::Tensor W, int64_t cfg, int64_t splits, c10::optional<at::Tensor> lz_x, c10::optional<at::Tensor> lz_coef,
                c10::optional<at::Tensor> lz_padz, c10::optional<at::Tensor> lz_padx) {
  check_rows(G, "G", G);
  check_rows(X, "X", G);
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == at::kFloat && W.dim() == 2 && W.stride(1) == 1,
              "W must be a 2-D fp32 GPU tensor with contiguous rows");
  const int64_t M = G.size(0), N = G.size(1), K = X.size(1);
  TORCH_CHECK(X.size(0) == M && W.size(0) == N && W.size(1) == K, "gemm_tn_acc: shape mismatch");
  TORCH_CHECK(gk::gemm_supported(N, K), "gemm_tn_acc: N and K must be multiples of 64");
  if (M == 0) return;
  gk::LazyArgs lz{};
  const bool has_lz = lazy_args(lz_x, lz_coef, lz_padz, lz_padx, G, N, &lz);
  c10::DeviceGuard guard(G.device());
  const int rc = gk::gemm_tn_acc(G.data_ptr(), G.stride(0), X.data_ptr(), X.stride(0), W.data_ptr<float>(), W.stride(0), M, (int)N,
                  (int)K, G.scalar_type() == at::kFloat, (int)cfg, (int)splits, has_lz ? &lz : nullptr, cur_stream(G));
  TORCH_CHECK(rc != -2, "gemm_tn_acc: the register-staged bf16x6 kernels (cfg digit 200000) take plain row GEMMs only");
}

// implicit-GEMM convolution over NHWC bf16 (x: [N, C, H, W] channels-last,
// w: [Cout, C, KH, KW] channels-last, y: [N, Cout, OH, OW] channels-last)
// the padding row: >= 128 zero bytes (one K slice of either dtype)
void check_zero(const at::Tensor& zero) {
  TORCH_CHECK(zero.is_cuda() && zero.is_contiguous() && zero.numel() * zero.element_size() >= 128,
              "zero must hold >= 128 zero bytes");
}

void check_conv(const at::Tensor& x, const at::Tensor& w, const at::Tensor& zero) {
  TORCH_CHECK(x.is_cuda() && is_gemm_dtype(x) && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv: x must be a channels-last bf16 or fp32 GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == x.scalar_type() && w.dim() == 4 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) == x.size(1),
              "conv: w must be a channels-last [Cout, C, KH, KW] GPU tensor of x's dtype");
  TORCH_CHECK(x.size(1) % 64 == 0 && w.size(0) % 64 == 0, "conv: C and Cout must be multiples of 64");
  check_zero(zero);
}

int64_t conv_nt(at::Tensor x, at::Tensor w, at::Tensor y, at::Tensor zero, int64_t stride, int64_t pad, int64_t cfg,
                int64_t max_blocks, c10::optional<at::Tensor> stats, c10::optional<at::Tensor> bias,
                c10::optional<at::Tensor> bn_h, c10::optional<at::Tensor> bn_dy2, c10::optional<at::Tensor> bn_mask,
                c10::optional<at::Tensor> lz_x, c10::optional<at::Tensor> lz_coef,
                c10::optional<at::Tensor> lz_padz, c10::optional<at::Tensor> lz_padx) {
  check_conv(x, w, zero);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Co = w.size(0), KH = w.size(2), KW = w.size(3);
  const int64_t OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(KH <= 4 && KW <= 4, "conv_nt: kernels up to 4x4 (gemm.hip kMaxTaps)");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == x.scalar_type() && y.dim() == 4 &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && y.size(0) == N && y.size(1) == Co &&
                  y.size(2) == OH && y.size(3) == OW,
              "conv_nt: y must be channels-last [N, Cout, OH, OW] of x's dtype");
  const int64_t M = N * OH * OW;
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 32), "conv_nt: M out of range");
  int rows = 0;
  float* sp = stats_ptr(stats, Co, &rows);
  gk::BnBwdArgs bn{};
  const bool has_bn = bn_bwd_args(bn_h, bn_dy2, bn_mask, M, Co, Co, sp != nullptr, y.scalar_type(), &bn);
  TORCH_CHECK(!has_bn || !bias.has_value() || !bias->defined(), "conv_nt: bias and BN epilogue are exclusive");
  gk::LazyArgs lz{};
  const bool has_lz = lazy_args(lz_x, lz_coef, lz_padz, lz_padx, x, C, &lz);
  c10::DeviceGuard guard(x.device());
  // cfg digit 10000: split-K over S = (cfg / 10000) % 10 fp32 partial planes of the (tap, channel) slices
  const int64_t S = (cfg / 10000) % 10;
  at::Tensor ws;
  if (S > 1) {
    TORCH_CHECK(x.scalar_type() == at::kFloat && !has_lz && S <= 16 && C % 32 == 0 && (KH * KW * C / 32) % S == 0,
                "conv_nt split-K: fp32, no lazy operand, S <= 16 dividing the K slices");
    ws = at::empty({S, M, Co}, x.options());
  }
  at::Tensor b3;
  if ((cfg / 100000) % 10 == 3) {
    const int64_t K = KH * KW * C;
    TORCH_CHECK(x.scalar_type() == at::kFloat, "conv_nt: cfg family 3 takes fp32 operands");
    b3 = at::empty({Co, 3 * K}, w.options().dtype(at::kBFloat16));
    gk::split3_rows(w.data_ptr<float>(), K, b3.data_ptr(), Co, (int)K, cur_stream(x));
  }
  const int r = gk::conv_nt(x.data_ptr(), zero.data_ptr(), (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)stride,
                            (int)pad, (int)KH, (int)KW, w.data_ptr(), y.data_ptr(), M, (int)Co,
                            x.scalar_type() == at::kFloat, (int)cfg, (int)max_blocks, sp, rows, bias_ptr(bias, Co),
                            has_bn ? &bn : nullptr, has_lz ? &lz : nullptr, cur_stream(x),
                            S > 1 ? ws.data_ptr<float>() : nullptr, b3.defined() ? b3.data_ptr() : nullptr);
  TORCH_CHECK(r != -2, "conv_nt: the register-staged bf16x6 kernels (cfg digit 200000/300000) take plain row GEMMs only");
  TORCH_CHECK(r >= 0, "conv_nt: the lazy operand's coefficient table does not fit this tile configuration");
  return r;
}

// Winograd F(2x2, 3x3) fp32 convolution (winograd.hip).  w: forward weight
// [K, C, 3, 3] channels-last fp32; flip = false: u = transform of w for the
// forward (Ci = C, Co = K); flip = true: of the grad-input filter (Ci = K,
// Co = C).  u: contiguous fp32 with 16 * K * C elements.
// ---------------------------------------------------------------------------
// batched per-step weight re-layouts (prep.hip; table packed by ops/weight_prep.py)
// ---------------------------------------------------------------------------
int64_t weight_prep_blocks(int64_t kind, int64_t R, int64_t S) { return gk::weight_prep_blocks((int)kind, (int)R, (int)S); }

void weight_prep(at::Tensor table, int64_t ndesc, int64_t total_blocks) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte && table.is_contiguous() &&
                  table.numel() == ndesc * (int64_t)sizeof(gk::PrepDesc),
              "weight_prep: table must be a contiguous GPU uint8 tensor of ndesc descriptors");
  TORCH_CHECK(ndesc > 0 && ndesc <= gk::weight_prep_max_descs(), "weight_prep: 1..", gk::weight_prep_max_descs(),
              " descriptors");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(table.data_ptr()) % 8 == 0, "weight_prep: table must be 8-byte aligned");
  c10::DeviceGuard guard(table.device());
  gk::weight_prep(reinterpret_cast<const gk::PrepDesc*>(table.data_ptr()), (int)ndesc, total_blocks,
                  cur_stream(table));
}

void wino_weights(at::Tensor w, at::Tensor u, bool flip) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wino_weights: w must be a channels-last fp32 [K, C, 3, 3] GPU tensor");
  const int64_t K = w.size(0), C = w.size(1);
  const int64_t Co = flip ? C : K, Ci = flip ? K : C;
  TORCH_CHECK(Ci % 8 == 0 && Co % 64 == 0, "wino_weights: input channels % 8 and output channels % 64");
  TORCH_CHECK(u.is_cuda() && u.scalar_type() == at::kFloat && u.is_contiguous() && u.numel() == 16 * K * C,
              "wino_weights: u must be a contiguous fp32 tensor of 16 * K * C elements");
  c10::DeviceGuard guard(w.device());
  gk::wino_weights(w.data_ptr<float>(), u.data_ptr<float>(), (int)Co, (int)Ci, flip ? 1 : 0, cur_stream(w));
}

// y = conv3x3(x) (stride 1, padding 1) from the transformed filter u;
// x: [N, Ci, H, W], y: [N, Co, H, W], both channels-last fp32.  Optional
// BatchNorm statistics partials / BN-backward epilogue as conv_nt.
int64_t wino_conv(at::Tensor x, at::Tensor u, at::Tensor y, int64_t max_blocks, c10::optional<at::Tensor> stats,
                  c10::optional<at::Tensor> bn_h, c10::optional<at::Tensor> bn_dy2, c10::optional<at::Tensor> bn_mask,
                  int64_t splits) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wino_conv: x must be a channels-last fp32 GPU tensor");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kFloat && y.dim() == 4 &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && y.size(0) == N && y.size(2) == H &&
                  y.size(3) == W,
              "wino_conv: y must be a channels-last fp32 [N, Co, H, W] GPU tensor");
  const int64_t Co = y.size(1);
  TORCH_CHECK(Ci % 8 == 0 && Co % 64 == 0, "wino_conv: Ci % 8 == 0 and Co % 64 == 0");
  TORCH_CHECK(u.is_cuda() && u.scalar_type() == at::kFloat && u.is_contiguous() && u.numel() == 16 * Ci * Co,
              "wino_conv: u must hold 16 * Ci * Co fp32 (wino_weights)");
  TORCH_CHECK(N * ((H + 1) / 2) * ((W + 1) / 2) < (int64_t(1) << 31) && x.numel() > 0 &&
                  x.numel() * 4 < (int64_t(1) << 31) && y.numel() * 4 < (int64_t(1) << 31),
              "wino_conv: size out of range (input / output bytes < 2^31: buffer-descriptor addressing)");
  int rows = 0;
  float* sp = stats_ptr(stats, Co, &rows);
  gk::BnBwdArgs bn{};
  const bool has_bn = bn_bwd_args(bn_h, bn_dy2, bn_mask, N * H * W, Co, Co, sp != nullptr, at::kFloat, &bn);
  c10::DeviceGuard guard(x.device());
  // splits > 1: input-channel split into fp32 partial planes + one reduce pass
  TORCH_CHECK(splits >= 1 && splits <= 16 && Ci % (8 * splits) == 0, "wino_conv: splits in [1, 16] dividing Ci / 8");
  at::Tensor ws;
  if (splits > 1) ws = at::empty({splits, N * H * W, Co}, x.options());
  const int r = gk::wino_conv(x.data_ptr<float>(), u.data_ptr<float>(), y.data_ptr<float>(), (int)N, (int)H, (int)W,
                              (int)Ci, (int)Co, (int)max_blocks, sp, rows, has_bn ? &bn : nullptr, cur_stream(x),
                              (int)splits, splits > 1 ? ws.data_ptr<float>() : nullptr);
  TORCH_CHECK(r >= 0, "wino_conv: split configuration refused");
  return r;
}

// bf16x6 Winograd (wino_x6.hip): u3 = bf16 [Ci/32 * 16 * 3 * Co * 32]
void wino_x6_weights(at::Tensor w, at::Tensor u3, bool flip) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wino_x6_weights: w must be a channels-last fp32 [K, C, 3, 3] GPU tensor");
  const int64_t K = w.size(0), C = w.size(1);
  const int64_t Co = flip ? C : K, Ci = flip ? K : C;
  TORCH_CHECK(Ci % 32 == 0 && Co % 32 == 0, "wino_x6_weights: input and output channels % 32");
  TORCH_CHECK(u3.is_cuda() && u3.scalar_type() == at::kBFloat16 && u3.is_contiguous() && u3.numel() == 48 * K * C,
              "wino_x6_weights: u3 must be a contiguous bf16 tensor of 48 * K * C elements");
  c10::DeviceGuard guard(w.device());
  gk::wino_x6_weights(w.data_ptr<float>(), reinterpret_cast<uint16_t*>(u3.data_ptr()), (int)Co, (int)Ci,
                      flip ? 1 : 0, cur_stream(w));
}

int64_t wino_x6_conv(at::Tensor x, at::Tensor u3, at::Tensor y, int64_t max_blocks, c10::optional<at::Tensor> stats,
                     c10::optional<at::Tensor> bn_h, c10::optional<at::Tensor> bn_dy2,
                     c10::optional<at::Tensor> bn_mask) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wino_x6_conv: x must be a channels-last fp32 GPU tensor");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kFloat && y.dim() == 4 &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && y.size(0) == N && y.size(2) == H &&
                  y.size(3) == W,
              "wino_x6_conv: y must be a channels-last fp32 [N, Co, H, W] GPU tensor");
  const int64_t Co = y.size(1);
  TORCH_CHECK(Ci % 32 == 0 && Co % 32 == 0, "wino_x6_conv: Ci % 32 == 0 and Co % 32 == 0");
  TORCH_CHECK(u3.is_cuda() && u3.scalar_type() == at::kBFloat16 && u3.is_contiguous() && u3.numel() == 48 * Ci * Co,
              "wino_x6_conv: u3 must hold 48 * Ci * Co bf16 (wino_x6_weights)");
  TORCH_CHECK(N * ((H + 1) / 2) * ((W + 1) / 2) < (int64_t(1) << 31) && x.numel() > 0 &&
                  x.numel() * 4 < (int64_t(1) << 31) && y.numel() * 4 < (int64_t(1) << 31),
              "wino_x6_conv: size out of range (input / output bytes < 2^31: buffer-descriptor addressing)");
  int rows = 0;
  float* sp = stats_ptr(stats, Co, &rows);
  gk::BnBwdArgs bn{};
  const bool has_bn = bn_bwd_args(bn_h, bn_dy2, bn_mask, N * H * W, Co, Co, sp != nullptr, at::kFloat, &bn);
  c10::DeviceGuard guard(x.device());
  const int r = gk::wino_x6_conv(x.data_ptr<float>(), reinterpret_cast<const uint16_t*>(u3.data_ptr()),
                                 y.data_ptr<float>(), (int)N, (int)H, (int)W, (int)Ci, (int)Co, (int)max_blocks, sp,
                                 rows, has_bn ? &bn : nullptr, cur_stream(x));
  TORCH_CHECK(r >= 0, "wino_x6_conv: configuration refused");
  return r;
}

// out ([K, C, 3, 3] channels-last fp32) += dW of the 3x3 stride-1 convolution
// x [N, C, H, W] -> dy [N, K, H, W] (channels-last fp32), Winograd F(2x2, 3x3);
// part: >= wino_wgrad_ws(...) fp32 workspace
int64_t wino_wgrad_ws(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K, int64_t splits) {
  return (int64_t)gk::wino_wgrad_splits((int)N, (int)H, (int)W, (int)C, (int)K, (int)splits) * 16 * K * C;
}

void wino_wgrad(at::Tensor x, at::Tensor dy, at::Tensor out, at::Tensor part, int64_t splits) {
  auto cl = [](const at::Tensor& t) {
    return t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast);
  };
  TORCH_CHECK(cl(x) && cl(dy) && cl(out), "wino_wgrad: x, dy, out must be channels-last fp32 GPU tensors");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "wino_wgrad: dy must be [N, K, H, W]");
  TORCH_CHECK(out.size(0) == K && out.size(1) == C && out.size(2) == 3 && out.size(3) == 3,
              "wino_wgrad: out must be [K, C, 3, 3]");
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0, "wino_wgrad: C and K must be multiples of 64");
  TORCH_CHECK(N * ((H + 1) / 2) * ((W + 1) / 2) < (int64_t(1) << 31) && x.numel() * 4 < (int64_t(1) << 31) &&
                  dy.numel() * 4 < (int64_t(1) << 31),
              "wino_wgrad: size out of range (x, dy bytes < 2^31: buffer-descriptor addressing)");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= wino_wgrad_ws(N, H, W, C, K, splits),
              "wino_wgrad: workspace too small (wino_wgrad_ws)");
  c10::DeviceGuard guard(x.device());
  gk::wino_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), part.data_ptr<float>(), out.data_ptr<float>(), (int)N,
                 (int)H, (int)W, (int)C, (int)K, (int)splits, cur_stream(x));
}

// grad-input of a stride-2 convolution (1x1 / pad 0 or 3x3 / pad 1) through the
// stride-1 MFMA kernels: dX = conv_transpose(dY, W) splits into the four
// (row, column) parity classes of dX; class (a, b) is a stride-1 KH'xKW' conv
// over dY (taps kh with kh = a + 1 mod 2: {1} for even rows, {2, 0} for odd)
// whose output lands on the class's pixels (gemm.hip ConvGeo remap).
// dy: [N, K, OH, OW] channels-last bf16; w: [K, C, k, k] channels-last bf16;
// dx: [N, C, H, W] channels-last bf16 (every pixel written).
void conv_dgrad_s2(at::Tensor dy, at::Tensor w, at::Tensor dx, at::Tensor zero, int64_t cfg, int64_t max_blocks,
                   c10::optional<at::Tensor> lz_x, c10::optional<at::Tensor> lz_coef,
                c10::optional<at::Tensor> lz_padz, c10::optional<at::Tensor> lz_padx) {
  TORCH_CHECK(dy.is_cuda() && is_gemm_dtype(dy) && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_s2: dy must be channels-last bf16 or fp32");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == dy.scalar_type() && w.dim() == 4 && w.size(0) == dy.size(1) &&
                  w.size(2) == w.size(3) && (w.size(2) == 1 || w.size(2) == 3),
              "conv_dgrad_s2: w must be [K, C, k, k] of dy's dtype, k in {1, 3}");
  TORCH_CHECK(dx.is_cuda() && dx.scalar_type() == dy.scalar_type() && dx.dim() == 4 && dx.size(0) == dy.size(0) &&
                  dx.size(1) == w.size(1) && dx.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_s2: dx must be channels-last [N, C, H, W] of dy's dtype");
  const bool f32 = dy.scalar_type() == at::kFloat;
  const int64_t N = dy.size(0), K = dy.size(1), OHd = dy.size(2), OWd = dy.size(3);
  const int64_t C = w.size(1), k = w.size(2), H = dx.size(2), W = dx.size(3);
  const int64_t p = k / 2;
  TORCH_CHECK((H + 2 * p - k) / 2 + 1 == OHd && (W + 2 * p - k) / 2 + 1 == OWd, "conv_dgrad_s2: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && C % 64 == 0, "conv_dgrad_s2: channels must be multiples of 64");
  check_zero(zero);
  TORCH_CHECK(N * H * W < (int64_t(1) << 31), "conv_dgrad_s2: too many pixels");
  gk::LazyArgs lzv{};
  const gk::LazyArgs* lz = lazy_args(lz_x, lz_coef, lz_padz, lz_padx, dy, K, &lzv) ? &lzv : nullptr;
  c10::DeviceGuard guard(dy.device());
  const hipStream_t st = cur_stream(dy);
  if (k == 1) {   // one class (even, even), zeros elsewhere; B = W^T [C][K]
    const at::Tensor wt = w.reshape({K, C}).t().contiguous();
    const int r = gk::conv_nt_remap(dy.data_ptr(), K, zero.data_ptr(), (int)OHd, (int)OWd, (int)K, (int)OHd,
                                    (int)OWd, 1, 1, wt.data_ptr(), dx.data_ptr(), N * OHd * OWd, (int)C, (int)H, (int)W,
                                    0, 0, 1, f32, (int)cfg, (int)max_blocks, lz, st);
    TORCH_CHECK(r >= 0, "conv_dgrad_s2: the lazy operand's coefficient table does not fit this tile configuration");
    return;
  }
  // [C][kh][kw][K] = W[K][C][kh][kw]
  const at::Tensor wt = w.permute({1, 2, 3, 0}).contiguous();
  for (int a = 0; a < 2; ++a) {
    for (int b = 0; b < 2; ++b) {
      const int64_t OHc = (H - a + 1) / 2, OWc = (W - b + 1) / 2;
      if (OHc <= 0 || OWc <= 0) continue;
      // class-conv tap j reads dY row oh + j: j = 0 <-> kh = 2 - a ... (a = 0: kh = 1; a = 1: kh = 2, 0)
      // taps as device-side slices (no index upload): {1} or {2, 0}
      at::Tensor wc = a == 0 ? wt.slice(1, 1, 2) : wt.slice(1, 0, 3, 2).flip({1});
      wc = b == 0 ? wc.slice(2, 1, 2) : wc.slice(2, 0, 3, 2).flip({2});
      wc = wc.contiguous();
      // a refused tile (lazy operand too large) must fail loudly: its class's pixels would stay unwritten
      const int r = gk::conv_nt_remap(dy.data_ptr(), K, zero.data_ptr(), (int)OHd, (int)OWd, (int)K, (int)OHc,
                                      (int)OWc, a == 0 ? 1 : 2, b == 0 ? 1 : 2, wc.data_ptr(), dx.data_ptr(),
                                      N * OHc * OWc, (int)C, (int)H, (int)W, a, b, 0, f32, (int)cfg, (int)max_blocks,
                                      lz, st);
      TORCH_CHECK(r >= 0, "conv_dgrad_s2: the lazy operand's coefficient table does not fit this tile configuration");
    }
  }
}

// tap-parallel 3x3 stride-1 grad-weight (wgrad3.hip): out (fp32 [K, C, 3, 3]) += dW
int64_t wgrad3_ws(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K) {
  return gk::wgrad3_ws_floats((int)N, (int)H, (int)W, (int)C, (int)K);
}

void conv3_wgrad(at::Tensor dy, at::Tensor x, at::Tensor out, at::Tensor part, at::Tensor zero) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3_wgrad: x must be channels-last bf16 [N, C, H, W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N &&
                  dy.size(2) == H && dy.size(3) == W && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3_wgrad: dy must be channels-last bf16 [N, K, H, W]");
  const int64_t K = dy.size(1);
  TORCH_CHECK(gk::wgrad3_supported((int)H, (int)W, (int)C, (int)K), "conv3_wgrad: unsupported shape");
  TORCH_CHECK(N * H * W < (int64_t(1) << 31), "conv3_wgrad: too many pixels");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(0) == K &&
                  out.size(1) == C && out.size(2) == 3 && out.size(3) == 3,
              "conv3_wgrad: out must be fp32 [K, C, 3, 3]");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= wgrad3_ws(N, H, W, C, K),
              "conv3_wgrad: part must hold wgrad3_ws floats");
  c10::DeviceGuard guard(x.device());
  TORCH_CHECK(zero.is_cuda() && zero.scalar_type() == at::kBFloat16 && zero.numel() >= 64, "zero: >= 64 bf16");
  gk::wgrad3_acc(dy.data_ptr(), x.data_ptr(), zero.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)K,
                 part.data_ptr<float>(),
                 out.data_ptr<float>(), out.stride(0), out.stride(1), out.stride(2), out.stride(3), cur_stream(x));
}

// wout: fp32 [Cout, C, KH, KW] channels-last (memory [Cout][KH][KW][C]); += dW
void conv_tn_acc(at::Tensor dy, at::Tensor x, at::Tensor wout, at::Tensor zero, int64_t stride, int64_t pad,
                 int64_t cfg, int64_t splits, c10::optional<at::Tensor> lz_x, c10::optional<at::Tensor> lz_coef,
                c10::optional<at::Tensor> lz_padz, c10::optional<at::Tensor> lz_padx) {
  TORCH_CHECK(wout.is_cuda() && wout.scalar_type() == at::kFloat && wout.dim() == 4 &&
                  wout.is_contiguous(at::MemoryFormat::ChannelsLast) && wout.size(1) == x.size(1),
              "conv_tn_acc: wout must be a channels-last fp32 [Cout, C, KH, KW] tensor");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Co = wout.size(0), KH = wout.size(2), KW = wout.size(3);
  TORCH_CHECK(x.is_cuda() && is_gemm_dtype(x) && x.is_contiguous(at::MemoryFormat::ChannelsLast) && C % 64 == 0 &&
                  Co % 64 == 0,
              "conv_tn_acc: x must be channels-last bf16 or fp32 with C, Cout % 64 == 0");
  check_zero(zero);
  TORCH_CHECK(x.numel() < (int64_t(1) << 31), "conv_tn_acc: x too large for 32-bit gather offsets");
  const int64_t OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == x.scalar_type() && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.size(0) == N && dy.size(1) == Co &&
                  dy.size(2) == OH && dy.size(3) == OW,
              "conv_tn_acc: dy must be channels-last [N, Cout, OH, OW] of x's dtype");
  const int64_t M = N * OH * OW;
  TORCH_CHECK(M < (int64_t(1) << 32), "conv_tn_acc: M out of range");
  if (M == 0) return;
  gk::LazyArgs lz{};
  const bool has_lz = lazy_args(lz_x, lz_coef, lz_padz, lz_padx, dy, Co, &lz);
  c10::DeviceGuard guard(x.device());
  const int rc = gk::conv_tn_acc(dy.data_ptr(), x.data_ptr(), zero.data_ptr(), (int)H, (int)W, (int)C, (int)OH, (int)OW,
                  (int)stride, (int)pad, (int)KH, (int)KW, wout.data_ptr<float>(), M, (int)Co,
                  x.scalar_type() == at::kFloat, (int)cfg, (int)splits, has_lz ? &lz : nullptr, cur_stream(x));
  TORCH_CHECK(rc != -2, "conv_tn_acc: the register-staged bf16x6 kernels (cfg digit 200000) take plain row GEMMs only");
}

// fused residual add (+ dropout) + LayerNorm (ln.hip)
bool add_ln_supported(int64_t H) { return gk::add_ln_supported((int)H); }
int64_t add_ln_ws_floats(int64_t R, int64_t H) { return 2 * gk::add_ln_partial_rows(R) * H; }

void check_rows_ln(const at::Tensor& t, const char* name, int64_t R, int64_t H, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous() && t.numel() == R * H &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous, 16-byte aligned GPU tensor of R*H elements (bf16 or fp32, all alike)");
}

void add_ln_forward(at::Tensor a, at::Tensor x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                    at::Tensor y, at::Tensor h, at::Tensor mean, at::Tensor rstd, double eps, double p, int64_t seed,
                    c10::optional<at::Tensor> seed_dev) {
  const int64_t H = x.size(-1), R = x.numel() / H;
  TORCH_CHECK(gk::add_ln_supported((int)H), "add_ln: unsupported hidden size");
  const auto dt = x.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "add_ln: bf16 or fp32 storage");
  for (auto* t : {&a, &x, &y, &h}) check_rows_ln(*t, "add_ln tensor", R, H, dt);
  TORCH_CHECK(mean.numel() >= R && rstd.numel() >= R && mean.scalar_type() == at::kFloat &&
                  rstd.scalar_type() == at::kFloat, "mean/rstd: fp32 [R]");
  const float* gp = gamma.has_value() && gamma->defined() ? gamma->data_ptr<float>() : nullptr;
  const float* bp = beta.has_value() && beta->defined() ? beta->data_ptr<float>() : nullptr;
  if (gp) TORCH_CHECK(gamma->numel() == H && gamma->is_contiguous(), "gamma: fp32 [H]");
  if (bp) TORCH_CHECK(beta->numel() == H && beta->is_contiguous(), "beta: fp32 [H]");
  c10::DeviceGuard guard(x.device());
  gk::add_ln_forward(a.data_ptr(), x.data_ptr(), gp, bp, y.data_ptr(), h.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), R, (int)H, (float)eps, (float)p, (uint32_t)seed, seed_word(seed_dev),
                     cur_stream(x), dt == at::kFloat);
}

void add_ln_backward(at::Tensor dy, at::Tensor h, at::Tensor mean, at::Tensor rstd, c10::optional<at::Tensor> gamma,
                     at::Tensor dx, c10::optional<at::Tensor> da, c10::optional<at::Tensor> dgamma,
                     c10::optional<at::Tensor> dbeta, bool accumulate, at::Tensor ws, double p, int64_t seed,
                     c10::optional<at::Tensor> seed_dev) {
  const int64_t H = h.size(-1), R = h.numel() / H;
  const auto dt = h.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "add_ln: bf16 or fp32 storage");
  for (auto* t : {&dy, &h, &dx}) check_rows_ln(*t, "add_ln tensor", R, H, dt);
  if (da.has_value() && da->defined()) check_rows_ln(*da, "da", R, H, dt);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= 2 * gk::add_ln_partial_rows(R) * H, "ws too small");
  auto f32 = [&](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == H && t->is_contiguous(), "fp32 [H] expected");
    return t->data_ptr<float>();
  };
  c10::DeviceGuard guard(h.device());
  gk::add_ln_backward(dy.data_ptr(), h.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), f32(gamma),
                      dx.data_ptr(), da.has_value() && da->defined() ? da->data_ptr() : nullptr, f32(dgamma),
                      f32(dbeta), accumulate ? 1 : 0, ws.data_ptr<float>(), R, (int)H, (float)p, (uint32_t)seed,
                      seed_word(seed_dev), cur_stream(h), dt == at::kFloat);
}

// fused softmax cross-entropy (xent.hip)
bool xent_supported(int64_t V) { return gk::xent_supported((int)V); }

void xent_forward(at::Tensor logits, at::Tensor labels, at::Tensor lse, at::Tensor loss, int64_t ignore) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "xent: logits must be contiguous bf16 [R, V]");
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(gk::xent_supported((int)V), "xent: V must be even");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == R && labels.is_contiguous(),
              "xent: labels int64 [R]");
  for (const at::Tensor* t : {&lse, &loss})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == R && t->is_contiguous(), "xent: fp32 [R]");
  c10::DeviceGuard guard(logits.device());
  gk::xent_forward(logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), loss.data_ptr<float>(), R,
                   (int)V, ignore, cur_stream(logits));
}

void xent_backward(at::Tensor logits, at::Tensor labels, at::Tensor lse, at::Tensor scale, at::Tensor grad,
                   int64_t ignore) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "xent: logits must be contiguous bf16 [R, V]");
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(gk::xent_supported((int)V), "xent: V must be even");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == R && labels.is_contiguous(), "xent: labels int64 [R]");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == R && scale.scalar_type() == at::kFloat &&
                  scale.numel() == 1 && scale.is_cuda(), "xent: lse fp32 [R], scale fp32 [1]");
  TORCH_CHECK(grad.scalar_type() == at::kBFloat16 && grad.sizes() == logits.sizes() && grad.is_contiguous(),
              "xent: grad bf16 like logits");
  c10::DeviceGuard guard(logits.device());
  gk::xent_backward(logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), scale.data_ptr<float>(),
                    grad.data_ptr(), R, (int)V, ignore, cur_stream(logits));
}

// fused BERT input embedding (embed.hip)
bool emb_supported(int64_t H, int64_t NT) { return gk::emb_supported((int)H, (int)NT); }
int64_t emb_part_floats(int64_t H) { return (int64_t)gk::emb_type_parts() * 2 * H; }

void emb_forward(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor Ww, at::Tensor Wp, at::Tensor Wt,
                 at::Tensor out) {
  const int64_t B = ids.size(0), T = ids.size(1), M = B * T, H = Ww.size(1);
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.dim() == 2 && ids.is_contiguous(),
              "emb: ids must be contiguous int64 [B, T]");
  const int64_t* tp = nullptr;
  if (tt.has_value() && tt->defined()) {
    TORCH_CHECK(tt->scalar_type() == at::kLong && tt->numel() == M && tt->is_contiguous(), "emb: tt int64 [B, T]");
    tp = tt->data_ptr<int64_t>();
  }
  for (const at::Tensor* t : {&Ww, &Wp, &Wt})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(1) == H && t->is_contiguous(),
                "emb: tables must be contiguous fp32 [*, H]");
  TORCH_CHECK(gk::emb_supported((int)H, (int)Wt.size(0)) && T <= Wp.size(0), "emb: unsupported shape");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() == M * H && out.is_contiguous(),
              "emb: out fp32 [B, T, H]");
  c10::DeviceGuard guard(ids.device());
  gk::emb_forward(ids.data_ptr<int64_t>(), tp, Ww.data_ptr<float>(), Wp.data_ptr<float>(), Wt.data_ptr<float>(),
                  out.data_ptr<float>(), M, (int)T, (int)H, cur_stream(ids));
}

int64_t emb_word_ws_ints(int64_t V, int64_t M) { return gk::emb_word_ws_ints(V, M); }
int64_t emb_word_part_floats(int64_t M, int64_t H) { return gk::emb_word_maxc(M) * H; }

void emb_backward(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor dx, c10::optional<at::Tensor> dWw,
                  c10::optional<at::Tensor> dWp, c10::optional<at::Tensor> dWt, at::Tensor part, at::Tensor sid,
                  at::Tensor order, at::Tensor wws, at::Tensor wpart) {
  const int64_t B = ids.size(0), T = ids.size(1), M = B * T, H = dx.size(-1);
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.dim() == 2 && ids.is_contiguous(),
              "emb: ids must be contiguous int64 [B, T]");
  TORCH_CHECK(dx.is_cuda() && dx.scalar_type() == at::kFloat && dx.numel() == M * H && dx.is_contiguous(),
              "emb: dx fp32 [B, T, H]");
  const int64_t* tp = nullptr;
  if (tt.has_value() && tt->defined()) {
    TORCH_CHECK(tt->scalar_type() == at::kLong && tt->numel() == M && tt->is_contiguous(), "emb: tt int64 [B, T]");
    tp = tt->data_ptr<int64_t>();
  }
  auto g = [&](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(1) == H &&
                    t->is_contiguous(), "emb: gradient tables must be contiguous fp32 [*, H]");
    return t->data_ptr<float>();
  };
  const int64_t P = dWp.has_value() && dWp->defined() ? dWp->size(0) : T;
  const int64_t NT = dWt.has_value() && dWt->defined() ? dWt->size(0) : 1;
  TORCH_CHECK(gk::emb_supported((int)H, (int)NT) && T <= P, "emb: unsupported shape");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= emb_part_floats(H), "emb: part too small");
  const int64_t V = dWw.has_value() && dWw->defined() ? dWw->size(0) : 0;
  if (V > 0) {
    TORCH_CHECK(sid.is_cuda() && sid.scalar_type() == at::kLong && sid.numel() == M && sid.is_contiguous() &&
                    order.is_cuda() && order.scalar_type() == at::kLong && order.numel() == M && order.is_contiguous(),
                "emb: sid / order must be the stable sort of ids (int64 [M])");
    TORCH_CHECK(wws.is_cuda() && wws.scalar_type() == at::kInt && wws.numel() >= gk::emb_word_ws_ints(V, M),
                "emb: word workspace int32 [emb_word_ws_ints(V, M)]");
    TORCH_CHECK(wpart.is_cuda() && wpart.scalar_type() == at::kFloat && wpart.numel() >= gk::emb_word_maxc(M) * H,
                "emb: word partials fp32 [emb_word_part_floats(M, H)]");
    TORCH_CHECK(V < (1ll << 31) && M < (1ll << 31), "emb: sizes must fit int32");
  }
  c10::DeviceGuard guard(ids.device());
  gk::emb_backward(ids.data_ptr<int64_t>(), tp, dx.data_ptr<float>(), g(dWw), g(dWp), g(dWt), part.data_ptr<float>(),
                   V > 0 ? sid.data_ptr<int64_t>() : nullptr, V > 0 ? order.data_ptr<int64_t>() : nullptr,
                   V > 0 ? wws.data_ptr<int>() : nullptr, V > 0 ? wpart.data_ptr<float>() : nullptr, V, M, (int)B,
                   (int)T, (int)P, (int)NT, (int)H, cur_stream(ids));
}

// fused self-attention (attn.hip)
void check_attn(const at::Tensor& t, const char* name, int64_t rows, int64_t cols) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() == rows * cols &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous 16-byte aligned bf16 GPU tensor of ", rows, " x ", cols, " elements");
}

void check_attn_f32(const at::Tensor& t, const char* name, int64_t n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n,
              name, " must be a contiguous fp32 GPU tensor of ", n, " elements");
}

void attn_fwd(at::Tensor qkv, at::Tensor out, at::Tensor lse, int64_t heads, double p, int64_t seed,
              c10::optional<at::Tensor> seed_dev) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * heads * 64, "qkv: [B, T, 3 * heads * 64]");
  const int64_t B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(gk::attn_supported((int)T, 64), "attn: T must be a multiple of 128");
  check_attn(qkv, "qkv", B * T, 3 * heads * 64);
  check_attn(out, "out", B * T, heads * 64);
  check_attn_f32(lse, "lse", B * heads * T);
  TORCH_CHECK(p >= 0.0 && p < 1.0, "attn: dropout p in [0, 1)");
  c10::DeviceGuard guard(qkv.device());
  gk::attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), (int)B, (int)T, (int)heads, (float)p,
               (uint32_t)seed, seed_word(seed_dev), cur_stream(qkv));
}

void attn_bwd(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, at::Tensor delta, at::Tensor dqkv,
              int64_t heads, double p, int64_t seed, c10::optional<at::Tensor> seed_dev) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * heads * 64, "qkv: [B, T, 3 * heads * 64]");
  const int64_t B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(gk::attn_supported((int)T, 64), "attn: T must be a multiple of 128");
  check_attn(qkv, "qkv", B * T, 3 * heads * 64);
  check_attn(dqkv, "dqkv", B * T, 3 * heads * 64);
  check_attn(out, "out", B * T, heads * 64);
  check_attn(dout, "dout", B * T, heads * 64);
  check_attn_f32(lse, "lse", B * heads * T);
  check_attn_f32(delta, "delta", B * heads * T);
  c10::DeviceGuard guard(qkv.device());
  gk::attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
               dqkv.data_ptr(), (int)B, (int)T, (int)heads, (float)p, (uint32_t)seed, seed_word(seed_dev),
               cur_stream(qkv));
}

void check_attn32(const at::Tensor& t, const char* name, int64_t rows, int64_t cols) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == rows * cols &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous 16-byte aligned fp32 GPU tensor of ", rows, " x ", cols, " elements");
}

void attn_f32_fwd(at::Tensor qkv, at::Tensor out, at::Tensor lse, int64_t heads, double p, int64_t seed,
                  c10::optional<at::Tensor> seed_dev) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * heads * 64, "qkv: [B, T, 3 * heads * 64]");
  const int64_t B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(gk::attn_f32_supported((int)T, 64), "attn_f32: T must be a multiple of 128");
  check_attn32(qkv, "qkv", B * T, 3 * heads * 64);
  check_attn32(out, "out", B * T, heads * 64);
  check_attn_f32(lse, "lse", B * heads * T);
  TORCH_CHECK(p >= 0.0 && p < 1.0, "attn: dropout p in [0, 1)");
  TORCH_CHECK(B * heads * T * (T / 2) < (int64_t(1) << 32), "attn: dropout hash index must fit 32 bits");
  c10::DeviceGuard guard(qkv.device());
  gk::attn_f32_fwd(qkv.data_ptr<float>(), out.data_ptr<float>(), lse.data_ptr<float>(), (int)B, (int)T, (int)heads,
                   (float)p, (uint32_t)seed, seed_word(seed_dev), cur_stream(qkv));
}

void attn_f32_bwd(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, at::Tensor delta, at::Tensor dqkv,
                  int64_t heads, double p, int64_t seed, c10::optional<at::Tensor> seed_dev) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * heads * 64, "qkv: [B, T, 3 * heads * 64]");
  const int64_t B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(gk::attn_f32_supported((int)T, 64), "attn_f32: T must be a multiple of 128");
  check_attn32(qkv, "qkv", B * T, 3 * heads * 64);
  check_attn32(dqkv, "dqkv", B * T, 3 * heads * 64);
  check_attn32(out, "out", B * T, heads * 64);
  check_attn32(dout, "dout", B * T, heads * 64);
  check_attn_f32(lse, "lse", B * heads * T);
  check_attn_f32(delta, "delta", B * heads * T);
  c10::DeviceGuard guard(qkv.device());
  gk::attn_f32_bwd(qkv.data_ptr<float>(), out.data_ptr<float>(), dout.data_ptr<float>(), lse.data_ptr<float>(),
                   delta.data_ptr<float>(), dqkv.data_ptr<float>(), (int)B, (int)T, (int)heads, (float)p,
                   (uint32_t)seed, seed_word(seed_dev), cur_stream(qkv));
}

void attn_dropout_mask(at::Tensor mask, int64_t B, int64_t heads, int64_t T, double p, int64_t seed,
                       c10::optional<at::Tensor> seed_dev) {
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
                  mask.numel() == B * heads * T * T, "mask: contiguous uint8 [B, heads, T, T]");
  c10::DeviceGuard guard(mask.device());
  gk::attn_dropout_mask(mask.data_ptr<uint8_t>(), (int)B, (int)heads, (int)T, (float)p, (uint32_t)seed,
                        seed_word(seed_dev), cur_stream(mask));
}

// linear-layer column passes (linear.hip): bias gradient / fused GELU backward
float* colsum_db(const c10::optional<at::Tensor>& db, int64_t N) {
  if (!db.has_value() || !db->defined()) return nullptr;
  TORCH_CHECK(db->is_cuda() && db->scalar_type() == at::kFloat && db->is_contiguous() && db->numel() == N,
              "db must be a contiguous fp32 [N] GPU tensor");
  return db->data_ptr<float>();
}

void check_col_2d(const at::Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == 2 && t.is_contiguous() && t.size(1) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous 16-byte aligned ", at::toString(dt),
              " [M, N] GPU tensor with N % 8 == 0 (bf16 or fp32, all operands alike)");
}

void colsum_acc(at::Tensor dy, at::Tensor db) {
  const bool f32 = dy.scalar_type() == at::kFloat;
  check_col_2d(dy, "dy", f32 ? at::kFloat : at::kBFloat16);
  float* d = colsum_db(db, dy.size(1));
  c10::DeviceGuard guard(dy.device());
  if (f32)
    gk::colsum_acc_f32(dy.data_ptr<float>(), d, dy.size(0), (int)dy.size(1), cur_stream(dy));
  else
    gk::colsum_acc_bf16(static_cast<const uint16_t*>(dy.data_ptr()), d, dy.size(0), (int)dy.size(1), cur_stream(dy));
}

void gelu_bwd_colsum(at::Tensor dy, at::Tensor pre, at::Tensor dpre, c10::optional<at::Tensor> db) {
  const bool f32 = dy.scalar_type() == at::kFloat;
  const auto dt = f32 ? at::kFloat : at::kBFloat16;
  check_col_2d(dy, "dy", dt);
  check_col_2d(pre, "pre", dt);
  check_col_2d(dpre, "dpre", dt);
  TORCH_CHECK(pre.sizes() == dy.sizes() && dpre.sizes() == dy.sizes(), "gelu_bwd_colsum: shape mismatch");
  float* d = colsum_db(db, dy.size(1));
  c10::DeviceGuard guard(dy.device());
  if (f32)
    gk::gelu_bwd_colsum_f32(dy.data_ptr<float>(), pre.data_ptr<float>(), dpre.data_ptr<float>(), d, dy.size(0),
                            (int)dy.size(1), cur_stream(dy));
  else
    gk::gelu_bwd_colsum_bf16(static_cast<const uint16_t*>(dy.data_ptr()), static_cast<const uint16_t*>(pre.data_ptr()),
                             static_cast<uint16_t*>(dpre.data_ptr()), d, dy.size(0), (int)dy.size(1), cur_stream(dy));
}

// LSTM cell (lstm.hip)
void check_lstm(const at::Tensor& t, at::ScalarType dt, int64_t numel, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous() && t.numel() == numel, name,
              " must be a contiguous ", at::toString(dt), " GPU tensor of ", numel, " elements");
}

// P: fp32 [S][B][N] K-slice partials of the step GEMM (N = 4Hp forward, Hp backward)
int64_t lstm_partials(const c10::optional<at::Tensor>& P, int64_t S, int64_t B, int64_t H, int64_t gates_mult,
                      const float** out) {
  *out = nullptr;
  if (!(P.has_value() && P->defined())) return 0;
  TORCH_CHECK(P->is_cuda() && P->scalar_type() == at::kFloat && P->is_contiguous() && P->dim() == 3 &&
                  P->size(0) >= S && S >= 1 && P->size(1) == B && P->size(2) % (64 * gates_mult) == 0 &&
                  P->size(2) / gates_mult >= H,
              "P must be a contiguous fp32 [>=S, B, ", gates_mult, "*Hp] tensor, Hp a multiple of 64 >= H");
  *out = P->data_ptr<float>();
  return P->size(2) / gates_mult;
}

void* lstm_pad(const c10::optional<at::Tensor>& t, int64_t rows, int64_t cols, const char* name,
               at::ScalarType dt = at::kBFloat16) {
  if (!(t.has_value() && t->defined())) return nullptr;
  check_lstm(*t, dt, rows * cols, name);
  return t->data_ptr();
}

// Split-K recurrent GEMM: P[s] = A[:, slice s] B[:, slice s]^T, A [M, K], B [N, K] (bf16, row-major)
void lstm_rec_gemm(at::Tensor A, at::Tensor Bm, at::Tensor P, int64_t S) {
  TORCH_CHECK(A.dim() == 2 && Bm.dim() == 2 && A.size(1) == Bm.size(1), "A [M, K] and B [N, K] expected");
  const int64_t M = A.size(0), K = A.size(1), N = Bm.size(0);
  TORCH_CHECK(S >= 1 && K % (64 * S) == 0 && N % 64 == 0, "lstm_rec_gemm: K % (64 S) and N % 64 must be 0");
  const bool f32 = A.scalar_type() == at::kFloat;
  const auto dt = f32 ? at::kFloat : at::kBFloat16;
  const int64_t al = f32 ? 4 : 8;   // elements per 16 bytes
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == dt && A.stride(1) == 1 && A.stride(0) % al == 0 &&
                  Bm.is_cuda() && Bm.scalar_type() == dt && Bm.stride(1) == 1 && Bm.stride(0) % al == 0,
              "lstm_rec_gemm: bf16 or fp32 GPU operands (both alike) with unit column stride and 16-byte aligned rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(Bm.data_ptr()) % 16 == 0,
              "lstm_rec_gemm: 16-byte aligned operands");
  check_lstm(P, at::kFloat, S * M * N, "P");
  c10::DeviceGuard guard(A.device());
  if (f32)
    gk::lstm_rec_gemm_f32(A.data_ptr<float>(), A.stride(0), Bm.data_ptr<float>(), Bm.stride(0), P.data_ptr<float>(),
                          (int)M, (int)N, (int)K, (int)S, cur_stream(A));
  else
    gk::lstm_rec_gemm(static_cast<const uint16_t*>(A.data_ptr()), A.stride(0),
                      static_cast<const uint16_t*>(Bm.data_ptr()), Bm.stride(0), P.data_ptr<float>(), (int)M, (int)N,
                      (int)K, (int)S, cur_stream(A));
}

// bf16x6 split-K recurrent GEMM: A fp32 [M, K]; B3 bf16 [3, N, K] = the exact
// hi / mid / lo split of an fp32 B (ops/lstm.py split3)
void lstm_rec_gemm_x6(at::Tensor A, at::Tensor B3, at::Tensor P, int64_t S) {
  TORCH_CHECK(A.dim() == 2 && B3.dim() == 3 && B3.size(0) == 3 && A.size(1) == B3.size(2),
              "lstm_rec_gemm_x6: A [M, K] fp32 and B3 [3, N, K] bf16 expected");
  const int64_t M = A.size(0), K = A.size(1), N = B3.size(1);
  TORCH_CHECK(S >= 1 && K % (64 * S) == 0 && N % 64 == 0, "lstm_rec_gemm_x6: K % (64 S) and N % 64 must be 0");
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == at::kFloat && A.stride(1) == 1 && A.stride(0) % 4 == 0 &&
                  B3.is_cuda() && B3.scalar_type() == at::kBFloat16 && B3.stride(2) == 1 && B3.stride(1) % 8 == 0 &&
                  B3.stride(0) % 8 == 0,
              "lstm_rec_gemm_x6: fp32 A / bf16 B3 GPU operands with unit column stride and 16-byte aligned rows");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B3.data_ptr()) % 16 == 0,
              "lstm_rec_gemm_x6: 16-byte aligned operands");
  check_lstm(P, at::kFloat, S * M * N, "P");
  c10::DeviceGuard guard(A.device());
  gk::lstm_rec_gemm_x6(A.data_ptr<float>(), A.stride(0), static_cast<const uint16_t*>(B3.data_ptr()), B3.stride(1),
                       B3.stride(0), P.data_ptr<float>(), (int)M, (int)N, (int)K, (int)S, cur_stream(A));
}

void lstm_cell_fwd(at::Tensor xg, c10::optional<at::Tensor> hg, c10::optional<at::Tensor> P, int64_t S, at::Tensor c_prev, at::Tensor c,
                   at::Tensor h, c10::optional<at::Tensor> h_pad, at::Tensor gates) {
  TORCH_CHECK(xg.dim() == 2 && xg.size(1) % 4 == 0, "xg must be [B, 4H]");
  const int64_t B = xg.size(0), H = xg.size(1) / 4;
  const bool f32 = xg.scalar_type() == at::kFloat;
  const auto dt = f32 ? at::kFloat : at::kBFloat16;   // xg / hg / h / h_pad storage (bf16 or fp32 alike)
  check_lstm(xg, dt, B * 4 * H, "xg");
  check_lstm(c_prev, at::kFloat, B * H, "c_prev");
  check_lstm(c, at::kFloat, B * H, "c");
  check_lstm(h, dt, B * H, "h");
  check_lstm(gates, at::kFloat, B * 4 * H, "gates");
  const float* pp = nullptr;
  int64_t Hp = lstm_partials(P, S, B, H, 4, &pp);
  if (!pp) S = 0, Hp = (H + 63) / 64 * 64;
  void* hp = lstm_pad(h_pad, B, Hp, "h_pad", dt);
  const void* ph = lstm_pad(hg, B, 4 * H, "hg", dt);
  c10::DeviceGuard guard(xg.device());
  if (f32)
    gk::lstm_cell_fwd_f32(xg.data_ptr<float>(), static_cast<const float*>(ph), pp, (int)S, c_prev.data_ptr<float>(),
                          c.data_ptr<float>(), h.data_ptr<float>(), static_cast<float*>(hp), gates.data_ptr<float>(),
                          (int)B, (int)H, (int)Hp, cur_stream(xg));
  else
    gk::lstm_cell_fwd(static_cast<const uint16_t*>(xg.data_ptr()), static_cast<const uint16_t*>(ph), pp, (int)S,
                      c_prev.data_ptr<float>(), c.data_ptr<float>(), static_cast<uint16_t*>(h.data_ptr()),
                      static_cast<uint16_t*>(hp), gates.data_ptr<float>(), (int)B, (int)H, (int)Hp, cur_stream(xg));
}

void lstm_cell_bwd(c10::optional<at::Tensor> dout, c10::optional<at::Tensor> dh_rec, c10::optional<at::Tensor> P,
                   int64_t S,
                   c10::optional<at::Tensor> dc_next, at::Tensor gates, at::Tensor c, at::Tensor c_prev, at::Tensor dG,
                   c10::optional<at::Tensor> dG_pad, at::Tensor dc_prev) {
  TORCH_CHECK(gates.dim() == 2 && gates.size(1) % 4 == 0, "gates must be [B, 4H]");
  const int64_t B = gates.size(0), H = gates.size(1) / 4;
  const bool f32 = dG.scalar_type() == at::kFloat;
  const auto dt = f32 ? at::kFloat : at::kBFloat16;   // dout / dh_rec / dG / dG_pad storage
  check_lstm(gates, at::kFloat, B * 4 * H, "gates");
  check_lstm(c, at::kFloat, B * H, "c");
  check_lstm(c_prev, at::kFloat, B * H, "c_prev");
  check_lstm(dG, dt, B * 4 * H, "dG");
  check_lstm(dc_prev, at::kFloat, B * H, "dc_prev");
  const void* po = nullptr;
  const float* pc = nullptr;
  if (dout.has_value() && dout->defined()) {
    check_lstm(*dout, dt, B * H, "dout");
    po = dout->data_ptr();
  }
  if (dc_next.has_value() && dc_next->defined()) {
    check_lstm(*dc_next, at::kFloat, B * H, "dc_next");
    pc = dc_next->data_ptr<float>();
  }
  const float* pp = nullptr;
  int64_t Hp = lstm_partials(P, S, B, H, 1, &pp);
  if (!pp) S = 0, Hp = (H + 63) / 64 * 64;
  void* gp = lstm_pad(dG_pad, B, 4 * Hp, "dG_pad", dt);
  const void* pr = lstm_pad(dh_rec, B, H, "dh_rec", dt);
  c10::DeviceGuard guard(gates.device());
  if (f32)
    gk::lstm_cell_bwd_f32(static_cast<const float*>(po), static_cast<const float*>(pr), pp, (int)S, pc,
                          gates.data_ptr<float>(), c.data_ptr<float>(), c_prev.data_ptr<float>(), dG.data_ptr<float>(),
                          static_cast<float*>(gp), dc_prev.data_ptr<float>(), (int)B, (int)H, (int)Hp, cur_stream(gates));
  else
    gk::lstm_cell_bwd(static_cast<const uint16_t*>(po), static_cast<const uint16_t*>(pr), pp, (int)S, pc,
                      gates.data_ptr<float>(), c.data_ptr<float>(), c_prev.data_ptr<float>(),
                      static_cast<uint16_t*>(dG.data_ptr()), static_cast<uint16_t*>(gp), dc_prev.data_ptr<float>(),
                      (int)B, (int)H, (int)Hp, cur_stream(gates));
}

}  // namespace


TORCH_LIBRARY(gksgd, m) {
  m.def("ctrl_bytes() -> int", &ctrl_bytes);
  m.def("workspace_bytes() -> int", &workspace_bytes);
  m.def(
      "compress(Tensor(a!) g, Tensor(b!) r, Tensor(c!) ctrl, Tensor(d!) ws, Tensor(e!) record, int mode, bool ec, "
      "bool zero_g, int loops, float z, float fixed_thr, float sample_p, int k, int k_cap, int seed, "
      "int n_stats, Tensor(f!)? stats_out=None, Tensor? valid=None, Tensor(g!)? u=None, Tensor? w=None, "
      "Tensor? chunks=None, int chunk_begin=0, int chunk_count=0, int chunk_base=0, float[] mc_mu=[], "
      "float[] mc_wd=[], Tensor? seed_dev=None, int handoff=-1) -> ()");
  m.def("apply_records_sgd(Tensor(a!) w, Tensor(b!)? w_bf16, Tensor records, int P, int k_cap, float scale, float lr, "
        "Tensor? lr_mult=None) -> ()");
  m.def("arena_digest(Tensor x, Tensor(a!) out, Tensor(b!) ws) -> ()");
  m.def("tensor_stats(Tensor x, Tensor(a!) ctrl, Tensor(b!) ws) -> ()");
  m.def("scatter_add_records(Tensor(a!) dst, Tensor records, int P, int k_cap, float scale, bool deterministic) -> ()");
  m.def("fill_zero(Tensor(a!) dst) -> ()");
  m.def("sign_bucket_workspace_bytes() -> int", &sign_bucket_workspace_bytes);
  m.def("sign_bucket_compress(Tensor(a!) x, Tensor(b!) mask, Tensor(c!) means, Tensor(d!) ws) -> ()");
  m.def("sign_bucket_decompress(Tensor(a!) x, Tensor mask, Tensor means) -> ()");
  m.def(
      "fused_sgd(Tensor(a!) w, Tensor(b!)? m, Tensor(c!) g, Tensor chunks, float[] lr, float[] momentum, "
      "float[] dampening, float[] weight_decay, int[] nesterov, int[] first_step, bool zero_grad, "
      "Tensor? grad_scale=None, Tensor(d!)? w_bf16=None, Tensor? lr_mult=None) -> ()");
  m.def("segmented_sumsq(Tensor w, Tensor g, Tensor chunks, Tensor(a!) out) -> ()");
  m.def(
      "fused_lars(Tensor(a!) w, Tensor(b!) m, Tensor g, Tensor chunks, Tensor seg_sumsq, float[] lr, "
      "float[] momentum, float[] weight_decay, float[] eeta, float[] epsilon) -> ()");
  m.def("clip_grad_norm(Tensor(a!) g, float max_norm, Tensor(b!) ws, Tensor(c!) coef, Tensor(d!) norm) -> ()");

  m.def("bn_workspace_floats(int M, int C, int elem_bytes) -> int", &bn_workspace_floats);
  m.def("bn_supported(int C, int elem_bytes) -> bool", &bn_supported);
  m.def("bn_set_blocks(int blocks) -> ()", [](int64_t b) { gk::bn_set_blocks((int)b); });
  m.def("bn_mask_bytes(int M, int C, int elem_bytes) -> int", &bn_mask_bytes);
  m.def(
      "bn_act_forward(Tensor x, Tensor? res, Tensor(a!) y, Tensor(i!)? mask, Tensor? w, Tensor? b, Tensor(b!)? run_mean, "
      "Tensor(c!)? run_var, Tensor(d!) save_mean, Tensor(e!) save_invstd, Tensor(f!) scale, Tensor(g!) shift, "
      "Tensor(h!) ws, float eps, float momentum, bool relu, Tensor(j!)? nbt=None, Tensor? pre=None, "
      "int pre_rows=0, Tensor(k!)? fin=None, Tensor? rscale=None, Tensor? rshift=None) -> ()");
  m.def(
      "bn_act_finalize(Tensor x, Tensor? w, Tensor? b, Tensor(a!)? run_mean, Tensor(b!)? run_var, "
      "Tensor(c!) save_mean, Tensor(d!) save_invstd, Tensor(e!) scale, Tensor(f!) shift, Tensor(g!) ws, float eps, "
      "float momentum, Tensor(h!)? nbt=None, Tensor? pre=None, int pre_rows=0) -> ()");
  m.def(
      "bn_relu_pool_forward(Tensor x, Tensor(a!) y, Tensor(b!) amax, Tensor? w, Tensor? b, Tensor(c!)? run_mean, "
      "Tensor(d!)? run_var, Tensor(e!) save_mean, Tensor(f!) save_invstd, Tensor(g!) scale, Tensor(h!) shift, "
      "Tensor(i!) ws, float eps, float momentum, int k, int s, int p, Tensor(j!)? nbt=None, Tensor? pre=None, "
      "int pre_rows=0) -> ()");
  m.def(
      "bn_relu_pool_backward(Tensor dy, Tensor amax, Tensor x, Tensor(a!) dx, Tensor? w, Tensor mean, "
      "Tensor invstd, Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor(d!) ws, int k, int s, int p, "
      "Tensor(e!)? gw_acc=None, Tensor(f!)? gb_acc=None, Tensor? dy2=None) -> ()");
  m.def(
      "bn_act_backward(Tensor dy, Tensor? mask, Tensor x, Tensor(a!) dx, Tensor(b!)? dres, Tensor? w, Tensor mean, "
      "Tensor invstd, Tensor(c!) dgamma, Tensor(d!) dbeta, Tensor(e!) ws, bool relu, Tensor(f!)? gw_acc=None, "
      "Tensor(g!)? gb_acc=None, Tensor? dy2=None, Tensor(h!)? fin=None) -> ()");
  m.def("accum_grad(Tensor(a!) dst, Tensor src) -> ()");
  m.def(
      "momentum_correct(Tensor(a!) u, Tensor(b!) g, Tensor w, Tensor chunks, int begin, int count, "
      "float[] momentum, float[] weight_decay) -> ()");
  m.def("mask_records(Tensor(a!) u, Tensor record, int k_cap) -> ()");
  m.def("cast_bf16(Tensor(a!) dst, Tensor src) -> ()");
  m.def("gemm_supported(int N, int K) -> bool", &gemm_supported);
  m.def("gemm_nt(Tensor A, Tensor B, Tensor(a!) C, int cfg=0, int max_blocks=0, Tensor(b!)? stats=None, "
        "Tensor? bias=None, Tensor? bn_h=None, Tensor? bn_dy2=None, Tensor? bn_mask=None, Tensor? lz_x=None, Tensor? lz_coef=None, Tensor? lz_padz=None, Tensor? lz_padx=None) -> int");
  m.def("gemm_tn_acc(Tensor G, Tensor X, Tensor(a!) W, int cfg=0, int splits=0, Tensor? lz_x=None, Tensor? lz_coef=None, Tensor? lz_padz=None, Tensor? lz_padx=None) -> ()");
  m.def("conv_nt(Tensor x, Tensor w, Tensor(a!) y, Tensor zero, int stride, int pad, int cfg=0, int max_blocks=0, "
        "Tensor(b!)? stats=None, Tensor? bias=None, Tensor? bn_h=None, Tensor? bn_dy2=None, Tensor? bn_mask=None, "
        "Tensor? lz_x=None, Tensor? lz_coef=None, Tensor? lz_padz=None, Tensor? lz_padx=None) -> int");
  m.def("stem_supported(int H, int W) -> bool", [](int64_t H, int64_t W) { return gk::stem_supported((int)H, (int)W); });
  m.def("stem_wgrad_ws(int N, int H, int W) -> int", &stem_wgrad_ws);
  m.def("stem_pack(Tensor w, Tensor(a!) wp) -> ()");
  m.def("stem_fwd(Tensor x, Tensor wp, Tensor(a!) y, Tensor(b!)? stats=None) -> int");
  m.def("stem_wgrad(Tensor x, Tensor dy, Tensor(a!) out, Tensor(b!) part) -> ()");
  m.def("stem_f32_supported(int H, int W) -> bool", [](int64_t H, int64_t W) { return gk::stem_f32_supported((int)H, (int)W); });
  m.def("stem_f32_fwd(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!)? stats=None) -> int");
  m.def("stem_f32x6_wplanes() -> int", &stem_f32x6_wplanes);
  m.def("stem_f32x6_fwd(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!)? stats, Tensor(c!) wp3) -> int");
  m.def("stem_f32_wgrad_ws(int N) -> int", &stem_f32_wgrad_ws);
  m.def("stem_f32_wgrad(Tensor x, Tensor dy, Tensor(a!) out, Tensor(b!) part, bool x6=False) -> ()");
  m.def("wgrad3_supported(int H, int W, int C, int K) -> bool", [](int64_t H, int64_t W, int64_t C, int64_t K) {
    return gk::wgrad3_supported((int)H, (int)W, (int)C, (int)K);
  });
  m.def("wgrad3_ws(int N, int H, int W, int C, int K) -> int", &wgrad3_ws);
  m.def("conv3_wgrad(Tensor dy, Tensor x, Tensor(a!) out, Tensor(b!) part, Tensor zero) -> ()");
  m.def("wino_weights(Tensor w, Tensor(a!) u, bool flip) -> ()");
  m.def("weight_prep(Tensor table, int ndesc, int total_blocks) -> ()");
  m.def("weight_prep_blocks(int kind, int R, int S) -> int", &weight_prep_blocks);
  m.def("wino_wgrad_ws(int N, int H, int W, int C, int K, int splits=0) -> int", &wino_wgrad_ws);
  m.def("wino_wgrad(Tensor x, Tensor dy, Tensor(a!) out, Tensor(b!) part, int splits=0) -> ()");
  m.def("wino_conv(Tensor x, Tensor u, Tensor(a!) y, int max_blocks=0, Tensor(b!)? stats=None, Tensor? bn_h=None, "
        "Tensor? bn_dy2=None, Tensor? bn_mask=None, int splits=1) -> int");
  m.def("wino_x6_weights(Tensor w, Tensor(a!) u3, bool flip) -> ()");
  m.def("wino_x6_conv(Tensor x, Tensor u3, Tensor(a!) y, int max_blocks=0, Tensor(b!)? stats=None, "
        "Tensor? bn_h=None, Tensor? bn_dy2=None, Tensor? bn_mask=None) -> int");
  m.def("conv_dgrad_s2(Tensor dy, Tensor w, Tensor(a!) dx, Tensor zero, int cfg=0, int max_blocks=0, "
        "Tensor? lz_x=None, Tensor? lz_coef=None, Tensor? lz_padz=None, Tensor? lz_padx=None) -> ()");
  m.def("bn_bwd_lazy_pre(Tensor x, Tensor part, int rows, Tensor? w, Tensor mean, Tensor invstd, "
        "Tensor(a!) dgamma, Tensor(b!) dbeta, Tensor(c!) coef, Tensor(d!) padz, Tensor(e!) padx, "
        "Tensor(f!)? gw_acc=None, Tensor(g!)? gb_acc=None) -> ()");
  m.def("bn_act_backward_lazy(Tensor dy, Tensor? dy2, Tensor? mask, Tensor x, Tensor(a!) dz, Tensor? w, "
        "Tensor mean, Tensor invstd, Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor(d!) ws, bool relu, "
        "Tensor(e!) coef, Tensor(f!) padz, Tensor(g!) padx, Tensor(h!)? gw_acc=None, Tensor(i!)? gb_acc=None) -> ()");
  m.def("bn_lazy_apply(Tensor dz, Tensor x, Tensor(a!) dx, Tensor coef) -> ()");
  m.def("bn_stats_partials(Tensor x, Tensor(a!) ws) -> ()");
  m.def(
      "bn_act_backward_pre_dual(Tensor dz, Tensor x, Tensor(a!) dx, Tensor? w, Tensor mean, Tensor invstd, "
      "Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor part, int rows, Tensor(d!)? gw_acc, Tensor(e!)? gb_acc, Tensor x2, "
      "Tensor(f!) dx2, Tensor? w2, Tensor mean2, Tensor invstd2, Tensor(g!) dgamma2, Tensor(h!) dbeta2, "
      "Tensor(i!) ws2, Tensor(j!)? gw2_acc, Tensor(k!)? gb2_acc) -> ()");
  m.def("bn_act_backward_pre(Tensor dz, Tensor x, Tensor(a!) dx, Tensor? w, Tensor mean, Tensor invstd, "
        "Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor part, int rows, Tensor(d!)? gw_acc=None, "
        "Tensor(e!)? gb_acc=None, Tensor(f!)? fin=None) -> ()");
  m.def("bn_fin_state_bytes(int C) -> int", &bn_fin_state_bytes);
  m.def("attn_supported(int T, int D) -> bool",
        [](int64_t T, int64_t D) { return gk::attn_supported((int)T, (int)D); });
  m.def("attn_fwd(Tensor qkv, Tensor(a!) out, Tensor(b!) lse, int heads, float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("attn_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, Tensor(a!) delta, Tensor(b!) dqkv, int heads, "
        "float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("attn_dropout_mask(Tensor(a!) mask, int B, int heads, int T, float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("attn_f32_fwd(Tensor qkv, Tensor(a!) out, Tensor(b!) lse, int heads, float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("attn_f32_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, Tensor(a!) delta, Tensor(b!) dqkv, int heads, "
        "float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("attn_f32_supported(int T, int D) -> bool",
        [](int64_t T, int64_t D) { return gk::attn_f32_supported((int)T, (int)D); });
  m.def("add_ln_supported(int H) -> bool", &add_ln_supported);
  m.def("add_ln_ws_floats(int R, int H) -> int", &add_ln_ws_floats);
  m.def("xent_supported(int V) -> bool", &xent_supported);
  m.def("xent_forward(Tensor logits, Tensor labels, Tensor(a!) lse, Tensor(b!) loss, int ignore) -> ()");
  m.def("xent_backward(Tensor logits, Tensor labels, Tensor lse, Tensor scale, Tensor(a!) grad, int ignore) -> ()");
  m.def("emb_supported(int H, int NT) -> bool", &emb_supported);
  m.def("emb_part_floats(int H) -> int", &emb_part_floats);
  m.def("emb_forward(Tensor ids, Tensor? tt, Tensor Ww, Tensor Wp, Tensor Wt, Tensor(a!) out) -> ()");
  m.def("emb_word_ws_ints(int V, int M) -> int", &emb_word_ws_ints);
  m.def("emb_word_part_floats(int M, int H) -> int", &emb_word_part_floats);
  m.def("emb_backward(Tensor ids, Tensor? tt, Tensor dx, Tensor(a!)? dWw, Tensor(b!)? dWp, Tensor(c!)? dWt, "
        "Tensor(d!) part, Tensor sid, Tensor order, Tensor(e!) wws, Tensor(f!) wpart) -> ()");
  m.def("add_ln_forward(Tensor a, Tensor x, Tensor? gamma, Tensor? beta, Tensor(a!) y, Tensor(b!) h, "
        "Tensor(c!) mean, Tensor(d!) rstd, float eps, float p, int seed, Tensor? seed_dev=None) -> ()");
  m.def("add_ln_backward(Tensor dy, Tensor h, Tensor mean, Tensor rstd, Tensor? gamma, Tensor(a!) dx, "
        "Tensor(b!)? da, Tensor(c!)? dgamma, Tensor(d!)? dbeta, bool accumulate, Tensor(e!) ws, float p, int seed, "
        "Tensor? seed_dev=None) -> ()");
  m.def("conv_tn_acc(Tensor dy, Tensor x, Tensor(a!) wout, Tensor zero, int stride, int pad, int cfg=0, int splits=0, "
        "Tensor? lz_x=None, Tensor? lz_coef=None, Tensor? lz_padz=None, Tensor? lz_padx=None) -> ()");
  m.def("colsum_acc(Tensor dy, Tensor(a!) db) -> ()");
  m.def("gelu_bwd_colsum(Tensor dy, Tensor pre, Tensor(a!) dpre, Tensor(b!)? db=None) -> ()");
  m.def("lstm_rec_gemm(Tensor A, Tensor B, Tensor(a!) P, int S) -> ()");
  m.def("lstm_rec_gemm_x6(Tensor A, Tensor B3, Tensor(a!) P, int S) -> ()");
  m.def("lstm_cell_fwd(Tensor xg, Tensor? hg, Tensor? P, int S, Tensor c_prev, Tensor(a!) c, Tensor(b!) h, Tensor(c!)? h_pad, "
        "Tensor(d!) gates) -> ()");
  m.def("lstm_cell_bwd(Tensor? dout, Tensor? dh_rec, Tensor? P, int S, Tensor? dc_next, Tensor gates, Tensor c, Tensor c_prev, "
        "Tensor(a!) dG, Tensor(b!)? dG_pad, Tensor(c!) dc_prev) -> ()");

  m.class_<RcclEngine>("RcclEngine")
      .def(torch::init<>())
      .def_static("unique_id", &RcclEngine::unique_id)
      .def("init", &RcclEngine::init)
      .def("init_async", &RcclEngine::init_async)
      .def("init_poll", &RcclEngine::init_poll)
      .def("init_wait", &RcclEngine::init_wait)
      .def("abort", &RcclEngine::abort)
      .def("set_op_timeout", &RcclEngine::set_op_timeout)
      .def("allgather", &RcclEngine::allgather)
      .def("allreduce", &RcclEngine::allreduce)
      .def("broadcast", &RcclEngine::broadcast)
      .def("allgather_many", &RcclEngine::allgather_many)
      .def("set_tracking", &RcclEngine::set_tracking)
      .def("start_watchdog", &RcclEngine::start_watchdog)
      .def("stop_watchdog", &RcclEngine::stop_watchdog)
      .def("poll", &RcclEngine::poll)
      .def("failed", &RcclEngine::failed)
      .def("error", &RcclEngine::error)
      .def("check", &RcclEngine::check)
      .def("in_flight", &RcclEngine::in_flight)
      .def("reset_stats", &RcclEngine::reset_stats)
      .def("stats", &RcclEngine::stats)
      .def("inject_failure", &RcclEngine::inject_failure)
      .def("destroy", &RcclEngine::destroy)
      .def("rank", &RcclEngine::rank)
      .def("world", &RcclEngine::world);
}

TORCH_LIBRARY_IMPL(gksgd, CUDA, m) {
  m.impl("compress", &compress);
  m.impl("tensor_stats", &tensor_stats);
  m.impl("scatter_add_records", &scatter_add_records);
  m.impl("apply_records_sgd", &apply_records_sgd);
  m.impl("arena_digest", &arena_digest);
  m.impl("fill_zero", &fill_zero);
  m.impl("sign_bucket_compress", &sign_bucket_compress);
  m.impl("sign_bucket_decompress", &sign_bucket_decompress);
  m.impl("fused_sgd", &fused_sgd);
  m.impl("segmented_sumsq", &segmented_sumsq);
  m.impl("fused_lars", &fused_lars);
  m.impl("clip_grad_norm", &clip_grad_norm);
  m.impl("bn_act_forward", &bn_act_forward);
  m.impl("bn_act_finalize", &bn_act_finalize);
  m.impl("bn_act_backward", &bn_act_backward);
  m.impl("bn_act_backward_pre", &bn_act_backward_pre);
  m.impl("bn_act_backward_pre_dual", &bn_act_backward_pre_dual);
  m.impl("bn_bwd_lazy_pre", &bn_bwd_lazy_pre);
  m.impl("bn_act_backward_lazy", &bn_act_backward_lazy);
  m.impl("bn_lazy_apply", &bn_lazy_apply);
  m.impl("bn_stats_partials", &bn_stats_partials);
  m.impl("stem_pack", &stem_pack);
  m.impl("conv_dgrad_s2", &conv_dgrad_s2);
  m.impl("conv3_wgrad", &conv3_wgrad);
  m.impl("stem_fwd", &stem_fwd);
  m.impl("stem_wgrad", &stem_wgrad);
  m.impl("stem_f32_fwd", &stem_f32_fwd);
  m.impl("stem_f32x6_fwd", &stem_f32x6_fwd);
  m.impl("stem_f32_wgrad", &stem_f32_wgrad);
  m.impl("bn_relu_pool_forward", &bn_relu_pool_forward);
  m.impl("bn_relu_pool_backward", &bn_relu_pool_backward);
  m.impl("accum_grad", &accum_grad);
  m.impl("momentum_correct", &momentum_correct);
  m.impl("mask_records", &mask_records);
  m.impl("cast_bf16", &cast_bf16);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("gemm_tn_acc", &gemm_tn_acc);
  m.impl("conv_nt", &conv_nt);
  m.impl("wino_weights", &wino_weights);
  m.impl("weight_prep", &weight_prep);
  m.impl("wino_conv", &wino_conv);
  m.impl("wino_x6_weights", &wino_x6_weights);
  m.impl("wino_x6_conv", &wino_x6_conv);
  m.impl("wino_wgrad", &wino_wgrad);
  m.impl("conv_tn_acc", &conv_tn_acc);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("attn_dropout_mask", &attn_dropout_mask);
  m.impl("attn_f32_fwd", &attn_f32_fwd);
  m.impl("attn_f32_bwd", &attn_f32_bwd);
  m.impl("add_ln_forward", &add_ln_forward);
  m.impl("xent_forward", &xent_forward);
  m.impl("xent_backward", &xent_backward);
  m.impl("emb_forward", &emb_forward);
  m.impl("emb_backward", &emb_backward);
  m.impl("add_ln_backward", &add_ln_backward);
  m.impl("colsum_acc", &colsum_acc);
  m.impl("gelu_bwd_colsum", &gelu_bwd_colsum);
  m.impl("lstm_rec_gemm", &lstm_rec_gemm);
  m.impl("lstm_rec_gemm_x6", &lstm_rec_gemm_x6);
  m.impl("lstm_cell_fwd", &lstm_cell_fwd);
  m.impl("lstm_cell_bwd", &lstm_cell_bwd);
}
