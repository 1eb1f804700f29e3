// torch <-> native bindings for pytorch_distributed_rnn_amd._C
//
// Thin host glue: validates tensors, allocates outputs/workspaces through the
// torch caching allocator, fills the POD argument structs of pdrnn/api.h and
// launches on torch's current HIP stream.  All math lives in csrc/kernels.
#include <torch/extension.h>
#include <cstdio>
#include <atomic>
#include <map>
#include <mutex>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include "pdrnn/api.h"
#include "pdrnn/runtime.h"

namespace {

using at::Tensor;

// PDRNN_LSTM_STAMPS=1: per-workgroup cycle stamps around the recurrence loop,
// summarised on stderr (diagnostic builds of the timing, never in benchmarks).
bool stamps_enabled() {
  static const bool on = std::getenv("PDRNN_LSTM_STAMPS") != nullptr;
  return on;
}
// PDRNN_SW=0: the fused motion step runs the gate-split / K-split kernel family
// instead of the sequence-in-wave kernels (A/B); PDRNN_SW=2 keeps the
// sequence-in-wave kernels but launches the latency regime's forward and
// BPTT separately (no one-launch step); read per call
bool sw_enabled() {
  const char* e = std::getenv("PDRNN_SW");
  return !(e && e[0] == '0');
}
bool sw_one_launch_enabled() {
  const char* e = std::getenv("PDRNN_SW");
  return !(e && (e[0] == '0' || e[0] == '2'));
}
void report_stamps(const char* what, const Tensor& st, int iters) {
  // [grid, 8]: loop start / end shader cycles, loop start / end real time,
  // workgroup entry / exit real time (100 MHz; entry/exit 0 when not stamped)
  auto h = st.cpu();
  const int64_t g = h.size(0);
  auto p = h.data_ptr<int64_t>();
  double cyc = 0, real = 0, pro = 0, epi = 0;
  int64_t in_min = INT64_MAX, in_max = 0, out_min = INT64_MAX, out_max = 0;
  for (int64_t i = 0; i < g; ++i) {
    const int64_t* r = p + i * 8;
    cyc += (double)(r[1] - r[0]);
    real += (double)(r[3] - r[2]);
    if (r[4] && r[5]) {
      pro += (double)(r[2] - r[4]);
      epi += (double)(r[5] - r[3]);
      in_min = std::min(in_min, r[4]); in_max = std::max(in_max, r[4]);
      out_min = std::min(out_min, r[5]); out_max = std::max(out_max, r[5]);
    }
  }
  cyc /= g; real /= g; pro /= g; epi /= g;
  const double us = real / 100.0;  // s_memrealtime ticks at 100 MHz
  fprintf(stderr, "[stamps] %s grid=%lld iters=%d loop=%.1f us cycles=%.0f clock=%.2f GHz cyc/iter=%.0f", what,
          (long long)g, iters, us, cyc, cyc / (us * 1e3), cyc / iters);
  if (in_max) {
    fprintf(stderr, " | prologue=%.1f us epilogue=%.1f us entry spread=%.1f us exit spread=%.1f us span=%.1f us",
            pro / 100.0, epi / 100.0, (in_max - in_min) / 100.0, (out_max - out_min) / 100.0,
            (out_max - in_min) / 100.0);
    std::map<int64_t, int> per_cu;  // placement census: workgroups per CU
    for (int64_t i = 0; i < g; ++i) per_cu[p[i * 8 + 6] & 0xFFFFFF]++;
    int lo = INT32_MAX, hi = 0;
    for (auto& kv : per_cu) { lo = std::min(lo, kv.second); hi = std::max(hi, kv.second); }
    fprintf(stderr, " | CUs used=%zu workgroups/CU min=%d max=%d", per_cu.size(), lo, hi);
    // loop time by the load of the workgroup's CU (mean / max us): is the
    // exit spread placement (more co-resident waves) or something else
    std::map<int, std::pair<double, double>> by_load;
    std::map<int, int> n_load;
    for (int64_t i = 0; i < g; ++i) {
      const int64_t* r = p + i * 8;
      const int k = per_cu[r[6] & 0xFFFFFF];
      const double t = (double)(r[3] - r[2]) / 100.0;
      auto& e = by_load[k];
      e.first += t; e.second = std::max(e.second, t); n_load[k]++;
    }
    for (auto& kv : by_load)
      fprintf(stderr, " | %d/CU: n=%d loop mean=%.1f max=%.1f", kv.first, n_load[kv.first],
              kv.second.first / n_load[kv.first], kv.second.second);
    // waves per SIMD (wave 0 always, wave 1 where stamped): loop time by the
    // busiest SIMD the workgroup's waves sit on, and by XCC
    std::map<int64_t, int> per_simd;
    for (int64_t i = 0; i < g; ++i) {
      const int64_t* r = p + i * 8;
      per_simd[r[6] & 0xFFFFFFFF]++;
      if (r[7] >> 32) per_simd[r[7] & 0xFFFFFFFF]++;
    }
    std::map<int, std::pair<double, double>> by_simd, by_xcc;
    std::map<int, int> n_simd, n_xcc;
    for (int64_t i = 0; i < g; ++i) {
      const int64_t* r = p + i * 8;
      int k = per_simd[r[6] & 0xFFFFFFFF];
      if (r[7] >> 32) k = std::max(k, per_simd[r[7] & 0xFFFFFFFF]);
      const int x = (int)((r[6] >> 16) & 0xF);
      const double t = (double)(r[3] - r[2]) / 100.0;
      auto& e = by_simd[k]; e.first += t; e.second = std::max(e.second, t); n_simd[k]++;
      auto& f = by_xcc[x]; f.first += t; f.second = std::max(f.second, t); n_xcc[x]++;
    }
    fprintf(stderr, "\n[stamps]   by busiest SIMD:");
    for (auto& kv : by_simd)
      fprintf(stderr, " %d waves: n=%d mean=%.1f max=%.1f |", kv.first, n_simd[kv.first],
              kv.second.first / n_simd[kv.first], kv.second.second);
    {  // are a workgroup's two waves on one SIMD (they then serialise the step)?
      double ts[2] = {0, 0}, tm[2] = {0, 0};
      int tn[2] = {0, 0};
      for (int64_t i = 0; i < g; ++i) {
        const int64_t* r = p + i * 8;
        if (!(r[7] >> 32)) continue;
        const int same = (r[6] & 0xFFFFFFFF) == (r[7] & 0xFFFFFFFF);
        const double t = (double)(r[3] - r[2]) / 100.0;
        ts[same] += t; tm[same] = std::max(tm[same], t); tn[same]++;
      }
      if (tn[0] + tn[1])
        fprintf(stderr, "\n[stamps]   waves on distinct SIMDs: n=%d mean=%.1f max=%.1f | same SIMD: n=%d mean=%.1f max=%.1f",
                tn[0], tn[0] ? ts[0] / tn[0] : 0., tm[0], tn[1], tn[1] ? ts[1] / tn[1] : 0., tm[1]);
    }
    {  // by launch order (blockIdx deciles): dispatch-age effects
      double ds[10] = {0}, dm[10] = {0};
      int dn[10] = {0};
      for (int64_t i = 0; i < g; ++i) {
        const int64_t* r = p + i * 8;
        const int d = (int)(i * 10 / g);
        const double t = (double)(r[3] - r[2]) / 100.0;
        ds[d] += t; dm[d] = std::max(dm[d], t); dn[d]++;
      }
      fprintf(stderr, "\n[stamps]   by blockIdx decile (mean/max):");
      for (int d = 0; d < 10; ++d)
        if (dn[d]) fprintf(stderr, " %.1f/%.1f", ds[d] / dn[d], dm[d]);
    }
    fprintf(stderr, "\n[stamps]   by XCC:");
    for (auto& kv : by_xcc)
      fprintf(stderr, " %d: mean=%.1f max=%.1f |", kv.first, kv.second.first / n_xcc[kv.first], kv.second.second);
  }
  fprintf(stderr, "\n");
}
// progress-ordered wave priority in the small-H recurrences (PDRNN_TUNE prio=0 off):
// B = 1440: 0.403 -> 0.387 ms/step (profiles/r3p_prio.md); rotation every 2^3 step pairs
int prio_env() {
  const int mode = pdrnn_tune_int("prio", 2);
  const int sh = 3;
  static int cus = 0;  // one GPU model per process
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return mode | (sh << 4) | (cus << 8);
}
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_HIP_TENSOR(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define HIP_LAUNCH_CHECK(expr)                                                               \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    TORCH_CHECK(_e == hipSuccess, "HIP launch failed: ", hipGetErrorString(_e), " @ " #expr); \
  } while (0)

const float* opt_ptr(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

int dtype_code(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, "16-bit (bf16/fp16) tensor expected");
  return t.scalar_type() == at::kBFloat16 ? 0 : 1;
}
// large-H LSTM storage: 0 bf16, 1 fp16, 2 fp32
int large_dtype(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 2;
  return dtype_code(t);
}
// element `off` of t, as an untyped pointer (large-H kernels take void* storage)
const void* eptr(const Tensor& t, int64_t off = 0) {
  return static_cast<const char*>(t.data_ptr()) + off * (int64_t)t.element_size();
}
void* eptrm(const Tensor& t, int64_t off = 0) { return static_cast<char*>(t.data_ptr()) + off * (int64_t)t.element_size(); }
const uint16_t* u16(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* u16m(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const uint16_t* opt_u16(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<const uint16_t*>(t->data_ptr()) : nullptr;
}

// Parameter layout of one fused LSTM stack, in nn.LSTM parameter order:
// per layer weight_ih, weight_hh, bias_ih, bias_hh (biases optional).
struct StackLayout {
  int64_t P = 0;
  int64_t off_wih[PDRNN_MAX_LAYERS], off_whh[PDRNN_MAX_LAYERS];
  int64_t off_bih[PDRNN_MAX_LAYERS], off_bhh[PDRNN_MAX_LAYERS];
};

StackLayout stack_layout(const std::vector<Tensor>& w, int64_t NL, bool has_bias) {
  StackLayout L;
  int64_t off = 0;
  for (int64_t l = 0; l < NL; ++l) {
    L.off_wih[l] = off; off += w[l * 4 + 0].numel();
    L.off_whh[l] = off; off += w[l * 4 + 1].numel();
    if (has_bias) {
      L.off_bih[l] = off; off += w[l * 4 + 2].numel();
      L.off_bhh[l] = off; off += w[l * 4 + 3].numel();
    } else {
      L.off_bih[l] = L.off_bhh[l] = -1;
    }
  }
  L.P = off;
  return L;
}

void check_stack(const std::vector<Tensor>& w, int64_t NL, int64_t H, int64_t I, bool& has_bias) {
  TORCH_CHECK((int64_t)w.size() == 4 * NL, "expected 4 tensors per layer (w_ih, w_hh, b_ih, b_hh)");
  TORCH_CHECK(NL >= 1 && NL <= PDRNN_MAX_LAYERS, "1..4 layers supported by the fused small-H LSTM");
  TORCH_CHECK(pdrnn_lstm_small_supported((int)H, (int)I, (int)NL), "fused small-H LSTM: unsupported (H=", H,
              ", I=", I, ", layers=", NL, ")");
  has_bias = w[2].defined();
  for (int64_t l = 0; l < NL; ++l) {
    const int64_t Iin = l == 0 ? I : H;
    const Tensor& wih = w[l * 4 + 0];
    const Tensor& whh = w[l * 4 + 1];
    CHECK_HIP_TENSOR(wih); CHECK_F32(wih); CHECK_F32(whh);
    TORCH_CHECK(wih.is_contiguous() && whh.is_contiguous(), "LSTM weights must be contiguous");
    TORCH_CHECK(wih.size(0) == 4 * H && wih.size(1) == Iin, "weight_ih_l", l, " shape mismatch");
    TORCH_CHECK(whh.size(0) == 4 * H && whh.size(1) == H, "weight_hh_l", l, " shape mismatch");
    if (has_bias) {
      TORCH_CHECK(w[l * 4 + 2].defined() && w[l * 4 + 3].defined(), "bias presence must be uniform");
      TORCH_CHECK(w[l * 4 + 2].is_contiguous() && w[l * 4 + 3].is_contiguous());
    }
  }
}

// Returns {out_or_hseq, hn, cn, act}.  x: [B,T,I] (batch_first) or [T,B,I];
// with idx, x is a [N,T,I] source table and B = len(idx).
std::vector<Tensor> lstm_small_fwd(const Tensor& x, const optional<Tensor>& idx, const std::vector<Tensor>& w,
                                   const optional<Tensor>& h0, const optional<Tensor>& c0, int64_t H, int64_t NL,
                                   bool batch_first, bool save, bool need_out, int64_t nb, int64_t split,
                                   int64_t cell) {
  CHECK_HIP_TENSOR(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be float32 or bfloat16");
  TORCH_CHECK(x.dim() == 3, "x must be 3-D");
  TORCH_CHECK(x.stride(2) == 1, "x innermost dim must be contiguous");
  const c10::DeviceGuard guard(x.device());
  const int64_t I = x.size(2);
  bool has_bias = false;
  check_stack(w, NL, H, I, has_bias);
  int64_t B, T, x_sb, x_st;
  if (idx.has_value() && idx->defined()) {
    TORCH_CHECK(batch_first, "gathered input requires batch_first");
    TORCH_CHECK(idx->scalar_type() == at::kLong && idx->is_contiguous());
    B = idx->size(0); T = x.size(1); x_sb = x.stride(0); x_st = x.stride(1);
  } else if (batch_first) {
    B = x.size(0); T = x.size(1); x_sb = x.stride(0); x_st = x.stride(1);
  } else {
    T = x.size(0); B = x.size(1); x_sb = x.stride(1); x_st = x.stride(0);
  }
  auto opts = x.options().dtype(at::kFloat);
  Tensor hn = at::empty({NL, B, H}, opts), cn = at::empty({NL, B, H}, opts);
  Tensor hseq, act, out;
  PdrnnLstmSmallFwdArgs a{};
  a.prio = prio_env();
  a.x = reinterpret_cast<const float*>(x.data_ptr());
  a.x_bf16 = x.scalar_type() == at::kBFloat16;
  a.idx = (idx.has_value() && idx->defined()) ? idx->data_ptr<int64_t>() : nullptr;
  a.x_sb = x_sb; a.x_st = x_st;
  for (int64_t l = 0; l < NL; ++l) {
    a.w_ih[l] = w[l * 4 + 0].data_ptr<float>();
    a.w_hh[l] = w[l * 4 + 1].data_ptr<float>();
    a.b_ih[l] = has_bias ? w[l * 4 + 2].data_ptr<float>() : nullptr;
    a.b_hh[l] = has_bias ? w[l * 4 + 3].data_ptr<float>() : nullptr;
  }
  if (h0.has_value() && h0->defined()) TORCH_CHECK(h0->is_contiguous() && h0->numel() == NL * B * H, "h0 shape");
  if (c0.has_value() && c0->defined()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == NL * B * H, "c0 shape");
  a.h0 = opt_ptr(h0); a.c0 = opt_ptr(c0);
  if (save) {
    hseq = at::empty({NL, B, T, H}, opts);
    act = at::empty({NL, B, T, 5, H}, opts);
    a.hseq = hseq.data_ptr<float>();
    a.act = act.data_ptr<float>();
    out = hseq;
  } else if (need_out) {
    out = batch_first ? at::empty({B, T, H}, opts) : at::empty({T, B, H}, opts);
    a.out = out.data_ptr<float>();
    a.o_sb = batch_first ? T * H : H;
    a.o_st = batch_first ? H : B * H;
  }
  a.hn = hn.data_ptr<float>(); a.cn = cn.data_ptr<float>();
  a.B = (int)B; a.T = (int)T; a.I = (int)I; a.NL = (int)NL; a.cell = (int)cell;
  if (split <= 0) split = pdrnn_lstm_small_max_split((int)H, (int)NL, 0);
  Tensor stamps;
  if (stamps_enabled()) {
    stamps = at::zeros({(B + nb - 1) / nb, 8}, opts.dtype(at::kLong));
    a.stamps = reinterpret_cast<uint64_t*>(stamps.data_ptr<int64_t>());
  }
  if (B > 0 && T > 0)
    HIP_LAUNCH_CHECK(pdrnn_lstm_small_fwd(&a, (int)H, (int)nb, (int)split, save ? 1 : 0, cur_stream()));
  if (stamps.defined()) report_stamps(save ? "fwd(train)" : "fwd(infer)", stamps, (int)(T + NL - 1));
  return {out, hn, cn, act};
}

// Returns {dparams_flat[P] (nn.LSTM parameter order), dx, dh0, dc0}.
std::vector<Tensor> lstm_small_bwd(const Tensor& x, const optional<Tensor>& idx, const std::vector<Tensor>& w,
                                   const optional<Tensor>& h0, const optional<Tensor>& c0, const Tensor& hseq,
                                   const Tensor& act, const optional<Tensor>& dout, const optional<Tensor>& dhn,
                                   const optional<Tensor>& dcn, int64_t H, int64_t NL, bool batch_first,
                                   bool need_dx, bool need_dh0, int64_t nb, int64_t split,
                                   const optional<Tensor>& grad_accum, int64_t cell) {
  CHECK_HIP_TENSOR(x);
  const c10::DeviceGuard guard(x.device());
  const int64_t I = x.size(2);
  bool has_bias = false;
  check_stack(w, NL, H, I, has_bias);
  const bool gathered = idx.has_value() && idx->defined();
  int64_t B, T, x_sb, x_st;
  if (gathered) {
    B = idx->size(0); T = x.size(1); x_sb = x.stride(0); x_st = x.stride(1);
  } else if (batch_first) {
    B = x.size(0); T = x.size(1); x_sb = x.stride(0); x_st = x.stride(1);
  } else {
    T = x.size(0); B = x.size(1); x_sb = x.stride(1); x_st = x.stride(0);
  }
  TORCH_CHECK(hseq.is_contiguous() && act.is_contiguous());
  StackLayout L = stack_layout(w, NL, has_bias);
  auto opts = x.options().dtype(at::kFloat);
  if (split <= 0) split = pdrnn_lstm_small_max_split((int)H, (int)NL, 1);
  const int grid = pdrnn_lstm_small_bwd_grid((int)H, (int)NL, (int)T, (int)B, (int)nb, (int)split);
  TORCH_CHECK(grid > 0, "unsupported backward tile nb=", nb);
  Tensor slab = at::empty({std::max(grid, 1), L.P}, opts);
  Tensor dx, dh0, dc0;
  PdrnnLstmSmallBwdArgs a{};
  a.prio = prio_env();
  a.x = reinterpret_cast<const float*>(x.data_ptr());
  a.x_bf16 = x.scalar_type() == at::kBFloat16;
  a.idx = gathered ? idx->data_ptr<int64_t>() : nullptr;
  a.x_sb = x_sb; a.x_st = x_st;
  for (int64_t l = 0; l < NL; ++l) {
    a.w_ih[l] = w[l * 4 + 0].data_ptr<float>();
    a.w_hh[l] = w[l * 4 + 1].data_ptr<float>();
    a.off_wih[l] = L.off_wih[l]; a.off_whh[l] = L.off_whh[l];
    a.off_bih[l] = L.off_bih[l]; a.off_bhh[l] = L.off_bhh[l];
  }
  a.h0 = opt_ptr(h0); a.c0 = opt_ptr(c0);
  a.hseq = hseq.data_ptr<float>(); a.act = act.data_ptr<float>();
  if (dout.has_value() && dout->defined()) {
    CHECK_F32(*dout);
    TORCH_CHECK(dout->stride(2) == 1, "dout innermost dim must be contiguous");
    a.dout = dout->data_ptr<float>();
    if (batch_first || gathered) { a.d_sb = dout->stride(0); a.d_st = dout->stride(1); }
    else { a.d_sb = dout->stride(1); a.d_st = dout->stride(0); }
  }
  if (dhn.has_value() && dhn->defined()) TORCH_CHECK(dhn->is_contiguous(), "dhn must be contiguous");
  if (dcn.has_value() && dcn->defined()) TORCH_CHECK(dcn->is_contiguous(), "dcn must be contiguous");
  a.dhn = opt_ptr(dhn); a.dcn = opt_ptr(dcn);
  if (need_dx) {
    TORCH_CHECK(!gathered, "input gradient of a gathered batch is not supported");
    dx = at::zeros(x.sizes(), x.options().dtype(at::kFloat));
    a.dx = dx.data_ptr<float>();
    a.dx_sb = batch_first ? dx.stride(0) : dx.stride(1);
    a.dx_st = batch_first ? dx.stride(1) : dx.stride(0);
  }
  if (need_dh0) {
    dh0 = at::empty({NL, B, H}, opts);
    dc0 = at::empty({NL, B, H}, opts);
    a.dh0 = dh0.data_ptr<float>(); a.dc0 = dc0.data_ptr<float>();
  }
  a.slab = slab.data_ptr<float>();
  a.P = L.P;
  a.B = (int)B; a.T = (int)T; a.I = (int)I; a.NL = (int)NL; a.cell = (int)cell;
  Tensor dparams;
  float beta = 0.f;
  if (grad_accum.has_value() && grad_accum->defined()) {
    TORCH_CHECK(grad_accum->numel() == L.P && grad_accum->is_contiguous(), "grad_accum must be flat [P]");
    dparams = *grad_accum;
    beta = 1.f;
  } else {
    dparams = at::empty({L.P}, opts);
  }
  if (B > 0 && T > 0) {
    Tensor stamps;
    if (stamps_enabled()) {
      stamps = at::zeros({grid, 8}, opts.dtype(at::kLong));
      a.stamps = reinterpret_cast<uint64_t*>(stamps.data_ptr<int64_t>());
    }
    HIP_LAUNCH_CHECK(pdrnn_lstm_small_bwd(&a, (int)H, (int)nb, (int)split, grid, cur_stream()));
    if (stamps.defined()) report_stamps("bwd", stamps, (int)(T + NL - 1));
    const int split = std::min<int>(64, std::max<int>(1, grid / 16));
    Tensor work = at::empty({split, L.P}, opts);
    HIP_LAUNCH_CHECK(pdrnn_slab_reduce(slab.data_ptr<float>(), grid, L.P, dparams.data_ptr<float>(), beta,
                                       work.data_ptr<float>(), split, cur_stream()));
  } else if (beta == 0.f) {
    dparams.zero_();
  }
  return {dparams, dx, dh0, dc0};
}

// Per-phase cycles per step of the phase-stamped four-wave forward (rows of
// 24: 8 loop stamps, then waves 0 / 2: five phase sums and the step count),
// averaged over the workgroups.
void report_phase_stamps(const Tensor& st) {
  auto h = st.cpu();
  const int64_t g = h.size(0);
  const int64_t* p = h.data_ptr<int64_t>();
  static const char* names[5] = {"reads", "products", "quad-reduce", "cell+stores", "barrier"};
  for (int w = 0; w < 2; ++w) {
    double m[5] = {0, 0, 0, 0, 0};
    int64_t used = 0;
    for (int64_t i = 0; i < g; ++i) {
      const int64_t* r = p + i * 24 + 8 + 8 * w;
      if (r[5] <= 0) continue;
      for (int k = 0; k < 5; ++k) m[k] += (double)r[k] / (double)r[5];
      ++used;
    }
    double tot = 0;
    fprintf(stderr, "[stamps] fwd4 phases layer %d (wave %d, %lld workgroups, cycles/step):", w, 2 * w, (long long)used);
    for (int k = 0; k < 5; ++k) {
      const double v = used ? m[k] / used : 0.0;
      tot += v;
      fprintf(stderr, " %s %.0f", names[k], v);
    }
    fprintf(stderr, " | total %.0f\n", tot);
  }
}

// Fused motion training step on the native path: LSTM stack forward with the
// classifier head + cross-entropy fused into its epilogue, BPTT backward, and
// one deterministic reduction that writes every parameter gradient straight
// into `flat_grad` (the model's flat gradient buffer = the DDP all-reduce
// bucket, parameter order: lstm.* then head weight, head bias) and the batch
// statistics [mean loss, n, n_correct] into `stats`.  No autograd graph, no
// per-op launches: 4 kernels per step, graph-capturable.
void lstm_head_train_step(const Tensor& x, const optional<Tensor>& idx, const Tensor& labels,
                          const std::vector<Tensor>& w, const Tensor& head_w, const optional<Tensor>& head_b,
                          Tensor flat_grad, Tensor stats, int64_t H, int64_t NL, int64_t split_fwd,
                          int64_t split_bwd, int64_t nb_fwd, int64_t nb_bwd,
                          const optional<std::vector<Tensor>>& adam_state,
                          const optional<std::vector<double>>& adam_hp, int64_t cell,
                          const optional<Tensor>& grad_colmap, const optional<Tensor>& stats_slot_step,
                          int64_t stats_slot_offset, bool round_bf16, const optional<Tensor>& adam_ticket) {
  CHECK_HIP_TENSOR(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be float32 or bfloat16");
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be [N, T, I] with contiguous rows");
  const c10::DeviceGuard guard(x.device());
  const int64_t I = x.size(2);
  bool has_bias = false;
  check_stack(w, NL, H, I, has_bias);
  TORCH_CHECK(has_bias, "fused train step expects LSTM biases");
  const bool gathered = idx.has_value() && idx->defined();
  const int64_t B = gathered ? idx->size(0) : x.size(0);
  const int64_t T = x.size(1);
  const int64_t C = head_w.size(0);
  TORCH_CHECK(head_w.dim() == 2 && head_w.size(1) == H && head_w.is_contiguous() && C <= 16, "head weight [C<=16, H]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous(), "labels must be int64");
  StackLayout L = stack_layout(w, NL, true);
  // GRU: `w` is the packed 4-block stack; the flat gradient buffer holds
  // nn.GRU's parameters, reached from the packed slab through grad_colmap
  const bool mapped = grad_colmap.has_value() && grad_colmap->defined();
  TORCH_CHECK(cell == 0 || mapped, "GRU train step needs the packed->nn.GRU gradient column map");
  const int64_t P_rnn = mapped ? grad_colmap->numel() : L.P;
  if (mapped)
    TORCH_CHECK(grad_colmap->scalar_type() == at::kInt && grad_colmap->is_contiguous() &&
                grad_colmap->device() == x.device(), "grad_colmap must be a contiguous int32 device tensor");
  const int* colmap = mapped ? grad_colmap->data_ptr<int>() : nullptr;
  const int64_t P_params = P_rnn + C * H + (head_b.has_value() && head_b->defined() ? C : 0);
  TORCH_CHECK(flat_grad.numel() == P_params && flat_grad.is_contiguous() && flat_grad.scalar_type() == at::kFloat,
              "flat_grad must be the model's flat fp32 gradient buffer (", P_params, " elements)");
  TORCH_CHECK(stats.numel() >= 3 && stats.is_contiguous() && stats.scalar_type() == at::kFloat);
  // stats_slot_step: `stats` is the whole [rows, 3] epoch ring; the row is read
  // on the device from the step count (graph replay, see slab_reduce_adam)
  const float* slot_step = nullptr;
  int ring_rows = 0;
  if (stats_slot_step.has_value() && stats_slot_step->defined()) {
    TORCH_CHECK(stats_slot_step->is_cuda() && stats_slot_step->scalar_type() == at::kFloat &&
                stats.dim() == 2 && stats.size(1) == 3, "stats_slot_step needs a float device step and a [rows, 3] ring");
    slot_step = stats_slot_step->data_ptr<float>();
    ring_rows = (int)stats.size(0);
  }
  const int64_t P_head = P_params - P_rnn;    // head weight (+ bias)
  const int64_t PH = P_head + 3;              // + [loss, count, correct]
  auto opts = x.options().dtype(at::kFloat);
  // hseq / act with the deferred-dW kernel's padding (one h row in front,
  // PDRNN_DW_PAD_ROWS rows behind: it streams whole stages without clamps)
  constexpr int64_t PADR = PDRNN_DW_PAD_ROWS;
  Tensor hseq_buf = at::empty({H + NL * B * T * H + PADR * H}, opts);
  Tensor act = at::empty({NL * B * T * 5 * H + PADR * 5 * H}, opts);
  Tensor hn = at::empty({NL, B, H}, opts), cn = at::empty({NL, B, H}, opts);
  Tensor dh_top = at::empty({B, H}, opts);
  if (split_fwd <= 0) split_fwd = pdrnn_lstm_small_max_split((int)H, (int)NL, 0);
  if (split_bwd <= 0) split_bwd = pdrnn_lstm_small_max_split((int)H, (int)NL, 1);
  if (cell == 1) split_fwd = 1;  // GRU: gate-split forward only
  TORCH_CHECK((split_fwd == 1 || split_fwd == 2) && split_bwd == 1,
              "fused train step runs on the gate-split or 2-lane K-split forward and the unit-group backward");
  if (nb_fwd <= 0) nb_fwd = 1;
  if (nb_bwd <= 0 || cell == 1) nb_bwd = 1;  // the GRU backward is single-sequence
  const int gridb = pdrnn_lstm_small_bwd_grid((int)H, (int)NL, (int)T, (int)B, (int)nb_bwd, (int)split_bwd);
  TORCH_CHECK(gridb > 0, "unsupported backward tile nb=", nb_bwd);
  // Sequence-in-wave kernels (lstm_sw.hip: a sequence's recurrence never
  // leaves its wave) for the motion shape; PDRNN_SW=0 keeps the gate-split /
  // K-split family below (A/B).  Weight gradients deferred to lstm_small_dw.
  // (their act / hseq byte offsets are 32-bit buffer offsets under one
  // 2 GiB descriptor: larger batches take the per-sequence-rebased family)
  const bool sw = sw_enabled() && pdrnn_lstm_sw_ok((int)H, (int)I, (int)NL, (int)cell) == 1 &&
                  pdrnn_lstm_small_dwout_ok((int)H, (int)NL, (int)T) != 0 && T <= 640 &&
                  pdrnn_lstm_sw_fits((int)NL, (int)B, (int)T) == 1;
  const int sw_fmode = sw ? pdrnn_lstm_sw_mode((int)NL, (int)B, 0) : -1;
  int sw_bmode = sw ? pdrnn_lstm_sw_mode((int)NL, (int)B, 1) : -1;
  if (sw_bmode == 4 && T % 4) sw_bmode = 2;  // register dW: whole 4-step K steps
  // sequence-in-wave latency regime (forward mode 5, backward mode 4): one
  // launch for forward + BPTT per step (lstm_sw_step_kernel)
  const bool sw_step = sw && sw_fmode == 5 && sw_bmode == 4 && !stamps_enabled() && sw_one_launch_enabled() &&
                       pdrnn_lstm_sw_step_ok((int)NL, (int)B, (int)T) == 1;
  Tensor head_slab = at::empty({B, PH}, opts);
  // Above one residency round the BPTT defers its weight gradients: the
  // recurrence writes the gate gradients (into `act`, in place) and the
  // matrix-core kernel lstm_small_dw forms dW / db over all B*T rows, one slab
  // row per K chunk (see pdrnn_lstm_small_bwd_dwout).  One round or less keeps
  // the one-launch step (register-resident dW, no extra launch).
  const int dw_mode = pdrnn_lstm_small_dwout_ok((int)H, (int)NL, (int)T);
  const bool dwout = sw || (nb_bwd == 1 && split_bwd == 1 && ((gridb < B && dw_mode == 1) || dw_mode == 2));
  // deferred dW: sequences per BPTT workgroup; the matrix-core launch forms
  // dW over fixed K chunks, one slab row each
  const int nb_dw = dwout ? pdrnn_lstm_small_bwd_dwout_nb((int)H, (int)NL, (int)T, (int)B) : (int)nb_bwd;
  // (sequence-in-wave mode 4: the BPTT waves form dW on the matrix cores, one
  // slab row per sequence, no dW launch)
  const bool sw_rdw = sw && sw_bmode == 4;
  const int slab_rows = sw_rdw ? (int)B : dwout ? pdrnn_lstm_small_dw_chunks((int)H, (int)NL, (int)B, (int)T) : gridb;
  Tensor slab = at::empty({slab_rows, L.P}, opts);

  PdrnnLstmSmallFwdArgs f{};
  f.prio = prio_env();
  f.x = reinterpret_cast<const float*>(x.data_ptr());
  f.x_bf16 = x.scalar_type() == at::kBFloat16;
  f.idx = gathered ? idx->data_ptr<int64_t>() : nullptr;
  f.x_sb = x.stride(0); f.x_st = x.stride(1);
  for (int64_t l = 0; l < NL; ++l) {
    f.w_ih[l] = w[l * 4 + 0].data_ptr<float>();
    f.w_hh[l] = w[l * 4 + 1].data_ptr<float>();
    f.b_ih[l] = w[l * 4 + 2].data_ptr<float>();
    f.b_hh[l] = w[l * 4 + 3].data_ptr<float>();
  }
  f.hseq = hseq_buf.data_ptr<float>() + H; f.act = act.data_ptr<float>();
  f.hn = hn.data_ptr<float>(); f.cn = cn.data_ptr<float>();
  f.head_w = head_w.data_ptr<float>();
  f.head_b = (head_b.has_value() && head_b->defined()) ? head_b->data_ptr<float>() : nullptr;
  f.labels = labels.data_ptr<int64_t>();
  f.slab = head_slab.data_ptr<float>(); f.dh_top = dh_top.data_ptr<float>();
  f.slab_P = PH; f.head_off_w = 0; f.head_off_b = C * H; f.stat_off = P_head;
  f.inv_batch = 1.f / (float)std::max<int64_t>(B, 1);
  f.C = (int)C;
  f.B = (int)B; f.T = (int)T; f.I = (int)I; f.NL = (int)NL; f.cell = (int)cell;
  f.w_bf16 = round_bf16 ? 1 : 0;
  hipStream_t st = cur_stream();
  // deferred dW: the fp32 copy of the gathered layer-0 input rows (written by
  // the sequence-in-wave forward, or by the gate-split deferred-dW backward)
  const int64_t xg_ld = (I + 3) / 4 * 4;
  Tensor xg;
  if (dwout) xg = at::empty({(B * T + PADR) * xg_ld + 256}, opts);  // + one DMA job past the last stage
  if (sw) { f.xg_out = xg.data_ptr<float>(); f.xg_ld = (int)xg_ld; }
  // sequences per sequence-in-wave workgroup: two in modes 1 / 3 (mode 5,
  // the four-wave forward, runs one)
  const int sw_fnb = sw ? pdrnn_lstm_sw_nb(sw_fmode) : 1, sw_bnb = sw ? pdrnn_lstm_sw_nb(sw_bmode) : 1;
  Tensor st_f, st_b;
  // PDRNN_TUNE sw_phase=1 (with PDRNN_LSTM_STAMPS): the phase-stamped build
  // of the four-wave forward, rows of 24 (report_phase_stamps)
  const bool phase = stamps_enabled() && sw && sw_fmode == 5 && cell == 0 && pdrnn_tune_int("sw_phase", 0) != 0;
  if (stamps_enabled()) {
    st_f = at::zeros({sw ? (B + sw_fnb - 1) / sw_fnb : (B + nb_fwd - 1) / nb_fwd, phase ? 24 : 8},
                     opts.dtype(at::kLong));
    f.phase_stamps = phase ? 1 : 0;
    st_b = at::zeros({sw ? (B + sw_bnb - 1) / sw_bnb : gridb, 8}, opts.dtype(at::kLong));
    f.stamps = reinterpret_cast<uint64_t*>(st_f.data_ptr<int64_t>());
  }
  // latency regime (one sequence per workgroup in both passes): forward,
  // head/CE and BPTT in one launch; otherwise the forward launches here
  const bool one_launch = !dwout && !st_f.defined() &&
      pdrnn_lstm_small_step_ok((int)H, (int)NL, (int)B, (int)nb_fwd, (int)split_fwd, (int)nb_bwd, (int)split_bwd,
                               gridb) == 1;
  if (sw_step) {
    // (launched with the backward below)
  } else if (sw) HIP_LAUNCH_CHECK(pdrnn_lstm_sw_fwd(&f, sw_fmode, st));
  else if (!one_launch) HIP_LAUNCH_CHECK(pdrnn_lstm_small_fwd(&f, (int)H, (int)nb_fwd, (int)split_fwd, 1, st));

  PdrnnLstmSmallBwdArgs bk{};
  bk.prio = prio_env();
  bk.x = f.x; bk.x_bf16 = f.x_bf16; bk.idx = f.idx; bk.x_sb = f.x_sb; bk.x_st = f.x_st;
  for (int64_t l = 0; l < NL; ++l) {
    bk.w_ih[l] = f.w_ih[l]; bk.w_hh[l] = f.w_hh[l];
    bk.off_wih[l] = L.off_wih[l]; bk.off_whh[l] = L.off_whh[l];
    bk.off_bih[l] = L.off_bih[l]; bk.off_bhh[l] = L.off_bhh[l];
  }
  bk.hseq = f.hseq; bk.act = f.act;
  bk.dhn = dh_top.data_ptr<float>(); bk.dhn_top_only = 1;
  bk.slab = slab.data_ptr<float>(); bk.P = L.P;
  bk.B = (int)B; bk.T = (int)T; bk.I = (int)I; bk.NL = (int)NL; bk.cell = (int)cell;
  bk.w_bf16 = f.w_bf16;
  int grid_dw = gridb;
  if (dwout) {
    grid_dw = sw ? (int)((B + sw_bnb - 1) / sw_bnb)
                 : pdrnn_lstm_small_bwd_dwout_grid((int)H, (int)NL, (int)T, (int)B, nb_dw);
    TORCH_CHECK(grid_dw > 0, "deferred-dW backward: no resident grid");
    if (st_f.defined() && !sw) {
      st_b = at::zeros({grid_dw, 8}, opts.dtype(at::kLong));
      bk.stamps = reinterpret_cast<uint64_t*>(st_b.data_ptr<int64_t>());
    }
    bk.dg_out = f.act;  // in place: each row lane overwrites the activation it has consumed
    bk.dg_st = 5 * H;
    bk.xg_out = xg.data_ptr<float>();
    bk.xg_ld = (int)xg_ld;
  }
  if (st_b.defined()) bk.stamps = reinterpret_cast<uint64_t*>(st_b.data_ptr<int64_t>());
  PdrnnLstmSmallDwArgs dw{};
  if (dwout) {
    dw.xg = xg.data_ptr<float>(); dw.xg_ld = bk.xg_ld;
    dw.hseq = f.hseq; dw.dg = f.act; dw.dg_st = 5 * H;
    dw.slab = slab.data_ptr<float>(); dw.P = L.P;
    for (int64_t l = 0; l < NL; ++l) {
      dw.off_wih[l] = L.off_wih[l]; dw.off_whh[l] = L.off_whh[l];
      dw.off_bih[l] = L.off_bih[l]; dw.off_bhh[l] = L.off_bhh[l];
    }
    dw.B = (int)B; dw.T = (int)T; dw.I = (int)I; dw.NL = (int)NL; dw.chunks = slab_rows;
  }
  if (sw_step) HIP_LAUNCH_CHECK(pdrnn_lstm_sw_step(&f, &bk, st));
  else if (sw) HIP_LAUNCH_CHECK(pdrnn_lstm_sw_bwd(&bk, sw_bmode, st));
  else if (one_launch) HIP_LAUNCH_CHECK(pdrnn_lstm_small_step(&f, &bk, (int)H, st));
  else if (dwout) HIP_LAUNCH_CHECK(pdrnn_lstm_small_bwd_dwout(&bk, (int)H, grid_dw, nb_dw, st));
  else HIP_LAUNCH_CHECK(pdrnn_lstm_small_bwd(&bk, (int)H, (int)nb_bwd, (int)split_bwd, gridb, st));
  if (dwout && !sw_rdw) HIP_LAUNCH_CHECK(pdrnn_lstm_small_dw(&dw, (int)H, st));
  if (st_f.defined()) {
    const int bw_iters = sw ? (int)(T + NL - 1)
                            : (int)(T + 2 * (NL - 1)) * (int)((B + (int64_t)grid_dw * nb_dw - 1) / ((int64_t)grid_dw * nb_dw));
    if (phase) report_phase_stamps(st_f);
    report_stamps(sw ? "fwd(head step, seq-in-wave)" : "fwd(head step)",
                  phase ? st_f.narrow(1, 0, 8).contiguous() : st_f, (int)(T + NL - 1));
    report_stamps(sw ? "bwd(head step, seq-in-wave, deferred dW)"
                     : dwout ? "bwd(head step, lean, deferred dW)" : "bwd(head step, lean)",
                  st_b, bw_iters);
  }

  // one-pass reduction of the slabs into the flat gradient (+ batch statistics),
  // with Adam folded in for a single process (slab_reduce_adam_kernel)
  PdrnnAdamArgs ad{};
  const bool fold_adam = adam_state.has_value() && adam_hp.has_value();
  if (fold_adam) {
    const auto& as = *adam_state;
    const auto& hp = *adam_hp;  // lr, beta1, beta2, eps, weight_decay, step, decoupled
    TORCH_CHECK(as.size() == 3 && hp.size() == 7, "adam_state = [param, exp_avg, exp_avg_sq], 7 hyper-parameters");
    for (const auto& t : as)
      TORCH_CHECK(t.is_contiguous() && t.numel() == P_params && t.scalar_type() == at::kFloat, "flat fp32 Adam buffers");
    ad.param = as[0].data_ptr<float>(); ad.exp_avg = as[1].data_ptr<float>(); ad.exp_avg_sq = as[2].data_ptr<float>();
    ad.n = P_params;
    ad.lr = (float)hp[0]; ad.beta1 = (float)hp[1]; ad.beta2 = (float)hp[2]; ad.eps = (float)hp[3];
    ad.weight_decay = (float)hp[4];
    ad.bias_correction1 = (float)(1.0 - std::pow(hp[1], hp[5]));
    ad.bias_correction2_sqrt = (float)std::sqrt(1.0 - std::pow(hp[2], hp[5]));
    ad.grad_scale = 1.f; ad.decoupled = hp[6] != 0.0 ? 1 : 0; ad.maximize = 0;
    // graph-replayed single-process epoch: the step count lives on the device
    // (the stats ring's slot step), advanced by the reduction's last workgroup
    if (adam_ticket.has_value() && adam_ticket->defined()) {
      TORCH_CHECK(slot_step != nullptr, "adam_ticket needs stats_slot_step (the device step count)");
      TORCH_CHECK(adam_ticket->is_cuda() && adam_ticket->scalar_type() == at::kInt && adam_ticket->numel() >= 1,
                  "adam_ticket: int32 device word");
      ad.step_advance = const_cast<float*>(slot_step);
      ad.ticket = reinterpret_cast<unsigned int*>(adam_ticket->data_ptr<int>());
    }
  }
  HIP_LAUNCH_CHECK(pdrnn_slab_reduce_adam(fold_adam ? &ad : nullptr, slab.data_ptr<float>(), slab_rows, P_rnn, L.P,
                                          colmap, head_slab.data_ptr<float>(), B, PH, P_params,
                                          flat_grad.data_ptr<float>(), stats.data_ptr<float>(), slot_step,
                                          (int)stats_slot_offset, ring_rows, st));
}

std::vector<Tensor> xent_fwd(const Tensor& logits, const Tensor& labels, int64_t ignore_index, bool need_grad) {
  CHECK_HIP_TENSOR(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, C] with contiguous rows");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == logits.size(0));
  const c10::DeviceGuard guard(logits.device());
  const int64_t N = logits.size(0), C = logits.size(1);
  auto f32 = logits.options().dtype(at::kFloat);
  PdrnnXentArgs a{};
  a.logits = logits.data_ptr();
  a.ld = logits.stride(0);
  switch (logits.scalar_type()) {
    case at::kFloat: a.dtype = 0; break;
    case at::kBFloat16: a.dtype = 1; break;
    case at::kHalf: a.dtype = 2; break;
    default: TORCH_CHECK(false, "xent: unsupported logits dtype");
  }
  a.labels = labels.data_ptr<int64_t>();
  a.N = N; a.C = C; a.ignore_index = ignore_index;
  Tensor dlogits;
  if (need_grad) { dlogits = at::empty({N, C}, f32); a.dlogits = dlogits.data_ptr<float>(); }
  const int nblocks = std::max(1, pdrnn_xent_partial_blocks(N, C));
  Tensor partial = at::empty({nblocks, 3}, f32);
  Tensor stats = at::empty({3}, f32);
  a.partial = partial.data_ptr<float>();
  a.out = stats.data_ptr<float>();
  HIP_LAUNCH_CHECK(pdrnn_xent_fwd(&a, cur_stream()));
  return {stats, dlogits};
}

// out_dtype: the gradient's dtype (fp32 default; bf16 / fp16 for a 16-bit head)
Tensor xent_bwd(const Tensor& dlogits, const Tensor& grad_out, const Tensor& stats, optional<at::ScalarType> out_dtype) {
  CHECK_HIP_TENSOR(dlogits);
  const c10::DeviceGuard guard(dlogits.device());
  Tensor g = grad_out.to(at::kFloat).contiguous();
  const at::ScalarType od = out_dtype.value_or(at::kFloat);
  TORCH_CHECK(od == at::kFloat || od == at::kBFloat16 || od == at::kHalf, "xent_bwd: fp32 / bf16 / fp16 output");
  Tensor out = at::empty_like(dlogits, dlogits.options().dtype(od));
  const int code = od == at::kFloat ? 2 : (od == at::kBFloat16 ? 0 : 1);
  HIP_LAUNCH_CHECK(pdrnn_xent_bwd(dlogits.data_ptr<float>(), g.data_ptr<float>(), stats.data_ptr<float>(),
                                  out.data_ptr(), dlogits.numel(), code, cur_stream()));
  return out;
}

void adam_flat(Tensor param, const Tensor& grad, Tensor exp_avg, Tensor exp_avg_sq,
               const optional<Tensor>& max_exp_avg_sq, double lr, double beta1, double beta2, double eps,
               double weight_decay, double step, double grad_scale, bool decoupled, bool maximize,
               const optional<Tensor>& lr_t, const optional<Tensor>& step_t, const optional<Tensor>& ticket,
               const optional<Tensor>& skip) {
  CHECK_HIP_TENSOR(param);
  for (const Tensor* t : std::initializer_list<const Tensor*>{&param, &grad, &exp_avg, &exp_avg_sq}) {
    CHECK_F32(*t);
    TORCH_CHECK(t->is_contiguous() && t->numel() == param.numel(), "adam_flat: flat contiguous buffers expected");
  }
  const c10::DeviceGuard guard(param.device());
  PdrnnAdamArgs a{};
  a.param = param.data_ptr<float>();
  a.grad = grad.data_ptr<float>();
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.max_exp_avg_sq = (max_exp_avg_sq.has_value() && max_exp_avg_sq->defined()) ? max_exp_avg_sq->data_ptr<float>() : nullptr;
  a.n = param.numel();
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.bias_correction1 = (float)(1.0 - std::pow(beta1, step));
  a.bias_correction2_sqrt = (float)std::sqrt(1.0 - std::pow(beta2, step));
  a.grad_scale = (float)grad_scale;
  a.decoupled = decoupled ? 1 : 0;
  a.maximize = maximize ? 1 : 0;
  a.lr_ptr = opt_ptr(lr_t);
  a.step_ptr = opt_ptr(step_t);
  if (ticket.has_value() && ticket->defined()) {
    // advance mode: step_t holds the count BEFORE this step and is bumped in-kernel
    TORCH_CHECK(step_t.has_value() && step_t->defined(), "adam_flat: ticket needs the device step tensor");
    TORCH_CHECK(ticket->is_cuda() && ticket->scalar_type() == at::kInt && ticket->numel() >= 1,
                "adam_flat: ticket must be a device int32 tensor (zero-initialised)");
    a.step_advance = step_t->data_ptr<float>();
    a.ticket = reinterpret_cast<unsigned int*>(ticket->data_ptr<int>());
    a.step_ptr = nullptr;
  }
  if (skip.has_value() && skip->defined()) {
    TORCH_CHECK(skip->is_cuda() && skip->scalar_type() == at::kInt && skip->numel() >= 1,
                "adam_flat: skip must be a device int32 tensor");
    a.skip = skip->data_ptr<int>();
  }
  HIP_LAUNCH_CHECK(pdrnn_adam_flat(&a, cur_stream()));
}

// Gradient-norm clipping of a flat fp32 gradient in place; returns the
// device tensor [scale, norm] (no host sync).
Tensor clip_flat(Tensor g, double max_norm, double eps) {
  CHECK_HIP_TENSOR(g); CHECK_F32(g);
  TORCH_CHECK(g.is_contiguous(), "clip_flat: contiguous gradient expected");
  const c10::DeviceGuard guard(g.device());
  const int64_t n = g.numel();
  int64_t nparts = (n + 256 * 16 - 1) / (256 * 16);
  nparts = std::max<int64_t>(1, std::min<int64_t>(nparts, 1024));
  Tensor work = at::empty({nparts + 2}, g.options());
  HIP_LAUNCH_CHECK(pdrnn_clip_flat(g.data_ptr<float>(), n, (float)max_norm, (float)eps, work.data_ptr<float>(),
                                   (int)nparts, work.data_ptr<float>() + nparts, cur_stream()));
  return work.narrow(0, nparts, 2);
}

Tensor embedding_fwd(const Tensor& weight, const Tensor& idx, optional<at::ScalarType> out_dtype) {
  CHECK_HIP_TENSOR(weight); CHECK_F32(weight);
  TORCH_CHECK(weight.is_contiguous() && weight.dim() == 2);
  TORCH_CHECK(idx.scalar_type() == at::kLong);
  const c10::DeviceGuard guard(weight.device());
  Tensor flat = idx.contiguous().view({-1});
  std::vector<int64_t> shape(idx.sizes().begin(), idx.sizes().end());
  shape.push_back(weight.size(1));
  const at::ScalarType odt = out_dtype.has_value() ? *out_dtype : at::kFloat;
  Tensor out = at::empty(shape, weight.options().dtype(odt));
  if (odt == at::kFloat) {
    HIP_LAUNCH_CHECK(pdrnn_embedding_fwd(weight.data_ptr<float>(), flat.data_ptr<int64_t>(), out.data_ptr<float>(),
                                         flat.numel(), weight.size(1), weight.size(0), cur_stream()));
  } else {
    HIP_LAUNCH_CHECK(pdrnn_embedding_fwd16(weight.data_ptr<float>(), flat.data_ptr<int64_t>(), u16m(out),
                                           flat.numel(), weight.size(1), weight.size(0), dtype_code(out),
                                           cur_stream()));
  }
  return out;
}

// out: accumulate into this fp32 [V, dim] gradient instead of returning a new one
Tensor embedding_bwd(const Tensor& dout, const Tensor& idx, int64_t num_embeddings, int64_t padding_idx,
                     const optional<Tensor>& out) {
  CHECK_HIP_TENSOR(dout);
  const c10::DeviceGuard guard(dout.device());
  const int64_t dim = dout.size(-1);
  Tensor g = dout.contiguous().view({-1, dim});
  int dt = 2;
  if (g.scalar_type() == at::kBFloat16) dt = 0;
  else if (g.scalar_type() == at::kHalf) dt = 1;
  else g = g.to(at::kFloat);
  Tensor flat = idx.contiguous().view({-1}).to(at::kLong);
  Tensor perm, offsets;
  if (num_embeddings <= 16384 && flat.numel() < ((int64_t)1 << 31)) {
    // in-tree stable counting sort (kernels/embedding.hip)
    perm = at::empty({flat.numel()}, flat.options());
    offsets = at::empty({num_embeddings + 1}, flat.options());
    Tensor scratch = at::empty({std::max<int64_t>(pdrnn_embedding_sort_scratch(flat.numel(), num_embeddings), 1)},
                               flat.options().dtype(at::kInt));
    HIP_LAUNCH_CHECK(pdrnn_embedding_sort(flat.data_ptr<int64_t>(), flat.numel(), num_embeddings,
                                          scratch.data_ptr<int>(), perm.data_ptr<int64_t>(),
                                          offsets.data_ptr<int64_t>(), cur_stream()));
  } else {  // large vocabularies: library stable sort + bucket bounds
    flat = at::where(flat < 0, flat + num_embeddings, flat);
    auto sorted = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
    Tensor vals = std::get<0>(sorted);
    perm = std::get<1>(sorted).contiguous();
    offsets = at::searchsorted(vals, at::arange(num_embeddings + 1, flat.options())).contiguous();
  }
  const bool acc = out.has_value() && out->defined();
  if (acc)
    TORCH_CHECK(out->scalar_type() == at::kFloat && out->is_contiguous() && out->size(0) == num_embeddings &&
                out->numel() == num_embeddings * dim, "embedding_bwd: out must be the fp32 [V, dim] gradient");
  // small vocabulary, many contributions per row: split each row's list
  const int64_t per_row = g.size(0) / std::max<int64_t>(num_embeddings, 1);
  if (num_embeddings <= 4096 && per_row >= 64) {
    Tensor dw = acc ? *out : at::empty({num_embeddings, dim}, dout.options().dtype(at::kFloat));
    const int pieces = (int)std::min<int64_t>(32, std::max<int64_t>(2, per_row / 32));
    Tensor part = at::empty({num_embeddings, pieces, dim}, dout.options().dtype(at::kFloat));
    HIP_LAUNCH_CHECK(pdrnn_embedding_bwd_pieces(g.data_ptr(), dt, perm.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(),
                                                part.data_ptr<float>(), pieces, dw.data_ptr<float>(), num_embeddings,
                                                dim, padding_idx, acc ? 1 : 0, cur_stream()));
    return dw;
  }
  Tensor dw = at::empty({num_embeddings, dim}, dout.options().dtype(at::kFloat));
  HIP_LAUNCH_CHECK(pdrnn_embedding_bwd_csr2(g.data_ptr(), dt, perm.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(),
                                            dw.data_ptr<float>(), num_embeddings, dim, padding_idx, cur_stream()));
  if (acc) {
    out->add_(dw.view_as(*out));
    return *out;
  }
  return dw;
}


// ---------------------------------------------------------------------------
// Persistent recurrence (one launch per layer direction set,
// W_hh register-resident; lstm_large.hip) when the shape is covered and
// PDRNN_LSTM_PERSIST != 0.  A grid-sync spin that times out (bounded at 2 s
// in the kernel: co-residency lost, e.g. to RCCL kernels on the comm stream)
// leaves that launch's outputs invalid.
//   * verify on (set_persist_verify(1) -- parallel/comm.py get_comm does it for every
//     multi-rank GPU job --
//     or PDRNN_LSTM_PERSIST_VERIFY=1): the host synchronises after the launch
//     and reads its error flag; on a timeout it warns, clears the sticky flag
//     and returns kPersistFailed, and the caller re-runs the layer on the
//     per-step kernels -- before anything (the next layer, the optimizer)
//     consumes the result.
//   * verify off (single rank: nothing else runs on the GPU): no
//     synchronisation; a sticky per-device flag is copied to pinned memory
//     after every launch and checked at the next one (fails loudly one call
//     later), and by persist_check() at epoch end.
//   * verify per step (set_persist_verify(2) -- only the LM trainer, which
//     carries the skip word and re-runs skipped steps, switches to it:
//     parallel/comm.py use_step_verification): no synchronisation at all; a timed-out launch leaves the sticky
//     flag set, the step's later persistent launches run per step, the
//     trainer all-reduces the flag on the stream and hands it to the Adam
//     launch as its skip word (persist_sticky_flag), reads its pinned copy
//     one step later and re-runs the skipped steps (train/lm.py settle;
//     persist_step_check clears and counts).  Launch-verify costs 6.7 % of
//     the char-LM step (profiles/r4/nb1_charlm_verify*.log).
enum PersistResult { kPersistNotRun = 0, kPersistOk = 1, kPersistFailed = 2 };
std::atomic<int> g_persist_verify{-1};     // -1: PDRNN_LSTM_PERSIST_VERIFY (default off); 1 launch, 2 step
std::atomic<int> g_persist_inject{0};      // tests: flag the next N launches as timed out
std::atomic<long long> g_persist_fallbacks{0};
std::atomic<long long> g_persist_tagx{0};  // launches on the tagged forward exchange
// after the first timed-out launch in a process the persistent path is off for
// good: a lost co-residency (RCCL kernels beside it) tends to recur every step,
// and each occurrence costs the 2 s spin bound plus the per-step re-run
std::atomic<int> g_persist_disabled{0};
int persist_verify_mode() {
  const int v = g_persist_verify.load();
  if (v >= 0) return v;
  static const int env = [] {
    const char* e = std::getenv("PDRNN_LSTM_PERSIST_VERIFY");
    return e ? std::atoi(e) : 0;
  }();
  return env;
}
bool persist_verify_on() { return persist_verify_mode() == 1; }
// leaked on purpose: no tensor destructor runs after the HIP runtime is gone
std::vector<Tensor>& persist_sticky() { static auto& v = *new std::vector<Tensor>(64); return v; }
// host mirrors: raw pinned words, never freed (a pinned tensor held in a
// static is released by the host caching allocator at exit, after tools such
// as the profiler have finalised)
int* pinned_word() {
  void* p = nullptr;
  TORCH_CHECK(hipHostMalloc(&p, sizeof(int), hipHostMallocDefault) == hipSuccess, "hipHostMalloc");
  *static_cast<int*>(p) = 0;
  return static_cast<int*>(p);
}
std::vector<int*>& persist_sticky_host() { static auto& v = *new std::vector<int*>(64, nullptr); return v; }

// Row tiles of the persistent recurrence for this launch, or 0 when the
// per-step kernels run it (PDRNN_LSTM_PERSIST=0, an explicit tile, the path
// turned off after a timeout, the fp32 forward, or a shape it does not cover).
int large_persist_plan(int B, int H, int ndir, bool backward, int dt, int64_t tile) {
  static const int env = [] {
    const char* e = std::getenv("PDRNN_LSTM_PERSIST");
    return e ? std::atoi(e) : 1;
  }();
  if (env == 0 || tile >= 0 || g_persist_disabled.load()) return 0;
  // fp32 storage: the persistent backward only -- the persistent forward ran
  // 8.3 us per step against 7.1 for the per-step kernels at the fp32 motion
  // model's H = 128, B = 1440 (its K = H is too short to pay for the 8-wave
  // K split's LDS reduction; the backward's K = 4H is not: 8.6 vs 11.7 us;
  // profiles/r4/h2/h2_persist_f32_cell*.json)
  if (dt == 2 && !backward) return 0;
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  int cus = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess, "CU count");
  // multi-rank: leave the CUs RCCL's kernels may take (comm.cpp, maxCTAs), so
  // a bucket all-reduce resident first never keeps the grid from co-residency
  return pdrnn_lstm_large_persist_mt(B, H, ndir, dt, cus - pdrnn::rccl_cta_reserve());
}

// Zeroed sync words for persistent launches without a fill dispatch per
// launch: slices of a per-(device, stream) pool handed out in order, the whole
// pool re-zeroed by one memset when it wraps.  Stream order makes that safe:
// every launch that used the pool before the memset has finished when it
// runs.  (Graph capture and the diagnostics take fresh zeros instead.)
int* persist_sync_words(int dev, hipStream_t st, int64_t n, const at::TensorOptions& opts) {
  struct Pool {
    Tensor buf;
    int64_t cur = 0;
  };
  constexpr int64_t kPool = 1 << 16;  // ints
  const int64_t need = (n + 63) & ~(int64_t)63;
  if (need > kPool) return nullptr;
  static std::mutex mu;
  static auto& pools = *new std::map<std::pair<int, hipStream_t>, Pool>();  // never destroyed (exit order)
  std::lock_guard<std::mutex> g(mu);
  Pool& p = pools[{dev, st}];
  if (!p.buf.defined()) p.buf = at::zeros({kPool}, opts.dtype(at::kInt));
  if (p.cur + need > kPool) {
    TORCH_CHECK(hipMemsetAsync(p.buf.data_ptr<int>(), 0, kPool * sizeof(int), st) == hipSuccess, "sync pool reset");
    p.cur = 0;
  }
  int* r = p.buf.data_ptr<int>() + p.cur;
  p.cur += need;
  return r;
}

int large_persist(const PdrnnLstmLargeStepArgs& a, int ndir, bool backward, int dt, int64_t tile,
                  const at::TensorOptions& opts, hipStream_t st) {
  static const bool check = [] {
    const char* e = std::getenv("PDRNN_LSTM_PERSIST_CHECK");
    return e && std::atoi(e) != 0;
  }();
  const int mode = 0;  // kernel mode bits: 16 = test hook (persist_inject_timeouts)
  const int mt = large_persist_plan(a.B, a.H, ndir, backward, dt, tile);
  if (mt == 0) return kPersistNotRun;
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  const int nmb = (a.B + 16 * mt - 1) / (16 * mt);
  std::vector<Tensor>& sticky = persist_sticky();
  std::vector<int*>& sticky_host = persist_sticky_host();
  TORCH_CHECK(dev >= 0 && dev < 64, "device index");
  if (!sticky[dev].defined()) {
    sticky[dev] = at::zeros({1}, opts.dtype(at::kInt));
    sticky_host[dev] = pinned_word();
  }
  if (__atomic_load_n(sticky_host[dev], __ATOMIC_RELAXED) != 0) {
    // per-step verification: an earlier launch of this step timed out -- the
    // step's check re-runs it; the rest of the step takes the per-step kernels
    if (persist_verify_mode() == 2) return kPersistNotRun;
    TORCH_CHECK(false, "persistent LSTM recurrence: a grid-sync wait timed out in an earlier launch (results invalid)");
  }
  // [counters | err | pad | stamps]; PDRNN_TUNE persist_stamps=1: workgroup
  // 0 records s_memtime at 7 points of steps 0..63 (kernel mode bit 8),
  // reported per phase after the launch (diagnostics: the launch synchronises)
  const bool pstamps = pdrnn_tune_int("persist_stamps", 0) != 0;
  const int64_t stamp_ints = pstamps ? 2 * 64 * 8 + 2 : 1;
  // 16-bit forward: the tagged h exchange (lstm_large.hip ps_poll_h), a
  // zeroed [2][ndir][B][H] dword buffer behind the counters (16-byte aligned)
  const bool tagx = !backward && dt != 2 && a.T < 65535 && pdrnn_tune_int("persist_tagx", 0) != 0;
  const int64_t head = (ndir * nmb + 1 + stamp_ints + 2 + 3) & ~(int64_t)3;
  const int nslots = tagx ? std::max(2, std::min(pdrnn_tune_int("persist_tagx_slots", 2), a.T)) : 0;
  const int64_t xints = (int64_t)nslots * ndir * a.B * a.H;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool pooled = !pstamps && !tagx && hipStreamIsCapturing(st, &cap) == hipSuccess &&
                      cap == hipStreamCaptureStatusNone;
  Tensor sync;
  int* cnt = pooled ? persist_sync_words(dev, st, head, opts) : nullptr;
  if (cnt == nullptr) {
    sync = at::zeros({head + xints}, opts.dtype(at::kInt));
    cnt = sync.data_ptr<int>();
  }
  uint32_t* xchg = tagx ? reinterpret_cast<uint32_t*>(cnt + head) : nullptr;
  int m = mode | (pstamps ? 8 : 0);
  for (int k = g_persist_inject.load(); k > 0; k = g_persist_inject.load())
    if (g_persist_inject.compare_exchange_weak(k, k - 1)) { m |= 16; break; }
  const hipError_t e = pdrnn_lstm_large_persist(&a, ndir, backward ? 1 : 0, dt, mt, cnt, cnt + ndir * nmb,
                                                sticky[dev].data_ptr<int>(), m, xchg, nslots, st);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // e.g. grid cannot be co-resident: per-step path
    return kPersistNotRun;
  }
  if (tagx) g_persist_tagx++;
  if (persist_verify_on()) {
    static std::vector<int*>& flag = *new std::vector<int*>(64, nullptr);
    if (!flag[dev]) flag[dev] = pinned_word();
    int* hf = flag[dev];
    hf[0] = 0;
    TORCH_CHECK(hipMemcpyAsync(hf, cnt + ndir * nmb, sizeof(int), hipMemcpyDeviceToHost, st) == hipSuccess, "flag copy");
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess, "persistent LSTM: stream synchronisation failed");
    if (hf[0] != 0) {
      g_persist_fallbacks++;
      const bool keep = std::getenv("PDRNN_LSTM_PERSIST_RETRY") != nullptr;  // tests: keep retrying
      if (!keep) g_persist_disabled = 1;
      std::fprintf(stderr, "[pdrnn] persistent LSTM recurrence (%s): a grid-sync wait timed out (co-residency "
                   "lost, fallback #%lld); re-running the layer on the per-step kernels%s\n",
                   backward ? "backward" : "forward", (long long)g_persist_fallbacks.load(),
                   keep ? "" : " and using them for the rest of the process");
      TORCH_CHECK(hipMemsetAsync(sticky[dev].data_ptr<int>(), 0, sizeof(int), st) == hipSuccess, "sticky reset");
      return kPersistFailed;
    }
  }
  TORCH_CHECK(hipMemcpyAsync(sticky_host[dev], sticky[dev].data_ptr<int>(), sizeof(int), hipMemcpyDeviceToHost, st) ==
                  hipSuccess, "sticky copy");
  if (pstamps) {
    // the kernel's stamp base: (err + 1) rounded up to 8 bytes (lstm_large.hip pdrnn_lstm_large_persist)
    const uintptr_t base = (reinterpret_cast<uintptr_t>(cnt + ndir * nmb + 1) + 7) & ~(uintptr_t)7;
    const int64_t off = (int64_t)(base - reinterpret_cast<uintptr_t>(sync.data_ptr<int>())) / 4;
    auto h = sync.narrow(0, off, 2 * 64 * 8).cpu();
    const int64_t* p = reinterpret_cast<const int64_t*>(h.data_ptr<int>());
    double d[6] = {0, 0, 0, 0, 0, 0}, step = 0;
    int n = 0;
    for (int s = 8; s < 63; ++s) {  // (steps 8..62: past the start-up, the next step's start closes the last phase)
      const int64_t* r = p + s * 8;
      const int64_t* q = p + (s + 1) * 8;
      if (!r[0] || !q[0]) continue;
      for (int k = 0; k < 6; ++k) d[k] += (double)(r[k + 1] - r[k]);
      step += (double)(q[0] - r[0]);
      ++n;
    }
    static const char* names[6] = {"wait", "loads+mfma", "lds partials", "cell+h store", "arrive", "acts/c stores"};
    fprintf(stderr, "[persist stamps] %s B=%d H=%d: cycles/step %.0f |", backward ? "bwd" : "fwd", a.B, a.H,
            n ? step / n : 0.0);
    for (int k = 0; k < 6; ++k) fprintf(stderr, " %s %.0f", names[k], n ? d[k] / n : 0.0);
    fprintf(stderr, "\n");
  }
  if (check && persist_verify_mode() != 2) {  // per-step verification re-runs the step instead
    int err = 0;  // (the flag may live in the pooled sync words: read it through the pointer)
    TORCH_CHECK(hipMemcpyAsync(&err, cnt + ndir * nmb, sizeof(int), hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess, "persistent LSTM: flag read failed");
    TORCH_CHECK(err == 0, "persistent LSTM grid sync timed out");
  }
  return kPersistOk;
}

// The current device's sticky timeout flag (device int32 [1], created on
// first use): the deferred per-step verification all-reduces it across ranks
// and hands it to the optimizer launch as its skip word.
Tensor persist_sticky_flag() {
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  TORCH_CHECK(dev >= 0 && dev < 64, "device index");
  std::vector<Tensor>& sticky = persist_sticky();
  if (!sticky[dev].defined()) {
    sticky[dev] = at::zeros({1}, at::TensorOptions().device(at::kCUDA, dev).dtype(at::kInt));
    persist_sticky_host()[dev] = pinned_word();
  }
  return sticky[dev];
}

// Row-owning fp32 recurrence at H = 128 (kernels/lstm_rows_f32.hip) instead of
// the per-step / persistent kernels; PDRNN_TUNE rows=0 turns it off (A/B).
bool rows_f32_on() {
  static const bool on = [] {
    return pdrnn_tune_int("rows", 1) != 0;
  }();
  return on;
}

// Per-step verification: true when a persistent launch on this device timed
// out since the last check (synchronises); the flag is cleared, the timeout
// counted, and the persistent path turned off for the process.
bool persist_step_check() {
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  if (dev < 0 || dev >= 64 || !persist_sticky()[dev].defined()) return false;
  if (persist_sticky()[dev].item<int>() == 0) return false;  // synchronises
  persist_sticky()[dev].zero_();
  if (persist_sticky_host()[dev]) __atomic_store_n(persist_sticky_host()[dev], 0, __ATOMIC_RELAXED);
  g_persist_fallbacks++;
  if (std::getenv("PDRNN_LSTM_PERSIST_RETRY") == nullptr) g_persist_disabled = 1;
  std::fprintf(stderr, "[pdrnn] persistent LSTM recurrence: a grid-sync wait timed out in this step (fallback #%lld); "
               "the step is re-run on the per-step kernels\n", (long long)g_persist_fallbacks.load());
  return true;
}

// End-of-epoch check of the deferred (verify-off) path: raises if any
// persistent launch on this device timed out since the last check.
void persist_check() {
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  if (dev < 0 || dev >= 64 || !persist_sticky()[dev].defined()) return;
  const int v = persist_sticky()[dev].item<int>();  // synchronises
  TORCH_CHECK(v == 0, "persistent LSTM recurrence: a grid-sync wait timed out (results of that step invalid)");
}

// Large-H LSTM layer (both directions in one launch per step).
// ---------------------------------------------------------------------------

// xp: [T, B, ndir*4H] (16-bit, bias included, gate-interleaved per direction)
// w:  ndir x [4H, H] gate-interleaved W_hh;  h0: [ndir, B, H] 16-bit;  c0: [ndir, B, H] f32
// returns hseq [T, B, ndir*H], cseq [ndir, T, B, H] f32, acts [ndir, T, B, 4H]
// cell 1 = GRU packed as [r|z|n_x|n_h] (ops/gru_large.py): c0 is the fp32
// initial hidden state and cseq the fp32 hidden states.
std::vector<Tensor> lstm_large_fwd(const Tensor& xp, const std::vector<Tensor>& w, const optional<Tensor>& h0,
                                   const optional<Tensor>& c0, int64_t H, int64_t reverse_mask, int64_t tile,
                                   int64_t cell) {
  CHECK_HIP_TENSOR(xp);
  const c10::DeviceGuard guard(xp.device());
  const int dt = large_dtype(xp);
  const int ndir = (int)w.size();
  TORCH_CHECK(ndir == 1 || ndir == 2, "1 or 2 directions");
  TORCH_CHECK(pdrnn_lstm_large_supported((int)H), "large LSTM path needs H % 64 == 0");
  TORCH_CHECK(xp.dim() == 3 && xp.size(2) == ndir * 4 * H && xp.stride(2) == 1, "xp must be [T, B, ndir*4H]");
  const int64_t T = xp.size(0), B = xp.size(1);
  TORCH_CHECK(xp.stride(1) == ndir * 4 * H && xp.stride(0) == B * ndir * 4 * H, "xp must be contiguous");
  for (auto& t : w) {
    TORCH_CHECK(t.is_contiguous() && t.size(0) == 4 * H && t.size(1) == H && large_dtype(t) == dt, "w: [4H, H] contiguous");
  }
  auto o16 = xp.options();
  auto o32 = xp.options().dtype(at::kFloat);
  Tensor hseq = at::empty({T, B, ndir * H}, o16);
  Tensor cseq = at::empty({ndir, T, B, H}, o32);
  Tensor acts = at::empty({ndir, T, B, 4 * H}, o16);
  const bool has_h0 = h0.has_value() && h0->defined();
  const bool has_c0 = c0.has_value() && c0->defined();
  if (has_h0) TORCH_CHECK(h0->is_contiguous() && large_dtype(*h0) == dt && h0->numel() == ndir * B * H, "h0 [ndir,B,H]");
  if (has_c0) TORCH_CHECK(c0->is_contiguous() && c0->scalar_type() == at::kFloat && c0->numel() == ndir * B * H, "c0");
  PdrnnLstmLargeStepArgs a{};
  a.B = (int)B; a.H = (int)H; a.T = (int)T; a.reverse_mask = (int)reverse_mask;
  TORCH_CHECK(cell == 0 || cell == 1, "cell: 0 = LSTM, 1 = GRU");
  a.cell = (int)cell;
  for (int d = 0; d < ndir; ++d) {
    PdrnnLstmLargeDir& dd = a.dir[d];
    dd.w = eptr(w[d]);
    dd.xp = eptr(xp, d * 4 * H); dd.xp_sb = ndir * 4 * H; dd.xp_st = B * ndir * 4 * H;
    dd.h0 = has_h0 ? eptr(*h0, d * B * H) : nullptr;
    dd.c0 = has_c0 ? c0->data_ptr<float>() + d * B * H : nullptr;
    dd.hseq = eptrm(hseq, d * H); dd.hseq_sb = ndir * H; dd.hseq_st = B * ndir * H;
    dd.cseq = cseq.data_ptr<float>() + d * T * B * H;
    dd.acts = eptrm(acts, d * T * B * 4 * H);
  }
  hipStream_t st = cur_stream();
  if (tile < 0 && rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, dt)) {
    HIP_LAUNCH_CHECK(pdrnn_lstm_rows_f32(&a, ndir, 0, st));
  } else if (large_persist(a, ndir, false, dt, tile, o32, st) != kPersistOk) {
    for (int64_t s = 0; s < T; ++s) {
      a.step = (int)s;
      HIP_LAUNCH_CHECK(pdrnn_lstm_large_step(&a, ndir, 0, dt, (int)tile, st));
    }
  }
  return {hseq, cseq, acts};
}

// Backward of one layer: returns dgates [ndir, T, B, 4H] (16-bit), dh0, dc0
// [ndir, B, H] f32.  wt: ndir x [H, 4H] (transposed gate-interleaved W_hh).
std::vector<Tensor> lstm_large_bwd(const optional<Tensor>& dout, const optional<Tensor>& dhn,
                                   const optional<Tensor>& dcn, const std::vector<Tensor>& wt, const Tensor& cseq,
                                   const Tensor& acts, const optional<Tensor>& c0, int64_t H, int64_t reverse_mask,
                                   int64_t tile, int64_t cell) {
  CHECK_HIP_TENSOR(acts);
  const c10::DeviceGuard guard(acts.device());
  const int dt = large_dtype(acts);
  const int ndir = (int)wt.size();
  const int64_t T = acts.size(1), B = acts.size(2);
  TORCH_CHECK(acts.is_contiguous() && acts.size(0) == ndir && acts.size(3) == 4 * H, "acts [ndir, T, B, 4H]");
  TORCH_CHECK(cseq.is_contiguous() && cseq.scalar_type() == at::kFloat, "cseq f32");
  for (auto& t : wt) TORCH_CHECK(t.is_contiguous() && t.size(0) == H && t.size(1) == 4 * H && large_dtype(t) == dt, "wt [H, 4H]");
  const bool has_dout = dout.has_value() && dout->defined();
  if (has_dout) {
    TORCH_CHECK(large_dtype(*dout) == dt && dout->dim() == 3 && dout->size(2) == ndir * H && dout->stride(2) == 1,
                "dout [T, B, ndir*H]");
  }
  auto o16 = acts.options();
  auto o32 = acts.options().dtype(at::kFloat);
  Tensor dgates = at::empty({ndir, T, B, 4 * H}, o16);
  Tensor carry = at::empty({ndir, B, H}, o32);
  Tensor dh0 = at::empty({ndir, B, H}, o32), dc0 = at::empty({ndir, B, H}, o32);
  auto f32p = [](const optional<Tensor>& t) -> const float* {
    if (!(t.has_value() && t->defined())) return nullptr;
    TORCH_CHECK(t->is_contiguous() && t->scalar_type() == at::kFloat, "f32 contiguous state grad expected");
    return t->data_ptr<float>();
  };
  const float* dhn_p = f32p(dhn);
  const float* dcn_p = f32p(dcn);
  const float* c0_p = f32p(c0);
  PdrnnLstmLargeStepArgs a{};
  a.B = (int)B; a.H = (int)H; a.T = (int)T; a.reverse_mask = (int)reverse_mask;
  TORCH_CHECK(cell == 0 || cell == 1, "cell: 0 = LSTM, 1 = GRU");
  a.cell = (int)cell;
  for (int d = 0; d < ndir; ++d) {
    PdrnnLstmLargeDir& dd = a.dir[d];
    dd.wt = eptr(wt[d]);
    dd.c0 = c0_p ? c0_p + d * B * H : nullptr;
    dd.cseq = cseq.data_ptr<float>() + d * T * B * H;
    dd.acts = eptrm(acts, d * T * B * 4 * H);
    dd.dgates = eptrm(dgates, d * T * B * 4 * H);
    if (has_dout) {
      dd.dout = eptr(*dout, d * H); dd.dout_sb = dout->stride(1); dd.dout_st = dout->stride(0);
    }
    dd.dhn = dhn_p ? dhn_p + d * B * H : nullptr;
    dd.dcn = dcn_p ? dcn_p + d * B * H : nullptr;
    dd.dc_carry = carry.data_ptr<float>() + d * B * H;
    dd.dh0 = dh0.data_ptr<float>() + d * B * H;
    dd.dc0 = dc0.data_ptr<float>() + d * B * H;
  }
  int big = 0;
  a.splitk = pdrnn_lstm_large_bwd_splitk((int)B, (int)H, ndir, &big);
  a.splitk_big = big;
  // large batch: ping-pong GEMM + cell kernel (fp32 dh through ws)
  a.bwd_pp = a.splitk == 1 ? pdrnn_lstm_large_bwd_pp((int)B, (int)H, ndir, dt) : 0;
  Tensor ws;
  if (a.splitk > 1 || a.bwd_pp) {
    ws = at::empty({a.splitk, 2, B, H}, o32);
    a.ws = ws.data_ptr<float>();
  }
  hipStream_t st = cur_stream();
  if (tile < 0 && rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, dt)) {
    HIP_LAUNCH_CHECK(pdrnn_lstm_rows_f32(&a, ndir, 1, st));  // (the first step's cell backward included)
    return {dgates, dh0, dc0};
  }
  HIP_LAUNCH_CHECK(pdrnn_lstm_large_bwd_first(&a, ndir, dt, st));
  const int pr = large_persist(a, ndir, true, dt, tile, o32, st);
  if (pr != kPersistOk) {
    // a failed launch may have advanced the dc carry: start the layer over
    if (pr == kPersistFailed) HIP_LAUNCH_CHECK(pdrnn_lstm_large_bwd_first(&a, ndir, dt, st));
    for (int64_t s = 0; s < T; ++s) {
      a.step = (int)s;
      HIP_LAUNCH_CHECK(pdrnn_lstm_large_step(&a, ndir, 1, dt, (int)tile, st));
    }
  }
  return {dgates, dh0, dc0};
}


// Time ranges of a unidirectional fp32 H = 128 layer on the row-owning
// kernels, into preallocated full-length tensors (the stacked-layer pipeline
// of ops/lstm_large.py: layer l + 1 runs chunk c while layer l runs chunk
// c + 1).  The state entering t0 > 0 is step t0 - 1 of the same tensors, so
// chunked and whole-sequence runs do the same arithmetic.
void check_rows_range(const Tensor& seq, int64_t width, int64_t T, int64_t B, const char* what) {
  CHECK_HIP_TENSOR(seq);
  TORCH_CHECK(seq.is_contiguous() && seq.scalar_type() == at::kFloat && seq.numel() == T * B * width, what,
              ": contiguous fp32 [T, B, ", width, "]");
}

// xp: [t1 - t0, B, 4H] (bias included, gate-interleaved); hseq / cseq [T, B, H],
// acts [T, B, 4H] written for t in [t0, t1)
void lstm_rows_fwd_range(const Tensor& xp, const Tensor& w, const optional<Tensor>& h0, const optional<Tensor>& c0,
                         const Tensor& hseq, const Tensor& cseq, const Tensor& acts, int64_t t0, int64_t t1,
                         int64_t cell) {
  CHECK_HIP_TENSOR(xp);
  const c10::DeviceGuard guard(xp.device());
  const int64_t H = w.size(1), T = hseq.size(0), B = hseq.size(1);
  TORCH_CHECK(rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, large_dtype(xp)), "row-owning fp32 kernels: H = 128");
  TORCH_CHECK(cell == 0 || cell == 1, "cell: 0 = LSTM, 1 = GRU");
  TORCH_CHECK(0 <= t0 && t0 < t1 && t1 <= T, "time range");
  TORCH_CHECK(w.is_contiguous() && w.size(0) == 4 * H && w.scalar_type() == at::kFloat, "w: [4H, H] fp32");
  check_rows_range(xp, 4 * H, t1 - t0, B, "xp");
  check_rows_range(hseq, H, T, B, "hseq");
  check_rows_range(cseq, H, T, B, "cseq");
  check_rows_range(acts, 4 * H, T, B, "acts");
  if (h0.has_value() && h0->defined()) check_rows_range(*h0, H, 1, B, "h0");
  if (c0.has_value() && c0->defined()) check_rows_range(*c0, H, 1, B, "c0");
  PdrnnLstmLargeStepArgs a{};
  a.B = (int)B; a.H = (int)H; a.T = (int)(t1 - t0); a.cell = (int)cell;
  PdrnnLstmLargeDir& d = a.dir[0];
  float* hs = hseq.data_ptr<float>();
  float* cs = cseq.data_ptr<float>();
  d.w = w.data_ptr<float>();
  d.xp = xp.data_ptr<float>(); d.xp_sb = 4 * H; d.xp_st = B * 4 * H;
  d.h0 = t0 > 0 ? hs + (t0 - 1) * B * H : (h0.has_value() && h0->defined() ? h0->data_ptr<float>() : nullptr);
  d.c0 = t0 > 0 ? cs + (t0 - 1) * B * H : (c0.has_value() && c0->defined() ? c0->data_ptr<float>() : nullptr);
  d.hseq = hs + t0 * B * H; d.hseq_sb = H; d.hseq_st = B * H;
  d.cseq = cs + t0 * B * H;
  d.acts = acts.data_ptr<float>() + t0 * B * 4 * H;
  HIP_LAUNCH_CHECK(pdrnn_lstm_rows_f32(&a, 1, 0, cur_stream()));
}

// Backward of [t0, t1) (run from the last range down): dout [t1 - t0, B, H]
// (any row strides), dhn / dcn the gradients entering step t1 - 1 from above
// (the final-state gradients, or dh / dc written by the range above); writes
// dgates for [t0, t1) and the gradients leaving t0 into dh0 / dc0 [B, H]
// (which may be the dhn / dcn buffers: the first-cell kernel reads them
// before the recurrence overwrites them).  carry: [B, H] scratch.
void lstm_rows_bwd_range(const optional<Tensor>& dout, const optional<Tensor>& dhn, const optional<Tensor>& dcn,
                         const Tensor& wt, const Tensor& cseq, const Tensor& acts, const optional<Tensor>& c0,
                         const Tensor& dgates, const Tensor& dh0, const Tensor& dc0, const Tensor& carry, int64_t t0,
                         int64_t t1, int64_t cell) {
  CHECK_HIP_TENSOR(acts);
  const c10::DeviceGuard guard(acts.device());
  const int64_t H = wt.size(0), T = cseq.size(0), B = cseq.size(1);
  TORCH_CHECK(rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, large_dtype(acts)), "row-owning fp32 kernels: H = 128");
  TORCH_CHECK(cell == 0 || cell == 1, "cell: 0 = LSTM, 1 = GRU");
  TORCH_CHECK(0 <= t0 && t0 < t1 && t1 <= T, "time range");
  TORCH_CHECK(wt.is_contiguous() && wt.size(1) == 4 * H && wt.scalar_type() == at::kFloat, "wt: [H, 4H] fp32");
  check_rows_range(cseq, H, T, B, "cseq");
  check_rows_range(acts, 4 * H, T, B, "acts");
  check_rows_range(dgates, 4 * H, T, B, "dgates");
  check_rows_range(dh0, H, 1, B, "dh0");
  check_rows_range(dc0, H, 1, B, "dc0");
  check_rows_range(carry, H, 1, B, "carry");
  if (dhn.has_value() && dhn->defined()) check_rows_range(*dhn, H, 1, B, "dhn");
  if (dcn.has_value() && dcn->defined()) check_rows_range(*dcn, H, 1, B, "dcn");
  if (c0.has_value() && c0->defined()) check_rows_range(*c0, H, 1, B, "c0");
  const bool has_dout = dout.has_value() && dout->defined();
  if (has_dout) {
    TORCH_CHECK(dout->scalar_type() == at::kFloat && dout->dim() == 3 && dout->size(0) == t1 - t0 &&
                dout->size(1) == B && dout->size(2) == H && dout->stride(2) == 1, "dout [t1 - t0, B, H] fp32");
  }
  PdrnnLstmLargeStepArgs a{};
  a.B = (int)B; a.H = (int)H; a.T = (int)(t1 - t0); a.cell = (int)cell;
  PdrnnLstmLargeDir& d = a.dir[0];
  const float* cs = cseq.data_ptr<float>();
  d.wt = wt.data_ptr<float>();
  d.c0 = t0 > 0 ? cs + (t0 - 1) * B * H : (c0.has_value() && c0->defined() ? c0->data_ptr<float>() : nullptr);
  d.cseq = const_cast<float*>(cs) + t0 * B * H;
  d.acts = acts.data_ptr<float>() + t0 * B * 4 * H;
  d.dgates = dgates.data_ptr<float>() + t0 * B * 4 * H;
  if (has_dout) {
    d.dout = dout->data_ptr<float>(); d.dout_sb = dout->stride(1); d.dout_st = dout->stride(0);
  }
  d.dhn = dhn.has_value() && dhn->defined() ? dhn->data_ptr<float>() : nullptr;
  d.dcn = dcn.has_value() && dcn->defined() ? dcn->data_ptr<float>() : nullptr;
  d.dc_carry = carry.data_ptr<float>();
  d.dh0 = dh0.data_ptr<float>();
  d.dc0 = dc0.data_ptr<float>();
  HIP_LAUNCH_CHECK(pdrnn_lstm_rows_f32(&a, 1, 1, cur_stream()));  // (the first step's cell backward included)
}

// Time-batched GEMM (kernels/gemm.hip).  A: a_kmajor ? [K, M] : [M, K];
// B: b_kmajor ? [K, N] : [N, K] (unit stride along the last dim, any row
// stride); optional second K segment A2 / B2 of the same layouts; output
// fp32 [M, N] (out16: the inputs' dtype, + fp32 bias[N]); `out` is written (or
// accumulated into, fp32) in place when given.
Tensor gemm16(const Tensor& A, bool a_kmajor, const Tensor& B, bool b_kmajor, const optional<Tensor>& A2,
              const optional<Tensor>& B2, const optional<Tensor>& bias, bool out16, const optional<Tensor>& out,
              bool accumulate, int64_t splitk, int64_t variant) {
  CHECK_HIP_TENSOR(A);
  CHECK_HIP_TENSOR(B);
  const c10::DeviceGuard guard(A.device());
  const int dt = dtype_code(A);
  TORCH_CHECK(dtype_code(B) == dt && A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1,
              "gemm16: 2-D 16-bit operands of one dtype with unit inner stride");
  TORCH_CHECK(!accumulate || (out.has_value() && out->defined()),
              "gemm16: accumulate=True needs the output tensor to accumulate into");
  const int64_t M = a_kmajor ? A.size(1) : A.size(0), K = a_kmajor ? A.size(0) : A.size(1);
  const int64_t N = b_kmajor ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == K, "gemm16: K mismatch");
  PdrnnGemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.lda = A.stride(0);
  a.ldb = B.stride(0);
  if (A2.has_value() || B2.has_value()) {
    TORCH_CHECK(A2.has_value() && B2.has_value(), "gemm16: A2 and B2 together");
    const Tensor& a2 = *A2;
    const Tensor& b2 = *B2;
    TORCH_CHECK(dtype_code(a2) == dt && dtype_code(b2) == dt && a2.stride(1) == 1 && b2.stride(1) == 1);
    const int64_t K2 = a_kmajor ? a2.size(0) : a2.size(1);
    TORCH_CHECK((a_kmajor ? a2.size(1) : a2.size(0)) == M && (b_kmajor ? b2.size(1) : b2.size(0)) == N &&
                (b_kmajor ? b2.size(0) : b2.size(1)) == K2, "gemm16: segment-2 shapes");
    a.A2 = a2.data_ptr();
    a.B2 = b2.data_ptr();
    a.lda2 = a2.stride(0);
    a.ldb2 = b2.stride(0);
    a.K2 = (int)K2;
  }
  // the operand DMA issues 16-byte loads from base + row * ld + 8 * chunk:
  // row strides a multiple of 8 elements, 16-byte aligned bases (else the
  // caller's torch fallback, ops/gemm.py:_rowmajor)
  for (const int64_t ld : {a.lda, a.ldb, a.A2 ? a.lda2 : (int64_t)8, a.B2 ? a.ldb2 : (int64_t)8})
    TORCH_CHECK(ld % 8 == 0, "gemm16: row strides must be multiples of 8 elements");
  for (const void* ptr : {a.A, a.B, a.A2, a.B2})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(ptr) % 16 == 0, "gemm16: operand bases must be 16-byte aligned");
  Tensor C;
  if (splitk > 1) {
    // fp32 partials [splitk, M, N], summed in fixed order
    TORCH_CHECK(!out16, "gemm16: split-K gives fp32 partials");
    C = at::empty({splitk, M, N}, A.options().dtype(at::kFloat));
    a.splitk = (int)splitk;
    a.c_split_stride = M * N;
  } else if (out.has_value()) {
    C = *out;
    TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.stride(1) == 1 &&
                (out16 ? C.scalar_type() == A.scalar_type() : C.scalar_type() == at::kFloat), "gemm16: out");
  } else {
    C = at::empty({M, N}, A.options().dtype(out16 ? A.scalar_type() : at::kFloat));
  }
  if (bias.has_value()) {
    TORCH_CHECK(out16 && bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == N,
                "gemm16: fp32 bias[N] with 16-bit output");
    a.bias = bias->data_ptr<float>();
  }
  a.C = C.data_ptr();
  a.ldc = splitk > 1 ? N : C.stride(0);
  a.variant = (int)variant;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.dtype = dt;
  a.a_kmajor = a_kmajor;
  a.b_kmajor = b_kmajor;
  a.c_16bit = out16;
  a.accumulate = splitk > 1 ? 0 : accumulate;
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31) && pdrnn_gemm_supported(&a),
              "gemm16: shape not covered (K % 64, k-major M/N % 8, 16-bit output N % 8)");
  HIP_LAUNCH_CHECK(pdrnn_gemm(&a, cur_stream()));
  if (splitk > 1) {
    // fixed-order sum of the partials (in-tree, deterministic)
    Tensor r = out.has_value() ? *out : at::empty({M, N}, A.options().dtype(at::kFloat));
    TORCH_CHECK(r.is_contiguous(), "gemm16: split-K output must be contiguous");
    HIP_LAUNCH_CHECK(pdrnn_splitk_sum(C.data_ptr<float>(), (int)splitk, M * N, r.data_ptr<float>(),
                                      out.has_value() && accumulate ? 1 : 0, cur_stream()));
    return r;
  }
  return C;
}

int any_dtype(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 2;
  return dtype_code(t);
}

// fp32-product GEMM (kernels/gemm_f32.hip): returns (C, rowsum) -- rowsum [M]
// fp32 = sums over K of op(A) when requested (the bias gradient of dW = G^T X).
std::vector<Tensor> gemm_f32(const Tensor& A, bool a_kmajor, const Tensor& B, bool b_kmajor,
                             const optional<Tensor>& A2, const optional<Tensor>& B2, const optional<Tensor>& bias,
                             bool out16, const optional<Tensor>& out, bool accumulate, int64_t splitk, bool rowsum) {
  CHECK_HIP_TENSOR(A);
  CHECK_HIP_TENSOR(B);
  const c10::DeviceGuard guard(A.device());
  const int dt = any_dtype(A);
  TORCH_CHECK(any_dtype(B) == dt && A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1,
              "gemm_f32: 2-D operands of one dtype with unit inner stride");
  TORCH_CHECK(!accumulate || (out.has_value() && out->defined()),
              "gemm_f32: accumulate=True needs the output tensor to accumulate into");
  const int64_t M = a_kmajor ? A.size(1) : A.size(0), K = a_kmajor ? A.size(0) : A.size(1);
  const int64_t N = b_kmajor ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kmajor ? B.size(0) : B.size(1)) == K, "gemm_f32: K mismatch");
  PdrnnGemmF32Args a{};
  a.A = A.data_ptr(); a.B = B.data_ptr(); a.lda = A.stride(0); a.ldb = B.stride(0);
  if (A2.has_value() || B2.has_value()) {
    TORCH_CHECK(A2.has_value() && B2.has_value(), "gemm_f32: A2 and B2 together");
    const Tensor& a2 = *A2;
    const Tensor& b2 = *B2;
    TORCH_CHECK(any_dtype(a2) == dt && any_dtype(b2) == dt && a2.dim() == 2 && b2.dim() == 2 && a2.stride(1) == 1 &&
                b2.stride(1) == 1, "gemm_f32: segment-2 operands");
    const int64_t K2 = a_kmajor ? a2.size(0) : a2.size(1);
    TORCH_CHECK((a_kmajor ? a2.size(1) : a2.size(0)) == M && (b_kmajor ? b2.size(1) : b2.size(0)) == N &&
                (b_kmajor ? b2.size(0) : b2.size(1)) == K2, "gemm_f32: segment-2 shapes");
    a.A2 = a2.data_ptr(); a.B2 = b2.data_ptr(); a.lda2 = a2.stride(0); a.ldb2 = b2.stride(0); a.K2 = (int)K2;
  }
  bool vec = true;
  for (const int64_t ld : {a.lda, a.ldb, a.A2 ? a.lda2 : (int64_t)4, a.B2 ? a.ldb2 : (int64_t)4}) vec = vec && ld % 4 == 0;
  for (const void* ptr : {a.A, a.B, a.A2, a.B2})
    vec = vec && reinterpret_cast<uintptr_t>(ptr) % (dt == 2 ? 16 : 8) == 0;
  a.vec = vec ? 1 : 0;
  if (splitk < 1) splitk = 1;
  Tensor C;
  if (splitk > 1) {
    TORCH_CHECK(!out16 && !bias.has_value(), "gemm_f32: split-K gives fp32 partials without bias");
    C = at::empty({splitk, M, N}, A.options().dtype(at::kFloat));
    a.c_split_stride = M * N;
  } else if (out.has_value()) {
    C = *out;
    TORCH_CHECK(C.dim() == 2 && C.size(0) == M && C.size(1) == N && C.stride(1) == 1 &&
                (out16 ? C.scalar_type() == A.scalar_type() : C.scalar_type() == at::kFloat), "gemm_f32: out");
  } else {
    C = at::empty({M, N}, A.options().dtype(out16 ? A.scalar_type() : at::kFloat));
  }
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == N,
                "gemm_f32: fp32 bias[N]");
    a.bias = bias->data_ptr<float>();
  }
  Tensor rs;
  if (rowsum) {
    rs = at::empty({splitk, M}, A.options().dtype(at::kFloat));
    a.rowsum = rs.data_ptr<float>();
  }
  a.C = C.data_ptr();
  a.ldc = splitk > 1 ? N : C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.in_dtype = dt;
  a.out_dtype = out16 ? dt : 2;
  TORCH_CHECK(!out16 || dt != 2, "gemm_f32: out16 needs 16-bit inputs");
  a.a_kmajor = a_kmajor; a.b_kmajor = b_kmajor;
  a.accumulate = splitk > 1 ? 0 : accumulate;
  a.splitk = (int)splitk;
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31) && pdrnn_gemm_f32_supported(&a),
              "gemm_f32: configuration not covered");
  hipStream_t st = cur_stream();
  HIP_LAUNCH_CHECK(pdrnn_gemm_f32(&a, st));
  if (splitk > 1) {
    Tensor r = out.has_value() ? *out : at::empty({M, N}, A.options().dtype(at::kFloat));
    TORCH_CHECK(r.is_contiguous(), "gemm_f32: split-K output must be contiguous");
    HIP_LAUNCH_CHECK(pdrnn_splitk_sum(C.data_ptr<float>(), (int)splitk, M * N, r.data_ptr<float>(),
                                      out.has_value() && accumulate ? 1 : 0, st));
    C = r;
  }
  if (rowsum && splitk > 1) {
    Tensor r = at::empty({M}, A.options().dtype(at::kFloat));
    HIP_LAUNCH_CHECK(pdrnn_splitk_sum(rs.data_ptr<float>(), (int)splitk, M, r.data_ptr<float>(), 0, st));
    rs = r;
  } else if (rowsum) {
    rs = rs.view({M});
  }
  return {C, rs};
}

// column sums of a 2-D tensor (fp32 or 16-bit; unit column stride) -> fp32 [cols]
// accumulate_into: add the sums into each of these fp32 [cols] tensors (the
// bias gradients themselves, ops/gradsink.py) instead of returning them
Tensor col_sum(const Tensor& X, const optional<std::vector<Tensor>>& accumulate_into) {
  CHECK_HIP_TENSOR(X);
  const c10::DeviceGuard guard(X.device());
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "col_sum: 2-D tensor with unit column stride");
  const int64_t rows = X.size(0), cols = X.size(1);
  const bool acc = accumulate_into.has_value() && !accumulate_into->empty();
  if (acc)
    for (const auto& o : *accumulate_into)
      TORCH_CHECK(o.scalar_type() == at::kFloat && o.is_contiguous() && o.numel() == cols && o.device() == X.device(),
                  "col_sum: accumulate_into takes fp32 [cols] tensors");
  Tensor out = acc ? (*accumulate_into)[0] : at::empty({cols}, X.options().dtype(at::kFloat));
  if (rows == 0) return acc ? out : out.zero_();
  const int g = pdrnn_col_sum_groups(rows, cols);
  Tensor part = at::empty({g, cols}, X.options().dtype(at::kFloat));
  hipStream_t st = cur_stream();
  HIP_LAUNCH_CHECK(pdrnn_col_sum(X.data_ptr(), any_dtype(X), rows, cols, X.stride(0), part.data_ptr<float>(), g, st));
  if (!acc) {
    HIP_LAUNCH_CHECK(pdrnn_splitk_sum(part.data_ptr<float>(), g, cols, out.data_ptr<float>(), 0, st));
    return out;
  }
  for (const auto& o : *accumulate_into)
    HIP_LAUNCH_CHECK(pdrnn_splitk_sum(part.data_ptr<float>(), g, cols, o.data_ptr<float>(), 1, st));
  return out;
}

// Weight shadows rebuilt in one launch (kernels/shadow_pack.hip; ops/shadow.py):
// jobs are (dst, src, src2 or None) 3-D views of equal shape, bf16 / fp16 /
// fp32 on either side, one device.  Launches ceil(n / 16).
int64_t shadow_pack(const std::vector<std::tuple<Tensor, Tensor, optional<Tensor>>>& jobs) {
  if (jobs.empty()) return 0;
  const c10::DeviceGuard guard(std::get<0>(jobs[0]).device());
  hipStream_t st = cur_stream();
  int64_t launches = 0;
  PdrnnPackBatch b{};
  auto flush = [&]() {
    if (b.njobs == 0) return;
    HIP_LAUNCH_CHECK(pdrnn_shadow_pack(&b, st));
    ++launches;
    b = PdrnnPackBatch{};
  };
  for (const auto& jt : jobs) {
    const Tensor& d = std::get<0>(jt);
    const Tensor& s = std::get<1>(jt);
    const optional<Tensor>& s2 = std::get<2>(jt);
    CHECK_HIP_TENSOR(d);
    CHECK_HIP_TENSOR(s);
    TORCH_CHECK(d.dim() == 3 && s.dim() == 3 && d.sizes() == s.sizes(), "shadow_pack: 3-D views of equal shape");
    auto code = [](const Tensor& t) {
      TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf,
                  "shadow_pack: bf16 / fp16 / fp32 tensors");
      return t.scalar_type() == at::kFloat ? 2 : (t.scalar_type() == at::kBFloat16 ? 0 : 1);
    };
    TORCH_CHECK(d.device() == s.device(), "shadow_pack: source on dst's device");
    PdrnnPackJob& j = b.job[b.njobs];
    j.src = s.data_ptr();
    j.sdtype = code(s);
    j.src2 = nullptr;
    if (s2.has_value() && s2->defined()) {
      TORCH_CHECK(s2->scalar_type() == s.scalar_type() && s2->sizes() == s.sizes() && s2->strides() == s.strides() &&
                      s2->device() == s.device(), "shadow_pack: src2 must match src's dtype, shape and strides");
      j.src2 = s2->data_ptr();
    }
    j.dst = d.data_ptr();
    for (int k = 0; k < 3; ++k) {
      TORCH_CHECK(d.size(k) < (int64_t)1 << 31, "shadow_pack: extent");
      j.n[k] = (int)d.size(k);
      j.ss[k] = s.stride(k);
      j.ds[k] = d.stride(k);
    }
    j.dtype = code(d);
    if (pdrnn_shadow_pack_tiles(&j) == 0) continue;
    if (++b.njobs == PDRNN_PACK_MAX_JOBS) flush();
  }
  flush();
  return launches;
}

// C[M, N] f32 = A[M, K] Bt[N, K]^T on the MFMA core (tests).
Tensor gemm_nt(const Tensor& A, const Tensor& Bt, int64_t tile) {
  CHECK_HIP_TENSOR(A);
  const c10::DeviceGuard guard(A.device());
  const int dt = large_dtype(A);
  TORCH_CHECK(A.is_contiguous() && Bt.is_contiguous() && A.size(1) == Bt.size(1) && large_dtype(Bt) == dt);
  const int64_t M = A.size(0), K = A.size(1), N = Bt.size(0);
  Tensor C = at::empty({M, N}, A.options().dtype(at::kFloat));
  HIP_LAUNCH_CHECK(pdrnn_gemm_nt(eptr(A), K, eptr(Bt), K, C.data_ptr<float>(), N, (int)M, (int)N, (int)K, dt,
                                 (int)tile, cur_stream()));
  return C;
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "pytorch_distributed_rnn_amd native runtime (gfx950 HIP kernels + RCCL runtime)";
  m.def("lstm_small_fwd", &lstm_small_fwd, "fused small-H LSTM / GRU stack forward", py::arg("x"), py::arg("idx"),
        py::arg("w"), py::arg("h0"), py::arg("c0"), py::arg("H"), py::arg("NL"), py::arg("batch_first"),
        py::arg("save"), py::arg("need_out"), py::arg("nb"), py::arg("split"), py::arg("cell") = 0);
  m.def("lstm_small_bwd", &lstm_small_bwd, "fused small-H LSTM / GRU stack BPTT backward", py::arg("x"),
        py::arg("idx"), py::arg("w"), py::arg("h0"), py::arg("c0"), py::arg("hseq"), py::arg("act"), py::arg("dout"),
        py::arg("dhn"), py::arg("dcn"), py::arg("H"), py::arg("NL"), py::arg("batch_first"), py::arg("need_dx"),
        py::arg("need_dh0"), py::arg("nb"), py::arg("split"), py::arg("grad_accum"), py::arg("cell") = 0);
  m.def("lstm_small_max_split", [](int64_t H, int64_t NL, bool backward) {
    return pdrnn_lstm_small_max_split((int)H, (int)NL, backward ? 1 : 0);
  });
  m.def("lstm_small_step_one_launch", [](int64_t H, int64_t NL, int64_t T, int64_t B, int64_t nb_fwd,
                                         int64_t split_fwd, int64_t nb_bwd, int64_t split_bwd) {
    if (split_fwd <= 0) split_fwd = pdrnn_lstm_small_max_split((int)H, (int)NL, 0);
    if (split_bwd <= 0) split_bwd = pdrnn_lstm_small_max_split((int)H, (int)NL, 1);
    if (nb_fwd <= 0) nb_fwd = 1;
    if (nb_bwd <= 0) nb_bwd = 1;
    const int gridb = pdrnn_lstm_small_bwd_grid((int)H, (int)NL, (int)T, (int)B, (int)nb_bwd, (int)split_bwd);
    return pdrnn_lstm_small_step_ok((int)H, (int)NL, (int)B, (int)nb_fwd, (int)split_fwd, (int)nb_bwd,
                                    (int)split_bwd, gridb) != 0;
  }, "the fused training step runs forward + head/CE + BPTT as one launch for this shape");
  m.def("lstm_small_step_deferred_dw", [](int64_t H, int64_t NL, int64_t T, int64_t B) {
    // the fused step's default single-sequence backward (nb = 1, unit-group map)
    const int split_bwd = pdrnn_lstm_small_max_split((int)H, (int)NL, 1);
    const int gridb = pdrnn_lstm_small_bwd_grid((int)H, (int)NL, (int)T, (int)B, 1, split_bwd);
    const int mode = pdrnn_lstm_small_dwout_ok((int)H, (int)NL, (int)T);
    return split_bwd == 1 && ((gridb < B && mode == 1) || mode == 2);
  }, "the fused training step defers the weight gradients to the matrix-core dW kernel for this shape");
  m.def("lstm_small_dwout_geometry", [](int64_t H, int64_t NL, int64_t T, int64_t B) {
    const int nb = pdrnn_lstm_small_bwd_dwout_nb((int)H, (int)NL, (int)T, (int)B);
    return py::make_tuple(nb, pdrnn_lstm_small_bwd_dwout_grid((int)H, (int)NL, (int)T, (int)B, nb));
  }, "(sequences per workgroup, grid) of the deferred-dW backward for this shape");
  m.def("lstm_sw_ok", [](int64_t H, int64_t I, int64_t NL, int64_t cell) {
    return pdrnn_lstm_sw_ok((int)H, (int)I, (int)NL, (int)cell) == 1;
  }, "the sequence-in-wave kernels (lstm_sw.hip) cover this LSTM (cell 0) / GRU (cell 1) stack in the fused train step",
        py::arg("H"), py::arg("I"), py::arg("NL"), py::arg("cell") = 0);
  m.def("lstm_sw_step_ok", [](int64_t NL, int64_t B, int64_t T) {
    return pdrnn_lstm_sw_step_ok((int)NL, (int)B, (int)T) == 1;
  }, "the one-launch sequence-in-wave step (forward + BPTT in one kernel) covers this batch");
  m.def("lstm_sw_fits", [](int64_t NL, int64_t B, int64_t T) { return pdrnn_lstm_sw_fits((int)NL, (int)B, (int)T) == 1; },
        "every act / hseq row of this batch fits the sequence-in-wave kernels' 2 GiB buffer descriptor");
  m.def("lstm_sw_mode", [](int64_t NL, int64_t B, bool backward) { return pdrnn_lstm_sw_mode((int)NL, (int)B, backward ? 1 : 0); },
        "wave map of the sequence-in-wave kernels for B sequences (0/1: a wave per 1/2 sequences, 2/3: a wave "
        "per layer of 1/2 sequences, 6: mode 2 at three waves per SIMD, forward only)",
        py::arg("NL"), py::arg("B"), py::arg("backward") = false);
  m.def("lstm_small_supported", [](int64_t H, int64_t I, int64_t NL) {
    return pdrnn_lstm_small_supported((int)H, (int)I, (int)NL) != 0;
  });
  m.def("lstm_head_train_step", &lstm_head_train_step, "fused LSTM + head + CE forward/backward -> flat grads",
        py::arg("x"), py::arg("idx"), py::arg("labels"), py::arg("w"), py::arg("head_w"), py::arg("head_b"),
        py::arg("flat_grad"), py::arg("stats"), py::arg("H"), py::arg("NL"), py::arg("split_fwd"),
        py::arg("split_bwd"), py::arg("nb_fwd"), py::arg("nb_bwd"), py::arg("adam_state") = py::none(),
        py::arg("adam_hp") = py::none(), py::arg("cell") = 0, py::arg("grad_colmap") = py::none(),
        py::arg("stats_slot_step") = py::none(), py::arg("stats_slot_offset") = 0, py::arg("round_bf16") = false,
        py::arg("adam_ticket") = py::none());
  m.def("gemm_f32", &gemm_f32, "fp32-product MFMA GEMM: (C, rowsum of op(A) over K)", py::arg("A"),
        py::arg("a_kmajor"), py::arg("B"), py::arg("b_kmajor"), py::arg("A2") = py::none(), py::arg("B2") = py::none(),
        py::arg("bias") = py::none(), py::arg("out16") = false, py::arg("out") = py::none(),
        py::arg("accumulate") = false, py::arg("splitk") = 1, py::arg("rowsum") = false);
  m.def("shadow_pack", &shadow_pack,
        "rebuild weight shadows: (dst, src, src2|None) 3-D views, fp32 sources, one launch per 16 jobs",
        py::arg("jobs"));
  m.def("col_sum", &col_sum, "deterministic fp32 column sums of a 2-D tensor (or added into accumulate_into)",
        py::arg("X"), py::arg("accumulate_into") = py::none());
  m.def("gemm_variants", []() {
    int v[8];
    const int n = pdrnn_gemm_variants(v, 8);
    return std::vector<int>(v, v + n);
  }, "schedule variants of the in-tree GEMM compiled into this build (first = default)");
  m.def("xent_fwd", &xent_fwd, "fused softmax cross-entropy + accuracy");
  m.def("xent_bwd", &xent_bwd, "cross-entropy backward (gradient in out_dtype, fp32 by default)",
        py::arg("dlogits"), py::arg("grad_out"), py::arg("stats"), py::arg("out_dtype") = py::none());
  m.def("adam_flat", &adam_flat, "fused Adam/AdamW step over a flat buffer", py::arg("param"), py::arg("grad"),
        py::arg("exp_avg"), py::arg("exp_avg_sq"), py::arg("max_exp_avg_sq"), py::arg("lr"), py::arg("beta1"),
        py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("step"), py::arg("grad_scale"),
        py::arg("decoupled"), py::arg("maximize"), py::arg("lr_t") = py::none(), py::arg("step_t") = py::none(),
        py::arg("ticket") = py::none(), py::arg("skip") = py::none());
  m.def("lstm_large_fwd", &lstm_large_fwd, "large-H LSTM layer forward (MFMA step kernels, both directions)");
  m.def("rccl_max_ctas", []() { return pdrnn::rccl_max_ctas(); },
        "workgroup cap of the native RCCL communicators' kernels (PDRNN_RCCL_MAX_CTAS)");
  m.def("rccl_cta_reserve", []() { return pdrnn::rccl_cta_reserve(); },
        "CUs a persistent recurrence leaves free for RCCL in this process");
  m.def("lstm_large_bwd_persistent",
        [](int64_t B, int64_t H, int64_t ndir, int64_t dtype, int64_t tile) {
          // the backward recurrence lstm_large_bwd would run as one grid-synced
          // persistent launch (dtype 0 bf16, 1 fp16, 2 fp32): such a launch must
          // not share the GPU with side-stream GEMMs (ops/lstm_large.py run_recurrence)
          if (tile < 0 && dtype == 2 && rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, 2)) return false;
          return large_persist_plan((int)B, (int)H, (int)ndir, true, (int)dtype, tile) != 0;
        },
        "1 when lstm_large_bwd's recurrence would take the grid-synced persistent path");
  m.def("lstm_large_bwd", &lstm_large_bwd, "large-H LSTM layer BPTT (MFMA step kernels) -> dgates, dh0, dc0");
  m.def("lstm_large_supported", [](int64_t H) { return pdrnn_lstm_large_supported((int)H) != 0; });
  m.def("lstm_rows_range_supported", [](int64_t H) { return rows_f32_on() && pdrnn_lstm_rows_f32_supported((int)H, 2) != 0; });
  m.def("lstm_rows_fwd_range", &lstm_rows_fwd_range, "row-owning fp32 recurrence over steps [t0, t1) (preallocated outputs)");
  m.def("lstm_rows_bwd_range", &lstm_rows_bwd_range, "row-owning fp32 BPTT over steps [t0, t1), last range first");
  m.def("set_persist_verify", [](int mode) { g_persist_verify = mode; },
        "0 off; 1 synchronise after every persistent-recurrence launch and re-run a timed-out layer on the "
        "per-step kernels; 2 per step: persist_step_check() before the optimizer update re-runs the step");
  m.def("persist_verify_mode", []() { return persist_verify_mode(); });
  m.def("clip_flat", &clip_flat, "in-place gradient-norm clipping of a flat fp32 gradient -> [scale, norm]",
        py::arg("g"), py::arg("max_norm"), py::arg("eps") = 1e-6);
  m.def("persist_sticky_flag", &persist_sticky_flag,
        "the current device's sticky persistent-timeout flag (device int32 [1])");
  m.def("persist_step_check", &persist_step_check,
        "per-step verification: True when a persistent launch timed out since the last check (synchronises)");
  m.def("persist_inject_timeouts", [](int64_t n) { g_persist_inject = (int)n; },
        "tests: flag the next n persistent launches as timed out");
  m.def("persist_tagx_launches", []() { return (int64_t)g_persist_tagx.load(); },
        "persistent forward launches that used the tagged h exchange (PDRNN_TUNE persist_tagx)");
  m.def("persist_fallbacks", []() { return (int64_t)g_persist_fallbacks.load(); },
        "persistent launches re-run on the per-step kernels after a timeout");
  m.def("persist_verify_on", []() { return persist_verify_mode() != 0; },
        "persistent launches are verified (per launch or per step) before the optimizer uses their results");
  m.def("persist_disabled", []() { return g_persist_disabled.load() != 0; },
        "the persistent recurrence is off for this process (after a timed-out launch)");
  m.def("persist_disable", []() { g_persist_disabled = 1; },
        "turn the persistent recurrence off for this process (a job-wide re-run after a timeout)");
  m.def("persist_reset", []() { g_persist_disabled = 0; g_persist_fallbacks = 0; },
        "tests: re-enable the persistent recurrence and clear the fallback count");
  m.def("debug_spin_cus", [](double ms, int64_t workgroups, int64_t threads, int64_t lds_bytes) {
    HIP_LAUNCH_CHECK(pdrnn_debug_spin_cus((uint64_t)(ms * 1e3), (int)workgroups, (int)threads, (int)lds_bytes,
                                          cur_stream()));
  }, "diagnostics: fill CUs with bounded spinning workgroups on the current stream");
  m.def("persist_check", &persist_check, "raise if a persistent launch on this device timed out (synchronises)");
  m.def("lstm_large_persist_mt", [](int64_t B, int64_t H, int64_t ndir, int64_t dtype) {
    int dev = 0, cus = 0;
    TORCH_CHECK(hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess);
    return pdrnn_lstm_large_persist_mt((int)B, (int)H, (int)ndir, (int)dtype, cus - pdrnn::rccl_cta_reserve());
  }, "persistent large-H recurrence: rows-per-workgroup / 16 for this shape on the current device (0 = not covered)");
  m.def("gemm_nt", &gemm_nt, "C = A Bt^T (bf16/fp16 in, f32 out) on the MFMA tile core", py::arg("A"),
        py::arg("Bt"), py::arg("tile") = -1);
  m.def("gemm16", &gemm16, "time-batched MFMA GEMM (kernels/gemm.hip): C = op(A) op(B) [+ A2 B2] [+ bias]",
        py::arg("A"), py::arg("a_kmajor"), py::arg("B"), py::arg("b_kmajor"), py::arg("A2") = py::none(),
        py::arg("B2") = py::none(), py::arg("bias") = py::none(), py::arg("out16") = false,
        py::arg("out") = py::none(), py::arg("accumulate") = false, py::arg("splitk") = 1,
        py::arg("variant") = 0);
  m.def("gemm16_supported", [](int64_t M, int64_t N, int64_t K, int64_t K2, bool akm, bool bkm, bool out16) {
    PdrnnGemmArgs a{};
    a.M = (int)M; a.N = (int)N; a.K = (int)K; a.K2 = (int)K2; a.a_kmajor = akm; a.b_kmajor = bkm;
    a.c_16bit = out16; a.ldc = N; a.A2 = a.B2 = K2 ? (const void*)1 : nullptr;
    return M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31) && pdrnn_gemm_supported(&a) != 0;
  });
  m.def("large_persist_mt", [](int64_t B, int64_t H, int64_t ndir, int64_t dtype, int64_t cus) {
    return g_persist_disabled.load() ? 0 : pdrnn_lstm_large_persist_mt((int)B, (int)H, (int)ndir, (int)dtype, (int)cus);
  }, "row tiles of the persistent recurrence for a grid of at most `cus` workgroups (0: not covered / turned off)");
  m.def("embedding_fwd", &embedding_fwd, py::arg("weight"), py::arg("idx"), py::arg("out_dtype") = py::none());
  m.def("embedding_sort", [](const Tensor& idx, int64_t V) {
    CHECK_HIP_TENSOR(idx);
    const c10::DeviceGuard guard(idx.device());
    Tensor flat = idx.contiguous().view({-1}).to(at::kLong);
    Tensor perm = at::empty({flat.numel()}, flat.options()), offsets = at::empty({V + 1}, flat.options());
    Tensor scratch = at::empty({std::max<int64_t>(pdrnn_embedding_sort_scratch(flat.numel(), V), 1)},
                               flat.options().dtype(at::kInt));
    HIP_LAUNCH_CHECK(pdrnn_embedding_sort(flat.data_ptr<int64_t>(), flat.numel(), V, scratch.data_ptr<int>(),
                                          perm.data_ptr<int64_t>(), offsets.data_ptr<int64_t>(), cur_stream()));
    return py::make_tuple(perm, offsets);
  }, "stable in-tree counting sort of indices by row (V <= 16384): (perm, row offsets)");
  m.def("embedding_bwd", &embedding_bwd, py::arg("dout"), py::arg("idx"), py::arg("num_embeddings"),
        py::arg("padding_idx"), py::arg("out") = py::none());
  m.attr("offload_arch") = "gfx950";
  pdrnn::register_runtime(m);
}
