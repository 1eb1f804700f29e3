// Gradient synchronisation engines + pybind registration of the runtime.
//
// GradReducer   -- replaces the C++ DDP Reducer of torch 1.4 that the reference
//                  gets from DistributedDataParallel (reference:
//                  src/motion/trainer/ddp.py:19).
//   * parameters are packed, in REVERSE registration order (the order BPTT
//     produces their gradients), into flat per-dtype buckets capped at
//     `bucket_cap_bytes`; every param.grad is a view into its bucket, so the
//     autograd engine / fused backward kernels accumulate straight into the
//     communication buffer (no pack copy),
//   * a bucket is launched as ONE all-reduce as soon as all of its params are
//     ready, strictly in bucket order (identical collective order on every
//     rank), on the communicator's own stream -> it overlaps the backward
//     kernels of the layers below,
//   * finalize() (queued at the end of backward) launches the stragglers and
//     makes the compute stream wait; averaging is done on the wire (ncclAvg)
//     or by one scale per bucket.
// FusionReducer -- replaces Horovod's tensor-fusion all-reduce that the
//                  reference uses through hvd.DistributedOptimizer (reference:
//                  src/motion/trainer/horovod.py:33-35):
//   per-tensor readiness from optimizer-side hooks, ready tensors are copied
//   (in canonical order) into a fusion buffer of `fusion_bytes`, one all-reduce
//   per full buffer, results copied back at synchronize().
#include <algorithm>
#include <map>

#include "pdrnn/runtime.h"

namespace pdrnn {
namespace py = pybind11;

class GradReducer {
 public:
  // flat_grad (optional): an existing flat gradient buffer in which the
  // params' gradients are laid out back to back in registration order (see
  // utils/flat.py).  Buckets then are plain slices of it -- zero copies.
  // groups (optional, one id per param): a bucket never spans two groups --
  // the DDP wrapper gives every (RNN layer, direction) its own id, so a
  // layer's buckets launch as soon as that layer's weight gradients exist
  // instead of waiting for the first parameters of the layer below.
  // A parameter larger than the cap is split into ceil(bytes / cap) equal
  // sub-tensor buckets (narrow views of its gradient, 4 KiB-aligned): a
  // 512 MiB bi-LSTM weight becomes 16 all-reduces of 32 MiB that pipeline on
  // the ring instead of one message whose first byte waits for the last.
  GradReducer(std::vector<at::Tensor> params, std::shared_ptr<Comm> comm, int64_t bucket_cap_bytes,
              int64_t first_bucket_cap_bytes, bool average, c10::optional<at::Tensor> flat_grad,
              std::vector<int64_t> groups = {})
      : params_(std::move(params)), comm_(std::move(comm)), average_(average) {
    TORCH_CHECK(groups.empty() || groups.size() == params_.size(), "groups: one id per parameter");
    const bool use_flat = flat_grad.has_value() && flat_grad->defined();
    std::vector<int64_t> flat_off;
    if (use_flat) {
      int64_t off = 0;
      for (const auto& p : params_) {
        TORCH_CHECK(p.scalar_type() == flat_grad->scalar_type() && p.device() == flat_grad->device(),
                    "flat_grad dtype/device must match every parameter");
        flat_off.push_back(off);
        off += p.numel();
      }
      TORCH_CHECK(off == flat_grad->numel() && flat_grad->is_contiguous(), "flat_grad size mismatch");
      flat_ = *flat_grad;
    }
    const int64_t n = (int64_t)params_.size();
    // Reverse order bucketing, split on dtype/device/group change or cap.
    // chunk_[b] = (offset, length) in elements when bucket b is a slice of one
    // oversized parameter, (-1, 0) for a bucket of whole parameters.
    std::vector<int64_t> cur;
    int64_t cur_bytes = 0;
    at::ScalarType cur_dtype = at::kFloat;
    c10::Device cur_dev = at::kCPU;
    int64_t cur_group = 0;
    auto close = [&]() {
      if (cur.empty()) return;
      buckets_idx_.push_back(cur);
      chunk_.push_back({-1, 0});
      cur.clear();
      cur_bytes = 0;
    };
    for (int64_t i = n - 1; i >= 0; --i) {
      const auto& p = params_[i];
      const int64_t cap = std::max<int64_t>(buckets_idx_.empty() ? first_bucket_cap_bytes : bucket_cap_bytes, 1);
      const int64_t bytes = p.numel() * p.element_size();
      const int64_t grp = groups.empty() ? 0 : groups[i];
      // a parameter is split by the regular cap, never by the (smaller)
      // first-bucket cap: a large weight right behind the small head bias
      // would otherwise become ceil(bytes / 1 MiB) latency-bound messages
      const int64_t split_cap = std::max<int64_t>(bucket_cap_bytes, 1);
      if (bytes > split_cap && p.numel() > 1) {
        close();
        // equal chunks rounded up to 4 KiB, issued from the parameter's end
        const int64_t k = (bytes + split_cap - 1) / split_cap;
        const int64_t align = std::max<int64_t>(4096 / p.element_size(), 1);
        const int64_t len = ((p.numel() + k - 1) / k + align - 1) / align * align;
        for (int64_t c = (p.numel() + len - 1) / len - 1; c >= 0; --c) {
          buckets_idx_.push_back({i});
          chunk_.push_back({c * len, std::min(len, p.numel() - c * len)});
        }
        cur_dtype = p.scalar_type(); cur_dev = p.device(); cur_group = grp;
        continue;
      }
      if (!cur.empty() && (p.scalar_type() != cur_dtype || p.device() != cur_dev || grp != cur_group ||
                           cur_bytes + bytes > cap))
        close();
      if (cur.empty()) { cur_dtype = p.scalar_type(); cur_dev = p.device(); cur_group = grp; }
      cur.push_back(i);
      cur_bytes += bytes;
    }
    close();
    views_.resize(n);
    param_buckets_.assign(n, {});
    std::map<int64_t, at::Tensor> own;  // non-flat: the gradient buffer of a split parameter
    for (size_t b = 0; b < buckets_idx_.size(); ++b) {
      for (int64_t i : buckets_idx_[b]) param_buckets_[i].push_back((int64_t)b);
      if (chunk_[b].first >= 0) {
        const int64_t i = buckets_idx_[b][0];
        const auto& p = params_[i];
        if (use_flat) {
          buckets_.push_back(flat_grad->narrow(0, flat_off[i] + chunk_[b].first, chunk_[b].second));
          views_[i] = flat_grad->narrow(0, flat_off[i], p.numel()).view(p.sizes());
        } else {
          auto it = own.find(i);
          if (it == own.end())
            it = own.emplace(i, at::zeros({p.numel()}, p.options().requires_grad(false))).first;
          buckets_.push_back(it->second.narrow(0, chunk_[b].first, chunk_[b].second));
          views_[i] = it->second.view(p.sizes());
        }
        continue;
      }
      int64_t total = 0;
      for (int64_t i : buckets_idx_[b]) total += params_[i].numel();
      if (use_flat) {
        // reverse-ordered bucket = descending contiguous index range
        const int64_t lo = buckets_idx_[b].back();
        const int64_t start = flat_off[lo];
        buckets_.push_back(flat_grad->narrow(0, start, total));
        for (int64_t i : buckets_idx_[b])
          views_[i] = buckets_[b].narrow(0, flat_off[i] - start, params_[i].numel()).view(params_[i].sizes());
      } else {
        auto flat = at::zeros({total}, params_[buckets_idx_[b][0]].options().requires_grad(false));
        int64_t off = 0;
        for (int64_t i : buckets_idx_[b]) {
          views_[i] = flat.narrow(0, off, params_[i].numel()).view(params_[i].sizes());
          off += params_[i].numel();
        }
        buckets_.push_back(flat);
      }
    }
    pending_.resize(buckets_.size());
    ready_.assign(n, 0);
    reset();
  }

  const std::vector<at::Tensor>& grad_views() const { return views_; }
  const std::vector<at::Tensor>& buckets() const { return buckets_; }
  const std::vector<std::vector<int64_t>>& bucket_indices() const { return buckets_idx_; }
  const std::vector<std::pair<int64_t, int64_t>>& bucket_chunks() const { return chunk_; }

  void reset() {
    for (size_t b = 0; b < buckets_.size(); ++b) pending_[b] = (int64_t)buckets_idx_[b].size();
    std::fill(ready_.begin(), ready_.end(), 0);
    next_ = 0;
    launched_ = 0;
  }

  // Returns true when the caller must re-point param.grad to grad_views()[i]
  // (the autograd engine produced a fresh tensor, which was copied in).
  bool mark_ready(int64_t i, const at::Tensor& grad) {
    TORCH_CHECK(i >= 0 && i < (int64_t)params_.size(), "bad parameter index");
    bool repoint = false;
    if (grad.defined() && grad.data_ptr() != views_[i].data_ptr()) {
      views_[i].copy_(grad);
      repoint = true;
    }
    if (ready_[i]) return repoint;  // grad accumulated twice in one backward (shared weight)
    ready_[i] = 1;
    for (int64_t b : param_buckets_[i]) --pending_[b];
    launch_ready();
    return repoint;
  }

  void finalize() {
    // Params that received no gradient this iteration contribute zeros.
    for (size_t i = 0; i < params_.size(); ++i) {
      if (ready_[i]) continue;
      ready_[i] = 1;
      for (int64_t b : param_buckets_[i]) --pending_[b];
    }
    launch_ready();
    comm_->wait();
    if (average_ && !comm_->native_avg() && comm_->world() > 1) {
      for (auto& f : buckets_) f.div_((double)comm_->world());
    }
    reset();
  }

  void zero_() {
    for (auto& f : buckets_) f.zero_();
  }

  // Synchronous all-reduce of every bucket (used by no-hook fallbacks / tests).
  void all_reduce_now() {
    for (size_t b = 0; b < buckets_.size(); ++b) comm_->all_reduce(buckets_[b], op());
    comm_->wait();
    if (average_ && !comm_->native_avg() && comm_->world() > 1)
      for (auto& f : buckets_) f.div_((double)comm_->world());
  }

  // Same, each bucket reduced straight on the caller's stream (nothing to
  // overlap: the fused motion step produces every gradient in one kernel).
  // The fused step's sync: the whole gradient is ready at once (after the
  // BPTT), so over a flat gradient it is ONE collective -- the per-bucket
  // split only serves the hook path that overlaps the backward, and at the
  // 8-GPU per-rank batch each extra call is a latency-bound RCCL launch.
  void all_reduce_inline() {
    if (flat_.defined()) {
      comm_->all_reduce_inline(flat_, op());
      if (average_ && !comm_->native_avg() && comm_->world() > 1) flat_.div_((double)comm_->world());
      return;
    }
    for (size_t b = 0; b < buckets_.size(); ++b) comm_->all_reduce_inline(buckets_[b], op());
    if (average_ && !comm_->native_avg() && comm_->world() > 1)
      for (auto& f : buckets_) f.div_((double)comm_->world());
  }

  int64_t launched() const { return launched_; }

 private:
  RedOp op() const { return (average_ && comm_->native_avg()) ? RedOp::kAvg : RedOp::kSum; }
  void launch_ready() {
    while (next_ < (int64_t)buckets_.size() && pending_[next_] == 0) {
      comm_->all_reduce(buckets_[next_], op());
      ++next_;
      ++launched_;
    }
  }

  std::vector<at::Tensor> params_;
  std::shared_ptr<Comm> comm_;
  bool average_;
  at::Tensor flat_;  // the flat gradient every bucket views (undefined without one)
  std::vector<std::vector<int64_t>> buckets_idx_;
  std::vector<at::Tensor> buckets_;
  std::vector<at::Tensor> views_;
  std::vector<std::pair<int64_t, int64_t>> chunk_;     // per bucket: (offset, length) of a split parameter
  std::vector<std::vector<int64_t>> param_buckets_;    // per parameter: the buckets it feeds
  std::vector<int64_t> pending_;
  std::vector<char> ready_;
  int64_t next_ = 0;
  int64_t launched_ = 0;
};

class FusionReducer {
 public:
  FusionReducer(std::shared_ptr<Comm> comm, int64_t fusion_bytes, bool average)
      : comm_(std::move(comm)), fusion_bytes_(std::max<int64_t>(fusion_bytes, 1024)), average_(average) {}

  // Register a tensor slot in canonical order; returns its handle.
  int64_t register_tensor(const std::string& name, const at::Tensor& like) {
    names_.push_back(name);
    entries_.push_back({at::Tensor(), false});
    (void)like;
    return (int64_t)names_.size() - 1;
  }

  // A gradient is ready: remember it; pack every ready tensor at the head of
  // the canonical order into the fusion buffer, all-reducing full buffers.
  void enqueue(int64_t h, const at::Tensor& grad) {
    TORCH_CHECK(h >= 0 && h < (int64_t)entries_.size(), "bad handle");
    entries_[h] = {grad, true};
    advance(false);
  }

  // Flush everything (missing tensors are skipped consistently: a rank only
  // skips what every rank skips when the model is identical), wait, unpack.
  void synchronize() {
    advance(true);
    flush();
    comm_->wait();
    for (auto& f : inflight_) unpack(f);
    inflight_.clear();
    for (auto& e : entries_) e = {at::Tensor(), false};
    cursor_ = 0;
  }

  int64_t collectives() const { return collectives_; }
  int64_t num_registered() const { return (int64_t)names_.size(); }

 private:
  struct Fused {
    at::Tensor buf;
    std::vector<std::pair<at::Tensor, int64_t>> members;  // (grad, offset)
  };
  RedOp op() const { return (average_ && comm_->native_avg()) ? RedOp::kAvg : RedOp::kSum; }

  void advance(bool final_pass) {
    while (cursor_ < (int64_t)entries_.size()) {
      auto& e = entries_[cursor_];
      if (!e.second) {
        if (!final_pass) return;
        ++cursor_;
        continue;
      }
      const at::Tensor& g = e.first;
      const int64_t bytes = g.numel() * g.element_size();
      if (!cur_.members.empty() &&
          (cur_used_ * cur_esize_ + bytes > fusion_bytes_ || g.scalar_type() != cur_dtype_ || g.device() != cur_dev_))
        flush();
      if (cur_.members.empty()) {
        cur_dtype_ = g.scalar_type();
        cur_dev_ = g.device();
        cur_esize_ = g.element_size();
        const int64_t cap = std::max<int64_t>(fusion_bytes_ / cur_esize_, g.numel());
        cur_.buf = at::empty({cap}, g.options());
        cur_used_ = 0;
      }
      cur_.buf.narrow(0, cur_used_, g.numel()).copy_(g.reshape({-1}));
      cur_.members.push_back({g, cur_used_});
      cur_used_ += g.numel();
      ++cursor_;
    }
  }

  void flush() {
    if (cur_.members.empty()) return;
    auto view = cur_.buf.narrow(0, 0, cur_used_);
    comm_->all_reduce(view, op());
    ++collectives_;
    inflight_.push_back(std::move(cur_));
    cur_ = Fused();
    cur_used_ = 0;
  }

  void unpack(Fused& f) {
    const bool div = average_ && !comm_->native_avg() && comm_->world() > 1;
    for (auto& m : f.members) {
      auto src = f.buf.narrow(0, m.second, m.first.numel()).view(m.first.sizes());
      if (div) m.first.copy_(src / (double)comm_->world());
      else m.first.copy_(src);
    }
  }

  std::shared_ptr<Comm> comm_;
  int64_t fusion_bytes_;
  bool average_;
  std::vector<std::string> names_;
  std::vector<std::pair<at::Tensor, bool>> entries_;
  int64_t cursor_ = 0;
  Fused cur_;
  int64_t cur_used_ = 0;
  int64_t cur_esize_ = 4;
  at::ScalarType cur_dtype_ = at::kFloat;
  c10::Device cur_dev_ = at::kCPU;
  std::vector<Fused> inflight_;
  int64_t collectives_ = 0;
};

static RedOp parse_op(const std::string& s) {
  if (s == "sum") return RedOp::kSum;
  if (s == "avg" || s == "mean") return RedOp::kAvg;
  if (s == "max") return RedOp::kMax;
  if (s == "min") return RedOp::kMin;
  TORCH_CHECK(false, "unknown reduce op ", s);
}

void register_runtime(py::module_& m) {
  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("native_avg", &Comm::native_avg)
      .def("all_reduce", [](Comm& c, at::Tensor t, const std::string& op) { c.all_reduce(t, parse_op(op)); },
           py::arg("tensor"), py::arg("op") = "sum")
      .def("broadcast", [](Comm& c, at::Tensor t, int root) { c.broadcast(t, root); })
      .def("all_gather", [](Comm& c, at::Tensor out, const at::Tensor& in) { c.all_gather(out, in); })
      .def("reduce_scatter", [](Comm& c, at::Tensor out, const at::Tensor& in, const std::string& op) {
             c.reduce_scatter(out, in, parse_op(op));
           }, py::arg("out"), py::arg("input"), py::arg("op") = "sum")
      .def("all_to_all", [](Comm& c, at::Tensor out, const at::Tensor& in) { c.all_to_all(out, in); })
      .def("send", &Comm::send)
      .def("recv", [](Comm& c, at::Tensor t, int peer) { c.recv(t, peer); })
      .def("all_reduce_inline", [](Comm& c, at::Tensor t, const std::string& op) { c.all_reduce_inline(t, parse_op(op)); },
           py::arg("tensor"), py::arg("op") = "sum")
      .def("wait", &Comm::wait)
      .def("barrier", &Comm::barrier)
      .def("debug_stall", &Comm::debug_stall, py::arg("seconds"))
      .def_property_readonly("aborted", &Comm::aborted)
      .def_property_readonly("timeout_s", &Comm::timeout_s)
      .def_property_readonly("tracked", &Comm::tracked)
      .def("track_current", &Comm::track_current)
      .def("close", &Comm::close, py::call_guard<py::gil_scoped_release>());
  m.attr("WATCHDOG_EXIT") = kWatchdogExit;
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("make_rccl_comm", [](py::bytes uid, int rank, int world, int device, bool high_priority, double timeout_s) {
    return make_rccl_comm(std::string(uid), rank, world, device, high_priority, timeout_s);
  }, py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("high_priority") = true,
     py::arg("timeout_s") = 600.0);
  m.def("make_pg_comm", &make_pg_comm, py::arg("process_group"));

  py::class_<GradReducer, std::shared_ptr<GradReducer>>(m, "GradReducer")
      .def(py::init<std::vector<at::Tensor>, std::shared_ptr<Comm>, int64_t, int64_t, bool, c10::optional<at::Tensor>,
                    std::vector<int64_t>>(),
           py::arg("params"), py::arg("comm"), py::arg("bucket_cap_bytes"), py::arg("first_bucket_cap_bytes"),
           py::arg("average") = true, py::arg("flat_grad") = py::none(), py::arg("groups") = std::vector<int64_t>{})
      .def("grad_views", &GradReducer::grad_views)
      .def("buckets", &GradReducer::buckets)
      .def("bucket_indices", &GradReducer::bucket_indices)
      .def("bucket_chunks", &GradReducer::bucket_chunks)
      .def("mark_ready", &GradReducer::mark_ready)
      .def("finalize", &GradReducer::finalize)
      .def("reset", &GradReducer::reset)
      .def("zero_", &GradReducer::zero_)
      .def("all_reduce_now", &GradReducer::all_reduce_now)
      .def("all_reduce_inline", &GradReducer::all_reduce_inline)
      .def_property_readonly("launched", &GradReducer::launched);

  py::class_<FusionReducer, std::shared_ptr<FusionReducer>>(m, "FusionReducer")
      .def(py::init<std::shared_ptr<Comm>, int64_t, bool>(), py::arg("comm"), py::arg("fusion_bytes"),
           py::arg("average") = true)
      .def("register_tensor", &FusionReducer::register_tensor)
      .def("enqueue", &FusionReducer::enqueue)
      .def("synchronize", &FusionReducer::synchronize)
      .def_property_readonly("collectives", &FusionReducer::collectives)
      .def_property_readonly("num_registered", &FusionReducer::num_registered);
}

}  // namespace pdrnn
