// Communicators: native RCCL (device) and a c10d ProcessGroup adapter (gloo /
// CPU plumbing).  See pdrnn/runtime.h.
//
// The RCCL communicator is the MI355X-native replacement of the reference's
// ProcessGroupMPI (reference: src/motion/trainer/ddp.py:18,
// src/example/example_distributed.py:18-19):
//  * bootstrapped from an ncclUniqueId that the Python side distributes
//    through the torch.distributed TCPStore rendezvous,
//  * every collective runs on ONE dedicated high-priority HIP stream per
//    communicator, fenced against the caller's compute stream with events, so
//    gradient all-reduce overlaps the BPTT kernels still running on the
//    compute stream,
//  * payloads are torch tensors; their storage is recorded on the comm stream
//    so the caching allocator never recycles memory a collective still reads.
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>

#include "pdrnn/runtime.h"

namespace pdrnn {
namespace {

namespace py = pybind11;

#define NCCL_CHECK(expr)                                                                   \
  do {                                                                                     \
    ncclResult_t _r = (expr);                                                              \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error: ", ncclGetErrorString(_r), " @ " #expr); \
  } while (0)
#define HIP_CHECK(expr)                                                                    \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " @ " #expr);     \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    default: TORCH_CHECK(false, "RCCL: unsupported dtype ", t);
  }
}

ncclRedOp_t to_nccl(RedOp op) {
  switch (op) {
    case RedOp::kSum: return ncclSum;
    case RedOp::kAvg: return ncclAvg;
    case RedOp::kMax: return ncclMax;
    case RedOp::kMin: return ncclMin;
  }
  return ncclSum;
}

class RcclComm final : public Comm {
 public:
  RcclComm(const std::string& uid, int rank, int world, int device, bool high_priority)
      : rank_(rank), world_(world), device_(device) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo));
    HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
    NCCL_CHECK(ncclCommInitRank(&comm_, world_, id, rank_));
  }
  ~RcclComm() override {
    if (comm_) {
      hipStreamSynchronize(stream_);
      ncclCommDestroy(comm_);
    }
    if (ev_in_) hipEventDestroy(ev_in_);
    if (ev_out_) hipEventDestroy(ev_out_);
    if (stream_) hipStreamDestroy(stream_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool native_avg() const override { return true; }

  void all_reduce(at::Tensor& t, RedOp op) override {
    check(t);
    // an in-place reduction over one rank is the identity: no collective, no
    // comm-stream hop (the autograd DDP path at N = 1).  The inline variant
    // below still issues it, so forced-sync timing runs keep the RCCL kernel.
    if (world_ == 1) return;
    enter();
    NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_nccl(op), comm_, stream_));
    leave({t});
  }
  void broadcast(at::Tensor& t, int root) override {
    check(t);
    enter();
    NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
    leave({t});
  }
  void all_gather(at::Tensor& out, const at::Tensor& in) override {
    check(out); check(in);
    TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: out must hold world * in elements");
    enter();
    NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, stream_));
    leave({out, in});
  }
  void reduce_scatter(at::Tensor& out, const at::Tensor& in, RedOp op) override {
    check(out); check(in);
    TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: in must hold world * out elements");
    enter();
    NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()), to_nccl(op),
                                 comm_, stream_));
    leave({out, in});
  }
  void all_to_all(at::Tensor& out, const at::Tensor& in) override {
    check(out); check(in);
    TORCH_CHECK(in.numel() % world_ == 0 && out.numel() == in.numel(), "all_to_all: equal splits required");
    const int64_t chunk = in.numel() / world_;
    const size_t esz = in.element_size();
    const auto dt = to_nccl(in.scalar_type());
    enter();
    NCCL_CHECK(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      NCCL_CHECK(ncclSend(static_cast<const char*>(in.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, stream_));
      NCCL_CHECK(ncclRecv(static_cast<char*>(out.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, stream_));
    }
    NCCL_CHECK(ncclGroupEnd());
    leave({out, in});
  }
  void send(const at::Tensor& t, int peer) override {
    check(t);
    enter();
    NCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
    leave({t});
  }
  void recv(at::Tensor& t, int peer) override {
    check(t);
    enter();
    NCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), peer, comm_, stream_));
    leave({t});
  }
  void all_reduce_inline(at::Tensor& t, RedOp op) override {
    check(t);
    // keep this communicator's collectives strictly ordered: join any still
    // queued on the comm stream first
    if (pending_) wait();
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    hipStream_t cs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream();
    if (cs == nullptr) {
      // never put RCCL on the legacy NULL stream (it synchronises with every
      // blocking stream): go through the comm stream instead
      all_reduce(t, op);
      wait();
      return;
    }
    NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_nccl(op), comm_, cs));
    if (serialize_comm()) HIP_CHECK(hipStreamSynchronize(cs));
  }
  void wait() override {
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    HIP_CHECK(hipEventRecord(ev_out_, stream_));
    HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream(), ev_out_, 0));
    pending_ = false;
  }
  void barrier() override {
    auto t = at::zeros({1}, at::TensorOptions().device(at::kCUDA, device_).dtype(at::kFloat));
    all_reduce(t, RedOp::kSum);
    wait();
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  hipStream_t stream() const { return stream_; }

 private:
  void check(const at::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "RCCL tensors must live on device ", device_);
    TORCH_CHECK(t.is_contiguous(), "RCCL tensors must be contiguous");
  }
  // Order the comm stream after everything enqueued on the caller's stream.
  void enter() {
    pending_ = true;
    c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    HIP_CHECK(hipEventRecord(ev_in_, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device_).stream()));
    HIP_CHECK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  void leave(std::initializer_list<at::Tensor> ts) {
    auto s = c10::hip::getStreamFromExternalMasqueradingAsCUDA(stream_, (c10::DeviceIndex)device_);
    for (const auto& t : ts)
      if (t.defined() && t.storage().data_ptr().get())
        c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(t.storage().data_ptr(), s);
    if (serialize_comm()) HIP_CHECK(hipStreamSynchronize(stream_));
  }

  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  bool pending_ = false;  // collectives on stream_ not yet joined by wait()
};

// c10d adapter: drives torch.distributed collectives (gloo on CPU, or torch's
// own RCCL process group) through Python.  Used for the CPU plumbing path and
// as a fallback; async work handles are waited in wait().
class ProcessGroupComm final : public Comm {
  void maybe_serialize() {
    if (serialize_comm()) wait();
  }

 public:
  explicit ProcessGroupComm(py::object pg) : pg_(std::move(pg)) {
    py::gil_scoped_acquire gil;
    dist_ = py::module_::import("torch.distributed");
    rank_ = dist_.attr("get_rank")(pg_).cast<int>();
    world_ = dist_.attr("get_world_size")(pg_).cast<int>();
    backend_ = py::str(dist_.attr("get_backend")(pg_)).cast<std::string>();
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool native_avg() const override { return backend_ == "nccl"; }

  void all_reduce(at::Tensor& t, RedOp op) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_reduce")(t, py::arg("op") = pyop(op), py::arg("group") = pg_,
                                               py::arg("async_op") = true));
    maybe_serialize();
  }
  void broadcast(at::Tensor& t, int root) override {
    py::gil_scoped_acquire gil;
    const int groot = dist_.attr("get_global_rank")(pg_, root).cast<int>();
    works_.push_back(dist_.attr("broadcast")(t, py::arg("src") = groot, py::arg("group") = pg_,
                                              py::arg("async_op") = true));
    maybe_serialize();
  }
  void all_gather(at::Tensor& out, const at::Tensor& in) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_gather_into_tensor")(out, in, py::arg("group") = pg_, py::arg("async_op") = true));
    maybe_serialize();
  }
  void reduce_scatter(at::Tensor& out, const at::Tensor& in, RedOp op) override {
    py::gil_scoped_acquire gil;
    if (backend_ == "gloo") {
      // gloo has no reduce_scatter: all_reduce a copy and slice.
      auto tmp = in.clone();
      dist_.attr("all_reduce")(tmp, py::arg("op") = pyop(op), py::arg("group") = pg_);
      out.copy_(tmp.view({world_, -1}).select(0, rank_).view_as(out));
      return;
    }
    works_.push_back(dist_.attr("reduce_scatter_tensor")(out, in, py::arg("op") = pyop(op), py::arg("group") = pg_,
                                                         py::arg("async_op") = true));
    maybe_serialize();
  }
  void all_to_all(at::Tensor& out, const at::Tensor& in) override {
    py::gil_scoped_acquire gil;
    works_.push_back(dist_.attr("all_to_all_single")(out, in, py::arg("group") = pg_, py::arg("async_op") = true));
    maybe_serialize();
  }
  void send(const at::Tensor& t, int peer) override {
    py::gil_scoped_acquire gil;
    const int g = dist_.attr("get_global_rank")(pg_, peer).cast<int>();
    dist_.attr("send")(t, g, py::arg("group") = pg_);
  }
  void recv(at::Tensor& t, int peer) override {
    py::gil_scoped_acquire gil;
    const int g = dist_.attr("get_global_rank")(pg_, peer).cast<int>();
    dist_.attr("recv")(t, g, py::arg("group") = pg_);
  }
  void wait() override {
    py::gil_scoped_acquire gil;
    for (auto& w : works_) w.attr("wait")();
    works_.clear();
  }
  void barrier() override {
    wait();
    py::gil_scoped_acquire gil;
    dist_.attr("barrier")(py::arg("group") = pg_);
  }

 private:
  py::object pyop(RedOp op) {
    auto R = dist_.attr("ReduceOp");
    switch (op) {
      case RedOp::kSum: return R.attr("SUM");
      case RedOp::kAvg: return R.attr("AVG");
      case RedOp::kMax: return R.attr("MAX");
      case RedOp::kMin: return R.attr("MIN");
    }
    return R.attr("SUM");
  }
  py::object pg_, dist_;
  std::vector<py::object> works_;
  int rank_ = 0, world_ = 1;
  std::string backend_;
};

}  // namespace

bool serialize_comm() {
  static const bool on = [] {
    const char* e = std::getenv("PDRNN_SERIALIZE_COMM");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::shared_ptr<Comm> make_rccl_comm(const std::string& uid, int rank, int world, int device, bool high_priority) {
  return std::make_shared<RcclComm>(uid, rank, world, device, high_priority);
}

std::shared_ptr<Comm> make_pg_comm(const pybind11::object& process_group) {
  return std::make_shared<ProcessGroupComm>(process_group);
}

}  // namespace pdrnn
