// Host runtime of pytorch_distributed_rnn_amd: communicators and gradient
// synchronisation engines (C++, g++-compiled, linked against torch + RCCL).
//
//  * Comm            abstract async collective interface
//  * RcclComm        native RCCL communicator on a dedicated high-priority HIP
//                    stream, ordered against the compute stream with events
//                    (replaces ProcessGroupMPI of the reference)
//  * ProcessGroupComm  the same interface over a c10d::ProcessGroup (gloo for
//                    the CPU plumbing configuration, or torch's RCCL group)
//  * GradReducer     DDP-style bucketed all-reduce driven by per-parameter
//                    readiness (replaces torch 1.4's C++ DDP Reducer, N7)
//  * FusionReducer   Horovod-style per-tensor all-reduce with a tensor-fusion
//                    buffer and an explicit synchronize() (replaces Horovod
//                    core, N9)
#pragma once

#include <torch/extension.h>

#include <memory>
#include <string>
#include <vector>

namespace pdrnn {

enum class RedOp { kSum = 0, kAvg = 1, kMax = 2, kMin = 3 };

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual bool native_avg() const = 0;  // does all_reduce(kAvg) divide on the wire?
  // All collectives are asynchronous w.r.t. the host.  For device tensors they
  // are ordered after all work already enqueued on the caller's current stream.
  virtual void all_reduce(at::Tensor& t, RedOp op) = 0;
  virtual void broadcast(at::Tensor& t, int root) = 0;
  virtual void all_gather(at::Tensor& out, const at::Tensor& in) = 0;
  virtual void reduce_scatter(at::Tensor& out, const at::Tensor& in, RedOp op) = 0;
  virtual void all_to_all(at::Tensor& out, const at::Tensor& in) = 0;
  virtual void send(const at::Tensor& t, int peer) = 0;
  virtual void recv(at::Tensor& t, int peer) = 0;
  // Make the caller's current stream (device) or the host (CPU) wait for every
  // collective issued so far.
  virtual void wait() = 0;
  virtual void barrier() = 0;
  // all_reduce whose result is ordered into the caller's current stream, for
  // call sites with nothing to overlap (the fused motion step): RCCL runs
  // straight on that stream, no cross-stream event hops.
  virtual void all_reduce_inline(at::Tensor& t, RedOp op) {
    all_reduce(t, op);
    wait();
  }
  // ---- failure detection (RcclComm: watchdog thread; others: their
  // backend's own timeouts) ----
  // Release the communicator now (watchdog joined, collectives drained with
  // a deadline, then destroyed or aborted); idempotent, later calls raise.
  // Called for every cached communicator at interpreter exit (parallel/comm.py)
  // so no watchdog thread is still polling the HIP runtime while the
  // process's exit handlers tear it down.
  virtual void close() {}
  virtual bool aborted() const { return false; }
  virtual double timeout_s() const { return 0.0; }
  virtual int64_t tracked() const { return 0; }  // collectives the watchdog has followed
  // bound the work enqueued so far on the caller's current stream like a
  // collective (a replayed graph that contains collectives: captured
  // collectives carry no completion event of their own)
  virtual void track_current() {}
  // test hook: occupy the comm stream for `seconds` like a collective whose
  // peer never arrives (bounded spin kernel)
  virtual void debug_stall(double seconds) {
    (void)seconds;
    TORCH_CHECK(false, "debug_stall: only the native RCCL communicator has a device-side stall");
  }
};

// exit status of a process whose communicator watchdog fired (see comm.cpp)
constexpr int kWatchdogExit = 86;

// PDRNN_SERIALIZE_COMM=1: every collective completes (device-synchronised)
// before the call returns -- A/B switch for overlap / stream-ordering bugs.
bool serialize_comm();

// CU budget of RCCL's kernels (PDRNN_RCCL_MAX_CTAS) and the CUs a persistent
// grid must leave free in this process (0 until a multi-rank RCCL
// communicator exists)
int rccl_max_ctas();
int rccl_cta_reserve();

std::shared_ptr<Comm> make_rccl_comm(const std::string& uid, int rank, int world, int device, bool high_priority,
                                     double timeout_s);
std::shared_ptr<Comm> make_pg_comm(const pybind11::object& process_group);
std::string rccl_unique_id();

void register_runtime(pybind11::module_& m);

}  // namespace pdrnn
