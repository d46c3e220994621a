// Native runtime pieces shared by the bindings: hipGraph capture/replay,
// HIP error helpers and the pinned-host batch prefetcher.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace mlt {

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// A captured sequence of launches replayed with one hipGraphLaunch.
// Capture happens on a private non-blocking stream in thread-local mode, so no
// other thread's work can leak into the graph; replay goes to any stream.
class HipGraph {
 public:
  HipGraph() = default;
  ~HipGraph() { reset(); }
  HipGraph(const HipGraph&) = delete;
  HipGraph& operator=(const HipGraph&) = delete;

  // Capture `body(stream)` into this graph.
  void capture(const std::function<void(hipStream_t)>& body);
  void launch(hipStream_t stream);
  bool valid() const { return exec_ != nullptr; }
  void reset();
  size_t num_nodes() const { return nodes_; }

 private:
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  hipStream_t cap_stream_ = nullptr;
  size_t nodes_ = 0;
};

// Pinned-host double/triple-buffered prefetcher: a worker thread fills pinned
// slots through a user callback (e.g. collating a batch on the host), and the
// consumer issues hipMemcpyAsync H2D on a dedicated copy stream, recording an
// event that the compute stream waits on. This is what feeds datasets that do
// not live in HBM (north star: "prefetches into pinned host memory with
// hipMemcpyAsync on a side stream").
class PinnedPrefetcher {
 public:
  // slot_bytes: bytes per batch; depth: number of pinned slots in flight.
  PinnedPrefetcher(size_t slot_bytes, int depth, int device);
  ~PinnedPrefetcher();
  void* slot_ptr(int i) const { return slots_[i]; }
  int depth() const { return depth_; }
  // Copy `bytes` of pinned slot `i` to `dst` on the copy stream and make
  // `compute` wait for it. The slot may be refilled once `slot_ready(i)`.
  void copy_to_device(int i, void* dst, size_t bytes, hipStream_t compute);
  bool slot_ready(int i);
  void wait_slot(int i);

 private:
  std::vector<void*> slots_;
  std::vector<hipEvent_t> events_;
  std::vector<hipEvent_t> before_;
  hipStream_t copy_stream_ = nullptr;
  size_t slot_bytes_;
  int depth_;
  int device_;
};

}  // namespace mlt
