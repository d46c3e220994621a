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

// Pinned-host ring prefetcher: `depth` persistent hipHostMalloc slots, each paired by the caller
// with a device buffer. The H2D hipMemcpyAsync runs on a dedicated copy stream and overlaps the
// compute stream's kernels; the two streams meet only where the data dependences are:
//   copy_to_device(i)  copy stream waits for release(i) -- the compute that last read device
//                      buffer i -- then copies slot i and records ready(i);
//   acquire(i, s)      stream s waits for ready(i) (at the point the batch is CONSUMED);
//   release(i, s)      records on s, after the consumer's work on buffer i was enqueued.
// With d buffers the copy of batch k + d - 1 runs while batch k computes. This is what feeds
// datasets that do not live in HBM (north star: "prefetches into pinned host memory with
// hipMemcpyAsync on a side stream").
class PinnedPrefetcher {
 public:
  // slot_bytes: bytes per batch; depth: number of pinned slots in flight.
  PinnedPrefetcher(size_t slot_bytes, int depth, int device);
  ~PinnedPrefetcher();
  void* slot_ptr(int i) const { return slots_[i]; }
  int depth() const { return depth_; }
  void copy_to_device(int i, void* dst, size_t bytes);
  void acquire(int i, hipStream_t compute);
  void release(int i, hipStream_t compute);
  // the host slot may be refilled once its copy is done
  bool slot_ready(int i);
  void wait_slot(int i);

 private:
  std::vector<void*> slots_;
  std::vector<hipEvent_t> events_;    // ready(i): copy of slot i done
  std::vector<hipEvent_t> released_;  // release(i): compute done reading device buffer i
  std::vector<char> has_release_;
  hipStream_t copy_stream_ = nullptr;
  size_t slot_bytes_;
  int depth_;
  int device_;
};

}  // namespace mlt
