// hipGraph executor + pinned-host prefetcher (see mlt_runtime.h).
#include "mlt_runtime.h"

namespace mlt {

void HipGraph::reset() {
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  if (cap_stream_) hipStreamDestroy(cap_stream_);
  exec_ = nullptr;
  graph_ = nullptr;
  cap_stream_ = nullptr;
  nodes_ = 0;
}

void HipGraph::capture(const std::function<void(hipStream_t)>& body) {
  reset();
  hip_check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
  hip_check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  try {
    body(cap_stream_);
  } catch (...) {
    hipGraph_t g = nullptr;
    hipStreamEndCapture(cap_stream_, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  hip_check(hipStreamEndCapture(cap_stream_, &graph_), "hipStreamEndCapture");
  hip_check(hipGetLastError(), "launch during capture");
  hip_check(hipGraphGetNodes(graph_, nullptr, &nodes_), "hipGraphGetNodes");
  hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
  // upload now so the first replay costs what every later one does
  hip_check(hipGraphUpload(exec_, cap_stream_), "hipGraphUpload");
  hip_check(hipStreamSynchronize(cap_stream_), "hipStreamSynchronize(upload)");
}

void HipGraph::launch(hipStream_t stream) {
  if (!exec_) throw std::runtime_error("HipGraph::launch on an empty graph");
  hip_check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
}

PinnedPrefetcher::PinnedPrefetcher(size_t slot_bytes, int depth, int device)
    : slot_bytes_(slot_bytes), depth_(depth), device_(device) {
  if (depth < 1 || depth > 64) throw std::invalid_argument("PinnedPrefetcher depth must be in [1, 64]");
  hip_check(hipSetDevice(device), "hipSetDevice");
  hip_check(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking), "hipStreamCreate(copy)");
  slots_.resize(depth, nullptr);
  events_.resize(depth, nullptr);
  released_.resize(depth, nullptr);
  has_release_.assign(depth, 0);
  for (int i = 0; i < depth; ++i) {
    hip_check(hipHostMalloc(&slots_[i], slot_bytes, hipHostMallocDefault), "hipHostMalloc");
    hip_check(hipEventCreateWithFlags(&events_[i], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&released_[i], hipEventDisableTiming), "hipEventCreate");
  }
}

PinnedPrefetcher::~PinnedPrefetcher() {
  for (int i = 0; i < depth_; ++i) {
    if (events_[i]) {
      hipEventSynchronize(events_[i]);
      hipEventDestroy(events_[i]);
    }
    if (released_[i]) hipEventDestroy(released_[i]);
    if (slots_[i]) hipHostFree(slots_[i]);
  }
  if (copy_stream_) hipStreamDestroy(copy_stream_);
}

void PinnedPrefetcher::copy_to_device(int i, void* dst, size_t bytes) {
  if (i < 0 || i >= depth_) throw std::out_of_range("prefetch slot");
  if (bytes > slot_bytes_) throw std::invalid_argument("prefetch copy larger than slot");
  // device buffer i may still be read by the batch that used it last: wait for ITS release only
  // (a wait captures the event's latest record, so re-recording it later is safe)
  if (has_release_[i]) hip_check(hipStreamWaitEvent(copy_stream_, released_[i], 0), "hipStreamWaitEvent");
  hip_check(hipMemcpyAsync(dst, slots_[i], bytes, hipMemcpyHostToDevice, copy_stream_), "hipMemcpyAsync");
  hip_check(hipEventRecord(events_[i], copy_stream_), "hipEventRecord");
}

void PinnedPrefetcher::acquire(int i, hipStream_t compute) {
  if (i < 0 || i >= depth_) throw std::out_of_range("prefetch slot");
  hip_check(hipStreamWaitEvent(compute, events_[i], 0), "hipStreamWaitEvent");
}

void PinnedPrefetcher::release(int i, hipStream_t compute) {
  if (i < 0 || i >= depth_) throw std::out_of_range("prefetch slot");
  hip_check(hipEventRecord(released_[i], compute), "hipEventRecord");
  has_release_[i] = 1;
}

bool PinnedPrefetcher::slot_ready(int i) { return hipEventQuery(events_[i]) == hipSuccess; }

void PinnedPrefetcher::wait_slot(int i) { hip_check(hipEventSynchronize(events_[i]), "hipEventSynchronize"); }

}  // namespace mlt
