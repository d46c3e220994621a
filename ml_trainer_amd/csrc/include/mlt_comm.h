// Native RCCL communicator (one process per GPU, xGMI inside the node).
//
// Replaces the reference's SMDDP backend (src/trainer.py:43-44,59): the
// unique id is generated on rank 0 and distributed by the caller (Python passes it
// through the torch.distributed store); collectives are enqueued on any HIP stream, so
// they can be captured into a hipGraph together with the compute of a training step
// (the LeNet engine's multi-step graphs contain the gradient all-reduce).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

namespace mlt {

struct XgmiFused;  // mlt_kernels.h

enum class CommDtype { F32 = 0, BF16 = 1, F16 = 2, I32 = 3, I64 = 4, U8 = 5 };
enum class CommOp { SUM = 0, AVG = 1, MAX = 2, MIN = 3 };

class Communicator {
 public:
  static std::string unique_id();  // NCCL_UNIQUE_ID_BYTES opaque bytes
  Communicator(const std::string& uid, int nranks, int rank, int device);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }

  void all_reduce(const void* send, void* recv, size_t count, CommDtype dt, CommOp op, hipStream_t st);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, CommDtype dt, CommOp op, hipStream_t st);
  void all_gather(const void* send, void* recv, size_t send_count, CommDtype dt, hipStream_t st);
  void broadcast(const void* send, void* recv, size_t count, CommDtype dt, int root, hipStream_t st);
  void all_to_all(const void* send, void* recv, size_t count_per_peer, CommDtype dt, hipStream_t st);
  // ncclCommGetAsyncError; returns "" when healthy
  std::string async_error() const;
  void abort();

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_ = 0, rank_ = 0, device_ = 0;
};

// One-shot all-reduce over xGMI (see kernels/allreduce.hip). Region = uncached device memory
// shared with the peers through IPC handles (dmabuf); exchange the handle() bytes out of band
// (Python passes them through the torch.distributed store) and call open() on every rank.
class XgmiAllReduce {
 public:
  XgmiAllReduce(int64_t cap_floats, int world, int rank, int device, int blocks);
  ~XgmiAllReduce();
  XgmiAllReduce(const XgmiAllReduce&) = delete;
  XgmiAllReduce& operator=(const XgmiAllReduce&) = delete;
  std::string handle() const;
  void open(const std::vector<std::string>& handles);
  bool ready() const { return opened_; }
  // in-place average (scale = 1/W) or sum of grad[0:n) across the ranks (every rank must make
  // the same sequence of calls)
  void launch(float* grad, int64_t n, float scale, hipStream_t st, const struct XgmiPostOpt* post = nullptr);
  // nonzero once a peer wait timed out (sticky; a plain host read of mapped memory, no sync)
  unsigned error() const;
  // peer-wait timeout; graphs captured earlier keep the value they were captured with
  void set_timeout_ms(long long ms);
  long long timeout_ms() const { return timeout_ms_; }
  int world() const { return world_; }
  int64_t capacity() const { return cap_; }
  // device alias of the sticky error word (a following launch can veto its work on it)
  const unsigned* error_dev() const { return err_; }
  // fault injection for tests: 1 = withhold half of this rank's slice flags (see allreduce.hip)
  void set_fault(int f) { fault_ = f; }
  int fault() const { return fault_; }
  // fused LeNet step: two-phase exchange (each 64-granule chunk reduced by its owner rank, which
  // publishes the sum for the others: 2 (W-1)/W of the granules per rank instead of W - 1)
  void set_fused_two(bool t) { two_ = t; }
  bool fused_two() const { return two_; }
  // 0 one-shot (pull everything), 1 two-shot (push reduce-scatter + push all-gather); every rank
  // must use the same algorithm for a given call. Graphs keep the algorithm they were captured with.
  void set_algo(int a);
  int algo() const { return algo_; }
  // the fused LeNet data-parallel step's view (kernels/lenet_mfma.hip): a granule array of its own
  // ([2][cap] x 8 bytes), per-block counters of its own, the device copy of the error word; timeout /
  // fault as set now (graphs keep the values they were captured with). World size 1 = loopback.
  static constexpr int kFusedBlocks = 128;
  // granules per parity of the fused LeNet exchange (its own index space, lenet_mfma.inc
  // xch_granules: conv elements + 256 lane-contiguous granules per fc weight-gradient wave)
  static constexpr int64_t kFusedGranules = 1 << 17;
  XgmiFused fused_view() const;

 private:
  int64_t cap_;
  int64_t slot_ = 0;  // two-shot: floats per rank slot of t1 / t2
  int algo_ = 0;
  int world_, rank_, device_, blocks_;
  void* region_ = nullptr;
  size_t bytes_ = 0;
  void* peer_base_[8] = {nullptr};
  unsigned* err_ = nullptr;       // device alias of err_host_
  unsigned* err_host_ = nullptr;  // coherent pinned host word
  long long timeout_ms_ = 2000;
  uint64_t* seqs_ = nullptr;
  uint64_t* fseqs_ = nullptr;
  uint64_t* fg_[8] = {nullptr};
  unsigned* derr_ = nullptr;  // device copy of the error word (in the region)
  bool opened_ = false;
  int fault_ = 0;
  bool two_ = false;
  uint64_t* fr_[8] = {nullptr};
  void* peers_host_ = nullptr;  // XgmiPeers
};

}  // namespace mlt
