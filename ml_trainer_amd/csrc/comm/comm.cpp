// Native RCCL communicator: see mlt_comm.h.
#include "mlt_comm.h"

#include <stdexcept>

namespace mlt {

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

static ncclDataType_t to_nccl(CommDtype d) {
  switch (d) {
    case CommDtype::F32: return ncclFloat32;
    case CommDtype::BF16: return ncclBfloat16;
    case CommDtype::F16: return ncclFloat16;
    case CommDtype::I32: return ncclInt32;
    case CommDtype::I64: return ncclInt64;
    case CommDtype::U8: return ncclUint8;
  }
  throw std::runtime_error("unsupported comm dtype");
}

static size_t dt_size(CommDtype d) {
  switch (d) {
    case CommDtype::F32: case CommDtype::I32: return 4;
    case CommDtype::BF16: case CommDtype::F16: return 2;
    case CommDtype::I64: return 8;
    case CommDtype::U8: return 1;
  }
  return 1;
}

static ncclRedOp_t to_nccl(CommOp o) {
  switch (o) {
    case CommOp::SUM: return ncclSum;
    case CommOp::AVG: return ncclAvg;
    case CommOp::MAX: return ncclMax;
    case CommOp::MIN: return ncclMin;
  }
  throw std::runtime_error("unsupported comm op");
}

std::string Communicator::unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

Communicator::Communicator(const std::string& uid, int nranks, int rank, int device)
    : nranks_(nranks), rank_(rank), device_(device) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id length");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("bad rank / world size");
  ncclUniqueId id;
  std::copy(uid.begin(), uid.end(), id.internal);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) throw std::runtime_error("hipGetDevice failed");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclResult_t r = ncclCommInitRank(&comm_, nranks, id, rank);
  (void)hipSetDevice(prev);
  nccl_check(r, "ncclCommInitRank");
}

Communicator::~Communicator() {
  if (comm_) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

void Communicator::all_reduce(const void* send, void* recv, size_t count, CommDtype dt, CommOp op, hipStream_t st) {
  nccl_check(ncclAllReduce(send, recv, count, to_nccl(dt), to_nccl(op), comm_, st), "ncclAllReduce");
}

void Communicator::reduce_scatter(const void* send, void* recv, size_t recv_count, CommDtype dt, CommOp op,
                                  hipStream_t st) {
  nccl_check(ncclReduceScatter(send, recv, recv_count, to_nccl(dt), to_nccl(op), comm_, st), "ncclReduceScatter");
}

void Communicator::all_gather(const void* send, void* recv, size_t send_count, CommDtype dt, hipStream_t st) {
  nccl_check(ncclAllGather(send, recv, send_count, to_nccl(dt), comm_, st), "ncclAllGather");
}

void Communicator::broadcast(const void* send, void* recv, size_t count, CommDtype dt, int root, hipStream_t st) {
  nccl_check(ncclBroadcast(send, recv, count, to_nccl(dt), root, comm_, st), "ncclBroadcast");
}

void Communicator::all_to_all(const void* send, void* recv, size_t count_per_peer, CommDtype dt, hipStream_t st) {
  // grouped point-to-point exchange: chunk p of `send` goes to peer p
  const size_t bytes = count_per_peer * dt_size(dt);
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  for (int p = 0; p < nranks_; ++p) {
    nccl_check(ncclSend(static_cast<const char*>(send) + p * bytes, count_per_peer, to_nccl(dt), p, comm_, st),
               "ncclSend");
    nccl_check(ncclRecv(static_cast<char*>(recv) + p * bytes, count_per_peer, to_nccl(dt), p, comm_, st),
               "ncclRecv");
  }
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

std::string Communicator::async_error() const {
  ncclResult_t e = ncclSuccess;
  if (comm_ && ncclCommGetAsyncError(comm_, &e) == ncclSuccess && e != ncclSuccess) return ncclGetErrorString(e);
  return "";
}

void Communicator::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

}  // namespace mlt
