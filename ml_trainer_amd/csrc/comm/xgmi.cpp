// Host side of the one-shot / two-shot xGMI all-reduce (kernels/allreduce.hip).
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "mlt_comm.h"
#include "mlt_kernels.h"

namespace mlt {

static void hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// region: data [2][cap] | flags [2][G][W] | t1 [2][W][slot] | t2 [2][W][slot] | f1 [2][G][W] | f2 [2][G][W]
//         | fg [2][max(cap, kFusedGranules)] (the fused step's granules) | fr [same] (its two-phase
//         variant's reduced granules) | fe (its device error word)
// (the t* / f* parts belong to the two-shot algorithm, ff to the fused LeNet step's exchange, which
// shares `data`), every part 256-byte aligned
struct RegionLayout {
  size_t flags, t1, t2, f1, f2, fg, fr, fe, bytes;
};
static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
// granules per parity half of the fused step's region, a multiple of 32 (256 B): the halves and the
// two-phase reduced array then sit back to back with no align256 padding between them, the layout
// fused_view() hands to the kernels (fr = fg + 2 cap)
static int64_t fused_cap(int64_t cap) {
  const int64_t c = cap > XgmiAllReduce::kFusedGranules ? cap : XgmiAllReduce::kFusedGranules;
  return (c + 31) & ~(int64_t)31;
}
static RegionLayout region_layout(int64_t cap, int world, int blocks, int64_t slot) {
  RegionLayout L;
  const size_t fl = (size_t)2 * blocks * world * sizeof(uint64_t), tb = (size_t)2 * world * slot * sizeof(float);
  L.flags = align256((size_t)2 * cap * sizeof(float));
  L.t1 = align256(L.flags + fl);
  L.t2 = align256(L.t1 + tb);
  L.f1 = align256(L.t2 + tb);
  L.f2 = align256(L.f1 + fl);
  L.fg = align256(L.f2 + fl);                                           // fused step: [2][fcap] granules
  L.fr = align256(L.fg + (size_t)2 * fused_cap(cap) * sizeof(uint64_t));  // two-phase: reduced granules
  L.fe = align256(L.fr + (size_t)2 * fused_cap(cap) * sizeof(uint64_t));  // fused step: device error word
  L.bytes = L.fe + 256;
  return L;
}

XgmiAllReduce::XgmiAllReduce(int64_t cap_floats, int world, int rank, int device, int blocks)
    : cap_((cap_floats + 3) & ~(int64_t)3), world_(world), rank_(rank), device_(device), blocks_(blocks) {
  if (world < 1 || world > kXgmiMaxRanks || rank < 0 || rank >= world) throw std::runtime_error("xgmi: bad world/rank");
  if (blocks < 1 || blocks > 1024) throw std::runtime_error("xgmi: bad block count");
  slot_ = ((cap_ + world - 1) / world + 3) & ~(int64_t)3;
  bytes_ = region_layout(cap_, world, blocks, slot_).bytes;
  hcheck(hipSetDevice(device), "hipSetDevice");
  hcheck(hipExtMallocWithFlags(&region_, bytes_, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  hcheck(hipMemset(region_, 0, bytes_), "hipMemset(region)");
  // error word in coherent pinned host memory: the kernel ORs into it at system scope and the
  // host reads it with a plain load after every replay (no device synchronisation)
  hcheck(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(unsigned),
                       hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc(err)");
  *err_host_ = 0u;
  hcheck(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_), err_host_, 0), "hipHostGetDevicePointer(err)");
  hcheck(hipMalloc(reinterpret_cast<void**>(&seqs_), sizeof(uint64_t) * blocks), "hipMalloc(seqs)");
  hcheck(hipMemset(seqs_, 0, sizeof(uint64_t) * blocks), "hipMemset(seqs)");
  hcheck(hipMalloc(reinterpret_cast<void**>(&fseqs_), sizeof(uint64_t) * kFusedBlocks), "hipMalloc(fseqs)");
  hcheck(hipMemset(fseqs_, 0, sizeof(uint64_t) * kFusedBlocks), "hipMemset(fseqs)");
  hcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  peers_host_ = new XgmiPeers();
  std::memset(peers_host_, 0, sizeof(XgmiPeers));
}

XgmiAllReduce::~XgmiAllReduce() {
  for (int q = 0; q < world_; ++q)
    if (q != rank_ && peer_base_[q]) (void)hipIpcCloseMemHandle(peer_base_[q]);
  if (region_) (void)hipFree(region_);
  if (err_host_) (void)hipHostFree(err_host_);
  if (seqs_) (void)hipFree(seqs_);
  if (fseqs_) (void)hipFree(fseqs_);
  delete static_cast<XgmiPeers*>(peers_host_);
}

std::string XgmiAllReduce::handle() const {
  hipIpcMemHandle_t h;
  hcheck(hipIpcGetMemHandle(&h, region_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiAllReduce::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("xgmi: need one handle per rank");
  hcheck(hipSetDevice(device_), "hipSetDevice");
  XgmiPeers* P = static_cast<XgmiPeers*>(peers_host_);
  const RegionLayout L = region_layout(cap_, world_, blocks_, slot_);
  for (int q = 0; q < world_; ++q) {
    void* base = nullptr;
    if (q == rank_) {
      base = region_;
    } else {
      if (handles[q].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("xgmi: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[q].data(), sizeof(h));
      hcheck(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      peer_base_[q] = base;
    }
    char* c = static_cast<char*>(base);
    P->data[q] = static_cast<float*>(base);
    P->flags[q] = reinterpret_cast<uint64_t*>(c + L.flags);
    P->t1[q] = reinterpret_cast<float*>(c + L.t1);
    P->t2[q] = reinterpret_cast<float*>(c + L.t2);
    P->f1[q] = reinterpret_cast<uint64_t*>(c + L.f1);
    P->f2[q] = reinterpret_cast<uint64_t*>(c + L.f2);
    fg_[q] = reinterpret_cast<uint64_t*>(c + L.fg);
    fr_[q] = reinterpret_cast<uint64_t*>(c + L.fr);
    if (q == rank_) derr_ = reinterpret_cast<unsigned*>(c + L.fe);
  }
  opened_ = true;
}

void XgmiAllReduce::launch(float* grad, int64_t n, float scale, hipStream_t st, const XgmiPostOpt* post) {
  if (!opened_) throw std::runtime_error("xgmi: open() the peer handles first");
  if (n > cap_) throw std::runtime_error("xgmi: vector larger than the region capacity");
  const long long ticks = timeout_ms_ * 100000LL;  // 100 MHz constant clock: 1e5 ticks per ms
  if (algo_ == 1)
    launch_xgmi_allreduce_2shot(grad, n, *static_cast<XgmiPeers*>(peers_host_), rank_, world_, slot_, blocks_, seqs_,
                                scale, err_, ticks, post, st, fault_);
  else
    launch_xgmi_allreduce(grad, n, *static_cast<XgmiPeers*>(peers_host_), rank_, world_, cap_, blocks_, seqs_, scale,
                          err_, ticks, post, st, fault_);
}

XgmiFused XgmiAllReduce::fused_view() const {
  if (!opened_) throw std::runtime_error("xgmi: open() the peer handles first");
  const XgmiPeers* P = static_cast<const XgmiPeers*>(peers_host_);
  XgmiFused X;
  std::memset(&X, 0, sizeof(X));
  (void)P;
  for (int q = 0; q < world_; ++q) {
    X.gran[q] = fg_[q];
    if (fr_[q] != fg_[q] + 2 * fused_cap(cap_)) throw std::runtime_error("xgmi: fused region layout");
  }
  X.two = two_ && world_ > 1 ? 1 : 0;
  X.seqs = fseqs_;
  X.err = err_;
  X.derr = derr_;
  X.cap = fused_cap(cap_);
  X.timeout = timeout_ms_ * 100000LL;
  X.rank = rank_;
  X.W = world_;
  X.G = kFusedBlocks;
  X.fault = fault_;
  return X;
}

void XgmiAllReduce::set_algo(int a) {
  if (a != 0 && a != 1) throw std::runtime_error("xgmi: algo 0 = one-shot, 1 = two-shot");
  algo_ = a;
}

unsigned XgmiAllReduce::error() const {
  return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
}

void XgmiAllReduce::set_timeout_ms(long long ms) {
  if (ms < 1 || ms > 3600LL * 1000) throw std::runtime_error("xgmi: timeout must be in [1 ms, 1 h]");
  timeout_ms_ = ms;
}

}  // namespace mlt
