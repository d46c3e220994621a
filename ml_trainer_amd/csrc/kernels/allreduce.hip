// One-shot all-reduce over xGMI for latency-bound gradient buckets (the LeNet step's single
// 248 KB bucket; SURVEY.md N12 "custom xGMI one-shot all-reduce for sub-MB buckets").
//
// Every rank owns an uncached (fine-grained) region, IPC-mapped into all peers:
//   data [2][cap] fp32        -- double-buffered by step parity
//   flags[2][G][W] uint64     -- flags[p][b][q] = last step at which rank q published slice b
// Block b of every rank owns slice b of the vector:
//   1. copy its slice of the local gradient into data[p] of its own region, fence (system);
//   2. store seq into flags[p][b][me] of EVERY peer's region (remote release stores);
//   3. spin on its own flags[p][b][*] until all W peers published seq (system acquire loads,
//      bounded by a wall-clock timeout);
//   4. sum slice b over the W regions in rank order (same order on every rank -> bit-identical
//      results everywhere), scale (1/W for AVG), write the local gradient.
// No second barrier: a rank can only reach step s+2 (and overwrite parity p) after it saw all
// peers publish step s+1, and a peer publishes s+1 only after its step-s kernel -- including
// its reads of parity p -- completed (stream order). seq is a per-block device launch counter
// (monotonic, never reset), so the kernel is replay-safe inside multi-step hipGraphs.
// Failure: a wait that exceeds the timeout sets the sticky error word (host-mapped, so the
// host polls it after every graph replay without a device sync) and the block returns WITHOUT
// reducing or updating -- no step ever runs on partial peer data. Every later launch on this
// rank sees the word and returns at once (it stops publishing), so every peer times out too and
// the whole job fails loudly instead of training divergent replicas; the parity argument
// above no longer matters because no launch after the error touches gradients or weights.
// With POST the averaged gradient slice is consumed right away by the flat optimizer update
// (the data-parallel step then needs no separate optimizer launch).
// The rank count is a template parameter (WT = 2..8): the W peer loads of a float4 are issued
// back to back and summed afterwards, so a thread waits ONE xGMI round trip, not W of them (with a
// runtime W hipcc emitted load -> s_waitcnt vmcnt(0) -> add per peer: 8 serial remote reads at
// W = 8). The optimizer operands are local and loaded before the peer loads are waited for.
#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_optim.h"

namespace mlt {

template <bool POST, int WT>
__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(float* __restrict__ grad, int64_t n, XgmiPeers P,
                                                             int rank, int W, int64_t cap,
                                                             uint64_t* __restrict__ seqs, float scale,
                                                             unsigned* __restrict__ err, long long timeout,
                                                             XgmiPostOpt O) {
  static_assert(WT >= 2 && WT <= kXgmiMaxRanks, "rank count");
  const int G = gridDim.x, b = blockIdx.x;
  __shared__ int failed;
  if (threadIdx.x == 0) failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  __syncthreads();
  if (failed) return;  // an earlier launch timed out: this rank no longer takes steps
  const uint64_t seq = seqs[b] + 1;  // per-block launch counter: identical on every block and rank
  const int p = (int)(seq & 1);
  const int64_t chunk = ((n + G - 1) / G + 3) & ~(int64_t)3;  // float4 granules
  const int64_t lo = (int64_t)b * chunk, hi = min(n, lo + chunk);
  float* mine = P.data[rank] + p * cap;
  const float* src[WT];  // this step's parity of every rank's region (uniform: SGPRs)
#pragma unroll
  for (int q = 0; q < WT; ++q) src[q] = P.data[q] + p * cap;
  // 1. publish this block's slice
  for (int64_t i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
    if (i + 4 <= hi) {
      *reinterpret_cast<float4*>(mine + i) = *reinterpret_cast<const float4*>(grad + i);
    } else {
      for (int64_t j = i; j < hi; ++j) mine[j] = grad[j];
    }
  }
  __threadfence_system();
  __syncthreads();
  // 2. signal every peer
  if (threadIdx.x < WT) {
    uint64_t* f = P.flags[threadIdx.x] + ((int64_t)p * G + b) * WT + rank;
    __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for all peers' slice b of this step
  if (threadIdx.x < WT) {
    uint64_t* f = P.flags[rank] + ((int64_t)p * G + b) * WT + threadIdx.x;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
      if (wall_clock64() - t0 > timeout) {  // wall_clock64 ticks at the 100 MHz constant clock
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        failed = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (failed) return;  // partial peer data: leave gradient, weights and the launch counter alone
  // 4. reduce in rank order (+ optimizer update)
  float lr = 0.f, tstep = 0.f;
  bool has_s1 = false, has_s2 = false;
  if constexpr (POST) {
    lr = O.lr_ptr ? O.lr_ptr[O.lr_index_ptr ? (*O.lr_index_ptr - 1) : 0] : O.h.lr;
    tstep = (float)(*O.step_ptr);
    has_s2 = O.h.kind == OPT_ADAM || O.h.kind == OPT_ADAMW || O.h.kind == OPT_ADAMAX;
    has_s1 = has_s2 || O.h.kind == OPT_ADAGRAD || (O.h.kind == OPT_SGD && O.h.momentum != 0.f);
  }
  for (int64_t i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
    if (i + 4 <= hi) {
      float4 v[WT];
#pragma unroll
      for (int q = 0; q < WT; ++q) v[q] = *reinterpret_cast<const float4*>(src[q] + i);
      // every peer load is issued before anything waits on one (hipcc otherwise interleaves the
      // adds with partial vmcnt waits between the loads)
      __builtin_amdgcn_sched_barrier(0);
      float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), av = pv, bv = pv;
      if constexpr (POST) {  // local optimizer operands: in flight together with the peer reads
        pv = *reinterpret_cast<const float4*>(O.p + i);
        if (has_s1) av = *reinterpret_cast<const float4*>(O.s1 + i);
        if (has_s2) bv = *reinterpret_cast<const float4*>(O.s2 + i);
      }
      float4 s = v[0];
#pragma unroll
      for (int q = 1; q < WT; ++q) {  // rank order: bit-identical on every rank
        s.x += v[q].x;
        s.y += v[q].y;
        s.z += v[q].z;
        s.w += v[q].w;
      }
      s.x *= scale;
      s.y *= scale;
      s.z *= scale;
      s.w *= scale;
      *reinterpret_cast<float4*>(grad + i) = s;
      if constexpr (POST) {
        opt_update(O.h, lr, tstep, pv.x, s.x, av.x, bv.x);
        opt_update(O.h, lr, tstep, pv.y, s.y, av.y, bv.y);
        opt_update(O.h, lr, tstep, pv.z, s.z, av.z, bv.z);
        opt_update(O.h, lr, tstep, pv.w, s.w, av.w, bv.w);
        *reinterpret_cast<float4*>(O.p + i) = pv;
        if (has_s1) *reinterpret_cast<float4*>(O.s1 + i) = av;
        if (has_s2) *reinterpret_cast<float4*>(O.s2 + i) = bv;
      }
    } else {
      for (int64_t j = i; j < hi; ++j) {
        float v[WT];
#pragma unroll
        for (int q = 0; q < WT; ++q) v[q] = src[q][j];
        float s = v[0];
#pragma unroll
        for (int q = 1; q < WT; ++q) s += v[q];
        s *= scale;
        grad[j] = s;
        if constexpr (POST) {
          float pv = O.p[j], av = has_s1 ? O.s1[j] : 0.f, bv = has_s2 ? O.s2[j] : 0.f;
          opt_update(O.h, lr, tstep, pv, s, av, bv);
          O.p[j] = pv;
          if (has_s1) O.s1[j] = av;
          if (has_s2) O.s2[j] = bv;
        }
      }
    }
  }
  if (threadIdx.x == 0) seqs[b] = seq;  // read again only by the next launch (stream order)
}

template <bool POST>
static void launch_w(int W, dim3 g, hipStream_t st, float* grad, int64_t n, const XgmiPeers& P, int rank, int64_t cap,
                     uint64_t* seqs, float scale, unsigned* err, long long timeout, const XgmiPostOpt& post) {
#define MLT_XGMI_W(WV)                                                                                       \
  case WV:                                                                                                   \
    hipLaunchKernelGGL((xgmi_allreduce_kernel<POST, WV>), g, dim3(256), 0, st, grad, n, P, rank, W, cap, seqs, \
                       scale, err, timeout, post);                                                           \
    break;
  switch (W) {
    MLT_XGMI_W(2)
    MLT_XGMI_W(3)
    MLT_XGMI_W(4)
    MLT_XGMI_W(5)
    MLT_XGMI_W(6)
    MLT_XGMI_W(7)
    MLT_XGMI_W(8)
    default: break;
  }
#undef MLT_XGMI_W
}

void launch_xgmi_allreduce(float* grad, int64_t n, const XgmiPeers& P, int rank, int W, int64_t cap, int blocks,
                           uint64_t* seqs, float scale, unsigned* err, long long timeout_ticks,
                           const XgmiPostOpt* post, hipStream_t st) {
  if (n <= 0 || W < 2 || W > kXgmiMaxRanks) return;  // (the host object rejects other world sizes)
  if (post)
    launch_w<true>(W, dim3(blocks), st, grad, n, P, rank, cap, seqs, scale, err, timeout_ticks, *post);
  else
    launch_w<false>(W, dim3(blocks), st, grad, n, P, rank, cap, seqs, scale, err, timeout_ticks, XgmiPostOpt{});
}

}  // namespace mlt
