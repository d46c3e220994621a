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
// reducing. Blocks whose peers did arrive still reduce their slices, so the training step does
// not fuse the update into this kernel (POST is for standalone use): the flat optimizer launch
// that follows reads the error word and applies NOTHING on a rank that saw any timeout -- the
// step is all-or-nothing per rank (a peer that finished its own wait may have applied it; the
// failing rank raises TransportError and the job stops). Every later launch on this
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
                                                             XgmiPostOpt O, int fault) {
  static_assert(WT >= 2 && WT <= kXgmiMaxRanks, "rank count");
  const int G = gridDim.x, b = blockIdx.x;
  const bool withhold = fault == 1 && b % (2 * WT) == rank;  // fault injection (tests only)
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
  if (threadIdx.x < WT && !withhold) {
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
                     uint64_t* seqs, float scale, unsigned* err, long long timeout, const XgmiPostOpt& post,
                     int fault) {
#define MLT_XGMI_W(WV)                                                                                       \
  case WV:                                                                                                   \
    hipLaunchKernelGGL((xgmi_allreduce_kernel<POST, WV>), g, dim3(256), 0, st, grad, n, P, rank, W, cap, seqs, \
                       scale, err, timeout, post, fault);                                                    \
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
                           const XgmiPostOpt* post, hipStream_t st, int fault) {
  if (n <= 0 || W < 2 || W > kXgmiMaxRanks) return;  // (the host object rejects other world sizes)
  if (post)
    launch_w<true>(W, dim3(blocks), st, grad, n, P, rank, cap, seqs, scale, err, timeout_ticks, *post, fault);
  else
    launch_w<false>(W, dim3(blocks), st, grad, n, P, rank, cap, seqs, scale, err, timeout_ticks, XgmiPostOpt{},
                    fault);
}

// ---- two-shot: reduce-scatter + all-gather, both by remote PUSHES -----------------------------
// The one-shot kernel pulls the whole vector from every peer ((W-1) x n floats per rank over
// xGMI); here each rank moves 2 (W-1)/W x n. Rank slice r = [r*ns, (r+1)*ns); block b owns
// sub-chunk [b*c, (b+1)*c) of every slice:
//   1. push sub-chunk b of slice q of the local gradient into rank q's t1[p][me] (posted remote
//      stores, no round trip), fence (system), flag f1 on rank q;
//   2. wait for f1 from all W ranks, sum t1[p][0..W-1] (LOCAL reads, rank order), scale, push
//      the reduced sub-chunk into EVERY rank's t2[p][me], fence, flag f2 everywhere;
//   3. wait for f2 from all W ranks, copy t2[p][q] (local) into the gradient (+ optimizer).
// Every element is summed by exactly one rank in rank order and copied everywhere, so all ranks
// hold bit-identical results. Reuse of parity p two launches later is safe for the one-shot's
// reason: a peer's step s+2 phase 1 (t1) needs this rank's step s+2 push, and its phase 2 (t2)
// needs this rank's step s+2 phase 1 -- both issued after this rank's step-s kernel retired.
// Failure: as the one-shot (sticky error word, no write to the gradient / weights).
template <int WT>
__device__ __forceinline__ bool xgmi_wait(uint64_t* f, uint64_t seq, long long timeout, unsigned* err, int* failed) {
  // threads 0..WT-1 each wait for one rank's flag; returns false on timeout
  if (threadIdx.x < WT) {
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f + threadIdx.x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
      if (wall_clock64() - t0 > timeout) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *failed = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return !*failed;
}

template <bool POST, int WT>
__global__ __launch_bounds__(256) void xgmi_twoshot_kernel(float* __restrict__ grad, int64_t n, XgmiPeers P, int rank,
                                                           int64_t S, uint64_t* __restrict__ seqs, float scale,
                                                           unsigned* __restrict__ err, long long timeout,
                                                           XgmiPostOpt O, int fault) {
  static_assert(WT >= 2 && WT <= kXgmiMaxRanks, "rank count");
  const int G = gridDim.x, b = blockIdx.x;
  const bool withhold = fault == 1 && b % (2 * WT) == rank;  // fault injection (tests only)
  __shared__ int failed;
  if (threadIdx.x == 0) failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  __syncthreads();
  if (failed) return;
  const uint64_t seq = seqs[b] + 1;
  const int p = (int)(seq & 1);
  const int64_t ns = ((n + WT - 1) / WT + 3) & ~(int64_t)3;   // slice length (float4 granules)
  const int64_t c = ((ns + G - 1) / G + 3) & ~(int64_t)3;     // sub-chunk per block
  const int64_t lo = min(ns, (int64_t)b * c), hi = min(ns, lo + c);
  const int nq4 = (int)((hi - lo) / 4);                        // float4s of this block per slice
  const int64_t fo = ((int64_t)p * G + b) * WT;                // flag row of (parity, block)
  // 1. scatter: sub-chunk b of slice q -> rank q's t1[p][rank]
  for (int idx = threadIdx.x; idx < WT * nq4; idx += blockDim.x) {
    const int q = idx / nq4, k = idx - q * nq4;
    const int64_t off = lo + 4 * k, gi = q * ns + off;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gi + 4 <= n) {
      v = *reinterpret_cast<const float4*>(grad + gi);
    } else {
      if (gi < n) v.x = grad[gi];
      if (gi + 1 < n) v.y = grad[gi + 1];
      if (gi + 2 < n) v.z = grad[gi + 2];
    }
    *reinterpret_cast<float4*>(P.t1[q] + ((int64_t)p * WT + rank) * S + off) = v;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < WT && !withhold)
    __hip_atomic_store(P.f1[threadIdx.x] + fo + rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!xgmi_wait<WT>(P.f1[rank] + fo, seq, timeout, err, &failed)) return;
  // 2. reduce my slice's sub-chunk b (local reads, rank order) and gather it to every rank
  const float* mine = P.t1[rank] + (int64_t)p * WT * S;
  for (int k = threadIdx.x; k < nq4; k += blockDim.x) {
    const int64_t off = lo + 4 * k;
    float4 v[WT];
#pragma unroll
    for (int q = 0; q < WT; ++q) v[q] = *reinterpret_cast<const float4*>(mine + (int64_t)q * S + off);
    float4 s = v[0];
#pragma unroll
    for (int q = 1; q < WT; ++q) {
      s.x += v[q].x;
      s.y += v[q].y;
      s.z += v[q].z;
      s.w += v[q].w;
    }
    s.x *= scale;
    s.y *= scale;
    s.z *= scale;
    s.w *= scale;
#pragma unroll
    for (int q = 0; q < WT; ++q) *reinterpret_cast<float4*>(P.t2[q] + ((int64_t)p * WT + rank) * S + off) = s;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < WT) __hip_atomic_store(P.f2[threadIdx.x] + fo + rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!xgmi_wait<WT>(P.f2[rank] + fo, seq, timeout, err, &failed)) return;
  // 3. the reduced vector (local) -> gradient (+ optimizer update)
  float lr = 0.f, tstep = 0.f;
  bool has_s1 = false, has_s2 = false;
  if constexpr (POST) {
    lr = O.lr_ptr ? O.lr_ptr[O.lr_index_ptr ? (*O.lr_index_ptr - 1) : 0] : O.h.lr;
    tstep = (float)(*O.step_ptr);
    has_s2 = O.h.kind == OPT_ADAM || O.h.kind == OPT_ADAMW || O.h.kind == OPT_ADAMAX;
    has_s1 = has_s2 || O.h.kind == OPT_ADAGRAD || (O.h.kind == OPT_SGD && O.h.momentum != 0.f);
  }
  const float* red = P.t2[rank] + (int64_t)p * WT * S;
  for (int idx = threadIdx.x; idx < WT * nq4; idx += blockDim.x) {
    const int q = idx / nq4, k = idx - q * nq4;
    const int64_t off = lo + 4 * k, gi = q * ns + off;
    if (gi >= n) continue;
    const float4 s4 = *reinterpret_cast<const float4*>(red + (int64_t)q * S + off);
    const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = gi + j;
      if (e >= n) break;
      grad[e] = sv[j];
      if constexpr (POST) {
        float pv = O.p[e], av = has_s1 ? O.s1[e] : 0.f, bv = has_s2 ? O.s2[e] : 0.f;
        float g = sv[j];
        opt_update(O.h, lr, tstep, pv, g, av, bv);
        O.p[e] = pv;
        if (has_s1) O.s1[e] = av;
        if (has_s2) O.s2[e] = bv;
      }
    }
  }
  if (threadIdx.x == 0) seqs[b] = seq;
}

template <bool POST>
static void launch_w2(int W, dim3 g, hipStream_t st, float* grad, int64_t n, const XgmiPeers& P, int rank, int64_t S,
                      uint64_t* seqs, float scale, unsigned* err, long long timeout, const XgmiPostOpt& post,
                      int fault) {
#define MLT_XGMI_W2(WV)                                                                                         \
  case WV:                                                                                                      \
    hipLaunchKernelGGL((xgmi_twoshot_kernel<POST, WV>), g, dim3(256), 0, st, grad, n, P, rank, S, seqs, scale, \
                       err, timeout, post, fault);                                                              \
    break;
  switch (W) {
    MLT_XGMI_W2(2)
    MLT_XGMI_W2(3)
    MLT_XGMI_W2(4)
    MLT_XGMI_W2(5)
    MLT_XGMI_W2(6)
    MLT_XGMI_W2(7)
    MLT_XGMI_W2(8)
    default: break;
  }
#undef MLT_XGMI_W2
}

void launch_xgmi_allreduce_2shot(float* grad, int64_t n, const XgmiPeers& P, int rank, int W, int64_t slot,
                                 int blocks, uint64_t* seqs, float scale, unsigned* err, long long timeout_ticks,
                                 const XgmiPostOpt* post, hipStream_t st, int fault) {
  if (n <= 0 || W < 2 || W > kXgmiMaxRanks) return;
  if (post)
    launch_w2<true>(W, dim3(blocks), st, grad, n, P, rank, slot, seqs, scale, err, timeout_ticks, *post, fault);
  else
    launch_w2<false>(W, dim3(blocks), st, grad, n, P, rank, slot, seqs, scale, err, timeout_ticks, XgmiPostOpt{},
                     fault);
}

}  // namespace mlt
