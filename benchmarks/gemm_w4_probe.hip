// Standalone probe for a one-wave-per-SIMD bf16 GEMM main loop (gfx950):
//   C[M,N] = A[M,K] . B[N,K]^T, bf16 operands, fp32 accumulation, bf16 out.
// 256 threads = 4 waves (2 x 2), block tile 256 x 256, wave tile 128 x 128 (8 x 8 fragments of
// v_mfma_f32_16x16x32_bf16, 256 accumulator registers), K staged 32 at a time into a 4-deep ring
// of LDS buffers by global_load_lds (3 K-steps in flight), ONE barrier per K-step, and the next
// K-step's fragments read LDS -> registers while the current step's 64 MFMAs run.
//
// LDS image of one operand per stage: 128 row PAIRS x 128 B; 16-B chunk position `pos` of pair R
// holds chunk p = pos ^ (R & 7) with row = 2R + (p >> 2), k-chunk = p & 3. Every ds_read_b128
// lane group of a 16x32 fragment read then touches 16 distinct 16-B slots (conflict-free).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o gemm_w4_probe gemm_w4_probe.hip
// Run:   ./gemm_w4_probe [M N K ...]   prints one JSON line per shape (TF, max error vs naive).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 32, NST = 4;
constexpr int OPB = BM * BK * 2;  // 16 KB per operand per stage
constexpr int STB = 2 * OPB;      // 32 KB per stage

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// byte offset (from the operand base, at k = 0) of image chunk e for this thread
__device__ __forceinline__ uint32_t src_off(int e, int mn0, int nmn, int64_t ld) {
  const int R = e >> 3, p = (e & 7) ^ (R & 7);
  const int row = min(mn0 + 2 * R + (p >> 2), nmn - 1);
  return (uint32_t)(row * ld * 2 + (p & 3) * 16);
}

// 16x32 fragment (rows r0..r0+15) of an operand image
__device__ __forceinline__ bf16x8 frag(const uint8_t* img, int r0) {
  const int lane = threadIdx.x & 63;
  const int r = r0 + (lane & 15), c = lane >> 4;
  const int R = r >> 1, p = ((r & 1) << 2) | c;
  return *reinterpret_cast<const bf16x8*>(img + R * 128 + ((p ^ (R & 7)) << 4));
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

template <int NW, int SCHED>
__global__ __launch_bounds__(NW * 64, 1) void gemm_w4(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                 uint16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                 int64_t ldb, int64_t ldc, int group_m) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM, tiles = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, tiles);
  int tm, tn;
  {
    const int gm = group_m > 0 ? group_m : tiles_m;
    const int per_group = gm * tiles_n, grp = id / per_group, first_m = grp * gm;
    const int gsize = min(tiles_m - first_m, gm), r = id - grp * per_group;
    tm = first_m + r % gsize;
    tn = r / gsize;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  constexpr int NT = NW * 64, WCN = NW / 2, TJ = 8 / (NW / 4), CH = 1024 / NT;  // chunks / operand / thread
  const int wr = wid / WCN, wc = wid % WCN;
  const int nk = K / BK;

  uint32_t sa[CH], sb[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    sa[i] = src_off(i * NT + tid, m0, M, lda);
    sb[i] = src_off(i * NT + tid, n0, N, ldb);
  }
  auto stage = [&](int kt) {
    uint8_t* base = smem + (kt & (NST - 1)) * STB;
    const uint8_t* a = A + (int64_t)kt * (BK * 2);
    const uint8_t* b = B + (int64_t)kt * (BK * 2);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(a + sa[i]), (lds_void*)(base + (i * NT + wid * 64) * 16), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b + sb[i]), (lds_void*)(base + OPB + (i * NT + wid * 64) * 16),
                                       16, 0, 0);
  };

  f32x4 acc[8][TJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[8], fb0[TJ], fa1[8], fb1[TJ];
  auto read = [&](int kt, bf16x8 (&fa)[8], bf16x8 (&fb)[TJ]) __attribute__((always_inline)) {
    const uint8_t* base = smem + (kt & (NST - 1)) * STB;
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = frag(base, wr * 128 + 16 * i);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = frag(base + OPB, wc * (16 * TJ) + 16 * j);
  };
  // one K-step: publish tile t+1, refill the ring with tile t+3, read tile t+1's fragments into
  // (na, nb) while the 64 MFMAs of tile t run on (ca, cb)
  auto step = [&](int t, bf16x8 (&ca)[8], bf16x8 (&cb)[TJ], bf16x8 (&na)[8], bf16x8 (&nb)[TJ])
                  __attribute__((always_inline)) {
    // branch-free: past the end the ring re-stages / re-reads the last tile (same bytes into its
    // own buffer), so every step keeps exactly 8 loads per thread behind the one it waits for
    if constexpr (CH == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (SCHED == 3) {
      // 64 MFMAs in 16 groups of 4; group q first issues one fragment read of the next step
      // (A for q < 8, B after) and, in even groups, one glds chunk of tile t+3
      const int kt3 = min(t + 3, nk - 1), kt1 = min(t + 1, nk - 1);
      uint8_t* sbase = smem + (kt3 & (NST - 1)) * STB;
      const uint8_t* ga = A + (int64_t)kt3 * (BK * 2);
      const uint8_t* gb = B + (int64_t)kt3 * (BK * 2);
      const uint8_t* rbase = smem + (kt1 & (NST - 1)) * STB;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q < 8)
          na[q] = frag(rbase, wr * 128 + 16 * q);
        else
          nb[q - 8] = frag(rbase + OPB, wc * (16 * TJ) + 16 * (q - 8));
        if ((q & 1) == 0) {
          const int c = q >> 1;  // 0..7: 4 A chunks then 4 B chunks
          if (c < CH)
            __builtin_amdgcn_global_load_lds((const void*)(ga + sa[c]), (lds_void*)(sbase + (c * NT + wid * 64) * 16), 16, 0, 0);
          else
            __builtin_amdgcn_global_load_lds((const void*)(gb + sb[c - CH]),
                                             (lds_void*)(sbase + OPB + ((c - CH) * NT + wid * 64) * 16), 16, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = q * 4 + u, i = f / TJ, j = f % TJ;
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(ca[i]), "v"(cb[j]));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      return;
    }
    stage(min(t + 3, nk - 1));
    read(min(t + 1, nk - 1), na, nb);
    if constexpr (SCHED >= 1) __builtin_amdgcn_sched_barrier(0);  // all loads issued before the MFMAs
    if constexpr (SCHED == 2) {
      // accumulators pinned to AGPRs (the register allocator otherwise splits the 256-register
      // accumulator file between VGPRs and AGPRs and shuffles it every step)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(ca[i]), "v"(cb[j]));
    } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i], cb[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (SCHED >= 1) {
      __builtin_amdgcn_sched_barrier(0);
      // the next set's reads (issued before the MFMAs) are long done: retire them HERE, where the
      // waitcnt pass sees it, so it does not put an lgkmcnt(0) ahead of the next step's MFMAs
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
  };

  // prologue: tiles 0..2 in flight, tile 0 landed + published, its fragments in set 0
  for (int s = 0; s < NST - 1; ++s) stage(min(s, nk - 1));
  if constexpr (CH == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  read(0, fa0, fb0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the loop header then has nothing pending

  int t = 0;
  for (; t + 1 < nk; t += 2) {
    step(t, fa0, fb0, fa1, fb1);
    step(t + 1, fa1, fb1, fa0, fb0);
  }
  if (t < nk) step(t, fa0, fb0, fa1, fb1);

  if constexpr (SCHED >= 2) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // asm MFMAs drained
  // epilogue: straight from registers (probe only)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wr * 128 + 16 * i + 4 * (lane >> 4) + r, gn = n0 + wc * (16 * TJ) + 16 * j + (lane & 15);
        if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = f2bf(acc[i][j][r]);
      }
}

__global__ void ref_gemm(const uint16_t* A, const uint16_t* B, float* C, int M, int N, int K) {
  const int m = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k)
    s += __uint_as_float((uint32_t)A[(int64_t)m * K + k] << 16) * __uint_as_float((uint32_t)B[(int64_t)n * K + k] << 16);
  C[(int64_t)m * N + n] = s;
}

__global__ void fill(uint16_t* p, int64_t n, uint32_t seed) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 2654435761u ^ seed;
  x ^= x >> 13;
  x *= 0x5bd1e995u;
  x ^= x >> 15;
  const float f = (float)(x & 0xffff) / 32768.f - 1.f;
  p[i] = (uint16_t)(__float_as_uint(f) >> 16);
}

template <int NW, int SCHED>
static double run(int M, int N, int K, uint16_t* A, uint16_t* B, uint16_t* C, int iters, int group_m) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t smem = NST * STB;
  CK(hipFuncSetAttribute((const void*)gemm_w4<NW, SCHED>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w)
    gemm_w4<NW, SCHED><<<tiles, NW * 64, smem>>>((const uint8_t*)A, (const uint8_t*)B, C, M, N, K, K, K, N, group_m);
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; ++it)
    gemm_w4<NW, SCHED><<<tiles, NW * 64, smem>>>((const uint8_t*)A, (const uint8_t*)B, C, M, N, K, K, K, N, group_m);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
  std::vector<int> shapes;
  for (int i = 1; i < argc; ++i) shapes.push_back(atoi(argv[i]));
  if (shapes.empty()) shapes = {8192, 8192, 8192};
  const int group_m = getenv("GROUP_M") ? atoi(getenv("GROUP_M")) : 4;
  for (size_t s = 0; s + 2 < shapes.size(); s += 3) {
    const int M = shapes[s], N = shapes[s + 1], K = shapes[s + 2];
    if (K % BK) {
      fprintf(stderr, "K must be a multiple of %d\n", BK);
      return 1;
    }
    uint16_t *A, *B, *C;
    float* R;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    fill<<<(M * (int64_t)K + 255) / 256, 256>>>(A, (int64_t)M * K, 1u);
    fill<<<(N * (int64_t)K + 255) / 256, 256>>>(B, (int64_t)N * K, 7u);
    // correctness on the first 256 rows
    const int MR = M < 512 ? M : 512;
    CK(hipMalloc(&R, (size_t)MR * N * 4));
    ref_gemm<<<dim3((N + 255) / 256, MR), 256>>>(A, B, R, MR, N, K);
    const int iters = (int)fmax(5.0, 2e13 / (2.0 * M * N * K));
    std::vector<uint16_t> hc((size_t)MR * N);
    std::vector<float> hr((size_t)MR * N);
    CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
    auto check = [&]() {
      CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
      double err = 0;
      for (size_t i = 0; i < hc.size(); ++i) {
        float v;
        uint32_t u = (uint32_t)hc[i] << 16;
        std::memcpy(&v, &u, 4);
        err = fmax(err, fabs(v - hr[i]) / (1.0 + fabs(hr[i])));
      }
      CK(hipMemset(C, 0, (size_t)M * N * 2));
      return err;
    };
    const double fl = 2.0 * M * N * K;
    double us[6], err[6];
    us[0] = run<4, 0>(M, N, K, A, B, C, iters, group_m); err[0] = check();
    us[1] = run<4, 1>(M, N, K, A, B, C, iters, group_m); err[1] = check();
    us[2] = run<8, 0>(M, N, K, A, B, C, iters, group_m); err[2] = check();
    us[3] = run<8, 1>(M, N, K, A, B, C, iters, group_m); err[3] = check();
    us[4] = run<4, 2>(M, N, K, A, B, C, iters, group_m); err[4] = check();
    us[5] = run<4, 3>(M, N, K, A, B, C, iters, group_m); err[5] = check();
    const char* nm[6] = {"w4", "w4s", "w8", "w8s", "w4a", "w4i"};
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"group_m\": %d", M, N, K, group_m);
    for (int v = 0; v < 6; ++v) printf(", \"%s_us\": %.2f, \"%s_tf\": %.1f, \"%s_err\": %.3g", nm[v], us[v], nm[v], fl / us[v] * 1e-6, nm[v], err[v]);
    printf("}\n");
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  return 0;
}
