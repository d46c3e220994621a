// MFMA shape A/B on gfx950 (round-4 verdict item "try v_mfma_f32_32x32x16_bf16"): the GEMM inner
// loop of one wave tile of 64 x 64 outputs, K consumed 32 per step, every A / B fragment re-read
// from LDS by ds_read_b128 each step (as in the ping-pong GEMM), on random bf16 data:
//   v16: v_mfma_f32_16x16x32_bf16 -- 4 x 4 tiles, 16 MFMAs + 8 fragment reads per 32-K step
//   v32: v_mfma_f32_32x32x16_bf16 -- 2 x 2 tiles x 2 k-halves, 8 MFMAs + 8 fragment reads per step
// Same wave tile => the same LDS bytes per FLOP; what differs is the instruction count and the
// clock the chip holds (MI355X_MICROARCH.md, DVFS give-back item 7). 8 waves per CU (2 per SIMD),
// 4 blocks of 512 per ... one 512-thread block per CU x 256 CUs x R rounds.
// Build: hipcc --offload-arch=gfx950 -O3 -o benchmarks/bin/mfma_shape_probe benchmarks/mfma_shape_probe.hip
// Run:   ./benchmarks/bin/mfma_shape_probe [iters=20000]   -> one JSON line per variant
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kThreads = 512;
constexpr int kLds = 64 * 1024;  // a 64-row A image + 64-row B image per wave pair region, reused

template <int V>
__global__ __launch_bounds__(kThreads, 1) void probe(const uint4* __restrict__ src, float* __restrict__ out,
                                                     int iters) {
  __shared__ uint4 lds[kLds / 16];
  for (int i = threadIdx.x; i < kLds / 16; i += kThreads) lds[i] = src[(blockIdx.x * 131 + i) & 65535];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // per wave: A rows [64][64 bf16 = 128 B] at region (w & 3) * 16 KB, B rows at + 8 KB; chunk XOR-
  // swizzled by (row >> 1) & 7 (conflict-free for both fragment shapes' lane groups)
  const uint8_t* base = reinterpret_cast<const uint8_t*>(lds) + (w & 3) * 16384;
  auto frag = [&](int img, int row, int chunk) __attribute__((always_inline)) {
    const uint8_t* p = base + img * 8192 + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
    return *reinterpret_cast<const bf16x8*>(p);
  };
  float res = 0.f;
  if constexpr (V == 16) {
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
      const int ks = it & 1;  // two 32-K steps of the 64-K image
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(0, 16 * i + (lane & 15), 4 * ks + (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag(1, 16 * j + (lane & 15), 4 * ks + (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) res += acc[i][j][0] + acc[i][j][3];
  } else {
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int it = 0; it < iters; ++it) {
      const int ks = it & 1;
      bf16x8 a[2][2], b[2][2];  // [tile][k-half of the 32-K step]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i][h] = frag(0, 32 * i + (lane & 31), 4 * ks + 2 * h + (lane >> 5));
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j][h] = frag(1, 32 * j + (lane & 31), 4 * ks + 2 * h + (lane >> 5));
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][h], b[j][h], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) res += acc[i][j][0] + acc[i][j][15];
  }
  out[blockIdx.x * kThreads + threadIdx.x] = res;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus;  // one 512-thread block (8 waves, 2 per SIMD) per CU
  std::vector<uint16_t> h(65536 * 8);
  uint32_t s = 12345u;
  for (auto& v : h) {  // random bf16 in [-1, 1): sign, exponent 126/127, random mantissa
    s = s * 1664525u + 1013904223u;
    v = (uint16_t)(((s >> 31) << 15) | ((126u + ((s >> 20) & 1u)) << 7) | ((s >> 8) & 0x7fu));
  }
  uint4* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, (size_t)blocks * kThreads * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int variants[2] = {16, 32};
  for (int rep = 0; rep < 3; ++rep) {
    for (int vi = 0; vi < 2; ++vi) {
      const int V = variants[vi];
      auto launch = [&]() {
        if (V == 16)
          hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(kThreads), 0, 0, src, out, iters);
        else
          hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(kThreads), 0, 0, src, out, iters);
      };
      launch();  // warm
      CHECK(hipDeviceSynchronize());
      const int reps = 10;
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      // per iteration a wave does a 64 x 64 x 32 MAC block
      const double flop = 2.0 * 64 * 64 * 32 * (double)iters * (kThreads / 64) * blocks * reps;
      printf("{\"variant\": \"v_mfma_f32_%s_bf16\", \"rep\": %d, \"waves_per_cu\": 8, \"wave_tile\": \"64x64\", "
             "\"iters\": %d, \"ms\": %.4f, \"tflops\": %.1f}\n",
             V == 16 ? "16x16x32" : "32x32x16", rep, iters, ms / reps, flop / (ms / reps * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
