// LayerNorm forward/backward and BERT embedding gather/scatter for gfx950.
//
// LayerNorm over rows of length D (768 / 1024): one wave per row, 4 rows per
// 256-thread block, bf16 in/out with 8-byte (4 x bf16) vector accesses, fp32
// statistics (two-pass mean / variance in registers), fp32 gamma/beta read
// directly from the master parameters. Backward: dx per row in one pass; dgamma /
// dbeta accumulated per lane across a grid-stride set of rows, reduced across the
// block's waves in LDS, written as per-block partials and summed over blocks by a
// second kernel in a fixed order (deterministic, no atomics).
#include <algorithm>

#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_fp8.h"

namespace mlt {

template <int VPL>  // 4-element vectors per lane: D = VPL * 256
__device__ __forceinline__ void load_row(const uint16_t* __restrict__ p, float (&x)[VPL * 4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const ushort4 u = reinterpret_cast<const ushort4*>(p)[lane + 64 * v];
    x[4 * v + 0] = bf16_to_f32(u.x);
    x[4 * v + 1] = bf16_to_f32(u.y);
    x[4 * v + 2] = bf16_to_f32(u.z);
    x[4 * v + 3] = bf16_to_f32(u.w);
  }
}

template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const uint16_t* __restrict__ X, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, uint16_t* __restrict__ Y,
                                                     float* __restrict__ mean, float* __restrict__ rstd, int64_t rows,
                                                     float eps) {
  constexpr int D = VPL * 256, E = VPL * 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float x[E];
  load_row<VPL>(X + row * D, x);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < E; ++i) s += x[i];
  const float mu = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const float d = x[i] - mu;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) * (1.f / D) + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = 4 * (lane + 64 * v);
    const float4 g = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b = *reinterpret_cast<const float4*>(beta + c);
    ushort4 o;
    o.x = f32_to_bf16((x[4 * v + 0] - mu) * rs * g.x + b.x);
    o.y = f32_to_bf16((x[4 * v + 1] - mu) * rs * g.y + b.y);
    o.z = f32_to_bf16((x[4 * v + 2] - mu) * rs * g.z + b.z);
    o.w = f32_to_bf16((x[4 * v + 3] - mu) * rs * g.w + b.w);
    reinterpret_cast<ushort4*>(Y + row * D)[lane + 64 * v] = o;
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)); partial dgamma/dbeta per block.
// DXS: also emit per-block column sums of the (bf16-rounded) dx -- the bias gradient of the
// linear layer whose output (plus residual) fed this LayerNorm, fused here for free.
template <int VPL, bool DXS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const uint16_t* __restrict__ DY, const uint16_t* __restrict__ X,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, uint16_t* __restrict__ DX,
                                                     float* __restrict__ part, int64_t rows,
                                                     const uint16_t* __restrict__ DRES) {
  constexpr int D = VPL * 256, E = VPL * 4;
  constexpr int NS = DXS ? 3 : 2;
  __shared__ float red[4][NS * D];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float dg[E], db[E], g[E], dxs[DXS ? E : 1];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    dg[i] = 0.f;
    db[i] = 0.f;
    if constexpr (DXS) dxs[i] = 0.f;
  }
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const float4 gv = *reinterpret_cast<const float4*>(gamma + 4 * (lane + 64 * v));
    g[4 * v] = gv.x;
    g[4 * v + 1] = gv.y;
    g[4 * v + 2] = gv.z;
    g[4 * v + 3] = gv.w;
  }
  // software-pipelined over the wave's rows: the next row's x / dy / statistics are in flight
  // while this row computes (each wave walks ~rows / 2048 rows; one row of latency per step otherwise)
  const int64_t rstep = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + wid;
  ushort4 nx[VPL], ndy[VPL];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    const int64_t rr = r < rows ? r : rows - 1;  // clamped, branch-free
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      nx[v] = reinterpret_cast<const ushort4*>(X + rr * D)[lane + 64 * v];
      ndy[v] = reinterpret_cast<const ushort4*>(DY + rr * D)[lane + 64 * v];
    }
    nmu = mean[rr];
    nrs = rstd[rr];
  };
  if (row < rows) fetch(row);
  for (; row < rows; row += rstep) {
    float x[E], dy[E];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      x[4 * v + 0] = bf16_to_f32(nx[v].x);
      x[4 * v + 1] = bf16_to_f32(nx[v].y);
      x[4 * v + 2] = bf16_to_f32(nx[v].z);
      x[4 * v + 3] = bf16_to_f32(nx[v].w);
      dy[4 * v + 0] = bf16_to_f32(ndy[v].x);
      dy[4 * v + 1] = bf16_to_f32(ndy[v].y);
      dy[4 * v + 2] = bf16_to_f32(ndy[v].z);
      dy[4 * v + 3] = bf16_to_f32(ndy[v].w);
    }
    const float mu = nmu, rs = nrs;
    fetch(row + rstep);  // unconditional: past the end it re-reads the last row (unused)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float xh = (x[i] - mu) * rs;
      x[i] = xh;
      const float t = dy[i] * g[i];
      s1 += t;
      s2 += t * xh;
      dg[i] += dy[i] * xh;
      db[i] += dy[i];
    }
    s1 = wave_sum(s1) * (1.f / D);
    s2 = wave_sum(s2) * (1.f / D);
    float dres[E];
    if (DRES) load_row<VPL>(DRES + row * D, dres);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 4 * v + q;
        o[q] = rs * (dy[i] * g[i] - s1 - x[i] * s2) + (DRES ? dres[i] : 0.f);
      }
      ushort4 u;
      u.x = f32_to_bf16(o[0]);
      u.y = f32_to_bf16(o[1]);
      u.z = f32_to_bf16(o[2]);
      u.w = f32_to_bf16(o[3]);
      reinterpret_cast<ushort4*>(DX + row * D)[lane + 64 * v] = u;
      if constexpr (DXS) {
        dxs[4 * v + 0] += bf16_to_f32(u.x);
        dxs[4 * v + 1] += bf16_to_f32(u.y);
        dxs[4 * v + 2] += bf16_to_f32(u.z);
        dxs[4 * v + 3] += bf16_to_f32(u.w);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * (lane + 64 * v) + q;
      red[wid][c] = dg[4 * v + q];
      red[wid][D + c] = db[4 * v + q];
      if constexpr (DXS) red[wid][2 * D + c] = dxs[4 * v + q];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < NS * D; c += 256)
    part[(int64_t)blockIdx.x * NS * D + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// fp8 variant (DXS, no DRES): the same dx, plus dx quantised for the fp8 GEMMs that consume it as
// their dY -- e5m2 Y [rows, D] and Y^T [D, rows] with the consumer's delayed scale, and its amax.
// Each quantised value is the bf16-rounded dx times the scale, the value the separate cast-transpose
// would read back, so Y / Y^T / amax equal ln_bwd + fp8_cast_transpose bit for bit (the dgamma /
// dbeta / column-sum partials cover other row sets, so those agree to fp32 rounding). A block
// walks 32-row chunks (wave w: rows 8 w .. 8 w + 7); the chunk's fp8 rows are staged in LDS and
// leave as 32-byte Y^T row pieces, 4 columns per thread.
template <int VPL>
__global__ __launch_bounds__(256) void ln_bwd_q8_kernel(const uint16_t* __restrict__ DY, const uint16_t* __restrict__ X,
                                                        const float* __restrict__ gamma, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, uint16_t* __restrict__ DX,
                                                        float* __restrict__ part, int64_t rows, uint8_t* __restrict__ Y8,
                                                        uint8_t* __restrict__ YT8, const float* __restrict__ qscale,
                                                        float* __restrict__ qamax) {
  constexpr int D = VPL * 256, E = VPL * 4, NS = 3, CR = 32;
  constexpr int RED_BYTES = 4 * NS * D * 4, TILE_BYTES = CR * D;
  __shared__ __attribute__((aligned(16))) uint8_t smem[RED_BYTES > TILE_BYTES ? RED_BYTES : TILE_BYTES];
  uint8_t* tile = smem;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float qs = *qscale;
  float dg[E], db[E], g[E], dxs[E], mx = 0.f;
#pragma unroll
  for (int i = 0; i < E; ++i) dg[i] = db[i] = dxs[i] = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const float4 gv = *reinterpret_cast<const float4*>(gamma + 4 * (lane + 64 * v));
    g[4 * v] = gv.x, g[4 * v + 1] = gv.y, g[4 * v + 2] = gv.z, g[4 * v + 3] = gv.w;
  }
  const int64_t nchunks = rows / CR;
  ushort4 nx[VPL], ndy[VPL];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    const int64_t rr = r < rows ? r : rows - 1;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      nx[v] = reinterpret_cast<const ushort4*>(X + rr * D)[lane + 64 * v];
      ndy[v] = reinterpret_cast<const ushort4*>(DY + rr * D)[lane + 64 * v];
    }
    nmu = mean[rr];
    nrs = rstd[rr];
  };
  int64_t ch = blockIdx.x;
  if (ch < nchunks) fetch(ch * CR + wid * 8);
  for (; ch < nchunks; ch += gridDim.x) {
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
      const int rl = wid * 8 + k;
      const int64_t row = ch * CR + rl;
      float x[E], dy[E];
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        x[4 * v + 0] = bf16_to_f32(nx[v].x), x[4 * v + 1] = bf16_to_f32(nx[v].y);
        x[4 * v + 2] = bf16_to_f32(nx[v].z), x[4 * v + 3] = bf16_to_f32(nx[v].w);
        dy[4 * v + 0] = bf16_to_f32(ndy[v].x), dy[4 * v + 1] = bf16_to_f32(ndy[v].y);
        dy[4 * v + 2] = bf16_to_f32(ndy[v].z), dy[4 * v + 3] = bf16_to_f32(ndy[v].w);
      }
      const float mu = nmu, rs = nrs;
      fetch(k < 7 ? row + 1 : (ch + gridDim.x) * CR + wid * 8);  // past the end: re-reads the last row
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < E; ++i) {
        const float xh = (x[i] - mu) * rs;
        x[i] = xh;
        const float t = dy[i] * g[i];
        s1 += t;
        s2 += t * xh;
        dg[i] += dy[i] * xh;
        db[i] += dy[i];
      }
      s1 = wave_sum(s1) * (1.f / D);
      s2 = wave_sum(s2) * (1.f / D);
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 4 * v + q;
          o[q] = bf16_to_f32(f32_to_bf16(rs * (dy[i] * g[i] - s1 - x[i] * s2)));  // dx as stored
          dxs[i] += o[q];
          mx = fmaxf(mx, fabsf(o[q]));
        }
        ushort4 u;
        u.x = f32_to_bf16(o[0]), u.y = f32_to_bf16(o[1]), u.z = f32_to_bf16(o[2]), u.w = f32_to_bf16(o[3]);
        reinterpret_cast<ushort4*>(DX + row * D)[lane + 64 * v] = u;
        const uint32_t q8 = pack4_fp8<1>(o[0] * qs, o[1] * qs, o[2] * qs, o[3] * qs);
        *reinterpret_cast<uint32_t*>(Y8 + row * D + 4 * (lane + 64 * v)) = q8;
        *reinterpret_cast<uint32_t*>(tile + rl * D + 4 * (lane + 64 * v)) = q8;
      }
    }
    __syncthreads();
    // Y^T: thread t takes columns 4 t .. 4 t + 3, the chunk's 32 rows -> 32 bytes per column
    if (threadIdx.x * 4 < D) {
      const int c4 = threadIdx.x * 4;
      uint32_t d[CR];
#pragma unroll
      for (int r = 0; r < CR; ++r) d[r] = *reinterpret_cast<const uint32_t*>(tile + r * D + c4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int sh = 8 * j;
        uint32_t w[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          w[q] = ((d[4 * q] >> sh) & 0xffu) | (((d[4 * q + 1] >> sh) & 0xffu) << 8) |
                 (((d[4 * q + 2] >> sh) & 0xffu) << 16) | (((d[4 * q + 3] >> sh) & 0xffu) << 24);
        uint4* tp = reinterpret_cast<uint4*>(YT8 + (int64_t)(c4 + j) * rows + ch * CR);
        tp[0] = make_uint4(w[0], w[1], w[2], w[3]);
        tp[1] = make_uint4(w[4], w[5], w[6], w[7]);
      }
    }
    __syncthreads();  // the tile is rewritten by the next chunk
  }
  float* red = reinterpret_cast<float*>(smem);  // [4][NS * D], after the last chunk's barrier
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * (lane + 64 * v) + q;
      red[wid * NS * D + c] = dg[4 * v + q];
      red[wid * NS * D + D + c] = db[4 * v + q];
      red[wid * NS * D + 2 * D + c] = dxs[4 * v + q];
    }
  mx = wave_max(mx);
  if (lane == 0) atomic_max_pos(qamax, mx);
  __syncthreads();
  for (int c = threadIdx.x; c < NS * D; c += 256)
    part[(int64_t)blockIdx.x * NS * D + c] =
        (red[c] + red[NS * D + c]) + (red[2 * NS * D + c] + red[3 * NS * D + c]);
}

// out_k[c] (+)= sum_r part[r][k*seg + c]: wave = 4 columns, lanes stride the rows, xor tree (fixed order)
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, int R, int64_t ld, int W,
                                                          int seg, SegOut o, int accmask) {
  const int lane = threadIdx.x & 63;
  const int c = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
  if (c >= W) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int r = lane; r < R; r += 64) {
    const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)r * ld + c);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s.x += __shfl_xor(s.x, off, 64);
    s.y += __shfl_xor(s.y, off, 64);
    s.z += __shfl_xor(s.z, off, 64);
    s.w += __shfl_xor(s.w, off, 64);
  }
  if (lane == 0) {
    const int k = c / seg;
    float* out = o.p[k] + (c - k * seg);
    if ((accmask >> k) & 1) {
      const float4 prev = *reinterpret_cast<const float4*>(out);
      s.x += prev.x;
      s.y += prev.y;
      s.z += prev.z;
      s.w += prev.w;
    }
    *reinterpret_cast<float4*>(out) = s;
  }
}

void launch_reduce_rows(const float* part, int R, int64_t ld, int W, int seg, SegOut outs, int accmask, hipStream_t st) {
  if (W <= 0 || R <= 0) return;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((W / 4 + 3) / 4), dim3(256), 0, st, part, R, ld, W, seg, outs, accmask);
}

static int ln_vpl(int D) { return D / 256; }

void launch_ln_fwd(const uint16_t* X, const float* gamma, const float* beta, uint16_t* Y, float* mean, float* rstd,
                   int64_t rows, int D, float eps, hipStream_t st) {
  if (rows <= 0) return;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (ln_vpl(D)) {
    case 1: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, block, 0, st, X, gamma, beta, Y, mean, rstd, rows, eps); break;
    case 2: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, block, 0, st, X, gamma, beta, Y, mean, rstd, rows, eps); break;
    case 3: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, block, 0, st, X, gamma, beta, Y, mean, rstd, rows, eps); break;
    case 4: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, block, 0, st, X, gamma, beta, Y, mean, rstd, rows, eps); break;
    default: break;
  }
}

// the fp8 variant's grid: 32-row chunks, up to 3 blocks per CU (48 KB of LDS each) -- its chunk
// barriers leave 2 blocks per CU short of latency hiding
int ln_bwd_q8_partial_blocks(int64_t rows) { return (int)std::min<int64_t>(std::max<int64_t>(rows / 32, 1), 768); }

int ln_bwd_partial_blocks(int64_t rows) {
  int64_t nb = (rows + 3) / 4;
  return (int)(nb < 512 ? nb : 512);
}

void launch_ln_bwd(const uint16_t* DY, const uint16_t* X, const float* gamma, const float* mean, const float* rstd,
                   uint16_t* DX, float* part, float* dgamma, float* dbeta, int64_t rows, int D, int accumulate,
                   const uint16_t* DRES, float* dxsum, int dxsum_acc, hipStream_t st) {
  if (rows <= 0) return;
  const int nb = ln_bwd_partial_blocks(rows);
  const dim3 grid(nb), block(256);
#define MLT_LN_BWD(V)                                                                                              \
  if (dxsum)                                                                                                       \
    hipLaunchKernelGGL((ln_bwd_kernel<V, true>), grid, block, 0, st, DY, X, gamma, mean, rstd, DX, part, rows, DRES); \
  else                                                                                                             \
    hipLaunchKernelGGL((ln_bwd_kernel<V, false>), grid, block, 0, st, DY, X, gamma, mean, rstd, DX, part, rows, DRES);
  switch (ln_vpl(D)) {
    case 1: MLT_LN_BWD(1) break;
    case 2: MLT_LN_BWD(2) break;
    case 3: MLT_LN_BWD(3) break;
    case 4: MLT_LN_BWD(4) break;
    default: return;
  }
#undef MLT_LN_BWD
  SegOut o{{dgamma, dbeta, dxsum}};
  launch_reduce_rows(part, nb, (dxsum ? 3 : 2) * D, (dxsum ? 3 : 2) * D, D, o, (accumulate ? 3 : 0) | (dxsum_acc ? 4 : 0), st);
}

bool launch_ln_bwd_q8(const uint16_t* DY, const uint16_t* X, const float* gamma, const float* mean, const float* rstd,
                      uint16_t* DX, float* part, float* dgamma, float* dbeta, int64_t rows, int D, int accumulate,
                      float* dxsum, int dxsum_acc, uint8_t* Y8, uint8_t* YT8, const float* qscale, float* qamax,
                      hipStream_t st) {
  if (rows <= 0 || rows % 32 || (D != 768 && D != 1024)) return false;
  const int nb = ln_bwd_q8_partial_blocks(rows);
  const dim3 grid(nb), block(256);
  if (D == 1024)
    hipLaunchKernelGGL(ln_bwd_q8_kernel<4>, grid, block, 0, st, DY, X, gamma, mean, rstd, DX, part, rows, Y8, YT8, qscale,
                       qamax);
  else
    hipLaunchKernelGGL(ln_bwd_q8_kernel<3>, grid, block, 0, st, DY, X, gamma, mean, rstd, DX, part, rows, Y8, YT8, qscale,
                       qamax);
  SegOut o{{dgamma, dbeta, dxsum}};
  launch_reduce_rows(part, nb, 3 * D, 3 * D, D, o, (accumulate ? 3 : 0) | (dxsum_acc ? 4 : 0), st);
  return true;
}

// ---------------------------------------------------------------------------
// BERT embeddings: out[t] = Wword[ids[t]] + Wpos[pos[t]] + Wtype[tt[t]]  (bf16 tables, bf16 out)
// ---------------------------------------------------------------------------
template <int VPL>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                        const uint16_t* __restrict__ Ww, const uint16_t* __restrict__ Wp,
                                                        const uint16_t* __restrict__ Wt, uint16_t* __restrict__ out,
                                                        int64_t rows, int S, int64_t vocab, int ntype) {
  constexpr int D = VPL * 256, E = VPL * 4;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  int64_t ty = tt ? tt[row] : 0;
  ty = ty < 0 ? 0 : (ty >= ntype ? ntype - 1 : ty);
  const int pos = (int)(row % S);
  float a[E], b[E], c[E];
  load_row<VPL>(Ww + id * D, a);
  load_row<VPL>(Wp + (int64_t)pos * D, b);
  load_row<VPL>(Wt + ty * D, c);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    ushort4 o;
    o.x = f32_to_bf16(a[4 * v] + b[4 * v] + c[4 * v]);
    o.y = f32_to_bf16(a[4 * v + 1] + b[4 * v + 1] + c[4 * v + 1]);
    o.z = f32_to_bf16(a[4 * v + 2] + b[4 * v + 2] + c[4 * v + 2]);
    o.w = f32_to_bf16(a[4 * v + 3] + b[4 * v + 3] + c[4 * v + 3]);
    reinterpret_cast<ushort4*>(out + row * D)[lane + 64 * v] = o;
  }
}

// word / position grads: fp32 atomics (the vocabulary rows hit are sparse and spread);
// token-type grads: per-block partials over the (few) type rows, reduced in fixed order.
// Embedding backward without atomics (bitwise reproducible):
//  * word rows: the token ids arrive sorted (stable, host-side torch.sort) with the permutation;
//    one wave per sorted entry, and the wave that starts a run of equal ids sums that run's
//    gradient rows in token order and adds the sum to its table row (one writer per row);
//  * positions / token types: one wave per position sums the B rows of that position in batch
//    order into gp, and leaves the per-type sums as a partial row for reduce_rows.
template <int VPL>
__global__ __launch_bounds__(256) void embed_bwd_word_kernel(const int64_t* __restrict__ sid,
                                                             const int64_t* __restrict__ perm,
                                                             const uint16_t* __restrict__ DX, float* __restrict__ gw,
                                                             int64_t rows, int64_t vocab) {
  constexpr int D = VPL * 256, E = VPL * 4;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows) return;
  const int64_t id = sid[i];
  if (i > 0 && sid[i - 1] == id) return;  // not the start of a run
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  for (int64_t j = i; j < rows && sid[j] == id; ++j) {
    float d[E];
    load_row<VPL>(DX + perm[j] * D, d);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] += d[e];
  }
  const int64_t row = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    float4* g = reinterpret_cast<float4*>(gw + row * D + 4 * (lane + 64 * v));
    float4 o = *g;
    o.x += acc[4 * v];
    o.y += acc[4 * v + 1];
    o.z += acc[4 * v + 2];
    o.w += acc[4 * v + 3];
    *g = o;
  }
}

template <int VPL>
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const int64_t* __restrict__ tt,
                                                            const uint16_t* __restrict__ DX, float* __restrict__ gp,
                                                            float* __restrict__ part_t, int64_t rows, int S) {
  constexpr int D = VPL * 256, E = VPL * 4;
  const int lane = threadIdx.x & 63;
  const int pos = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pos >= S) return;
  float a[E], t0[E], t1[E];
#pragma unroll
  for (int e = 0; e < E; ++e) a[e] = t0[e] = t1[e] = 0.f;
  for (int64_t r = pos; r < rows; r += S) {
    float d[E];
    load_row<VPL>(DX + r * D, d);
    const bool one = tt && tt[r] != 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      a[e] += d[e];
      t0[e] += one ? 0.f : d[e];
      t1[e] += one ? d[e] : 0.f;
    }
  }
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = 4 * (lane + 64 * v);
    float4* g = reinterpret_cast<float4*>(gp + (int64_t)pos * D + c);
    float4 o = *g;
    o.x += a[4 * v];
    o.y += a[4 * v + 1];
    o.z += a[4 * v + 2];
    o.w += a[4 * v + 3];
    *g = o;
    *reinterpret_cast<float4*>(part_t + (int64_t)pos * 2 * D + c) =
        make_float4(t0[4 * v], t0[4 * v + 1], t0[4 * v + 2], t0[4 * v + 3]);
    *reinterpret_cast<float4*>(part_t + (int64_t)pos * 2 * D + D + c) =
        make_float4(t1[4 * v], t1[4 * v + 1], t1[4 * v + 2], t1[4 * v + 3]);
  }
}

void launch_embed_fwd(const int64_t* ids, const int64_t* tt, const uint16_t* Ww, const uint16_t* Wp,
                      const uint16_t* Wt, uint16_t* out, int64_t rows, int S, int D, int64_t vocab, int ntype,
                      hipStream_t st) {
  if (rows <= 0) return;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (D / 256) {
    case 3: hipLaunchKernelGGL(embed_fwd_kernel<3>, grid, block, 0, st, ids, tt, Ww, Wp, Wt, out, rows, S, vocab, ntype); break;
    case 4: hipLaunchKernelGGL(embed_fwd_kernel<4>, grid, block, 0, st, ids, tt, Ww, Wp, Wt, out, rows, S, vocab, ntype); break;
    case 1: hipLaunchKernelGGL(embed_fwd_kernel<1>, grid, block, 0, st, ids, tt, Ww, Wp, Wt, out, rows, S, vocab, ntype); break;
    case 2: hipLaunchKernelGGL(embed_fwd_kernel<2>, grid, block, 0, st, ids, tt, Ww, Wp, Wt, out, rows, S, vocab, ntype); break;
    default: break;
  }
}

void launch_embed_bwd(const int64_t* sid, const int64_t* perm, const int64_t* tt, const uint16_t* DX, float* gw,
                      float* gp, float* gt, float* part, int64_t rows, int S, int D, int64_t vocab, int ntype,
                      hipStream_t st) {
  if (rows <= 0) return;
  const dim3 gw_grid((unsigned)((rows + 3) / 4)), gp_grid((unsigned)((S + 3) / 4)), block(256);
#define MLT_EMB_BWD(V)                                                                                          \
  hipLaunchKernelGGL(embed_bwd_word_kernel<V>, gw_grid, block, 0, st, sid, perm, DX, gw, rows, vocab);         \
  hipLaunchKernelGGL(embed_bwd_pos_kernel<V>, gp_grid, block, 0, st, tt, DX, gp, part, rows, S);
  switch (D / 256) {
    case 1: MLT_EMB_BWD(1) break;
    case 2: MLT_EMB_BWD(2) break;
    case 3: MLT_EMB_BWD(3) break;
    case 4: MLT_EMB_BWD(4) break;
    default: return;
  }
#undef MLT_EMB_BWD
  // token types 0 and 1 (ntype <= 2): the S partial rows summed in position order into gt
  SegOut o{{gt, gt + D, nullptr}};
  launch_reduce_rows(part, S, 2 * D, ntype >= 2 ? 2 * D : D, D, o, ntype >= 2 ? 3 : 1, st);
}

}  // namespace mlt
