// Small utility kernels.
//
// transpose_b16: out[c][r] = x[r][c] for 2-byte elements, the K-contiguous
// x^T operand of the transposed weight-gradient GEMM (ops/linear.py).  No LDS:
// each lane loads an 8x8 block as 8 row pieces of 16 bytes, transposes it in
// registers (32 byte permutes) and stores 8 column pieces of 16 bytes.  Lanes
// (cb = lane & 7, rb = lane >> 3) are laid out so every load instruction reads
// 8 whole 128-byte row segments and every store writes 8 whole 128-byte output
// row segments: both directions move full cache lines.
//
// gpu_sleep: one wave spins on s_memrealtime (100 MHz constant clock) for the
// requested time.  Used by the stream-overlap tests (upstream conftest's
// cuda_sleep idea): two sleeps on streams that truly overlap take ~max, not sum.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {
__global__ void sleep_kernel(uint64_t ticks) {
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  // Bounded spin: exits after `ticks` of the 100 MHz real-time counter.
  while (__builtin_amdgcn_s_memrealtime() - start < ticks) {
    __builtin_amdgcn_s_sleep(8);
  }
}
// One wave per 64x64 tile; a block's 4 waves take 4 neighbouring column tiles.
__global__ __launch_bounds__(256) void transpose_b16_kernel(const uint16_t* __restrict__ x, int64_t rows,
                                                            int64_t cols, int64_t ldx, uint16_t* __restrict__ out,
                                                            int64_t ldo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 64 + 8 * (lane >> 3);
  const int64_t c = ((int64_t)blockIdx.y * 4 + wave) * 64 + 8 * (lane & 7);
  if (r >= rows || c >= cols) return;  // rows, cols are multiples of 8
  uint4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const uint4*>(x + (r + i) * ldx + c);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(v);  // w[4 i + d] = (x[r+i][c+2d], x[r+i][c+2d+1])
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint4 lo, hi;  // output rows c + 2d (low halves) and c + 2d + 1 (high halves)
    uint32_t* pl = reinterpret_cast<uint32_t*>(&lo);
    uint32_t* ph = reinterpret_cast<uint32_t*>(&hi);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = w[4 * (2 * k) + d], b = w[4 * (2 * k + 1) + d];
      pl[k] = (a & 0xffffu) | (b << 16);
      ph[k] = (a >> 16) | (b & 0xffff0000u);
    }
    *reinterpret_cast<uint4*>(out + (c + 2 * d) * ldo + r) = lo;
    *reinterpret_cast<uint4*>(out + (c + 2 * d + 1) * ldo + r) = hi;
  }
}
}  // namespace

void transpose_b16(const uint16_t* x, int64_t rows, int64_t cols, int64_t ldx, uint16_t* out, int64_t ldo,
                   hipStream_t s) {
  if (rows <= 0 || cols <= 0) return;
  const dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((cols + 255) / 256));
  hipLaunchKernelGGL(transpose_b16_kernel, grid, dim3(256), 0, s, x, rows, cols, ldx, out, ldo);
}

void gpu_sleep(int64_t microseconds, hipStream_t s) {
  if (microseconds <= 0) return;
  const uint64_t ticks = (uint64_t)microseconds * 100ull;  // 100 MHz
  hipLaunchKernelGGL(sleep_kernel, dim3(1), dim3(64), 0, s, ticks);
}

}  // namespace mipipe
