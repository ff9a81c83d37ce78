// Micro-benchmark: bf16 output-tile store patterns of a 256x256-tile GEMM epilogue.
// Each of 256 persistent workgroups (512 threads, 8 waves of 128x64 sub-tiles) writes its
// tiles of an M x N bf16 matrix.  pattern 0: lane = (row l&15, 16 cols at 16(l>>4)), two
// 16-B stores (the MFMA-native row-vector layout); pattern 1: lane = (row l>>3 (+8), 8 cols at
// 8(l&7)), each instruction 8 full 128-B row segments.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int P>
__global__ void __launch_bounds__(512) k_store(__bf16* C, int M, int N, int nTn, int tiles) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = wave >> 2, wc = wave & 3;
  bf16x8 val;
  for (int k = 0; k < 8; ++k) val[k] = (__bf16)(float)(lane + k);
  for (int v = blockIdx.x; v < tiles; v += gridDim.x) {
    const int tm = v / nTn, tn = v % nTn;
    const int r0 = tm * 256 + wr * 128, c0 = tn * 256 + wc * 64;
    for (int mf = 0; mf < 8; ++mf) {
      if (P == 0) {
        __bf16* p = C + (size_t)(r0 + mf * 16 + (lane & 15)) * N + c0 + 16 * (lane >> 4);
        *reinterpret_cast<bf16x8*>(p) = val;
        *reinterpret_cast<bf16x8*>(p + 8) = val;
      } else if (P == 2) {
        // MFMA-native non-swapped layout with a 4-column W permutation: lane (c = l&15, g = l>>4)
        // holds 4 consecutive columns 4c.. of rows 4g + r: one 8-B store per r, 4 full rows
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v4;
        for (int k = 0; k < 4; ++k) v4[k] = val[k];
        for (int r = 0; r < 4; ++r) {
          __bf16* p = C + (size_t)(r0 + mf * 16 + 4 * (lane >> 4) + r) * N + c0 + 4 * (lane & 15);
          *reinterpret_cast<bf16x4*>(p) = v4;
        }
      } else {
        for (int h = 0; h < 2; ++h) {
          __bf16* p = C + (size_t)(r0 + mf * 16 + 8 * h + (lane >> 3)) * N + c0 + 8 * (lane & 7);
          *reinterpret_cast<bf16x8*>(p) = val;
        }
      }
    }
  }
}

int main() {
  const int M = 65536, N = 3072, nTn = N / 256, tiles = (M / 256) * nTn;
  __bf16* C;
  hipMalloc(&C, (size_t)M * N * 2);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int P = 0; P < 3; ++P) {
    for (int grid : {32, 64, 128, 256}) {
      for (int it = 0; it < 3; ++it) {
        if (P == 0) k_store<0><<<grid, 512>>>(C, M, N, nTn, tiles);
        else if (P == 1) k_store<1><<<grid, 512>>>(C, M, N, nTn, tiles);
        else k_store<2><<<grid, 512>>>(C, M, N, nTn, tiles);
      }
      hipEventRecord(a);
      for (int it = 0; it < 10; ++it) {
        if (P == 0) k_store<0><<<grid, 512>>>(C, M, N, nTn, tiles);
        else if (P == 1) k_store<1><<<grid, 512>>>(C, M, N, nTn, tiles);
        else k_store<2><<<grid, 512>>>(C, M, N, nTn, tiles);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 10;
      printf("pattern %d grid %4d: %.1f us  %.0f GB/s\n", P, grid, ms * 1e3, (double)M * N * 2 / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
