// Micro-benchmark: how much operand LDS-DMA issue costs an MFMA stream, at one and at two waves per
// SIMD (the question behind the GEMM's two-waves-per-SIMD variant).
//
// Each wave runs K-tile iterations shaped like k_gemm_w4's K-loop: phase A = NJ*8 v_mfma_f32_16x16x32_bf16
// on register operands set 0 while (8 + NJ) ds_read_b128 fetch set 1 and PA LDS-DMA pieces (1 KiB
// each) are issued; wait lgkmcnt(0) + vmcnt + s_barrier; phase B = the same on set 1 / set 0 with PB
// pieces. Mode 1 (ping-pong, 8 waves): waves 0-3 and 4-7 alternate a compute segment (both phases'
// MFMAs) and a load segment (all reads + pieces, then waits), one barrier between segments.
// The DMA streams from a per-XCD window (L2-resident at 2 MiB, partly Infinity Cache at 8 MiB).
// Printed: shader cycles per iteration (s_memtime, median over workgroups; the ideal is 16 cycles per
// MFMA per SIMD = 2048 for 128 MFMAs per SIMD) and MFMA TF/s from the wall time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_dma tools/micro/mfma_dma.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int NW, int NJ, int PA, int PB, int MODE, int WIN_MB>
__global__ void __launch_bounds__(NW * 64, NW / 4) k_mfma_dma(const char* src, int iters, unsigned long long* cyc,
                                                             float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NR = 8 + NJ;  // fragment reads per phase
  // read region: 64 KiB of operand image (random bf16 copied in), DMA region behind it
  char* rd = smem;
  char* dm = smem + 65536;
  for (int i = threadIdx.x; i < 65536 / 16; i += NW * 64)
    *reinterpret_cast<float4*>(rd + i * 16) = *reinterpret_cast<const float4*>(src + (size_t)i * 16);
  __syncthreads();
  const size_t win = (size_t)WIN_MB << 20;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(src + (size_t)(blockIdx.x & 7) * win), (short)0, (int)win, 0x00020000);
  const int off0 = (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
  const int off1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  bf16x8 a0[8], b0[NJ], a1[8], b1[NJ];
  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a0[i] = *reinterpret_cast<const bf16x8*>(rd + i * 2048 + off0);
    a1[i] = a0[i];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    b0[j] = *reinterpret_cast<const bf16x8*>(rd + 32768 + j * 2048 + off0);
    b1[j] = b0[j];
  }
  int voff = (int)(((blockIdx.x >> 3) * 4096 + wave * 64 + lane) * 16 % win);
  int piece = 0;
  auto dma = [&](int p) {
    char* dst = dm + ((wave * 16 + p) & 63) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, voff,
                                             ((piece++) * NW * 1024) & (int)(win - 1) & ~1023, 0, 0);
  };
  auto rd0 = [&](int i) {
    const char* b = rd + (i < 8 ? i * 2048 : 32768 + (i - 8) * 2048) + off0;
    if (i < 8) a0[i] = *reinterpret_cast<const bf16x8*>(b);
    else b0[i - 8] = *reinterpret_cast<const bf16x8*>(b);
  };
  auto rd1 = [&](int i) {
    const char* b = rd + (i < 8 ? i * 2048 : 32768 + (i - 8) * 2048) + off1;
    if (i < 8) a1[i] = *reinterpret_cast<const bf16x8*>(b);
    else b1[i - 8] = *reinterpret_cast<const bf16x8*>(b);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
      // phase A: MFMAs on set 0, reads of set 1, PA pieces
#pragma unroll
      for (int p = 0; p < (PA > NR ? PA : NR); ++p) {
        if (p < PA) dma(p);
        if (p < NR) rd1(p);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
#pragma unroll
      for (int g = 0; g < NR; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, (8 * NJ) / NR > 0 ? (8 * NJ) / NR : 1, 0);
        if (g < PA) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      // phase B: MFMAs on set 1, reads of set 0, PB pieces
#pragma unroll
      for (int p = 0; p < (PB > NR ? PB : NR); ++p) {
        if (p < PB) dma(p + PA);
        if (p < NR) rd0(p);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
#pragma unroll
      for (int g = 0; g < NR; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, (8 * NJ) / NR > 0 ? (8 * NJ) / NR : 1, 0);
        if (g < PB) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else {
    // ping-pong: group g = wave >> 2; group 1 starts with a load segment
    const int grp = wave >> 2;
    auto compute = [&]() {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
    };
    auto load = [&]() {
#pragma unroll
      for (int p = 0; p < (PA + PB > NR ? PA + PB : NR); ++p) {
        if (p < PA + PB) dma(p);
        if (p < NR) { rd0(p); rd1(p); }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    // group 0: compute, bar, load, bar, ...; group 1: load, bar, compute, bar, ... (same barrier count)
    if (grp == 1) {
      load();
      bar();
    }
    for (int it = 0; it < iters; ++it) {
      __builtin_amdgcn_s_setprio(1);
      compute();
      __builtin_amdgcn_s_setprio(0);
      bar();
      load();
      bar();
    }
    if (grp == 0) bar();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 1234.5f) sink[threadIdx.x] = s;
}

template <int NW, int NJ, int PA, int PB, int MODE, int WIN_MB>
void run(const char* label, const char* src, unsigned long long* cyc, float* sink) {
  const int iters = 3000;
  const int grid = 256;
  const size_t lds = 65536 + 65536;
  auto k = k_mfma_dma<NW, NJ, PA, PB, MODE, WIN_MB>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, 0, src, iters, cyc, sink);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, 0, src, iters, cyc, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  std::vector<unsigned long long> h(grid);
  hipMemcpy(h.data(), cyc, grid * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double cyc_it = (double)h[grid / 2] / iters;
  const double mfma_simd = (double)NW / 4 * 16 * NJ;  // MFMAs per SIMD per iteration
  const double flops = (double)grid * NW * 16 * NJ * 16384.0 * iters;
  const double pieces_cu = (double)NW * (PA + PB);
  printf("%-34s waves %d NJ %d pieces/wave %2d win %dMiB: %7.0f cyc/iter (ideal %5.0f, eff %.3f) %6.0f TF/s  "
         "DMA %5.1f B/cyc/CU  clk %.2f GHz\n",
         label, NW, NJ, PA + PB, WIN_MB, cyc_it, mfma_simd * 16, mfma_simd * 16 / cyc_it, flops / (ms * 1e-3) / 1e12,
         pieces_cu * 1024 / cyc_it, cyc_it * iters / (ms * 1e-3) / 1e9);
}

int main() {
  char* src;
  unsigned long long* cyc;
  float* sink;
  const size_t bytes = (size_t)8 * (8 << 20) + (1 << 20);
  (void)hipMalloc(&src, bytes);
  std::vector<unsigned short> h(bytes / 2);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (unsigned short)(0x3c00 + ((x >> 16) & 0x3ff) - 0x200) ^ ((x >> 8) & 0x8000);  // bf16 ~ +-[0.4, 1.6]
  }
  hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice);
  (void)hipMalloc(&cyc, 256 * 8);
  (void)hipMalloc(&sink, 512 * 4);
  run<4, 8, 0, 0, 0, 2>("w4 no DMA", src, cyc, sink);
  run<4, 8, 0, 16, 0, 2>("w4 16 pieces in phase B", src, cyc, sink);
  run<4, 8, 8, 8, 0, 2>("w4 8+8 pieces", src, cyc, sink);
  run<4, 8, 0, 16, 0, 8>("w4 16 pieces in phase B", src, cyc, sink);
  run<4, 8, 8, 8, 0, 8>("w4 8+8 pieces", src, cyc, sink);
  run<8, 4, 0, 0, 0, 2>("w8 coop no DMA", src, cyc, sink);
  run<8, 4, 0, 8, 0, 2>("w8 coop 8 pieces in phase B", src, cyc, sink);
  run<8, 4, 4, 4, 0, 2>("w8 coop 4+4 pieces", src, cyc, sink);
  run<8, 4, 0, 8, 0, 8>("w8 coop 8 pieces in phase B", src, cyc, sink);
  run<8, 4, 4, 4, 0, 8>("w8 coop 4+4 pieces", src, cyc, sink);
  run<8, 4, 0, 0, 1, 2>("w8 ping-pong no DMA", src, cyc, sink);
  run<8, 4, 0, 8, 1, 2>("w8 ping-pong 8 pieces", src, cyc, sink);
  run<8, 4, 0, 8, 1, 8>("w8 ping-pong 8 pieces", src, cyc, sink);
  run<4, 8, 0, 16, 0, 2>("w4 16 pieces in phase B (again)", src, cyc, sink);
  return 0;
}
