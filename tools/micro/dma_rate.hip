// Micro-benchmark: per-CU L2->LDS (global_load_lds_dwordx4), L2->VGPR (global_load_dwordx4) and
// L2->VGPR->LDS (global_load_dwordx4 + ds_write_b128) throughput. 256 workgroups of 4 or 8 waves;
// each wave streams 1-KiB pieces of a 2 MiB L2-resident window, `depth` instructions per round.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/dma_rate tools/micro/dma_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE, int DEPTH, int NW>
__global__ void __launch_bounds__(512) k_dma(const char* src, int iters, unsigned long long* cyc, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each block reads a 2 MiB window (L2 resident after warmup), offset per block
  const char* base = src + (size_t)(blockIdx.x & 7) * (2 << 20);
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  typedef float f4v __attribute__((ext_vector_type(4)));
  for (int it = 0; it < iters; ++it) {
    f4v xs[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const size_t off = ((size_t)((it * DEPTH + d) * NW + wave) * 1024 + lane * 16) & ((2 << 20) - 1);
      if (MODE == 0) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off),
                                         (__attribute__((address_space(3))) void*)(smem + (wave * DEPTH + d) * 1024),
                                         16, 0, 0);
      } else if (MODE == 1) {
        const float4 x = *reinterpret_cast<const float4*>(base + off);
        acc += x.x + x.y + x.z + x.w;
      } else {
        xs[d] = *reinterpret_cast<const f4v*>(base + off);  // all DEPTH loads in flight, then the LDS stores
      }
    }
    if (MODE == 2) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        f4v x = xs[d];
        asm volatile("" : "+v"(x));  // keep every load and its LDS store
        const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(smem + (wave * DEPTH + d) * 1024 + lane * 16);
        asm volatile("ds_write_b128 %0, %1" ::"v"(la), "v"(x) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (MODE == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (acc == 12345.f) sink[0] = acc;
}

template <int MODE, int DEPTH, int NW>
void run(const char* src, unsigned long long* cyc, float* sink) {
  const int iters = 2000;
  hipLaunchKernelGGL((k_dma<MODE, DEPTH, NW>), dim3(256), dim3(64 * NW), NW * DEPTH * 1024, 0, src, iters, cyc, sink);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_dma<MODE, DEPTH, NW>), dim3(256), dim3(64 * NW), NW * DEPTH * 1024, 0, src, iters, cyc, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double mc = 0; for (int i = 0; i < 256; ++i) mc += h[i]; mc /= 256;
  const double bytes_cu = (double)iters * DEPTH * NW * 1024;
  printf("mode %s waves %d depth %2d: %.1f us, %.1f B/cycle/CU (memtime), %.1f GB/s per CU, chip %.1f TB/s\n",
         MODE == 0 ? "glds     " : (MODE == 1 ? "vgpr     " : "vgpr+ds_w"), NW, DEPTH, ms * 1e3, bytes_cu / mc,
         bytes_cu / (ms * 1e-3) / 1e9, bytes_cu * 256 / (ms * 1e-3) / 1e12);
}

int main() {
  char* src; unsigned long long* cyc; float* sink;
  (void)hipMalloc(&src, 16 << 20); (void)hipMemset(src, 1, 16 << 20);
  (void)hipMalloc(&cyc, 256 * 8); (void)hipMalloc(&sink, 4);
  run<0, 2, 4>(src, cyc, sink); run<0, 4, 4>(src, cyc, sink); run<0, 8, 4>(src, cyc, sink); run<0, 16, 4>(src, cyc, sink);
  run<1, 2, 4>(src, cyc, sink); run<1, 4, 4>(src, cyc, sink); run<1, 8, 4>(src, cyc, sink); run<1, 16, 4>(src, cyc, sink);
  run<2, 2, 4>(src, cyc, sink); run<2, 4, 4>(src, cyc, sink); run<2, 8, 4>(src, cyc, sink); run<2, 16, 4>(src, cyc, sink);
  run<0, 4, 8>(src, cyc, sink); run<0, 8, 8>(src, cyc, sink); run<1, 4, 8>(src, cyc, sink); run<2, 4, 8>(src, cyc, sink);
  return 0;
}
