// The eight-wave ping-pong GEMM (k_gemm_w8): C[M,N] = epi(A[M,K] . W[N,K]^T) on 16-bit operands,
// dispatched from rf_gemm.hip (knob gemm_w8). Replaces the same nn.Linear addmm's as k_gemm_w4
// (TF:504-506, 1064-1069, 1107-1116, 1123-1128 via recformer/models.py:335-343).
#include <type_traits>

#include "rf_common.h"
#include "rf_gemm_epi.h"

namespace rf {
// ---- 8-wave 256x256 GEMM: two waves per SIMD in ping-pong (knob gemm_w8) -----------------------
// The four-wave kernel above issues its 16 operand DMA pieces and 32 fragment reads per K-tile inside
// its own MFMA stream; with one wave per SIMD each piece's issue stalls that stream (tools/micro/
// mfma_dma.hip, profiles/r06/micro_mfma_dma.txt: the w4 K-loop shape runs 3,286 cycles per K-tile for
// 2,048 of MFMAs, eff 0.62; 2,782 without any DMA). Here each SIMD holds two waves of one 512-thread
// workgroup, one from each group (waves 0-3, 4-7), and the groups alternate roles segment by segment,
// one s_barrier apart: while a wave runs the 64 MFMAs of its 128 x 64 block for one K-tile (both k-steps,
// operands already in registers), its partner issues its share of the operand DMA, reads its fragments
// of the next K-tile and runs any epilogue (same micro-benchmark: 2,156 cycles per K-tile, eff 0.95).
// Step m = (tile T, K-tile kt) of this workgroup's persistent sequence; buffer m & 1.
//   segment 2m:   group 0 computes m     | group 1 reads m's fragments, DMAs the W rows of m + 1
//   segment 2m+1: group 1 computes m     | group 0 reads m+1's fragments, DMAs the A rows of m + 2
// (a buffer is refilled only after both groups read it; every DMA lands, counted vmcnt, before the
// barrier that ends its issuing segment). A tile's epilogue runs in each group's load segment right
// after its last compute, beside the partner's MFMAs. Wave (group g, local l): rows 128 (l >> 1) ..,
// columns 64 (2 g + (l & 1)) ..; the W image rows are permuted so a lane owns 4 consecutive output
// columns (8-B stores, 16 lanes = one 128-B line per row). Same LDS image and swizzle as k_gemm_w4.
constexpr int W8_BUF = 4 * PP_HALF;   // one K-tile: A rows 0-255 | W image rows 0-255
constexpr int W8_CV = 2 * W8_BUF;     // column vectors [parity][1 KiB]
constexpr int W8_LDS = W8_CV + 2 * 1024;

template <typename E, int EPI>
__global__ void __launch_bounds__(512, 2)
    k_gemm_w8(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e, int nTm,
              int nTn) {
  typedef typename H16<E>::x8 V8;
  static_assert(EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU,
                "k_gemm_w8: 16-bit EPI_NONE / EPI_BIAS / EPI_BIAS_GELU");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = nTm * nTn;
  if ((int)blockIdx.x >= tiles) return;
  const int GN = e.gn > 0 ? min(e.gn, nTn) : nTn;
  auto tile_origin = [&](int vv, int& om0, int& on0) {
    const int wg = xcd_remap(vv, tiles);
    const int g = wg / (nTm * GN);
    const int gw = min(GN, nTn - g * GN);
    const int rem = wg - g * nTm * GN;
    const int tm = rem / gw;
    om0 = tm * 256;
    on0 = (g * GN + rem - tm * gw) * 256;
  };
  const int ntile = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // tiles of this WG
  const int nk = K >> 6;
  const int J = ntile * nk;  // steps
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wl = wave & 3;
  const int wr = wl >> 1, wq = 2 * grp + (wl & 1);  // compute block: rows 128 wr, columns 64 wq
  // DMA role: group 0 stages A rows 64 wl + 8 p + lane / 8, group 1 the W image rows 64 wl + 8 p + lane / 8
  // = W rows 64 wl + 32 (p & 1) + 4 (lane / 8) + (p >> 1) (image row 64 q + 16 j + c holds W row 64 q + 4 c + j)
  const __amdgpu_buffer_rsrc_t rs =
      grp == 0 ? __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0,
                                                   (int)min((int64_t)e.M * lda * 2, (int64_t)0x7FFFFFFF), 0x00020000)
               : __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0,
                                                   (int)min((int64_t)e.N * ldw * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const int ldo = grp == 0 ? lda : ldw;
  const int pch = ((lane & 7) ^ (lane >> 3)) * 8;
  const int drow = grp == 0 ? 64 * wl + (lane >> 3) : 64 * wl + 4 * (lane >> 3);
  char* dbase = smem + (grp == 0 ? 0 : 2 * PP_HALF) + 64 * wl * 128;
  // the operand rows (A: tile row origin, W: tile column origin) and K-tile of step s
  auto step_tile = [&](int s, int& om0, int& on0, int& kt) {
    const int T = s / nk;
    kt = s - T * nk;
    tile_origin((int)blockIdx.x + T * (int)gridDim.x, om0, on0);
  };
  auto dma_step = [&](int s) {  // this wave's 8 pieces of step s into buffer s & 1
    int om0, on0, kt;
    step_tile(s, om0, on0, kt);
    const int vo = ((grp == 0 ? om0 : on0) + drow) * ldo * 2 + pch * 2;
    char* dst = dbase + (s & 1) * W8_BUF;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int roff = grp == 0 ? 8 * p : 32 * (p & 1) + (p >> 1);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + 8 * p * 128), 16,
                                               vo, kt * 128 + roff * ldo * 2, 0, 0);
    }
  };
  auto dma_cols = [&](int s) {  // wave 0: the column vector of step s's tile into its parity slot
    if (EPI == RF_EPI_NONE) return;
    int om0, on0, kt;
    step_tile(s, om0, on0, kt);
    glds16(e.bias + min(on0 + 4 * lane, e.N - 4), smem + W8_CV + ((s / nk) & 1) * 1024);
  };
  const int lr = lane & 15;
  const int off0 = lr * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
  const int off1 = lr * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  const int aOff = wr * PP_HALF + off0, bOff = 2 * PP_HALF + wq * 64 * 128 + off0;
  const int dks = off1 - off0;
  V8 a0[8], a1[8], b0[4], b1[4];
  f32x4 acc[8][4];
  auto read_step = [&](int s) {
    const char* base = smem + (s & 1) * W8_BUF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b0[j] = *reinterpret_cast<const V8*>(base + bOff + j * 16 * 128);
      b1[j] = *reinterpret_cast<const V8*>(base + bOff + j * 16 * 128 + dks);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a0[i] = *reinterpret_cast<const V8*>(base + aOff + i * 16 * 128);
      a1[i] = *reinterpret_cast<const V8*>(base + aOff + i * 16 * 128 + dks);
    }
  };
  auto compute = [&](bool first) {
    __builtin_amdgcn_s_setprio(1);
    if (first) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a0[i], b0[j], f32x4{0.f, 0.f, 0.f, 0.f});
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int NST = 32;  // epilogue stores per wave (interior tile): 8 blocks x 4 rows
  // epilogue of the tile of step s (its last K-tile just computed): lane (c = l & 15, g = l >> 4) holds
  // rows 4 g + r of each 16-row block i and the output columns 4 c .. 4 c + 3 of the wave's 64
  auto epilogue = [&](int s) {
    int m0, n0, kt;
    step_tile(s, m0, n0, kt);
    const bool interior = (m0 + 256 <= e.M) && (n0 + 256 <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    const int erow = m0 + wr * 128 + 4 * (el >> 4);
    const int ecol = n0 + wq * 64 + 4 * (el & 15);
    float bv[4], gm[4], bt[4];
    const float* cb = reinterpret_cast<const float*>(smem + W8_CV + ((s / nk) & 1) * 1024);
    lds_cols<EPI, 4>(cb, ecol - n0, bv, gm, bt);
    constexpr bool FSC = EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU;
    float csc = 1.f;
    if (FSC) {
      csc = ecol < e.scale_cols ? e.col_scale : 1.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) bv[k] *= csc;
    }
    const void* tbase = reinterpret_cast<const E*>(e.C) + (int64_t)m0 * e.ldc;
    auto body = [&](auto check) {
      constexpr bool CK = decltype(check)::value;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float vv[4] = {acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]};
          epi_seg<E, EPI, false, false, 4, CK, !CK, FSC>(e, erow + i * 16 + r, ecol, vv, bv, gm, bt, 0.f, tbase, m0,
                                                         csc);
        }
    };
    if (interior) body(std::false_type{});
    else body(std::true_type{});
    return interior ? NST : 0;
  };
  auto wait_lgkm0 = []() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  // the counted wait of a load segment: its DMA pieces (issued first) landed, the epilogue's stores
  // (issued after them) may stay in flight
  auto wait_dma = [&](int nst) {
    if (nst >= NST) wait_vmcnt<NST>();
    else wait_vmcnt<0>();
  };

  // prologue: step 0 (both operands), tile 0's column vector; group 0 reads step 0 and DMAs A of step 1.
  // Both groups then run the same loop shape (load segment, barrier, compute segment, barrier; only the
  // accumulators are carried across iterations), group 0 one segment ahead: it computes step 0 first.
  dma_step(0);
  if (wave == 0) dma_cols(0);
  wait_vmcnt<0>();
  bar();
  if (grp == 0) {
    if (J > 1) dma_step(1);
    read_step(0);
    wait_lgkm0();
    wait_vmcnt<0>();
  }
  bar();
  if (grp == 0) {
    compute(true);
    bar();
  }
  // group 0's iteration m: load segment of step m (A of m + 1, epilogue of m - 1 if it ended a tile, the
  // fragments of m) beside group 1's compute of m - 1, then its compute of m beside group 1's load of m.
  // Group 1's iteration m: load segment of step m (W of m + 1, epilogue of m - 1, fragments of m) beside
  // group 0's compute of m, then its compute of m beside group 0's load of m + 1.
  for (int m = grp == 0 ? 1 : 0; m < J; ++m) {
    const int kt = m % nk;
    if (m + 1 < J) dma_step(m + 1);
    // the next tile's column vector (wave 0, at the tile's second K-tile: its parity slot was last read by
    // group 1's epilogue of the tile before, one segment earlier; nk >= 2)
    if (wave == 0 && kt == 1 && m - 1 + nk < J) dma_cols(m - 1 + nk);
    int nst = 0;
    if (kt == 0 && m > 0) nst = epilogue(m - 1);
    if (kt == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);  // the fragment reads after the epilogue (register pressure)
    read_step(m);
    wait_lgkm0();
    wait_dma(nst);
    bar();
    compute(false);
    bar();
  }
  if (grp == 0) {  // group 0's last load segment: the last tile's epilogue, beside group 1's last compute
    epilogue(J - 1);
    bar();
  } else {
    epilogue(J - 1);
  }
  wait_vmcnt<0>();
}

template <typename E, int EPI>
void launch_w8(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                      hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_w8<E, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)W8_LDS);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 255) / 256;
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_w8<E, EPI><<<grid, 512, W8_LDS, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm, nTn);
}

#define RF_W8_INST(E, EPI)                                                                                     \
  template void launch_w8<E, EPI>(int, int, int, const void*, int, const void*, int, const EpiArgs&, hipStream_t);
RF_W8_INST(bf16, RF_EPI_NONE)
RF_W8_INST(bf16, RF_EPI_BIAS)
RF_W8_INST(bf16, RF_EPI_BIAS_GELU)
RF_W8_INST(f16, RF_EPI_NONE)
RF_W8_INST(f16, RF_EPI_BIAS)
RF_W8_INST(f16, RF_EPI_BIAS_GELU)
#undef RF_W8_INST

}  // namespace rf
