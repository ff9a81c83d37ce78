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
#if defined(RF_W8_STAMPS)
constexpr int W8_NSTAMP = 128;
constexpr int W8_LDS = W8_CV + 2 * 1024 + 2 * W8_NSTAMP * 8;
#else
constexpr int W8_LDS = W8_CV + 2 * 1024;
#endif

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
  // origin of this workgroup's T-th tile (xcd-aware raster as k_gemm_w4); evaluated once per tile
  auto tile_origin = [&](int T, int& om0, int& on0) {
    const int wg = xcd_remap((int)blockIdx.x + T * (int)gridDim.x, tiles);
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
  // Operand DMA of step s (into buffer s & 1), each piece 8 image rows x 128 B, lane: row + lane / 8,
  // 16-B chunk (lane & 7) ^ (row & 7) from the source (the read swizzle). Group g stages the rows
  // 128 g + 32 wl + 8 p (p < 4) of the A image and of the W image, 4 + 4 pieces per wave and step: its
  // W half (the image rows of its own columns) and its A half during its load segment of step s - 1,
  // except that group 1's A half (rows 128-255, which group 0 reads one segment before group 1) goes out
  // at the start of its compute segment of step s - 2 (the buffer's previous step was read by then). W image
  // row r = 64 q + 16 j + c holds W row 64 q + 4 c + j, so lane (r0 + lane / 8) of a piece at r0 (a
  // multiple of 8) reads W row 4 (lane / 8) + wrow(r0). Every piece has two segments to land before its
  // first reader: the issuing wave waits for it (counted vmcnt) at the end of its following segment.
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)min((int64_t)e.M * lda * 2, (int64_t)0x7FFFFFFF),
                                        0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)min((int64_t)e.N * ldw * 2, (int64_t)0x7FFFFFFF),
                                        0x00020000);
  const int pch = ((lane & 7) ^ (lane >> 3)) * 8;
  const int r0g = 128 * grp + 32 * wl;                         // this wave's first A / W image row
  const int voA = ((r0g + (lane >> 3)) * lda + pch) * 2;      // + tile row origin * lda * 2
  const int voW = (4 * (lane >> 3) * ldw + pch) * 2;           // + (tile column origin + wrow) * ldw * 2
  auto wrow = [](int r0) { return 64 * (r0 >> 6) + 4 * (r0 & 15) + ((r0 >> 4) & 3); };
  auto dma_A = [&](int s, int om0, int kt) {
    char* buf = smem + (s & 1) * W8_BUF;
    const int vo = voA + om0 * lda * 2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int so = kt * 128 + 8 * p * lda * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(buf + (r0g + 8 * p) * 128),
                                               16, vo, so, 0, 0);
    }
  };
  auto dma_W = [&](int s, int on0, int kt) {
    char* buf = smem + (s & 1) * W8_BUF + 2 * PP_HALF;
    const int vw = voW + on0 * ldw * 2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r0 = r0g + 8 * p;
      const int so = kt * 128 + wrow(r0) * ldw * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (__attribute__((address_space(3))) void*)(buf + r0 * 128), 16,
                                               vw, so, 0, 0);
    }
  };
  auto dma_cols = [&](int T, int on0) {  // wave 0: tile T's column vector into its parity slot
    if (EPI == RF_EPI_NONE) return;
    glds16(e.bias + min(on0 + 4 * lane, e.N - 4), smem + W8_CV + (T & 1) * 1024);
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
  auto compute = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
#if defined(RF_W8_STAMPS)  // diagnostic build (tools/w8_stamps.py): waves 0 and 4 stamp s_memtime around
  // every barrier into LDS (no vector-memory op, so the counted vmcnt waits stay exact), flushed at the end
  unsigned long long* lst = reinterpret_cast<unsigned long long*>(smem + W8_CV + 2048) + grp * W8_NSTAMP;
  int nstp = 0;
  auto stamp = [&]() {
    if (wl == 0 && nstp < W8_NSTAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) lst[nstp] = t;
    }
    ++nstp;
  };
#else
  auto stamp = [&]() {};
#endif
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    stamp();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stamp();
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int NST = 32;  // epilogue stores per wave (interior tile): 8 blocks x 4 rows
  // epilogue of tile T at (m0, n0): lane (c = l & 15, g = l >> 4) holds rows 4 g + r of each 16-row block
  // i and the output columns 4 c .. 4 c + 3 of the wave's 64. Returns the stores it left in flight.
  auto epilogue = [&](int T, int m0, int n0) {
    const bool interior = (m0 + 256 <= e.M) && (n0 + 256 <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    const int erow = m0 + wr * 128 + 4 * (el >> 4);
    const int ecol = n0 + wq * 64 + 4 * (el & 15);
    float bv[4], gm[4], bt[4];
    const float* cb = reinterpret_cast<const float*>(smem + W8_CV + (T & 1) * 1024);
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
  // counted wait: every vector-memory op of this wave but the `younger` newest has completed (DMA pieces
  // come in fours, an interior epilogue issues NST stores)
  auto wait_n = [&](int younger) {
    switch (younger) {
      case 4: wait_vmcnt<4>(); break;
      case 8: wait_vmcnt<8>(); break;
      case NST: wait_vmcnt<NST>(); break;
      case NST + 4: wait_vmcnt<NST + 4>(); break;
      case NST + 8: wait_vmcnt<NST + 8>(); break;
      default: wait_vmcnt<0>(); break;
    }
  };

  // tile bookkeeping of step m (read / computed this iteration): its tile T and origin, the tile before
  // (for its epilogue) and the tile after (for the DMA of steps m + 1, m + 2 and the next column vector)
  int T = 0, kt = 0, cm0, cn0, pm0 = 0, pn0 = 0, nm0 = 0, nn0 = 0;
  tile_origin(0, cm0, cn0);
  if (ntile > 1) tile_origin(1, nm0, nn0);
  // prologue: step 0 (every wave its halves), tile 0's column vector; then step 1 (group 0 its halves, group 1
  // its A half, which must land before group 0 reads step 1) while group 0 reads step 0; group 0 computes
  // step 0 (one segment ahead of group 1)
  dma_A(0, cm0, 0);
  dma_W(0, cn0, 0);
  if (wave == 0) dma_cols(0, cn0);
  wait_vmcnt<0>();
  bar();
  if (J > 1) {
    const bool same = nk > 1;
    dma_A(1, same ? cm0 : nm0, same ? 1 : 0);
    if (grp == 0) dma_W(1, same ? cn0 : nn0, same ? 1 : 0);
  }
  if (grp == 0) {
    read_step(0);
    wait_lgkm0();
  }
  bar();
  int nst = 0;
  zero_acc();  // tile 0 (later tiles: after each epilogue)
  if (grp == 0) {
    compute();
    wait_vmcnt<0>();
    bar();
  }
  // Iteration m: the load segment of step m (beside the partner's compute: group 0's beside group 1's
  // compute of m - 1, group 1's beside group 0's compute of m) — the DMA of step m + 1, the previous
  // tile's epilogue when step m starts a tile, the fragments of step m — then the compute segment of
  // step m (group 1: headed by its A half of step m + 2). Only the accumulators are carried across
  // iterations.
  const int m_first = grp == 0 ? 1 : 0;
  for (int m = m_first; m < J; ++m) {
    if (m > 0) kt = kt + 1 == nk ? 0 : kt + 1;  // kt = m % nk (kt of step 0 set above)
    const bool tstart = kt == 0 && m > 0;
    if (tstart) {
      ++T;
      pm0 = cm0; pn0 = cn0;
      cm0 = nm0; cn0 = nn0;
      if (T + 1 < ntile) tile_origin(T + 1, nm0, nn0);
    }
    const bool n1 = m + 1 < J;
    if (n1) {
      const bool same = kt + 1 < nk;
      if (grp == 0) dma_A(m + 1, same ? cm0 : nm0, same ? kt + 1 : 0);
      dma_W(m + 1, same ? cn0 : nn0, same ? kt + 1 : 0);
    }
    // the next tile's column vector (wave 0, at the tile's second K-tile: its parity slot was last read by
    // group 1's epilogue of the tile before, one segment earlier; nk >= 2)
    if (wave == 0 && kt == 1 && T + 1 < ntile) dma_cols(T + 1, nn0);
    nst = 0;
    if (tstart) {
      nst = epilogue(T - 1, pm0, pn0);
      zero_acc();
    }
    __builtin_amdgcn_sched_barrier(0);  // the fragment reads after the epilogue (register pressure)
#if defined(RF_W8_LATE)
    // A/B: every wait in the load segment, before the reads: all but this segment's pieces and stores
    wait_n((n1 ? (grp == 0 ? 8 : 4) : 0) + nst);
    read_step(m);
#else
    read_step(m);
    if (grp == 1) wait_n((n1 ? 4 : 0) + nst);  // its A half of step m + 1 (issued a segment ago) landed
#endif
    wait_lgkm0();
    bar();
    bool n2 = false;
    if (grp == 1 && m + 2 < J) {
      const bool same = kt + 2 < nk;
      dma_A(m + 2, same ? cm0 : nm0, same ? kt + 2 : kt + 2 - nk);
      n2 = true;
    }
    compute();
#if !defined(RF_W8_LATE)
    wait_n(nst + (n2 ? 4 : 0));  // this wave's pieces of the load segment (step m + 1) landed
#endif
    bar();
  }
  if (grp == 0) {  // group 0's last load segment: the last tile's epilogue, beside group 1's last compute
    epilogue(T, cm0, cn0);
    bar();
  } else {
    epilogue(T, cm0, cn0);
  }
#if defined(RF_W8_STAMPS)
  if (e.stamps && wl == 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int i = lane; i < W8_NSTAMP; i += 64)
      e.stamps[((size_t)blockIdx.x * 2 + grp) * W8_NSTAMP + i] = i < nstp ? lst[i] : 0ull;
  }
#endif
  wait_vmcnt<0>();
}

template <typename E, int EPI>
static void launch_w8(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
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

// the entry rf_gemm.hip calls (a plain function: the kernel templates are instantiated implicitly here,
// as the dispatcher of rf_gemm.hip does for its own kernels)
void gemm_w8(bool half, int epi, int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
             hipStream_t s) {
  if (half) {
    if (epi == RF_EPI_NONE) launch_w8<f16, RF_EPI_NONE>(M, N, K, A, lda, W, ldw, e, s);
    else if (epi == RF_EPI_BIAS) launch_w8<f16, RF_EPI_BIAS>(M, N, K, A, lda, W, ldw, e, s);
    else launch_w8<f16, RF_EPI_BIAS_GELU>(M, N, K, A, lda, W, ldw, e, s);
  } else {
    if (epi == RF_EPI_NONE) launch_w8<bf16, RF_EPI_NONE>(M, N, K, A, lda, W, ldw, e, s);
    else if (epi == RF_EPI_BIAS) launch_w8<bf16, RF_EPI_BIAS>(M, N, K, A, lda, W, ldw, e, s);
    else launch_w8<bf16, RF_EPI_BIAS_GELU>(M, N, K, A, lda, W, ldw, e, s);
  }
}

}  // namespace rf

namespace rf {

// ---- the four-wave kernel on ks-split LDS planes (knob gemm_w4p) -----------------------------------------
// k_gemm_w4's 256 x 256 tile, 4 waves of 128 x 128 (one per SIMD), the same MFMA sequence per accumulator
// (so bit-identical outputs), with the operand image of a K-tile split by k-step: plane ks holds k
// [32 ks, 32 ks + 32) of the 256 A and the 256 W rows as 64-B rows (TileGeo<32>'s chunk swizzle). A plane is
// free as soon as every wave has read its fragments, so each phase refills the plane the PREVIOUS phase
// finished with: phase A(t) (MFMAs on k-step 0, reads of k-step 1 of K-tile t) DMAs plane 0 of K-tile t + 2;
// phase B(t) (k-step 1, reads of k-step 0 of t + 1) DMAs plane 1 of t + 2 — 8 pieces per wave per phase
// instead of 16 in phase B only (k_gemm_w4), with one barrier per phase, and every piece two barriers
// (three phases) ahead of its first read. tools/micro/mfma_dma.hip: the w4 loop shape runs 3,286 cycles
// per K-tile with its 16 pieces in one phase, 2,816 with 8 + 8 (2,782 without any DMA).
constexpr int WP_BUF = 4 * PP_HALF;       // one K-tile: plane 0 | plane 1, each A rows 0-255 | W image rows 0-255
constexpr int WP_PLANE = 2 * PP_HALF;     // 32 KiB: 512 rows x 64 B
constexpr int WP_CV = 2 * WP_BUF;         // column vectors [parity][3][1 KiB]
constexpr int WP_LDS = WP_CV + 6 * 1024;

template <typename E, int EPI, bool CF32>
__global__ void __launch_bounds__(256, 1)
    k_gemm_w4p(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e, int nTm,
               int nTn) {
  typedef typename H16<E>::x8 V8;
  constexpr bool RF32 = false;
  constexpr bool OUT32 = CF32 || EPI == RF_EPI_COS;
  constexpr int NJ = 8, TN = 256;
  constexpr int S = (OUT32 || EPI == RF_EPI_BIAS_GELU_AUX) ? 64 : 32;  // epilogue stores per wave (interior)
  constexpr int C = (EPI == RF_EPI_NONE || EPI == RF_EPI_DGELU) ? 0 : 1;  // column-vector DMA per wave and tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = nTm * nTn;
  int v = blockIdx.x;
  if (v >= tiles) return;
  const int GN = e.gn > 0 ? min(e.gn, nTn) : nTn;
  auto tile_origin = [&](int vv, int& om0, int& on0) {
    const int wg = xcd_remap(vv, tiles);
    const int g = wg / (nTm * GN);
    const int gw = min(GN, nTn - g * GN);
    const int rem = wg - g * nTm * GN;
    const int tm = rem / gw;
    om0 = tm * 256;
    on0 = (g * GN + rem - tm * gw) * TN;
  };
  int m0, n0, nm0 = 0, nn0 = 0;
  tile_origin(v, m0, n0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // compute block: A rows 128 wr, W image rows 128 wc
  const int nk = K >> 6;
  // DMA: a piece is 16 plane rows x 64 B (lane: row + lane / 4, 16-B slot lane & 3, fetched from source
  // chunk slot ^ f(row), f(r) = (-(r >> 2)) & 3 — TileGeo<32>'s swizzle, row = the plane row, a multiple of
  // 16 plus lane / 4). Wave w stages A rows 64 w .. 64 w + 63 (pieces p = 0..3) and the W image rows of
  // fragments f = 4 (w & 1) + p of W-half w >> 1 (image row 16 f + j of a half holds W row 8 j + f, or
  // 64 (f >> 2) + 4 j + (f & 3) for fp32 out: whole-line epilogue stores, as k_gemm_w4's wperm).
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)min((int64_t)e.M * lda * 2, (int64_t)0x7FFFFFFF),
                                        0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)min((int64_t)e.N * ldw * 2, (int64_t)0x7FFFFFFF),
                                        0x00020000);
  const int jl = lane >> 2;                                              // plane row within a piece
  const int sch = ((lane & 3) ^ ((-(jl >> 2)) & 3)) * 8;                 // source chunk (elements)
  const int arow_l = 64 * wave + jl;                                     // + 16 p
  const int whalf = wave >> 1;
  const int wrow_l = 128 * whalf + (OUT32 ? 4 * jl : 8 * jl);           // + wfrag(f)
  auto wfrag = [](int f) { return OUT32 ? 64 * (f >> 2) + (f & 3) : f; };
  auto voffA = [&](int bm0) { return ((bm0 + arow_l) * lda + sch) * 2; };
  auto voffW = [&](int bn0) { return ((bn0 + wrow_l) * ldw + sch) * 2; };
  int vA = voffA(m0), vW = voffW(n0), vAn = vA, vWn = vW;
  auto launder = [&]() { asm volatile("" : "+v"(vA), "+v"(vW), "+v"(vAn), "+v"(vWn)); };
  // piece p (0-3 A, 4-7 W) of plane ks of virtual K-tile kv (>= nk: the next tile's K-tile kv - nk), issued
  // p = 0..7 in order: the soffsets run as two chains (A: +16 rows per piece, W: +1 row per piece) so only
  // three row-step scalars stay live (per-piece products were kept as SGPR spills in VGPR lanes and
  // reloaded with v_readlane inside the MFMA stream — k_gemm_w4's round-3 finding)
  const int stA = 16 * lda * 2, stW = ldw * 2, wb = wfrag(4 * (wave & 1)) * ldw * 2;
  int sA = 0, sW = 0;
  auto dma_piece = [&](int kv, int ks, int p) {
    const bool nxt = kv >= nk;
    const int kt = nxt ? kv - nk : kv;
    char* plane = smem + (kv & 1) * WP_BUF + ks * WP_PLANE;
    if (p == 0) { sA = kt * 128 + ks * 64; asm volatile("" : "+s"(sA)); }
    if (p == 4) { sW = kt * 128 + ks * 64 + wb; asm volatile("" : "+s"(sW)); }
    if (p < 4) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(plane + (64 * wave + 16 * p) * 64),
                                               16, nxt ? vAn : vA, sA, 0, 0);
      int st = stA;
      asm volatile("" : "+s"(st));
      sA += st;
    } else {
      const int f = 4 * (wave & 1) + (p - 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsW, (__attribute__((address_space(3))) void*)(plane + PP_HALF + (128 * whalf + 16 * f) * 64), 16,
          nxt ? vWn : vW, sW, 0, 0);
      int st = stW;
      asm volatile("" : "+s"(st));
      sW += st;
    }
  };
  auto dma_cols = [&](int tm0, int tn0, int par) {
    if (C == 0) return;
    const int vec = wave % 3;
    const float* src = EPI == RF_EPI_COS ? e.rw : e.bias;
    int idx = min(tn0 + 4 * lane, e.N - 4);
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 1) src = e.lgamma;
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 2) src = e.lbeta;
    if (EPI == RF_EPI_COS && vec == 1) {
      src = e.ra;
      idx = min(tm0 + 4 * lane, e.M - 4);
    }
    glds16(src + idx, smem + WP_CV + (par * 3 + vec) * 1024);
  };
  // fragment reads: 16 rows (lane & 15) x the 4 chunks (lane >> 4) of a plane's 64-B rows, swizzled
  const int lr = lane & 15;
  const int offr = lr * 64 + (((lane >> 4) ^ ((-(lr >> 2)) & 3)) << 4);
  const int aOff = 128 * wr * 64 + offr, bOff = PP_HALF + 128 * wc * 64 + offr;
  V8 a0[8], b0[8], a1[8], b1[8];
  f32x4 acc[8][8];
  auto readp = [&](int kv, int ks, int idx) {  // fragment idx (0-7 A, 8-15 W) of plane ks of K-tile kv
    const char* plane = smem + (kv & 1) * WP_BUF + ks * WP_PLANE;
    const V8 x = *reinterpret_cast<const V8*>(plane + (idx < 8 ? aOff + idx * 16 * 64 : bOff + (idx - 8) * 16 * 64));
    if (ks == 0) {
      if (idx < 8) a0[idx] = x; else b0[idx - 8] = x;
    } else {
      if (idx < 8) a1[idx] = x; else b1[idx - 8] = x;
    }
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // the counted wait before a barrier: everything but the `younger` newest vector-memory ops of this wave
  auto sync = [&](int younger) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int R1 = 16 + S + C < 63 ? 16 + S + C : 63;  // vmcnt is 6 bits: a larger count waits more, safely
    if (younger == 16) wait_vmcnt<16>();
    else if (younger == 16 + S + C) wait_vmcnt<R1>();
    else wait_vmcnt<0>();
    bar();
  };

  // prologue: both planes of K-tiles 0 and 1, the first tile's column vectors; k-step 0 of K-tile 0
  dma_cols(m0, n0, 0);
#pragma unroll
  for (int kv = 0; kv < 2; ++kv)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int p = 0; p < 8; ++p) dma_piece(kv, ks, p);
  wait_vmcnt<0>();
  bar();
#pragma unroll
  for (int i = 0; i < 16; ++i) readp(0, 0, i);
  int tix = 0;
  int relax = 0;  // vector-memory ops of the previous tile's epilogue (+ column DMA) still counted in vmcnt
  bool first_tile = true;
  for (;;) {
    const bool has_next = v + (int)gridDim.x < tiles;
    if (has_next) {
      tile_origin(v + gridDim.x, nm0, nn0);
    } else {
      nm0 = m0;
      nn0 = n0;
    }
    vAn = voffA(nm0);
    vWn = voffW(nn0);
    // ---- phase A(t): k-step 0 MFMAs of K-tile t; k-step 1 fragments of t; plane 0 of K-tile t + 2 ----
    auto phaseA = [&](int t, auto zero) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        dma_piece(t + 2, 0, p);
        readp(t, 1, p < 4 ? 8 + 2 * p : 2 * (p - 4));  // W fragments first (phase B's MFMA order)
        readp(t, 1, p < 4 ? 8 + 2 * p + 1 : 2 * (p - 4) + 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = mfma16(a0[i], b0[j], decltype(zero)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 DS reads
      }
    };
    // ---- phase B(t): k-step 1 MFMAs of K-tile t; k-step 0 fragments of t + 1; plane 1 of K-tile t + 2 ----
    auto phaseB = [&](int t) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        dma_piece(t + 2, 1, p);
        readp(t + 1, 0, p < 4 ? 8 + 2 * p : 2 * (p - 4));
        readp(t + 1, 0, p < 4 ? 8 + 2 * p + 1 : 2 * (p - 4) + 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    };
    // S(t) before phase A(t): every wave's reads of plane 0 of K-tile t (phase B(t - 1)) done, plane 1 of K-tile
    // t landed; M(t) before phase B(t): the reads of plane 1 of t done, plane 0 of t + 1 landed. The first
    // three barriers of a tile also count the previous tile's epilogue stores and column DMA (relax).
    if (!first_tile) sync(16 + relax);
    launder();
    phaseA(0, std::true_type{});
    sync(16 + relax);
    launder();
    phaseB(0);
    for (int t = 1; t < nk; ++t) {
      sync(t == 1 ? 16 + relax : 16);
      launder();
      phaseA(t, std::false_type{});
      sync(16);
      launder();
      phaseB(t);
    }
    first_tile = false;
    // epilogue straight from the accumulators (k_gemm_w4's): lane (c = l & 15, g = l >> 4) holds rows
    // 4 g + r of each 16-row block i and the columns [8c, 8c+8) (16-bit) / [4c, 4c+4) u [64+4c, ..)
    const bool interior = (m0 + 256 <= e.M) && (n0 + TN <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    const int erow = m0 + wr * 128 + 4 * (el >> 4);
    const int ecol = n0 + wc * 128 + (OUT32 ? 4 : 8) * (el & 15);
    float bv[8], gm[8], bt[8];
    const float* cb = reinterpret_cast<const float*>(smem + WP_CV + (tix & 1) * 3 * 1024);
    {
      const int co = ecol - n0;
      if (OUT32) {
        lds_cols<EPI, 4>(cb, co, bv, gm, bt);
        lds_cols<EPI, 4>(cb, co + 64, bv + 4, gm + 4, bt + 4);
      } else {
        lds_cols<EPI, 8>(cb, co, bv, gm, bt);
      }
    }
    const int em0 = m0;
    const void* tbase = reinterpret_cast<const E*>(e.C) + (int64_t)m0 * e.ldc;
    constexpr bool FSC = !OUT32 && (EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX);
    float csc = 1.f;
    if (FSC) {
      csc = ecol < e.scale_cols ? e.col_scale : 1.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) bv[k] *= csc;
    }
    auto epilogue = [&](auto check) {
      constexpr bool CK = decltype(check)::value;
      constexpr bool ZP = !CK && !OUT32 && EPI == RF_EPI_DGELU;
      if constexpr (ZP) {
        constexpr int ZD = 16;
        const char* zbase = reinterpret_cast<const char*>(e.R) + (int64_t)em0 * e.ldr * (int)sizeof(E);
        auto zload = [&](int k) {
          const int row = erow + (k >> 2) * 16 + (k & 3);
          return *reinterpret_cast<const V8*>(zbase + (uint32_t)(((row - em0) * e.ldr + ecol) * (int)sizeof(E)));
        };
        V8 zv[ZD];
#pragma unroll
        for (int k = 0; k < ZD; ++k) zv[k] = zload(k);
#pragma unroll
        for (int k = 0; k < 32; ++k) {
          const int i = k >> 2, r = k & 3;
          const V8 z = zv[k % ZD];
          if (k + ZD < 32) zv[k % ZD] = zload(k + ZD);
          float vv[8];
#pragma unroll
          for (int f = 0; f < 8; ++f) vv[f] = acc[i][f][r];
          epi_seg<E, EPI, CF32, RF32, 8, CK, true, FSC, true>(e, erow + i * 16 + r, ecol, vv, bv, gm, bt, 0.f, tbase,
                                                              em0, csc, z);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float vv[8];
#pragma unroll
            for (int f = 0; f < 8; ++f) vv[f] = acc[i][f][r];
            const int row = erow + i * 16 + r;
            const float rsc = EPI == RF_EPI_COS ? cb[256 + row - em0] : 0.f;
            if (OUT32) {
              epi_seg<E, EPI, CF32, RF32, 4, CK>(e, row, ecol, vv, bv, gm, bt, rsc);
              epi_seg<E, EPI, CF32, RF32, 4, CK>(e, row, ecol + 64, vv + 4, bv + 4, gm + 4, bt + 4, rsc);
            } else {
              epi_seg<E, EPI, CF32, RF32, 8, CK, !CK, FSC>(e, row, ecol, vv, bv, gm, bt, rsc, tbase, em0, csc);
            }
          }
      }
    };
    if (interior) epilogue(std::false_type{});
    else epilogue(std::true_type{});
    asm volatile("" ::: "memory");
    // the next tile's column vectors into the other parity slot (last read by the previous tile's epilogue,
    // before this tile's first barrier); waited for by the next tile's S(1) barrier at the latest
    if (has_next) dma_cols(nm0, nn0, (tix + 1) & 1);
    ++tix;
    if (!has_next) break;
    v += gridDim.x;
    m0 = nm0;
    n0 = nn0;
    vA = vAn;
    vW = vWn;
    relax = interior ? S + C : 0;
  }
  wait_vmcnt<0>();
}

template <typename E, int EPI, bool CF32>
static void launch_w4p(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                       hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_w4p<E, EPI, CF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)WP_LDS);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 255) / 256;
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_w4p<E, EPI, CF32><<<grid, 256, WP_LDS, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm, nTn);
}

// rf_gemm.hip's entry: the 16-bit-output forms of the encoder GEMMs (EPI_NONE / BIAS / BIAS_GELU); false when
// the combination is not instantiated here (the caller then takes k_gemm_w4)
bool gemm_w4p(bool half, int epi, bool cf32, int M, int N, int K, const void* A, int lda, const void* W, int ldw,
              const EpiArgs& e, hipStream_t s) {
  if (cf32) return false;
#define WP_(EE)                                                                                      \
  switch (epi) {                                                                                     \
    case RF_EPI_NONE: launch_w4p<EE, RF_EPI_NONE, false>(M, N, K, A, lda, W, ldw, e, s); return true; \
    case RF_EPI_BIAS: launch_w4p<EE, RF_EPI_BIAS, false>(M, N, K, A, lda, W, ldw, e, s); return true; \
    case RF_EPI_BIAS_GELU: launch_w4p<EE, RF_EPI_BIAS_GELU, false>(M, N, K, A, lda, W, ldw, e, s); return true; \
    default: return false;                                                                           \
  }
  if (half) {
    WP_(f16)
  } else {
    WP_(bf16)
  }
#undef WP_
}

}  // namespace rf
