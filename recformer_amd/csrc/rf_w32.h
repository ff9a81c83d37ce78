// The four-wave 256x256 persistent main loop on v_mfma_f32_32x32x16 (k_gemm_w32's, rf_gemm.hip),
// shared by the encoder GEMMs and the fused catalog score + rank kernel (rf_retrieval.hip): w32_run
// walks the tiles and the K-loop; a policy object supplies the epilogue and its column vectors.
#pragma once
#include <utility>

#include "rf_common.h"

namespace rf {

constexpr int W32_HALF = 128 * 128;              // bytes per 128-row half of a K-tile operand
constexpr int W32_BUF = 4 * W32_HALF;            // one K-tile: A rows 0-127, 128-255, W rows 0-127, 128-255
constexpr int W32_CV = 2 * W32_BUF;              // column vectors [parity][3][1 KiB]
constexpr int W32_PF = W32_CV + 6 * 1024;        // L2-prefetch landing area, 256 B per wave (never read)
constexpr int W32_SCR = W32_PF + 1024;           // epilogue scratch (policies), up to the 160 KiB of a CU
constexpr int W32_SCR_BYTES = 163840 - W32_SCR;
constexpr int W32_LDS = 163840;

template <int N>
__device__ __forceinline__ void w32_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- 4-wave 256x256 GEMM on v_mfma_f32_32x32x16: one wave per SIMD, 4 x 4 blocks of 32 x 32 -----
// k_gemm_w4's structure (256 x 256 tile, 4 waves x 128 x 128 accumulators = 256 AGPRs, two 64-KiB
// K-tile buffers, one barrier per K-tile, the next tile's first two K-tiles fetched across the tile
// boundary) with the 32x32x16 MFMA instead of 16x16x32: the same 2,048 MFMA cycles and 32
// ds_read_b128 per wave and K-tile, but 64 instead of 128 MFMA issues, each holding the SIMD's
// vector issue for 8 of its 32 cycles instead of 8 of 16 (MI355X_MICROARCH.md cycle table) — 1,536
// instead of 1,024 free issue cycles per K-tile for the LDS reads and the 16 LDS-DMA pieces.
// K-tile = 4 k-steps of 16: phase A runs k-steps 0, 1 (32 MFMAs) while the fragments of k-steps 2, 3
// are read; phase B runs 2, 3 while the next K-tile's 0, 1 are read and the K-tile after it is
// DMA'd into the buffer just released (one MFMA, one DMA piece, one MFMA, one read per group).
// LDS image: 128-B rows, 16-B chunk c of row R at slot c ^ ((R >> 1) & 7) — the 32-row operand
// read (lane l: row l & 31, chunk 2s + (l >> 5)) hits 16 distinct bank quads in each of
// ds_read_b128's four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...).
// Output: lane l holds column l & 31 of each 32 x 32 block and rows 8(r>>2) + 4(l>>5) + (r&3); the
// W rows are permuted so lane c owns output columns 4c .. 4c+3 of the wave's 128 (LDS row
// 32 jb + c holds W row 4c + jb): every store instruction writes two whole 256-B row segments.
template <int N, typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// what a policy's epilogue sees of the tile: origin, the wave's 128 x 128 quadrant (wr: A half,
// wc: W half), lane, the tile's column vectors in LDS (pol.cols' slots) and its LDS scratch
struct W32Tile {
  int m0, n0, wr, wc, lane, wave;
  const float* cb;
  char* scr;
};

// Policy interface:
//   static constexpr int S;                          memory ops a wave issues per epilogue, every tile
//   void cols(char* slot, int wave, int lane, int tm0, int tn0) const;   LDS-DMA of the tile's vectors
//                                                    into slot[0..3 KiB) (one glds16 per wave at most)
//   void epilogue(f32x16 (&acc)[4][4], const W32Tile&) const;
//     acc[i][jb][r]: A row 32i + 8(r>>2) + 4(l>>5) + (r&3) of the wave's half, W row (output column)
//     4(l&31) + jb of the wave's half (the W image is permuted).
template <typename E, typename Pol>
__device__ __forceinline__ void w32_run(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw,
                                        int M, int N, int gn, int pf, int nTm, int nTn, const Pol& pol) {
  typedef typename H16<E>::x8 V8;
  constexpr int S = Pol::S;  // memory operations a wave issues in a tile's epilogue (>= 64 for the relax)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = nTm * nTn;
  int v = blockIdx.x;
  if (v >= tiles) return;
  const int GN = gn > 0 ? min(gn, nTn) : nTn;
  auto tile_origin = [&](int vv, int& om0, int& on0) {
    const int wg = xcd_remap(vv, tiles);
    const int g = wg / (nTm * GN);
    const int gw = min(GN, nTn - g * GN);
    const int rem = wg - g * nTm * GN;
    const int tm = rem / gw;
    om0 = tm * 256;
    on0 = (g * GN + rem - tm * gw) * 256;
  };
  int m0, n0, nm0 = 0, nn0 = 0;
  tile_origin(v, m0, n0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // A half (rows 128 wr..) and W half (columns 128 wc..)
  const int nk = K >> 6;
  // Operand DMA (buffer_load ... lds, rows past M / N read as zeros): wave w stages LDS rows
  // [64(w&1), +64) of A-half w>>1 and W-half w>>1 as 8 pieces pp of 8 rows; lane: LDS row
  // 64(w&1) + 8pp + (l>>3), slot l&7, so it fetches chunk (l&7) ^ ((row>>1)&7) = (l&7) ^ (4(pp&1) + (l>>4)):
  // two per-lane source offsets (even / odd pieces). W: LDS row rho holds W row 4(rho&31) + (rho>>5),
  // i.e. per lane 4(l>>3) + 2(w&1) and per piece 32(pp&3) + (pp>>2) rows.
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)min((int64_t)M * lda * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)min((int64_t)N * ldw * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const int half = wave >> 1;
  const int pchE = ((lane & 7) ^ (lane >> 4)) * 8;
  const int pchO = ((lane & 7) ^ (4 + (lane >> 4))) * 8;
  const int arow_l = half * 128 + (wave & 1) * 64 + (lane >> 3);
  const int wrow_l = half * 128 + 4 * (lane >> 3) + 2 * (wave & 1);
  auto voffA = [&](int bm0, int pch) { return ((bm0 + arow_l) * lda + pch) * 2; };
  auto voffW = [&](int bn0, int pch) { return ((bn0 + wrow_l) * ldw + pch) * 2; };
  int vAE = voffA(m0, pchE), vAO = voffA(m0, pchO), vWE = voffW(n0, pchE), vWO = voffW(n0, pchO);
  int vAEn = vAE, vAOn = vAO, vWEn = vWE, vWOn = vWO;
  auto launder = [&]() {
    asm volatile("" : "+v"(vAE), "+v"(vAO), "+v"(vWE), "+v"(vWO));
    asm volatile("" : "+v"(vAEn), "+v"(vAOn), "+v"(vWEn), "+v"(vWOn));
  };
  // soffset chains: A +8 rows per piece; W pieces pp = 0..7 at rows +0, 32, 64, 96, 1, 33, 65, 97
  const int stA = 8 * lda * 2, stW = 32 * ldw * 2, stWj = -95 * ldw * 2;
  int sA = 0, sW = 0;
  auto dma_piece = [&](int kv, int buf, int p) {
    const bool nxt = kv >= nk;
    const int kt = nxt ? kv - nk : kv;
    const bool isA = p < 8;
    const int pp = p & 7;
    char* dst = smem + buf * W32_BUF + (isA ? half : 2 + half) * W32_HALF + ((wave & 1) * 64 + 8 * pp) * 128;
    if (p == 0) { sA = kt * 128; asm volatile("" : "+s"(sA)); }
    if (p == 8) { sW = kt * 128; asm volatile("" : "+s"(sW)); }
    const int soff = isA ? sA : sW;
    {
      int st = isA ? stA : (pp == 3 ? stWj : stW);
      asm volatile("" : "+s"(st));  // no hoisting of per-piece products out of the K-loop
      if (isA) sA += st; else sW += st;
    }
    const int vo = isA ? ((pp & 1) ? (nxt ? vAOn : vAO) : (nxt ? vAEn : vAE))
                       : ((pp & 1) ? (nxt ? vWOn : vWO) : (nxt ? vWEn : vWE));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsA : rsW, (__attribute__((address_space(3))) void*)dst, 16, vo,
                                             soff, 0, 0);
  };
  auto dma_cols = [&](int tm0, int tn0, int par) { pol.cols(smem + W32_CV + par * 3 * 1024, wave, lane, tm0, tn0); };
  // fragment reads: k-step s of 32-row block f at LDS row 32f + (l&31), chunk 2s + (l>>5)
  int offS[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    offS[s] = (lane & 31) * 128 + (((2 * s + (lane >> 5)) ^ ((lane >> 1) & 7)) << 4);
  }
  const int aOff = wr * W32_HALF, bOff = (2 + wc) * W32_HALF;
  V8 xa[2][4], xb[2][4], ya[2][4], yb[2][4];
  f32x16 acc[4][4];
  // set X = k-steps 0, 1; set Y = k-steps 2, 3; idx 0-3 A blocks, 4-7 W blocks; s = 0, 1 within the set
  auto readX = [&](int buf, int s, int idx) {
    const char* base = smem + buf * W32_BUF + (idx < 4 ? aOff : bOff) + (idx & 3) * 32 * 128 + offS[s];
    if (idx < 4) xa[s][idx] = *reinterpret_cast<const V8*>(base);
    else xb[s][idx - 4] = *reinterpret_cast<const V8*>(base);
  };
  auto readY = [&](int buf, int s, int idx) {
    const char* base = smem + buf * W32_BUF + (idx < 4 ? aOff : bOff) + (idx & 3) * 32 * 128 + offS[2 + s];
    if (idx < 4) ya[s][idx] = *reinterpret_cast<const V8*>(base);
    else yb[s][idx - 4] = *reinterpret_cast<const V8*>(base);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int pfd = pf & 0xff;
  const int npf = pfd ? 1 + ((pf >> 8) & 1) : 0;
  auto prefetch = [&](int kv) {
    const bool nxt = kv >= nk;
    const int kt = min(nxt ? kv - nk : kv, nk - 1);
    const int prow = wave * 64 + lane;
    auto* dst = (__attribute__((address_space(3))) void*)(smem + W32_PF + wave * 256);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 4, ((nxt ? nm0 : m0) + prow) * lda * 2, kt * 128, 0, 0);
    if (npf == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, dst, 4, ((nxt ? nn0 : n0) + prow) * ldw * 2, kt * 128, 0, 0);
  };

  dma_cols(m0, n0, 0);
#pragma unroll
  for (int p = 0; p < 16; ++p) dma_piece(0, 0, p);
#pragma unroll
  for (int p = 0; p < 16; ++p) dma_piece(1, 1, p);
  w32_wait_vmcnt<16>();
  bar();
#pragma unroll
  for (int i = 0; i < 16; ++i) readX(0, i >> 3, i & 7);
  int kb = 0, tix = 0, relax = 0;
  for (;;) {
    const bool has_next = v + (int)gridDim.x < tiles;
    if (has_next) {
      tile_origin(v + gridDim.x, nm0, nn0);
    } else {
      nm0 = m0;
      nn0 = n0;
    }
    vAEn = voffA(nm0, pchE);
    vAOn = voffA(nm0, pchO);
    vWEn = voffW(nn0, pchE);
    vWOn = voffW(nn0, pchO);
    // ---- phase A: k-steps 0, 1 of K-tile t on MFMA; k-steps 2, 3 of K-tile t from LDS ----
    auto phaseA = [&](auto zero) {
#pragma unroll
      for (int i = 0; i < 16; ++i) readY(kb, i >> 3, ((i & 7) + 4) & 7);  // W blocks first
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma32(xa[s][i], xb[s][j], (decltype(zero)::value && s == 0) ? f32x16{} : acc[i][j]);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      }
    };
    auto midsync = [&](int t) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t == 0 && relax) w32_wait_vmcnt<(S < 63 ? S : 63)>();
      else if (t > 0 && npf == 1) w32_wait_vmcnt<1>();
      else if (t > 0 && npf == 2) w32_wait_vmcnt<2>();
      else w32_wait_vmcnt<0>();
      bar();
    };
    // ---- phase B: k-steps 2, 3 on MFMA; K-tile t+1's k-steps 0, 1 from LDS; DMA of K-tile t+2 ----
    auto phaseB = [&](int t) {
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        dma_piece(t + 2, kb, p);
        readX(kb ^ 1, p >> 3, ((p & 7) + 4) & 7);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(ya[s][i], yb[s][j], acc[i][j]);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      }
      if (npf && t + 1 < nk && t + 2 + pfd < 2 * nk) prefetch(t + 2 + pfd);
      kb ^= 1;
    };
    launder();
    phaseA(std::true_type{});
    for (int t = 0; t + 1 < nk; ++t) {
      midsync(t);
      phaseB(t);
      launder();
      phaseA(std::false_type{});
    }
    midsync(nk - 1);
    phaseB(nk - 1);
    // no accumulator copy-out may move into the MFMA stream (it would hold 256 VGPRs next to the next
    // tile's fragments); the epilogue streams 8 accumulators per row pair (sched_barrier per pair)
    __builtin_amdgcn_sched_barrier(0);
    // the accumulators are read below by inline asm, which the hazard recognizer does not see: 24 wait
    // states cover the 32x32x16 MFMA's write -> VALU read distance (18) for the last MFMAs' blocks
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    pol.epilogue(acc, W32Tile{m0, n0, wr, wc, lane, wave,
                              reinterpret_cast<const float*>(smem + W32_CV + (tix & 1) * 3 * 1024), smem + W32_SCR});
    asm volatile("" ::: "memory");
    if (has_next) dma_cols(nm0, nn0, (tix + 1) & 1);
    ++tix;
    if (!has_next) break;
    v += gridDim.x;
    m0 = nm0;
    n0 = nn0;
    vAE = vAEn;
    vAO = vAOn;
    vWE = vWEn;
    vWO = vWOn;
    relax = S;  // every tile issues its S stores (out-of-range ones are dropped, not skipped)
  }
  w32_wait_vmcnt<0>();
}


}  // namespace rf
