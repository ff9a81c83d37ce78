// MFMA GEMMs with fused epilogues: C[M,N] = epi(A[M,K] . W[N,K]^T).
//
// Replaces the nn.Linear addmm's of the Longformer layer (TF:504-506, 982-984,
// 1064-1071, 1107, 1123) and the scoring product of Similarity (models.py:358-369).
//
// bf16 path (k_gemm_bf16<BM,BN,WM,WN,...>): v_mfma_f32_16x16x32_bf16, BK = 64. Operands are
// DMA'd HBM->LDS by 16-B global_load_lds into a lane-linear image; the XOR swizzle that
// makes the ds_read_b128 operand reads conflict-free is applied to the per-lane SOURCE
// address and to the read (guide §5.4 rule 21, §5.5 T2). Two LDS stages: tile k+1's DMA
// is in flight while tile k's MFMAs run. Blocks are remapped bijectively so consecutive
// tiles (sharing an A panel) land on one XCD's L2 (guide §5 T1).
//   * 256x256 tile, 8 waves of 128x64 — the production shape: 128 flop per staged byte,
//     so the L2->LDS stream needs ~20 TB/s at MFMA peak (a 128^2 tile would need ~39 TB/s,
//     above what the XCD L2s deliver);
//   * 128x128 tile, 4 waves of 64x64 — for small M or N (global rows, scoring).
// Epilogue: whole rows of 16 columns per lane with 16-B vector stores (bias / q-scale /
// GELU / residual / LayerNorm-recompute / cosine scale applied in fp32 on the way) — straight
// from the accumulators in the ping-pong kernel, through LDS slabs in k_gemm_bf16.
// fp32 path: exact-f32 v_mfma_f32_16x16x4_f32, 64x64x16 tiles, register staging.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "rf_common.h"
#include "rf_gemm_epi.h"
#include "rf_w32.h"

namespace rf {




// ------------------------------------------------------------------------------------
// bf16
constexpr int EPI_LD = 68;  // fp32 staging row stride (floats): conflict-free write + b128 read

// bias[c0, c0+16) as 4 float4 loads (zeros for EPI_NONE / EPI_COS or a ragged right edge)
template <int EPI>
__device__ __forceinline__ void load_bias16(const EpiArgs& e, int c0, float* b) {
  if (EPI == RF_EPI_NONE || EPI == RF_EPI_COS || EPI == RF_EPI_DGELU || c0 + 16 > e.N) {
#pragma unroll
    for (int k = 0; k < 16; ++k) b[k] = 0.f;
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 x = *reinterpret_cast<const float4*>(e.bias + c0 + 4 * q);
    b[4 * q] = x.x; b[4 * q + 1] = x.y; b[4 * q + 2] = x.z; b[4 * q + 3] = x.w;
  }
}

// 16 consecutive columns [c0, c0+16) of one output row: vector epilogue. `bv` is the bias
// slice from load_bias16 (hoisted by the caller).
template <typename E, int EPI, bool CF32, bool RF32>
__device__ __forceinline__ void epi_row16(const EpiArgs& e, int row, int c0, float* v, const float* bv) {
  if (row >= e.M) return;
  if (c0 + 16 > e.N) {  // ragged right edge: scalar path
#pragma unroll
    for (int k = 0; k < 16; ++k) epi_store<E, EPI, CF32, RF32>(e, row, c0 + k, v[k]);
    return;
  }
  if (EPI == RF_EPI_COS) {
    const float s = e.ra[row] * e.col_scale;
    float* out = reinterpret_cast<float*>(e.C) + (int64_t)row * e.ldc + c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 w = *reinterpret_cast<const float4*>(e.rw + c0 + 4 * q);
      *reinterpret_cast<float4*>(out + 4 * q) =
          make_float4(v[4 * q] * s * w.x, v[4 * q + 1] * s * w.y, v[4 * q + 2] * s * w.z, v[4 * q + 3] * s * w.w);
    }
    return;
  }
  if (EPI == RF_EPI_DGELU) {
    const E* z = reinterpret_cast<const E*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] *= dgelu_erf(to_f32(z[k]));
  } else if (EPI != RF_EPI_NONE) {
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] += bv[k];
  }
  if (c0 < e.scale_cols) {
    // scale_cols is a multiple of 16 on every call site (head-aligned q columns)
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] *= e.col_scale;
  }
  if (EPI == RF_EPI_BIAS_GELU_AUX) {
    E* z = reinterpret_cast<E*>(const_cast<void*>(e.R)) + (int64_t)row * e.ldr + c0;
#pragma unroll
    for (int h8 = 0; h8 < 2; ++h8) {
      typename H16<E>::x8 x;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (E)v[8 * h8 + k];
      *reinterpret_cast<typename H16<E>::x8*>(z + 8 * h8) = x;
    }
  }
  if (EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX) {
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = CF32 ? gelu_erf(v[k]) : gelu_bf16out(v[k]);
  }
  if (EPI == RF_EPI_BIAS_RESID) {
    if (RF32) {
      const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(r + 4 * q);
        v[4 * q] += x.x; v[4 * q + 1] += x.y; v[4 * q + 2] += x.z; v[4 * q + 3] += x.w;
      }
    } else {
      const E* r = reinterpret_cast<const E*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const typename H16<E>::x8 x = *reinterpret_cast<const typename H16<E>::x8*>(r + 8 * q);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[8 * q + k] += (float)x[k];
      }
    }
  }
  if (EPI == RF_EPI_BIAS_RESID_LN) {
    // same expression as the LayerNorm kernel's output: (x - mean) * rstd * gamma + beta
    const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)row * e.ldr + c0;
    const float mu = e.lmean[row], rs = e.lrstd[row];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(r + 4 * q);
      const float4 gm = *reinterpret_cast<const float4*>(e.lgamma + c0 + 4 * q);
      const float4 bt = *reinterpret_cast<const float4*>(e.lbeta + c0 + 4 * q);
      v[4 * q] += (x.x - mu) * rs * gm.x + bt.x;
      v[4 * q + 1] += (x.y - mu) * rs * gm.y + bt.y;
      v[4 * q + 2] += (x.z - mu) * rs * gm.z + bt.z;
      v[4 * q + 3] += (x.w - mu) * rs * gm.w + bt.w;
    }
  }
  if (CF32) {
    float* out = reinterpret_cast<float*>(e.C) + (int64_t)row * e.ldc + c0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<f32x4*>(out + 4 * q) = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  } else {
    E* out = reinterpret_cast<E*>(e.C) + (int64_t)row * e.ldc + c0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      typename H16<E>::x8 x;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (E)v[8 * q + k];
      *reinterpret_cast<typename H16<E>::x8*>(out + 8 * q) = x;
    }
  }
}

// Operand tile geometry for a BK-deep stage: rows of BK bf16 (BK*2 bytes), 16-B chunks.
//  BK = 64: 128-B rows, chunk slot = c ^ (r & 7)            (guide §5.5 T2)
//  BK = 32:  64-B rows, chunk slot = c ^ f(r), f = (-(r>>2)) & 3: makes every 16-lane group
//            of the ds_read_b128 operand read (rows l&15, chunk l>>4) hit 16 distinct slots.
template <int BK> struct TileGeo;
template <> struct TileGeo<64> {
  static constexpr int ROWB = 128, PIECE_ROWS = 8;
  static __device__ __forceinline__ int slot(int r, int c) { return c ^ (r & 7); }
};
template <> struct TileGeo<32> {
  static constexpr int ROWB = 64, PIECE_ROWS = 16;
  static __device__ __forceinline__ int slot(int r, int c) { return c ^ ((-(r >> 2)) & 3); }
};


// NSTAGE-deep LDS ring, prefetch distance NSTAGE-1. Each wave waits only for ITS pieces of
// the tile it is about to read (counted vmcnt, the younger tiles stay in flight across the
// raw s_barrier — guide §5 'Pipelining across barriers'), then the barrier publishes every
// wave's pieces. The slot refilled in iteration kt was last read in kt-1, which every wave
// has finished before passing this iteration's barrier.
constexpr int gemm_min_waves(int bm, int bn, int wm, int wn, int bk, int nstage) {
  // waves per SIMD the LDS budget admits (1..8): lets the register allocator size for it
  return (163840 / (nstage * (bm + bn) * bk * 2)) * ((bm / wm) * (bn / wn)) / 4 < 1
             ? 1
             : ((163840 / (nstage * (bm + bn) * bk * 2)) * ((bm / wm) * (bn / wn)) / 4 > 8
                    ? 8
                    : (163840 / (nstage * (bm + bn) * bk * 2)) * ((bm / wm) * (bn / wn)) / 4);
}

template <typename E, int BM, int BN, int WM, int WN, int BK, int NSTAGE, int EPI, bool CF32, bool RF32>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, gemm_min_waves(BM, BN, WM, WN, BK, NSTAGE))
    k_gemm_bf16(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw,
                EpiArgs e, int nTn) {
  using G = TileGeo<BK>;
  constexpr int NWN = BN / WN;
  constexpr int NWAVES = (BM / WM) * NWN;
  constexpr int FM = WM / 16, FN = WN / 16;          // 16x16 fragments per wave
  constexpr int A_BYTES = BM * G::ROWB, B_BYTES = BN * G::ROWB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CHUNKS = (BM + BN) / G::PIECE_ROWS;  // 1-KiB DMA pieces per stage
  constexpr int CPW = CHUNKS / NWAVES;               // per wave
  constexpr int ACH = BM / G::PIECE_ROWS;            // A pieces come first
  constexpr int LPR = G::ROWB / 16;                  // lanes per row in a piece
  static_assert(CHUNKS % NWAVES == 0, "staging split");
  static_assert(NWAVES * 16 * EPI_LD * 4 <= NSTAGE * STAGE, "epilogue scratch");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wg / nTn, tn = wg - tm * nTn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / NWN, wn = wave % NWN;

  typedef typename H16<E>::x8 V8;
  const E* src[CPW];
  int dst[CPW];
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int c = wave * CPW + i;
    const bool isA = c < ACH;
    const int row = (isA ? c : c - ACH) * G::PIECE_ROWS + lane / LPR;
    const int ch = G::slot(row, lane % LPR);  // slot is an involution on the chunk index
    if (isA)
      src[i] = A + (int64_t)min(m0 + row, e.M - 1) * lda + ch * 8;
    else
      src[i] = W + (int64_t)min(n0 + row, e.N - 1) * ldw + ch * 8;
    dst[i] = isA ? c * 1024 : A_BYTES + (c - ACH) * 1024;
  }
  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * STAGE;
    const int koff = kt * BK;
#pragma unroll
    for (int i = 0; i < CPW; ++i) glds16(src[i] + koff, base + dst[i]);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  if constexpr (BK == 32 && NSTAGE == 4) {
    // Register-pipelined ring: iteration kt computes tile kt from fragment set X while the
    // ds_reads of tile kt+1 fill set Y and the DMA of tile kt+3 is in flight, so neither the
    // LDS latency nor the HBM/L2 latency sits on the MFMA stream (guide T14 idea applied to
    // the LDS->register stage). Slot (kt+3)%4 = (kt-1)%4 was last read (frag prefetch of tile
    // kt-1) in iteration kt-2 and drained by that wave's lgkmcnt(0) before iteration kt-1's
    // barrier.
    auto read_frags = [&](int kt, V8 (&a)[FM], V8 (&b)[FN]) {
      const char* as = smem + (kt & 3) * STAGE;
      const char* ws = as + A_BYTES;
      const int ch = lane >> 4;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WM + i * 16 + (lane & 15);
        a[i] = *reinterpret_cast<const V8*>(as + r * G::ROWB + (G::slot(r, ch) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WN + j * 16 + (lane & 15);
        b[j] = *reinterpret_cast<const V8*>(ws + r * G::ROWB + (G::slot(r, ch) << 4));
      }
    };
    auto mma = [&](const V8 (&a)[FM], const V8 (&b)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    };
    auto sync_tile = [&](int kt) {  // tile kt landed in every wave's pieces
      const int ahead = nk - 1 - kt;  // tiles kt+1.. that may still be in flight (at most 1)
      if (ahead >= 1) wait_vmcnt<CPW>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    V8 a0[FM], b0[FN], a1[FM], b1[FN];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < nk) stage(i, i);
    // tile 0 landed (tiles 1, 2 may be in flight)
    if (nk >= 3) wait_vmcnt<2 * CPW>();
    else if (nk == 2) wait_vmcnt<CPW>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_frags(0, a0, b0);
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      sync_tile(kt + 1);
      if (kt + 3 < nk) stage(kt + 3, (kt + 3) & 3);
      read_frags(kt + 1, a1, b1);
      mma(a0, b0);
      if (kt + 2 < nk) {
        sync_tile(kt + 2);
        if (kt + 4 < nk) stage(kt + 4, (kt + 4) & 3);
        read_frags(kt + 2, a0, b0);
      }
      mma(a1, b1);
    }
    if (kt < nk) mma(a0, b0);
  } else {
#pragma unroll
  for (int i = 0; i < NSTAGE - 1; ++i)
    if (i < nk) stage(i, i);
  for (int kt = 0; kt < nk; ++kt) {
    // tiles kt+1 .. min(kt+NSTAGE-2, nk-1) may stay in flight
    const int ahead = min(NSTAGE - 2, nk - 1 - kt);
    if (NSTAGE >= 4 && ahead >= 2) wait_vmcnt<2 * CPW>();
    else if (NSTAGE >= 3 && ahead >= 1) wait_vmcnt<CPW>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) stage(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    const char* as = smem + (kt % NSTAGE) * STAGE;
    const char* ws = as + A_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int ch = 4 * s + (lane >> 4);
      V8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WM + i * 16 + (lane & 15);
        a[i] = *reinterpret_cast<const V8*>(as + r * G::ROWB + (G::slot(r, ch) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WN + j * 16 + (lane & 15);
        b[j] = *reinterpret_cast<const V8*>(ws + r * G::ROWB + (G::slot(r, ch) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    }
  }
  }
  __syncthreads();  // every wave is done with the ring before it becomes epilogue scratch

  // ---- epilogue: per wave, 16-row slabs through LDS, then row-major vector stores ----
  float* scr = reinterpret_cast<float*>(smem) + wave * 16 * EPI_LD;
  const int rr = lane >> 2, cc = (lane & 3) * 16;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j0 = 0; j0 < FN; j0 += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          scr[((lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[i][j0 + j][r];
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(scr + rr * EPI_LD + cc + 4 * q);
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
      float bv[16];
      load_bias16<EPI>(e, n0 + wn * WN + j0 * 16 + cc, bv);
      epi_row16<E, EPI, CF32, RF32>(e, m0 + wm * WM + i * 16 + rr, n0 + wn * WN + j0 * 16 + cc, v, bv);
    }
  }
}

// ------------------------------------------------------------------------------------
// fp32 (exact f32 MFMA). 64x64x16 tile, 4 waves (2x2) of 32x32.
constexpr int GF_M = 64, GF_N = 64, GF_K = 16, GF_LD = 20;  // padded LDS row (floats)

template <int EPI>
__global__ void __launch_bounds__(256) k_gemm_f32(int K, const float* __restrict__ A, int lda,
                                                   const float* __restrict__ W, int ldw, EpiArgs e,
                                                   int nTn) {
  __shared__ __attribute__((aligned(16))) float As[GF_M * GF_LD];
  __shared__ __attribute__((aligned(16))) float Ws[GF_N * GF_LD];
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / nTn, tn = wg - tm * nTn;
  const int m0 = tm * GF_M, n0 = tn * GF_N;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = t >> 2, lc = (t & 3) * 4;
  const float* ap = A + (int64_t)min(m0 + lr, e.M - 1) * lda + lc;
  const float* wp = W + (int64_t)min(n0 + lr, e.N - 1) * ldw + lc;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 ra = *reinterpret_cast<const float4*>(ap);
  float4 rw = *reinterpret_cast<const float4*>(wp);
  const int nk = K / GF_K;
  for (int kt = 0; kt < nk; ++kt) {
    *reinterpret_cast<float4*>(&As[lr * GF_LD + lc]) = ra;
    *reinterpret_cast<float4*>(&Ws[lr * GF_LD + lc]) = rw;
    __syncthreads();
    if (kt + 1 < nk) {
      ra = *reinterpret_cast<const float4*>(ap + (kt + 1) * GF_K);
      rw = *reinterpret_cast<const float4*>(wp + (kt + 1) * GF_K);
    }
    float4 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = *reinterpret_cast<const float4*>(&As[(wm * 32 + i * 16 + (lane & 15)) * GF_LD + 4 * (lane >> 4)]);
      b[i] = *reinterpret_cast<const float4*>(&Ws[(wn * 32 + i * 16 + (lane & 15)) * GF_LD + 4 * (lane >> 4)]);
    }
    // lane group g supplies k = 4g + kk at step kk — the same permutation for A and B,
    // so every k of the 16-deep tile is summed exactly once.
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
      }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi_store<float, EPI, false, false>(e, m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r,
                                            n0 + wn * 32 + j * 16 + (lane & 15), acc[i][j][r]);
}

// ------------------------------------------------------------------------------------
// bf16 256x256 ping-pong kernel (guide §5 "256² 8-phase template", rebuilt here).
//
// 8 waves = two groups of four (wr = wave>>2 owns output rows wr*128.., wc = wave&3 owns
// columns wc*64..), one wave of each group per SIMD. Group 1 runs one barrier behind group 0,
// so on every SIMD one wave issues its LDS reads and DMA while the other runs its MFMAs.
// Each K-tile (BK = 64) is 4 phases; a phase = [ds_read the register sub-tile it needs,
// DMA one 16-KiB half-tile, (counted vmcnt)] barrier [16 MFMAs on one 64x32 C-quadrant]
// barrier. LDS: 2 buffers (even / odd K-tile) x 4 halves {A rows 0-127, A rows 128-255,
// W rows 0-127, W rows 128-255} x 16 KiB = 128 KiB; each half is 128 rows x 128 B with the
// chunk swizzle c ^ (r & 7) applied on the DMA source address.
// Reads per K-tile:  P1 a0 + a1 (16) + b0 (4) -> (a0,b0);  P2 b1 (4) -> (a0,b1);
//                    P3 -> (a1,b1);  P4 -> (a1,b0)   (every read of a buffer happens in P1-P2).
// DMA per iteration (K-tiles t = 2i in buffer 0, t+1 in buffer 1):  P1 W1-half of t+1;
// P2..P5 A0, A1, W0, W1 of t+2;  P6..P8 A0, A1, W0 of t+3. Restaging a half waits >= 1 phase
// after its last read when only the leading group reads it (A0), >= 2 phases otherwise (the
// lgkmcnt(0) before each MFMA block retires a wave's reads; the stagger adds one phase).
// vmcnt(6) in P4 and P8 (3 half-tiles = 6 DMAs stay in flight) retires the buffer that is
// read from the next phase on.

// W-row order in LDS (per 128-row half): LDS row 16f + j (N-fragment f = 0..7, MFMA column j)
// holds the W row that makes lane group c = l&15 own whole vectors of output columns:
//   bf16 output: column 8j + f          -> lane c holds columns 8c..8c+7 (one 16-B store)
//   fp32 output: column 64(f>>2) + 4j + (f&3) -> columns 4c..4c+3 and 64+4c..: two 16-B
//                stores, each instruction writing 4 full 256-B row segments.
// Each store instruction then writes whole 128-B lines (4 rows x 16 lanes): measured 2.3-3.6x
// the per-CU store rate of the 16-row x 4-lane pattern (tools/micro/store_pattern.hip).
template <bool OUT32>
__device__ __forceinline__ int wperm(int rho) {
  const int f = (rho >> 4) & 7, j = rho & 15;
  return OUT32 ? 64 * (f >> 2) + 4 * j + (f & 3) : 8 * j + f;
}

#if defined(RF_GEMM_EXPERIMENTS)  // retired main loop (tools/build_variant.sh builds only)
constexpr int CV_OFF = 8 * PP_HALF + 1024;  // LDS: ring, stamp area, then 2 x 3 column vectors

// s_waitcnt vmcnt(n) for a wave-uniform n from the small set the ping-pong kernel uses
template <int S>
__device__ __forceinline__ void wait_vm_rt(int n) {
  if (n == 0) wait_vmcnt<0>();
  else if (n == 6) wait_vmcnt<6>();
  else if (n == 8) wait_vmcnt<8>();
  else if (n == S) wait_vmcnt<S>();
  else if (n == 6 + S) wait_vmcnt<6 + S>();
  else if (n == 8 + S) wait_vmcnt<8 + S>();
  else wait_vmcnt<0>();
}

// Persistent: one workgroup per CU walks tiles v = blockIdx.x, +gridDim.x, ... The next tile's
// prologue DMAs are issued BEFORE the current tile's epilogue (most of them during its last
// K-iteration), so (vmcnt retiring in issue order) the next tile can start while the
// epilogue's S stores are still draining: the prologue wait and the first P4 wait count them
// as allowed-outstanding (interior tiles only, where S is exact).
template <typename E, int EPI, bool CF32, bool RF32>
__global__ void __launch_bounds__(512, 1)
    k_gemm_pp(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e,
              int nTm, int nTn) {
  typedef typename H16<E>::x8 V8;
  constexpr bool OUT32 = CF32 || EPI == RF_EPI_COS;  // fp32 output layout
  constexpr int S = OUT32 ? 32 : 16;                  // epilogue stores per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = nTm * nTn;
  int v = blockIdx.x;
  if (v >= tiles) return;
  int m0 = 0, n0 = 0;
  // Tile order: XCD-contiguous ranges (xcd_remap) of a column-grouped raster: GN columns of
  // tiles at a time, all row panels down, so the tiles one XCD runs concurrently share a W
  // slice of GN x 256 rows that stays resident in its L2 across rounds.
  const int GN = e.gn > 0 ? min(e.gn, nTn) : nTn;
  auto tile_origin = [&](int vv, int& om0, int& on0) {
    const int wg = xcd_remap(vv, tiles);
    const int g = wg / (nTm * GN);
    const int gw = min(GN, nTn - g * GN);  // width of this (possibly last, narrower) group
    const int rem = wg - g * nTm * GN;
    const int tm = rem / gw;
    om0 = tm * 256;
    on0 = (g * GN + rem - tm * gw) * 256;
  };
  auto set_tile = [&](int vv) { tile_origin(vv, m0, n0); };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave (wr, wc) owns output rows 64wr.. and columns 128wc..; group = wr >> 1 (waves 0-3 / 4-7)
  const int grp = wave >> 2, wr = wave >> 1, wc = wave & 1;

  // DMA sources: this thread's two 8-row pieces of each half (rows 16*wave + 8p + lane/8),
  // chunk (lane&7) ^ (row&7) = (lane&7) ^ (lane>>3); rows clamped into the matrix. Offsets
  // are recomputed per DMA (a few VALU ops in the load phase) to keep VGPRs for the MMA.
  // The per-lane row terms are laundered through an empty asm at every K-step so the compiler
  // recomputes the few address ops per DMA instead of hoisting 8+ live offsets out of the
  // tile loop (VGPRs belong to the MMA operands and accumulators).
  int xa = 16 * wave + (lane >> 3);               // A piece row (p = 0; p = 1 is +8)
  int xw0 = wperm<OUT32>(xa), xw1 = wperm<OUT32>(xa + 8);  // permuted W piece rows
  int pch = ((lane & 7) ^ (lane >> 3)) * 8;
  const int nk = K >> 6;
  auto launder = [&]() { asm volatile("" : "+v"(xa), "+v"(xw0), "+v"(xw1), "+v"(pch)); };
  // half index: 0 = A rows 0-127, 1 = A rows 128-255, 2 = W rows 0-127, 3 = W rows 128-255
  // K-tiles nk, nk+1 of the current tile are K-tiles 0, 1 of the NEXT tile when `pf` is set
  // (nk even, so the buffer parity carries over): the last iteration's idle DMA slots prefetch
  // the next tile's prologue behind this tile's MFMAs.
  int nm0 = 0, nn0 = 0;
  bool pf = false;
  auto dma = [&](int t, int half) {
    int kt = t, bm0 = m0, bn0 = n0;
    if (t >= nk) {  // wave-uniform
      if (!pf || t >= nk + 2) return;
      kt = t - nk;
      bm0 = nm0;
      bn0 = nn0;
    }
    char* dst = smem + ((t & 1) * 4 + half) * PP_HALF + wave * 2048;
    const bool isA = half < 2;
    const E* base = isA ? A : W;
    const int ld = isA ? lda : ldw;
    const int lim = (isA ? e.M : e.N) - 1;
    const int r0 = (isA ? bm0 : bn0) + (half & 1) * 128;
    const int ra = r0 + (isA ? xa : xw0), rb = r0 + (isA ? xa + 8 : xw1);
#if !(defined(RF_GEMM_DIAG) && (RF_GEMM_DIAG & 2))  // diagnostic: no operand DMA
    glds16(base + (min(ra, lim) * ld + kt * 64 + pch), dst);
    glds16(base + (min(rb, lim) * ld + kt * 64 + pch), dst + 1024);
#endif
  };
  // Epilogue column vectors of a tile (bias or EPI_COS item norms; LN gamma, beta) as one
  // 1-KiB DMA per wave into LDS slot [parity][vector]: wave w loads vector w % 3 (vectors an
  // epilogue does not have repeat the bias), so every wave issues exactly one DMA and the
  // counted waits stay uniform. Source columns are clamped into [0, N): the ragged last
  // column tile's out-of-range segments take the scalar epi_store path, never these values.
  auto dma_cols = [&](int tm0, int tn0, int par) {
    if (EPI == RF_EPI_NONE || EPI == RF_EPI_DGELU) return;
    const int vec = wave % 3;
    const float* src = EPI == RF_EPI_COS ? e.rw : e.bias;
    int idx = min(tn0 + 4 * lane, e.N - 4);
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 1) src = e.lgamma;
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 2) src = e.lbeta;
    if (EPI == RF_EPI_COS && vec == 1) {  // EPI_COS: the tile's 256 row norms
      src = e.ra;
      idx = min(tm0 + 4 * lane, e.M - 4);
    }
    glds16(src + idx, smem + CV_OFF + (par * 3 + vec) * 1024);
  };
  auto prologue_dma = [&]() {  // K-tiles 0 and 1 complete
    dma(0, 0); dma(0, 1); dma(0, 2); dma(0, 3);
    dma(1, 0); dma(1, 1); dma(1, 2); dma(1, 3);
  };

  // fragment read offsets: row l&15 of a 16-row block, chunk ks*4 + (l>>4), swizzled
  const int lr = lane & 15;
  const int off0 = lr * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
  const int off1 = lr * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  const int aBase = grp * PP_HALF + (wr & 1) * 64 * 128;  // A-half of the group, 64-row band
  const int bBase = (2 + wc) * PP_HALF;                    // the whole W-half

  // quadrant (qm, qn) = 32 rows x 64 columns of the wave's 64 x 128 tile
  V8 a[2][2][2], b[2][4][2];
  f32x4 acc[4][8];

  auto read_a = [&](int buf, int qm) {
#if defined(RF_GEMM_DIAG) && (RF_GEMM_DIAG & 1)  // timing diagnostic: no LDS operand reads
    for (int i = 0; i < 2; ++i) asm volatile("" : "=v"(a[qm][i][0]), "=v"(a[qm][i][1]));
    return;
#endif
    const char* base = smem + buf * 4 * PP_HALF + aBase + qm * 32 * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[qm][i][0] = *reinterpret_cast<const V8*>(base + i * 16 * 128 + off0);
      a[qm][i][1] = *reinterpret_cast<const V8*>(base + i * 16 * 128 + off1);
    }
  };
  auto read_b = [&](int buf, int qn) {
#if defined(RF_GEMM_DIAG) && (RF_GEMM_DIAG & 1)
    for (int j = 0; j < 4; ++j) asm volatile("" : "=v"(b[qn][j][0]), "=v"(b[qn][j][1]));
    return;
#endif
    const char* base = smem + buf * 4 * PP_HALF + bBase + qn * 64 * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b[qn][j][0] = *reinterpret_cast<const V8*>(base + j * 16 * 128 + off0);
      b[qn][j][1] = *reinterpret_cast<const V8*>(base + j * 16 * 128 + off1);
    }
  };
  auto mma = [&](int qm, int qn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[qm * 2 + i][qn * 4 + j] =
              mfma16(a[qm][i][ks], b[qn][j][ks], acc[qm * 2 + i][qn * 4 + j]);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // the MFMA half of a phase: barrier, retire this phase's LDS reads, MFMAs at raised priority
  auto compute = [&](int qm, int qn, bool live) {
#ifndef RF_GEMM_PRIO
#define RF_GEMM_PRIO 1
#endif
#if defined(RF_GEMM_DIAG) && (RF_GEMM_DIAG & 4)  // diagnostic: no barriers around the MFMAs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (live) {
      __builtin_amdgcn_s_setprio(RF_GEMM_PRIO);
      mma(qm, qn);
      __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    return;
#endif
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (live) {
      __builtin_amdgcn_s_setprio(RF_GEMM_PRIO);
      mma(qm, qn);
      __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    bar();
  };

  // diagnostic timeline (tools/gemm_stamps.py): wave 0 records s_memtime at 6 points of each
  // tile into LDS past the ring (no vmcnt traffic), copied out at the end
  unsigned long long* stl = reinterpret_cast<unsigned long long*>(smem + 8 * PP_HALF);
  int tix = 0;
  auto stamp = [&](int k) {
    if (e.stamps != nullptr && wave == 0) {
      const unsigned long long tt = __builtin_amdgcn_s_memtime();
      if (lane == 0 && tix < 16) stl[tix * 8 + k] = tt;
    }
  };
  set_tile(v);
  dma_cols(m0, n0, 0);
  prologue_dma();
  int relax = 0;  // S stores of the previous (interior) tile may still be outstanding
  for (;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    wait_vm_rt<S>((nk > 1 ? 8 : 0) + relax);  // K-tile 0 landed
    bar();
    stamp(0);
    if (grp == 1) bar();  // group 1 runs one barrier behind
    const bool has_next = v + (int)gridDim.x < tiles;
    pf = has_next && !(nk & 1);
    if (has_next) tile_origin(v + gridDim.x, nm0, nn0);
    const int lim = nk + (pf ? 2 : 0);  // DMA-able virtual K-tiles

    for (int t = 0; t < nk; t += 2) {
      const bool odd_live = t + 1 < nk;
      launder();
      // ---- even K-tile t (buffer 0) ----
      read_a(0, 0); read_b(0, 0); read_a(0, 1);
      if (t > 0) dma(t + 1, 3);
      compute(0, 0, true);
      read_b(0, 1); dma(t + 2, 0);
      compute(0, 1, true);
      dma(t + 2, 1);
      compute(1, 1, true);
      dma(t + 2, 2);
      wait_vm_rt<S>((t + 2 < lim ? 6 : 0) + (t == 0 ? relax : 0));  // retires tile t+1 (buffer 1)
      if (t == 0) stamp(1);
      compute(1, 0, true);
      // ---- odd K-tile t+1 (buffer 1) ----
      read_a(1, 0); read_b(1, 0); read_a(1, 1); dma(t + 2, 3);
      compute(0, 0, odd_live);
      read_b(1, 1); dma(t + 3, 0);
      compute(0, 1, odd_live);
      dma(t + 3, 1);
      compute(1, 1, odd_live);
      dma(t + 3, 2);
      if (t + 2 < nk) wait_vm_rt<S>(t + 3 < lim ? 6 : 0);  // retires tile t+2 (buffer 0)
      if (t == 0) stamp(2);
      compute(1, 0, odd_live);
    }
    if (grp == 0) bar();  // equalise the barrier count of the two groups: every LDS read is done
    stamp(3);

    const int em0 = m0, en0 = n0;
    const bool interior = (em0 + 256 <= e.M) && (en0 + 256 <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    // lane (c = l&15, g = l>>4) holds rows 4g + r of each 16-row block mf and the columns
    // [8c, 8c+8) (bf16) or [4c, 4c+4) u [64+4c, 64+4c+4) (fp32) of the wave's 128 (wperm)
    const int erow = em0 + wr * 64 + 4 * (el >> 4);
    const int ecol = en0 + wc * 128 + (OUT32 ? 4 : 8) * (el & 15);
    // column vectors of this tile: DMA'd into LDS with its prologue (retired by the K-loop's
    // counted waits, published by its barriers), so the epilogue issues no global load
    float bv[8], gm[8], bt[8];
    const float* cb = reinterpret_cast<const float*>(smem + CV_OFF + (tix & 1) * 3 * 1024);
    {
      const int co = ecol - en0;
      if (OUT32) {
        lds_cols<EPI, 4>(cb, co, bv, gm, bt);
        lds_cols<EPI, 4>(cb, co + 64, bv + 4, gm + 4, bt + 4);
      } else {
        lds_cols<EPI, 8>(cb, co, bv, gm, bt);
      }
    }
    v += gridDim.x;
    if (has_next) {
      set_tile(v);
      launder();
      dma_cols(m0, n0, (tix + 1) & 1);  // before the prologue DMAs: the first counted waits cover it
      if (pf) dma(1, 3);  // the rest of the next tile's K-tiles 0, 1 went out in the last iteration
      else prologue_dma();
    }
    asm volatile("" ::: "memory");
    stamp(4);
    // Epilogue straight from the accumulators: whole-line vector stores
    auto epilogue = [&](auto check) {
      constexpr bool CK = decltype(check)::value;
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float vv[8];
#pragma unroll
          for (int f = 0; f < 8; ++f) vv[f] = acc[mf][f][r];
          const int row = erow + mf * 16 + r;
          const float rsc = EPI == RF_EPI_COS ? cb[256 + row - em0] : 0.f;
          if (OUT32) {
            epi_seg<E, EPI, CF32, RF32, 4, CK>(e, row, ecol, vv, bv, gm, bt, rsc);
            epi_seg<E, EPI, CF32, RF32, 4, CK>(e, row, ecol + 64, vv + 4, bv + 4, gm + 4, bt + 4, rsc);
          } else {
            epi_seg<E, EPI, CF32, RF32, 8, CK>(e, row, ecol, vv, bv, gm, bt, rsc);
          }
        }
    };
    if (interior) epilogue(std::false_type{});
    else epilogue(std::true_type{});
    asm volatile("" ::: "memory");
    stamp(5);
    ++tix;
    if (!has_next) break;
    relax = interior ? S : 0;
  }
  wait_vmcnt<0>();
  if (e.stamps != nullptr && wave == 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int i = lane; i < 16 * 8; i += 64) e.stamps[blockIdx.x * 128 + i] = stl[i];
  }
}

#endif  // RF_GEMM_EXPERIMENTS


#if defined(RF_GEMM_EXPERIMENTS)  // retired main loop (tools/build_variant.sh builds only)
template <typename E, int EPI, bool CF32, bool RF32>
static void launch_pp(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                      hipStream_t s) {
  constexpr size_t lds = CV_OFF + 6 * 1024;  // ring + diagnostic stamp area + column vectors
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_pp<E, EPI, CF32, RF32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 255) / 256;
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_pp<E, EPI, CF32, RF32><<<grid, 512, lds, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm, nTn);
}

#endif  // RF_GEMM_EXPERIMENTS

// ---- 4-wave 256x256 GEMM: one wave per SIMD, 128x128 accumulator block per wave ----------------
// The alternative main loop to the ping-pong (knob gemm_variant 6): 4 waves (2 x 2), each owning a
// 128 x 128 block of the tile (256 accumulator registers), so a K-tile costs 32 ds_read_b128 per wave
// (128 KiB per CU, vs 192 KiB for 8 waves of 64 x 128) against 128 MFMAs. One continuous MFMA stream
// per SIMD with the LDS reads and the operand DMA interleaved into it (no second wave to alternate
// with): each K-tile is two phases of 64 MFMAs — phase A on the ks = 0 fragments while the ks = 1
// fragments of the same K-tile are read, phase B on ks = 1 while the next K-tile's ks = 0 fragments
// are read and the K-tile after that is DMA'd into the buffer this one just released. One barrier
// per K-tile (between the phases) publishes the next K-tile and releases the current buffer. Same
// LDS image (XOR-swizzled 128-B rows), W-row permutation and epilogue as the ping-pong kernel; the
// next tile's first two K-tiles are fetched across the tile boundary (virtual K-tiles nk, nk+1).
constexpr int W4_BUF = 4 * PP_HALF;          // one K-tile: A rows 0-127, 128-255, W rows 0-127, 128-255
constexpr int W4_CV = 2 * W4_BUF;            // column vectors [parity][3][1 KiB]
constexpr int W4_PF = W4_CV + 6 * 1024;     // L2-prefetch landing area, 256 B per wave (never read)
constexpr int W4_LDS = W4_PF + 1024;

// NJ = 16-column W fragments per wave: 8 = the 256 x 256 tile; 6 = a 256 x 192 tile (each wave 128 x 96,
// W halves of 96 rows) for the N = 768 products at the training batch, whose 192 tiles of 256^2 leave a
// quarter of the 256 CUs idle while 256 tiles of 256 x 192 fill them in one round (EPI_NONE / EPI_BIAS,
// 16-bit C; a lane then owns 6 consecutive output columns: 12-B stores).
template <typename E, int EPI, bool CF32, bool RF32, bool IL, int NJ = 8>
__global__ void __launch_bounds__(256, 1)
    k_gemm_w4(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e,
              int nTm, int nTn) {
  typedef typename H16<E>::x8 V8;
  constexpr bool OUT32 = CF32 || EPI == RF_EPI_COS;
  static_assert(NJ == 8 || (NJ == 6 && IL && !OUT32 && !RF32 &&
                            (EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_RESID)),
                "k_gemm_w4: the 192-column tile takes the 16-bit EPI_NONE / EPI_BIAS / EPI_BIAS_RESID forms only");
  constexpr int TN = 32 * NJ;   // tile columns (256 or 192)
  constexpr int NP = 8 + NJ;    // DMA pieces (and fragment reads) per wave and K-tile: 8 of A, NJ of W
  // epilogue stores per wave (interior tile); EPI_BIAS_GELU_AUX stores the pre-activation too
  constexpr int S = (OUT32 || EPI == RF_EPI_BIAS_GELU_AUX) ? 64 : 32;
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
  const int wr = wave >> 1, wc = wave & 1;  // A half (rows 128 wr..) and W half (columns 16 NJ wc..)
  const int nk = K >> 6;
  // Operand DMA through buffer resources (buffer_load ... lds): rows past M / N read as zeros
  // (num_records), the per-piece row step and the K-tile offset are scalars (soffset), so a piece
  // costs no VALU. Wave w stages rows [64(w&1), +64) of A-half w>>1 and of W-half w>>1 as 8 pieces
  // of 8 rows; lane: row 8p + lane/8 of the piece, 16-B chunk (lane&7)^(row&7). W rows permuted
  // by wperm (whole-line epilogue stores): W row of piece p = 8(l>>3) + 4(w&1) + 64(p&1) + (p>>1)
  // (16-bit out) or 64(w&1) + 4(l>>3) + 32(p&1) + (p>>1) (fp32 out), relative to the half.
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)min((int64_t)e.M * lda * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)min((int64_t)e.N * ldw * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const int half = wave >> 1;
  const int pch = ((lane & 7) ^ (lane >> 3)) * 8;                      // element offset of the chunk
  const int arow_l = half * 128 + (wave & 1) * 64 + (lane >> 3);      // + 8p
  // NJ = 6: W-half rows 48 (w&1) + 8 p + r of the LDS image hold fragment j = 3 (w&1) + (p>>1), column c =
  // 8 (p&1) + r, i.e. W row 6 c + j = 48 (p&1) + 6 r + 3 (w&1) + (p>>1) of the 96-row half
  const int wrow_l = NJ == 6 ? half * 96 + 6 * (lane >> 3) + 3 * (wave & 1)
                             : half * 128 + (OUT32 ? 64 * (wave & 1) + 4 * (lane >> 3) : 8 * (lane >> 3) + 4 * (wave & 1));
  auto voffA = [&](int bm0) { return ((bm0 + arow_l) * lda + pch) * 2; };
  auto voffW = [&](int bn0) { return ((bn0 + wrow_l) * ldw + pch) * 2; };
  int vA = voffA(m0), vW = voffW(n0), vAn = vA, vWn = vW;
  auto launder = [&]() { asm volatile("" : "+v"(vA), "+v"(vW), "+v"(vAn), "+v"(vWn)); };
  // The per-piece soffsets run as two chains (A: +8 rows per piece; W pieces issued in the order
  // pp = 0,2,4,6,1,3,5,7, i.e. rows +0..3 then +64..67 (+32..35 fp32 out): +1 row, +61 (+29) once).
  // Three row-step scalars stay live instead of 14 loop-invariant products, which hipcc spilled to
  // VGPR lanes and reloaded with v_readlane inside phase B (one per piece).
  const int stA = 8 * lda * 2, stW1 = ldw * 2, stWj = (NJ == 6 ? 46 : OUT32 ? 29 : 61) * ldw * 2;
  int sA = 0, sW = 0;
  // piece p (0-7 A, 8-15 W) of virtual K-tile kv (>= nk: the next tile's K-tile kv - nk) into buffer
  // buf; pieces 0 and 8 start their chain, so every K-tile issues p = 0..7 and 8..15 in order
  auto dma_piece = [&](int kv, int buf, int p) {
#if defined(RF_W4_DIAG) && (RF_W4_DIAG & 2)  // timing diagnostic: no operand DMA in the K-loop
    if (kv >= 2) return;
#endif
    const bool nxt = kv >= nk;
    const int kt = nxt ? kv - nk : kv;
    const bool isA = p < 8;
    const int q = isA ? p : p - 8;
    const int pp = isA ? q : (q < NJ / 2 ? 2 * q : 2 * (q - NJ / 2) + 1);
    char* dst = smem + buf * W4_BUF + (isA ? half : 2 + half) * PP_HALF +
                ((wave & 1) * (isA ? 64 : 8 * NJ) + 8 * pp) * 128;
    if (p == 0) { sA = kt * 128; asm volatile("" : "+s"(sA)); }
    if (p == 8) { sW = kt * 128; asm volatile("" : "+s"(sW)); }
    const int soff = isA ? sA : sW;
    {
      int st = isA ? stA : (q == NJ / 2 - 1 ? stWj : stW1);
      asm volatile("" : "+s"(st));  // no hoisting of per-piece products out of the K-loop
      if (isA) sA += st; else sW += st;
    }
#if defined(RF_W4_DIAG) && (RF_W4_DIAG & 8)
    const int rstep = isA ? 8 * pp : (OUT32 ? 32 * (pp & 1) + (pp >> 1) : 64 * (pp & 1) + (pp >> 1));
#endif
    const int vo = isA ? (nxt ? vAn : vA) : (nxt ? vWn : vW);
#if defined(RF_W4_DIAG) && (RF_W4_DIAG & 8)  // timing diagnostic: every DMA reads K-tile 0 (L2-hot)
    const int soffd = rstep * (isA ? lda : ldw) * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsA : rsW, (__attribute__((address_space(3))) void*)dst, 16, vo,
                                             kv < 2 ? soff : soffd, 0, 0);
#else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rsA : rsW, (__attribute__((address_space(3))) void*)dst, 16, vo,
                                             soff, 0, 0);
#endif
  };
  auto dma_cols = [&](int tm0, int tn0, int par) {
    if (EPI == RF_EPI_NONE || EPI == RF_EPI_DGELU) return;
    const int vec = wave % 3;
    const float* src = EPI == RF_EPI_COS ? e.rw : e.bias;
    int idx = min(tn0 + 4 * lane, e.N - 4);
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 1) src = e.lgamma;
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 2) src = e.lbeta;
    if (EPI == RF_EPI_COS && vec == 1) {
      src = e.ra;
      idx = min(tm0 + 4 * lane, e.M - 4);
    }
    glds16(src + idx, smem + W4_CV + (par * 3 + vec) * 1024);
  };
  const int lr = lane & 15;
  const int off0 = lr * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
  const int off1 = lr * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  const int aOff = wr * PP_HALF, bOff = (2 + wc) * PP_HALF;
  V8 a0[8], b0[NJ], a1[8], b1[NJ];
  f32x4 acc[8][NJ];
  auto read0 = [&](int buf, int idx) {  // ks = 0 fragment idx (0-7 A, 8..8+NJ-1 W)
#if defined(RF_W4_DIAG) && (RF_W4_DIAG & 4)  // timing diagnostic: no LDS operand reads
    if (idx < 8) asm volatile("" : "=v"(a0[idx])); else asm volatile("" : "=v"(b0[idx - 8]));
    return;
#endif
    const char* base = smem + buf * W4_BUF + (idx < 8 ? aOff : bOff) + (idx < 8 ? idx : idx - 8) * 16 * 128 + off0;
    if (idx < 8) a0[idx] = *reinterpret_cast<const V8*>(base);
    else b0[idx - 8] = *reinterpret_cast<const V8*>(base);
  };
  auto read1 = [&](int buf, int idx) {
#if defined(RF_W4_DIAG) && (RF_W4_DIAG & 4)
    if (idx < 8) asm volatile("" : "=v"(a1[idx])); else asm volatile("" : "=v"(b1[idx - 8]));
    return;
#endif
    const char* base = smem + buf * W4_BUF + (idx < 8 ? aOff : bOff) + (idx < 8 ? idx : idx - 8) * 16 * 128 + off1;
    if (idx < 8) a1[idx] = *reinterpret_cast<const V8*>(base);
    else b1[idx - 8] = *reinterpret_cast<const V8*>(base);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // L2 prefetch (e.pf): at the end of phase B(t), one dword per operand row (lane = row) of virtual
  // K-tile t + 2 + pfd, as a 4-B LDS-DMA into a landing area nothing reads (no register is written
  // asynchronously). It is the youngest memory operation at the next mid-sync, which waits for all
  // but it (vmcnt(npf)): a prefetch has two phases to land before a wait covers it, and the DMA of
  // its K-tile later hits L2 instead of waiting one HBM latency. Not issued in a tile's last phase B
  // (the relaxed wait of the next tile's first mid-sync counts only the epilogue stores).
  const int pfd = e.pf & 0xff;
  const int npf = pfd ? 1 + ((e.pf >> 8) & 1) : 0;
  auto prefetch = [&](int kv) {
    const bool nxt = kv >= nk;
    const int kt = min(nxt ? kv - nk : kv, nk - 1);
    const int prow = wave * 64 + lane;
    auto* dst = (__attribute__((address_space(3))) void*)(smem + W4_PF + wave * 256);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 4, ((nxt ? nm0 : m0) + prow) * lda * 2, kt * 128, 0, 0);
    if (npf == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, dst, 4, ((nxt ? nn0 : n0) + prow) * ldw * 2, kt * 128, 0, 0);
  };

  // prologue: K-tiles 0, 1 of the first tile, its column vectors
  dma_cols(m0, n0, 0);
#pragma unroll
  for (int p = 0; p < NP; ++p) dma_piece(0, 0, p);
#pragma unroll
  for (int p = 0; p < NP; ++p) dma_piece(1, 1, p);
  wait_vmcnt<NP>();
  bar();
#pragma unroll
  for (int i = 0; i < NP; ++i) read0(0, i);
  int kb = 0;      // LDS buffer of the current K-tile (running parity across tiles)
  int tix = 0;     // tile counter (column-vector parity)
  int relax = 0;   // epilogue stores of the previous (interior) tile still counted in vmcnt
  for (;;) {
    const bool has_next = v + (int)gridDim.x < tiles;  // virtual K-tiles nk, nk+1 = its K-tiles 0, 1
    if (has_next) {
      tile_origin(v + gridDim.x, nm0, nn0);
    } else {
      nm0 = m0;
      nn0 = n0;
    }
    vAn = voffA(nm0);
    vWn = voffW(nn0);
    // ---- phase A: ks = 0 MFMAs of K-tile t; ks = 1 fragments of K-tile t from LDS ----
    auto phaseA = [&](auto zero) {
      // W fragments first: phase B's MFMA order (i outer, j inner) needs all of b1 and a1[0] first
#pragma unroll
      for (int i = 0; i < NP; ++i) read1(kb, i < NJ ? 8 + i : i - NJ);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = mfma16(a0[i], b0[j], decltype(zero)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
      if constexpr (NJ == 8) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
      } else {
#pragma unroll
        for (int g = 0; g < NP; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // 3 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8 * NJ - 3 * NP, 0);
      }
    };
    // ---- mid-sync: this wave's reads of buffer kb done; K-tile t+1 (buffer kb^1) landed ----
    auto midsync = [&](int t) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t == 0 && relax) wait_vmcnt<(S < 63 ? S : 63)>();  // the previous tile's stores may stay in flight
      else if (t > 0 && npf == 1) wait_vmcnt<1>();          // the prefetch of phase B(t-1) may stay in flight
      else if (t > 0 && npf == 2) wait_vmcnt<2>();
      else wait_vmcnt<0>();
#if !(defined(RF_W4_DIAG) && (RF_W4_DIAG & 1))  // timing diagnostic: no barrier (wrong results)
      bar();
#endif
    };
    // ---- phase B: ks = 1 MFMAs; K-tile t+1's ks = 0 fragments; DMA of K-tile t+2 into kb ----
    // unconditional (branch-free phase): past the last tile the reads and the DMA (of the last
    // tile's own rows, into the buffer nothing reads any more) are harmless. The LDS reads may not
    // move above an LDS-DMA write the compiler cannot tell apart from them, so program order
    // alternates them (IL) or puts the DMAs first, and the groups follow that order.
    auto phaseB = [&](int t) {
      if (IL) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          dma_piece(t + 2, kb, p);
          read0(kb ^ 1, p < NJ ? 8 + p : p - NJ);  // b0 first (phase A's MFMA order)
        }
      } else {
#pragma unroll
        for (int p = 0; p < 16; ++p) dma_piece(t + 2, kb, p);
      }
      if (!IL) {
#pragma unroll
        for (int i = 0; i < 16; ++i) read0(kb ^ 1, i);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
      if (IL && NJ == 8) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
      } else if (IL) {
#pragma unroll
        for (int g = 0; g < NP; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8 * NJ - 3 * NP, 0);
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
      } else {
#pragma unroll
        for (int g = 0; g < 17; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
        }
#pragma unroll
        for (int g = 0; g < 15; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if (npf && t + 1 < nk && t + 2 + pfd < 2 * nk) prefetch(t + 2 + pfd);
      kb ^= 1;
    };
    if (IL) {  // the first phase A initialises the accumulators (MFMA with a zero C operand)
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
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int t = 0; t < nk; ++t) {
        launder();
        phaseA(std::false_type{});
        midsync(t);
        phaseB(t);
      }
    }
    // epilogue straight from the accumulators (as k_gemm_pp): lane (c = l&15, g = l>>4) holds rows
    // 4g + r of each 16-row block i and the columns [8c, 8c+8) (16-bit) / [4c, 4c+4) u [64+4c, ..)
    const bool interior = (m0 + 256 <= e.M) && (n0 + TN <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    const int erow = m0 + wr * 128 + 4 * (el >> 4);
    const int ecol = n0 + wc * (16 * NJ) + (OUT32 ? 4 : NJ) * (el & 15);
    float bv[8], gm[8], bt[8];
    const float* cb = reinterpret_cast<const float*>(smem + W4_CV + (tix & 1) * 3 * 1024);
    {
      const int co = ecol - n0;
      if (NJ == 6) {  // 6 columns at a 24-B offset: 8-B reads
#pragma unroll
        for (int k = 0; k < 8; ++k) bv[k] = gm[k] = bt[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 6; k += 2) {
          const f32x2 b = *reinterpret_cast<const f32x2*>(cb + co + k);
          bv[k] = b[0];
          bv[k + 1] = b[1];
        }
      } else if (OUT32) {
        lds_cols<EPI, 4>(cb, co, bv, gm, bt);
        lds_cols<EPI, 4>(cb, co + 64, bv + 4, gm + 4, bt + 4);
      } else {
        lds_cols<EPI, 8>(cb, co, bv, gm, bt);
      }
    }
    const int em0 = m0;
    const void* tbase = reinterpret_cast<const E*>(e.C) + (int64_t)m0 * e.ldc;
    constexpr bool FSC = !OUT32 && (EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX ||
                                    EPI == RF_EPI_BIAS_RESID);
    float csc = 1.f;
    if (FSC) {
      csc = ecol < e.scale_cols ? e.col_scale : 1.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) bv[k] *= csc;
    }
    auto epilogue = [&](auto check) {
      constexpr bool CK = decltype(check)::value;
      // interior EPI_DGELU tiles: the lane's pre-activation rows stream ZD rows ahead of their use
      // (row k + ZD is loaded before row k is computed), so a row's wait covers one load issued ZD
      // rows earlier instead of a memory round trip per row (a load next to its use made hipcc wait
      // vmcnt(0), draining the row's previous store and the next tile's operand DMA with it)
      // (the same for a 16-bit residual row, EPI_BIAS_RESID: the training dA GEMM that adds the other
      // consumer's gradient, train._GradMailbox)
      constexpr bool ZP = !CK && !OUT32 && (EPI == RF_EPI_DGELU || (EPI == RF_EPI_BIAS_RESID && !RF32));
      if constexpr (ZP) {
        constexpr int ZD = 16;  // rows in flight (4 VGPRs each)
        const char* zbase = reinterpret_cast<const char*>(e.R) + (int64_t)em0 * e.ldr * (int)sizeof(E);
        auto zload = [&](int k) {
          const int row = erow + (k >> 2) * 16 + (k & 3);
          const char* zp = zbase + (uint32_t)(((row - em0) * e.ldr + ecol) * (int)sizeof(E));
          if constexpr (NJ == 6) {  // the lane's 6 columns: one 12-B load
            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
            typedef uint32_t u32x3_t __attribute__((ext_vector_type(3)));
            const u32x3_t w = *reinterpret_cast<const u32x3_t*>(zp);
            return __builtin_bit_cast(V8, u32x4_t{w[0], w[1], w[2], 0u});
          } else {
            return *reinterpret_cast<const V8*>(zp);
          }
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
          for (int f = 0; f < 8; ++f) vv[f] = f < NJ ? acc[i][f < NJ ? f : 0][r] : 0.f;
          epi_seg<E, EPI, CF32, RF32, NJ == 6 ? 6 : 8, CK, true, FSC, true>(e, erow + i * 16 + r, ecol, vv, bv, gm, bt,
                                                                           0.f, tbase, em0, csc, z);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float vv[8];
#pragma unroll
            for (int f = 0; f < 8; ++f) vv[f] = f < NJ ? acc[i][f < NJ ? f : 0][r] : 0.f;
            const int row = erow + i * 16 + r;
            const float rsc = EPI == RF_EPI_COS ? cb[256 + row - em0] : 0.f;
            if (NJ == 6) {
              epi_seg<E, EPI, CF32, RF32, 6, CK, !CK, FSC>(e, row, ecol, vv, bv, gm, bt, rsc, tbase, em0, csc);
            } else if (OUT32) {
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
    // the next tile's column vectors into the other parity slot, once per tile and outside the
    // K-loop: that slot was last read by the previous tile's epilogue, which every wave finished
    // before this tile's first barrier; the next tile's second mid-sync waits for it
    if (has_next) dma_cols(nm0, nn0, (tix + 1) & 1);
    ++tix;
    if (!has_next) break;
    v += gridDim.x;
    m0 = nm0;
    n0 = nn0;
    vA = vAn;
    vW = vWn;
    relax = interior ? S : 0;
  }
  wait_vmcnt<0>();
}

template <typename E, int EPI, bool CF32, bool RF32, bool IL, int NJ = 8>
static void launch_w4(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                      hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_w4<E, EPI, CF32, RF32, IL, NJ>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)W4_LDS);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 32 * NJ - 1) / (32 * NJ);
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_w4<E, EPI, CF32, RF32, IL, NJ><<<grid, 256, W4_LDS, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm,
                                                                   nTn);
}



// the eight-wave ping-pong kernel (rf_gemm_w8.hip): EPI_NONE / EPI_BIAS / EPI_BIAS_GELU, 16-bit C
void gemm_w8(bool half, int epi, int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
             hipStream_t s);
// the four-wave kernel on k-step-split LDS planes (rf_gemm_w8.hip, knob gemm_w4p); false: not instantiated there
bool gemm_w4p(bool half, int epi, bool cf32, int M, int N, int K, const void* A, int lda, const void* W, int ldw,
              const EpiArgs& e, hipStream_t s);

// ---- k_gemm_w32: the encoder GEMMs on w32_run (rf_w32.h) ----------------------------------------
template <typename E, int EPI, bool CF32>
struct W32GemmPol {
  static constexpr int S = 64;  // 64 stores per wave (the DGELU / AUX extras only make the wait stricter)
  EpiArgs e;
  __device__ __forceinline__ void cols(char* slot, int wave, int lane, int tm0, int tn0) const {
    if (EPI == RF_EPI_NONE || EPI == RF_EPI_DGELU) return;
    const int vec = wave % 3;
    const float* src = EPI == RF_EPI_COS ? e.rw : e.bias;
    int idx = min(tn0 + 4 * lane, e.N - 4);
    if (EPI == RF_EPI_COS && vec == 1) {
      src = e.ra;
      idx = min(tm0 + 4 * lane, e.M - 4);
    }
    if (EPI != RF_EPI_COS && vec != 0) return;
    glds16(src + idx, slot + vec * 1024);
  }
  __device__ __forceinline__ void epilogue(f32x16 (&acc)[4][4], const W32Tile& t) const {
    constexpr bool OUT32 = CF32 || EPI == RF_EPI_COS;
  // epilogue: lane (c = l&31, g = l>>5): rows 32i + 8(r>>2) + 4g + (r&3), columns 4c .. 4c+3.
  // One branch-free path for every tile: outputs (and the DGELU / AUX pre-activation rows) go
  // through buffer resources based at the tile's first row with num_records = its valid rows, so
  // rows past M are dropped / read as zeros by the range check, and a lane whose 4 columns lie past
  // N (N % 8 == 0: a 4-column group is all in or all out) gets a base offset >= 2^31, past any
  // num_records. Each row pair's 8 accumulators stream out under a sched_barrier (no copy-out of all
  // 256 next to the next tile's fragments); the DGELU pre-activations are loaded ZD pairs ahead.
  const int m0 = t.m0, n0 = t.n0, wr = t.wr, wc = t.wc;
  const float* cb = t.cb;
  int el = t.lane;
  asm volatile("" : "+v"(el));
  const int rowl = wr * 128 + 4 * (el >> 5);   // tile-relative row (+ 32i + 8(r>>2) + (r&3))
  const int coll = wc * 128 + 4 * (el & 31);   // tile-relative column
  const int ecol = n0 + coll;
  const bool col_ok = ecol < e.N;
  const int rows_valid = min(256, e.M - m0);
  constexpr int CB = OUT32 ? 4 : (int)sizeof(E);
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(e.C) + (int64_t)m0 * e.ldc * CB, (short)0, rows_valid * e.ldc * CB, 0x00020000);
  const uint32_t lbC = col_ok ? (uint32_t)((rowl * e.ldc + ecol) * CB) : 0x80000000u;
  const int rstepC = e.ldc * CB;
  constexpr bool HAS_R = EPI == RF_EPI_DGELU || EPI == RF_EPI_BIAS_GELU_AUX;
  __amdgpu_buffer_rsrc_t rsR = rsC;
  uint32_t lbR = 0;
  int rstepR = 0;
  if (HAS_R) {
    rsR = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(e.R)) + (int64_t)m0 * e.ldr * (int)sizeof(E), (short)0,
        rows_valid * e.ldr * (int)sizeof(E), 0x00020000);
    lbR = col_ok ? (uint32_t)((rowl * e.ldr + ecol) * (int)sizeof(E)) : 0x80000000u;
    rstepR = e.ldr * (int)sizeof(E);
  }
  float bv[4], gm[4], bt[4];
  lds_cols<EPI, 4>(cb, coll, bv, gm, bt);
  float csc = 1.f;
  if (!OUT32) {
    csc = ecol < e.scale_cols ? e.col_scale : 1.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[k] *= csc;
  }
  typedef __attribute__((ext_vector_type(2))) unsigned int U2;
  typedef __attribute__((ext_vector_type(4))) unsigned int U4;
  constexpr int ZD = 8;  // DGELU pre-activation prefetch distance (row pairs)
  U2 zr[ZD][2];
  auto prow = [](int P) { return 32 * (P >> 3) + 8 * ((2 * (P & 7)) >> 2) + ((2 * (P & 7)) & 3); };
  auto zload = [&](int P, U2 (&dst)[2]) {
    const uint32_t o = lbR + (uint32_t)(prow(P) * rstepR);
    dst[0] = __builtin_amdgcn_raw_buffer_load_b64(rsR, o, 0, 0);
    dst[1] = __builtin_amdgcn_raw_buffer_load_b64(rsR, o + rstepR, 0, 0);
  };
  if (EPI == RF_EPI_DGELU) {
#pragma unroll
    for (int P = 0; P < ZD; ++P) zload(P, zr[P]);
  }
  auto pack4 = [](const float* x) {
    typename H16<E>::x4 h;
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = (E)x[k];
    return __builtin_bit_cast(U2, h);
  };
  // compile-time pair index (a runtime loop here, which hipcc leaves for the long DGELU / AUX bodies,
  // indexes the accumulators dynamically and demotes them to scratch)
  static_for<32>([&](auto ir) {
    constexpr int P = decltype(ir)::value;
    constexpr int i = P >> 3, r = 2 * (P & 7);
    constexpr int pr = 32 * i + 8 * (r >> 2) + (r & 3);
    float v[8];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {  // copy-out at the point of use (hipcc otherwise hoists all 256)
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[jb]) : "a"(acc[i][jb][r]));
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[4 + jb]) : "a"(acc[i][jb][r + 1]));
    }
    const uint32_t oC = lbC + (uint32_t)(pr * rstepC);
    if (EPI == RF_EPI_COS) {
      const float s0 = cb[256 + rowl + pr] * e.col_scale, s1 = cb[256 + rowl + pr + 1] * e.col_scale;
      const U4 w0 = __builtin_bit_cast(U4, f32x4{v[0] * s0 * bv[0], v[1] * s0 * bv[1], v[2] * s0 * bv[2], v[3] * s0 * bv[3]});
      const U4 w1 = __builtin_bit_cast(U4, f32x4{v[4] * s1 * bv[0], v[5] * s1 * bv[1], v[6] * s1 * bv[2], v[7] * s1 * bv[3]});
      __builtin_amdgcn_raw_buffer_store_b128(w0, rsC, oC, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(w1, rsC, oC + rstepC, 0, 2);
    } else {
      if (EPI == RF_EPI_DGELU) {
        const U2 z0 = zr[P % ZD][0], z1 = zr[P % ZD][1];
        if (P + ZD < 32) zload(P + ZD, zr[P % ZD]);
        const typename H16<E>::x4 h0 = __builtin_bit_cast(typename H16<E>::x4, z0);
        const typename H16<E>::x4 h1 = __builtin_bit_cast(typename H16<E>::x4, z1);
        float zf[8], d[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          zf[k] = (float)h0[k];
          zf[4 + k] = (float)h1[k];
        }
        dgelu8_erf(zf, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= d[k];
      } else if (EPI != RF_EPI_NONE) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], csc, bv[k & 3]);
      } else if (!CF32) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= csc;
      }
      if (EPI == RF_EPI_BIAS_GELU_AUX) {
        const uint32_t oR = lbR + (uint32_t)(pr * rstepR);
        __builtin_amdgcn_raw_buffer_store_b64(pack4(v), rsR, oR, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(pack4(v + 4), rsR, oR + rstepR, 0, 0);
      }
      if (EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX) {
        f32x2 y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = (f32x2){v[2 * k], v[2 * k + 1]};
        gelu8_bf16out(y);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] = y[k].x;
          v[2 * k + 1] = y[k].y;
        }
      }
      if (CF32) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, f32x4{v[0], v[1], v[2], v[3]}), rsC, oC, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, f32x4{v[4], v[5], v[6], v[7]}), rsC,
                                               oC + rstepC, 0, 2);
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(pack4(v), rsC, oC, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b64(pack4(v + 4), rsC, oC + rstepC, 0, 2);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  });
  }
};

template <typename E, int EPI, bool CF32>
__global__ void __launch_bounds__(256, 1)
    k_gemm_w32(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e,
               int nTm, int nTn) {
  w32_run<E>(K, A, lda, W, ldw, e.M, e.N, e.gn, e.pf, nTm, nTn, W32GemmPol<E, EPI, CF32>{e});
}

template <typename E, int EPI, bool CF32>
static void launch_w32(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                       hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_w32<E, EPI, CF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)W32_LDS);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 255) / 256;
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_w32<E, EPI, CF32><<<grid, 256, W32_LDS, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm, nTn);
}

#if defined(RF_GEMM_EXPERIMENTS)  // retired main loop (tools/build_variant.sh builds only)
// ---- 4-wave 256x256 GEMM on a 4-deep BK = 32 ring (knob gemm_variant 7) ----------------------------
// As k_gemm_w4 (one wave per SIMD, 128 x 128 accumulators per wave), but the K loop walks 32-wide
// K-tiles through a 4-slot LDS ring: iteration g runs the 64 MFMAs of K-tile g from one register set
// while the 16 ds_read_b128 of K-tile g+1 fill the other and the 8 DMA pieces of K-tile g+4 go into
// the slot K-tile g just left (read into registers during iteration g-1, released by its barrier).
// So every DMA has three iterations (~3 x 64 MFMAs) to land, the DMA and LDS reads spread evenly
// over the MFMA stream (8 + 16 per 64), and one barrier per iteration publishes K-tile g+2 and
// releases slot g+1. LDS image: 64-B rows, chunk slot c ^ ((-(r>>2)) & 3) (TileGeo<32>); W rows
// permuted by wperm like the ping-pong kernel, so the epilogue is the same.
constexpr int R4_STAGE = 2 * 256 * 64;       // A 256 x 32 + W 256 x 32 (16-bit)
constexpr int R4_CV = 4 * R4_STAGE;          // column vectors [parity][3][1 KiB], then a dummy slot
constexpr int R4_LDS = R4_CV + 7 * 1024;

template <typename E, int EPI, bool CF32, bool RF32>
__global__ void __launch_bounds__(256, 1)
    k_gemm_w4r(int K, const E* __restrict__ A, int lda, const E* __restrict__ W, int ldw, EpiArgs e,
               int nTm, int nTn) {
  typedef typename H16<E>::x8 V8;
  constexpr bool OUT32 = CF32 || EPI == RF_EPI_COS;
  constexpr int S = OUT32 ? 64 : 32;   // epilogue stores per wave (interior tile)
  constexpr int PER = 9;               // VMEM ops per iteration: 8 operand pieces + 1 column vector
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
    on0 = (g * GN + rem - tm * gw) * 256;
  };
  int m0, n0, nm0, nn0;
  tile_origin(v, m0, n0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = K >> 5;  // 32-wide K-tiles (even: K % 64 == 0)
  // DMA: wave w stages rows [64w, 64w + 64) of the A image and of the W image as 4 pieces of 16 rows
  // each; lane: row 16p + l/4 of the piece, chunk slot l&3 holding source chunk (l&3) ^ ((-(l>>4))&3).
  // W image row rho (0..255) holds W row 128(rho>>7) + wperm(rho & 127): 16-bit out
  // 8(l>>2) + 4(w&1) + p, fp32 out 64(w&1) + 4(l>>2) + p, relative to the half.
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A, (short)0, (int)min((int64_t)e.M * lda * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)min((int64_t)e.N * ldw * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const int sch = ((lane & 3) ^ ((-(lane >> 4)) & 3)) * 8;  // source chunk (elements)
  const int arow_l = 64 * wave + (lane >> 2);
  const int wrow_l = 128 * (wave >> 1) + (OUT32 ? 64 * (wave & 1) + 4 * (lane >> 2) : 8 * (lane >> 2) + 4 * (wave & 1));
  auto voffA = [&](int bm0) { return ((bm0 + arow_l) * lda + sch) * 2; };
  auto voffW = [&](int bn0) { return ((bn0 + wrow_l) * ldw + sch) * 2; };
  int vA = voffA(m0), vW = voffW(n0), vAn = vA, vWn = vW;
  // the 8 pieces of virtual K-tile kv (>= nk: the next output tile's K-tile kv - nk) into ring slot
  // `slot`, then one column-vector piece (cols of the next tile into parity slot cpar, or the dummy)
  auto dma_tile = [&](int kv, int slot) {
    const bool nxt = kv >= nk;
    const int kt = nxt ? kv - nk : kv;
    const int va = nxt ? vAn : vA, vw = nxt ? vWn : vW;
    char* base = smem + slot * R4_STAGE + wave * 64 * 64;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(base + p * 1024), 16,
                                               va, kt * 64 + 16 * p * lda * 2, 0, 0);
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (__attribute__((address_space(3))) void*)(base + 256 * 64 + p * 1024),
                                               16, vw, kt * 64 + p * ldw * 2, 0, 0);
  };
  auto dma_cols = [&](int tm0, int tn0, int dst_off) {
    const int vec = wave % 3;
    const float* src = EPI == RF_EPI_COS ? e.rw : (e.bias != nullptr && EPI != RF_EPI_DGELU ? e.bias
                                                                                              : reinterpret_cast<const float*>(A));
    int idx = min(tn0 + 4 * lane, e.N - 4);
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 1) src = e.lgamma;
    if (EPI == RF_EPI_BIAS_RESID_LN && vec == 2) src = e.lbeta;
    if (EPI == RF_EPI_COS && vec == 1) {
      src = e.ra;
      idx = min(tm0 + 4 * lane, e.M - 4);
    }
    if (EPI == RF_EPI_NONE || EPI == RF_EPI_DGELU) idx = 0;  // a harmless piece (fixed VMEM count)
    glds16(src + idx, smem + dst_off + (dst_off == R4_CV + 6 * 1024 ? 0 : vec * 1024));
  };
  const int lr = lane & 15, ch = lane >> 4;
  const int aRd = (wr * 128 + lr) * 64 + ((ch ^ ((-(lr >> 2)) & 3)) << 4);
  const int bRd = 256 * 64 + (wc * 128 + lr) * 64 + ((ch ^ ((-(lr >> 2)) & 3)) << 4);
  V8 a0[8], b0[8], a1[8], b1[8];
  f32x4 acc[8][8];
  // (16-row blocks keep the row's low bits, so one swizzle offset serves all 8 fragments)
  auto rd = [&](V8 (&a)[8], V8 (&b)[8], int slot, int idx) {
    const char* base = smem + slot * R4_STAGE + (idx & 7) * 16 * 64;
    if (idx < 8) a[idx] = *reinterpret_cast<const V8*>(base + aRd);
    else b[idx - 8] = *reinterpret_cast<const V8*>(base + bRd);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto launder = [&]() { asm volatile("" : "+v"(vA), "+v"(vW), "+v"(vAn), "+v"(vWn)); };

  // one iteration: MFMAs of K-tile t from (xa, xb), reads of K-tile t+1 into (ya, yb), DMA of t+4
  auto iter = [&](V8 (&xa)[8], V8 (&xb)[8], V8 (&ya)[8], V8 (&yb)[8], int t, int g, int cdst) {
    dma_tile(t + 4, g & 3);
    dma_cols(nm0, nn0, cdst);
#pragma unroll
    for (int i = 0; i < 16; ++i) rd(ya, yb, (g + 1) & 3, i);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(xa[i], xb[j], acc[i][j]);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 DMA piece
    }
#pragma unroll
    for (int q = 0; q < 15; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // 3 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 LDS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  };

  // prologue: K-tiles 0..3 of the first tile (+ its column vectors, 9 VMEM ops per K-tile)
  nm0 = m0;
  nn0 = n0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    dma_tile(k, k);
    dma_cols(m0, n0, R4_CV);
  }
  wait_vmcnt<2 * PER>();  // K-tiles 0, 1 landed
  bar();
#pragma unroll
  for (int i = 0; i < 16; ++i) rd(a0, b0, 0, i);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();  // every wave has read slot 0 before iteration 0 refills it
  int g = 0;       // running K-tile counter (ring slot, register-set parity) across tiles
  int tix = 0;     // output-tile counter (column-vector parity)
  int relax = 0;   // epilogue stores of the previous (interior) tile counted in vmcnt
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool has_next = v + (int)gridDim.x < tiles;
    if (has_next) tile_origin(v + gridDim.x, nm0, nn0);
    else {
      nm0 = m0;
      nn0 = n0;
    }
    vAn = voffA(nm0);
    vWn = voffW(nn0);
    const int cslot = R4_CV + ((tix + 1) & 1) * 3 * 1024;
    for (int t = 0; t < nk; t += 2) {
      launder();
      // iteration 0 of a tile writes the dummy slot: a slower wave may still read the other
      // parity slot in the previous tile's epilogue
      iter(a0, b0, a1, b1, t, g, t == 0 ? R4_CV + 6 * 1024 : cslot);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t == 0 && relax) wait_vmcnt<(2 * PER + S < 63 ? 2 * PER + S : 63)>();
      else wait_vmcnt<2 * PER>();
      bar();
      iter(a1, b1, a0, b0, t + 1, g + 1, cslot);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t == 0 && relax) wait_vmcnt<(2 * PER + S < 63 ? 2 * PER + S : 63)>();
      else wait_vmcnt<2 * PER>();
      bar();
      g += 2;
    }
    // epilogue straight from the accumulators (as k_gemm_pp / k_gemm_w4)
    const bool interior = (m0 + 256 <= e.M) && (n0 + 256 <= e.N);
    int el = lane;
    asm volatile("" : "+v"(el));
    const int erow = m0 + wr * 128 + 4 * (el >> 4);
    const int ecol = n0 + wc * 128 + (OUT32 ? 4 : 8) * (el & 15);
    float bv[8], gm[8], bt[8];
    const float* cb = reinterpret_cast<const float*>(smem + R4_CV + (tix & 1) * 3 * 1024);
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
    auto epilogue = [&](auto check) {
      constexpr bool CK = decltype(check)::value;
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
            epi_seg<E, EPI, CF32, RF32, 8, CK>(e, row, ecol, vv, bv, gm, bt, rsc);
          }
        }
    };
    if (interior) epilogue(std::false_type{});
    else epilogue(std::true_type{});
    asm volatile("" ::: "memory");
    ++tix;
    if (!has_next) break;
    v += gridDim.x;
    m0 = nm0;
    n0 = nn0;
    vA = vAn;
    vW = vWn;
    relax = interior ? S : 0;
  }
  wait_vmcnt<0>();
}

template <typename E, int EPI, bool CF32, bool RF32>
static void launch_w4r(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                       hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_w4r<E, EPI, CF32, RF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)R4_LDS);
    attr_set = true;
  }
  const int nTm = (M + 255) / 256, nTn = (N + 255) / 256;
  const int grid = min(nTm * nTn, num_cus());
  k_gemm_w4r<E, EPI, CF32, RF32><<<grid, 256, R4_LDS, s>>>(K, (const E*)A, lda, (const E*)W, ldw, e, nTm, nTn);
}

#endif  // RF_GEMM_EXPERIMENTS

template <typename E, int BM, int BN, int WM, int WN, int BK, int NSTAGE, int EPI, bool CF32, bool RF32>
static void launch_bf16(int M, int N, int K, const void* A, int lda, const void* W, int ldw,
                        const EpiArgs& e, hipStream_t s) {
  constexpr int threads = (BM / WM) * (BN / WN) * 64;
  constexpr size_t lds = (size_t)NSTAGE * (BM + BN) * BK * 2;
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_gemm_bf16<E, BM, BN, WM, WN, BK, NSTAGE, EPI, CF32, RF32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int nTm = (M + BM - 1) / BM, nTn = (N + BN - 1) / BN;
  k_gemm_bf16<E, BM, BN, WM, WN, BK, NSTAGE, EPI, CF32, RF32><<<nTm * nTn, threads, lds, s>>>(
      K, (const E*)A, lda, (const E*)W, ldw, e, nTn);
}

// ---- a few rows (M <= 64): k_gemm_skinny ----------------------------------------------------------
// The CLS-only last layer (B rows: the batch's CLS vectors) and the global query rows: with 128 x 128
// tiles a 64-row product has N / 128 workgroups, each walking all of K alone (FFN2's 64 x 768 x 3072:
// 6 workgroups, ~44 us). Here a workgroup owns 16 output columns and all M (<= 64) rows; its four
// waves split K into quarters (v_mfma_f32_16x16x32: A fragments = 16 rows, B = the 16 W rows), and
// the four partial 64 x 16 tiles are summed in LDS in a fixed order, then the scalar epilogue
// (epi_store: bias and column scale, GELU, the pre-activation output, the GELU backward) writes them.
// Fragments come straight from HBM / L2 (16 B per lane per operand and k-step); N / 16 workgroups.
template <typename E, int EPI, bool CF32>
__global__ void __launch_bounds__(256) k_gemm_skinny(int M, int K, const E* __restrict__ A, int lda,
                                                      const E* __restrict__ W, int ldw, EpiArgs e) {
  typedef typename H16<E>::x8 V8;
  __shared__ float red[4][64][17];
  const int n0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int nmb = (M + 15) >> 4;
  const int kq = K >> 2;  // this wave's quarter of K (a multiple of 32)
  const int k0 = wave * kq;
  const E* wrow = W + (int64_t)(n0 + li) * ldw + k0 + 8 * g;
  const E* arow[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) arow[mb] = A + (int64_t)min(16 * mb + li, M - 1) * lda + k0 + 8 * g;
  f32x4 acc[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = 0; k < kq; k += 32) {
    const V8 b = *reinterpret_cast<const V8*>(wrow + k);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      if (mb < nmb) acc[mb] = mfma16(*reinterpret_cast<const V8*>(arow[mb] + k), b, acc[mb]);
  }
  // D[row 4g + r][col li] of each 16-row block
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][16 * mb + 4 * g + r][li] = acc[mb][r];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx >> 4, col = idx & 15;
    if (row < M) {
      const float v = ((red[0][row][col] + red[1][row][col]) + red[2][row][col]) + red[3][row][col];
      epi_store<E, EPI, CF32, false>(e, row, n0 + col, v);
    }
  }
}

template <typename E, int EPI, bool CF32>
static bool launch_skinny(int M, int N, int K, const void* A, int lda, const void* W, int ldw, const EpiArgs& e,
                          hipStream_t s) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!(M >= 1 && M <= 64 && N % 16 == 0 && K % 128 == 0 && lda % 8 == 0 && ldw % 8 == 0 && al16(A) && al16(W)))
    return false;
  k_gemm_skinny<E, EPI, CF32><<<N / 16, 256, 0, s>>>(M, K, (const E*)A, lda, (const E*)W, ldw, e);
  return true;
}

// Variant selector for A/B timing (knob gemm_variant), tools/gemm_gn.py with the bench epilogues:
//   8 (default) four-wave, phase B DMA and LDS reads alternating, zero-C first MFMAs, W fragments
//     read first; with the stage-wise GELU: qkv 198, out-proj 68.5, FFN1 285, FFN2 247 us
//   6 four-wave, phase B DMAs then reads, accumulators zeroed per tile: 204 / 74 / 303 / 264 us
//   5 ping-pong (8 waves): 220 / 77 / 321 / 264 us
//   7 four-wave on a BK32 4-slot ring, one barrier per 64 MFMAs (slower than 6: 217 / 77 / 315 / 275)
//   1 -> 256^2 BK64 x2, 0 -> 256^2 BK32 x4 register-pipelined ring, 2/3/4 -> 256x128 / 128^2 tiles.
static unsigned long long* g_stamps = nullptr;  // set by rf_debug_gemm_stamps (tools only)

// column groups of 6 tiles: qkv -2.7%, FFN1/FFN2 -1% vs 4 (tools/gemm_gn.py); full width loses on FFN1
static int gemm_gn() { return g_knob[KNOB_GEMM_GN]; }
// L2 prefetch 2 K-tiles ahead for long K only: FFN2 (K = 3072) waits on its A-panel DMA from HBM,
// 241.8 -> 230.2 us in a same-process C2 step A/B; at K = 768 (qkv, out-proj, FFN1) the A panel is
// re-read from L2 by the tiles of its row and the extra loads cost 1-4 % (tools/gemm_gn.py gemm_pf)
static int gemm_pf(int K) { return g_knob[KNOB_GEMM_PF] >= 0 ? g_knob[KNOB_GEMM_PF] : (K >= 2048 ? 2 : 0); }

#if defined(RF_GEMM_EXPERIMENTS)
static int gemm_variant() { return g_knob[KNOB_GEMM_VARIANT]; }
#endif


// The ping-pong kernel DMAs its epilogue column vectors (and EPI_COS row norms) as 16-B
// pieces: they must be 16-B aligned with N (M for the row norms) a multiple of 4.
static bool pp_cols_ok(int M, int N, const EpiArgs& e) {
  auto al16 = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return N >= 4 && N % 4 == 0 && al16(e.bias) && al16(e.rw) && al16(e.lgamma) && al16(e.lbeta) &&
         (e.ra == nullptr || (M >= 4 && M % 4 == 0 && al16(e.ra)));
}

template <typename E, int EPI, bool CF32, bool RF32>
static void dispatch_tile(int M, int N, int K, const void* A, int lda, const void* W, int ldw,
                          const EpiArgs& e, hipStream_t s) {
  if constexpr (!RF32 && (EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU ||
                          EPI == RF_EPI_BIAS_GELU_AUX || EPI == RF_EPI_DGELU)) {
    if (M <= 64 && g_knob[KNOB_GEMM_SKINNY] && launch_skinny<E, EPI, CF32>(M, N, K, A, lda, W, ldw, e, s)) return;
  }
  // 256x256 when the grid still covers the chip; 128x128 for skinny problems
  const long tiles256 = (long)((M + 255) / 256) * ((N + 255) / 256);
  const bool w4_ok = pp_cols_ok(M, N, e) && K % 64 == 0 && K >= 128 && (int64_t)M * lda * 2 < 0x7FFFFFFF &&
                     (int64_t)N * ldw * 2 < 0x7FFFFFFF;
  if (tiles256 >= 128) {
#if defined(RF_GEMM_EXPERIMENTS)
    // retired main loops, compiled only into tools/build_variant.sh builds (A/B of the knob)
    switch (gemm_variant()) {
      case 1: launch_bf16<E, 256, 256, 128, 64, 64, 2, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return;
      case 2: launch_bf16<E, 256, 128, 64, 64, 32, 3, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return;
      case 3: launch_bf16<E, 128, 128, 64, 64, 32, 3, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return;
      case 4: launch_bf16<E, 256, 128, 64, 64, 64, 2, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return;
      case 7: if (w4_ok) { launch_w4r<E, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return; } break;
      case 6: if (w4_ok) { launch_w4<E, EPI, CF32, RF32, false>(M, N, K, A, lda, W, ldw, e, s); return; } break;
      case 5: if (pp_cols_ok(M, N, e)) { launch_pp<E, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s); return; } break;
      default: break;
    }
#endif
    if constexpr (EPI == RF_EPI_DGELU || EPI == RF_EPI_BIAS_GELU_AUX) {
      // A/B: smaller tiles with several workgroups per CU for the epilogue-heavy training shapes
      if (g_knob[KNOB_EPI_TILE] == 1) {
        launch_bf16<E, 128, 128, 64, 64, 32, 4, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
        return;
      }
      if (g_knob[KNOB_EPI_TILE] == 2) {
        launch_bf16<E, 256, 128, 64, 64, 64, 2, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
        return;
      }
    }
    if constexpr (!RF32 && (EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS)) {
      // A/B: the N = 768 GEMMs at the training batch (16k rows: 192 tiles of 256^2 for 256 CUs) on
      // smaller tiles that cover the chip
      if (g_knob[KNOB_MID_TILE] && tiles256 < num_cus()) {
        if (g_knob[KNOB_MID_TILE] == 1) {
          launch_bf16<E, 128, 128, 64, 64, 32, 4, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
          return;
        }
        launch_bf16<E, 256, 128, 64, 64, 64, 2, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
        return;
      }
    }
    if constexpr (!CF32 && !RF32 && (EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_RESID)) {
      // 256 x 192 tiles when the 256^2 grid leaves CUs idle and the 192-wide one fills at most one round
      // (the N = 768 products at the training batch: 192 -> 256 tiles at 16k rows)
      const long tiles192 = (long)((M + 255) / 256) * ((N + 191) / 192);
      if (w4_ok && g_knob[KNOB_GEMM_N192] && tiles256 < num_cus() && tiles192 > tiles256 && tiles192 <= num_cus() &&
          e.scale_cols % 192 == 0 && !g_knob[KNOB_GEMM_MFMA32]) {
        launch_w4<E, EPI, false, false, true, 6>(M, N, K, A, lda, W, ldw, e, s);
        return;
      }
    }
    if constexpr (!RF32 && EPI != RF_EPI_BIAS_RESID && EPI != RF_EPI_BIAS_RESID_LN) {
      const int64_t cb = (CF32 || EPI == RF_EPI_COS) ? 4 : 2;
      const bool w32_ok = N % 8 == 0 && (int64_t)256 * e.ldc * cb < 0x7FFFFFFF &&
                          (int64_t)256 * (e.ldr > 0 ? e.ldr : 0) * 2 < 0x7FFFFFFF;
      if (w4_ok && w32_ok && g_knob[KNOB_GEMM_MFMA32]) {
        launch_w32<E, EPI, CF32>(M, N, K, A, lda, W, ldw, e, s);
        return;
      }
    }
    if constexpr (!CF32 && !RF32 && (EPI == RF_EPI_NONE || EPI == RF_EPI_BIAS || EPI == RF_EPI_BIAS_GELU)) {
      if (w4_ok && g_knob[KNOB_GEMM_W8] && !g_knob[KNOB_GEMM_MFMA32]) {
        gemm_w8(std::is_same<E, f16>::value, EPI, M, N, K, A, lda, W, ldw, e, s);
        return;
      }
    }
    if constexpr (!RF32) {
      if (w4_ok && g_knob[KNOB_GEMM_W4P] && !g_knob[KNOB_GEMM_MFMA32] &&
          gemm_w4p(std::is_same<E, f16>::value, EPI, CF32, M, N, K, A, lda, W, ldw, e, s))
        return;
    }
    if (w4_ok) launch_w4<E, EPI, CF32, RF32, true>(M, N, K, A, lda, W, ldw, e, s);
    else launch_bf16<E, 256, 256, 128, 64, 32, 4, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
  } else {
    launch_bf16<E, 128, 128, 64, 64, 32, 4, EPI, CF32, RF32>(M, N, K, A, lda, W, ldw, e, s);
  }
}

// the 16-bit epilogue / io combinations rf_gemm accepts, for one operand type
template <typename E>
static void gemm16(int epilogue, bool cf, bool rf, int M, int N, int K, const void* A, int lda, const void* W,
                   int ldw, const EpiArgs& e, hipStream_t s) {
  switch (epilogue) {
    case RF_EPI_NONE:
      if (cf) dispatch_tile<E, RF_EPI_NONE, true, false>(M, N, K, A, lda, W, ldw, e, s);
      else dispatch_tile<E, RF_EPI_NONE, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_BIAS:
      if (cf) dispatch_tile<E, RF_EPI_BIAS, true, false>(M, N, K, A, lda, W, ldw, e, s);
      else dispatch_tile<E, RF_EPI_BIAS, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_BIAS_GELU:
      dispatch_tile<E, RF_EPI_BIAS_GELU, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_BIAS_GELU_AUX:
      dispatch_tile<E, RF_EPI_BIAS_GELU_AUX, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_DGELU:
      dispatch_tile<E, RF_EPI_DGELU, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_BIAS_RESID:
      if (cf && rf) dispatch_tile<E, RF_EPI_BIAS_RESID, true, true>(M, N, K, A, lda, W, ldw, e, s);
      else if (cf) dispatch_tile<E, RF_EPI_BIAS_RESID, true, false>(M, N, K, A, lda, W, ldw, e, s);
      else if (rf) dispatch_tile<E, RF_EPI_BIAS_RESID, false, true>(M, N, K, A, lda, W, ldw, e, s);
      else dispatch_tile<E, RF_EPI_BIAS_RESID, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
    case RF_EPI_COS:
      dispatch_tile<E, RF_EPI_COS, false, false>(M, N, K, A, lda, W, ldw, e, s);
      break;
  }
}

}  // namespace rf

using namespace rf;

extern "C" int rf_gemm(int dtype, int M, int N, int K, const void* A, int lda, const void* W,
                       int ldw, const float* bias, const void* resid, int ldr, void* C, int ldc,
                       int io_flags, int epilogue, int scale_cols, float col_scale, const float* ra,
                       const float* rw, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && K > 0, "rf_gemm: bad shape M=%d N=%d K=%d", M, N, K);
  RF_REQUIRE(lda >= K && ldw >= K && ldc >= N, "rf_gemm: bad leading dims");
  RF_REQUIRE((epilogue >= RF_EPI_NONE && epilogue <= RF_EPI_COS) || epilogue == RF_EPI_BIAS_GELU_AUX ||
                 epilogue == RF_EPI_DGELU,
             "rf_gemm: bad epilogue %d", epilogue);
  RF_REQUIRE(epilogue != RF_EPI_DGELU || (dtype != RF_F32 && resid && ldr >= N && !(io_flags & 3)),
             "rf_gemm: EPI_DGELU needs 16-bit operands and the pre-activation (resid) of that type");
  RF_REQUIRE(epilogue != RF_EPI_BIAS_GELU_AUX || (dtype != RF_F32 && resid && ldr >= N && !(io_flags & 3)),
             "rf_gemm: EPI_BIAS_GELU_AUX needs 16-bit operands and a pre-activation output (resid) of that type");
  RF_REQUIRE(epilogue == RF_EPI_NONE || epilogue == RF_EPI_COS || epilogue == RF_EPI_DGELU || bias,
             "rf_gemm: bias required");
  RF_REQUIRE(epilogue != RF_EPI_BIAS_RESID || (resid && ldr >= N), "rf_gemm: residual required");
  RF_REQUIRE(epilogue != RF_EPI_COS || (ra && rw), "rf_gemm: norms required for EPI_COS");
  if (M == 0) return RF_OK;
  EpiArgs e{M, N, bias, resid, ldr, C, ldc, scale_cols, col_scale, ra, rw,
            nullptr, nullptr, nullptr, nullptr, g_stamps, gemm_gn(), gemm_pf(K)};
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16 || dtype == RF_F16) {
    RF_REQUIRE(K % 64 == 0, "rf_gemm(16-bit): K=%d must be a multiple of 64", K);
    RF_REQUIRE(lda % 8 == 0 && ldw % 8 == 0, "rf_gemm(16-bit): lda/ldw must be multiples of 8");
    RF_REQUIRE(ldc % 8 == 0 && (resid == nullptr || ldr % 8 == 0),
               "rf_gemm(16-bit): ldc/ldr must be multiples of 8 (16-B vector epilogue)");
    RF_REQUIRE(scale_cols % 16 == 0, "rf_gemm(16-bit): scale_cols must be a multiple of 16");
    const bool cf = io_flags & RF_IO_C_F32, rf = io_flags & RF_IO_R_F32;
    if (dtype == RF_F16) gemm16<f16>(epilogue, cf, rf, M, N, K, A, lda, W, ldw, e, s);
    else gemm16<bf16>(epilogue, cf, rf, M, N, K, A, lda, W, ldw, e, s);
  } else if (dtype == RF_F32) {
    RF_REQUIRE(K % GF_K == 0, "rf_gemm(f32): K=%d must be a multiple of %d", K, GF_K);
    RF_REQUIRE(lda % 4 == 0 && ldw % 4 == 0, "rf_gemm(f32): lda/ldw must be multiples of 4");
    const int nTm = (M + GF_M - 1) / GF_M, nTn = (N + GF_N - 1) / GF_N;
    switch (epilogue) {
#define C_(E) case E: k_gemm_f32<E><<<nTm * nTn, 256, 0, s>>>(K, (const float*)A, lda, (const float*)W, ldw, e, nTn); break;
      C_(RF_EPI_NONE) C_(RF_EPI_BIAS) C_(RF_EPI_BIAS_GELU) C_(RF_EPI_BIAS_RESID) C_(RF_EPI_COS)
#undef C_
    }
  } else {
    RF_REQUIRE(false, "rf_gemm: bad dtype %d", dtype);
  }
  RF_LAUNCH_CHECK("rf_gemm");
}

extern "C" int rf_gemm_resid_ln(int dtype, int M, int N, int K, const void* A, int lda,
                                const void* W, int ldw, const float* bias, const float* resid_pre,
                                int ldr, const float* r_mean, const float* r_rstd,
                                const float* r_gamma, const float* r_beta, float* C, int ldc,
                                rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && K > 0, "rf_gemm_resid_ln: bad shape M=%d N=%d K=%d", M, N, K);
  RF_REQUIRE(lda >= K && ldw >= K && ldc >= N && ldr >= N, "rf_gemm_resid_ln: bad leading dims");
  RF_REQUIRE(bias && resid_pre && r_mean && r_rstd && r_gamma && r_beta && C,
             "rf_gemm_resid_ln: null pointer");
  if (M == 0) return RF_OK;
  EpiArgs e{M, N, bias, resid_pre, ldr, C, ldc, 0, 1.0f, nullptr, nullptr,
            r_mean, r_rstd, r_gamma, r_beta, g_stamps, gemm_gn(), gemm_pf(K)};
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16) {
    RF_REQUIRE(K % 64 == 0, "rf_gemm_resid_ln(bf16): K=%d must be a multiple of 64", K);
    RF_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 && ldr % 8 == 0,
               "rf_gemm_resid_ln(bf16): leading dims must be multiples of 8");
    dispatch_tile<bf16, RF_EPI_BIAS_RESID_LN, true, true>(M, N, K, A, lda, W, ldw, e, s);
  } else if (dtype == RF_F32) {
    RF_REQUIRE(K % GF_K == 0 && lda % 4 == 0 && ldw % 4 == 0, "rf_gemm_resid_ln(f32): alignment");
    const int nTm = (M + GF_M - 1) / GF_M, nTn = (N + GF_N - 1) / GF_N;
    k_gemm_f32<RF_EPI_BIAS_RESID_LN><<<nTm * nTn, 256, 0, s>>>(K, (const float*)A, lda, (const float*)W,
                                                              ldw, e, nTn);
  } else {
    RF_REQUIRE(false, "rf_gemm_resid_ln: bad dtype %d", dtype);
  }
  RF_LAUNCH_CHECK("rf_gemm_resid_ln");
}

// Diagnostic only (tools/gemm_stamps.py): device buffer of >= gridDim*128 uint64 that the
// ping-pong GEMM fills with per-tile s_memtime stamps; nullptr disables. Not part of the ABI.
extern "C" void rf_debug_gemm_stamps(void* buf) { g_stamps = reinterpret_cast<unsigned long long*>(buf); }
