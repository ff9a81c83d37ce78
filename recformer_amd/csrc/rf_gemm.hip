// MFMA GEMMs with fused epilogues: C[M,N] = epi(A[M,K] . W[N,K]^T).
//
// Replaces the nn.Linear addmm's of the Longformer layer (TF:504-506, 982-984,
// 1064-1071, 1107, 1123) and the scoring product of Similarity (models.py:358-369).
//
// bf16 path: 128x128x64 block tile, 4 waves (2x2) of 64x64, v_mfma_f32_16x16x32_bf16,
// operands staged HBM->LDS by 16-B global_load_lds (lane-linear LDS image, XOR swizzle
// applied on the per-lane SOURCE address and on the ds_read_b128 — guide §5.4 rule 21,
// §5.5 T2), two LDS buffers so the next K tile's DMA overlaps this tile's MFMAs,
// bijective XCD-aware block remap (guide §5 'XCD swizzle must be bijective').
// fp32 path: exact-f32 v_mfma_f32_16x16x4_f32, 64x64x16 tiles, register staging.
#include "rf_common.h"

namespace rf {

struct EpiArgs {
  int M, N;
  const float* bias;
  const void* R;
  int ldr;
  void* C;
  int ldc;
  int scale_cols;
  float col_scale;
  const float* ra;
  const float* rw;
};

template <typename TIN, int EPI, bool CF32, bool RF32>
__device__ __forceinline__ void epi_store(const EpiArgs& e, int row, int col, float v) {
  if (row >= e.M || col >= e.N) return;
  if (EPI == RF_EPI_COS) {
    reinterpret_cast<float*>(e.C)[(int64_t)row * e.ldc + col] = v * e.ra[row] * e.rw[col] * e.col_scale;
    return;
  }
  if (EPI != RF_EPI_NONE) v += e.bias[col];
  if (col < e.scale_cols) v *= e.col_scale;
  if (EPI == RF_EPI_BIAS_GELU) v = gelu_erf(v);
  if (EPI == RF_EPI_BIAS_RESID) {
    if (RF32)
      v += reinterpret_cast<const float*>(e.R)[(int64_t)row * e.ldr + col];
    else
      v += to_f32(reinterpret_cast<const TIN*>(e.R)[(int64_t)row * e.ldr + col]);
  }
  if (CF32)
    reinterpret_cast<float*>(e.C)[(int64_t)row * e.ldc + col] = v;
  else
    reinterpret_cast<TIN*>(e.C)[(int64_t)row * e.ldc + col] = from_f32<TIN>(v);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ------------------------------------------------------------------------------------
// bf16
constexpr int GB_M = 128, GB_N = 128, GB_K = 64;
constexpr int GB_TILE_BYTES = GB_M * GB_K * 2;  // 16 KiB per operand tile

template <int EPI, bool CF32, bool RF32>
__global__ void __launch_bounds__(256) k_gemm_bf16(int K, const bf16* __restrict__ A, int lda,
                                                    const bf16* __restrict__ W, int ldw, EpiArgs e,
                                                    int nTn) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (A tile + W tile) = 64 KiB
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / nTn, tn = wg - tm * nTn;
  const int m0 = tm * GB_M, n0 = tn * GB_N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // per-lane staging sources: wave stages chunks c = wave*4+i (8 rows each) of each tile
  const bf16* asrc[4];
  const bf16* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int ar = min(m0 + row, e.M - 1);
    const int wr = min(n0 + row, e.N - 1);
    asrc[i] = A + (int64_t)ar * lda + ch * 8;
    wsrc[i] = W + (int64_t)wr * ldw + ch * 8;
  }
  auto stage = [&](int kt, int buf) {
    char* as = smem + buf * 2 * GB_TILE_BYTES;
    char* ws = as + GB_TILE_BYTES;
    const int koff = kt * GB_K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(asrc[i] + koff, as + (wave * 4 + i) * 1024);
      glds16(wsrc[i] + koff, ws + (wave * 4 + i) * 1024);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GB_K;
  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* as = smem + cur * 2 * GB_TILE_BYTES;
    const char* ws = as + GB_TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + (lane >> 4);
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = *reinterpret_cast<const bf16x8*>(as + swz128(wm * 64 + i * 16 + (lane & 15), ch));
        b[i] = *reinterpret_cast<const bf16x8*>(ws + swz128(wn * 64 + i * 16 + (lane & 15), ch));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    wait_vmcnt0();
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi_store<bf16, EPI, CF32, RF32>(e, m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r,
                             n0 + wn * 64 + j * 16 + (lane & 15), acc[i][j][r]);
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

}  // namespace rf

using namespace rf;

extern "C" int rf_gemm(int dtype, int M, int N, int K, const void* A, int lda, const void* W,
                       int ldw, const float* bias, const void* resid, int ldr, void* C, int ldc,
                       int io_flags, int epilogue, int scale_cols, float col_scale, const float* ra,
                       const float* rw, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && K > 0, "rf_gemm: bad shape M=%d N=%d K=%d", M, N, K);
  RF_REQUIRE(lda >= K && ldw >= K && ldc >= N, "rf_gemm: bad leading dims");
  RF_REQUIRE(epilogue >= RF_EPI_NONE && epilogue <= RF_EPI_COS, "rf_gemm: bad epilogue %d", epilogue);
  RF_REQUIRE(epilogue == RF_EPI_NONE || epilogue == RF_EPI_COS || bias, "rf_gemm: bias required");
  RF_REQUIRE(epilogue != RF_EPI_BIAS_RESID || (resid && ldr >= N), "rf_gemm: residual required");
  RF_REQUIRE(epilogue != RF_EPI_COS || (ra && rw), "rf_gemm: norms required for EPI_COS");
  if (M == 0) return RF_OK;
  EpiArgs e{M, N, bias, resid, ldr, C, ldc, scale_cols, col_scale, ra, rw};
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16) {
    RF_REQUIRE(K % GB_K == 0, "rf_gemm(bf16): K=%d must be a multiple of %d", K, GB_K);
    RF_REQUIRE(lda % 8 == 0 && ldw % 8 == 0, "rf_gemm(bf16): lda/ldw must be multiples of 8");
    const int nTm = (M + GB_M - 1) / GB_M, nTn = (N + GB_N - 1) / GB_N;
    const size_t lds = 4 * GB_TILE_BYTES;
    const bool cf = io_flags & RF_IO_C_F32, rf = io_flags & RF_IO_R_F32;
    const dim3 grid(nTm * nTn);
    const bf16* Ab = (const bf16*)A;
    const bf16* Wb = (const bf16*)W;
    switch (epilogue) {
      case RF_EPI_NONE:
        if (cf) k_gemm_bf16<RF_EPI_NONE, true, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        else k_gemm_bf16<RF_EPI_NONE, false, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        break;
      case RF_EPI_BIAS:
        if (cf) k_gemm_bf16<RF_EPI_BIAS, true, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        else k_gemm_bf16<RF_EPI_BIAS, false, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        break;
      case RF_EPI_BIAS_GELU:
        k_gemm_bf16<RF_EPI_BIAS_GELU, false, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        break;
      case RF_EPI_BIAS_RESID:
        if (cf && rf) k_gemm_bf16<RF_EPI_BIAS_RESID, true, true><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        else if (cf) k_gemm_bf16<RF_EPI_BIAS_RESID, true, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        else if (rf) k_gemm_bf16<RF_EPI_BIAS_RESID, false, true><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        else k_gemm_bf16<RF_EPI_BIAS_RESID, false, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        break;
      case RF_EPI_COS:
        k_gemm_bf16<RF_EPI_COS, false, false><<<grid, 256, lds, s>>>(K, Ab, lda, Wb, ldw, e, nTn);
        break;
    }
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
