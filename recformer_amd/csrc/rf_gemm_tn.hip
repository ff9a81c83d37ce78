// Weight gradients of the encoder's Linears on MFMA: dW = dC^T A (training backward of every
// nn.Linear, TF:504-514, 1064-1130 and the LM head, models.py:499-510, as autograd computes it).
//
//   C[n][k] = sum_m X[m][n] Y[m][k]      X = dC (M x N), Y = A (M x K), 16-bit, row-major,
//                                        C fp32 (the master weight's dtype), N x K
//
// The reduction runs over the M = B*Lp token rows — long (16k-130k) against a small output (at most
// 3072 x 768 = 36 tiles of 256^2) — so the rows are split S ways (split-K in GEMM terms): S x tiles
// workgroups, each one 256 x 256 output tile over its row range into an fp32 slab, then a fixed-order
// column-parallel reduction of the S slabs (deterministic; optionally adding into an existing
// gradient, the accumulation of several passes' contributions).
//
// k_gemm_tn: 4 waves, one per SIMD, each owning a 128 x 128 block of the tile (256 accumulator
// registers) — the four-wave structure of k_gemm_w4 (rf_gemm.hip) with the operands staged the other
// way round: a K-step is 64 m-rows of X (256 columns n) and of Y (256 columns k), DMA'd as 512-B rows
// (buffer_load ... lds, 16 B per lane, rows past M read as zeros), and the MFMA fragments — 8
// consecutive m for one n (or k) — are read with ds_read_b64_tr_b16 (the 4-row x 16-column transposed
// read, guide T10). The 32-B column blocks of each m-row are XOR-permuted by h(r) = (r & 3) |
// ((r >> 3) & 1) << 2, so the 8 rows one transposed read instruction touches per 32-lane half fall on 8
// different 32-B bank groups (conflict-free); the permutation is applied on the DMA's source address
// (the LDS image stays lane-linear). Per K-step and wave: 128 MFMAs (v_mfma_f32_16x16x32), 64
// transposed reads, 16 DMA pieces; phase A runs the ks = 0 MFMAs while the ks = 1 fragments are read,
// phase B the ks = 1 MFMAs while the next K-step's ks = 0 fragments are read and the K-step after it
// is DMA'd into the buffer this one released; one barrier per K-step.
#include <type_traits>

#include "rf_common.h"

namespace rf {

constexpr int TN_ROWB = 512;             // bytes per staged m-row (256 columns, 16-bit)
constexpr int TN_TILE = 64 * TN_ROWB;    // 32 KiB: 64 m-rows of one operand
constexpr int TN_BUF = 2 * TN_TILE;      // one K-step: X tile, then Y tile
constexpr int TN_LDS = 2 * TN_BUF;       // 128 KiB, two buffers

template <int N>
__device__ __forceinline__ void tn_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ds_read_b64_tr_b16 as inline asm: hipcc (ROCm 7.2) puts an s_waitcnt vmcnt(0) in front of every
// transposed-read builtin that follows an LDS-DMA (it cannot rule out that the DMA writes the bytes
// read), which drains the K-step in flight at each read; plain LDS loads do not get it. The asm reads
// are invisible to the wait pass, so each phase waits for its own reads explicitly (lgkmcnt(0) before
// the MFMAs that consume them), and every read group is pinned between sched_barriers.
template <typename V4>
__device__ __forceinline__ V4 tr_read4(uint32_t addr) {
  V4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

template <typename E>
__global__ void __launch_bounds__(256, 1)
    k_gemm_tn(int M, int N, int K, const E* __restrict__ X, int ldx, const E* __restrict__ Y, int ldy,
              float* __restrict__ slabs, int ldc, int64_t slab_stride, int mchunk, int nTn, int nTk, int S) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T = nTn * nTk;
  const int wg = xcd_remap(blockIdx.x, T * S);  // one XCD runs whole splits: a split's tiles share rows
  const int split = wg / T, tile = wg - split * T;
  const int tn = tile / nTk, tk = tile - tn * nTk;
  const int n0 = tn * 256, k0 = tk * 256;
  const int m_begin = split * mchunk;
  const int m_end = min(M, m_begin + mchunk);
  if (m_begin >= m_end) return;
  const int nk = (m_end - m_begin + 63) >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // X half (columns n 128 wr..) and Y half (columns k 128 wc..)

  // ---- DMA: wave w stages pieces 8w..8w+7 of each operand tile (piece = 2 m-rows x 512 B); lane L
  // writes 16-B chunk position L & 31 of m-row 2p + (L >> 5); that position holds the chunk of
  // logical 32-B block t = (pos >> 1) ^ h(row), half (pos & 1). Rows past M (the last split's tail)
  // read as zeros through the buffer resource; the split boundaries are multiples of 64 rows.
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)min((int64_t)M * ldx * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY =
      __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0, (int)min((int64_t)M * ldy * 2, (int64_t)0x7FFFFFFF), 0x00020000);
  const int prow = lane >> 5;  // + 2p
  const int pos = lane & 31;
  // row parity of the piece's rows: h depends on row & 3 and (row >> 3) & 1; rows 2p + prow
  auto src_col = [&](int row) {
    const int h = (row & 3) | (((row >> 3) & 1) << 2);
    return 16 * ((pos >> 1) ^ h) + 8 * (pos & 1);
  };
  int vX[8], vY[8];  // per-piece voffset (bytes) for the K-step at m_begin
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 2 * (8 * wave + i) + prow;
    vX[i] = ((m_begin + row) * ldx + n0 + src_col(row)) * 2;
    vY[i] = ((m_begin + row) * ldy + k0 + src_col(row)) * 2;
  }
  auto dma = [&](int kt, int buf, int p) {  // piece p: 0-7 X, 8-15 Y
    const bool isX = p < 8;
    const int i = p & 7;
    char* dst = smem + buf * TN_BUF + (isX ? 0 : TN_TILE) + (8 * wave + i) * 1024;
    const int soff = kt * 64 * (isX ? ldx : ldy) * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isX ? rsX : rsY, (__attribute__((address_space(3))) void*)dst, 16,
                                             isX ? vX[i] : vY[i], soff, 0, 0);
  };

  // ---- fragment reads: operand tile f (16 columns), ks (32 m), lane (g = l>>4, q = (l&15)>>2, p = l&3)
  // reads m-rows 32 ks + 8 g + 4 hh + q, columns 16 f + 4 p .. + 3 (block f ^ h, h = q | (g & 1) << 2)
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int hsw = q | ((g & 1) << 2);
  const int rbase = (8 * g + q) * TN_ROWB + 8 * pp;
  int co[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) co[f] = rbase + ((f ^ hsw) << 5);
  const int xoff = wr * 8 * 32, yoff = TN_TILE + wc * 8 * 32;  // the wave's 128-column halves
  V8 xa0[8], yb0[8], xa1[8], yb1[8];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // one transposed read: operand X (or Y) tile f, ks, half hh (m-rows +4) of buffer buf
  auto rd = [&](int buf, int ks, int f, bool isX, int hh) -> V4 {
    return tr_read4<V4>(lds0 + buf * TN_BUF + (isX ? xoff : yoff) + co[f] + ks * 32 * TN_ROWB + hh * 4 * TN_ROWB);
  };
  auto pack = [](V4 lo, V4 hi) { return V8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}; };
  V4 tmp[32];  // one phase's reads: fragment idx (0-7 Y, 8-15 X), halves lo / hi
  // read r (0-31) of a phase: fragment r >> 1 (0-7 Y, 8-15 X: Y first, the MFMA order), half r & 1
  auto issue = [&](int buf, int ks, int r) {
    const int idx = r >> 1;
    tmp[r] = rd(buf, ks, idx & 7, idx >= 8, r & 1);
  };
  auto land = [&](V8 (&xa)[8], V8 (&yb)[8]) {  // after the phase's lgkmcnt(0)
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      yb[f] = pack(tmp[2 * f], tmp[2 * f + 1]);
      xa[f] = pack(tmp[16 + 2 * f], tmp[17 + 2 * f]);
    }
  };
  f32x4 acc[8][8];

  // prologue: K-steps 0 and 1
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(0, 0, p);
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(1, 1, p);
  tn_wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int r = 0; r < 32; ++r) issue(0, 0, r);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);  // nothing that reads the asm loads' registers moves above the wait
  land(xa0, yb0);

  int kb = 0;
  // ---- phase A: ks = 0 MFMAs of K-step t (zero C operand on the first); ks = 1 fragments of t:
  // 32 groups of [2 MFMA, 1 transposed read], pinned in this order ----
  auto phaseA = [&](auto zero) {
#pragma unroll
    for (int s = 0; s < 32; ++s) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = (2 * s + u) >> 3, j = (2 * s + u) & 7;
        acc[i][j] = mfma16(xa0[i], yb0[j], decltype(zero)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
      }
      issue(kb, 1, s);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // ---- mid-sync: this wave's reads of buffer kb done; K-step t+1 (buffer kb^1) landed ----
  auto midsync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    tn_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    land(xa1, yb1);
  };
  // ---- phase B: ks = 1 MFMAs; K-step t+1's ks = 0 fragments; DMA of K-step t+2 into kb ----
  // branch-free (one scheduling region, so the DMA pieces and reads interleave with the MFMAs):
  // past the split's last K-step the DMA fills a buffer nothing reads any more and the reads load
  // fragments nothing uses (rows past M read as zeros, others are in bounds)
  auto phaseB = [&](int t) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = (4 * s + u) >> 3, j = (4 * s + u) & 7;
        acc[i][j] = mfma16(xa1[i], yb1[j], acc[i][j]);
      }
      dma(t + 2, kb, s);
#pragma unroll
      for (int u = 2; u < 4; ++u) {
        const int i = (4 * s + u) >> 3, j = (4 * s + u) & 7;
        acc[i][j] = mfma16(xa1[i], yb1[j], acc[i][j]);
      }
      issue(kb ^ 1, 0, 2 * s);
      issue(kb ^ 1, 0, 2 * s + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // K-step t+1's ks = 0 fragments
    __builtin_amdgcn_sched_barrier(0);
    land(xa0, yb0);
    kb ^= 1;
  };
  phaseA(std::true_type{});
  for (int t = 0; t + 1 < nk; ++t) {
    midsync();
    phaseB(t);
    phaseA(std::false_type{});
  }
  midsync();
  phaseB(nk - 1);

  // ---- epilogue: this split's fp32 slab. Lane (c = l & 15, g) holds rows n = 16 i + 4 g + r and
  // column k = 16 j + c of the wave's block.
  float* out = slabs + (int64_t)split * slab_stride;
  const int col = k0 + wc * 128 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = n0 + wr * 128 + 16 * i + 4 * g + r;
      if (row < N) {
        float* o = out + (int64_t)row * ldc;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (col + 16 * j < K) o[col + 16 * j] = acc[i][j][r];
      }
    }
  tn_wait_vm<0>();  // the (unused) DMA of the last phase B has landed before the workgroup exits
}

// C (=|+=) sum_s slabs[s]: fixed order over s, 4 consecutive floats per thread; rows n < scale_n of the
// sum multiplied by scale first (a Linear's output-column scale, e.g. the query's 1/8: its dW rows)
__global__ void __launch_bounds__(256) k_tn_reduce(int N, int K, const float* __restrict__ slabs, int ld_slab,
                                                   int64_t slab_stride, int S, float* __restrict__ C, int ldc,
                                                   int accumulate, int scale_n, float scale) {
  const int kq = K >> 2;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * kq) return;
  const int n = (int)(idx / kq), k = (int)(idx - (int64_t)n * kq) * 4;
  const float* s0 = slabs + (int64_t)n * ld_slab + k;
  auto ld = [&](int s) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s0 + s * slab_stride));
    return make_float4(v[0], v[1], v[2], v[3]);
  };
  float4 a = ld(0);
  int s = 1;
  // four slabs' loads in flight per step (the adds keep the order s = 1, 2, ...: same sums as one
  // at a time, which waited one memory round trip per slab)
  for (; s + 4 <= S; s += 4) {
    const float4 b0 = ld(s), b1 = ld(s + 1), b2 = ld(s + 2), b3 = ld(s + 3);
    a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w;
    a.x += b1.x; a.y += b1.y; a.z += b1.z; a.w += b1.w;
    a.x += b2.x; a.y += b2.y; a.z += b2.z; a.w += b2.w;
    a.x += b3.x; a.y += b3.y; a.z += b3.z; a.w += b3.w;
  }
  for (; s < S; ++s) {
    const float4 b = ld(s);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  if (n < scale_n) {
    a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
  }
  float* c = C + (int64_t)n * ldc + k;
  if (accumulate) {
    const float4 b = *reinterpret_cast<const float4*>(c);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  *reinterpret_cast<float4*>(c) = a;
}

static int tn_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    n = c > 0 ? c : 256;
  }
  return n;
}

// split count and row chunk: at most one workgroup per CU (the kernel holds a CU: 128 KiB LDS,
// 512 registers a lane), so all of them run in ONE round — ceil(CUs / tiles) splits put 4-32 of them
// into a second round that doubled the kernel's time; each split at least 512 rows
static void tn_plan(int M, int N, int K, int& S, int& mchunk) {
  const int T = ((N + 255) / 256) * ((K + 255) / 256);
  const int cus = g_knob[KNOB_TN_WGS] > 0 ? g_knob[KNOB_TN_WGS] : tn_cus();
  int s = cus / T;
  const int max_s = max(1, M / 512);
  s = max(1, min(s, max_s));
  mchunk = ((M + s - 1) / s + 63) / 64 * 64;
  S = (M + mchunk - 1) / mchunk;
}

template <typename E>
static int launch_tn(int M, int N, int K, const void* X, int ldx, const void* Y, int ldy, float* C, int ldc,
                     int accumulate, int scale_n, float scale, void* ws, size_t ws_bytes, hipStream_t s) {
  int S, mchunk;
  tn_plan(M, N, K, S, mchunk);
  const int nTn = (N + 255) / 256, nTk = (K + 255) / 256;
  const int64_t slab = (int64_t)N * K;
  RF_REQUIRE(ws_bytes >= (size_t)S * slab * 4, "rf_weight_grad: workspace of %zu bytes < %lld needed", ws_bytes,
             (long long)(S * slab * 4));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_gemm_tn<E>, hipFuncAttributeMaxDynamicSharedMemorySize, TN_LDS);
    attr = true;
  }
  k_gemm_tn<E><<<nTn * nTk * S, 256, TN_LDS, s>>>(M, N, K, (const E*)X, ldx, (const E*)Y, ldy, (float*)ws, K, slab,
                                                  mchunk, nTn, nTk, S);
  const int64_t work = (int64_t)N * (K / 4);
  k_tn_reduce<<<(unsigned)((work + 255) / 256), 256, 0, s>>>(N, K, (const float*)ws, K, slab, S, C, ldc, accumulate,
                                                                 scale_n, scale);
  return RF_OK;
}

}  // namespace rf

using namespace rf;

extern "C" size_t rf_weight_grad_workspace(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  int S, mchunk;
  tn_plan(M, N, K, S, mchunk);
  return (size_t)S * N * K * 4;
}

extern "C" int rf_weight_grad(int dtype, int M, int N, int K, const void* X, int ldx, const void* Y, int ldy,
                              float* C, int ldc, int accumulate, int scale_rows, float row_scale, void* workspace,
                              size_t ws_bytes, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && K > 0 && scale_rows >= 0, "rf_weight_grad: bad shape M=%d N=%d K=%d", M, N, K);
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_weight_grad: 16-bit operands only (dtype %d)", dtype);
  RF_REQUIRE(N % 16 == 0 && K % 16 == 0, "rf_weight_grad: N=%d and K=%d must be multiples of 16", N, K);
  RF_REQUIRE(ldx >= N && ldy >= K && ldx % 8 == 0 && ldy % 8 == 0 && ldc >= K && ldc % 4 == 0,
             "rf_weight_grad: bad leading dims");
  RF_REQUIRE((reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(C) & 15) == 0,
             "rf_weight_grad: operands must be 16-byte aligned");
  RF_REQUIRE((int64_t)M * ldx * 2 < 0x7FFFFFFF && (int64_t)M * ldy * 2 < 0x7FFFFFFF,
             "rf_weight_grad: operands above 2 GiB");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (!accumulate) {
      for (int n = 0; n < N; ++n) (void)hipMemsetAsync(C + (int64_t)n * ldc, 0, (size_t)K * 4, s);
    }
    RF_LAUNCH_CHECK("rf_weight_grad");
  }
  int rc = dtype == RF_BF16
               ? launch_tn<bf16>(M, N, K, X, ldx, Y, ldy, C, ldc, accumulate, scale_rows, row_scale, workspace, ws_bytes, s)
               : launch_tn<f16>(M, N, K, X, ldx, Y, ldy, C, ldc, accumulate, scale_rows, row_scale, workspace, ws_bytes, s);
  if (rc != RF_OK) return rc;
  RF_LAUNCH_CHECK("rf_weight_grad");
}
