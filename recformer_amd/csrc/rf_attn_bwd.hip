// Backward of the local (sliding-window) attention branch, bf16 operands / fp32 math
// (the gradient of LongformerSelfAttention's local branch,
// TF:482-604 with the global keys of TF:898-962; the overwritten global query rows TF:612-629
// receive no local gradient).
//
// Forward per query i (non-global, valid): keys = band keys j (|i-j| <= 32, flag 1) plus the
// local K/V rows at the global positions; P = softmax(S), O = P V, S = q k^T (q pre-scaled).
// Backward with dO: dP = dO V^T, delta_i = dO_i . O_i, dS = P o (dP - delta),
//   dq = dS K,  dk_j = sum_i dS_ij q_i,  dv_j = sum_i P_ij dO_i.
//
//   k_band_bwd_q   one workgroup per (64-query block, head, sequence): recomputes S and dP for
//                  its queries (band + global keys), writes dq, the row log-sum-exp (log2
//                  domain) and delta, and dS / P of the global-key columns (reduced over all
//                  queries of the sequence on the host side: they are few).
//   k_band_bwd_kv  one workgroup per (64-key block, head, sequence): for its keys the queries
//                  in band are rows [64y-32, 64y+96); recomputes S^T and dP^T from the saved
//                  log-sum-exp and delta and writes dk, dv (band part; global-key rows get
//                  their gradient from the host reduction).
// Query rows that are padding or global (flag != 1) carry no local gradient: their dO is
// treated as 0 (lse = +inf, delta = 0).
#include <type_traits>

#include "rf_common.h"

namespace rf {

constexpr float BW_NEG_INF = -__builtin_inff();
constexpr float BW_LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_b;
template <typename E>
__device__ __forceinline__ typename H16<E>::x4 trr(const char* p) {  // 16-bit transposed read (bit patterns)
  return __builtin_bit_cast(typename H16<E>::x4, __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_b*)p));
}
__device__ __forceinline__ int bswz128(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }
__device__ __forceinline__ int bswz_el(int row, int col) {
  return row * 128 + (((col >> 3) ^ (row & 7)) << 4) + ((col & 7) << 1);
}
template <typename V4>
__device__ __forceinline__ auto cat8(V4 a, V4 b) {
  typedef decltype(a[0]) E0;
  typedef typename std::remove_cv<typename std::remove_reference<E0>::type>::type E;
  return typename H16<E>::x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// 8-row x 128-B DMA piece `pc` of a [rows][64 bf16] image: rows pc*8 + lane/8 of `base`
// (row index clamped into [0, Lp)), source chunk swizzled so the image is XOR-swizzled.
template <typename E>
__device__ __forceinline__ void dma_rows(const E* base, int ld, int row0, int Lp, char* img, int pc,
                                         int lane) {
  const int row = pc * 8 + (lane >> 3);
  const int ch = (lane & 7) ^ (row & 7);
  const int r = min(max(row0 + row, 0), Lp - 1);
  glds16(base + (int64_t)r * ld + ch * 8, img + pc * 1024);
}

// LDS carve of k_band_bwd_q
constexpr int BQ_Q = 0;        // 64 x 128 B
constexpr int BQ_DO = 8192;    // 64 x 128 B
constexpr int BQ_K = 16384;    // 128 x 128 B (window rows 64x-32 ..)
constexpr int BQ_V = 32768;    // 128 x 128 B
constexpr int BQ_KG = 49152;   // 32 x 128 B
constexpr int BQ_VG = 53248;   // 32 x 128 B
constexpr int BQ_GP = 57344;   // 32 int
constexpr int BQ_MK = 57472;   // 2 x uint64 window ballots (valid & local)
constexpr int BQ_LDS = 57488;

// 4 consecutive gradient values: fp32 (16 B) or bf16 (8 B) output
__device__ __forceinline__ void store_g4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void store_g4(bf16* p, f32x4 v) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}
__device__ __forceinline__ void store_g4(f16* p, f32x4 v) {
  *reinterpret_cast<f16x4*>(p) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
}

template <typename E, typename GT>
__global__ void __launch_bounds__(256) k_band_bwd_q(int Lp, int H, const E* __restrict__ q,
                                                     const E* __restrict__ k, const E* __restrict__ v,
                                                     int ld, const E* __restrict__ o, int ldo,
                                                     const E* __restrict__ dout, int ldd,
                                                     const uint8_t* __restrict__ flags,
                                                     const int32_t* __restrict__ gidx, int gmax,
                                                     GT* __restrict__ dq, int lddq, float* __restrict__ lse2,
                                                     float* __restrict__ delta, float* __restrict__ gds,
                                                     float* __restrict__ gpr, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = Lp >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int x = wg % nqb, bh = wg / nqb;
  const int h = bh % H, b = bh / H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int i0 = 64 * x;
  const E* qh = q + rb * ld + h * 64;
  const E* kh = k + rb * ld + h * 64;
  const E* vh = v + rb * ld + h * 64;
  const E* dh = dout + rb * ldd + h * 64;
  int* gp = reinterpret_cast<int*>(smem + BQ_GP);
  unsigned long long* mk = reinterpret_cast<unsigned long long*>(smem + BQ_MK);
  const int gt = gmax > 16 ? 2 : (gmax > 0 ? 1 : 0);

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    dma_rows(qh, ld, i0, Lp, smem + BQ_Q, 2 * wave + j, lane);
    dma_rows(dh, ldd, i0, Lp, smem + BQ_DO, 2 * wave + j, lane);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    dma_rows(kh, ld, i0 - 32, Lp, smem + BQ_K, 4 * wave + j, lane);
    dma_rows(vh, ld, i0 - 32, Lp, smem + BQ_V, 4 * wave + j, lane);
  }
  if (gt > 0) {
    const int row = wave * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int p = row < gmax ? gidx[(int64_t)b * gmax + row] : -1;
    const int64_t off = (int64_t)(p >= 0 ? p : 0) * ld + ch * 8;
    glds16(kh + off, smem + BQ_KG + wave * 1024);
    glds16(vh + off, smem + BQ_VG + wave * 1024);
  }
  if (threadIdx.x < 32) gp[threadIdx.x] = (int)threadIdx.x < gmax ? gidx[(int64_t)b * gmax + threadIdx.x] : -1;
  if (wave < 2) {  // window rows [64 wave, 64 wave + 64): valid & local key flags
    const int row = i0 - 32 + 64 * wave + lane;
    const int f = (row >= 0 && row < Lp) ? flags[rb + row] : 0;
    const unsigned long long ml = __ballot(f == 1);
    if (lane == 0) mk[wave] = ml;
  }
  // this lane's query and its O fragment (delta = dO . O)
  const int myq = i0 + 16 * wave + li;
  const bool qv = flags[rb + myq] == 1;
  V8 of[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    of[s2] = *reinterpret_cast<const V8*>(o + (rb + myq) * ldo + h * 64 + 32 * s2 + 8 * g);
  wait_vmcnt0();
  __syncthreads();

  V8 qf[2], df[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    qf[s2] = *reinterpret_cast<const V8*>(smem + BQ_Q + bswz128(16 * wave + li, 4 * s2 + g));
    df[s2] = qv ? *reinterpret_cast<const V8*>(smem + BQ_DO + bswz128(16 * wave + li, 4 * s2 + g)) : V8{};
  }
  float dl = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf((float)df[s2][j], (float)of[s2][j], dl);
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);

  // S^T and dP^T over the wave's band (window rows 16w + 16t, t < 5) and the global keys
  f32x4 st[5], dp[5], sg[2], dg[2];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    dp[t] = st[t];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int off = bswz128(16 * wave + 16 * t + li, 4 * s2 + g);
      st[t] = mfma16(*reinterpret_cast<const V8*>(smem + BQ_K + off), qf[s2],
                                                      st[t]);
      dp[t] = mfma16(*reinterpret_cast<const V8*>(smem + BQ_V + off), df[s2],
                                                      dp[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    dg[t] = sg[t];
    if (t < gt) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int off = bswz128(16 * t + li, 4 * s2 + g);
        sg[t] = mfma16(*reinterpret_cast<const V8*>(smem + BQ_KG + off),
                                                        qf[s2], sg[t]);
        dg[t] = mfma16(*reinterpret_cast<const V8*>(smem + BQ_VG + off),
                                                        df[s2], dg[t]);
      }
    }
  }
  // allowed: valid & local window key, |key - query| <= 32 (span bits [li, li + 64]), global
  // slot occupied
  unsigned int aw[3];
  {
    const int ks = 16 * wave;
    const unsigned long long ml0 = mk[0], ml1 = mk[1];
    const unsigned long long lo = ks ? ((ml0 >> ks) | (ml1 << (64 - ks))) : ml0;
    const unsigned long long hi = ml1 >> ks;
    aw[0] = ((unsigned int)lo & (~0u << li)) >> (4 * g);
    aw[1] = (unsigned int)(lo >> 32) >> (4 * g);
    aw[2] = ((unsigned int)hi & ((2u << li) - 1u)) >> (4 * g);
  }
  float mx = BW_NEG_INF;
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = (aw[t >> 1] >> (16 * (t & 1) + r)) & 1u;
      st[t][r] = ok ? st[t][r] : BW_NEG_INF;
      mx = fmaxf(mx, st[t][r]);
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = t < gt && gp[16 * t + 4 * g + r] >= 0;
      sg[t][r] = ok ? sg[t][r] : BW_NEG_INF;
      mx = fmaxf(mx, sg[t][r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float nmu = mx == BW_NEG_INF ? 0.f : -mx * BW_LOG2E;
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      st[t][r] = __builtin_amdgcn_exp2f(fmaf(st[t][r], BW_LOG2E, nmu));
      l += st[t][r];
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sg[t][r] = __builtin_amdgcn_exp2f(fmaf(sg[t][r], BW_LOG2E, nmu));
      l += sg[t][r];
    }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const bool live = qv && l > 0.f;
  const float il = live ? 1.0f / l : 0.f;
  // P and dS = P (dP - delta); with attention dropout (TF:585-586) the forward used P o Z (Z the
  // regenerated keep mask times 1/(1-p)), so dP = Z o (dO V^T) and delta = dO . O is unchanged
  const uint64_t drow = ((uint64_t)b * H + h) * Lp + myq;
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      st[t][r] *= il;
      const float z = dr.thresh ? attn_keep_scale(dr, drow, Lp, i0 - 32 + 16 * wave + 16 * t + 4 * g + r) : 1.f;
      dp[t][r] = st[t][r] * (z * dp[t][r] - dl);
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sg[t][r] *= il;
      float z = 1.f;
      if (dr.thresh) {
        const int gk = gp[16 * t + 4 * g + r];
        z = gk >= 0 ? attn_keep_scale(dr, drow, Lp, gk) : 0.f;
      }
      dg[t][r] = sg[t][r] * (z * dg[t][r] - dl);
      sg[t][r] *= z;  // gpr: the dropped probabilities (dv of the global-key columns)
    }
  // dq^T[dim][query] = K^T dS^T over 3 key steps of 32 (the last pairs tile 4 with zeros) + globals
  f32x4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rr = 4 * g + (li >> 2);
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    V8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = 2 * s2 + (j >> 2);
      pf[j] = (E)(t < 5 ? dp[t < 5 ? t : 4][j & 3] : 0.f);
    }
    const int ga = 16 * wave + 32 * s2, gb = s2 < 2 ? ga + 16 : ga;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V8 kf = cat8(trr<E>(smem + BQ_K + bswz_el(ga + rr, col)), trr<E>(smem + BQ_K + bswz_el(gb + rr, col)));
      acc[dt] = mfma16(kf, pf, acc[dt]);
    }
  }
  if (gt > 0) {
    V8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (E)dg[j >> 2][j & 3];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V8 kf = cat8(trr<E>(smem + BQ_KG + bswz_el(rr, col)), trr<E>(smem + BQ_KG + bswz_el(16 + rr, col)));
      acc[dt] = mfma16(kf, pf, acc[dt]);
    }
  }
  GT* dqr = dq + (rb + myq) * lddq + h * 64 + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) store_g4(dqr + 16 * dt, live ? acc[dt] : f32x4{0.f, 0.f, 0.f, 0.f});
  const int64_t ri = ((int64_t)b * H + h) * Lp + myq;
  if (g == 0) {
    lse2[ri] = live ? -nmu + __log2f(l) : __builtin_inff();
    delta[ri] = live ? dl : 0.f;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gk = 16 * t + 4 * g + r;
      if (gk < gmax) {
        gds[ri * gmax + gk] = live ? dg[t][r] : 0.f;
        gpr[ri * gmax + gk] = live ? sg[t][r] : 0.f;
      }
    }
}

// LDS carve of k_band_bwd_kv
constexpr int BK_K = 0;        // 64 x 128 B (key block)
constexpr int BK_V = 8192;
constexpr int BK_Q = 16384;    // 128 x 128 B (query window rows 64y-32 ..)
constexpr int BK_DO = 32768;   // 128 x 128 B
constexpr int BK_L = 49152;    // 128 float lse2
constexpr int BK_D = 49664;    // 128 float delta
constexpr int BK_LDS = 50176;

template <typename E, typename GT>
__global__ void __launch_bounds__(256) k_band_bwd_kv(int Lp, int H, const E* __restrict__ q,
                                                      const E* __restrict__ k, const E* __restrict__ v,
                                                      int ld, const E* __restrict__ dout, int ldd,
                                                      const uint8_t* __restrict__ flags,
                                                      const float* __restrict__ lse2,
                                                      const float* __restrict__ delta, GT* __restrict__ dk,
                                                      GT* __restrict__ dv, int lddkv, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = Lp >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int y = wg % nqb, bh = wg / nqb;
  const int h = bh % H, b = bh / H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int j0 = 64 * y;
  const E* qh = q + rb * ld + h * 64;
  const E* kh = k + rb * ld + h * 64;
  const E* vh = v + rb * ld + h * 64;
  const E* dh = dout + rb * ldd + h * 64;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    dma_rows(kh, ld, j0, Lp, smem + BK_K, 2 * wave + j, lane);
    dma_rows(vh, ld, j0, Lp, smem + BK_V, 2 * wave + j, lane);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    dma_rows(qh, ld, j0 - 32, Lp, smem + BK_Q, 4 * wave + j, lane);
    dma_rows(dh, ldd, j0 - 32, Lp, smem + BK_DO, 4 * wave + j, lane);
  }
  float* ls = reinterpret_cast<float*>(smem + BK_L);
  float* ds = reinterpret_cast<float*>(smem + BK_D);
  if (threadIdx.x < 128) {
    const int r = j0 - 32 + threadIdx.x;
    const bool in = r >= 0 && r < Lp;
    const int64_t ri = ((int64_t)b * H + h) * Lp + r;
    ls[threadIdx.x] = in ? lse2[ri] : __builtin_inff();
    ds[threadIdx.x] = in ? delta[ri] : 0.f;
  }
  const int myk = j0 + 16 * wave + li;
  const bool kv1 = flags[rb + myk] == 1;
  wait_vmcnt0();
  __syncthreads();

  V8 kb[2], vb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    kb[s2] = *reinterpret_cast<const V8*>(smem + BK_K + bswz128(16 * wave + li, 4 * s2 + g));
    vb[s2] = *reinterpret_cast<const V8*>(smem + BK_V + bswz128(16 * wave + li, 4 * s2 + g));
  }
  // S and dP for query window rows 16w + 16t + 4g + r (t < 5) against this lane's key
  f32x4 st[5], dp[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    dp[t] = st[t];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int off = bswz128(16 * wave + 16 * t + li, 4 * s2 + g);
      st[t] = mfma16(*reinterpret_cast<const V8*>(smem + BK_Q + off), kb[s2],
                                                      st[t]);
      dp[t] = mfma16(*reinterpret_cast<const V8*>(smem + BK_DO + off), vb[s2],
                                                      dp[t]);
    }
  }
  // band: query span index 16t + 4g + r in [li, li + 64]; P from the saved row lse (log2)
  const unsigned int b0 = kv1 ? (~0u << li) : 0u, b2 = kv1 ? ((2u << li) - 1u) : 0u;
  const unsigned int bw[3] = {b0 >> (4 * g), kv1 ? (~0u >> (4 * g)) : 0u, b2 >> (4 * g)};
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const f32x4 lq = *reinterpret_cast<const f32x4*>(ls + 16 * wave + 16 * t + 4 * g);
    const f32x4 dq4 = *reinterpret_cast<const f32x4*>(ds + 16 * wave + 16 * t + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = (bw[t >> 1] >> (16 * (t & 1) + r)) & 1u;
      const float p = ok ? __builtin_amdgcn_exp2f(fmaf(st[t][r], BW_LOG2E, -lq[r])) : 0.f;
      // dropout (TF:585-586): dv from P o Z, dS = P (Z dP' - delta); query row j0 - 32 + 16 w + 16 t + 4 g + r
      const float z = (dr.thresh && ok)
                          ? attn_keep_scale(dr, ((uint64_t)b * H + h) * Lp + (j0 - 32 + 16 * wave + 16 * t + 4 * g + r),
                                            Lp, myk)
                          : 1.f;
      st[t][r] = p * z;
      dp[t][r] = p * (z * dp[t][r] - dq4[r]);
    }
  }
  // dv^T[dim][key] = dO^T P, dk^T[dim][key] = Q^T dS over 3 query steps of 32
  f32x4 av[4], ak[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    av[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    ak[dt] = av[dt];
  }
  const int rr = 4 * g + (li >> 2);
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2) {
    V8 pf, sf;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = 2 * s2 + (j >> 2);
      pf[j] = (E)(t < 5 ? st[t < 5 ? t : 4][j & 3] : 0.f);
      sf[j] = (E)(t < 5 ? dp[t < 5 ? t : 4][j & 3] : 0.f);
    }
    const int ga = 16 * wave + 32 * s2, gb = s2 < 2 ? ga + 16 : ga;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V8 df = cat8(trr<E>(smem + BK_DO + bswz_el(ga + rr, col)), trr<E>(smem + BK_DO + bswz_el(gb + rr, col)));
      const V8 qf = cat8(trr<E>(smem + BK_Q + bswz_el(ga + rr, col)), trr<E>(smem + BK_Q + bswz_el(gb + rr, col)));
      av[dt] = mfma16(df, pf, av[dt]);
      ak[dt] = mfma16(qf, sf, ak[dt]);
    }
  }
  GT* dkr = dk + (rb + myk) * lddkv + h * 64 + 4 * g;
  GT* dvr = dv + (rb + myk) * lddkv + h * 64 + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    store_g4(dkr + 16 * dt, ak[dt]);
    store_g4(dvr + 16 * dt, av[dt]);
  }
}

}  // namespace rf

using namespace rf;

template <typename E, typename GT>
static void launch_band_bwd(int B, int Lp, int H, const void* q, const void* k, const void* v, int ld_qkv,
                            const void* o, int ld_o, const void* dout, int ld_do, const uint8_t* flags,
                            const int32_t* gidx, int gmax, GT* dq, GT* dk, GT* dv, int ld_grad, float* lse2,
                            float* delta, float* gds, float* gpr, const AttnDrop& dr, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_band_bwd_q<E, GT>, hipFuncAttributeMaxDynamicSharedMemorySize, BQ_LDS);
    (void)hipFuncSetAttribute((const void*)k_band_bwd_kv<E, GT>, hipFuncAttributeMaxDynamicSharedMemorySize, BK_LDS);
    attr = true;
  }
  const int nblk = (Lp / 64) * H * B;
  k_band_bwd_q<E, GT><<<nblk, 256, BQ_LDS, s>>>(Lp, H, (const E*)q, (const E*)k, (const E*)v, ld_qkv,
                                             (const E*)o, ld_o, (const E*)dout, ld_do, flags, gidx, gmax, dq,
                                             ld_grad, lse2, delta, gds, gpr, dr);
  k_band_bwd_kv<E, GT><<<nblk, 256, BK_LDS, s>>>(Lp, H, (const E*)q, (const E*)k, (const E*)v, ld_qkv,
                                              (const E*)dout, ld_do, flags, lse2, delta, dk, dv, ld_grad, dr);
}

extern "C" int rf_band_attn_bwd_drop(int dtype, int grad_dtype, int B, int Lp, int H, int hd, int half_w,
                                     const void* q, const void* k, const void* v, int ld_qkv, const void* o, int ld_o,
                                     const void* dout, int ld_do, const uint8_t* flags, const int32_t* gidx,
                                     int gmax, void* dq, void* dk, void* dv, int ld_grad, float* lse2, float* delta,
                                     float* gds, float* gpr, float p_drop, uint64_t seed, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_band_attn_bwd: operands must be bf16 or fp16 (got %d)", dtype);
  RF_REQUIRE(grad_dtype == RF_F32 || grad_dtype == dtype,
             "rf_band_attn_bwd: gradients fp32 or the operand type (got %d for %d)", grad_dtype, dtype);
  RF_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "rf_band_attn_bwd: dropout p=%g outside [0, 1)", p_drop);
  const AttnDrop dr{seed, drop_thresh(p_drop), 1.0f / (1.0f - p_drop), g_seed_dev};
  RF_REQUIRE(hd == 64 && half_w == 32, "rf_band_attn_bwd: head_dim 64 and window 64 only (got %d, %d)", hd,
             2 * half_w);
  RF_REQUIRE(B >= 0 && H > 0 && Lp >= 0 && gmax >= 0 && gmax <= 32, "rf_band_attn_bwd: bad shape");
  RF_REQUIRE(Lp % 64 == 0, "rf_band_attn_bwd: Lp=%d must be a multiple of 64", Lp);
  RF_REQUIRE(ld_qkv % 8 == 0 && ld_o % 8 == 0 && ld_do % 8 == 0 && ld_grad % 4 == 0,
             "rf_band_attn_bwd: alignment");
  RF_REQUIRE(ld_qkv >= H * 64 && ld_o >= H * 64 && ld_do >= H * 64 && ld_grad >= H * 64,
             "rf_band_attn_bwd: bad leading dims");
  RF_REQUIRE(gmax == 0 || (gidx && gds && gpr), "rf_band_attn_bwd: gidx / global outputs required");
  if (B == 0 || Lp == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
#define LB_(E, GT) launch_band_bwd<E, GT>(B, Lp, H, q, k, v, ld_qkv, o, ld_o, dout, ld_do, flags, gidx, gmax, (GT*)dq, \
                                          (GT*)dk, (GT*)dv, ld_grad, lse2, delta, gds, gpr, dr, s)
  if (dtype == RF_F16) {
    if (grad_dtype == RF_F16) LB_(f16, f16);
    else LB_(f16, float);
  } else {
    if (grad_dtype == RF_BF16) LB_(bf16, bf16);
    else LB_(bf16, float);
  }
#undef LB_
  RF_LAUNCH_CHECK("rf_band_attn_bwd");
}

extern "C" int rf_band_attn_bwd_dt(int grad_dtype, int B, int Lp, int H, int hd, int half_w, const void* q,
                                   const void* k, const void* v, int ld_qkv, const void* o, int ld_o,
                                   const void* dout, int ld_do, const uint8_t* flags, const int32_t* gidx, int gmax,
                                   void* dq, void* dk, void* dv, int ld_grad, float* lse2, float* delta, float* gds,
                                   float* gpr, rf_stream_t stream) {
  return rf_band_attn_bwd_drop(RF_BF16, grad_dtype, B, Lp, H, hd, half_w, q, k, v, ld_qkv, o, ld_o, dout, ld_do,
                               flags, gidx, gmax, dq, dk, dv, ld_grad, lse2, delta, gds, gpr, 0.f, 0, stream);
}

extern "C" int rf_band_attn_bwd(int B, int Lp, int H, int hd, int half_w, const void* q, const void* k,
                                const void* v, int ld_qkv, const void* o, int ld_o, const void* dout, int ld_do,
                                const uint8_t* flags, const int32_t* gidx, int gmax, float* dq, float* dk,
                                float* dv, int ld_grad, float* lse2, float* delta, float* gds, float* gpr,
                                rf_stream_t stream) {
  return rf_band_attn_bwd_dt(RF_F32, B, Lp, H, hd, half_w, q, k, v, ld_qkv, o, ld_o, dout, ld_do, flags, gidx, gmax,
                             dq, dk, dv, ld_grad, lse2, delta, gds, gpr, stream);
}
