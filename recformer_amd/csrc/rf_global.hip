// Global-token attention rows via the key/value-projection fold (SURVEY.md §8a row A6, §7
// 'Global-path algebra').
//
// The reference projects key_global / value_global over ALL L tokens of every layer
// (TF:983-984) only to serve the G global query rows (TF:964-1057). Per head h:
//     s_j   = qg_h . (Wkg_h h_j + bkg_h) = u_h . h_j + c_h,   u_h = Wkg_h^T qg_h, c_h = qg_h . bkg_h
//     out_h = sum_j p_j (Wvg_h h_j + bvg_h) = Wvg_h w_h + bvg_h,  w_h = sum_j p_j h_j  (sum p = 1)
// so the two d x d projections over L tokens (4 L d^2 flops/layer, 2/5 of the fused QKV
// GEMM) collapse to two per-head GEMVs plus one streaming pass over h. Same algebra,
// different rounding (fp32 throughout here; checked against the oracle in the tests).
//
//   k_gfold_u       (H, B*G):    u = Wkg_h^T qg_h, c = qg_h . bkg_h        (fp32 workspace)
//   k_gfold_partial (Lp/CH, B*G): per CH-row chunk: s = u.h_j + c (masked to valid keys),
//                                chunk max/sum per head, w_part = sum_j p_j h_j
//   k_gfold_out     (H, B*G):    merge chunks (log-sum-exp), out = Wvg_h w_h + bvg_h,
//                                written into ctx at the global token's row
#include "rf_common.h"

namespace rf {

constexpr float GF_NEG_INF = -__builtin_inff();
constexpr int GF_CH = 64;     // rows per partial chunk
constexpr int GF_HMAX = 16;   // heads handled per block (H <= 16)

struct GfoldWs {
  float* u;      // [R][H][Dp]   (Dp = D + 4, padded rows)
  float* c;      // [R][H]
  float* m;      // [R][nch][H]
  float* l;      // [R][nch][H]
  float* w;      // [R][nch][H][D]
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

__device__ __forceinline__ void load4(const float* p, float* x) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
}
__device__ __forceinline__ void load4(const bf16* p, float* x) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  x[0] = (float)v[0]; x[1] = (float)v[1]; x[2] = (float)v[2]; x[3] = (float)v[3];
}

__host__ __device__ inline GfoldWs gfold_carve(void* ws, int R, int nch, int H, int D) {
  char* p = (char*)ws;
  GfoldWs w;
  w.u = (float*)p; p += align256((size_t)R * H * (D + 4) * 4);
  w.c = (float*)p; p += align256((size_t)R * H * 4);
  w.m = (float*)p; p += align256((size_t)R * nch * H * 4);
  w.l = (float*)p; p += align256((size_t)R * nch * H * 4);
  w.w = (float*)p;
  return w;
}

inline size_t gfold_bytes(int R, int nch, int H, int D) {
  return align256((size_t)R * H * (D + 4) * 4) + align256((size_t)R * H * 4) +
         2 * align256((size_t)R * nch * H * 4) + (size_t)R * nch * H * D * 4;
}

template <typename T>
__global__ void __launch_bounds__(256) k_gfold_u(int D, int H, int gmax, const T* __restrict__ qg,
                                                  int ld_qg, const T* __restrict__ wkg,
                                                  const float* __restrict__ bkg,
                                                  const int32_t* __restrict__ gidx, GfoldWs ws) {
  __shared__ float qs[64];
  const int h = blockIdx.x, r = blockIdx.y;
  if (gidx[r] < 0) return;
  const int t = threadIdx.x;
  if (t < 64) qs[t] = to_f32(qg[(int64_t)r * ld_qg + h * 64 + t]);
  __syncthreads();
  const T* wb = wkg + (int64_t)h * 64 * D;
  float* urow = ws.u + ((int64_t)r * H + h) * (D + 4);
  for (int k = t; k < D; k += 256) {
    float a = 0.f;
#pragma unroll 8
    for (int d = 0; d < 64; ++d) a = fmaf(qs[d], to_f32(wb[(int64_t)d * D + k]), a);
    urow[k] = a;
  }
  if (t < 64) {
    float cv = wave_sum(qs[t] * bkg[h * 64 + t]);
    if (t == 0) ws.c[(int64_t)r * H + h] = cv;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_gfold_partial(int Lp, int D, int H, int gmax,
                                                        const T* __restrict__ hs, int ldh,
                                                        const uint8_t* __restrict__ flags,
                                                        const int32_t* __restrict__ gidx,
                                                        GfoldWs ws) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // u: H x (D+4), p: H x CH
  const int ch = blockIdx.x, r = blockIdx.y, nch = gridDim.x;
  if (gidx[r] < 0) return;
  const int b = r / gmax;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int Dp = D + 4;
  float* us = sm;
  float* ps = sm + H * Dp;
  const float* ug = ws.u + (int64_t)r * H * Dp;
  for (int i = t; i < H * Dp; i += 256) us[i] = ug[i];
  __syncthreads();

  const int j0 = ch * GF_CH;
  const T* hb = hs + (int64_t)b * Lp * ldh;
  // ---- scores: thread -> (row j = t/4, heads hg, hg+4, hg+8, ...) ----
  {
    const int jl = t >> 2, hg = t & 3;
    const int j = j0 + jl;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (j < Lp) {
      const T* hr = hb + (int64_t)j * ldh;
      for (int k = 0; k < D; k += 4) {
        float x[4];
        load4(hr + k, x);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int hh = hg + 4 * i;
          if (hh < H) {
            const float4 uu = *reinterpret_cast<const float4*>(us + hh * Dp + k);
            s[i] = fmaf(x[0], uu.x, fmaf(x[1], uu.y, fmaf(x[2], uu.z, fmaf(x[3], uu.w, s[i]))));
          }
        }
      }
    }
    const bool ok = j < Lp && flags[(int64_t)b * Lp + j] != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hh = hg + 4 * i;
      if (hh < H) ps[hh * GF_CH + jl] = ok ? s[i] + ws.c[(int64_t)r * H + hh] : GF_NEG_INF;
    }
  }
  __syncthreads();
  // ---- chunk softmax statistics per head (one wave per head, lane = row) ----
  for (int hh = wave; hh < H; hh += 4) {
    const float sv = ps[hh * GF_CH + lane];
    const float mx = wave_max(sv);
    const float mu = (mx == GF_NEG_INF) ? 0.f : mx;
    const float p = __expf(sv - mu);
    const float lsum = wave_sum(p);
    ps[hh * GF_CH + lane] = p;
    if (lane == 0) {
      ws.m[((int64_t)r * nch + ch) * H + hh] = mx;
      ws.l[((int64_t)r * nch + ch) * H + hh] = lsum;
    }
  }
  __syncthreads();
  // ---- w_part[h][k] = sum_j p[h][j] h[j][k]; thread -> columns k = t + 256 i ----
  const int jn = min(GF_CH, Lp - j0);
  for (int k0 = 0; k0 < D; k0 += 256) {
    const int k = k0 + t;
    if (k >= D) break;
    float acc[GF_HMAX];
#pragma unroll
    for (int hh = 0; hh < GF_HMAX; ++hh) acc[hh] = 0.f;
    for (int jl = 0; jl < jn; ++jl) {
      const float x = to_f32(hb[(int64_t)(j0 + jl) * ldh + k]);
#pragma unroll
      for (int hh = 0; hh < GF_HMAX; ++hh)
        if (hh < H) acc[hh] = fmaf(ps[hh * GF_CH + jl], x, acc[hh]);
    }
    float* wout = ws.w + (((int64_t)r * nch + ch) * H) * D + k;
#pragma unroll
    for (int hh = 0; hh < GF_HMAX; ++hh)
      if (hh < H) wout[(int64_t)hh * D] = acc[hh];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_gfold_out(int Lp, int D, int H, int gmax, int nch,
                                                    const T* __restrict__ wvg,
                                                    const float* __restrict__ bvg,
                                                    const int32_t* __restrict__ gidx, GfoldWs ws,
                                                    T* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];  // D floats + nch scales
  float* scl = wsm + D;
  __shared__ float lsum_s;
  const int h = blockIdx.x, r = blockIdx.y;
  const int pos = gidx[r];
  if (pos < 0) return;
  const int b = r / gmax;
  const int t = threadIdx.x;
  if (t < 64) {
    float mx = GF_NEG_INF;
    for (int c = t; c < nch; c += 64) mx = fmaxf(mx, ws.m[((int64_t)r * nch + c) * H + h]);
    mx = wave_max(mx);
    float ls = 0.f;
    for (int c = t; c < nch; c += 64) {
      const float mc = ws.m[((int64_t)r * nch + c) * H + h];
      const float sc = (mc == GF_NEG_INF) ? 0.f : __expf(mc - mx);
      scl[c] = sc;
      ls += sc * ws.l[((int64_t)r * nch + c) * H + h];
    }
    ls = wave_sum(ls);
    if (t == 0) lsum_s = ls;
  }
  __syncthreads();
  const float inv = lsum_s > 0.f ? 1.0f / lsum_s : 0.f;
  for (int k = t; k < D; k += 256) {
    float a = 0.f;
    for (int c = 0; c < nch; ++c) a = fmaf(scl[c], ws.w[(((int64_t)r * nch + c) * H + h) * D + k], a);
    wsm[k] = a * inv;
  }
  __syncthreads();
  // out[d] = Wvg[h*64+d] . w + bvg: 4 threads per output row of Wvg
  const int d = t >> 2, qtr = t & 3;
  const T* wr = wvg + (int64_t)(h * 64 + d) * D;
  float a = 0.f;
  for (int k = qtr; k < D; k += 4) a = fmaf(to_f32(wr[k]), wsm[k], a);
  a += __shfl_xor(a, 1, 64);
  a += __shfl_xor(a, 2, 64);
  if (qtr == 0) out[((int64_t)b * Lp + pos) * ldo + h * 64 + d] = from_f32<T>(a + bvg[h * 64 + d]);
}

}  // namespace rf

using namespace rf;

extern "C" size_t rf_global_fold_workspace(int B, int Lp, int D, int H, int gmax) {
  if (B <= 0 || gmax <= 0) return 0;
  const int nch = (Lp + GF_CH - 1) / GF_CH;
  return gfold_bytes(B * gmax, nch, H, D);
}

extern "C" int rf_global_attn_fold_fwd(int dtype, int B, int Lp, int D, int H, const void* qg,
                                       int ld_qg, const void* h, int ldh, const void* wkg,
                                       const float* bkg, const void* wvg, const float* bvg,
                                       const uint8_t* flags, const int32_t* gidx, int gmax,
                                       void* workspace, void* out, int ld_out,
                                       rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && H > 0, "rf_global_attn_fold_fwd: bad shape");
  RF_REQUIRE(D == H * 64, "rf_global_attn_fold_fwd: D=%d must be H*64", D);
  RF_REQUIRE(H <= GF_HMAX, "rf_global_attn_fold_fwd: at most %d heads", GF_HMAX);
  RF_REQUIRE(D % 4 == 0 && ldh >= D && ld_qg >= D && ld_out >= D, "rf_global_attn_fold_fwd: dims");
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(workspace && gidx && flags, "rf_global_attn_fold_fwd: null workspace/gidx/flags");
  const int R = B * gmax;
  const int nch = (Lp + GF_CH - 1) / GF_CH;
  GfoldWs ws = gfold_carve(workspace, R, nch, H, D);
  hipStream_t s = as_stream(stream);
  const size_t lds_p = (size_t)(H * (D + 4) + H * GF_CH) * sizeof(float);
  RF_REQUIRE(lds_p <= 160 * 1024, "rf_global_attn_fold_fwd: D too large for LDS");
  const size_t lds_o = (size_t)(D + nch) * sizeof(float);
  if (dtype == RF_BF16) {
    (void)hipFuncSetAttribute((const void*)k_gfold_partial<bf16>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_p);
    k_gfold_u<bf16><<<dim3(H, R), 256, 0, s>>>(D, H, gmax, (const bf16*)qg, ld_qg, (const bf16*)wkg, bkg, gidx, ws);
    k_gfold_partial<bf16><<<dim3(nch, R), 256, lds_p, s>>>(Lp, D, H, gmax, (const bf16*)h, ldh, flags, gidx, ws);
    k_gfold_out<bf16><<<dim3(H, R), 256, lds_o, s>>>(Lp, D, H, gmax, nch, (const bf16*)wvg, bvg, gidx, ws,
                                                      (bf16*)out, ld_out);
  } else if (dtype == RF_F32) {
    (void)hipFuncSetAttribute((const void*)k_gfold_partial<float>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_p);
    k_gfold_u<float><<<dim3(H, R), 256, 0, s>>>(D, H, gmax, (const float*)qg, ld_qg, (const float*)wkg, bkg, gidx, ws);
    k_gfold_partial<float><<<dim3(nch, R), 256, lds_p, s>>>(Lp, D, H, gmax, (const float*)h, ldh, flags, gidx, ws);
    k_gfold_out<float><<<dim3(H, R), 256, lds_o, s>>>(Lp, D, H, gmax, nch, (const float*)wvg, bvg, gidx, ws,
                                                       (float*)out, ld_out);
  } else {
    RF_REQUIRE(false, "rf_global_attn_fold_fwd: bad dtype %d", dtype);
  }
  RF_LAUNCH_CHECK("rf_global_attn_fold_fwd");
}
