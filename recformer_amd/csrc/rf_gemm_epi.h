// Epilogue helpers and shared constants of the MFMA GEMM kernels (rf_gemm.hip, rf_gemm_w8.hip).
#pragma once
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
  // RF_EPI_BIAS_RESID_LN: residual = LayerNorm(R) recomputed from the fp32 pre-LN rows R and
  // the row statistics the LayerNorm kernel stored (no fp32 copy of the LN output in HBM)
  const float* lmean;
  const float* lrstd;
  const float* lgamma;
  const float* lbeta;
  unsigned long long* stamps;  // diagnostic s_memtime stamps (tools only), nullptr = off
  int gn;                      // ping-pong kernel: column tiles per raster group (0 = all)
  int pf;                      // four-wave kernel: L2 prefetch distance in K-tiles (0 = off); bit 8: W rows too
};

// scalar epilogue (fp32 kernel and ragged tails)
template <typename TIN, int EPI, bool CF32, bool RF32>
__device__ __forceinline__ void epi_store(const EpiArgs& e, int row, int col, float v) {
  if (row >= e.M || col >= e.N) return;
  if (EPI == RF_EPI_COS) {
    // same association as the vector epilogues (v * (ra * scale) * rw): one score, one rounding
    reinterpret_cast<float*>(e.C)[(int64_t)row * e.ldc + col] = v * (e.ra[row] * e.col_scale) * e.rw[col];
    return;
  }
  if (EPI == RF_EPI_DGELU) {  // GELU backward: dz = du * gelu'(z), R = z (16-bit)
    v *= dgelu_erf(to_f32(reinterpret_cast<const TIN*>(e.R)[(int64_t)row * e.ldr + col]));
    if (CF32)
      reinterpret_cast<float*>(e.C)[(int64_t)row * e.ldc + col] = v;
    else
      reinterpret_cast<TIN*>(e.C)[(int64_t)row * e.ldc + col] = from_f32<TIN>(v);
    return;
  }
  if (EPI != RF_EPI_NONE) v += e.bias[col];
  if (col < e.scale_cols) v *= e.col_scale;
  if (EPI == RF_EPI_BIAS_GELU_AUX)
    reinterpret_cast<TIN*>(const_cast<void*>(e.R))[(int64_t)row * e.ldr + col] = from_f32<TIN>(v);
  if (EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX)
    v = (CF32 || sizeof(TIN) == 4) ? gelu_erf(v) : gelu_bf16out(v);  // 16-bit outputs: the fitted form
  if (EPI == RF_EPI_BIAS_RESID) {
    if (RF32)
      v += reinterpret_cast<const float*>(e.R)[(int64_t)row * e.ldr + col];
    else
      v += to_f32(reinterpret_cast<const TIN*>(e.R)[(int64_t)row * e.ldr + col]);
  }
  if (EPI == RF_EPI_BIAS_RESID_LN) {
    const float x = reinterpret_cast<const float*>(e.R)[(int64_t)row * e.ldr + col];
    v += (x - e.lmean[row]) * e.lrstd[row] * e.lgamma[col] + e.lbeta[col];
  }
  if (CF32)
    reinterpret_cast<float*>(e.C)[(int64_t)row * e.ldc + col] = v;
  else
    reinterpret_cast<TIN*>(e.C)[(int64_t)row * e.ldc + col] = from_f32<TIN>(v);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int PP_HALF = 128 * 128;  // bytes per half-tile

// n (4 or 8) consecutive columns [c0, c0 + n) of one output row; bv/gm/bt = bias / LN gamma /
// LN beta for those columns (hoisted by the caller). Mirrors epi_row16 / epi_store.
// CHECK = false: interior tile (no bounds tests, EPI_COS row norm `rsc` from LDS), so the
// epilogue holds no global load and hipcc places no vmcnt wait between its stores.
// FS: the caller pre-scaled bv by this lane's column scale cs (its columns lie on one side of
// scale_cols, a multiple of 16): v = fma(v, cs, bv) instead of (v + bv) * col_scale under a per-lane
// branch — bit-identical for cs = 1 and for power-of-two scales (1/sqrt(64)).
// ZV (NV = 8): EPI_DGELU's pre-activations / EPI_BIAS_RESID's 16-bit residual come in zv, loaded by
// the caller ahead of use
template <typename E, int EPI, bool CF32, bool RF32, int NV, bool CHECK = true, bool TB = false, bool FS = false,
          bool ZV = false>
__device__ __forceinline__ void epi_seg(const EpiArgs& e, int row, int c0, float* v, const float* bv,
                                        const float* gm, const float* bt, float rsc = 0.f,
                                        const void* tbase = nullptr, int tm0 = 0, float cs = 1.f,
                                        typename H16<E>::x8 zv = {}) {
  if (CHECK && row >= e.M) return;
  if (CHECK && c0 + NV > e.N) {
#pragma unroll
    for (int k = 0; k < NV; ++k) epi_store<E, EPI, CF32, RF32>(e, row, c0 + k, v[k]);
    return;
  }
  if (EPI == RF_EPI_COS) {
    const float sc = (CHECK ? e.ra[row] : rsc) * e.col_scale;
    float* out = reinterpret_cast<float*>(e.C) + (int64_t)row * e.ldc + c0;
#pragma unroll
    for (int q = 0; q < NV / 4; ++q)
      *reinterpret_cast<f32x4*>(out + 4 * q) =
          f32x4{v[4 * q] * sc * bv[4 * q], v[4 * q + 1] * sc * bv[4 * q + 1], v[4 * q + 2] * sc * bv[4 * q + 2],
                v[4 * q + 3] * sc * bv[4 * q + 3]};
    return;
  }
  if (EPI == RF_EPI_DGELU) {
    const E* z = reinterpret_cast<const E*>(e.R) + (int64_t)row * e.ldr + c0;
    if (NV == 8) {
      const typename H16<E>::x8 x = ZV ? zv : *reinterpret_cast<const typename H16<E>::x8*>(z);
      float zf[8], d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) zf[k] = (float)x[k];
      dgelu8_erf(zf, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= d[k];
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] *= dgelu_erf(to_f32(z[k]));
    }
  } else if (EPI != RF_EPI_NONE) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = FS ? fmaf(v[k], cs, bv[k]) : v[k] + bv[k];
  }
  if (!FS && c0 < e.scale_cols) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] *= e.col_scale;
  }
  if (EPI == RF_EPI_BIAS_GELU_AUX) {  // the pre-activation, bf16 (NV = 8 on this path)
    E* z = reinterpret_cast<E*>(const_cast<void*>(e.R)) + (int64_t)row * e.ldr + c0;
    if (NV == 8) {
      typename H16<E>::x8 x;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (E)v[k];
      // non-temporal: read again only by the backward's GELU-derivative GEMM, a whole pass later
      __builtin_nontemporal_store(x, reinterpret_cast<typename H16<E>::x8*>(z));
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) z[k] = (E)v[k];
    }
  }
  if (EPI == RF_EPI_BIAS_GELU || EPI == RF_EPI_BIAS_GELU_AUX) {
    if (CF32) {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = gelu_erf(v[k]);
    } else if (NV == 8) {
      f32x2 y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = (f32x2){v[2 * k], v[2 * k + 1]};
      gelu8_bf16out(y);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = y[k].x;
        v[2 * k + 1] = y[k].y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; k += 2) {
        const f32x2 y = gelu2_bf16out((f32x2){v[k], v[k + 1]});
        v[k] = y.x;
        v[k + 1] = y.y;
      }
    }
  }
  if (EPI == RF_EPI_BIAS_RESID) {
    if (RF32) {
      const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
      for (int q = 0; q < NV / 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(r + 4 * q);
        v[4 * q] += x.x; v[4 * q + 1] += x.y; v[4 * q + 2] += x.z; v[4 * q + 3] += x.w;
      }
    } else if (ZV && (NV == 8 || NV == 6)) {  // the caller's prefetched residual row segment
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] += (float)zv[k];
    } else if (NV == 6) {  // 4-B aligned: three 2-element loads
      const E* r = reinterpret_cast<const E*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const typename H16<E>::x2 x = *reinterpret_cast<const typename H16<E>::x2*>(r + 2 * q);
        v[2 * q] += (float)x[0];
        v[2 * q + 1] += (float)x[1];
      }
    } else {
      const E* r = reinterpret_cast<const E*>(e.R) + (int64_t)row * e.ldr + c0;
#pragma unroll
      for (int q = 0; q < NV / 4; ++q) {
        const typename H16<E>::x4 x = *reinterpret_cast<const typename H16<E>::x4*>(r + 4 * q);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 * q + k] += (float)x[k];
      }
    }
  }
  if (EPI == RF_EPI_BIAS_RESID_LN) {
    const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)row * e.ldr + c0;
    const float mu = e.lmean[row], rs = e.lrstd[row];
#pragma unroll
    for (int q = 0; q < NV / 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(r + 4 * q);
      v[4 * q] += (x.x - mu) * rs * gm[4 * q] + bt[4 * q];
      v[4 * q + 1] += (x.y - mu) * rs * gm[4 * q + 1] + bt[4 * q + 1];
      v[4 * q + 2] += (x.z - mu) * rs * gm[4 * q + 2] + bt[4 * q + 2];
      v[4 * q + 3] += (x.w - mu) * rs * gm[4 * q + 3] + bt[4 * q + 3];
    }
  }
  if (CF32) {
    float* out = reinterpret_cast<float*>(e.C) + (int64_t)row * e.ldc + c0;
#pragma unroll
    for (int q = 0; q < NV / 4; ++q)
      *reinterpret_cast<f32x4*>(out + 4 * q) = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  } else {
    // TB (interior tiles): the tile's first output row as a wave-uniform base (tbase = row tm0): a
    // 32-bit per-lane offset from it (one v_add per store, global_store's SGPR-base form) instead of
    // 64-bit address arithmetic per store
    E* out;
    if constexpr (TB)
      out = reinterpret_cast<E*>(const_cast<char*>(reinterpret_cast<const char*>(tbase)) +
                                 (uint32_t)(((row - tm0) * e.ldc + c0) * (int)sizeof(E)));
    else out = reinterpret_cast<E*>(e.C) + (int64_t)row * e.ldc + c0;
    if (NV == 8) {
      typename H16<E>::x8 x;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (E)v[k];
#if !defined(RF_GEMM_PLAIN_STORE)
      // non-temporal: the tile's output is not re-read by this kernel; measured +0.8% per C2
      // step (tools/gpu/gemm_var.sh: qkv -4%, FFN -1.5%). Plain stores for only the outputs the
      // next kernel reads at once (out-proj / FFN2 -> LayerNorm, qkv -> band attention), for
      // Infinity-Cache hits, measured slower too (same-process step A/B, round 3: LayerNorm
      // unchanged, the GEMMs 1-3% slower)
      __builtin_nontemporal_store(x, reinterpret_cast<typename H16<E>::x8*>(out));
#else
      *reinterpret_cast<typename H16<E>::x8*>(out) = x;
#endif
    } else if (NV == 6) {  // the 192-column tile's 6 columns: one 12-B store (4-B aligned)
      // the fp32 value is rounded to 16 bits as a separate step, as in the 8-column forms: hipcc otherwise
      // folds the bias FMA and the fp16 conversion into one v_fma_mix (one rounding instead of two: 1 ulp
      // apart from the 256-column tile in ~2e-5 of the fp16 outputs)
#pragma unroll
      for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(v[k]));
      typename H16<E>::x8 x;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (E)(k < 6 ? v[k < 6 ? k : 0] : 0.f);
      typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
      typedef uint32_t u32x3_t __attribute__((ext_vector_type(3)));
      const u32x4_t w = __builtin_bit_cast(u32x4_t, x);
      __builtin_nontemporal_store(u32x3_t{w[0], w[1], w[2]}, reinterpret_cast<u32x3_t*>(out));
    } else {
      typename H16<E>::x4 x;
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = (E)v[k];
      *reinterpret_cast<typename H16<E>::x4*>(out) = x;
    }
  }
}

// per-column epilogue vectors (bias or, for EPI_COS, the item inverse norms; LN gamma / beta)
template <int EPI, int NV>
__device__ __forceinline__ void load_cols(const EpiArgs& e, int c0, float* bv, float* gm, float* bt) {
  const bool in = c0 + NV <= e.N;
#pragma unroll
  for (int q = 0; q < NV / 4; ++q) {
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f), g = b, t = b;
    if (in) {
      if (EPI == RF_EPI_COS) b = *reinterpret_cast<const float4*>(e.rw + c0 + 4 * q);
      else if (EPI != RF_EPI_NONE && EPI != RF_EPI_DGELU) b = *reinterpret_cast<const float4*>(e.bias + c0 + 4 * q);
      if (EPI == RF_EPI_BIAS_RESID_LN) {
        g = *reinterpret_cast<const float4*>(e.lgamma + c0 + 4 * q);
        t = *reinterpret_cast<const float4*>(e.lbeta + c0 + 4 * q);
      }
    }
    bv[4 * q] = b.x; bv[4 * q + 1] = b.y; bv[4 * q + 2] = b.z; bv[4 * q + 3] = b.w;
    gm[4 * q] = g.x; gm[4 * q + 1] = g.y; gm[4 * q + 2] = g.z; gm[4 * q + 3] = g.w;
    bt[4 * q] = t.x; bt[4 * q + 1] = t.y; bt[4 * q + 2] = t.z; bt[4 * q + 3] = t.w;
  }
}


template <int EPI, int NV>
__device__ __forceinline__ void lds_cols(const float* cb, int co, float* bv, float* gm, float* bt) {
#pragma unroll
  for (int q = 0; q < NV / 4; ++q) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(cb + co + 4 * q);
    f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f}, t = g;
    if (EPI == RF_EPI_BIAS_RESID_LN) {
      g = *reinterpret_cast<const f32x4*>(cb + 256 + co + 4 * q);
      t = *reinterpret_cast<const f32x4*>(cb + 512 + co + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bv[4 * q + k] = b[k];
      gm[4 * q + k] = g[k];
      bt[4 * q + k] = t[k];
    }
  }
}


inline int num_cus() {
  static int n[16] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) dev = 0;
  if (!n[dev]) {
    int c = 0;
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    n[dev] = c > 0 ? c : 256;
  }
  return n[dev];
}

}  // namespace rf
