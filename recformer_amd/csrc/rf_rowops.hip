// Row-wise HBM-bound kernels: input prologue, fused embedding+LayerNorm, LayerNorm,
// inverse row norms, global-row gather, candidate cosine scores.
// One wave64 per row; each lane owns D/64 elements loaded as 8-16 B vectors
// (cdna_hip_programming.md Guideline 13). All statistics in fp32.
#include <stdarg.h>
#include <stdio.h>

#include <string.h>

#include "rf_common.h"

namespace rf {

static thread_local char g_err[512];
int g_knob[KNOB_COUNT] = {6, 8, 0, 3, 0, 8, -1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0};
const uint64_t* g_seed_dev = nullptr;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

// ------------------------------------------------------------------------------------
// vector load/store of VEC elements at p (VEC*sizeof(T) bytes, naturally aligned)
template <typename T, int VEC> struct Vec;
template <> struct Vec<float, 4> {
  static __device__ __forceinline__ void load(const float* p, float* o) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* o) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
};
template <> struct Vec<float, 2> {
  static __device__ __forceinline__ void load(const float* p, float* o) {
    float2 v = *reinterpret_cast<const float2*>(p);
    o[0] = v.x; o[1] = v.y;
  }
  static __device__ __forceinline__ void store(float* p, const float* o) {
    *reinterpret_cast<float2*>(p) = make_float2(o[0], o[1]);
  }
};
template <> struct Vec<float, 1> {
  static __device__ __forceinline__ void load(const float* p, float* o) { o[0] = *p; }
  static __device__ __forceinline__ void store(float* p, const float* o) { *p = o[0]; }
};
template <> struct Vec<bf16, 4> {
  static __device__ __forceinline__ void load(const bf16* p, float* o) {
    bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* o) {
    bf16x4 v;
    v[0] = (bf16)o[0]; v[1] = (bf16)o[1]; v[2] = (bf16)o[2]; v[3] = (bf16)o[3];
    *reinterpret_cast<bf16x4*>(p) = v;
  }
};
template <> struct Vec<bf16, 2> {
  static __device__ __forceinline__ void load(const bf16* p, float* o) {
    bf16x2 v = *reinterpret_cast<const bf16x2*>(p);
    o[0] = (float)v[0]; o[1] = (float)v[1];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* o) {
    bf16x2 v;
    v[0] = (bf16)o[0]; v[1] = (bf16)o[1];
    *reinterpret_cast<bf16x2*>(p) = v;
  }
};
template <> struct Vec<bf16, 1> {
  static __device__ __forceinline__ void load(const bf16* p, float* o) { o[0] = (float)*p; }
  static __device__ __forceinline__ void store(bf16* p, const float* o) { *p = (bf16)o[0]; }
};
template <> struct Vec<f16, 4> {
  static __device__ __forceinline__ void load(const f16* p, float* o) {
    f16x4 v = *reinterpret_cast<const f16x4*>(p);
    o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
  }
  static __device__ __forceinline__ void store(f16* p, const float* o) {
    f16x4 v;
    v[0] = (f16)o[0]; v[1] = (f16)o[1]; v[2] = (f16)o[2]; v[3] = (f16)o[3];
    *reinterpret_cast<f16x4*>(p) = v;
  }
};
template <> struct Vec<f16, 2> {
  static __device__ __forceinline__ void load(const f16* p, float* o) {
    f16x2 v = *reinterpret_cast<const f16x2*>(p);
    o[0] = (float)v[0]; o[1] = (float)v[1];
  }
  static __device__ __forceinline__ void store(f16* p, const float* o) {
    f16x2 v;
    v[0] = (f16)o[0]; v[1] = (f16)o[1];
    *reinterpret_cast<f16x2*>(p) = v;
  }
};
template <> struct Vec<f16, 1> {
  static __device__ __forceinline__ void load(const f16* p, float* o) { o[0] = (float)*p; }
  static __device__ __forceinline__ void store(f16* p, const float* o) { *p = (f16)o[0]; }
};

// VEC consecutive elements of the split fp32 stream (rf_common.h split_f32 / join_f32)
template <int VEC>
__device__ __forceinline__ void load_split(const uint16_t* hi, const uint16_t* lo, float* o) {
  typedef __attribute__((ext_vector_type(VEC))) uint16_t u16v;
  const u16v h = *reinterpret_cast<const u16v*>(hi);
#if !defined(RF_LN_PLAIN_LOAD)
  const u16v l = __builtin_nontemporal_load(reinterpret_cast<const u16v*>(lo));
#else
  const u16v l = *reinterpret_cast<const u16v*>(lo);
#endif
#pragma unroll
  for (int j = 0; j < VEC; ++j) o[j] = join_f32(h[j], l[j]);
}
template <int VEC>
__device__ __forceinline__ void store_split(uint16_t* hi, uint16_t* lo, const float* o) {
  typedef __attribute__((ext_vector_type(VEC))) uint16_t u16v;
  u16v h, l;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    uint16_t a, b;
    split_f32(o[j], a, b);
    h[j] = a;
    l[j] = b;
  }
#if defined(RF_LN_NT_HI)
  __builtin_nontemporal_store(h, reinterpret_cast<u16v*>(hi));
#else
  *reinterpret_cast<u16v*>(hi) = h;
#endif
#if !defined(RF_LN_PLAIN_LO)
  // non-temporal: the lo plane is next read by the following LayerNorm, after a GEMM and the
  // attention have streamed through the caches (+0.5% per C2 step; the hi plane, the next GEMM's
  // operand, stays a normal store)
  __builtin_nontemporal_store(l, reinterpret_cast<u16v*>(lo));
#else
  *reinterpret_cast<u16v*>(lo) = l;
#endif
}

// ------------------------------------------------------------------------------------
// 256-thread block exclusive scan of one int per thread.
__device__ __forceinline__ int block_excl_scan256(int v, int* lds /*[8]*/, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    int s = lds[w];
    if (w < wid) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// A2 prologue. One 256-thread block per sequence.
__global__ void __launch_bounds__(256) k_prepare(
    const int64_t* __restrict__ ids_in, const int64_t* __restrict__ am_in,
    const int64_t* __restrict__ gm_in, const int64_t* __restrict__ tt_in,
    const int64_t* __restrict__ ip_in, const int64_t* __restrict__ pos_in, int L, int Lp,
    int pad_id, int gmax, int32_t* __restrict__ ids, int32_t* __restrict__ pos,
    int32_t* __restrict__ tt, int32_t* __restrict__ ip, uint8_t* __restrict__ flags,
    int32_t* __restrict__ gidx, int32_t* __restrict__ gstat) {
  __shared__ int scan_lds[8];
  const int b = blockIdx.x;
  const int per = (Lp + 255) / 256;
  const int p0 = threadIdx.x * per;
  const int p1 = min(p0 + per, Lp);
  const int64_t* idr = ids_in + (int64_t)b * L;
  int cnt_tok = 0, cnt_glob = 0;
  for (int p = p0; p < p1; ++p) {
    int64_t id = p < L ? idr[p] : pad_id;
    cnt_tok += (id != pad_id);
    if (p < L) {
      int64_t am = am_in ? am_in[(int64_t)b * L + p] : 1;
      int64_t m = gm_in ? am * (gm_in[(int64_t)b * L + p] + 1) : am;
      cnt_glob += (m > 1);
    }
  }
  int tot_tok, tot_glob;
  int run_tok = block_excl_scan256(cnt_tok, scan_lds, &tot_tok);
  int run_glob = block_excl_scan256(cnt_glob, scan_lds, &tot_glob);
  for (int p = p0; p < p1; ++p) {
    const int64_t o = (int64_t)b * Lp + p;
    const int64_t i = (int64_t)b * L + p;
    int64_t id = p < L ? idr[p] : pad_id;
    int nonpad = id != pad_id;
    run_tok += nonpad;
    int32_t posv;
    if (pos_in)
      posv = p < L ? (int32_t)pos_in[i] : pad_id;
    else
      posv = nonpad ? run_tok + pad_id : pad_id;
    uint8_t f = 0;
    int32_t ttv = 0, ipv = pad_id;
    if (p < L) {
      int64_t am = am_in ? am_in[i] : 1;
      int64_t m = gm_in ? am * (gm_in[i] + 1) : am;
      f = m <= 0 ? 0 : (m == 1 ? 1 : 2);
      ttv = tt_in ? (int32_t)tt_in[i] : 0;
      ipv = (int32_t)ip_in[i];
      if (f == 2) {
        if (run_glob < gmax) gidx[(int64_t)b * gmax + run_glob] = p;
        ++run_glob;
      }
    }
    ids[o] = (int32_t)id;
    pos[o] = posv;
    tt[o] = ttv;
    ip[o] = ipv;
    flags[o] = f;
  }
  for (int g = tot_glob + threadIdx.x; g < gmax; g += 256) gidx[(int64_t)b * gmax + g] = -1;
  if (gstat && threadIdx.x == 0) {
    // per sequence: its number of global tokens and whether position 0 (the CLS) is one — the same
    // flag rule as above, so the host's global-slot count matches the flags exactly
    const int64_t am0 = am_in ? am_in[(int64_t)b * L] : 1;
    const int64_t m0 = gm_in ? am0 * (gm_in[(int64_t)b * L] + 1) : am0;
    gstat[2 * b] = tot_glob;
    gstat[2 * b + 1] = m0 > 1 ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------
// Fused embedding gather + LayerNorm (A3). One wave per token. Tables in TT (fp32 keeps the
// reference's fp32 embedding sum under autocast), output in T plus an optional fp32 copy
// (the fp32 residual stream of the bf16 path).
template <typename TT, typename T, int VEC, int NCH>
__global__ void __launch_bounds__(256) k_embed_ln(
    int M, const int32_t* __restrict__ ids, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ tt, const int32_t* __restrict__ ip, const TT* __restrict__ we,
    const TT* __restrict__ pe, const TT* __restrict__ te, const TT* __restrict__ ie,
    const float* __restrict__ lw, const float* __restrict__ lb, float eps, T* __restrict__ out,
    float* __restrict__ out32, uint16_t* __restrict__ out_lo) {
  constexpr int D = 64 * VEC * NCH;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int64_t r0 = (int64_t)ids[row] * D, r1 = (int64_t)pos[row] * D;
  const int64_t r2 = (int64_t)tt[row] * D, r3 = (int64_t)ip[row] * D;
  float x[NCH][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * 64 * VEC + lane * VEC;
    float a[VEC], b2[VEC], c2[VEC], d2[VEC];
    Vec<TT, VEC>::load(we + r0 + e, a);
    Vec<TT, VEC>::load(pe + r1 + e, b2);
    Vec<TT, VEC>::load(te + r2 + e, c2);
    Vec<TT, VEC>::load(ie + r3 + e, d2);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      // summation order of models.py:135: ((word + pos) + type) + item_pos
      x[c][j] = ((a[j] + b2[j]) + c2[j]) + d2[j];
      s += x[c][j];
    }
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float d = x[c][j] - mean;
      v += d * d;
    }
  const float rstd = rsqrtf(wave_sum(v) * (1.0f / D) + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * 64 * VEC + lane * VEC;
    float w[VEC], bb[VEC], y[VEC];
    Vec<float, VEC>::load(lw + e, w);
    Vec<float, VEC>::load(lb + e, bb);
#pragma unroll
    for (int j = 0; j < VEC; ++j) y[j] = (x[c][j] - mean) * rstd * w[j] + bb[j];
    if (out_lo) {  // split fp32 stream: out holds the hi plane (T is bf16 here)
      store_split<VEC>(reinterpret_cast<uint16_t*>(out) + (int64_t)row * D + e, out_lo + (int64_t)row * D + e, y);
    } else {
      Vec<T, VEC>::store(out + (int64_t)row * D + e, y);
    }
    if (out32) Vec<float, VEC>::store(out32 + (int64_t)row * D + e, y);
  }
}

// LayerNorm of one row per wave; with `res` (fp32, row stride D) the row is x + res first:
// the reference's LayerNorm(dense(h) + input_tensor) (TF:1064-1071, 1123-1130) where, under
// autocast, dense() returns bf16 and the residual input is fp32. y32 may alias res (the fp32
// residual stream updated in place: every lane reads its whole row before the first store).
template <typename TX, typename T, int VEC, int NCH>
__global__ void __launch_bounds__(256) k_layernorm(int M, const TX* __restrict__ x, int ldx,
                                                    const float* res,
                                                    const float* __restrict__ lw,
                                                    const float* __restrict__ lb, float eps,
                                                    T* __restrict__ y, int ldy,
                                                    float* y32,
                                                    float* __restrict__ mean_out,
                                                    float* __restrict__ rstd_out) {
  constexpr int D = 64 * VEC * NCH;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float xv[NCH][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    Vec<TX, VEC>::load(x + (int64_t)row * ldx + c * 64 * VEC + lane * VEC, xv[c]);
    if (res) {
      float rv[VEC];
      Vec<float, VEC>::load(res + (int64_t)row * D + c * 64 * VEC + lane * VEC, rv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) xv[c][j] += rv[j];
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += xv[c][j];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float d = xv[c][j] - mean;
      v += d * d;
    }
  const float rstd = rsqrtf(wave_sum(v) * (1.0f / D) + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * 64 * VEC + lane * VEC;
    float w[VEC], bb[VEC], o[VEC];
    Vec<float, VEC>::load(lw + e, w);
    Vec<float, VEC>::load(lb + e, bb);
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (xv[c][j] - mean) * rstd * w[j] + bb[j];
    Vec<T, VEC>::store(y + (int64_t)row * ldy + e, o);
    if (y32) Vec<float, VEC>::store(y32 + (int64_t)row * D + e, o);
  }
}

// The residual-add LayerNorm on the split fp32 stream (split_f32 / join_f32): y = LN(x + r)
// with x the bf16 dense output and r = join(r_hi, r_lo) exactly the fp32 stream of the
// reference's autocast run (TF:1064-1071, 1123-1130). Outputs: the new stream as planes
// (y_hi is also the next GEMM's bf16 operand) and/or an fp32 copy y32. Planes may alias the
// inputs (in-place update: every lane reads its whole row before its first store).
// Traffic per row: 2 B (x) + 4 B (r) in, 4 B out per element, vs 2 + 4 in, 4 + 2 out with a
// separate fp32 stream and bf16 operand.
// LPR lanes per row (a group of 8..64 lanes), 8 elements (16-B loads of each plane) per lane
// and chunk: D = LPR * 8 * NCH; 256 / LPR rows per block (D = 768: half a wave per row).
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int LPR, int NCH>
__global__ void __launch_bounds__(256) k_add_ln_split(int M, const bf16* __restrict__ x, int ldx,
                                                       const uint16_t* r_hi, const uint16_t* r_lo,
                                                       const float* __restrict__ lw,
                                                       const float* __restrict__ lb, float eps,
                                                       uint16_t* y_hi, uint16_t* y_lo, float* y32) {
  constexpr int VEC = 8, D = LPR * VEC * NCH;
  const int gl = threadIdx.x % LPR;
  const int row = blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
  if (row >= M) return;  // whole lane groups exit together: the shuffles below stay in-group
  float xv[NCH][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * LPR * VEC + gl * VEC;
#if !defined(RF_LN_PLAIN_LOAD)  // the dense output and the lo plane are read once: non-temporal
    const bf16x8 xb = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(x + (int64_t)row * ldx + e));
#else
    const bf16x8 xb = *reinterpret_cast<const bf16x8*>(x + (int64_t)row * ldx + e);
#endif
#pragma unroll
    for (int j = 0; j < VEC; ++j) xv[c][j] = (float)xb[j];
    if (r_hi) {
      float rv[VEC];
      load_split<VEC>(r_hi + (int64_t)row * D + e, r_lo + (int64_t)row * D + e, rv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) xv[c][j] += rv[j];
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += xv[c][j];
  }
  const float mean = group_sum<LPR>(s) * (1.0f / D);
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float d = xv[c][j] - mean;
      v += d * d;
    }
  const float rstd = rsqrtf(group_sum<LPR>(v) * (1.0f / D) + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * LPR * VEC + gl * VEC;
    float w[VEC], bb[VEC], o[VEC];
    Vec<float, 4>::load(lw + e, w);
    Vec<float, 4>::load(lw + e + 4, w + 4);
    Vec<float, 4>::load(lb + e, bb);
    Vec<float, 4>::load(lb + e + 4, bb + 4);
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (xv[c][j] - mean) * rstd * w[j] + bb[j];
    if (y_hi) store_split<VEC>(y_hi + (int64_t)row * D + e, y_lo + (int64_t)row * D + e, o);
    if (y32) {
      Vec<float, 4>::store(y32 + (int64_t)row * D + e, o);
      Vec<float, 4>::store(y32 + (int64_t)row * D + e + 4, o + 4);
    }
  }
}

// ---- training path: hidden dropout + residual add + LayerNorm (TF:1068-1071, 1127-1130) ----
// Forward: x = dropout(t) + res, y = LN(x) in one pass (t the bf16 dense output, res the fp32
// stream); x (the backward's input) and the row stats are written. The keep mask is a counter
// hash of (seed, element index) — regenerated by the backward, never stored.

template <typename E, int VEC, int NCH>
__global__ void __launch_bounds__(256) k_drop_add_ln_fwd(int M, const E* __restrict__ t, int ldt,
                                                          const float* __restrict__ res, uint32_t thresh,
                                                          float keep_scale, uint64_t seed, const uint64_t* seed_dev,
                                                          const float* __restrict__ lw, const float* __restrict__ lb,
                                                          float eps, float* __restrict__ xo, float* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          E* __restrict__ y16, int mrow) {
  constexpr int D = 64 * VEC * NCH;
  if (thresh) seed = seed_resolve(seed, seed_dev);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float xv[NCH][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * 64 * VEC + lane * VEC;
    float tv[VEC], rv[VEC];
    Vec<E, VEC>::load(t + (int64_t)row * ldt + e, tv);
    Vec<float, VEC>::load(res + (int64_t)row * D + e, rv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const bool keep = thresh == 0 || drop_keep(seed, (uint64_t)row * mrow * D + e + j, thresh);
      xv[c][j] = (keep ? tv[j] * keep_scale : 0.f) + rv[j];
      s += xv[c][j];
    }
    Vec<float, VEC>::store(xo + (int64_t)row * D + e, xv[c]);
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float d = xv[c][j] - mean;
      v += d * d;
    }
  const float rstd = rsqrtf(wave_sum(v) * (1.0f / D) + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = c * 64 * VEC + lane * VEC;
    float w[VEC], bb[VEC], o[VEC];
    Vec<float, VEC>::load(lw + e, w);
    Vec<float, VEC>::load(lb + e, bb);
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (xv[c][j] - mean) * rstd * w[j] + bb[j];
    Vec<float, VEC>::store(y + (int64_t)row * D + e, o);
    if (y16) Vec<E, VEC>::store(y16 + (int64_t)row * D + e, o);  // the next GEMM's operand
  }
}

// LayerNorm backward (training path; TF:1071, 1130 under autograd): per row, with
// xhat = (x - mean) * rstd and g = dy * w,
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat))
// and per-column partial sums of dy * xhat (dw) and dy (db) over this block's rows, written to
// part[blockIdx][2][D] and reduced by k_colsum2 (deterministic; no float atomics).
// One wave per row, LNB_ROWS rows per 256-thread block.
constexpr int LNB_ROWS = 32;

// With dt != null (the dropout + residual form above) it also writes the dense branch's
// gradient dt = dx * keep * keep_scale in bf16 (the mask regenerated from the seed).
template <typename E, int VEC, int NCH>
__global__ void __launch_bounds__(256) k_layernorm_bwd(int M, const float* __restrict__ dy,
                                                        const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ w, float* __restrict__ dx,
                                                        float* __restrict__ part, E* __restrict__ dt,
                                                        uint32_t thresh, float keep_scale, uint64_t seed,
                                                        const uint64_t* seed_dev, const E* __restrict__ dy2,
                                                        int tb, int mrow) {
  constexpr int D = 64 * VEC * NCH;
  if (thresh) seed = seed_resolve(seed, seed_dev);
  __shared__ float red[4][3][D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ns = tb ? 3 : 2;  // partial slots per block: dw, db (+ the column sums of dt)
  float pw[NCH][VEC], pb[NCH][VEC], pt[NCH][VEC], wr[NCH][VEC];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    Vec<float, VEC>::load(w + c * 64 * VEC + lane * VEC, wr[c]);
#pragma unroll
    for (int j = 0; j < VEC; ++j) pw[c][j] = pb[c][j] = pt[c][j] = 0.f;
  }
  const int r0 = blockIdx.x * LNB_ROWS;
  for (int rr = wv; rr < LNB_ROWS; rr += 4) {
    const int row = r0 + rr;
    if (row >= M) break;
    const float mu = mean[row], rs = rstd[row];
    float g[NCH][VEC], xh[NCH][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int e = c * 64 * VEC + lane * VEC;
      float d[VEC], xv[VEC];
      if (dy) {
        Vec<float, VEC>::load(dy + (int64_t)row * D + e, d);
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) d[j] = 0.f;
      }
      if (dy2) {  // second consumer's gradient (bf16), summed as autograd would
        float d2[VEC];
        Vec<E, VEC>::load(dy2 + (int64_t)row * D + e, d2);
#pragma unroll
        for (int j = 0; j < VEC; ++j) d[j] += d2[j];
      }
      Vec<float, VEC>::load(x + (int64_t)row * ldx + e, xv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        xh[c][j] = (xv[j] - mu) * rs;
        g[c][j] = d[j] * wr[c][j];
        s1 += g[c][j];
        s2 += g[c][j] * xh[c][j];
        pw[c][j] += d[j] * xh[c][j];
        pb[c][j] += d[j];
      }
    }
    const float c1 = wave_sum(s1) * (1.0f / D), c2 = wave_sum(s2) * (1.0f / D);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = rs * (g[c][j] - c1 - xh[c][j] * c2);
      const int e = c * 64 * VEC + lane * VEC;
      Vec<float, VEC>::store(dx + (int64_t)row * D + e, o);
      if (dt) {
        float od[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          od[j] = (thresh == 0 || drop_keep(seed, (uint64_t)row * mrow * D + e + j, thresh)) ? o[j] * keep_scale
                                                                                             : 0.f;
        Vec<E, VEC>::store(dt + (int64_t)row * D + e, od);
        if (tb) {  // the dense branch's bias gradient: column sums of dt as stored (16-bit)
#pragma unroll
          for (int j = 0; j < VEC; ++j) pt[c][j] += (float)(E)od[j];
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      red[wv][0][c * 64 * VEC + lane * VEC + j] = pw[c][j];
      red[wv][1][c * 64 * VEC + lane * VEC + j] = pb[c][j];
      red[wv][2][c * 64 * VEC + lane * VEC + j] = pt[c][j];
    }
  __syncthreads();
  for (int i = threadIdx.x; i < ns * D; i += 256) {
    const int k = i / D, col = i - k * D;
    part[((int64_t)blockIdx.x * ns + k) * D + col] = red[0][k][col] + red[1][k][col] + red[2][k][col] + red[3][k][col];
  }
}

// Deterministic column sums of an (M, N) row-major matrix (T = fp32 or bf16) in two stages:
// k_colsum_part: block (column group of 64, row slice z) -> part[z][N] (4 row phases per block
// combined in LDS); k_colsum_fin: out[n] = sum_z part[z][n]. Used for LayerNorm dgamma / dbeta
// (over k_layernorm_bwd's per-block partials) and for bias gradients (column sums of dC).
// dst[rows[r]] += src[r] for r < R (rows[r] < 0: skipped), two (src, dst) pairs per launch; one
// thread per column walks the rows in order, so repeated destination rows add up in a fixed
// order (no atomics). The training path's global-key gradient columns (a few rows per sequence).
template <typename T>
__global__ void __launch_bounds__(256) k_scatter_add_rows(int R, int D, const int32_t* __restrict__ rows,
                                                           const T* __restrict__ s0, const T* __restrict__ s1,
                                                           int lds, T* __restrict__ d0, T* __restrict__ d1,
                                                           int ldd) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= D) return;
  const T* src = blockIdx.y ? s1 : s0;
  T* dst = blockIdx.y ? d1 : d0;
  for (int r = 0; r < R; ++r) {
    const int row = rows[r];
    if (row < 0) continue;
    T* p = dst + (int64_t)row * ldd + col;
    *p = from_f32<T>(to_f32(*p) + to_f32(src[(int64_t)r * lds + col]));
  }
}

// row slices of the column-sum stage (at most; 64 rows each at least). 256 slices (every row load of a wave
// in flight at once) measured no faster in the captured C3 step (16.53 vs 16.49 ms, knob colsum_slices,
// gpurun_out/r05i): the training bias-gradient sums run beside the weight-gradient stream
constexpr int CS_SLICES = 64;

template <typename T, bool VECOK>
__global__ void __launch_bounds__(256) k_colsum_part(int M, int N, const T* __restrict__ x, int64_t ldx,
                                                      float* __restrict__ part) {
  // 64 lanes x 4 consecutive columns = 256 columns per block; 4 row phases (waves) combined in LDS
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + 4 * lane;
  const int per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(M, r0 + per);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (VECOK && c + 4 <= N) {  // 4-element vector loads (aligned rows), 8 rows in flight
#pragma unroll 8
    for (int r = r0 + ph; r < r1; r += 4) {
      float v[4];
      Vec<T, 4>::load(x + (int64_t)r * ldx + c, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += v[k];
    }
  } else {
    for (int r = r0 + ph; r < r1; r += 4)
      for (int k = 0; k < 4 && c + k < N; ++k) a[k] += to_f32(x[(int64_t)r * ldx + c + k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[ph][4 * lane + k] = a[k];
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < N)
    part[(int64_t)blockIdx.y * N + cc] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// 16-bit x with 16-B rows (N % 8 == 0, ldx % 8 == 0, 16-B aligned): one 16-B load per lane and row (8
// columns), 512 columns per block, the same slice / phase split and the same per-column order of the
// additions as k_colsum_part (rows r0 + ph, r0 + ph + 4, ... per phase, then the 4 phases in order), so the
// partials are bit-identical to it; the 8-B loads of k_colsum_part moved the training bias-gradient sums
// at ~3.6 TB/s
template <typename E>
__global__ void __launch_bounds__(256) k_colsum_part16(int M, int N, const E* __restrict__ x, int64_t ldx,
                                                        float* __restrict__ part) {
  typedef typename H16<E>::x8 V8;
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + 8 * lane;
  const int per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(M, r0 + per);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < N) {
#pragma unroll 8
    for (int r = r0 + ph; r < r1; r += 4) {
      const V8 v = *reinterpret_cast<const V8*>(x + (int64_t)r * ldx + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += (float)v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[ph][8 * lane + k] = a[k];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int cc = blockIdx.x * 512 + i;
    if (cc < N) part[(int64_t)blockIdx.y * N + cc] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

// out[n] = sum_z part[z][n]: 64 slice phases x 4 columns per block (phase z adds slices z, z + 64, ... in
// order), tree-reduced in LDS (fixed order)
// scale_n > 0: out[c] for c < scale_n multiplied by scale (a Linear's column scale, e.g. the query's 1/8)
__global__ void __launch_bounds__(256) k_colsum_fin(int S, int N, const float* __restrict__ part, float* __restrict__ out,
                                                     float* __restrict__ out2, int split, float* __restrict__ out3,
                                                     int scale_n = 0, float scale = 1.f) {
  __shared__ float red[64][5];
  const int z = threadIdx.x >> 2, k = threadIdx.x & 3;
  const int c = blockIdx.x * 4 + k;
  float a = 0.f;
  if (c < N)
    for (int zz = z; zz < S; zz += 64) a += part[(int64_t)zz * N + c];
  red[z][k] = a;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (z < o) red[z][k] += red[z + o][k];
    __syncthreads();
  }
  if (z == 0 && c < N) {
    if (out3 && c >= 2 * split) out3[c - 2 * split] = red[0][k];
    else if (out2 && c >= split) out2[c - split] = red[0][k];
    else out[c] = c < scale_n ? red[0][k] * scale : red[0][k];
  }
}

template <typename T>
static void colsum(int M, int N, const T* x, int64_t ldx, float* part, float* out, float* out2, int split,
                   hipStream_t s, float* out3 = nullptr, int scale_n = 0, float scale = 1.f) {
  const int cap = g_knob[KNOB_COLSUM_SLICES] > 0 ? min(g_knob[KNOB_COLSUM_SLICES], CS_SLICES) : CS_SLICES;
  const int S = max(1, min(cap, (M + 63) / 64));
  const bool vec = ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % (4 * sizeof(T))) == 0;
  if constexpr (sizeof(T) == 2) {
    if (N % 8 == 0 && ldx % 8 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0) {
      k_colsum_part16<T><<<dim3((N + 511) / 512, S), 256, 0, s>>>(M, N, x, ldx, part);
      k_colsum_fin<<<(N + 3) / 4, 256, 0, s>>>(S, N, part, out, out2, split, out3, scale_n, scale);
      return;
    }
  }
  if (vec) k_colsum_part<T, true><<<dim3((N + 255) / 256, S), 256, 0, s>>>(M, N, x, ldx, part);
  else k_colsum_part<T, false><<<dim3((N + 255) / 256, S), 256, 0, s>>>(M, N, x, ldx, part);
  k_colsum_fin<<<(N + 3) / 4, 256, 0, s>>>(S, N, part, out, out2, split, out3, scale_n, scale);
}

template <typename T, int VEC, int NCH>
__global__ void __launch_bounds__(256) k_row_inv_norm(int M, const T* __restrict__ x, int ldx,
                                                       float eps, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    float xv[VEC];
    Vec<T, VEC>::load(x + (int64_t)row * ldx + c * 64 * VEC + lane * VEC, xv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += xv[j] * xv[j];
  }
  s = wave_sum(s);
  if (lane == 0) out[row] = 1.0f / fmaxf(sqrtf(s), eps);
}

template <typename T>
__global__ void __launch_bounds__(256) k_gather_rows(int Lp, int D, int gmax, const T* __restrict__ x,
                                                      int ldx, const int32_t* __restrict__ gidx,
                                                      T* __restrict__ out) {
  const int r = blockIdx.x;  // r = b*gmax + g
  const int b = r / gmax;
  const int p = gidx[r];
  for (int e = threadIdx.x; e < D; e += 256)
    out[(int64_t)r * D + e] = p >= 0 ? x[((int64_t)b * Lp + p) * ldx + e] : from_f32<T>(0.f);
}

template <typename T>
__global__ void __launch_bounds__(256) k_cos_cand(int B, int C, int D, const T* __restrict__ z,
                                                   int ldz, const float* __restrict__ rz,
                                                   const T* __restrict__ items, int ldi,
                                                   const float* __restrict__ ri,
                                                   const int64_t* __restrict__ cand,
                                                   float inv_temp, float* __restrict__ scores) {
  const int lane = threadIdx.x & 63;
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (idx >= B * C) return;
  const int b = idx / C;
  const int64_t n = cand[idx];
  float s = 0.f;
  for (int e = lane; e < D; e += 64) s += to_f32(z[(int64_t)b * ldz + e]) * to_f32(items[n * ldi + e]);
  s = wave_sum(s);
  if (lane == 0) scores[idx] = s * rz[b] * ri[n] * inv_temp;
}

// Backward of the cosine scoring head (Similarity, models.py:358-369, trained through the
// CrossEntropyLoss of models.py:583-599): logits s[b, c] = inv_temp (z_b . t_n) rz_b ri_n with
// n = c (full catalog) or n = cand[b, c] (sampled softmax, models.py:592-597). With g = dL/ds:
//   dz_b = rz_b (inv_temp sum_c g_bc ri_n t_n - (sum_c g_bc s_bc) rz_b z_b)
// Pass 1 (k_cos_bwd_part): a workgroup takes COS_NCH columns of ROWS rows (16 for the full catalog —
// the rows share every item row, so the table is read once — 1 for sampled rows, whose items differ),
// thread t owns columns d = t + 256 k of the partial sum over its columns; the (g s) row sums too.
// Pass 2 (k_cos_bwd_fin): the partials of a row summed in chunk order (deterministic), then dz.
constexpr int COS_NCH = 64;

template <typename T, int ROWS, int KD>
__global__ void __launch_bounds__(256) k_cos_bwd_part(int B, int C, int D, const T* __restrict__ items, int ldi,
                                                      const float* __restrict__ ri, const int64_t* __restrict__ cand,
                                                      const float* __restrict__ g, int64_t ldg,
                                                      const float* __restrict__ s, int64_t lds,
                                                      float* __restrict__ part, float* __restrict__ partc) {
  __shared__ float sg[ROWS][COS_NCH];
  __shared__ float sgs[ROWS][COS_NCH];
  __shared__ int64_t sidx[COS_NCH];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * COS_NCH, b0 = blockIdx.y * ROWS;
  const int ncol = min(COS_NCH, C - c0);
  for (int e = tid; e < ROWS * COS_NCH; e += 256) {
    const int r = e / COS_NCH, c = e - r * COS_NCH;
    const int b = b0 + r, col = c0 + c;
    const bool ok = b < B && c < ncol;
    const float gv = ok ? g[(int64_t)b * ldg + col] : 0.f;
    sg[r][c] = gv;
    sgs[r][c] = ok ? gv * s[(int64_t)b * lds + col] : 0.f;
    if (ROWS == 1 && r == 0) sidx[c] = ok ? cand[(int64_t)b * C + col] : 0;
  }
  __syncthreads();
  if (tid < ROWS && b0 + tid < B) {
    float a = 0.f;
    for (int c = 0; c < COS_NCH; ++c) a += sgs[tid][c];
    partc[(int64_t)blockIdx.x * B + b0 + tid] = a;
  }
  float acc[ROWS][KD];
#pragma unroll
  for (int r = 0; r < ROWS; ++r)
#pragma unroll
    for (int k = 0; k < KD; ++k) acc[r][k] = 0.f;
  int c = 0;
  for (; c + 4 <= ncol; c += 4) {  // 4 item rows in flight
    float t[4][KD];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t n = ROWS == 1 ? sidx[c + u] : (int64_t)(c0 + c + u);
      const float w = ri[n];
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int d = tid + 256 * k;
        t[u][k] = d < D ? to_f32(items[n * ldi + d]) * w : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int k = 0; k < KD; ++k) acc[r][k] = fmaf(sg[r][c + u], t[u][k], acc[r][k]);
  }
  for (; c < ncol; ++c) {
    const int64_t n = ROWS == 1 ? sidx[c] : (int64_t)(c0 + c);
    const float w = ri[n];
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = tid + 256 * k;
      const float t = d < D ? to_f32(items[n * ldi + d]) * w : 0.f;
#pragma unroll
      for (int r = 0; r < ROWS; ++r) acc[r][k] = fmaf(sg[r][c], t, acc[r][k]);
    }
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    float* dst = part + ((int64_t)blockIdx.x * B + b0 + r) * D;
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int d = tid + 256 * k;
      if (b0 + r < B && d < D) dst[d] = acc[r][k];
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_cos_bwd_fin(int B, int D, int nch, const T* __restrict__ z, int ldz,
                                                     const float* __restrict__ rz, float inv_temp,
                                                     const float* __restrict__ part, const float* __restrict__ partc,
                                                     float* __restrict__ dz, int64_t lddz) {
  const int b = blockIdx.y;
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= D) return;
  float a = 0.f, cs = 0.f;
  for (int ch = 0; ch < nch; ++ch) {
    a += part[((int64_t)ch * B + b) * D + d];
    cs += partc[(int64_t)ch * B + b];
  }
  const float r = rz[b];
  dz[(int64_t)b * lddz + d] = r * (inv_temp * a - cs * r * to_f32(z[(int64_t)b * ldz + d]));
}

// ------------------------------------------------------------------------------------
// D dispatch: 64*VEC*NCH == D
#define RF_ROW_DISPATCH(D, LAUNCH)                                      \
  do {                                                                  \
    switch (D) {                                                        \
      case 64: LAUNCH(1, 1); break;                                     \
      case 128: LAUNCH(2, 1); break;                                    \
      case 256: LAUNCH(4, 1); break;                                    \
      case 384: LAUNCH(2, 3); break;                                    \
      case 512: LAUNCH(4, 2); break;                                    \
      case 768: LAUNCH(4, 3); break;                                    \
      case 1024: LAUNCH(4, 4); break;                                   \
      default:                                                          \
        ::rf::set_error("row kernel: unsupported width D=%d", (int)D);  \
        return RF_ERR_ARG;                                              \
    }                                                                   \
  } while (0)

// Cross entropy of one logits row against an integer label (torch CrossEntropyLoss with
// ignore_index, the losses of models.py:494-510 and :589-597): loss = logsumexp(x) - x[label],
// 0 for ignored rows; also the row's argmax (first max, as torch.argmax) for cl_correct_num.
// One block per row, two passes over the row (max + first argmax, then sum of exp(x - max)):
// branch-free, ~4 VALU ops per element.
template <typename T>
__global__ void __launch_bounds__(256) k_cross_entropy(int N, const T* __restrict__ x, int64_t ldx,
                                                        const int64_t* __restrict__ labels, int64_t ignore,
                                                        float* __restrict__ loss, int32_t* __restrict__ amax) {
  __shared__ float sm[4];
  __shared__ int si[4];
  __shared__ float ss[4];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const T* xr = x + (int64_t)row * ldx;
  float m = -__builtin_inff();
  int im = 0x7fffffff;
  for (int c = t; c < N; c += 256) {
    const float v = to_f32(xr[c]);
    if (v > m) { m = v; im = c; }  // per thread columns ascend: keeps the first maximum
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int i2 = __shfl_xor(im, o, 64);
    if (m2 > m || (m2 == m && i2 < im)) { m = m2; im = i2; }
  }
  if (lane == 0) { sm[wave] = m; si[wave] = im; }
  __syncthreads();
  float M = sm[0];
  int I = si[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (sm[w] > M || (sm[w] == M && si[w] < I)) { M = sm[w]; I = si[w]; }
  const float mu = M == -__builtin_inff() ? 0.f : M;
  float l = 0.f;
  for (int c = t; c < N; c += 256) l += __expf(to_f32(xr[c]) - mu);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
  if (lane == 0) ss[wave] = l;
  __syncthreads();
  if (t == 0) {
    const float Lq = ss[0] + ss[1] + ss[2] + ss[3];
    const int64_t lab = labels[row];
    float out = 0.f;
    if (lab != ignore) out = (mu + __logf(Lq)) - to_f32(xr[lab]);
    loss[row] = out;
    if (amax) amax[row] = I;
  }
}

// Gradient of the mean cross entropy w.r.t. the logits (the backward of models.py:499-510's
// CrossEntropyLoss after the LM-head decoder): dx[c] = (softmax(x)[c] - [c == label]) * gs[0], 0 for
// ignored rows; gs = upstream gradient / number of counted rows, on the device (no host read).
// One block per row: max, then sum of exp(x - max), then the write — fp32 math, output in the
// logits' dtype (the decoder GEMMs' operand), so no fp32 probability matrix is materialised.
template <typename T>
__global__ void __launch_bounds__(256) k_cross_entropy_bwd(int N, const T* __restrict__ x, int64_t ldx,
                                                            const int64_t* __restrict__ labels, int64_t ignore,
                                                            const float* __restrict__ gs, T* __restrict__ dx,
                                                            int64_t ldd) {
  __shared__ float sm[4], ss[4];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const T* xr = x + (int64_t)row * ldx;
  T* dr = dx + (int64_t)row * ldd;
  const int64_t lab = labels[row];
  if (lab == ignore) {
    for (int c = t; c < N; c += 256) dr[c] = from_f32<T>(0.f);
    return;
  }
  float m = -__builtin_inff();
  for (int c = t; c < N; c += 256) m = fmaxf(m, to_f32(xr[c]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) sm[wave] = m;
  __syncthreads();
  const float M = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  const float mu = M == -__builtin_inff() ? 0.f : M;
  float l = 0.f;
  for (int c = t; c < N; c += 256) l += __expf(to_f32(xr[c]) - mu);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
  if (lane == 0) ss[wave] = l;
  __syncthreads();
  const float g = gs[0];
  const float sc = g / (ss[0] + ss[1] + ss[2] + ss[3]);
  for (int c = t; c < N; c += 256) {
    const float p = __expf(to_f32(xr[c]) - mu) * sc;
    dr[c] = from_f32<T>(c == lab ? p - g : p);
  }
}

// Ranker counts (utils.py:76-108) over a block of fp32 scores: per row b,
//   gt[b]    += #{n : s[b,n] > s_label[b]}   (rank, strict — predicts < scores)
//   valid[b] += #{n : s[b,n] > -max_val}     (valid_length)
//   sexp[b]  += sum_n exp(s[b,n] - shift)   (optional: bounded log-sum-exp for the CE of a
//                                             cosine / temp score row, |s| <= shift = 1/temp)
// grid (rows, column splits); integer atomics, so the counts are exact for any split.
__global__ void __launch_bounds__(256) k_rank_accum(int N, const float* __restrict__ sc, int64_t ld,
                                                     const float* __restrict__ slab, float max_val, float shift,
                                                     int32_t* __restrict__ gt, int32_t* __restrict__ valid,
                                                     float* __restrict__ sexp) {
  __shared__ int sg[4], sv[4];
  __shared__ float se[4];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (N + gridDim.y - 1) / gridDim.y;
  const int c0 = blockIdx.y * per, c1 = min(N, c0 + per);
  const float* sr = sc + (int64_t)row * ld;
  const float lab = slab[row];
  int cg = 0, cv = 0;
  float e = 0.f;
  for (int c = c0 + t; c < c1; c += 256) {
    const float v = sr[c];
    cg += v > lab;
    cv += v > -max_val;
    if (sexp) e += __expf(v - shift);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cg += __shfl_xor(cg, o, 64);
    cv += __shfl_xor(cv, o, 64);
    e += __shfl_xor(e, o, 64);
  }
  if (lane == 0) { sg[wave] = cg; sv[wave] = cv; se[wave] = e; }
  __syncthreads();
  if (t == 0) {
    atomicAdd(gt + row, sg[0] + sg[1] + sg[2] + sg[3]);
    atomicAdd(valid + row, sv[0] + sv[1] + sv[2] + sv[3]);
    if (sexp) atomicAdd(sexp + row, se[0] + se[1] + se[2] + se[3]);
  }
}

template <typename TT, typename T>
static int launch_embed(int M, int D, const int32_t* ids, const int32_t* pos, const int32_t* tt,
                        const int32_t* ip, const void* we, const void* pe, const void* te,
                        const void* ie, const float* lw, const float* lb, float eps, void* out,
                        float* out32, uint16_t* out_lo, hipStream_t s) {
  dim3 grid((M + 3) / 4);
#define L_(V, N)                                                                                 \
  k_embed_ln<TT, T, V, N><<<grid, 256, 0, s>>>(M, ids, pos, tt, ip, (const TT*)we, (const TT*)pe, \
                                               (const TT*)te, (const TT*)ie, lw, lb, eps, (T*)out, \
                                               out32, out_lo)
  RF_ROW_DISPATCH(D, L_);
#undef L_
  RF_LAUNCH_CHECK("rf_embed_ln_fwd");
}

template <typename TX, typename T>
static int launch_ln(int M, int D, const void* x, int ldx, const float* res, const float* w, const float* b,
                     float eps, void* y, int ldy, float* y32, float* mean, float* rstd,
                     hipStream_t s) {
  dim3 grid((M + 3) / 4);
#define L_(V, N) \
  k_layernorm<TX, T, V, N><<<grid, 256, 0, s>>>(M, (const TX*)x, ldx, res, w, b, eps, (T*)y, ldy, y32, mean, rstd)
  RF_ROW_DISPATCH(D, L_);
#undef L_
  RF_LAUNCH_CHECK("rf_layernorm_fwd");
}

}  // namespace rf

using namespace rf;

extern "C" {

const char* rf_last_error(void) { return rf::g_err; }

static int knob_index(const char* name) {
  static const char* names[rf::KNOB_COUNT] = {"gemm_gn", "gemm_variant", "band_qpb", "band_path", "gfold_path",
                                              "gfold_qsplit", "gemm_pf", "gemm_mfma32", "rank_w32",
                                              "gfold_chunk", "gemm_skinny", "epi_tile", "tn_wgs", "mid_tile",
                                              "colsum_slices", "gemm_n192", "adam_nt", "gemm_w8", "gemm_w4p"};
  for (int i = 0; i < rf::KNOB_COUNT; ++i)
    if (name && names[i] && strcmp(name, names[i]) == 0) return i;
  rf::set_error("rf_debug_knob: unknown knob '%s'", name ? name : "(null)");
  return -1;
}

int rf_debug_set_knob(const char* name, int value) {
  const int i = knob_index(name);
  if (i < 0) return INT32_MIN;
  const int old = rf::g_knob[i];
  rf::g_knob[i] = value;
  return old;
}

int rf_debug_get_knob(const char* name) {
  const int i = knob_index(name);
  return i < 0 ? INT32_MIN : rf::g_knob[i];
}
int rf_abi_version(void) { return 2; }  // recformer_amd/_lib.py ABI_VERSION

int rf_prepare_inputs(const int64_t* input_ids, const int64_t* attention_mask,
                      const int64_t* global_attention_mask, const int64_t* token_type_ids,
                      const int64_t* item_position_ids, const int64_t* position_ids, int B,
                      int L, int Lp, int pad_id, int gmax, int32_t* ids, int32_t* pos,
                      int32_t* tt, int32_t* ip, uint8_t* flags, int32_t* gidx, int32_t* gstat,
                      rf_stream_t stream) {
  RF_REQUIRE(input_ids && item_position_ids && ids && pos && tt && ip && flags,
             "rf_prepare_inputs: null pointer");
  RF_REQUIRE(B > 0 && L > 0 && Lp >= L, "rf_prepare_inputs: bad shape B=%d L=%d Lp=%d", B, L, Lp);
  RF_REQUIRE(gmax == 0 || gidx, "rf_prepare_inputs: gidx required when gmax>0");
  k_prepare<<<B, 256, 0, as_stream(stream)>>>(input_ids, attention_mask, global_attention_mask,
                                               token_type_ids, item_position_ids, position_ids,
                                               L, Lp, pad_id, gmax, ids, pos, tt, ip, flags,
                                               gidx, gstat);
  RF_LAUNCH_CHECK("rf_prepare_inputs");
}

int rf_embed_ln_fwd(int table_dtype, int out_dtype, int M, int D, const int32_t* ids,
                    const int32_t* pos, const int32_t* tt, const int32_t* ip, const void* word_emb,
                    const void* pos_emb, const void* type_emb, const void* ipos_emb,
                    const float* ln_w, const float* ln_b, float eps, void* out, float* out32,
                    rf_stream_t stream) {
  RF_REQUIRE(M >= 0, "rf_embed_ln_fwd: bad M");
  if (M == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (table_dtype == RF_F32 && out_dtype == RF_F32)
    return launch_embed<float, float>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b, eps, out, out32, nullptr, s);
  if (table_dtype == RF_F32 && out_dtype == RF_BF16)
    return launch_embed<float, bf16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b, eps, out, out32, nullptr, s);
  if (table_dtype == RF_BF16 && out_dtype == RF_BF16)
    return launch_embed<bf16, bf16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b, eps, out, out32, nullptr, s);
  if (table_dtype == RF_F32 && out_dtype == RF_F16)
    return launch_embed<float, f16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b, eps, out, out32, nullptr, s);
  if (table_dtype == RF_F16 && out_dtype == RF_F16)
    return launch_embed<f16, f16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b, eps, out, out32, nullptr, s);
  RF_REQUIRE(false, "rf_embed_ln_fwd: unsupported dtypes table=%d out=%d", table_dtype, out_dtype);
}

int rf_layernorm_fwd(int x_dtype, int y_dtype, int M, int D, const void* x, int ldx,
                     const float* w, const float* b, float eps, void* y, int ldy, float* y32,
                     float* mean, float* rstd, rf_stream_t stream) {
  return rf_add_layernorm_fwd(x_dtype, y_dtype, M, D, x, ldx, nullptr, w, b, eps, y, ldy, y32, mean, rstd,
                              stream);
}

int rf_add_layernorm_fwd(int x_dtype, int y_dtype, int M, int D, const void* x, int ldx, const float* res,
                         const float* w, const float* b, float eps, void* y, int ldy, float* y32,
                         float* mean, float* rstd, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && ldx >= D && ldy >= D, "rf_layernorm_fwd: bad shape");
  if (M == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (x_dtype == RF_BF16 && y_dtype == RF_BF16)
    return launch_ln<bf16, bf16>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_F32 && y_dtype == RF_BF16)
    return launch_ln<float, bf16>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_F32 && y_dtype == RF_F32)
    return launch_ln<float, float>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_BF16 && y_dtype == RF_F32)
    return launch_ln<bf16, float>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_F16 && y_dtype == RF_F16)
    return launch_ln<f16, f16>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_F32 && y_dtype == RF_F16)
    return launch_ln<float, f16>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  if (x_dtype == RF_F16 && y_dtype == RF_F32)
    return launch_ln<f16, float>(M, D, x, ldx, res, w, b, eps, y, ldy, y32, mean, rstd, s);
  RF_REQUIRE(false, "rf_layernorm_fwd: bad dtypes %d/%d", x_dtype, y_dtype);
}

int rf_embed_ln_split_fwd(int table_dtype, int M, int D, const int32_t* ids, const int32_t* pos,
                          const int32_t* tt, const int32_t* ip, const void* word_emb, const void* pos_emb,
                          const void* type_emb, const void* ipos_emb, const float* ln_w, const float* ln_b,
                          float eps, uint16_t* out_hi, uint16_t* out_lo, rf_stream_t stream) {
  RF_REQUIRE(M >= 0, "rf_embed_ln_split_fwd: bad M");
  if (M == 0) return RF_OK;
  RF_REQUIRE(out_hi && out_lo, "rf_embed_ln_split_fwd: null output plane");
  hipStream_t s = as_stream(stream);
  if (table_dtype == RF_F32)
    return launch_embed<float, bf16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b,
                                     eps, out_hi, nullptr, out_lo, s);
  if (table_dtype == RF_BF16)
    return launch_embed<bf16, bf16>(M, D, ids, pos, tt, ip, word_emb, pos_emb, type_emb, ipos_emb, ln_w, ln_b,
                                    eps, out_hi, nullptr, out_lo, s);
  RF_REQUIRE(false, "rf_embed_ln_split_fwd: unsupported table dtype %d", table_dtype);
}

int rf_add_layernorm_split_fwd(int M, int D, const void* x, int ldx, const uint16_t* res_hi,
                               const uint16_t* res_lo, const float* w, const float* b, float eps,
                               uint16_t* y_hi, uint16_t* y_lo, float* y32, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && ldx >= D, "rf_add_layernorm_split_fwd: bad shape");
  RF_REQUIRE((res_hi == nullptr) == (res_lo == nullptr) && (y_hi == nullptr) == (y_lo == nullptr),
             "rf_add_layernorm_split_fwd: planes come in (hi, lo) pairs");
  RF_REQUIRE(y_hi || y32, "rf_add_layernorm_split_fwd: no output");
  if (M == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  RF_REQUIRE(ldx % 8 == 0, "rf_add_layernorm_split_fwd: ldx must be a multiple of 8");
#define LS_(LPR, NCH) k_add_ln_split<LPR, NCH><<<(M + 256 / LPR - 1) / (256 / LPR), 256, 0, s>>>( \
      M, (const bf16*)x, ldx, res_hi, res_lo, w, b, eps, y_hi, y_lo, y32)
  switch (D) {
    case 64: LS_(8, 1); break;
    case 128: LS_(16, 1); break;
    case 256: LS_(32, 1); break;
    case 384: LS_(16, 3); break;
    case 512: LS_(64, 1); break;
    case 768: LS_(32, 3); break;
    case 1024: LS_(32, 4); break;
    default: RF_REQUIRE(false, "rf_add_layernorm_split_fwd: unsupported width D=%d", D);
  }
#undef LS_
  RF_LAUNCH_CHECK("rf_add_layernorm_split_fwd");
}

size_t rf_layernorm_bwd_workspace(int M, int D) {
  if (M <= 0 || D <= 0) return 0;
  return ((size_t)((M + LNB_ROWS - 1) / LNB_ROWS) + CS_SLICES) * 3 * D * sizeof(float);
}

size_t rf_colsum_workspace(int M, int N) { return (size_t)CS_SLICES * (N > 0 ? N : 0) * sizeof(float); }

int rf_scatter_add_rows(int dtype, int R, int D, const int32_t* rows, const void* src0, const void* src1,
                        int ld_src, void* dst0, void* dst1, int ld_dst, rf_stream_t stream) {
  RF_REQUIRE(R >= 0 && D >= 0 && ld_src >= D && ld_dst >= D, "rf_scatter_add_rows: bad shape");
  if (R == 0 || D == 0) return RF_OK;
  RF_REQUIRE(rows && src0 && dst0 && (!src1 == !dst1), "rf_scatter_add_rows: null pointer");
  hipStream_t s = as_stream(stream);
  dim3 grid((D + 255) / 256, src1 ? 2 : 1);
  if (dtype == RF_BF16)
    k_scatter_add_rows<bf16><<<grid, 256, 0, s>>>(R, D, rows, (const bf16*)src0, (const bf16*)src1, ld_src,
                                                  (bf16*)dst0, (bf16*)dst1, ld_dst);
  else if (dtype == RF_F16)
    k_scatter_add_rows<f16><<<grid, 256, 0, s>>>(R, D, rows, (const f16*)src0, (const f16*)src1, ld_src, (f16*)dst0,
                                                 (f16*)dst1, ld_dst);
  else if (dtype == RF_F32)
    k_scatter_add_rows<float><<<grid, 256, 0, s>>>(R, D, rows, (const float*)src0, (const float*)src1, ld_src,
                                                   (float*)dst0, (float*)dst1, ld_dst);
  else
    RF_REQUIRE(false, "rf_scatter_add_rows: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_scatter_add_rows");
}

int rf_colsum(int dtype, int M, int N, const void* x, int64_t ldx, float* out, int scale_cols, float col_scale,
              void* workspace, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && ldx >= N && scale_cols >= 0, "rf_colsum: bad shape");
  RF_REQUIRE(out && workspace && (M == 0 || x), "rf_colsum: null pointer");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    (void)hipMemsetAsync(out, 0, (size_t)N * sizeof(float), s);
    RF_LAUNCH_CHECK("rf_colsum");
  }
  float* ws = (float*)workspace;
  if (dtype == RF_BF16) colsum<bf16>(M, N, (const bf16*)x, ldx, ws, out, nullptr, N, s, nullptr, scale_cols, col_scale);
  else if (dtype == RF_F16) colsum<f16>(M, N, (const f16*)x, ldx, ws, out, nullptr, N, s, nullptr, scale_cols, col_scale);
  else if (dtype == RF_F32)
    colsum<float>(M, N, (const float*)x, ldx, ws, out, nullptr, N, s, nullptr, scale_cols, col_scale);
  else RF_REQUIRE(false, "rf_colsum: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_colsum");
}

extern "C++" {
template <typename E>
static int ln_bwd_impl(int M, int D, const float* dy, const float* x, int ldx, const float* mean,
                       const float* rstd, const float* w, float* dx, float* dw, float* db, void* workspace,
                       E* dt, uint32_t thresh, float keep_scale, uint64_t seed, rf_stream_t stream,
                       const E* dy2 = nullptr, float* dbias_t = nullptr, int mrow = 1);
}


const uint64_t* rf_set_seed_source(const uint64_t* step_counter) {
  const uint64_t* old = g_seed_dev;
  g_seed_dev = step_counter;
  return old;
}

int rf_drop_add_ln_fwd(int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                       const float* w, const float* b, float eps, float* x, float* y, float* mean, float* rstd,
                       rf_stream_t stream) {
  return rf_drop_add_ln_fwd_dual(M, D, t, ldt, res, p, seed, w, b, eps, x, y, mean, rstd, nullptr, stream);
}

int rf_drop_add_ln_fwd_dual(int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                            const float* w, const float* b, float eps, float* x, float* y, float* mean,
                            float* rstd, void* y16, rf_stream_t stream) {
  return rf_drop_add_ln_fwd_t(RF_BF16, M, D, t, ldt, res, p, seed, w, b, eps, x, y, mean, rstd, y16, 1, stream);
}
int rf_drop_add_ln_fwd_t(int dtype, int M, int D, const void* t, int ldt, const float* res, float p, uint64_t seed,
                         const float* w, const float* b, float eps, float* x, float* y, float* mean, float* rstd,
                         void* y16, int mask_row_mul, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_drop_add_ln_fwd: dtype must be bf16 or fp16");
  RF_REQUIRE(M >= 0 && ldt >= D && p >= 0.f && p < 1.f && mask_row_mul >= 1, "rf_drop_add_ln_fwd: bad arguments");
  if (M == 0) return RF_OK;
  RF_REQUIRE(t && res && w && b && x && y && mean && rstd, "rf_drop_add_ln_fwd: null pointer");
  RF_REQUIRE(ldt % 4 == 0, "rf_drop_add_ln_fwd: ldt must be a multiple of 4");
  hipStream_t s = as_stream(stream);
  const uint32_t th = drop_thresh(p);
  const float ks = 1.0f / (1.0f - p);
  dim3 grid((M + 3) / 4);
#define L_(V, N)                                                                                   \
  k_drop_add_ln_fwd<E, V, N><<<grid, 256, 0, s>>>(M, (const E*)t, ldt, res, th, ks, seed, g_seed_dev, w, b, eps, x, y, \
                                                  mean, rstd, (E*)y16, mask_row_mul)
  if (dtype == RF_F16) {
    typedef f16 E;
    RF_ROW_DISPATCH(D, L_);
  } else {
    typedef bf16 E;
    RF_ROW_DISPATCH(D, L_);
  }
#undef L_
  RF_LAUNCH_CHECK("rf_drop_add_ln_fwd");
}

int rf_drop_add_ln_bwd(int M, int D, const float* dy, const float* x, const float* mean, const float* rstd,
                       const float* w, float p, uint64_t seed, float* dres, void* dt, float* dw, float* db,
                       void* workspace, rf_stream_t stream) {
  RF_REQUIRE(M == 0 || dy, "rf_drop_add_ln_bwd: null dy");
  return rf_drop_add_ln_bwd_dual(M, D, dy, nullptr, x, mean, rstd, w, p, seed, dres, dt, dw, db, workspace, stream);
}

int rf_drop_add_ln_bwd_dual(int M, int D, const float* dy, const void* dy16, const float* x, const float* mean,
                            const float* rstd, const float* w, float p, uint64_t seed, float* dres, void* dt,
                            float* dw, float* db, void* workspace, rf_stream_t stream) {
  return rf_drop_add_ln_bwd_t(RF_BF16, M, D, dy, dy16, x, mean, rstd, w, p, seed, dres, dt, dw, db, workspace, 1,
                              stream);
}
int rf_drop_add_ln_bwd_t(int dtype, int M, int D, const float* dy, const void* dy16, const float* x,
                         const float* mean, const float* rstd, const float* w, float p, uint64_t seed, float* dres,
                         void* dt, float* dw, float* db, void* workspace, int mask_row_mul, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_drop_add_ln_bwd: dtype must be bf16 or fp16");
  RF_REQUIRE(M >= 0 && p >= 0.f && p < 1.f && mask_row_mul >= 1, "rf_drop_add_ln_bwd: bad arguments");
  RF_REQUIRE(M == 0 || dt, "rf_drop_add_ln_bwd: null dt");
  if (dtype == RF_F16)
    return ln_bwd_impl<f16>(M, D, dy, x, D, mean, rstd, w, dres, dw, db, workspace, (f16*)dt, drop_thresh(p),
                            1.0f / (1.0f - p), seed, stream, (const f16*)dy16, nullptr, mask_row_mul);
  return ln_bwd_impl<bf16>(M, D, dy, x, D, mean, rstd, w, dres, dw, db, workspace, (bf16*)dt, drop_thresh(p),
                           1.0f / (1.0f - p), seed, stream, (const bf16*)dy16, nullptr, mask_row_mul);
}

int rf_drop_add_ln_bwd_tb(int dtype, int M, int D, const float* dy, const void* dy16, const float* x,
                          const float* mean, const float* rstd, const float* w, float p, uint64_t seed, float* dres,
                          void* dt, float* dw, float* db, float* dbias_t, void* workspace, int mask_row_mul,
                          rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_drop_add_ln_bwd_tb: dtype must be bf16 or fp16");
  RF_REQUIRE(M >= 0 && p >= 0.f && p < 1.f && mask_row_mul >= 1, "rf_drop_add_ln_bwd_tb: bad arguments");
  RF_REQUIRE(M == 0 || (dt && dbias_t), "rf_drop_add_ln_bwd_tb: null dt / dbias_t");
  if (dtype == RF_F16)
    return ln_bwd_impl<f16>(M, D, dy, x, D, mean, rstd, w, dres, dw, db, workspace, (f16*)dt, drop_thresh(p),
                            1.0f / (1.0f - p), seed, stream, (const f16*)dy16, dbias_t, mask_row_mul);
  return ln_bwd_impl<bf16>(M, D, dy, x, D, mean, rstd, w, dres, dw, db, workspace, (bf16*)dt, drop_thresh(p),
                           1.0f / (1.0f - p), seed, stream, (const bf16*)dy16, dbias_t, mask_row_mul);
}

int rf_layernorm_bwd(int M, int D, const float* dy, const float* x, int ldx, const float* mean,
                     const float* rstd, const float* w, float* dx, float* dw, float* db, void* workspace,
                     rf_stream_t stream) {
  return ln_bwd_impl<bf16>(M, D, dy, x, ldx, mean, rstd, w, dx, dw, db, workspace, nullptr, 0u, 1.f, 0ull, stream);
}

extern "C++" {
template <typename E>
static int ln_bwd_impl(int M, int D, const float* dy, const float* x, int ldx, const float* mean,
                       const float* rstd, const float* w, float* dx, float* dw, float* db, void* workspace,
                       E* dt, uint32_t thresh, float keep_scale, uint64_t seed, rf_stream_t stream,
                       const E* dy2, float* dbias_t, int mrow) {
  RF_REQUIRE(M >= 0 && ldx >= D, "rf_layernorm_bwd: bad shape");
  if (M == 0) return RF_OK;
  RF_REQUIRE((dy || dy2) && x && mean && rstd && w && dx && dw && db && workspace, "rf_layernorm_bwd: null pointer");
  RF_REQUIRE(ldx % 4 == 0, "rf_layernorm_bwd: ldx must be a multiple of 4");
  hipStream_t s = as_stream(stream);
  const int nb = (M + LNB_ROWS - 1) / LNB_ROWS;
  float* part = reinterpret_cast<float*>(workspace);
  const int tb = dt && dbias_t ? 1 : 0;
  const int ns = 2 + tb;
#define L_(V, N) k_layernorm_bwd<E, V, N><<<nb, 256, 0, s>>>(M, dy, x, ldx, mean, rstd, w, dx, part, dt, thresh, keep_scale, seed, g_seed_dev, dy2, tb, mrow)
  RF_ROW_DISPATCH(D, L_);
#undef L_
  // [dw | db (| dbias_t)] columns
  colsum<float>(nb, ns * D, part, ns * D, part + (size_t)nb * ns * D, dw, db, D, s, tb ? dbias_t : nullptr);
  RF_LAUNCH_CHECK("rf_layernorm_bwd");
}
}

int rf_row_inv_norm(int dtype, int M, int D, const void* x, int ldx, float eps, float* out,
                    rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && ldx >= D, "rf_row_inv_norm: bad shape");
  if (M == 0) return RF_OK;
  dim3 grid((M + 3) / 4);
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16) {
#define L_(V, N) k_row_inv_norm<bf16, V, N><<<grid, 256, 0, s>>>(M, (const bf16*)x, ldx, eps, out)
    RF_ROW_DISPATCH(D, L_);
#undef L_
  } else if (dtype == RF_F32) {
#define L_(V, N) k_row_inv_norm<float, V, N><<<grid, 256, 0, s>>>(M, (const float*)x, ldx, eps, out)
    RF_ROW_DISPATCH(D, L_);
#undef L_
  } else if (dtype == RF_F16) {
#define L_(V, N) k_row_inv_norm<f16, V, N><<<grid, 256, 0, s>>>(M, (const f16*)x, ldx, eps, out)
    RF_ROW_DISPATCH(D, L_);
#undef L_
  } else {
    RF_REQUIRE(false, "rf_row_inv_norm: bad dtype %d", dtype);
  }
  RF_LAUNCH_CHECK("rf_row_inv_norm");
}

int rf_gather_global_rows(int dtype, int B, int Lp, int D, int gmax, const void* x, int ldx,
                          const int32_t* gidx, void* out, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && gmax >= 0 && ldx >= D, "rf_gather_global_rows: bad shape");
  if (B == 0 || gmax == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16)
    k_gather_rows<bf16><<<B * gmax, 256, 0, s>>>(Lp, D, gmax, (const bf16*)x, ldx, gidx, (bf16*)out);
  else if (dtype == RF_F16)
    k_gather_rows<f16><<<B * gmax, 256, 0, s>>>(Lp, D, gmax, (const f16*)x, ldx, gidx, (f16*)out);
  else if (dtype == RF_F32)
    k_gather_rows<float><<<B * gmax, 256, 0, s>>>(Lp, D, gmax, (const float*)x, ldx, gidx, (float*)out);
  else
    RF_REQUIRE(false, "rf_gather_global_rows: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_gather_global_rows");
}

int rf_cos_score_cand(int dtype, int B, int C, int D, const void* z, int ldz, const float* rz,
                      const void* items, int ldi, const float* ri, const int64_t* cand,
                      float inv_temp, float* scores, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && C >= 0 && D > 0, "rf_cos_score_cand: bad shape");
  if (B == 0 || C == 0) return RF_OK;
  dim3 grid((B * C + 3) / 4);
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16)
    k_cos_cand<bf16><<<grid, 256, 0, s>>>(B, C, D, (const bf16*)z, ldz, rz, (const bf16*)items, ldi,
                                          ri, cand, inv_temp, scores);
  else if (dtype == RF_F16)
    k_cos_cand<f16><<<grid, 256, 0, s>>>(B, C, D, (const f16*)z, ldz, rz, (const f16*)items, ldi, ri, cand, inv_temp,
                                         scores);
  else if (dtype == RF_F32)
    k_cos_cand<float><<<grid, 256, 0, s>>>(B, C, D, (const float*)z, ldz, rz, (const float*)items,
                                           ldi, ri, cand, inv_temp, scores);
  else
    RF_REQUIRE(false, "rf_cos_score_cand: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_cos_score_cand");
}

size_t rf_cos_score_bwd_workspace(int B, int C, int D) {
  const int64_t nch = (C + COS_NCH - 1) / COS_NCH;
  return (size_t)(nch * B * ((int64_t)D + 1) * sizeof(float));
}

int rf_cos_score_bwd(int dtype, int B, int C, int D, const void* z, int ldz, const float* rz, const void* items,
                     int ldi, const float* ri, const int64_t* cand, float inv_temp, const float* g, int64_t ldg,
                     const float* s, int64_t lds, void* ws, float* dz, int64_t lddz, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && C >= 0 && D > 0 && D <= 1024, "rf_cos_score_bwd: bad shape B=%d C=%d D=%d", B, C, D);
  RF_REQUIRE(ldz >= D && ldi >= D && ldg >= C && lds >= C && lddz >= D, "rf_cos_score_bwd: bad leading dims");
  if (B == 0) return RF_OK;
  RF_REQUIRE(z && rz && items && ri && g && s && ws && dz, "rf_cos_score_bwd: null pointer");
  const int nch = (C + COS_NCH - 1) / COS_NCH;
  hipStream_t st = as_stream(stream);
  float* part = reinterpret_cast<float*>(ws);
  float* partc = part + (int64_t)nch * B * D;
  if (C == 0) {
    RF_REQUIRE(hipMemsetAsync(dz, 0, sizeof(float) * (size_t)lddz * (B - 1) + sizeof(float) * D, st) == hipSuccess,
               "rf_cos_score_bwd: memset failed");
    return RF_OK;
  }
  const int KD = (D + 255) / 256;
#define COS_PART(T, ROWS, KDV)                                                                                  \
  k_cos_bwd_part<T, ROWS, KDV><<<dim3(nch, (B + ROWS - 1) / ROWS), 256, 0, st>>>(                               \
      B, C, D, (const T*)items, ldi, ri, cand, g, ldg, s, lds, part, partc)
#define COS_KD(T, ROWS)                                   \
  switch (KD) {                                           \
    case 1: COS_PART(T, ROWS, 1); break;                  \
    case 2: COS_PART(T, ROWS, 2); break;                  \
    case 3: COS_PART(T, ROWS, 3); break;                  \
    default: COS_PART(T, ROWS, 4); break;                 \
  }
#define COS_ROWS(T)                \
  if (cand) { COS_KD(T, 1) }       \
  else { COS_KD(T, 16) }
  const dim3 fgrid((D + 255) / 256, B);
  if (dtype == RF_F32) {
    COS_ROWS(float)
    k_cos_bwd_fin<float><<<fgrid, 256, 0, st>>>(B, D, nch, (const float*)z, ldz, rz, inv_temp, part, partc, dz, lddz);
  } else if (dtype == RF_BF16) {
    COS_ROWS(bf16)
    k_cos_bwd_fin<bf16><<<fgrid, 256, 0, st>>>(B, D, nch, (const bf16*)z, ldz, rz, inv_temp, part, partc, dz, lddz);
  } else if (dtype == RF_F16) {
    COS_ROWS(f16)
    k_cos_bwd_fin<f16><<<fgrid, 256, 0, st>>>(B, D, nch, (const f16*)z, ldz, rz, inv_temp, part, partc, dz, lddz);
  } else {
    RF_REQUIRE(false, "rf_cos_score_bwd: bad dtype %d", dtype);
  }
#undef COS_ROWS
#undef COS_KD
#undef COS_PART
  RF_LAUNCH_CHECK("rf_cos_score_bwd");
}

int rf_cross_entropy_bwd(int dtype, int M, int N, const void* logits, int64_t ldx, const int64_t* labels,
                        int64_t ignore_index, const float* grad_scale, void* dlogits, int64_t ldd, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && ldx >= N && ldd >= N, "rf_cross_entropy_bwd: bad shape");
  if (M == 0) return RF_OK;
  RF_REQUIRE(logits && labels && grad_scale && dlogits, "rf_cross_entropy_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16)
    k_cross_entropy_bwd<bf16><<<M, 256, 0, s>>>(N, (const bf16*)logits, ldx, labels, ignore_index, grad_scale,
                                                (bf16*)dlogits, ldd);
  else if (dtype == RF_F16)
    k_cross_entropy_bwd<f16><<<M, 256, 0, s>>>(N, (const f16*)logits, ldx, labels, ignore_index, grad_scale,
                                               (f16*)dlogits, ldd);
  else if (dtype == RF_F32)
    k_cross_entropy_bwd<float><<<M, 256, 0, s>>>(N, (const float*)logits, ldx, labels, ignore_index, grad_scale,
                                                 (float*)dlogits, ldd);
  else
    RF_REQUIRE(false, "rf_cross_entropy_bwd: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_cross_entropy_bwd");
}

int rf_cross_entropy_fwd(int dtype, int M, int N, const void* logits, int64_t ldx, const int64_t* labels,
                         int64_t ignore_index, float* loss, int32_t* argmax, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N > 0 && ldx >= N, "rf_cross_entropy_fwd: bad shape");
  RF_REQUIRE(logits && labels && loss, "rf_cross_entropy_fwd: null pointer");
  if (M == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16)
    k_cross_entropy<bf16><<<M, 256, 0, s>>>(N, (const bf16*)logits, ldx, labels, ignore_index, loss, argmax);
  else if (dtype == RF_F16)
    k_cross_entropy<f16><<<M, 256, 0, s>>>(N, (const f16*)logits, ldx, labels, ignore_index, loss, argmax);
  else if (dtype == RF_F32)
    k_cross_entropy<float><<<M, 256, 0, s>>>(N, (const float*)logits, ldx, labels, ignore_index, loss, argmax);
  else
    RF_REQUIRE(false, "rf_cross_entropy_fwd: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_cross_entropy_fwd");
}

int rf_rank_accum(int M, int N, const float* scores, int64_t ld, const float* s_label, float max_val,
                  float shift, int32_t* gt, int32_t* valid, float* sexp, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && N >= 0 && ld >= N, "rf_rank_accum: bad shape");
  RF_REQUIRE(scores && s_label && gt && valid, "rf_rank_accum: null pointer");
  if (M == 0 || N == 0) return RF_OK;
  const int splits = min(64, (N + 8191) / 8192);
  k_rank_accum<<<dim3(M, splits), 256, 0, as_stream(stream)>>>(N, scores, ld, s_label, max_val, shift, gt, valid,
                                                              sexp);
  RF_LAUNCH_CHECK("rf_rank_accum");
}

}  // extern "C"
