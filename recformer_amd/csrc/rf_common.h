// Shared device/host helpers for librecformer_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/recformer_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef _Float16 f16;  // fp16 operands (the reference's torch.cuda.amp default, finetune.py:106-110)
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace rf {

// ---- error plumbing (no C++ exception crosses the C ABI) ------------------------------
void set_error(const char* fmt, ...);
void clear_error();

#define RF_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      ::rf::set_error(__VA_ARGS__);           \
      return RF_ERR_ARG;                      \
    }                                         \
  } while (0)

#define RF_LAUNCH_CHECK(name)                                                         \
  do {                                                                                \
    hipError_t _e = hipGetLastError();                                                \
    if (_e != hipSuccess) {                                                           \
      ::rf::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));          \
      return RF_ERR_HIP;                                                              \
    }                                                                                 \
    return RF_OK;                                                                     \
  } while (0)

inline hipStream_t as_stream(rf_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- tuning knobs (A/B tools only) -------------------------------------------------------
// Launch-path choices measured once and compiled in as defaults; tools/ switch them through
// rf_debug_set_knob (one host call, no environment lookups on any launch).
enum Knob {
  KNOB_GEMM_GN = 0,     // ping-pong GEMM raster: column-group width (6)
  KNOB_GEMM_VARIANT,    // bf16 GEMM kernel family (8 = four-wave interleaved, 6 = four-wave, 5 = ping-pong, 7 = BK32 ring)
  KNOB_BAND_QPB,        // band attention query blocks per workgroup (0 = auto)
  KNOB_BAND_PATH,       // band attention kernel: 3 pipe3 (default), 0 pipe2, 1 pipe (v1), 2 one-shot
  KNOB_GFOLD_PATH,      // global fold: 0 auto, 1 GEMV, 2 MFMA, 3 auto without the ring partial kernel, 4 ring at any Lp
  KNOB_GFOLD_QSPLIT,    // global fold query/key kernel: max column splits (8)
  KNOB_GEMM_PF,         // four-wave GEMM L2 prefetch: -1 auto (2 for K >= 2048), else distance in K-tiles (0 = off), + 256: W rows too
  KNOB_GEMM_MFMA32,     // four-wave GEMM on v_mfma_f32_32x32x16 (k_gemm_w32): 1 on, 0 the 16x16x32 kernel (k_gemm_w4)
  KNOB_RANK_W32,        // catalog score + rank on the 32x32x16 four-wave loop (k_rank_w32 + k_label_score32): 1 on
                        // (0 by default; ranker.rank_catalog / retrieve(k=0) take it for their counts-only
                        // pass: 1M x 4096 6.96 vs 7.89 ms; the top-k mode is faster on 16x16x32, r04h)
  KNOB_GFOLD_CHUNK,     // inference global fold: rows per chunk of the pass over h (0 = 256; 64 / 128)
  KNOB_GEMM_SKINNY,     // 16-bit GEMMs with M <= 64 rows on k_gemm_skinny (1, default) or the 128 x 128 kernel (0)
  KNOB_EPI_TILE,        // training GELU GEMMs (EPI_DGELU, EPI_BIAS_GELU_AUX): 0 the four-wave 256x256 kernel,
                        // 1 the 128x128 tile kernel, 2 the 256x128 tile kernel (several workgroups per CU,
                        // so one's epilogue overlaps another's MFMAs)
  KNOB_TN_WGS,          // weight-gradient GEMM: workgroups its row split aims at (0 = one per CU)
  KNOB_MID_TILE,        // EPI_NONE / EPI_BIAS GEMMs whose 256x256 grid leaves CUs idle: 0 the four-wave kernel,
                        // 1 the 128x128 tile kernel, 2 the 256x128 one (captured C3: 17.77 / 18.20 vs
                        // 16.26 / 16.36 ms, r04z: the older tile kernels lose more than the idle CUs cost)
  KNOB_COLSUM_SLICES,   // column sums (bias gradients): row slices at most (0 = CS_SLICES; A/B of the slice count)
  KNOB_GEMM_N192,       // EPI_NONE / EPI_BIAS / 16-bit EPI_BIAS_RESID GEMMs whose 256^2 grid leaves CUs idle: 1 the
                        // four-wave kernel on 256 x 192 tiles when those fill one round; 0 (default): the captured
                        // C3 step measured slower with it (16.01 vs 15.92 ms, gpurun_out/r05n): the narrower
                        // tile issues 14 operand DMA pieces per 96 MFMAs instead of 16 per 128
  KNOB_ADAM_NT,         // AdamW: non-temporal operand loads / stores (1, default: captured C3 16.03 vs 16.07 ms,
                        // gpurun_out/r05q) or plain (0)
  KNOB_GEMM_W8,         // 16-bit EPI_NONE / EPI_BIAS / EPI_BIAS_GELU GEMMs on the eight-wave ping-pong kernel
                        // (k_gemm_w8: two waves per SIMD, one computing while its partner loads): 1 on, 0 the
                        // four-wave kernel
  KNOB_GEMM_W4P,        // 16-bit EPI_NONE / EPI_BIAS / EPI_BIAS_GELU GEMMs on the four-wave kernel with k-step-split
                        // LDS planes (k_gemm_w4p: operand DMA spread over both phases): 1 on, 0 k_gemm_w4
  KNOB_COUNT
};
extern int g_knob[KNOB_COUNT];

// ---- scalar conversions ---------------------------------------------------------------
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f32(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f32<f16>(float x) { return (f16)x; }

// ---- 16-bit operand types: bf16 (autocast bfloat16) and fp16 (torch.cuda.amp default) ----------
template <typename E> struct H16;
template <> struct H16<bf16> {
  typedef bf16x8 x8;
  typedef bf16x4 x4;
  typedef bf16x2 x2;
  static constexpr bool bf = true;
};
template <> struct H16<f16> {
  typedef f16x8 x8;
  typedef f16x4 x4;
  typedef f16x2 x2;
  static constexpr bool bf = false;
};
// v_mfma_f32_16x16x32_{bf16,f16}: one instruction shape, the element type picks the opcode
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// erf with |error| <= 1.5e-7 (Abramowitz & Stegun 7.1.26): one v_rcp, one v_exp and a
// degree-5 Horner chain — ~4x fewer VALU issues than the libm erff, which dominated the
// FFN1 GEMM epilogue (it runs after the MFMA loop, so its VALU cost is not hidden).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float y = fmaf(-p * t, __expf(-ax * ax), 1.0f);
  return copysignf(y, x);
}

// exact-erf GELU (transformers ACT2FN['gelu'] = x * Phi(x), TF:1115), |error| < 1e-6 |x|
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// derivative of the exact-erf GELU, d/dz [z Phi(z)] = Phi(z) + z phi(z), as torch's gelu_backward
// (approximate='none') computes it in fp32
// (erf through erf_fast's form with its exp(-x^2) = exp(-z^2 / 2) shared with phi: one v_exp, one
// v_rcp per value)
__device__ __forceinline__ float dgelu_erf(float z) {
  const float ax = fabsf(z) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float e = __expf(-ax * ax);
  const float erf = copysignf(fmaf(-p * t, e, 1.0f), z);
  return fmaf(0.5f, erf, 0.5f) + z * 0.3989422804014327f * e;
}
// the same on 8 values, one stage at a time across 4 pairs (independent chains fill the transcendental
// hazards; see gelu8_bf16out), the multiplies, FMAs and adds as packed-fp32 (v_pk_*) pairs: the same
// operations per value in the same order, so bit-identical to dgelu_erf (hipcc left this scalar: ~13
// VALU + 2 transcendentals per value, a third of the GELU-backward GEMM's tile time at 16k x 3072 x 768)
__device__ __forceinline__ void dgelu8_erf(const float (&z)[8], float (&d)[8]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 c0 = {0.70710678118654752f, 0.70710678118654752f};
  f2 zz[4], ax[4], t[4], p[4], e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) zz[k] = (f2){z[2 * k], z[2 * k + 1]};
#pragma unroll
  for (int k = 0; k < 4; ++k) ax[k] = __builtin_elementwise_abs(zz[k]) * c0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f2 q = __builtin_elementwise_fma((f2){0.3275911f, 0.3275911f}, ax[k], (f2){1.0f, 1.0f});
    t[k] = (f2){__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f2 a2 = -ax[k] * ax[k];
    e[k] = (f2){__expf(a2.x), __expf(a2.y)};
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = __builtin_elementwise_fma(t[k], (f2){1.061405429f, 1.061405429f},
                                                               (f2){-1.453152027f, -1.453152027f});
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = __builtin_elementwise_fma(t[k], p[k], (f2){1.421413741f, 1.421413741f});
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = __builtin_elementwise_fma(t[k], p[k], (f2){-0.284496736f, -0.284496736f});
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = __builtin_elementwise_fma(t[k], p[k], (f2){0.254829592f, 0.254829592f});
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f2 y = __builtin_elementwise_fma(-p[k] * t[k], e[k], (f2){1.0f, 1.0f});
    const f2 erf = __builtin_elementwise_copysign(y, zz[k]);
    const f2 r = __builtin_elementwise_fma((f2){0.5f, 0.5f}, erf, (f2){0.5f, 0.5f}) +
                 zz[k] * (f2){0.3989422804014327f, 0.3989422804014327f} * e[k];
    d[2 * k] = r.x;
    d[2 * k + 1] = r.y;
  }
}

// GELU for 16-bit outputs: x * sigmoid(x (a + b x^2 + c x^4)) with (a, b, c) fitted minimax to
// the exact-erf GELU, x^2 clamped at 64; |error| <= 2.6e-5 absolute on all of R (fp32): below the
// bf16 rounding of the stored value, and below fp16's for |y| >= 0.03 (smaller outputs differ by
// at most 2.6e-5 absolute). 8 VALU + 2 transcendental vs ~18 + 2 for gelu_erf.
// Constants are pre-multiplied by -log2(e) so the exponential is one v_exp_f32.
__device__ __forceinline__ float gelu_bf16out(float x) {
  const float x2 = fminf(x * x, 64.0f);
  const float p = fmaf(fmaf(0.0010142630552196598f, x2, -0.1067757240026454f), x2, -2.3011213394567367f);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * p));
}

// gelu_bf16out on a pair (the same operations, so bit-identical): the multiplies, adds and
// FMAs issue as v_pk_*_f32, one instruction per pair.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2_bf16out(f32x2 x) {
  const f32x2 x2 = __builtin_elementwise_min(x * x, (f32x2){64.0f, 64.0f});
  const f32x2 p = __builtin_elementwise_fma(
      __builtin_elementwise_fma((f32x2){0.0010142630552196598f, 0.0010142630552196598f}, x2,
                                (f32x2){-0.1067757240026454f, -0.1067757240026454f}),
      x2, (f32x2){-2.3011213394567367f, -2.3011213394567367f});
  const f32x2 t = x * p;
  const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
  return x * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// gelu_bf16out on 4 pairs, one stage at a time across the pairs (the same operations per value, so
// bit-identical): the four chains interleave, so the transcendental and packed-op hazards fill with
// the other chains' instructions instead of s_nop (the per-pair form compiled to a serial chain).
// The clamp runs as one packed multiply with the VOP3P clamp bit: s = clamp(x (x / 64)) in [0, 1] =
// min(x^2, 64) / 64, and the quadratic's coefficients are scaled by 64 and 4096 — powers of two, so
// every rounding equals the unscaled form's (bit-identical to gelu2_bf16out) for two v_min_f32 less
// per pair.
__device__ __forceinline__ void gelu8_bf16out(f32x2 (&x)[4]) {
  f32x2 x2[4], t[4], d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x64 = x[k] * (f32x2){0.015625f, 0.015625f};
    asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(x2[k]) : "v"(x[k]), "v"(x64));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    t[k] = __builtin_elementwise_fma((f32x2){0.0010142630552196598f * 4096.0f, 0.0010142630552196598f * 4096.0f},
                                     x2[k], (f32x2){-0.1067757240026454f * 64.0f, -0.1067757240026454f * 64.0f});
#pragma unroll
  for (int k = 0; k < 4; ++k)
    t[k] = __builtin_elementwise_fma(t[k], x2[k], (f32x2){-2.3011213394567367f, -2.3011213394567367f});
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = x[k] * t[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = (f32x2){__builtin_amdgcn_exp2f(t[k].x), __builtin_amdgcn_exp2f(t[k].y)};
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = d[k] + 1.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = (f32x2){__builtin_amdgcn_rcpf(d[k].x), __builtin_amdgcn_rcpf(d[k].y)};
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = x[k] * d[k];
}

// ---- split fp32 residual stream ------------------------------------------------
// An fp32 value v is stored as two 16-bit planes: hi = the top half of bits(v) rounded half-up
// (a bf16 within half an ulp of v: the GEMM operand), lo = the low 16 bits of bits(v). The
// pair decodes to bits(v) exactly: hi was rounded up iff bit 15 of lo is set. Rounding half-up
// differs from the round-to-nearest-even bf16 cast only on exact ties (by one bf16 ulp).
__device__ __forceinline__ void split_f32(float v, uint16_t& hi, uint16_t& lo) {
  const uint32_t u = __float_as_uint(v);
  hi = (uint16_t)((u + 0x8000u) >> 16);
  lo = (uint16_t)(u & 0xFFFFu);
}
__device__ __forceinline__ float join_f32(uint32_t hi, uint32_t lo) {
  return __uint_as_float(((hi - (lo >> 15)) << 16) | lo);
}

// ---- dropout keep masks (training path) ------------------------------------------------------
// Counter hash of (seed, element index): regenerated by each backward, never stored. P(keep) =
// 1 - thresh / 2^32 with thresh = drop_thresh(p); kept values are scaled by 1 / (1 - p)
// (nn.functional.dropout). recformer_amd/dropout.py restates it bit-exactly in torch.
__host__ __device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  uint32_t h = (uint32_t)idx * 0x9E3779B1u ^ (uint32_t)(idx >> 32) * 0x85EBCA77u ^ (uint32_t)seed;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= (uint32_t)(seed >> 32);
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h >= thresh;
}
inline uint32_t drop_thresh(float p) {
  return p <= 0.f ? 0u : (p >= 1.f ? 0xFFFFFFFFu : (uint32_t)((double)p * 4294967296.0));
}
// Attention-probability dropout (TF:585-586 local rows, TF:1036-1037 global rows): one mask entry
// per (sequence b, head h, query position i, key position j), index ((b H + h) Lp + i) Lp + j.
struct AttnDrop {
  uint64_t seed;
  uint32_t thresh;                   // 0: off
  float scale;                       // 1 / (1 - p)
  const uint64_t* seed_dev = nullptr;  // step counter in device memory (g_seed_dev), mixed in at kernel start
};
// Device-side dropout seeds for captured (hipGraph) training steps: rf_set_seed_source() registers a
// device uint64 step counter; every dropout launch made while it is set passes the pointer, and the
// kernel uses seed + counter * SEED_STEP_MIX, so one captured graph draws fresh masks on each replay
// (the caller advances the counter inside the graph) while the forward and the backward of one step
// agree. Unset (the default) the seeds are exactly the host values.
extern const uint64_t* g_seed_dev;
constexpr uint64_t SEED_STEP_MIX = 0x9E3779B97F4A7C15ull;
__device__ __forceinline__ uint64_t seed_resolve(uint64_t seed, const uint64_t* dev) {
  return dev ? seed + *dev * SEED_STEP_MIX : seed;
}
__device__ __forceinline__ void drop_resolve(AttnDrop& d) {
  if (d.thresh && d.seed_dev) d.seed = seed_resolve(d.seed, d.seed_dev);
  d.seed_dev = nullptr;
}
__device__ __forceinline__ float attn_keep_scale(const AttnDrop& d, uint64_t row, int Lp, int key) {
  return drop_keep(d.seed, row * (uint64_t)Lp + (uint64_t)key, d.thresh) ? d.scale : 0.f;
}

// Bijective XCD-aware remap of a 1-D block id (guide §5 T1): the hardware deals block ids
// round-robin over the 8 XCDs; the returned index is contiguous per XCD, so blocks that share
// data (neighbouring tiles, windows) run on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ---- wave64 reductions ----------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 16-byte global->LDS DMA: LDS destination is (wave-uniform base + lane*16); the global
// source is per lane (cdna_hip_programming.md §5 'Async global->LDS copy').
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// the same with the non-temporal cache policy (read-once streams)
__device__ __forceinline__ void glds16_nt(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 2);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Byte offset of 16-B chunk `ch` (0..7) of row `row` in a [rows][64 x bf16] LDS tile
// (128-B rows) with the XOR swizzle ch ^ (row & 7): conflict-free ds_read_b128 of the
// MFMA 16x16x32 operand pattern (rows l&15, chunk l>>4) — guide §5.5 T2.
__device__ __forceinline__ int swz128(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

}  // namespace rf
