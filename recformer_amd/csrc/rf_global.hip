// Global-token attention rows via the key/value-projection fold (SURVEY.md §8a row A6, §7
// 'Global-path algebra').
//
// The reference projects key_global / value_global over ALL L tokens of every layer
// (TF:983-984) only to serve the G global query rows (TF:964-1057). Per head h:
//     s_j   = qg_h . (Wkg_h h_j + bkg_h) = u_h . h_j + c_h,   u_h = Wkg_h^T qg_h
//     out_h = sum_j p_j (Wvg_h h_j + bvg_h) = Wvg_h w_h + bvg_h,  w_h = sum_j p_j h_j  (sum p = 1)
// c_h = qg_h . bkg_h is the same for every key j, so softmax removes it. The two d x d
// projections over L tokens (4 L d^2 flops/layer, 2/5 of the fused QKV GEMM) collapse to
// per-head GEMVs plus one streaming pass over h. Same algebra, different rounding.
//
//   k_gfold_u        (16, R):     u_h = Wkg_h^T qg_h  (bf16 path: bf16 [R][16][D], heads>=H = 0;
//                                                      fp32 path: fp32 [R][H][D+4])
//   k_gfold_partial  (Lp/64, R):  one 64-row chunk of h: s = u.h_j over valid keys, chunk
//                                 max / sum per head, w_part[c][h] = sum_j p_j h_j[c].
//                                 bf16: the 64 x D chunk is DMA'd to LDS once; S^T = H.U^T and
//                                 W^T = H^T.P^T run on v_mfma_f32_16x16x32_bf16 (H^T and P^T
//                                 through ds_read_b64_tr_b16), like the band-attention kernel
//                                 with "keys = values = h" and the heads as 16 queries.
//   k_gfold_out      (H, R):      log-sum-exp merge of the chunks, out = Wvg_h w_h + bvg_h,
//                                 written into ctx at the global token's row (TF:621-629).
#include "rf_common.h"

namespace rf {

constexpr float GF_NEG_INF = -__builtin_inff();
#ifndef RF_GF_CH
#define RF_GF_CH 256
#endif
constexpr int GF_CH = RF_GF_CH;  // rows per chunk (bf16 kernel walks it in 64-row sub-chunks)
constexpr int GF_CHF = 64;
#if defined(RF_GF_DIAG)  // timing diagnostics of k_gfold_partial_bf16 (tools/build_variant.sh only)
constexpr bool RF_GF_DIAG_SC = (RF_GF_DIAG & 1) != 0;  // no score MFMAs
constexpr bool RF_GF_DIAG_PH = (RF_GF_DIAG & 4) != 0;  // no P.H products
#else
constexpr bool RF_GF_DIAG_SC = false, RF_GF_DIAG_PH = false;
#endif    // rows per chunk of the fp32 VALU kernel
// the partial pass's image stream: RF_GF_NT (A/B builds) reads it with the non-temporal policy — measured
// slower (C2: kernel 30.1 vs 27.9 us, step 12.28 vs 12.13 ms, profiles/r05/gfold_partial_ab.txt): the
// layer's next reader of h then misses the Infinity Cache
#if defined(RF_GF_NT)
#define GF_IMG_DMA glds16_nt
#else
#define GF_IMG_DMA glds16
#endif
// RF_GF_STAMPS (tools/build_variant.sh only, inference): k_gfold_partial_bf16's wave 0 records
// s_memrealtime (100 MHz) at 16 points into free LDS and copies them to the (unused without dropout)
// ws.ld slots of its (row, chunk) — tools/gfold_stamps.py reads the timeline.
#if defined(RF_GF_STAMPS)
#define GF_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (threadIdx.x == 0) gf_lds_st32(red + GF_RED_LD + (k), __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_s_memrealtime())); \
  } while (0)
#else
#define GF_STAMP(k) do { } while (0)
#endif
constexpr int GF_HP = 16;     // heads padded to one MFMA column tile (H <= 16)
constexpr int GF_RED_LD = 176;  // partial kernels' LDS reduction area: dropped sums at red + 176
constexpr int GF_RED_FLOATS = GF_RED_LD + 64;

struct GfoldWs {
  bf16* u16;     // [R][2 planes hi/lo][16][D]
  float* u32;    // [R][H][D+4]
  float* m;      // [R][nch][16]
  float* l;      // [R][nch][16]
  float* ld;     // [R][nch][16]  sum of the dropped probabilities (attention dropout only)
  float* w;      // [R][nch][16][D]
};

// Rows per chunk of the training forward's 16-bit partial pass (rf_global_attn_fold_fwd_drop; one
// block per (chunk, global row)): GF_CH = 256 when the grid fills the chip, halved down to 64 while it
// has fewer blocks than the chip has CUs and at most 16 chunks (C3, B = 16: 64 -> 256 blocks; C4 at 4
// per rank: 16 -> 64) — every block streams its chunk once, so a short grid leaves CUs idle. The
// backward reads the forward's chunk partials with the same count. The inference entry points keep
// GF_CH: the chunking sets the rounding of the softmax merge, and a sequence's scores there must
// not depend on the batch it is encoded in (test_c2_full_size_properties).
constexpr int GF_FILL = 256;  // MI355X CUs
inline int gfold_chunk(int dtype, int R, int Lp) {
  if (dtype == RF_F32) return GF_CHF;
  int ch = GF_CH;
  while (ch > 64 && (int64_t)R * ((Lp + ch - 1) / ch) < GF_FILL && (Lp + ch / 2 - 1) / (ch / 2) <= 16) ch /= 2;
  return ch;
}

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline GfoldWs gfold_carve(void* ws, int R, int nch, int H, int D) {
  char* p = (char*)ws;
  GfoldWs w;
  w.u16 = (bf16*)p; p += align256((size_t)R * 2 * GF_HP * D * 2);
  w.u32 = (float*)p; p += align256((size_t)R * H * (D + 4) * 4);
  w.m = (float*)p; p += align256((size_t)R * nch * GF_HP * 4);
  w.l = (float*)p; p += align256((size_t)R * nch * GF_HP * 4);
  w.ld = (float*)p; p += align256((size_t)R * nch * GF_HP * 4);
  w.w = (float*)p;
  return w;
}

inline size_t gfold_bytes(int R, int nch, int H, int D) {
  return align256((size_t)R * 2 * GF_HP * D * 2) + align256((size_t)R * H * (D + 4) * 4) +
         3 * align256((size_t)R * nch * GF_HP * 4) + (size_t)R * nch * D * GF_HP * 4;
}

__device__ __forceinline__ void load4(const float* p, float* x) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
}
__device__ __forceinline__ void load4(const bf16* p, float* x) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  x[0] = (float)v[0]; x[1] = (float)v[1]; x[2] = (float)v[2]; x[3] = (float)v[3];
}

__device__ __forceinline__ void load4(const f16* p, float* x) {
  const f16x4 v = *reinterpret_cast<const f16x4*>(p);
  x[0] = (float)v[0]; x[1] = (float)v[1]; x[2] = (float)v[2]; x[3] = (float)v[3];
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_g;
template <typename E>
__device__ __forceinline__ typename H16<E>::x4 tr_read_g(const char* p) {  // 16-bit bit patterns
  return __builtin_bit_cast(typename H16<E>::x4, __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_g*)p));
}
// The same read as inline asm, for reads that overlap an LDS-DMA in flight: hipcc puts an
// s_waitcnt vmcnt(0) in front of every transposed-read builtin issued after an LDS-DMA (it cannot
// rule out that the DMA writes the bytes read), which drained the partial kernel's refill of the
// other image half before each P.H product. The asm read is invisible to hipcc's wait bookkeeping:
// the caller retires it with tr_wait() (lgkmcnt(0) + a scheduling fence) before any use.
template <typename E>
__device__ __forceinline__ typename H16<E>::x4 tr_read_ga(const char* p) {
  typename H16<E>::x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
__device__ __forceinline__ void tr_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// 16-bit plane type of the u planes for an element type (fp32 mode writes none)
template <typename T> struct Plane16 { typedef T type; };
template <> struct Plane16<float> { typedef bf16 type; };

__device__ __forceinline__ void gf_lds_st32(const void* p, float v) {  // LDS store invisible to hipcc's waits
  asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p),
               "v"(v) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- u = Wkg_h^T qg_h ------------------------------------------------------------------
// grid (16 heads, R): one block per (head, global row); thread t owns columns 4t..4t+3 of
// Wkg_h (64 rows x D), reads them with 8-B vector loads (L2-resident weights) and dots them
// with the head's 64 query values (LDS broadcast). bf16 path writes u as hi + lo bf16 planes
// (u ~= hi + lo to ~16 mantissa bits) so the MFMA score product keeps fp32-like precision
// in u: s = hi.h + lo.h; heads >= H are written as zeros (padding of the 16-head tile).
template <typename T>
__global__ void __launch_bounds__(256) k_gfold_u(int D, int H, int R, const T* __restrict__ qg,
                                                  int ld_qg, const T* __restrict__ wkg,
                                                  const int32_t* __restrict__ gidx, GfoldWs ws,
                                                  bool out_bf16) {
  typedef typename Plane16<T>::type P16;
  __shared__ float qs[64];
  const int h = blockIdx.x, r = blockIdx.y;
  if (gidx[r] < 0) return;
  const int t = threadIdx.x;
  if (h < H && t < 64) qs[t] = to_f32(qg[(int64_t)r * ld_qg + h * 64 + t]);
  __syncthreads();
  for (int k = 4 * t; k < D; k += 4 * blockDim.x) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (h < H) {
      const T* wp = wkg + (int64_t)(h * 64) * D + k;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) {
        float x[4];
        load4(wp + (int64_t)d * D, x);
        const float qd = qs[d];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fmaf(qd, x[i], a[i]);
      }
    }
    if (out_bf16) {
      P16* hi = reinterpret_cast<P16*>(ws.u16) + ((int64_t)r * 2 * GF_HP + h) * D + k;
      P16* lo = hi + (int64_t)GF_HP * D;
      typename H16<P16>::x4 vh, vl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vh[i] = (P16)a[i];
        vl[i] = (P16)(a[i] - (float)vh[i]);
      }
      *reinterpret_cast<typename H16<P16>::x4*>(hi) = vh;
      *reinterpret_cast<typename H16<P16>::x4*>(lo) = vl;
    } else if (h < H) {
      *reinterpret_cast<float4*>(ws.u32 + ((int64_t)r * H + h) * (D + 4) + k) = make_float4(a[0], a[1], a[2], a[3]);
    }
  }
}

// ---- qg_h and u_h straight from the layer input ----------------------------------------------
// grid (16 heads, R): qg_h = (Wqg_h h_g + bqg_h) * q_scale for the global row's hidden vector h_g
// (rounded to the compute dtype, as the qg GEMM would store it), then u_h = Wkg_h^T qg_h as in
// k_gfold_u. Replaces gather + qg GEMM + u (three launches) for the fold path.
template <typename T>
__global__ void __launch_bounds__(256) k_gfold_qu(int Lp, int D, int H, int gmax, const T* __restrict__ hs,
                                                   int ldh, const T* __restrict__ wqg,
                                                   const float* __restrict__ bqg, float q_scale,
                                                   const T* __restrict__ wkg, const int32_t* __restrict__ gidx,
                                                   GfoldWs ws, bool out_bf16) {
  typedef typename Plane16<T>::type P16;
  __shared__ float hrow[1024];
  __shared__ float qs[64];
  const int h = blockIdx.x, r = blockIdx.y;
  const int pos = gidx[r];
  if (pos < 0) return;
  const int b = r / gmax;
  const int t = threadIdx.x;
  if (h < H) {
    const T* hr = hs + ((int64_t)b * Lp + pos) * ldh;
    for (int k = t; k < D; k += blockDim.x) hrow[k] = to_f32(hr[k]);
    __syncthreads();
    {
      const int d = t >> 2, part = t & 3;  // 4 threads per output of qg_h (64 outputs)
      const T* wr = wqg + (int64_t)(h * 64 + d) * D;
      float a = 0.f;
      for (int k = 8 * part; k < D; k += 32) {
        float x[8];
        load4(wr + k, x);
        load4(wr + k + 4, x + 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) a = fmaf(x[i], hrow[k + i], a);
      }
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      if (part == 0) qs[d] = to_f32(from_f32<T>((a + bqg[h * 64 + d]) * q_scale));
    }
  }
  __syncthreads();
  for (int k = 4 * t; k < D; k += 4 * blockDim.x) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (h < H) {
      const T* wp = wkg + (int64_t)(h * 64) * D + k;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) {
        float x[4];
        load4(wp + (int64_t)d * D, x);
        const float qd = qs[d];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fmaf(qd, x[i], a[i]);
      }
    }
    if (out_bf16) {
      P16* hi = reinterpret_cast<P16*>(ws.u16) + ((int64_t)r * 2 * GF_HP + h) * D + k;
      P16* lo = hi + (int64_t)GF_HP * D;
      typename H16<P16>::x4 vh, vl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vh[i] = (P16)a[i];
        vl[i] = (P16)(a[i] - (float)vh[i]);
      }
      *reinterpret_cast<typename H16<P16>::x4*>(hi) = vh;
      *reinterpret_cast<typename H16<P16>::x4*>(lo) = vl;
    } else if (h < H) {
      *reinterpret_cast<float4*>(ws.u32 + ((int64_t)r * H + h) * (D + 4) + k) = make_float4(a[0], a[1], a[2], a[3]);
    }
  }
}

// ---- bf16 partial: MFMA over a 64-row chunk -----------------------------------------------
// LDS image of the chunk: segment-major [D/64][64 rows][128 B] with the 16-B slot XOR
// (row & 7) inside each 128-B segment (lane-linear DMA pieces of 8 rows x 128 B).
__device__ __forceinline__ int gimg(int row, int col) {
  return (((col >> 6) * 64 + row) << 7) + ((((col >> 3) & 7) ^ (row & 7)) << 4) + ((col & 7) << 1);
}

// ---- bf16 qg_h and u_h on MFMA, 64 global rows per block -------------------------------------
// grid (H, ceil(R/64)), 4 waves x 16 global rows. The head's 64 x D slice of Wqg, then of Wkg,
// is DMA'd once into an LDS image shared by the block's 64 rows (the GEMV kernels above read it
// once per row: L2-bound when R is large, e.g. a catalog of short item sequences).
//   qg[row][d] = bf16((h_g[row] . Wqg[h*64+d] + bqg) * q_scale)   (A: h rows from HBM, B: LDS)
//   u[row][c]  = sum_d qg[row][d] Wkg[h*64+d][c]                    (A: Wkg^T via ds_read_tr,
//                                                                    B: qg^T via ds_read_tr)
// u is written as the hi + lo bf16 planes k_gfold_partial_bf16 reads; heads >= H are not
// written (the partial kernel does not load them). Column split (gridDim.z): a block stages only
// the 64-column segments of Wkg its u columns need; with `sep` that slice has its own LDS region
// and its DMA goes out with Wqg's at the start (one wait), else it reuses the Wqg region after
// the qg phase.
template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_qu_mfma(int Lp, int R, int gmax, const E* __restrict__ hs,
                                                        int ldh, const E* __restrict__ wqg,
                                                        const float* __restrict__ bqg, float q_scale,
                                                        const E* __restrict__ wkg,
                                                        const int32_t* __restrict__ gidx, GfoldWs ws,
                                                        int sep) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  const int h = blockIdx.x, r0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int q4 = li >> 2, p4 = li & 3;
  // u columns of this block and the Wkg segments they span
  const int nct = D / 16 / gridDim.z, ct0 = blockIdx.z * nct;
  const int sg0 = (16 * ct0) >> 6, sg1 = (16 * (ct0 + nct) + 63) >> 6;
  char* kimg = sep ? smem + nseg * 64 * 128 : smem;                  // Wkg slice image
  char* pimg = smem + (nseg + (sep ? sg1 - sg0 : 0)) * 64 * 128 + wave * 2048;  // qg^T [64 d][16 rows]
  const int r = r0 + 16 * wave + li;
  const int pos = r < R ? gidx[r] : -1;

  V8 a[NK];
  if (pos >= 0) {
    const E* hr = hs + ((int64_t)(r / gmax) * Lp + pos) * ldh + 8 * g;
#pragma unroll
    for (int s = 0; s < NK; ++s) a[s] = *reinterpret_cast<const V8*>(hr + 32 * s);
  } else {
#pragma unroll
    for (int s = 0; s < NK; ++s) a[s] = V8{};
  }
  // segments [s0, s1) of the head's 64-row weight slice into image `dst` (segment s at s - s0)
  auto dma_head = [&](const E* w, char* dst, int s0, int s1) {
    for (int p = wave + 8 * s0; p < s1 * 8; p += 4) {
      const int seg = p >> 3, row = (p & 7) * 8 + (lane >> 3);
      const int chk = (lane & 7) ^ (row & 7);
      glds16(w + (int64_t)(h * 64 + row) * D + seg * 64 + chk * 8, dst + ((seg - s0) * 64 + (p & 7) * 8) * 128);
    }
  };
  dma_head(wqg, smem, 0, nseg);
  if (sep) dma_head(wkg, kimg, sg0, sg1);
  wait_vmcnt0();
  __syncthreads();
  {
    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NK; ++s)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const V8 b = *reinterpret_cast<const V8*>(smem + gimg(16 * nt + li, 32 * s + 8 * g));
        acc[nt] = mfma16(a[s], b, acc[nt]);
      }
    // C[row 4g+i][d 16nt+li] -> qg^T image [d][row]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int d = 16 * nt + li;
      const float bb = bqg[h * 64 + d];
      V4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (E)((acc[nt][i] + bb) * q_scale);
      *reinterpret_cast<V4*>(pimg + (d * 16 + 4 * g) * 2) = v;
    }
  }
  __syncthreads();  // every wave is done with the Wqg image
#if defined(RF_GF_DIAG) && (RF_GF_DIAG & 2)
  return;
#endif
  if (!sep) {
    dma_head(wkg, kimg, sg0, sg1);
    wait_vmcnt0();
  }
  __syncthreads();
  V8 pb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int rb = 32 * s + 8 * g + q4;
    const V4 v0 = tr_read_g<E>(pimg + (rb * 16 + 4 * p4) * 2);
    const V4 v1 = tr_read_g<E>(pimg + ((rb + 4) * 16 + 4 * p4) * 2);
    pb[s] = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  }
  const int rw = r0 + 16 * wave + li;  // C column n = li -> this wave's row li
  const bool wr = rw < R && gidx[rw] >= 0;
  E* hi = reinterpret_cast<E*>(ws.u16) + ((int64_t)rw * 2 * GF_HP + h) * D + 4 * g;
  E* lo = hi + (int64_t)GF_HP * D;
  // column split (gridDim.z): this block writes u columns [z D / nz, (z + 1) D / nz)
  for (int ct = ct0; ct < ct0 + nct; ++ct) {
    const int c0 = 16 * ct, cl = c0 - 64 * sg0;  // column within the staged slice
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int rb = 32 * s + 8 * g + q4;
      const V4 v0 = tr_read_g<E>(kimg + gimg(rb, cl + 4 * p4));
      const V4 v1 = tr_read_g<E>(kimg + gimg(rb + 4, cl + 4 * p4));
      const V8 wa = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      acc = mfma16(wa, pb[s], acc);
    }
    // C[col c0+4g+i][row li]
#if defined(RF_GF_DIAG) && (RF_GF_DIAG & 1)
    if (acc[0] == 1234.5f) {
#else
    if (wr) {
#endif
      V4 vh, vl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vh[i] = (E)acc[i];
        vl[i] = (E)(acc[i] - (float)vh[i]);
      }
      *reinterpret_cast<V4*>(hi + c0) = vh;
      *reinterpret_cast<V4*>(lo + c0) = vl;
    }
  }
}

// ---- bf16 merge + out on MFMA, 64 global rows per block ----------------------------------------
// grid (H, ceil(R/64)). w_h[row] = sum_c exp(m_c - M) w_c / sum_c exp(m_c - M) l_c is formed in
// registers from the fp32 chunk partials and split into hi + lo bf16 (MFMA B operand);
// out[row][h*64+d] = Wvg[h*64+d] . w_h[row] + bvg, with the head's Wvg slice in LDS.
template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_out_mfma(int Lp, int R, int gmax, int nch,
                                                         const E* __restrict__ wvg,
                                                         const float* __restrict__ bvg,
                                                         const int32_t* __restrict__ gidx, GfoldWs ws,
                                                         E* __restrict__ out, int ldo, bool drop) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  const int h = blockIdx.x, r0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  for (int p = wave; p < nseg * 8; p += 4) {
    const int seg = p >> 3, row = (p & 7) * 8 + (lane >> 3);
    const int chk = (lane & 7) ^ (row & 7);
    glds16(wvg + (int64_t)(h * 64 + row) * D + seg * 64 + chk * 8, smem + (seg * 64 + (p & 7) * 8) * 128);
  }
  const int r = r0 + 16 * wave + li;
  const int pos = r < R ? gidx[r] : -1;
  const int rr = pos >= 0 ? r : 0;  // rows without a global token read row 0's partials, unused
  float mx = GF_NEG_INF;
  for (int c = 0; c < nch; ++c) mx = fmaxf(mx, ws.m[((int64_t)rr * nch + c) * GF_HP + h]);
  float lsum = 0.f, dsum = 0.f;
  for (int c = 0; c < nch; ++c) {
    const float mc = ws.m[((int64_t)rr * nch + c) * GF_HP + h];
    const float sc = mc == GF_NEG_INF ? 0.f : __expf(mc - mx);
    lsum += sc * ws.l[((int64_t)rr * nch + c) * GF_HP + h];
    if (drop) dsum += sc * ws.ld[((int64_t)rr * nch + c) * GF_HP + h];
  }
  const float inv = lsum > 0.f ? 1.0f / lsum : 0.f;
  // the value bias enters with the weight sum_j p'_j (1 without dropout: the p_j sum to 1)
  const float bw = drop ? dsum * inv : 1.f;
  wait_vmcnt0();
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* wbase = ws.w + ((int64_t)rr * nch * GF_HP + h) * D + 8 * g;
#pragma unroll 2
  for (int s = 0; s < NK; ++s) {
    float w8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nch; ++c) {
      const float mc = ws.m[((int64_t)rr * nch + c) * GF_HP + h];
      const float sc = (mc == GF_NEG_INF ? 0.f : __expf(mc - mx)) * inv;
      const float* wp = wbase + (int64_t)c * GF_HP * D + 32 * s;
#if defined(RF_GF_DIAG) && (RF_GF_DIAG & 4)
      const float4 x0 = make_float4(sc, sc, sc, (float)s), x1 = x0; (void)wp;
#else
      const float4 x0 = *reinterpret_cast<const float4*>(wp);
      const float4 x1 = *reinterpret_cast<const float4*>(wp + 4);
#endif
      w8[0] = fmaf(sc, x0.x, w8[0]); w8[1] = fmaf(sc, x0.y, w8[1]);
      w8[2] = fmaf(sc, x0.z, w8[2]); w8[3] = fmaf(sc, x0.w, w8[3]);
      w8[4] = fmaf(sc, x1.x, w8[4]); w8[5] = fmaf(sc, x1.y, w8[5]);
      w8[6] = fmaf(sc, x1.z, w8[6]); w8[7] = fmaf(sc, x1.w, w8[7]);
    }
    V8 bh, bl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bh[i] = (E)w8[i];
      bl[i] = (E)(w8[i] - (float)bh[i]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const V8 wa = *reinterpret_cast<const V8*>(smem + gimg(16 * nt + li, 32 * s + 8 * g));
      acc[nt] = mfma16(wa, bh, acc[nt]);
      acc[nt] = mfma16(wa, bl, acc[nt]);
    }
  }
  // C[d 16nt+4g+i][row li]
  if (pos >= 0) {
    E* o = out + ((int64_t)(r / gmax) * Lp + pos) * ldo + h * 64 + 4 * g;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      V4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (E)(acc[nt][i] + (drop ? bvg[h * 64 + 16 * nt + 4 * g + i] * bw
                                                                 : bvg[h * 64 + 16 * nt + 4 * g + i]));
      *reinterpret_cast<V4*>(o + 16 * nt) = v;
    }
  }
}

// The chunk image is filled in two column halves (segments [0, D/128) and [D/128, D/64)),
// each 12 (D=768) DMA pieces per wave: the scores' k-steps over half A run while half B lands,
// and the next sub-chunk's half A / half B are issued as soon as every wave's P.H products
// over that half are done — so the h stream overlaps the MFMA work instead of alternating
// with it. Row validity comes from per-sub-chunk ballots taken in the prologue (no global
// load inside the loop, whose hipcc wait would drain the DMA queue).
template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_partial_bf16(int Lp, int gmax, int chr,
                                                             const E* __restrict__ hs, int ldh,
                                                             const uint8_t* __restrict__ flags,
                                                             const int32_t* __restrict__ gidx,
                                                             GfoldWs ws, int H, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  constexpr int hseg = nseg / 2;        // segments per half
  constexpr int nmt = D >> 6;            // 16-column tiles of W per wave (D/16 over 4 waves)
  constexpr int hmt = nmt / 2;           // ... per half
  constexpr int PPW = hseg * 8 / 4;      // DMA pieces per wave per half
  if constexpr (nseg % 2 != 0) return;  // D not a multiple of 128: k_gfold_partial_bf16_1 instead
  const int ch = blockIdx.x, r = blockIdx.y, nch = gridDim.x;
  char* pimg = smem + nseg * 64 * 128;                         // P [64 rows][16 heads] bf16
  float* red = reinterpret_cast<float*>(pimg + 64 * 16 * 2);    // [max 4x16][sum 4x16][m 16][alpha 16]
  GF_STAMP(0);
  if (gidx[r] < 0) return;
  const int b = r / gmax;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int q4 = li >> 2, p4 = li & 3;
  float* m_run = red + 128;
  float* alpha_s = red + 144;
  unsigned long long* vmask = reinterpret_cast<unsigned long long*>(red + 160);  // per sub-chunk
  const E* hb = hs + (int64_t)b * Lp * ldh;
  const int row_begin = ch * chr;
  const int row_end = min(row_begin + chr, Lp);
  const int nsub = (row_end - row_begin + 63) >> 6;

  auto dma_half = [&](int j0, int half) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wave * PPW + i;                     // piece within the half
      const int seg = half * hseg + (p >> 3), row = (p & 7) * 8 + (lane >> 3);
      const int chk = (lane & 7) ^ (row & 7);
      const int jr = min(j0 + row, Lp - 1);
      GF_IMG_DMA(reinterpret_cast<const char*>(hb) + (uint32_t)((jr * ldh + seg * 64 + chk * 8) * (int)sizeof(E)),
             smem + (seg * 64 + (p & 7) * 8) * 128);
    }
  };
  // u (B operand of S^T = H.U^T, hi and lo planes; heads >= H score 0). D <= 768: u is DMA'd once per
  // block into LDS in fragment order ([plane][k-step][lane] x 16 B, conflict-free ds_read_b128) with
  // the first image, instead of every wave loading all of it into registers — 4x fewer u bytes (the
  // register loads were 50 MB per C2 launch against the 25 MB first image, and the prologue waited
  // 4.9 us for them before the image went out: s_memrealtime stamps, tools/gfold_stamps.py).
#if defined(RF_GF_OLD_PROLOGUE)  // A/B builds only: the round-4 register-u prologue
  constexpr bool ULDS = false;
#else
  constexpr bool ULDS = D <= 768;
#endif
  constexpr int UPW = 2 * NK / 4;  // u pieces per wave
  char* uimg = reinterpret_cast<char*>(red + GF_RED_FLOATS);
  V8 uh[ULDS ? 1 : NK], ul[ULDS ? 1 : NK];
  if constexpr (!ULDS) {
    const E* uhi = reinterpret_cast<const E*>(ws.u16) + ((int64_t)r * 2 * GF_HP + li) * D + 8 * g;
    const E* ulo = uhi + (int64_t)GF_HP * D;
#pragma unroll
    for (int s2 = 0; s2 < NK; ++s2) {
      uh[s2] = li < H ? *reinterpret_cast<const V8*>(uhi + 32 * s2) : V8{};
      ul[s2] = li < H ? *reinterpret_cast<const V8*>(ulo + 32 * s2) : V8{};
    }
    if (wave < nsub) {  // validity ballots of the (up to 4) 64-row sub-chunks
      const int jr = row_begin + 64 * wave + lane;
      const bool ok = jr < Lp && flags[(int64_t)b * Lp + jr] != 0;
      const unsigned long long m = __ballot(ok);
      if (lane == 0) vmask[wave] = m;
    }
    if (threadIdx.x < 16) m_run[threadIdx.x] = GF_NEG_INF;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // u fragments and flags, before the DMA stream
    GF_STAMP(1);
    dma_half(row_begin, 0);
    dma_half(row_begin, 1);
    GF_STAMP(2);
  } else {
    const int jf = row_begin + 64 * wave + lane;
    int fv = (wave < nsub && jf < Lp) ? (int)flags[(int64_t)b * Lp + jf] : 0;
    // piece (plane, k-step s2): lane (li, g) <- u[plane][head li][32 s2 + 8 g ..]; rows >= H read row
    // H - 1 (an in-bounds source), zeroed in LDS once landed (below)
    const E* ub = reinterpret_cast<const E*>(ws.u16) + ((int64_t)r * 2 * GF_HP + min(li, H - 1)) * D + 8 * g;
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int pc = wave * UPW + i, plane = pc / NK, s2 = pc % NK;
      glds16(ub + (int64_t)plane * GF_HP * D + 32 * s2, uimg + pc * 1024);
    }
    dma_half(row_begin, 0);
    dma_half(row_begin, 1);
    GF_STAMP(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // u, the first image and the flags landed
    // padding heads (li >= H) were DMA'd from head H - 1 (a finite in-bounds source): zero their u so
    // their score columns and workspace slots (m, l, W of heads >= H) are those of u = 0, not copies of
    // a real head's. No reader uses them (the out / backward kernels loop h < H); this keeps it so.
    // The same wave wrote these bytes by DMA and waited for them above, so the stores land after them.
    if (li >= H) {
#pragma unroll
      for (int i = 0; i < UPW; ++i) *reinterpret_cast<V8*>(uimg + (wave * UPW + i) * 1024 + lane * 16) = V8{};
    }
    asm volatile("" : "+v"(fv));
    if (wave < nsub) {
      const unsigned long long m = __ballot(fv != 0);
      if (lane == 0) vmask[wave] = m;
    }
    if (threadIdx.x < 16) m_run[threadIdx.x] = GF_NEG_INF;
    GF_STAMP(2);
  }
  float l_run = 0.f, ld_run = 0.f;  // per head li (valid in wave 0, g == 0)
  const uint64_t drow = ((uint64_t)b * H + li) * Lp + (uint64_t)max(gidx[r], 0);  // dropout mask row
  f32x4 acc[nmt];
#pragma unroll
  for (int i = 0; i < nmt; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int sub = 0; sub < nsub; ++sub) {
    const int j0 = row_begin + 64 * sub;
    const bool more = sub + 1 < nsub;
    // S^T[j = 16*wave + 4g + q][head = li]: k-steps over half A, then half B
    f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
    const int arow = 16 * wave + li;
    wait_vm_n<PPW>();  // half A landed (half B's PPW pieces may still fly)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (sub < 4) GF_STAMP(3 + 3 * sub);
#pragma unroll
    for (int s2 = 0; s2 < (RF_GF_DIAG_SC ? 0 : NK / 2); ++s2) {
      const V8 a = *reinterpret_cast<const V8*>(smem + gimg(arow, 32 * s2 + 8 * g));
      if constexpr (ULDS) {
        st = mfma16(a, *reinterpret_cast<const V8*>(uimg + (s2 * 64 + lane) * 16), st);
        st = mfma16(a, *reinterpret_cast<const V8*>(uimg + ((NK + s2) * 64 + lane) * 16), st);
      } else {
        st = mfma16(a, uh[s2], st);
        st = mfma16(a, ul[s2], st);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // half B landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int s2 = NK / 2; s2 < (RF_GF_DIAG_SC ? NK / 2 : NK); ++s2) {
      const V8 a = *reinterpret_cast<const V8*>(smem + gimg(arow, 32 * s2 + 8 * g));
      if constexpr (ULDS) {
        st = mfma16(a, *reinterpret_cast<const V8*>(uimg + (s2 * 64 + lane) * 16), st);
        st = mfma16(a, *reinterpret_cast<const V8*>(uimg + ((NK + s2) * 64 + lane) * 16), st);
      } else {
        st = mfma16(a, uh[s2], st);
        st = mfma16(a, ul[s2], st);
      }
    }
    const unsigned long long vm = vmask[sub];
    float mx = GF_NEG_INF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jj = 16 * wave + 4 * g + q;
      const bool ok = (vm >> jj) & 1ull;
      st[q] = ok ? st[q] : GF_NEG_INF;
      mx = fmaxf(mx, st[q]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (g == 0) red[wave * 16 + li] = mx;
    __syncthreads();
    const float m_old = m_run[li];
    const float m_new = fmaxf(m_old, fmaxf(fmaxf(red[li], red[16 + li]), fmaxf(red[32 + li], red[48 + li])));
    const float mu = (m_new == GF_NEG_INF) ? 0.f : m_new;
    float ls = 0.f, lsd = 0.f;
    E* pt = reinterpret_cast<E*>(pimg);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p = __expf(st[q] - mu);
      ls += p;
      if (dr.thresh) {  // TF:1036-1037: W and the value-bias weight use the dropped probabilities
        p *= attn_keep_scale(dr, drow, Lp, j0 + 16 * wave + 4 * g + q);
        lsd += p;
      }
      pt[(16 * wave + 4 * g + q) * 16 + li] = (E)p;
    }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    if (g == 0) red[64 + wave * 16 + li] = ls;
    if (dr.thresh) {
      lsd += __shfl_xor(lsd, 16, 64);
      lsd += __shfl_xor(lsd, 32, 64);
      if (g == 0) red[GF_RED_LD + wave * 16 + li] = lsd;
    }
    __syncthreads();  // P, sums and every wave's read of m_run are done
    if (wave == 0 && g == 0) {
      const float a = __expf(m_old - mu);  // 0 when m_old = -inf
      l_run = l_run * a + red[64 + li] + red[80 + li] + red[96 + li] + red[112 + li];
      if (dr.thresh)
        ld_run = ld_run * a + red[GF_RED_LD + li] + red[GF_RED_LD + 16 + li] + red[GF_RED_LD + 32 + li] +
                 red[GF_RED_LD + 48 + li];
      alpha_s[li] = a;
      m_run[li] = m_new;
    }
    __syncthreads();
    if (sub < 4) GF_STAMP(4 + 3 * sub);
    // rescale W rows (head 4g + q) by alpha, then W[head][c] += sum_j p[j][head] h[j][c]
    float al[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) al[q] = alpha_s[4 * g + q];
    // P.H over each image half: transposed reads as asm (no vmcnt(0) in front of them: the other
    // half's refill stays in flight), in batches of PB column tiles, each retired by tr_wait()
    V8 pa[2];
    {
      V4 pv[4];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int rb = 32 * s2 + 8 * g + q4;
        pv[2 * s2] = tr_read_ga<E>(pimg + (rb * 16 + 4 * p4) * 2);
        pv[2 * s2 + 1] = tr_read_ga<E>(pimg + ((rb + 4) * 16 + 4 * p4) * 2);
      }
      tr_wait();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        pa[s2] = V8{pv[2 * s2][0], pv[2 * s2][1], pv[2 * s2][2], pv[2 * s2][3],
                    pv[2 * s2 + 1][0], pv[2 * s2 + 1][1], pv[2 * s2 + 1][2], pv[2 * s2 + 1][3]};
    }
    constexpr int PB = D >= 1024 ? 1 : (hmt % 3 == 0 ? 3 : (hmt % 2 == 0 ? 2 : 1));  // D = 1024: u fills the VGPRs
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int i0 = 0; i0 < (RF_GF_DIAG_PH ? 0 : hmt); i0 += PB) {
        V4 hv[PB][4];
#pragma unroll
        for (int ii = 0; ii < PB; ++ii) {
          const int col = (half * (nmt * 2) + wave * hmt + i0 + ii) * 16 + 4 * p4;  // column tile of this half
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int rb = 32 * s2 + 8 * g + q4;
            hv[ii][2 * s2] = tr_read_ga<E>(smem + gimg(rb, col));
            hv[ii][2 * s2 + 1] = tr_read_ga<E>(smem + gimg(rb + 4, col));
          }
        }
        tr_wait();
#pragma unroll
        for (int ii = 0; ii < PB; ++ii) {
          const int i = half * hmt + i0 + ii;
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[i][q] *= al[q];
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const V4 v0 = hv[ii][2 * s2], v1 = hv[ii][2 * s2 + 1];
            const V8 hb8 = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
            acc[i] = mfma16(pa[s2], hb8, acc[i]);
          }
        }
      }
      // every wave is done reading this half of the image: refill it with the next sub-chunk
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#if !(defined(RF_GF_DIAG) && (RF_GF_DIAG & 2))  // diagnostic: no refill DMA (stale image)
      if (more) dma_half(j0 + 64, half);
#endif
    }
    if (sub < 4) GF_STAMP(5 + 3 * sub);
  }
  if (wave == 0 && g == 0) {
    ws.m[((int64_t)r * nch + ch) * GF_HP + li] = m_run[li];
    ws.l[((int64_t)r * nch + ch) * GF_HP + li] = l_run;
    if (dr.thresh) ws.ld[((int64_t)r * nch + ch) * GF_HP + li] = ld_run;
  }
  float* wout = ws.w + ((int64_t)r * nch + ch) * GF_HP * D;
#pragma unroll
  for (int half = 0; half < 2; ++half)
#pragma unroll
    for (int ii = 0; ii < hmt; ++ii) {
      const int i = half * hmt + ii;
      const int c0 = (half * (nmt * 2) + wave * hmt + ii) * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * g + q < H) wout[(int64_t)(4 * g + q) * D + c0 + li] = acc[i][q];
    }
#if defined(RF_GF_STAMPS)
  GF_STAMP(15);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 16) ws.ld[((int64_t)r * nch + ch) * GF_HP + threadIdx.x] = red[GF_RED_LD + threadIdx.x];
#endif
}

// ---- partial pass on a 3-slot ring of 32-row sub-chunks (round 3; D a multiple of 128, <= 768) ------
// The two-half image above keeps one 64-row sub-chunk in flight and waits one memory latency per
// sub-chunk. Here the chunk walks 32-row sub-chunks through three LDS slots with two of them in flight
// while the third is computed. The score product S^T = H.U^T splits its D-reduction over the four waves
// (each wave holds only its quarter of u: 12 fragments instead of 48, so the loop has registers to
// spare) and sums the partial scores in LDS; the online softmax runs with one head per 16 lanes (max
// and sum by lane shuffles, the running statistics in registers); P.H as the old kernel (transposed LDS
// reads, accumulators rescaled by alpha). LDS stores that follow an LDS-DMA in flight are inline asm:
// hipcc would otherwise wait for every DMA outstanding before each of them.
template <int D>
__device__ __forceinline__ int gimg32(int row, int col) {
  return (((col >> 6) * 32 + row) << 7) + ((((col >> 3) & 7) ^ (row & 7)) << 4) + ((col & 7) << 1);
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void lds_st32(const void* p, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st16(const void* p, uint32_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_fence_barrier() {  // the asm stores above are complete, then barrier
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_partial_ring(int Lp, int gmax, int chr, const E* __restrict__ hs, int ldh,
                                                            const uint8_t* __restrict__ flags,
                                                            const int32_t* __restrict__ gidx, GfoldWs ws, int H,
                                                            AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int KW = NK / 4 > 0 ? NK / 4 : 1;  // score k-steps per wave
  constexpr int nseg = D >> 6;
  constexpr int SLOT = 32 * D * 2;    // bytes per 32-row sub-chunk image
  constexpr int PPW = nseg * 4 / 4;   // DMA pieces (8 rows x 128 B) per wave per sub-chunk
  constexpr int nmt = D >> 6;         // P.H column tiles per wave
  if constexpr (NK % 4 != 0 || D > 768) return;  // D a multiple of 128 up to 768 (host dispatch)
  float* red = reinterpret_cast<float*>(smem + 3 * SLOT);            // [4 waves][32 rows][16 heads]
  char* pimg = smem + 3 * SLOT + 4 * 32 * 16 * 4;                     // P [32 rows][16 heads] 16-bit
  float* alpha_s = reinterpret_cast<float*>(pimg + 32 * 16 * 2);      // [16]
  const int ch = blockIdx.x, r = blockIdx.y, nch = gridDim.x;
  if (gidx[r] < 0) return;
  const int pos = gidx[r];
  const int b = r / gmax;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int q4 = li >> 2, p4 = li & 3;
  const E* hb = hs + (int64_t)b * Lp * ldh;
  const int row_begin = ch * chr;
  const int row_end = min(row_begin + chr, Lp);
  const int nsub = (row_end - row_begin + 31) >> 5;
  // validity flags of the chunk's rows (up to 256), loaded with u (one memory round trip in all)
  uint32_t fl[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) fl[q] = flags[(int64_t)b * Lp + min(row_begin + 64 * q + lane, Lp - 1)];
  // u fragments of this wave's k range (hi and lo planes); heads >= H score 0
  V8 uh[KW], ul[KW];
  {
    const E* uhi = reinterpret_cast<const E*>(ws.u16) + ((int64_t)r * 2 * GF_HP + li) * D + 8 * g;
    const E* ulo = uhi + (int64_t)GF_HP * D;
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {
      const int s2 = wave * KW + kk;
      uh[kk] = li < H ? *reinterpret_cast<const V8*>(uhi + 32 * s2) : V8{};
      ul[kk] = li < H ? *reinterpret_cast<const V8*>(ulo + 32 * s2) : V8{};
    }
  }
  unsigned long long vm[4];  // row validity, ballots of 64 rows
#pragma unroll
  for (int q = 0; q < 4; ++q) vm[q] = __ballot(row_begin + 64 * q + lane < row_end && fl[q] != 0);
  // u and the flags are in registers before the DMA stream starts: the fence makes hipcc wait for them
  // here, not (with vmcnt(0), draining the ring) at their first use inside the loop
#pragma unroll
  for (int kk = 0; kk < KW; ++kk) asm volatile("" : "+v"(uh[kk]), "+v"(ul[kk]));
  // sub-chunk k (rows row_begin + 32 k ..) into slot k % 3; rows past the chunk read clamped rows
  auto dma = [&](int k) {
    char* slot = smem + (k % 3) * SLOT;
    const int j0 = row_begin + 32 * k;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;                  // piece: segment pc / 4, rows 8 (pc % 4) ..
      const int seg = pc >> 2, row = (pc & 3) * 8 + (lane >> 3);
      const int chk = (lane & 7) ^ (row & 7);
      const int jr = min(j0 + row, Lp - 1);
      glds16(reinterpret_cast<const char*>(hb) + (uint32_t)((jr * ldh + seg * 64 + chk * 8) * (int)sizeof(E)),
             slot + (seg * 32 + (pc & 3) * 8) * 128);
    }
  };
  dma(0);
  dma(1);
  // running statistics of head hh = lane-group of 16 (thread -> head t / 16, rows 2 (t % 16) + {0, 1})
  const int hh = threadIdx.x >> 4, tr = threadIdx.x & 15;
  float m_run = GF_NEG_INF, l_run = 0.f, ld_run = 0.f;
  const uint64_t drow = ((uint64_t)b * H + min(hh, H - 1)) * Lp + (uint64_t)pos;
  f32x4 acc[nmt];
#pragma unroll
  for (int i = 0; i < nmt; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sub = 0; sub < nsub; ++sub) {
    dma(sub + 2);  // into the slot sub - 1 used (released by the barrier ending the last iteration)
    wait_vm_n<2 * PPW>();  // sub-chunk sub landed (sub + 1, sub + 2 may fly)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* slot = smem + (sub % 3) * SLOT;
    // ---- partial scores over this wave's k range, two 16-row tiles ----
    f32x4 st0 = f32x4{0.f, 0.f, 0.f, 0.f}, st1 = st0;
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {
      const int s2 = wave * KW + kk;
      const V8 a0 = *reinterpret_cast<const V8*>(slot + gimg32<D>(li, 32 * s2 + 8 * g));
      const V8 a1 = *reinterpret_cast<const V8*>(slot + gimg32<D>(16 + li, 32 * s2 + 8 * g));
      st0 = mfma16(a0, uh[kk], st0);
      st0 = mfma16(a0, ul[kk], st0);
      st1 = mfma16(a1, uh[kk], st1);
      st1 = mfma16(a1, ul[kk], st1);
    }
    // C[row 4g + i (+16)][head li] -> red[wave][row][head]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lds_st32(red + (wave * 32 + 4 * g + i) * 16 + li, st0[i]);
      lds_st32(red + (wave * 32 + 16 + 4 * g + i) * 16 + li, st1[i]);
    }
    lds_fence_barrier();
    // ---- online softmax: head hh, rows 2 tr, 2 tr + 1 ----
    {
      const int j0 = row_begin + 32 * sub;
      float sv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int jr = 2 * tr + u;
        float sc = ((red[(0 * 32 + jr) * 16 + hh] + red[(1 * 32 + jr) * 16 + hh]) + red[(2 * 32 + jr) * 16 + hh]) +
                   red[(3 * 32 + jr) * 16 + hh];
        const int jl = 32 * sub + jr;  // row within the chunk
        const bool ok = ((vm[jl >> 6] >> (jl & 63)) & 1ull) && hh < H;
        sv[u] = ok ? sc : GF_NEG_INF;
      }
      float mx = fmaxf(sv[0], sv[1]);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 16));
      const float m_new = fmaxf(m_run, mx);
      const float mu = m_new == GF_NEG_INF ? 0.f : m_new;
      float ls = 0.f, lsd = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int jr = 2 * tr + u;
        float pv = __expf(sv[u] - mu);
        ls += pv;
        if (dr.thresh) {
          pv *= attn_keep_scale(dr, drow, Lp, j0 + jr);
          lsd += pv;
        }
        lds_st16(pimg + (jr * 16 + hh) * 2, (uint32_t)__builtin_bit_cast(uint16_t, (E)pv));
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        ls += __shfl_xor(ls, o, 16);
        lsd += __shfl_xor(lsd, o, 16);
      }
      const float a = __expf(m_run - mu);  // 0 when m_run = -inf
      l_run = l_run * a + ls;
      ld_run = ld_run * a + lsd;
      m_run = m_new;
      if (tr == 0) lds_st32(alpha_s + hh, a);
    }
    lds_fence_barrier();
    // ---- W[head][c] = alpha W + sum_j p[j][head] h[j][c] (K = 32 rows) ----
    float al[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) al[q] = alpha_s[4 * g + q];
    V8 pa;
    {
      const int rb = 8 * g + q4;
      const V4 v0 = tr_read_ga<E>(pimg + (rb * 16 + 4 * p4) * 2);
      const V4 v1 = tr_read_ga<E>(pimg + ((rb + 4) * 16 + 4 * p4) * 2);
      tr_wait();
      pa = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
    constexpr int PB = nmt % 3 == 0 ? 3 : (nmt % 2 == 0 ? 2 : 1);
#pragma unroll
    for (int i0 = 0; i0 < nmt; i0 += PB) {
      V4 hv[PB][2];
#pragma unroll
      for (int ii = 0; ii < PB; ++ii) {
        const int col = (wave * nmt + i0 + ii) * 16 + 4 * p4;
        const int rb = 8 * g + q4;
        hv[ii][0] = tr_read_ga<E>(slot + gimg32<D>(rb, col));
        hv[ii][1] = tr_read_ga<E>(slot + gimg32<D>(rb + 4, col));
      }
      tr_wait();
#pragma unroll
      for (int ii = 0; ii < PB; ++ii) {
        const int i = i0 + ii;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] *= al[q];
        const V4 v0 = hv[ii][0], v1 = hv[ii][1];
        acc[i] = mfma16(pa, V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]}, acc[i]);
      }
    }
    // every wave is done with this slot, pimg and alpha before the next iteration's DMA / stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the (unused) tail DMAs land before the stores / exit
  if (tr == 0 && hh < GF_HP) {
    ws.m[((int64_t)r * nch + ch) * GF_HP + hh] = m_run;
    ws.l[((int64_t)r * nch + ch) * GF_HP + hh] = l_run;
    if (dr.thresh) ws.ld[((int64_t)r * nch + ch) * GF_HP + hh] = ld_run;
  }
  float* wout = ws.w + ((int64_t)r * nch + ch) * GF_HP * D;
#pragma unroll
  for (int i = 0; i < nmt; ++i) {
    const int c0 = (wave * nmt + i) * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < H) wout[(int64_t)(4 * g + q) * D + c0 + li] = acc[i][q];
  }
}

// Single-buffered form for D not a multiple of 128 (one 64-row DMA, then compute).
template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_partial_bf16_1(int Lp, int gmax, int chr,
                                                             const E* __restrict__ hs, int ldh,
                                                             const uint8_t* __restrict__ flags,
                                                             const int32_t* __restrict__ gidx,
                                                             GfoldWs ws, int H, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  constexpr int nmt = D >> 6;  // 16-column tiles of W per wave (D/16 tiles over 4 waves)
  const int ch = blockIdx.x, r = blockIdx.y, nch = gridDim.x;
  if (gidx[r] < 0) return;
  const int b = r / gmax;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int q4 = li >> 2, p4 = li & 3;
  // u fragments (B operand of S^T = H.U^T): hi and lo planes, issued before the first DMA wait
  V8 uh[NK], ul[NK];
  {
    const E* uhi = reinterpret_cast<const E*>(ws.u16) + ((int64_t)r * 2 * GF_HP + li) * D + 8 * g;
    const E* ulo = uhi + (int64_t)GF_HP * D;
#pragma unroll
    for (int s = 0; s < NK; ++s) {  // heads >= H: zero scores (their u rows are not written)
      uh[s] = li < H ? *reinterpret_cast<const V8*>(uhi + 32 * s) : V8{};
      ul[s] = li < H ? *reinterpret_cast<const V8*>(ulo + 32 * s) : V8{};
    }
  }
  char* pimg = smem + nseg * 64 * 128;                         // P [64 rows][16 heads] bf16
  float* red = reinterpret_cast<float*>(pimg + 64 * 16 * 2);    // [max 4x16][sum 4x16][m 16][alpha 16]
  float* m_run = red + 128;
  float* alpha_s = red + 144;
  const E* hb = hs + (int64_t)b * Lp * ldh;
  if (threadIdx.x < 16) m_run[threadIdx.x] = GF_NEG_INF;
  float l_run = 0.f, ld_run = 0.f;  // per head li (valid in wave 0, g == 0)
  const uint64_t drow = ((uint64_t)b * H + li) * Lp + (uint64_t)max(gidx[r], 0);  // dropout mask row
  f32x4 acc[nmt];
#pragma unroll
  for (int i = 0; i < nmt; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int row_begin = ch * chr;
  const int row_end = min(row_begin + chr, Lp);
  for (int j0 = row_begin; j0 < row_end; j0 += 64) {
    __syncthreads();  // previous sub-chunk's LDS reads are done
    for (int p = wave; p < nseg * 8; p += 4) {
      const int seg = p >> 3, row = (p & 7) * 8 + (lane >> 3);
      const int chk = (lane & 7) ^ (row & 7);
      const int jr = min(j0 + row, Lp - 1);
      glds16(reinterpret_cast<const char*>(hb) + (uint32_t)((jr * ldh + seg * 64 + chk * 8) * (int)sizeof(E)),
             smem + (seg * 64 + (p & 7) * 8) * 128);
    }
    wait_vmcnt0();
    __syncthreads();

    // S^T[j = 16*wave + 4g + q][head = li]
    f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
    const int arow = 16 * wave + li;
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      const V8 a = *reinterpret_cast<const V8*>(smem + gimg(arow, 32 * s + 8 * g));
      st = mfma16(a, uh[s], st);
      st = mfma16(a, ul[s], st);
    }
    float mx = GF_NEG_INF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + 16 * wave + 4 * g + q;
      const bool ok = j < Lp && flags[(int64_t)b * Lp + j] != 0;
      st[q] = ok ? st[q] : GF_NEG_INF;
      mx = fmaxf(mx, st[q]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (g == 0) red[wave * 16 + li] = mx;
    __syncthreads();
    const float m_old = m_run[li];
    const float m_new = fmaxf(m_old, fmaxf(fmaxf(red[li], red[16 + li]), fmaxf(red[32 + li], red[48 + li])));
    const float mu = (m_new == GF_NEG_INF) ? 0.f : m_new;
    float ls = 0.f, lsd = 0.f;
    E* pt = reinterpret_cast<E*>(pimg);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p = __expf(st[q] - mu);
      ls += p;
      if (dr.thresh) {  // TF:1036-1037: W and the value-bias weight use the dropped probabilities
        p *= attn_keep_scale(dr, drow, Lp, j0 + 16 * wave + 4 * g + q);
        lsd += p;
      }
      pt[(16 * wave + 4 * g + q) * 16 + li] = (E)p;
    }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    if (g == 0) red[64 + wave * 16 + li] = ls;
    if (dr.thresh) {
      lsd += __shfl_xor(lsd, 16, 64);
      lsd += __shfl_xor(lsd, 32, 64);
      if (g == 0) red[GF_RED_LD + wave * 16 + li] = lsd;
    }
    __syncthreads();  // P, sums and every wave's read of m_run are done
    if (wave == 0 && g == 0) {
      const float a = __expf(m_old - mu);  // 0 when m_old = -inf
      l_run = l_run * a + red[64 + li] + red[80 + li] + red[96 + li] + red[112 + li];
      if (dr.thresh)
        ld_run = ld_run * a + red[GF_RED_LD + li] + red[GF_RED_LD + 16 + li] + red[GF_RED_LD + 32 + li] +
                 red[GF_RED_LD + 48 + li];
      alpha_s[li] = a;
      m_run[li] = m_new;
    }
    __syncthreads();
    // rescale W rows (head 4g + q) by alpha, then W[head][c] += sum_j p[j][head] h[j][c]
    float al[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) al[q] = alpha_s[4 * g + q];
    V8 pa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int rb = 32 * s + 8 * g + q4;
      const V4 v0 = tr_read_g<E>(pimg + (rb * 16 + 4 * p4) * 2);
      const V4 v1 = tr_read_g<E>(pimg + ((rb + 4) * 16 + 4 * p4) * 2);
      pa[s] = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
#pragma unroll
    for (int i = 0; i < nmt; ++i) {
      const int col = (wave * nmt + i) * 16 + 4 * p4;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[i][q] *= al[q];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int rb = 32 * s + 8 * g + q4;
        const V4 v0 = tr_read_g<E>(smem + gimg(rb, col));
        const V4 v1 = tr_read_g<E>(smem + gimg(rb + 4, col));
        const V8 hb8 = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        acc[i] = mfma16(pa[s], hb8, acc[i]);
      }
    }
  }
  if (wave == 0 && g == 0) {
    ws.m[((int64_t)r * nch + ch) * GF_HP + li] = m_run[li];
    ws.l[((int64_t)r * nch + ch) * GF_HP + li] = l_run;
    if (dr.thresh) ws.ld[((int64_t)r * nch + ch) * GF_HP + li] = ld_run;
  }
  float* wout = ws.w + ((int64_t)r * nch + ch) * GF_HP * D;
#pragma unroll
  for (int i = 0; i < nmt; ++i) {
    const int c0 = (wave * nmt + i) * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < H) wout[(int64_t)(4 * g + q) * D + c0 + li] = acc[i][q];
  }
}

// ---- fp32 partial (VALU; parity path) ------------------------------------------------------
__global__ void __launch_bounds__(256) k_gfold_partial_f32(int Lp, int D, int H, int gmax,
                                                            const float* __restrict__ hs, int ldh,
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
  const float* ug = ws.u32 + (int64_t)r * H * Dp;
  for (int i = t; i < H * Dp; i += 256) us[i] = ug[i];
  __syncthreads();
  const int j0 = ch * GF_CHF;
  const float* hb = hs + (int64_t)b * Lp * ldh;
  {
    const int jl = t >> 2, hg = t & 3;
    const int j = j0 + jl;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (j < Lp) {
      const float* hr = hb + (int64_t)j * ldh;
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
      if (hh < H) ps[hh * GF_CHF+ jl] = ok ? s[i] : GF_NEG_INF;
    }
  }
  __syncthreads();
  for (int hh = wave; hh < H; hh += 4) {
    const float sv = ps[hh * GF_CHF+ lane];
    const float mx = wave_max(sv);
    const float mu = (mx == GF_NEG_INF) ? 0.f : mx;
    const float p = __expf(sv - mu);
    const float lsum = wave_sum(p);
    ps[hh * GF_CHF+ lane] = p;
    if (lane == 0) {
      ws.m[((int64_t)r * nch + ch) * GF_HP + hh] = mx;
      ws.l[((int64_t)r * nch + ch) * GF_HP + hh] = lsum;
    }
  }
  __syncthreads();
  const int jn = min(GF_CHF, Lp - j0);
  float* wout = ws.w + ((int64_t)r * nch + ch) * D * GF_HP;
  for (int k = t; k < D; k += 256) {
    float acc[GF_HP];
#pragma unroll
    for (int hh = 0; hh < GF_HP; ++hh) acc[hh] = 0.f;
    for (int jl = 0; jl < jn; ++jl) {
      const float x = hb[(int64_t)(j0 + jl) * ldh + k];
#pragma unroll
      for (int hh = 0; hh < GF_HP; ++hh)
        if (hh < H) acc[hh] = fmaf(ps[hh * GF_CHF+ jl], x, acc[hh]);
    }
#pragma unroll
    for (int hh = 0; hh < GF_HP; ++hh)
      if (hh < H) wout[(int64_t)hh * D + k] = acc[hh];
  }
}

// ---- bf16 merge + out on MFMA, 16 global rows per block (few global rows) ---------------------
// grid (H, ceil(R/16)). For the C2 shape (R = 64: one CLS row per sequence) the 64-row kernel
// launches only H blocks and the per-row GEMV kernel re-reads the head's Wvg slice once per row
// (768 blocks x 96 KiB of L2 reads, phases serialised by barriers); here 4 x H blocks each DMA the
// head's slice once, merge the chunk partials of 16 rows with all loads of a chunk in flight
// (thread = row t/16, 4-column groups 4(t%16) + 64j), keep w as hi + lo 16-bit planes in LDS (rows
// padded by 16 B: conflict-free B-operand reads) and wave w computes output columns 16w..16w+15 of
// the 16 rows with v_mfma_f32_16x16x32 (A: the Wvg image, B: the w planes).
template <typename E, int D>
__global__ void __launch_bounds__(256) k_gfold_out16(int Lp, int R, int gmax, int nch,
                                                      const E* __restrict__ wvg, const float* __restrict__ bvg,
                                                      const int32_t* __restrict__ gidx, GfoldWs ws,
                                                      E* __restrict__ out, int ldo, bool drop) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  constexpr int WLD = D + 8;  // w plane row stride (elements)
  E* whi = reinterpret_cast<E*>(smem + D * 128);
  E* wlo = whi + 16 * WLD;
  float* bws = reinterpret_cast<float*>(wlo + 16 * WLD);
  const int h = blockIdx.x, r0 = blockIdx.y * 16;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int g = lane >> 4, li = lane & 15;
  for (int p = wave; p < nseg * 8; p += 4) {
    const int seg = p >> 3, row = (p & 7) * 8 + (lane >> 3);
    const int chk = (lane & 7) ^ (row & 7);
    glds16(wvg + (int64_t)(h * 64 + row) * D + seg * 64 + chk * 8, smem + (seg * 64 + (p & 7) * 8) * 128);
  }
  // ---- merge: w[i] = sum_c exp(m_c - M) w_c / sum_c exp(m_c - M) l_c for row i = t / 16 ----
  const int i = t >> 4, cb = 4 * (t & 15);
  const int r = r0 + i;
  const int pos = r < R ? gidx[r] : -1;
  float4 acc[D / 64];
#pragma unroll
  for (int j = 0; j < D / 64; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the row's 16 threads hold chunk q = t % 16's max / sum (nch <= 16: one round of loads, lane
  // shuffles instead of a load per chunk), then all of a chunk pair's w loads are in flight at once
  float inv = 0.f, bw = 1.f;
  if (pos >= 0) {
    const int q = t & 15;
    const int64_t mo = ((int64_t)r * nch + q) * GF_HP + h;
    const float mq = q < nch ? ws.m[mo] : GF_NEG_INF;
    const float lq = q < nch ? ws.l[mo] : 0.f;
    const float dq = (drop && q < nch) ? ws.ld[mo] : 0.f;
    float mx = mq;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 16));
    const float scq = mq == GF_NEG_INF ? 0.f : __expf(mq - mx);
    float lsum = scq * lq, dsum = scq * dq;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      lsum += __shfl_xor(lsum, o, 16);
      dsum += __shfl_xor(dsum, o, 16);
    }
    inv = lsum > 0.f ? 1.0f / lsum : 0.f;
    bw = drop ? dsum * inv : 1.f;
    const float scn = scq * inv;
    const float* wrow = ws.w + ((int64_t)r * nch * GF_HP + h) * D + cb;
    for (int c = 0; c < nch; c += 2) {
      float4 x0[D / 64], x1[D / 64];
      const bool two = c + 1 < nch;
#pragma unroll
      for (int j = 0; j < D / 64; ++j) {
        x0[j] = *reinterpret_cast<const float4*>(wrow + (int64_t)c * GF_HP * D + 64 * j);
        x1[j] = two ? *reinterpret_cast<const float4*>(wrow + (int64_t)(c + 1) * GF_HP * D + 64 * j)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const float s0 = __shfl(scn, c, 16), s1 = two ? __shfl(scn, c + 1, 16) : 0.f;
#pragma unroll
      for (int j = 0; j < D / 64; ++j) {
        acc[j].x = fmaf(s1, x1[j].x, fmaf(s0, x0[j].x, acc[j].x));
        acc[j].y = fmaf(s1, x1[j].y, fmaf(s0, x0[j].y, acc[j].y));
        acc[j].z = fmaf(s1, x1[j].z, fmaf(s0, x0[j].z, acc[j].z));
        acc[j].w = fmaf(s1, x1[j].w, fmaf(s0, x0[j].w, acc[j].w));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < D / 64; ++j) {
    const float v[4] = {acc[j].x, acc[j].y, acc[j].z, acc[j].w};
    V4 vh, vl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      vh[k] = (E)v[k];
      vl[k] = (E)(v[k] - (float)vh[k]);
    }
    *reinterpret_cast<V4*>(whi + i * WLD + cb + 64 * j) = vh;
    *reinterpret_cast<V4*>(wlo + i * WLD + cb + 64 * j) = vl;
  }
  if ((t & 15) == 0) bws[i] = bw;
  wait_vmcnt0();
  __syncthreads();
  // ---- out[row li][16 wave + 4g + k] = Wvg_h[16 wave + 4g + k] . w[li] + bvg ----
  f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int s = 0; s < NK; ++s) {
    const V8 wa = *reinterpret_cast<const V8*>(smem + gimg(16 * wave + li, 32 * s + 8 * g));
    const V8 bh = *reinterpret_cast<const V8*>(whi + li * WLD + 32 * s + 8 * g);
    const V8 bl = *reinterpret_cast<const V8*>(wlo + li * WLD + 32 * s + 8 * g);
    o = mfma16(wa, bh, o);
    o = mfma16(wa, bl, o);
  }
  const int ro = r0 + li;
  const int po = ro < R ? gidx[ro] : -1;
  if (po >= 0) {
    const float bwr = bws[li];
    const int d0 = h * 64 + 16 * wave + 4 * g;
    V4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (E)(o[k] + (drop ? bvg[d0 + k] * bwr : bvg[d0 + k]));
    *reinterpret_cast<V4*>(out + ((int64_t)(ro / gmax) * Lp + po) * ldo + d0) = v;
  }
}

// ---- merge chunks + out = Wvg_h w_h + bvg_h -------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) k_gfold_out(int Lp, int D, int gmax, int nch,
                                                    const T* __restrict__ wvg,
                                                    const float* __restrict__ bvg,
                                                    const int32_t* __restrict__ gidx, GfoldWs ws,
                                                    T* __restrict__ out, int ldo, bool drop) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];  // D floats + nch scales
  float* scl = wsm + D;
  __shared__ float lsum_s, dsum_s;
  const int h = blockIdx.x, r = blockIdx.y;
  const int pos = gidx[r];
  if (pos < 0) return;
  const int b = r / gmax;
  const int t = threadIdx.x;
  if (t < 64) {
    float mx = GF_NEG_INF;
    for (int c = t; c < nch; c += 64) mx = fmaxf(mx, ws.m[((int64_t)r * nch + c) * GF_HP + h]);
    mx = wave_max(mx);
    float ls = 0.f, ds = 0.f;
    for (int c = t; c < nch; c += 64) {
      const float mc = ws.m[((int64_t)r * nch + c) * GF_HP + h];
      const float sc = (mc == GF_NEG_INF) ? 0.f : __expf(mc - mx);
      scl[c] = sc;
      ls += sc * ws.l[((int64_t)r * nch + c) * GF_HP + h];
      if (drop) ds += sc * ws.ld[((int64_t)r * nch + c) * GF_HP + h];
    }
    ls = wave_sum(ls);
    if (drop) ds = wave_sum(ds);
    if (t == 0) {
      lsum_s = ls;
      dsum_s = ds;
    }
  }
  __syncthreads();
  const float inv = lsum_s > 0.f ? 1.0f / lsum_s : 0.f;
  const float bw = drop ? dsum_s * inv : 1.f;  // value-bias weight sum_j p'_j (see k_gfold_out_mfma)
  for (int k = t; k < D; k += 256) {
    float a = 0.f;
    for (int c = 0; c < nch; ++c) a = fmaf(scl[c], ws.w[(((int64_t)r * nch + c) * GF_HP + h) * D + k], a);
    wsm[k] = a * inv;
  }
  __syncthreads();
  // GEMV out[d] = Wvg_h[d, :] . w: 4 threads per output row d (64 rows), each a quarter of the
  // row in interleaved 8-element vectors, all loads issued up front; partial sums via shuffles
  {
    const int d = t >> 2, part = t & 3;
    const T* wr = wvg + (int64_t)(h * 64 + d) * D;
    float a = 0.f;
    for (int k = 8 * part; k < D; k += 32) {
      float x[8];
      load4(wr + k, x);
      load4(wr + k + 4, x + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) a = fmaf(x[i], wsm[k + i], a);
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (part == 0)
      out[((int64_t)b * Lp + pos) * ldo + h * 64 + d] = from_f32<T>(a + (drop ? bvg[h * 64 + d] * bw : bvg[h * 64 + d]));
  }
}

}  // namespace rf

using namespace rf;

extern "C" size_t rf_global_fold_workspace(int B, int Lp, int D, int H, int gmax) {
  if (B <= 0 || gmax <= 0 || Lp <= 0) return 0;
  const int nch = (Lp + GF_CHF - 1) / GF_CHF;  // the larger chunk count of the two paths
  return gfold_bytes(B * gmax, nch, H, D);
}

// The 64-row MFMA kernels for qg/u and out amortise each head's weight slice over 64 global rows
// but launch only H * R/64 blocks; qg/u splits u's columns over up to 4 blocks and wins at any
// R, while for out below a few hundred global rows (one CLS row per 1024-token sequence, C2)
// the per-row GEMV kernel fills the chip better (tools/gfold_bench.py: C2 R=64 out 14.5 vs
// 45 us; catalog R=4096 qu+out 970 vs 155 us). Knob gfold_path (1 GEMV, 2 MFMA) forces one.
static bool gfold_use_mfma(int R, bool qu) {
  if (g_knob[KNOB_GFOLD_PATH] == 1) return false;
  if (g_knob[KNOB_GFOLD_PATH] == 2) return true;
  return qu || R >= 256;  // qg/u: MFMA with a column split wins at any R (C2: 20 -> 12.5 us)
}

// partial + out stages of the 16-bit path (bf16 / fp16 operands)
template <typename E>
static int fold_partial_out16(int B, int Lp, int D, int H, const void* h, int ldh, const void* wvg,
                              const float* bvg, const uint8_t* flags, const int32_t* gidx, int gmax, GfoldWs ws,
                              int nch, int chr, void* out, int ld_out, hipStream_t s, bool do_partial,
                              bool do_out, AttnDrop dr) {
  const int R = B * gmax;
  const size_t lds_o = (size_t)(D + nch) * sizeof(float);
    const size_t lds_p = (size_t)(D / 64) * 64 * 128 + 64 * 16 * 2 + GF_RED_FLOATS * sizeof(float);
    const size_t lds_r = (size_t)3 * 32 * D * 2 + 4 * 32 * 16 * 4 + 32 * 16 * 2 + 16 * 4;
    RF_REQUIRE(lds_p <= 160 * 1024, "rf_global_attn_fold: D too large for LDS");
#define GP_(DD)                                                                                 \
  case DD:                                                                                      \
    if (DD % 128 == 0 && DD <= 768 && (Lp <= 128 || g_knob[KNOB_GFOLD_PATH] == 4) && g_knob[KNOB_GFOLD_PATH] != 3) {                \
      (void)hipFuncSetAttribute((const void*)k_gfold_partial_ring<E, DD>,                          \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_r);        \
      k_gfold_partial_ring<E, DD><<<dim3(nch, R), 256, lds_r, s>>>(Lp, gmax, chr, (const E*)h, ldh,  \
                                                                flags, gidx, ws, H, dr);        \
    } else if (DD % 128 == 0) {                                                                 \
      const size_t lds_pu = lds_p + (DD <= 768 ? (size_t)2 * (DD / 32) * 1024 : 0); /* u image */     \
      (void)hipFuncSetAttribute((const void*)k_gfold_partial_bf16<E, DD>,                          \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pu);       \
      k_gfold_partial_bf16<E, DD><<<dim3(nch, R), 256, lds_pu, s>>>(Lp, gmax, chr, (const E*)h, ldh, \
                                                                flags, gidx, ws, H, dr);        \
    } else {                                                                                    \
      (void)hipFuncSetAttribute((const void*)k_gfold_partial_bf16_1<E, DD>,                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_p);        \
      k_gfold_partial_bf16_1<E, DD><<<dim3(nch, R), 256, lds_p, s>>>(Lp, gmax, chr, (const E*)h, ldh, \
                                                                  flags, gidx, ws, H, dr);      \
    }                                                                                           \
    break;
    if (do_partial) switch (D) {
      GP_(64) GP_(128) GP_(192) GP_(256) GP_(384) GP_(512) GP_(768) GP_(1024)
      default:
        RF_REQUIRE(false, "rf_global_attn_fold(16-bit): unsupported hidden size %d", D);
    }
#undef GP_
    const size_t lds_16 = (size_t)D * 128 + (size_t)2 * 16 * (D + 8) * 2 + 16 * 4;
    if (!do_out) {
    } else if (ld_out % 4 == 0 && !gfold_use_mfma(R, false) && g_knob[KNOB_GFOLD_PATH] != 1 && nch <= 16 &&
               (D == 64 || D == 128 || D == 192 || D == 256 || D == 384 || D == 512 || D == 768) &&
               lds_16 <= 160 * 1024) {
#define G16_(DD)                                                                                \
  case DD:                                                                                      \
    (void)hipFuncSetAttribute((const void*)k_gfold_out16<E, DD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              (int)lds_16);                                                     \
    k_gfold_out16<E, DD><<<dim3(H, (R + 15) / 16), 256, lds_16, s>>>(Lp, R, gmax, nch, (const E*)wvg, bvg, gidx, \
                                                                  ws, (E*)out, ld_out, dr.thresh != 0); \
    break;
      switch (D) { G16_(64) G16_(128) G16_(192) G16_(256) G16_(384) G16_(512) G16_(768) default: break; }
#undef G16_
    } else if (ld_out % 4 == 0 && gfold_use_mfma(R, false)) {
      const size_t lds_w = (size_t)D * 128;
#define GO_(DD)                                                                                 \
  case DD:                                                                                      \
    (void)hipFuncSetAttribute((const void*)k_gfold_out_mfma<E, DD>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_w);          \
    k_gfold_out_mfma<E, DD><<<dim3(H, (R + 63) / 64), 256, lds_w, s>>>(Lp, R, gmax, nch, (const E*)wvg, \
                                                                   bvg, gidx, ws, (E*)out, ld_out, \
                                                                   dr.thresh != 0);                 \
    break;
      switch (D) { GO_(64) GO_(128) GO_(192) GO_(256) GO_(384) GO_(512) GO_(768) GO_(1024) }
#undef GO_
    } else {
      k_gfold_out<E><<<dim3(H, R), 256, lds_o, s>>>(Lp, D, gmax, nch, (const E*)wvg, bvg, gidx, ws,
                                                        (E*)out, ld_out, dr.thresh != 0);
    }
  return RF_OK;
}

// partial + out stages shared by both entry points (u already in the workspace)
static int fold_partial_out(int dtype, int B, int Lp, int D, int H, const void* h, int ldh, const void* wvg,
                            const float* bvg, const uint8_t* flags, const int32_t* gidx, int gmax,
                            GfoldWs ws, int nch, int chr, void* out, int ld_out, hipStream_t s, bool do_partial = true,
                            bool do_out = true, AttnDrop dr = AttnDrop{0, 0, 1.f}) {
  const int R = B * gmax;
  const size_t lds_o = (size_t)(D + nch) * sizeof(float);
  if (dtype == RF_BF16 || dtype == RF_F16) {
    return dtype == RF_F16
               ? fold_partial_out16<f16>(B, Lp, D, H, h, ldh, wvg, bvg, flags, gidx, gmax, ws, nch, chr, out, ld_out, s,
                                         do_partial, do_out, dr)
               : fold_partial_out16<bf16>(B, Lp, D, H, h, ldh, wvg, bvg, flags, gidx, gmax, ws, nch, chr, out, ld_out, s,
                                          do_partial, do_out, dr);
  } else {
    const size_t lds_p = (size_t)(H * (D + 4) + H * GF_CHF) * sizeof(float);
    RF_REQUIRE(lds_p <= 160 * 1024, "rf_global_attn_fold: D too large for LDS");
    (void)hipFuncSetAttribute((const void*)k_gfold_partial_f32,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_p);
    if (do_partial)
      k_gfold_partial_f32<<<dim3(nch, R), 256, lds_p, s>>>(Lp, D, H, gmax, (const float*)h, ldh, flags, gidx, ws);
    if (do_out)
      k_gfold_out<float><<<dim3(H, R), 256, lds_o, s>>>(Lp, D, gmax, nch, (const float*)wvg, bvg, gidx, ws,
                                                       (float*)out, ld_out, false);
  }
  return RF_OK;
}

extern "C" int rf_global_attn_fold_fwd_stage(int stage, int dtype, int B, int Lp, int D, int H, const void* qg,
                                             int ld_qg, const void* h, int ldh, const void* wkg,
                                             const float* bkg, const void* wvg, const float* bvg,
                                             const uint8_t* flags, const int32_t* gidx, int gmax,
                                             void* workspace, void* out, int ld_out, float p_drop,
                                             uint64_t seed, rf_stream_t stream) {
  (void)bkg;  // softmax-invariant (see header comment)
  RF_REQUIRE(stage >= 1 && stage <= 3, "rf_global_attn_fold_fwd_stage: stage %d not in 1..3", stage);
  RF_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "rf_global_attn_fold_fwd: p_drop %f not in [0, 1)", p_drop);
  RF_REQUIRE(p_drop == 0.f || dtype != RF_F32, "rf_global_attn_fold_fwd: attention dropout needs 16-bit operands");
  const AttnDrop dr{seed, drop_thresh(p_drop), p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.f, g_seed_dev};
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && H > 0, "rf_global_attn_fold_fwd: bad shape");
  RF_REQUIRE(D == H * 64, "rf_global_attn_fold_fwd: D=%d must be H*64", D);
  RF_REQUIRE(H <= GF_HP, "rf_global_attn_fold_fwd: at most %d heads", GF_HP);
  RF_REQUIRE(ldh >= D && ld_qg >= D && ld_out >= D, "rf_global_attn_fold_fwd: dims");
  RF_REQUIRE((int64_t)Lp * ldh * 4 < 0x7FFFFFFF, "rf_global_attn_fold: one sequence's rows must span < 2 GiB");
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16 || dtype == RF_F32, "rf_global_attn_fold_fwd: bad dtype %d", dtype);
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(workspace && gidx && flags, "rf_global_attn_fold_fwd: null workspace/gidx/flags");
  RF_REQUIRE(dtype == RF_F32 || ldh % 8 == 0, "rf_global_attn_fold_fwd(16-bit): ldh must be a multiple of 8");
  RF_REQUIRE(dtype != RF_F32 || ldh % 4 == 0, "rf_global_attn_fold_fwd(f32): ldh must be a multiple of 4");
  const int R = B * gmax;
  const int chr = gfold_chunk(dtype, R, Lp);
  const int nch = (Lp + chr - 1) / chr;
  GfoldWs ws = gfold_carve(workspace, R, nch, H, D);
  hipStream_t s = as_stream(stream);
  if (!(stage & 1)) {
  } else if (dtype == RF_BF16)
    k_gfold_u<bf16><<<dim3(GF_HP, R), 192, 0, s>>>(D, H, R, (const bf16*)qg, ld_qg, (const bf16*)wkg, gidx,
                                                    ws, true);
  else if (dtype == RF_F16)
    k_gfold_u<f16><<<dim3(GF_HP, R), 192, 0, s>>>(D, H, R, (const f16*)qg, ld_qg, (const f16*)wkg, gidx, ws, true);
  else
    k_gfold_u<float><<<dim3(H, R), 192, 0, s>>>(D, H, R, (const float*)qg, ld_qg, (const float*)wkg, gidx,
                                                 ws, false);
  const int rc =
      fold_partial_out(dtype, B, Lp, D, H, h, ldh, wvg, bvg, flags, gidx, gmax, ws, nch, chr, out, ld_out, s,
                       (stage & 1) != 0, (stage & 2) != 0, dr);
  if (rc != RF_OK) return rc;
  RF_LAUNCH_CHECK("rf_global_attn_fold_fwd");
}

extern "C" int rf_global_attn_fold_fwd_drop(int dtype, int B, int Lp, int D, int H, const void* qg,
                                            int ld_qg, const void* h, int ldh, const void* wkg,
                                            const float* bkg, const void* wvg, const float* bvg,
                                            const uint8_t* flags, const int32_t* gidx, int gmax,
                                            void* workspace, void* out, int ld_out, float p_drop,
                                            uint64_t seed, rf_stream_t stream) {
  return rf_global_attn_fold_fwd_stage(3, dtype, B, Lp, D, H, qg, ld_qg, h, ldh, wkg, bkg, wvg, bvg, flags, gidx,
                                       gmax, workspace, out, ld_out, p_drop, seed, stream);
}

extern "C" int rf_global_attn_fold_fwd(int dtype, int B, int Lp, int D, int H, const void* qg, int ld_qg,
                                       const void* h, int ldh, const void* wkg, const float* bkg, const void* wvg,
                                       const float* bvg, const uint8_t* flags, const int32_t* gidx, int gmax,
                                       void* workspace, void* out, int ld_out, rf_stream_t stream) {
  return rf_global_attn_fold_fwd_drop(dtype, B, Lp, D, H, qg, ld_qg, h, ldh, wkg, bkg, wvg, bvg, flags, gidx, gmax,
                                      workspace, out, ld_out, 0.f, 0, stream);
}

// Attention-dropout scale of the global query rows (TF:1036-1037) for the training backward:
// z[((b H + h) gmax + g) Lp + l] = keep(row (b H + h) Lp + gidx[b][g], key l) / (1 - p); an empty
// slot (gidx < 0) uses position 0 (its gradient is zero). recformer_amd/train.py _global_keep.
__global__ void k_attn_global_keep(int B, int H, int Lp, int gmax, const int32_t* __restrict__ gidx, AttnDrop dr,
                                   float* __restrict__ z) {
  drop_resolve(dr);  // device step counter (captured training steps)
  const int bhg = blockIdx.y;  // (b H + h) gmax + g
  const int g = bhg % gmax, bh = bhg / gmax, b = bh / H;
  const uint64_t row = (uint64_t)bh * Lp + (uint64_t)max(gidx[b * gmax + g], 0);
  for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < Lp; l += gridDim.x * blockDim.x)
    z[(int64_t)bhg * Lp + l] = attn_keep_scale(dr, row, Lp, l);
}

extern "C" int rf_attn_global_keep(int B, int H, int Lp, const int32_t* gidx, int gmax, float p_drop, uint64_t seed,
                                   float* z, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && H > 0 && Lp >= 0 && gmax >= 0, "rf_attn_global_keep: bad shape");
  RF_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "rf_attn_global_keep: p_drop %f not in [0, 1)", p_drop);
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(gidx && z, "rf_attn_global_keep: null pointer");
  const AttnDrop dr{seed, drop_thresh(p_drop), p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.f, g_seed_dev};
  k_attn_global_keep<<<dim3((Lp + 255) / 256, B * H * gmax), 256, 0, as_stream(stream)>>>(B, H, Lp, gmax, gidx, dr, z);
  RF_LAUNCH_CHECK("rf_attn_global_keep");
}

extern "C" int rf_global_attn_fold_h_stage(int stage, int dtype, int B, int Lp, int D, int H, const void* h,
                                           int ldh, const void* wqg, const float* bqg, float q_scale,
                                           const void* wkg, const float* bkg, const void* wvg, const float* bvg,
                                           const uint8_t* flags, const int32_t* gidx, int gmax,
                                           void* workspace, void* out, int ld_out, rf_stream_t stream) {
  (void)bkg;
  RF_REQUIRE(stage >= 1 && stage <= 3, "rf_global_attn_fold_h_stage: stage %d not in 1..3", stage);
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && H > 0, "rf_global_attn_fold_h: bad shape");
  RF_REQUIRE(D == H * 64 && D <= 1024, "rf_global_attn_fold_h: D=%d must be H*64 <= 1024", D);
  RF_REQUIRE(H <= GF_HP, "rf_global_attn_fold_h: at most %d heads", GF_HP);
  RF_REQUIRE(ldh >= D && ld_out >= D, "rf_global_attn_fold_h: dims");
  RF_REQUIRE((int64_t)Lp * ldh * 4 < 0x7FFFFFFF, "rf_global_attn_fold: one sequence's rows must span < 2 GiB");
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16 || dtype == RF_F32, "rf_global_attn_fold_h: bad dtype %d", dtype);
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(workspace && gidx && flags && wqg && bqg, "rf_global_attn_fold_h: null pointer");
  RF_REQUIRE(dtype == RF_F32 || ldh % 8 == 0, "rf_global_attn_fold_h(16-bit): ldh must be a multiple of 8");
  RF_REQUIRE(dtype != RF_F32 || ldh % 4 == 0, "rf_global_attn_fold_h(f32): ldh must be a multiple of 4");
  const int R = B * gmax;
  // fixed chunks here (inference): a sequence's result does not depend on the batch it is in (knob
  // gfold_chunk: 64 / 128 / 256 rows, at most 16 chunks per sequence; 0 = GF_CH)
  int chr = dtype != RF_F32 ? GF_CH : GF_CHF;
  if (dtype != RF_F32 && (g_knob[KNOB_GFOLD_CHUNK] == 64 || g_knob[KNOB_GFOLD_CHUNK] == 128)) {
    chr = g_knob[KNOB_GFOLD_CHUNK];
    while ((Lp + chr - 1) / chr > 16 && chr < GF_CH) chr *= 2;
  }
  const int nch = (Lp + chr - 1) / chr;
  GfoldWs ws = gfold_carve(workspace, R, nch, H, D);
  hipStream_t s = as_stream(stream);
  if (!(stage & 1)) {
  } else if (dtype != RF_F32 && gfold_use_mfma(R, true)) {
    RF_REQUIRE(D % 64 == 0 && D <= 1024, "rf_global_attn_fold_h: D=%d", D);
    // few row tiles: split u's columns over more blocks (each recomputes its tile's qg)
    int qsplit = 1;
    // C2 (R = 64): 8 column splits 51.3 vs 52.9 us for 4 (tools/gfold_bench.py)
    const int qmax = std::max(1, g_knob[KNOB_GFOLD_QSPLIT]);
    while (qsplit < qmax && H * ((R + 63) / 64) * qsplit < 32 * qmax && (D / 16) % (2 * qsplit) == 0) qsplit *= 2;
    // Wkg slice: at most ceil(cols / 64) + 1 segments of 8 KiB; its own region when it fits
    const int nslice = std::min(D / 64, (D / qsplit + 63) / 64 + 1);
    const int sep = (size_t)D * 128 + (size_t)nslice * 8192 + 4 * 2048 <= 160 * 1024 ? 1 : 0;
    const size_t lds_q = (size_t)D * 128 + (sep ? (size_t)nslice * 8192 : 0) + 4 * 2048;
#define GQ_(DD)                                                                                   \
  case DD:                                                                                        \
    (void)hipFuncSetAttribute((const void*)k_gfold_qu_mfma<E, DD>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_q);            \
    k_gfold_qu_mfma<E, DD><<<dim3(H, (R + 63) / 64, qsplit), 256, lds_q, s>>>(Lp, R, gmax, (const E*)h, ldh, \
                                                                     (const E*)wqg, bqg, q_scale,  \
                                                                     (const E*)wkg, gidx, ws, sep); \
    break;
    if (dtype == RF_F16) {
      typedef f16 E;
      switch (D) { GQ_(64) GQ_(128) GQ_(192) GQ_(256) GQ_(384) GQ_(512) GQ_(768) GQ_(1024) default: break; }
    } else {
      typedef bf16 E;
      switch (D) { GQ_(64) GQ_(128) GQ_(192) GQ_(256) GQ_(384) GQ_(512) GQ_(768) GQ_(1024) default: break; }
    }
#undef GQ_
  } else if (dtype == RF_BF16)
    k_gfold_qu<bf16><<<dim3(GF_HP, R), 256, 0, s>>>(Lp, D, H, gmax, (const bf16*)h, ldh, (const bf16*)wqg, bqg,
                                                     q_scale, (const bf16*)wkg, gidx, ws, true);
  else if (dtype == RF_F16)
    k_gfold_qu<f16><<<dim3(GF_HP, R), 256, 0, s>>>(Lp, D, H, gmax, (const f16*)h, ldh, (const f16*)wqg, bqg, q_scale,
                                                    (const f16*)wkg, gidx, ws, true);
  else
    k_gfold_qu<float><<<dim3(H, R), 256, 0, s>>>(Lp, D, H, gmax, (const float*)h, ldh, (const float*)wqg, bqg,
                                                  q_scale, (const float*)wkg, gidx, ws, false);
  const int rc = fold_partial_out(dtype, B, Lp, D, H, h, ldh, wvg, bvg, flags, gidx, gmax, ws, nch, chr, out, ld_out,
                                  s, (stage & 1) != 0, (stage & 2) != 0);
  if (rc != RF_OK) return rc;
  RF_LAUNCH_CHECK("rf_global_attn_fold_h_stage");
}

extern "C" int rf_global_attn_fold_h_fwd(int dtype, int B, int Lp, int D, int H, const void* h, int ldh,
                                         const void* wqg, const float* bqg, float q_scale, const void* wkg,
                                         const float* bkg, const void* wvg, const float* bvg,
                                         const uint8_t* flags, const int32_t* gidx, int gmax,
                                         void* workspace, void* out, int ld_out, rf_stream_t stream) {
  return rf_global_attn_fold_h_stage(3, dtype, B, Lp, D, H, h, ldh, wqg, bqg, q_scale, wkg, bkg, wvg, bvg, flags,
                                     gidx, gmax, workspace, out, ld_out, stream);
}


// =====================================================================================================
// Backward of the global rows through the fold algebra (TF:964-1057 under autograd; the closed form of
// recformer_amd/train.py _global_bwd) in ONE pass over h, from the forward's fold workspace (u planes,
// per-chunk softmax statistics and w partials, which the caller keeps between forward and backward).
// Per global row r and head h, with dw_h = Wvg_h^T do_h (given, fp32) and c_h = do_h . bvg_h (dropout):
//   M, L       the merged softmax statistics;  w_h = sum_j p'_j h_j (merged partials);  S'_h = sum_j p'_j
//   Delta_h    = dw_h . w_h + c_h S'_h  (= sum_j p_j dp_j: no pass over h needed for it)
//   s_j = u_h . h_j,  p_j = exp(s_j - M) / L,  p'_j = p_j z_j,  dp_j = (dw_h . h_j + c_h) z_j,
//   ds_j = p_j (dp_j - Delta_h),  du_h = sum_j ds_j h_j,  dh_j = sum_{g, h} (p'_j dw_h + ds_j u_h)
// k_gbwd_prep (R, 16): merges w, S' and the statistics, writes dw as hi + lo 16-bit planes and the
//   dh product's operand [dw_hi ; u_hi] transposed (per column, 32 values: 16 B per MFMA fragment);
// k_gbwd_main (Lp/64, B): one 64-row chunk of one sequence for all of its global rows: the chunk DMA'd
//   once; the s and dp products on MFMA with the reduction over D split by k range across the 4 waves
//   and summed in LDS (the u / dw fragments of a quarter of D fit the registers); the softmax backward
//   per (row, head); du partial = dS^T.H (transposed LDS reads, as the forward's P.H); dh = [p' | ds] .
//   [dw ; u] on MFMA (K = 32 per global row), staged through LDS and stored as whole lines;
// k_gbwd_reduce: du = sum of the chunk partials in chunk order (deterministic).
namespace rf {

constexpr int GB_ROWS = 64;  // rows per k_gbwd_main block
constexpr int GB_GMAX = 4;   // global rows per sequence the kernel takes (more: the torch path)

// Per (global row r, head h). FROM_DOUT (rf_global_fold_bwd_full): dw_h = Wvg_h^T do_h and
// c_h = do_h . bvg_h from the attention output gradient's global row and the weights, else given.
// The chunk statistics are merged by one lane per chunk (nch <= 64) and the per-chunk scales kept in
// LDS, so the w merge issues its chunk loads together instead of one dependent load per chunk.
template <typename E, bool FROM_DOUT>
__global__ void __launch_bounds__(256) k_gbwd_prep(int D, int H, int nch, int Lp, int gmax,
                                                   const int32_t* __restrict__ gidx, GfoldWs ws,
                                                   const float* __restrict__ dw, const float* __restrict__ cb,
                                                   const E* __restrict__ dout, int ldd, const E* __restrict__ wvg,
                                                   const float* __restrict__ bvg, float* __restrict__ cbw, int drop,
                                                   float* __restrict__ wout, float* __restrict__ st,
                                                   E* __restrict__ dwp, E* __restrict__ bt) {
  __shared__ float red[4];
  __shared__ float scs[64];    // per-chunk scale exp(m_c - M) / L
  __shared__ float dos[64];    // do_h (FROM_DOUT)
  __shared__ float stat[4];    // M, 1/L, S', c
  const int r = blockIdx.x, h = blockIdx.y, t = threadIdx.x;
  const int pos = gidx[r];
  const bool live = h < H && pos >= 0;
  if (t < 64) {
    float mc = GF_NEG_INF, lc = 0.f, ldc = 0.f;
    if (live && t < nch) {
      const int64_t o = ((int64_t)r * nch + t) * GF_HP + h;
      mc = ws.m[o];
      lc = ws.l[o];
      if (drop) ldc = ws.ld[o];
    }
    const float M = wave_max(mc);
    const float sc = mc == GF_NEG_INF ? 0.f : __expf(mc - M);
    const float L = wave_sum(sc * lc);
    const float LD = drop ? wave_sum(sc * ldc) : 0.f;
    const float inv = L > 0.f ? 1.0f / L : 0.f;
    if (t < nch) scs[t] = sc * inv;
    if (t == 0) {
      stat[0] = live ? M : 0.f;
      stat[1] = inv;
      stat[2] = live ? (drop ? LD * inv : 1.f) : 0.f;
    }
  } else if (t < 128) {
    float c = 0.f;
    if (FROM_DOUT) {
      const int d = t - 64;
      const float v = live ? to_f32(dout[((int64_t)(r / gmax) * Lp + pos) * ldd + h * 64 + d]) : 0.f;
      dos[d] = v;
      // bvg holds H * 64 values: the padding heads h >= H (the grid covers GF_HP) must not read it (they
      // once did, 4 KiB past the bias at C1's H = 2 — an illegal address whenever the bias sat at the end of
      // a mapped block: the round-4/5 suite fault first blamed on the gradient mailbox)
      if (drop) c = wave_sum(live ? v * bvg[h * 64 + d] : 0.f);
    } else if (live && cb) {
      c = cb[r * GF_HP + h];
    }
    if (t == 64) {
      stat[3] = c;
      if (FROM_DOUT && cbw) cbw[r * GF_HP + h] = c;
    }
  }
  __syncthreads();
  const float inv = stat[1], Sp = stat[2], c = stat[3];
  const E* u16 = reinterpret_cast<const E*>(ws.u16);
  float dsum = 0.f;
  for (int k = t; k < D; k += 256) {
    float wv = 0.f, dv = 0.f;
    E uh = (E)0.f;
    if (live) {
      const float* wp = ws.w + ((int64_t)r * nch * GF_HP + h) * D + k;
#pragma unroll 4
      for (int cc = 0; cc < nch; ++cc) wv += scs[cc] * wp[(int64_t)cc * GF_HP * D];
      if (FROM_DOUT) {
        const E* vp = wvg + (int64_t)(h * 64) * D + k;
#pragma unroll 16
        for (int d = 0; d < 64; ++d) dv = fmaf(dos[d], to_f32(vp[(int64_t)d * D]), dv);
      } else {
        dv = dw[((int64_t)r * GF_HP + h) * D + k];
      }
      uh = u16[((int64_t)r * 2 * GF_HP + h) * D + k];
    }
    wout[((int64_t)r * GF_HP + h) * D + k] = wv;
    dsum += dv * wv;
    const E hi = (E)dv, lo = (E)(dv - (float)hi);
    dwp[((int64_t)r * 2 * GF_HP + h) * D + k] = hi;
    dwp[((int64_t)r * 2 * GF_HP + GF_HP + h) * D + k] = lo;
    bt[((int64_t)r * D + k) * 32 + h] = hi;
    bt[((int64_t)r * D + k) * 32 + 16 + h] = uh;
  }
  dsum = wave_sum(dsum);
  if ((t & 63) == 0) red[t >> 6] = dsum;
  __syncthreads();
  if (t == 0) {
    float* o = st + ((int64_t)r * GF_HP + h) * 4;
    o[0] = stat[0];
    o[1] = inv;
    o[2] = ((red[0] + red[1]) + red[2]) + red[3] + c * Sp;
    o[3] = Sp;
  }
}

template <typename E, int D>
__global__ void __launch_bounds__(256) k_gbwd_main(int Lp, int gmax, int H, const E* __restrict__ hs, int ldh,
                                                   const uint8_t* __restrict__ flags, const int32_t* __restrict__ gidx,
                                                   GfoldWs ws, const E* __restrict__ dwp, const E* __restrict__ bt,
                                                   const float* __restrict__ st, const float* __restrict__ cb,
                                                   float* __restrict__ dupart, E* __restrict__ dh, int lddh,
                                                   AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NK = D / 32;
  constexpr int nseg = D >> 6;
  constexpr int KW = NK / 4;   // k-steps of the s / dp products per wave
  constexpr int nmt = D >> 6;  // du column tiles per wave
  char* himg = smem;
  float* red = reinterpret_cast<float*>(smem + D * 128);                  // [2][4][64][16]
  E* pds = reinterpret_cast<E*>(smem + D * 128 + 2 * 4 * 64 * 16 * 4);    // [GB_GMAX][64][32]
  const int ch = blockIdx.x, b = blockIdx.y, nch2 = gridDim.x;
  const int j0 = ch * GB_ROWS;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int q4 = li >> 2, p4 = li & 3;
  const E* hb = hs + (int64_t)b * Lp * ldh;
  for (int p = wave; p < nseg * 8; p += 4) {
    const int seg = p >> 3, row = (p & 7) * 8 + (lane >> 3);
    const int chk = (lane & 7) ^ (row & 7);
    const int jr = min(j0 + row, Lp - 1);
    glds16(reinterpret_cast<const char*>(hb) + (uint32_t)((jr * ldh + seg * 64 + chk * 8) * (int)sizeof(E)),
           himg + (seg * 64 + (p & 7) * 8) * 128);
  }
  const int jv = j0 + lane;
  const bool okv = jv < Lp && flags[(int64_t)b * Lp + min(jv, Lp - 1)] != 0;
  const unsigned long long vm = __ballot(okv);
  wait_vmcnt0();
  __syncthreads();
  const E* u16 = reinterpret_cast<const E*>(ws.u16);
  int ng = 0;
  for (int gq = 0; gq < gmax; ++gq) {
    const int r = b * gmax + gq;
    const int pos = gidx[r];
    if (pos < 0) continue;
    // ---- s and dp over this wave's k range: S^T[row][head] = h_row . u_head ----
    {
      V8 uhf[KW], ulf[KW], dhf[KW], dlf[KW];
      const E* up = u16 + ((int64_t)r * 2 * GF_HP + li) * D + 8 * g;
      const E* dq = dwp + ((int64_t)r * 2 * GF_HP + li) * D + 8 * g;
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        const int s2 = wave * KW + kk;
        uhf[kk] = *reinterpret_cast<const V8*>(up + 32 * s2);
        ulf[kk] = *reinterpret_cast<const V8*>(up + GF_HP * D + 32 * s2);
        dhf[kk] = *reinterpret_cast<const V8*>(dq + 32 * s2);
        dlf[kk] = *reinterpret_cast<const V8*>(dq + GF_HP * D + 32 * s2);
      }
      f32x4 sa[4], da[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) sa[t] = da[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        const int s2 = wave * KW + kk;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const V8 a = *reinterpret_cast<const V8*>(himg + gimg(16 * t + li, 32 * s2 + 8 * g));
          sa[t] = mfma16(a, uhf[kk], sa[t]);
          sa[t] = mfma16(a, ulf[kk], sa[t]);
          da[t] = mfma16(a, dhf[kk], da[t]);
          da[t] = mfma16(a, dlf[kk], da[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * t + 4 * g + i;
          red[((0 * 4 + wave) * 64 + row) * 16 + li] = sa[t][i];
          red[((1 * 4 + wave) * 64 + row) * 16 + li] = da[t][i];
        }
    }
    __syncthreads();
    // ---- softmax backward per (row, head): thread -> row t/4, heads 4 (t%4) .. +3 ----
    {
      const int jr = threadIdx.x >> 2, h0 = (threadIdx.x & 3) * 4;
      const int j = j0 + jr;
      const bool ok = (vm >> jr) & 1ull;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int hh = h0 + k;
        float s = 0.f, dpv = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          s += red[((0 * 4 + w) * 64 + jr) * 16 + hh];
          dpv += red[((1 * 4 + w) * 64 + jr) * 16 + hh];
        }
        const float* sp = st + ((int64_t)r * GF_HP + hh) * 4;
        const bool live = ok && hh < H;
        const float p = live ? __expf(s - sp[0]) * sp[1] : 0.f;
        const float z = (live && dr.thresh) ? attn_keep_scale(dr, ((uint64_t)b * H + hh) * Lp + pos, Lp, j) : 1.f;
        const float c = cb ? cb[r * GF_HP + hh] : 0.f;
        const float ds = p * ((dpv + c) * z - sp[2]);
        pds[(ng * 64 + jr) * 32 + hh] = (E)(p * z);
        pds[(ng * 64 + jr) * 32 + 16 + hh] = (E)ds;
      }
    }
    __syncthreads();
    // ---- du partial: du[head][col] = sum_j ds[j][head] h_j[col] (the forward's P.H with ds) ----
    {
      const char* pbase = reinterpret_cast<const char*>(pds + ng * 64 * 32);
      V8 pa[2];
      {
        V4 pv[4];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int rb = 32 * s2 + 8 * g + q4;
          pv[2 * s2] = tr_read_ga<E>(pbase + (rb * 32 + 16 + 4 * p4) * 2);
          pv[2 * s2 + 1] = tr_read_ga<E>(pbase + ((rb + 4) * 32 + 16 + 4 * p4) * 2);
        }
        tr_wait();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          pa[s2] = V8{pv[2 * s2][0], pv[2 * s2][1], pv[2 * s2][2], pv[2 * s2][3],
                      pv[2 * s2 + 1][0], pv[2 * s2 + 1][1], pv[2 * s2 + 1][2], pv[2 * s2 + 1][3]};
      }
      float* dout = dupart + ((int64_t)r * nch2 + ch) * GF_HP * D;
#pragma unroll
      for (int i = 0; i < nmt; ++i) {
        const int c0 = (wave * nmt + i) * 16;
        V4 hv[4];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int rb = 32 * s2 + 8 * g + q4;
          hv[2 * s2] = tr_read_ga<E>(himg + gimg(rb, c0 + 4 * p4));
          hv[2 * s2 + 1] = tr_read_ga<E>(himg + gimg(rb + 4, c0 + 4 * p4));
        }
        tr_wait();
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const V4 v0 = hv[2 * s2], v1 = hv[2 * s2 + 1];
          acc = mfma16(pa[s2], V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]}, acc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) dout[(int64_t)(4 * g + q) * D + c0 + li] = acc[q];
      }
    }
    ++ng;
    __syncthreads();  // red is rewritten by the next global row
  }
  // ---- dh[j][col] = sum over the global rows of [p' | ds][j] . [dw ; u][col]; staged in the image ----
  E* stg = reinterpret_cast<E*>(himg);
  constexpr int NT = D / 16;  // column tiles
  for (int cb0 = 0; cb0 < NT; cb0 += 12) {
    f32x4 acc[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int slot = 0;
    for (int gq = 0; gq < gmax; ++gq) {
      const int r = b * gmax + gq;
      if (gidx[r] < 0) continue;
      const V8 a = *reinterpret_cast<const V8*>(pds + (slot * 64 + 16 * wave + li) * 32 + 8 * g);
      const E* bp = bt + ((int64_t)r * D + 16 * cb0 + li) * 32 + 8 * g;
#pragma unroll
      for (int i = 0; i < 12; ++i)
        if (cb0 + i < NT) acc[i] = mfma16(a, *reinterpret_cast<const V8*>(bp + (int64_t)16 * i * 32), acc[i]);
      ++slot;
    }
#pragma unroll
    for (int i = 0; i < 12; ++i)
      if (cb0 + i < NT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) stg[(16 * wave + 4 * g + q) * D + 16 * (cb0 + i) + li] = (E)acc[i][q];
      }
  }
  __syncthreads();
  for (int e = threadIdx.x * 8; e < GB_ROWS * D; e += 256 * 8) {
    const int row = e / D, col = e - row * D;
    if (j0 + row < Lp)
      *reinterpret_cast<V8*>(dh + ((int64_t)b * Lp + j0 + row) * lddh + col) = *reinterpret_cast<const V8*>(stg + e);
  }
}

// du[r][h][col] = sum over the chunks, in chunk order (empty global slots: 0, their partials unwritten)
__global__ void __launch_bounds__(256) k_gbwd_reduce(int R, int D, int nch2, const int32_t* __restrict__ gidx,
                                                     const float* __restrict__ dupart, float* __restrict__ du) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)R * GF_HP * D) return;
  const int64_t r = idx / ((int64_t)GF_HP * D), rem = idx - r * GF_HP * D;
  float s = 0.f;
  if (gidx[r] >= 0)
    for (int c = 0; c < nch2; ++c) s += dupart[(r * nch2 + c) * GF_HP * D + rem];
  du[idx] = s;
}

// dqg / dWkg / dWvg / dbvg / dbkg of the global branch from du, w and S' (rf_global_fold_bwd_full);
// grid R*H + 2*D blocks. Block (r, h) < R*H: dqg[r][h*64+i] = sum_c du[r][h][c] Wkg[h*64+i][c] (four
// threads per output over the row of Wkg). Then one block per output row o of dWkg (which = 0) or
// dWvg (which = 1), h = o / 64, over the global rows (K = R, a few):
//   dWkg[o][c] = sum_r qg[r][o] du[r][h][c],  dWvg[o][c] = sum_r do[r][o] w[r][h][c],
//   dbvg[o] = sum_r do[r][o] S'[r][h],  dbkg[o] = 0 (softmax-invariant); empty slots contribute 0.
template <typename E>
__global__ void __launch_bounds__(256) k_gbwd_post(int D, int H, int Lp, int gmax, int R,
                                                   const int32_t* __restrict__ gidx, const E* __restrict__ dout,
                                                   int ldd, const E* __restrict__ qg, int ldq,
                                                   const E* __restrict__ wkg, const float* __restrict__ du,
                                                   const float* __restrict__ w, const float* __restrict__ st,
                                                   float* __restrict__ dqg, float* __restrict__ dwkg,
                                                   float* __restrict__ dwvg, float* __restrict__ dbvg,
                                                   float* __restrict__ dbkg) {
  __shared__ float sh[1024];
  const int bid = blockIdx.x, t = threadIdx.x;
  if (bid < R * H) {
    const int r = bid / H, h = bid - (bid / H) * H;
    const bool live = gidx[r] >= 0;
    for (int k = t; k < D; k += 256) sh[k] = live ? du[((int64_t)r * GF_HP + h) * D + k] : 0.f;
    __syncthreads();
    const int i = t >> 2, part = t & 3;
    const E* wr = wkg + (int64_t)(h * 64 + i) * D;
    float a = 0.f;
    for (int k = 8 * part; k < D; k += 32) {
      float x[8];
      load4(wr + k, x);
      load4(wr + k + 4, x + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) a = fmaf(x[j], sh[k + j], a);
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (part == 0) dqg[(int64_t)r * D + h * 64 + i] = a;
    return;
  }
  const int o2 = bid - R * H, which = o2 >= D ? 1 : 0, o = o2 - which * D, h = o >> 6;
  for (int rr = t; rr < R; rr += 256) {
    const int pos = gidx[rr];
    float c = 0.f;
    if (pos >= 0)
      c = which == 0 ? to_f32(qg[(int64_t)rr * ldq + o]) : to_f32(dout[((int64_t)(rr / gmax) * Lp + pos) * ldd + o]);
    sh[rr] = c;
  }
  __syncthreads();
  const float* src = (which == 0 ? du : w) + (int64_t)h * D;
  float* dst = (which == 0 ? dwkg : dwvg) + (int64_t)o * D;
  for (int c = t; c < D; c += 256) {
    float a = 0.f;
#pragma unroll 4
    for (int rr = 0; rr < R; ++rr) a = fmaf(sh[rr], src[(int64_t)rr * GF_HP * D + c], a);
    dst[c] = a;
  }
  if (t == 0) {
    if (which == 1) {
      float a = 0.f;
      for (int rr = 0; rr < R; ++rr) a = fmaf(sh[rr], st[((int64_t)rr * GF_HP + h) * 4 + 3], a);
      dbvg[o] = a;
    } else if (dbkg) {
      dbkg[o] = 0.f;
    }
  }
}

// Gradient of the global-key (value) rows of the local branch: the band backward's dS (P) columns of
// the global keys, reduced over every query of the sequence and added at the global positions:
//   dk[b*Lp + gidx[b][g]][h*64+d] += sum_i gds[b][h][i][g] q[b*Lp+i][h*64+d]   (blockIdx.y = 0)
//   dv[b*Lp + gidx[b][g]][h*64+d] += sum_i gpr[b][h][i][g] dout[b*Lp+i][h*64+d] (blockIdx.y = 1)
// Block (b*H + h, k|v): thread (32 row groups x 8 column octets, 16-B loads, 8 rows in flight), 4
// global slots per pass, fp32 accumulation in a fixed order (row group, then the 32 groups summed in
// order), one rounding into dk.
template <typename E>
__global__ void __launch_bounds__(256) k_global_kv_grad(int Lp, int H, int gmax, const float* __restrict__ gds,
                                                        const float* __restrict__ gpr, const E* __restrict__ q,
                                                        int ldq, const E* __restrict__ dout, int ldd,
                                                        const int32_t* __restrict__ gidx, E* __restrict__ dk,
                                                        int ldk, E* __restrict__ dv, int ldv) {
  typedef typename H16<E>::x8 V8;
  __shared__ float red[32][4][64];
  const int bh = blockIdx.x, b = bh / H, h = bh - (bh / H) * H, kv = blockIdx.y;
  const float* wsrc = (kv ? gpr : gds) + (int64_t)bh * Lp * gmax;
  const E* x = (kv ? dout : q) + (int64_t)b * Lp * (kv ? ldd : ldq) + h * 64;
  const int ldx = kv ? ldd : ldq;
  E* dst = kv ? dv : dk;
  const int ldo = kv ? ldv : ldk;
  const int t = threadIdx.x, c8 = (t & 7) * 8, rg = t >> 3;
  for (int g0 = 0; g0 < gmax; g0 += 4) {
    const int gn = min(4, gmax - g0);
    float acc[4][8];
#pragma unroll
    for (int gg = 0; gg < 4; ++gg)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[gg][j] = 0.f;
    // rows rg, rg + 32, ...: 8 rows per batch, their loads issued together
    for (int i0 = rg; i0 < Lp; i0 += 32 * 8) {
      V8 xv[8];
      float wv[8][4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 32 * u;
        xv[u] = i < Lp ? *reinterpret_cast<const V8*>(x + (int64_t)i * ldx + c8) : V8{};
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) wv[u][gg] = (i < Lp && gg < gn) ? wsrc[(int64_t)i * gmax + g0 + gg] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[gg][j] = fmaf(wv[u][gg], to_f32(xv[u][j]), acc[gg][j]);
    }
#pragma unroll
    for (int gg = 0; gg < 4; ++gg)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[rg][gg][c8 + j] = acc[gg][j];
    __syncthreads();
    const int gg = t >> 6, col = t & 63;
    if (gg < gn) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 32; ++k) sum += red[k][gg][col];
      const int pos = gidx[b * gmax + g0 + gg];
      if (pos >= 0) {
        E* o = dst + ((int64_t)b * Lp + pos) * ldo + h * 64 + col;
        *o = (E)(to_f32(*o) + sum);
      }
    }
    __syncthreads();
  }
}

// Backward of the query_global projection of the global rows, qg = (h_g Wqg^T + bqg) * q_scale
// (TF:966-967), from dqg (R x D fp32; 0 for empty slots) — rf_global_query_bwd, grid D + R * (D / 64):
//   block o < D:  dWqg[o][c] = q_scale sum_r dqg[r][o] h[row r][c],  dbqg[o] = q_scale sum_r dqg[r][o]
//   then (r, 64 columns c): dh[row r][c] += sum_o dqg[r][o] WqgT[c][o]   (WqgT: the transposed weight
//   with q_scale folded in, the packed training copy; four threads per output over its row).
template <typename E>
__global__ void __launch_bounds__(256) k_gq_bwd(int D, int Lp, int gmax, int R, const int32_t* __restrict__ gidx,
                                                const float* __restrict__ dqg, float q_scale,
                                                const E* __restrict__ hs, int ldh, const E* __restrict__ wqgT,
                                                float* __restrict__ dwqg, float* __restrict__ dbqg,
                                                E* __restrict__ dh, int lddh) {
  __shared__ float sh[1024];
  __shared__ int64_t rowof[1024];
  const int bid = blockIdx.x, t = threadIdx.x;
  if (bid < D) {
    const int o = bid;
    for (int r = t; r < R; r += 256) {
      const int pos = gidx[r];
      sh[r] = pos >= 0 ? q_scale * dqg[(int64_t)r * D + o] : 0.f;
      rowof[r] = pos >= 0 ? (int64_t)(r / gmax) * Lp + pos : -1;
    }
    __syncthreads();
    for (int c = t; c < D; c += 256) {
      float a = 0.f;
#pragma unroll 4
      for (int r = 0; r < R; ++r)
        if (rowof[r] >= 0) a = fmaf(sh[r], to_f32(hs[rowof[r] * ldh + c]), a);
      dwqg[(int64_t)o * D + c] = a;
    }
    if (t == 0) {
      float a = 0.f;
      for (int r = 0; r < R; ++r) a += sh[r];
      dbqg[o] = a;
    }
    return;
  }
  const int nct = D / 64, b2 = bid - D, r = b2 / nct, ct = b2 - (b2 / nct) * nct;
  const int pos = gidx[r];
  if (pos < 0) return;
  for (int k = t; k < D; k += 256) sh[k] = dqg[(int64_t)r * D + k];
  __syncthreads();
  const int c = ct * 64 + (t >> 2), part = t & 3;
  const E* wr = wqgT + (int64_t)c * D;
  float a = 0.f;
  for (int k = 8 * part; k < D; k += 32) {
    float x[8];
    load4(wr + k, x);
    load4(wr + k + 4, x + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) a = fmaf(x[j], sh[k + j], a);
  }
  a += __shfl_xor(a, 1, 64);
  a += __shfl_xor(a, 2, 64);
  if (part == 0) {
    E* o = dh + ((int64_t)(r / gmax) * Lp + pos) * lddh + c;
    *o = (E)(to_f32(*o) + a);
  }
}

struct GbwdWs {
  char* dwp;
  char* bt;
  float* dupart;
};

inline size_t gbwd_bytes(int R, int Lp, int D) {
  const int nch2 = (Lp + GB_ROWS - 1) / GB_ROWS;
  return align256((size_t)R * 2 * GF_HP * D * 2) + align256((size_t)R * D * 32 * 2) +
         (size_t)R * nch2 * GF_HP * D * 4;
}

}  // namespace rf

extern "C" size_t rf_global_fold_bwd_workspace(int B, int Lp, int D, int gmax) {
  if (B <= 0 || gmax <= 0 || Lp <= 0) return 0;
  return gbwd_bytes(B * gmax, Lp, D);
}

// shared by rf_global_fold_bwd (dw / cb given) and rf_global_fold_bwd_full (FROM_DOUT: dw / c from
// the output gradient's global rows and Wvg / bvg inside the prep kernel; cbw receives c)
static void gbwd_run(int dtype, int B, int Lp, int D, int H, const void* h, int ldh, const uint8_t* flags,
                     const int32_t* gidx, int gmax, const void* fwd_workspace, const float* dw, const float* cb,
                     const void* dout, int ldd, const void* wvg, const float* bvg, float* cbw, float p_drop,
                     uint64_t seed, void* dh, int lddh, float* du, float* w, float* stats, void* workspace,
                     hipStream_t s) {
  const bool from_dout = dout != nullptr;
  const int R = B * gmax;
  const int nch = (Lp + gfold_chunk(dtype, R, Lp) - 1) / gfold_chunk(dtype, R, Lp);  // the forward's chunks
  const int nch2 = (Lp + GB_ROWS - 1) / GB_ROWS;
  GfoldWs fws = gfold_carve(const_cast<void*>(fwd_workspace), R, nch, H, D);
  char* p = reinterpret_cast<char*>(workspace);
  GbwdWs bw;
  bw.dwp = p; p += align256((size_t)R * 2 * GF_HP * D * 2);
  bw.bt = p; p += align256((size_t)R * D * 32 * 2);
  bw.dupart = reinterpret_cast<float*>(p);
  const AttnDrop dr{seed, drop_thresh(p_drop), p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.f, g_seed_dev};
  const int drop = p_drop > 0.f ? 1 : 0;
  const float* cbm = from_dout ? (drop ? cbw : nullptr) : cb;  // the main kernel's c terms
  const size_t lds = (size_t)D * 128 + 2 * 4 * 64 * 16 * 4 + (size_t)GB_GMAX * 64 * 32 * 2;
#define GB_(EE, DD)                                                                                          \
  case DD:                                                                                                   \
    if (from_dout)                                                                                           \
      k_gbwd_prep<EE, true><<<dim3(R, GF_HP), 256, 0, s>>>(D, H, nch, Lp, gmax, gidx, fws, nullptr, nullptr,  \
                                                           (const EE*)dout, ldd, (const EE*)wvg, bvg, cbw,    \
                                                           drop, w, stats, (EE*)bw.dwp, (EE*)bw.bt);          \
    else                                                                                                     \
      k_gbwd_prep<EE, false><<<dim3(R, GF_HP), 256, 0, s>>>(D, H, nch, Lp, gmax, gidx, fws, dw, cb, nullptr,  \
                                                            0, nullptr, nullptr, nullptr, drop, w, stats,     \
                                                            (EE*)bw.dwp, (EE*)bw.bt);                         \
    (void)hipFuncSetAttribute((const void*)k_gbwd_main<EE, DD>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                              (int)lds);                                                                       \
    k_gbwd_main<EE, DD><<<dim3(nch2, B), 256, lds, s>>>(Lp, gmax, H, (const EE*)h, ldh, flags, gidx, fws,      \
                                                        (const EE*)bw.dwp, (const EE*)bw.bt, stats, cbm,       \
                                                        bw.dupart, (EE*)dh, lddh, dr);                         \
    break;
  if (dtype == RF_F16) {
    switch (D) { GB_(f16, 128) GB_(f16, 256) GB_(f16, 384) GB_(f16, 512) GB_(f16, 640) GB_(f16, 768) default: break; }
  } else {
    switch (D) { GB_(bf16, 128) GB_(bf16, 256) GB_(bf16, 384) GB_(bf16, 512) GB_(bf16, 640) GB_(bf16, 768) default: break; }
  }
#undef GB_
  const int64_t n = (int64_t)R * GF_HP * D;
  k_gbwd_reduce<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(R, D, nch2, gidx, bw.dupart, du);
}

static int gbwd_check(int dtype, int B, int Lp, int D, int H, int gmax, float p_drop, const char* name) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "%s: 16-bit operands only", name);
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && H > 0 && H <= GF_HP && D == 64 * H,
             "%s: bad shape B=%d Lp=%d D=%d H=%d", name, B, Lp, D, H);
  RF_REQUIRE(D % 128 == 0 && D <= 768, "%s: D=%d (multiples of 128 up to 768)", name, D);
  RF_REQUIRE(gmax <= GB_GMAX, "%s: at most %d global rows per sequence", name, GB_GMAX);
  RF_REQUIRE(Lp <= 64 * 64, "%s: Lp=%d (at most 64 chunks of the forward pass)", name, Lp);
  RF_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "%s: p_drop %f", name, p_drop);
  return RF_OK;
}

extern "C" int rf_global_fold_bwd(int dtype, int B, int Lp, int D, int H, const void* h, int ldh,
                                  const uint8_t* flags, const int32_t* gidx, int gmax, const void* fwd_workspace,
                                  const float* dw, const float* cb, float p_drop, uint64_t seed, void* dh, int lddh,
                                  float* du, float* w, float* stats, void* workspace, rf_stream_t stream) {
  const int rc = gbwd_check(dtype, B, Lp, D, H, gmax, p_drop, "rf_global_fold_bwd");
  if (rc != RF_OK) return rc;
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(h && flags && gidx && fwd_workspace && dw && dh && du && w && stats && workspace,
             "rf_global_fold_bwd: null pointer");
  RF_REQUIRE(ldh % 8 == 0 && lddh % 8 == 0 && ldh >= D && lddh >= D, "rf_global_fold_bwd: leading dims");
  RF_REQUIRE((int64_t)Lp * ldh * 4 < 0x7FFFFFFF, "rf_global_attn_fold: one sequence's rows must span < 2 GiB");
  gbwd_run(dtype, B, Lp, D, H, h, ldh, flags, gidx, gmax, fwd_workspace, dw, cb, nullptr, 0, nullptr, nullptr,
           nullptr, p_drop, seed, dh, lddh, du, w, stats, workspace, as_stream(stream));
  RF_LAUNCH_CHECK("rf_global_fold_bwd");
}

extern "C" size_t rf_global_fold_bwd_full_workspace(int B, int Lp, int D, int gmax) {
  if (B <= 0 || gmax <= 0 || Lp <= 0) return 0;
  const size_t R = (size_t)B * gmax;
  return gbwd_bytes(B * gmax, Lp, D) + 2 * align256(R * GF_HP * D * 4) + align256(R * GF_HP * 4 * 4) +
         align256(R * GF_HP * 4) + 256;
}

extern "C" int rf_global_fold_bwd_full(int dtype, int B, int Lp, int D, int H, const void* h, int ldh,
                                       const uint8_t* flags, const int32_t* gidx, int gmax,
                                       const void* fwd_workspace, const void* dout, int lddout, const void* qg,
                                       int ldqg, const void* wkg, const void* wvg, const float* bvg, float p_drop,
                                       uint64_t seed, void* dh, int lddh, float* dqg, float* dwkg, float* dwvg,
                                       float* dbvg, float* dbkg, void* workspace, rf_stream_t stream) {
  const int rc = gbwd_check(dtype, B, Lp, D, H, gmax, p_drop, "rf_global_fold_bwd_full");
  if (rc != RF_OK) return rc;
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(h && flags && gidx && fwd_workspace && dout && qg && wkg && wvg && bvg && dh && dqg && dwkg && dwvg &&
                 dbvg && workspace,
             "rf_global_fold_bwd_full: null pointer");
  RF_REQUIRE(ldh % 8 == 0 && lddh % 8 == 0 && ldh >= D && lddh >= D && lddout >= D && ldqg >= D,
             "rf_global_fold_bwd_full: leading dims");
  RF_REQUIRE(B * gmax <= 1024, "rf_global_fold_bwd_full: at most 1024 global rows");
  RF_REQUIRE((int64_t)Lp * ldh * 4 < 0x7FFFFFFF, "rf_global_attn_fold: one sequence's rows must span < 2 GiB");
  const int R = B * gmax;
  char* p = reinterpret_cast<char*>(workspace) + gbwd_bytes(R, Lp, D);
  p = reinterpret_cast<char*>(((uintptr_t)p + 255) & ~(uintptr_t)255);
  float* du = reinterpret_cast<float*>(p); p += align256((size_t)R * GF_HP * D * 4);
  float* w = reinterpret_cast<float*>(p); p += align256((size_t)R * GF_HP * D * 4);
  float* st = reinterpret_cast<float*>(p); p += align256((size_t)R * GF_HP * 4 * 4);
  float* cbw = reinterpret_cast<float*>(p);
  hipStream_t s = as_stream(stream);
  gbwd_run(dtype, B, Lp, D, H, h, ldh, flags, gidx, gmax, fwd_workspace, nullptr, nullptr, dout, lddout, wvg, bvg,
           cbw, p_drop, seed, dh, lddh, du, w, st, workspace, s);
  if (dtype == RF_F16)
    k_gbwd_post<f16><<<R * H + 2 * D, 256, 0, s>>>(D, H, Lp, gmax, R, gidx, (const f16*)dout, lddout, (const f16*)qg,
                                                   ldqg, (const f16*)wkg, du, w, st, dqg, dwkg, dwvg, dbvg, dbkg);
  else
    k_gbwd_post<bf16><<<R * H + 2 * D, 256, 0, s>>>(D, H, Lp, gmax, R, gidx, (const bf16*)dout, lddout,
                                                    (const bf16*)qg, ldqg, (const bf16*)wkg, du, w, st, dqg, dwkg,
                                                    dwvg, dbvg, dbkg);
  RF_LAUNCH_CHECK("rf_global_fold_bwd_full");
}

extern "C" int rf_global_kv_grad(int dtype, int B, int Lp, int H, int gmax, const float* gds, const float* gpr,
                                 const void* q, int ldq, const void* dout, int lddout, const int32_t* gidx, void* dk,
                                 int ldk, void* dv, int ldv, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_global_kv_grad: 16-bit operands only");
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && H > 0, "rf_global_kv_grad: bad shape");
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(gds && gpr && q && dout && gidx && dk && dv, "rf_global_kv_grad: null pointer");
  RF_REQUIRE(ldq % 8 == 0 && lddout % 8 == 0 && ldq >= 64 * H && lddout >= 64 * H && ldk >= 64 * H && ldv >= 64 * H,
             "rf_global_kv_grad: leading dims");
  RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)dout & 15) == 0, "rf_global_kv_grad: q / dout 16-B aligned");
  hipStream_t s = as_stream(stream);
  if (dtype == RF_F16)
    k_global_kv_grad<f16><<<dim3(B * H, 2), 256, 0, s>>>(Lp, H, gmax, gds, gpr, (const f16*)q, ldq, (const f16*)dout,
                                                         lddout, gidx, (f16*)dk, ldk, (f16*)dv, ldv);
  else
    k_global_kv_grad<bf16><<<dim3(B * H, 2), 256, 0, s>>>(Lp, H, gmax, gds, gpr, (const bf16*)q, ldq,
                                                          (const bf16*)dout, lddout, gidx, (bf16*)dk, ldk, (bf16*)dv,
                                                          ldv);
  RF_LAUNCH_CHECK("rf_global_kv_grad");
}

extern "C" int rf_global_query_bwd(int dtype, int B, int Lp, int D, int gmax, const int32_t* gidx, const float* dqg,
                                   float q_scale, const void* h, int ldh, const void* wqgT, float* dwqg, float* dbqg,
                                   void* dh, int lddh, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_global_query_bwd: 16-bit operands only");
  RF_REQUIRE(B >= 0 && Lp >= 0 && gmax >= 0 && D > 0 && D % 64 == 0, "rf_global_query_bwd: bad shape");
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  RF_REQUIRE(B * gmax <= 1024, "rf_global_query_bwd: at most 1024 global rows");
  RF_REQUIRE(gidx && dqg && h && wqgT && dwqg && dbqg && dh, "rf_global_query_bwd: null pointer");
  RF_REQUIRE(ldh >= D && lddh >= D && ((uintptr_t)wqgT & 7) == 0, "rf_global_query_bwd: leading dims / alignment");
  const int R = B * gmax;
  hipStream_t s = as_stream(stream);
  if (dtype == RF_F16)
    k_gq_bwd<f16><<<D + R * (D / 64), 256, 0, s>>>(D, Lp, gmax, R, gidx, dqg, q_scale, (const f16*)h, ldh,
                                                    (const f16*)wqgT, dwqg, dbqg, (f16*)dh, lddh);
  else
    k_gq_bwd<bf16><<<D + R * (D / 64), 256, 0, s>>>(D, Lp, gmax, R, gidx, dqg, q_scale, (const bf16*)h, ldh,
                                                     (const bf16*)wqgT, dwqg, dbqg, (bf16*)dh, lddh);
  RF_LAUNCH_CHECK("rf_global_query_bwd");
}
