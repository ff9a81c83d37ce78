// Longformer sliding-window + global attention.
//
// Local branch, bf16 (k_band_attn_bf16): one workgroup = (64-query block, head, sequence),
// 4 waves x 16 queries. The block's 128-row K/V window [i0-32, i0+96) and a 32-row chunk
// of global-token K/V rows are DMA'd into LDS (16-B global_load_lds, XOR-swizzled image).
// Per wave: S^T = K.Q^T on v_mfma_f32_16x16x32_bf16 (keys on the MFMA row, the wave's 16
// queries on the lane), so each lane holds one query's scores and the softmax row
// reductions are two shuffles (lanes l, l^16, l^32, l^48). O^T = V^T.P^T takes P straight
// from the S^T accumulators (cdna_hip_programming.md §3 'accumulator as next operand')
// and V^T through ds_read_b64_tr_b16 (§5.5 T10). Online softmax over segments
// {window, global chunk 0, 1, ...} supports any number of global tokens.
//
// Masking contract (Appendix A / TF:519-579, 743-757, 898-926): a local query i sees the
// keys j with |i-j| <= 32 that are valid and NOT global, plus every global key of its
// sequence (local K/V). Padded query rows are written as exactly 0. Global query rows are
// computed here too and then overwritten by k_global_attn (TF:612-629).
#include <stdlib.h>

#include "rf_common.h"

namespace rf {

constexpr float RF_NEG_INF = -__builtin_inff();
constexpr float LOG2E = 1.4426950408889634f;

// LDS carve (bytes)
constexpr int AT_KW = 0;            // 128 x 128 B
constexpr int AT_VW = 16384;        // 128 x 128 B
constexpr int AT_KG = 32768;        // 32 x 128 B
constexpr int AT_VG = 36864;        // 32 x 128 B
constexpr int AT_FL = 40960;        // 128 window flags
constexpr int AT_GP = 41088;        // 32 x int global positions
constexpr int AT_LDS = 41216;

// byte offset of bf16 element (row, col) in a swizzled [rows][64] image
__device__ __forceinline__ int swz_el(int row, int col) {
  return row * 128 + (((col >> 3) ^ (row & 7)) << 4) + ((col & 7) << 1);
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// Two ds_read_b64_tr_b16 + lgkmcnt(0) as one asm statement. With an LDS-DMA in flight hipcc
// treats the transposed-read builtin as possibly aliasing it and waits vmcnt(0) first, which
// would drain the prefetch pipeline; as asm the read is ordered only by the kernel's own
// counted vmcnt + barrier protocol (the slots read here were retired before the barrier).
__device__ __forceinline__ void tr_read2(uint32_t a0, uint32_t a1, bf16x4& v0, bf16x4& v1) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %2\n\t"
      "ds_read_b64_tr_b16 %1, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v0), "=&v"(v1)
      : "v"(a0), "v"(a1)
      : "memory");
}

template <typename E>
__device__ __forceinline__ typename H16<E>::x4 tr_read(const char* lds_base, int off) {
  // the transposed 16-bit read moves bit patterns: one instruction for bf16 and fp16
  return __builtin_bit_cast(typename H16<E>::x4, __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds_base + off)));
}

template <typename E>
__global__ void __launch_bounds__(256) k_band_attn_bf16(int Lp, const E* __restrict__ q,
                                                         const E* __restrict__ k,
                                                         const E* __restrict__ v, int ld,
                                                         const uint8_t* __restrict__ flags,
                                                         const int32_t* __restrict__ gidx,
                                                         int gmax, E* __restrict__ out,
                                                         int ldo, int H) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  __shared__ __attribute__((aligned(16))) char smem[AT_LDS];
  // 1-D grid, XCD-remapped: the Lp/64 query blocks of one (sequence, head) are consecutive
  // on one XCD, so the half-overlapping K/V windows of neighbouring blocks hit its L2
  const int nqb = Lp >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = wg % nqb, bh = wg / nqb;
  const int i0 = qb * 64, h = bh % H, b = bh / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  int* gp = reinterpret_cast<int*>(smem + AT_GP);
  uint8_t* fl = reinterpret_cast<uint8_t*>(smem + AT_FL);

  // ---- stage the K/V window (16 chunks of 8 rows; 4 per wave) ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = wave * 4 + i;
    const int row = c * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int kp = min(max(i0 - 32 + row, 0), Lp - 1);
    const int64_t off = (rb + kp) * ld + hoff + ch * 8;
    glds16(k + off, smem + AT_KW + c * 1024);
    glds16(v + off, smem + AT_VW + c * 1024);
  }
  auto stage_global = [&](int cg) {
    const int row = wave * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int gi = cg * 32 + row;
    const int p = gi < gmax ? gidx[(int64_t)b * gmax + gi] : -1;
    const int64_t off = (rb + (p >= 0 ? p : 0)) * ld + hoff + ch * 8;
    glds16(k + off, smem + AT_KG + wave * 1024);
    glds16(v + off, smem + AT_VG + wave * 1024);
    if (threadIdx.x < 32) {
      const int gj = cg * 32 + threadIdx.x;
      gp[threadIdx.x] = gj < gmax ? gidx[(int64_t)b * gmax + gj] : -1;
    }
  };
  const int nchunks = (gmax + 31) / 32;
  if (nchunks > 0) stage_global(0);
  if (threadIdx.x < 128) {
    const int kp = i0 - 32 + threadIdx.x;
    fl[threadIdx.x] = (kp >= 0 && kp < Lp) ? flags[rb + kp] : 0;
  }

  // ---- this wave's queries: Q^T fragments (B operand) straight from HBM ----
  const int qw = i0 + 16 * wave;
  const int myq = qw + li;
  const int ks = min(16 * wave, 32);  // first LDS window row of the wave's 96-key span
  V8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    qf[s] = *reinterpret_cast<const V8*>(q + (rb + myq) * ld + hoff + 32 * s + 8 * g);

  wait_vmcnt0();
  __syncthreads();

  // ---- window segment: 6 key tiles of 16 ----
  f32x4 st[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const V8 kf = *reinterpret_cast<const V8*>(smem + AT_KW + swz128(ks + 16 * t + li, 4 * s + g));
      st[t] = mfma16(kf, qf[s], st[t]);
    }
  }
  float mx = RF_NEG_INF;
#pragma unroll
  for (int t = 0; t < 6; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kr = ks + 16 * t + 4 * g + r;     // LDS window row
      const int kp = i0 - 32 + kr;                 // absolute key position
      const bool ok = (abs(kp - myq) <= 32) && (fl[kr] == 1);
      const float sv = ok ? st[t][r] : RF_NEG_INF;
      st[t][r] = sv;
      mx = fmaxf(mx, sv);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float m = mx;
  float lsum = 0.f;
  {
    const float mu = (m == RF_NEG_INF) ? 0.f : m;
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f((st[t][r] - mu) * LOG2E);
        st[t][r] = p;
        lsum += p;
      }
  }
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // PV: 3 k-steps of 32 keys; key(g, j) = 32*s + 16*(j>>2) + 4*g + (j&3)
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    V8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (E)st[2 * s + (j >> 2)][j & 3];
    const int r0 = ks + 32 * s + 4 * g + (li >> 2);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V4 v0 = tr_read<E>(smem + AT_VW, swz_el(r0, col));
      const V4 v1 = tr_read<E>(smem + AT_VW, swz_el(r0 + 16, col));
      V8 vf;
      vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
      vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
      o[dt] = mfma16(vf, pf, o[dt]);
    }
  }

  // ---- global-key segments (local K/V at global positions) ----
  for (int cg = 0; cg < nchunks; ++cg) {
    if (cg > 0) {
      __syncthreads();
      stage_global(cg);
      wait_vmcnt0();
      __syncthreads();
    }
    f32x4 sg[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const V8 kf = *reinterpret_cast<const V8*>(smem + AT_KG + swz128(16 * t + li, 4 * s + g));
        sg[t] = mfma16(kf, qf[s], sg[t]);
      }
    }
    float cmx = RF_NEG_INF;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = gp[16 * t + 4 * g + r] >= 0;
        const float sv = ok ? sg[t][r] : RF_NEG_INF;
        sg[t][r] = sv;
        cmx = fmaxf(cmx, sv);
      }
    cmx = fmaxf(cmx, __shfl_xor(cmx, 16, 64));
    cmx = fmaxf(cmx, __shfl_xor(cmx, 32, 64));
    const float mn = fmaxf(m, cmx);
    const float mu = (mn == RF_NEG_INF) ? 0.f : mn;
    const float alpha = exp2f((m - mu) * LOG2E);
    lsum *= alpha;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f((sg[t][r] - mu) * LOG2E);
        sg[t][r] = p;
        lsum += p;
      }
    m = mn;
    V8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (E)sg[j >> 2][j & 3];
    const int r0 = 4 * g + (li >> 2);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V4 v0 = tr_read<E>(smem + AT_VG, swz_el(r0, col));
      const V4 v1 = tr_read<E>(smem + AT_VG, swz_el(r0 + 16, col));
      V8 vf;
      vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
      vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
      o[dt] = mfma16(vf, pf, o[dt]);
    }
  }

  // ---- normalise and store O[q][16dt + 4g + r] ----
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const bool qvalid = fl[32 + 16 * wave + li] != 0;
  const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;
  E* orow = out + (rb + myq) * ldo + hoff + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    V4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = (E)(qvalid ? o[dt][r] * inv : 0.f);
    *reinterpret_cast<V4*>(orow + 16 * dt) = w;
  }
}

// ------------------------------------------------------------------------------------
// Local branch, 16-bit, any window (k_band_attn_wide): the layout of k_band_attn_bf16 with
// the key span of a 64-query block, rows [i0 - w, i0 + 63 + w], walked in 64-row chunks under
// the online softmax (one more chunk per 64 of window), then the global-key chunks. Chunk c's
// K/V rows are DMA'd to LDS once per workgroup; each wave skips the 16-key tiles outside its
// own span [qw - w, qw + 15 + w]. Any half window and any Lp (query rows past Lp are not
// stored). The window-64 kernels above stay the production path; this one serves the other
// per-layer windows the reference accepts (models.py:179-187, e.g. the 512 offline preset).
constexpr int AW_K = 0;        // 64 x 128 B
constexpr int AW_V = 8192;     // 64 x 128 B
constexpr int AW_KG = 16384;   // 32 x 128 B
constexpr int AW_VG = 20480;   // 32 x 128 B
constexpr int AW_FL = 24576;   // 64 chunk-row flags
constexpr int AW_GP = 24640;   // 32 x int
constexpr int AW_LDS = 24768;

template <typename E>
__global__ void __launch_bounds__(256) k_band_attn_wide(int Lp, int half_w, const E* __restrict__ q,
                                                         const E* __restrict__ k,
                                                         const E* __restrict__ v, int ld,
                                                         const uint8_t* __restrict__ flags,
                                                         const int32_t* __restrict__ gidx,
                                                         int gmax, E* __restrict__ out,
                                                         int ldo, int H) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  __shared__ __attribute__((aligned(16))) char smem[AW_LDS];
  const int nqb = (Lp + 63) >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = wg % nqb, bh = wg / nqb;
  const int i0 = qb * 64, h = bh % H, b = bh / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  const int w = half_w;
  int* gp = reinterpret_cast<int*>(smem + AW_GP);
  uint8_t* fl = reinterpret_cast<uint8_t*>(smem + AW_FL);

  const int qw = i0 + 16 * wave;
  const int myq = qw + li;
  const int qrow = min(myq, Lp - 1);
  V8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    qf[s] = *reinterpret_cast<const V8*>(q + (rb + qrow) * ld + hoff + 32 * s + 8 * g);
  const bool qvalid = myq < Lp && flags[rb + qrow] != 0;

  float m = RF_NEG_INF, lsum = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one segment of up to 64 keys (4 tiles of 16) against the wave's 16 queries: scores for the
  // tiles in [t_lo, t_hi), masked by `ok(key tile row)`, online-softmax update, P.V
  auto segment = [&](const char* kbase, const char* vbase, int ntile, auto ok) {
    f32x4 st[4];
    float cmx = RF_NEG_INF;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < ntile) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const V8 kf = *reinterpret_cast<const V8*>(kbase + swz128(16 * t + li, 4 * s + g));
          st[t] = mfma16(kf, qf[s], st[t]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sv = (t < ntile && ok(16 * t + 4 * g + r)) ? st[t][r] : RF_NEG_INF;
        st[t][r] = sv;
        cmx = fmaxf(cmx, sv);
      }
    }
    cmx = fmaxf(cmx, __shfl_xor(cmx, 16, 64));
    cmx = fmaxf(cmx, __shfl_xor(cmx, 32, 64));
    const float mn = fmaxf(m, cmx);
    const float mu = (mn == RF_NEG_INF) ? 0.f : mn;
    const float alpha = exp2f((m - mu) * LOG2E);
    lsum *= alpha;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f((st[t][r] - mu) * LOG2E);
        st[t][r] = p;
        lsum += p;
      }
    m = mn;
    // PV: k-steps of 32 keys; key(g, j) = 32*s + 16*(j>>2) + 4*g + (j&3)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (2 * s < ntile) {
        V8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (E)st[2 * s + (j >> 2)][j & 3];
        const int r0 = 32 * s + 4 * g + (li >> 2);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int col = 16 * dt + 4 * (li & 3);
          const V4 v0 = tr_read<E>(vbase, swz_el(r0, col));
          const V4 v1 = tr_read<E>(vbase, swz_el(r0 + 16, col));
          V8 vf;
          vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
          vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
          o[dt] = mfma16(vf, pf, o[dt]);
        }
      }
    }
  };

  // ---- window chunks ----
  const int k_first = i0 - w;
  const int nck = (64 + 2 * w + 63) / 64;
  for (int c = 0; c < nck; ++c) {
    const int kb0 = k_first + 64 * c;
    __syncthreads();  // the previous chunk's LDS reads are done
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cc = wave * 2 + i;
      const int row = cc * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (row & 7);
      const int kp = min(max(kb0 + row, 0), Lp - 1);
      const int64_t off = (rb + kp) * ld + hoff + ch * 8;
      glds16(k + off, smem + AW_K + cc * 1024);
      glds16(v + off, smem + AW_V + cc * 1024);
    }
    if (threadIdx.x < 64) {
      const int kp = kb0 + threadIdx.x;
      fl[threadIdx.x] = (kp >= 0 && kp < Lp) ? flags[rb + kp] : 0;
    }
    wait_vmcnt0();
    __syncthreads();
    // tiles of this chunk that meet the wave's span [qw - w, qw + 15 + w]
    const int lo = qw - w - kb0, hi = qw + 15 + w - kb0;
    if (hi < 0 || lo > 63) continue;
    const int ntile = min(4, (hi >> 4) + 1);
    segment(smem + AW_K, smem + AW_V, ntile, [&](int kr) {
      const int kp = kb0 + kr;
      return abs(kp - myq) <= w && fl[kr] == 1;
    });
  }

  // ---- global-key chunks (local K/V at global positions) ----
  const int nchunks = (gmax + 31) / 32;
  for (int cg = 0; cg < nchunks; ++cg) {
    __syncthreads();
    {
      const int row = wave * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (row & 7);
      const int gi = cg * 32 + row;
      const int p = gi < gmax ? gidx[(int64_t)b * gmax + gi] : -1;
      const int64_t off = (rb + (p >= 0 ? p : 0)) * ld + hoff + ch * 8;
      glds16(k + off, smem + AW_KG + wave * 1024);
      glds16(v + off, smem + AW_VG + wave * 1024);
      if (threadIdx.x < 32) {
        const int gj = cg * 32 + threadIdx.x;
        gp[threadIdx.x] = gj < gmax ? gidx[(int64_t)b * gmax + gj] : -1;
      }
    }
    wait_vmcnt0();
    __syncthreads();
    segment(smem + AW_KG, smem + AW_VG, 2, [&](int kr) { return gp[kr] >= 0; });
  }

  // ---- normalise and store O[q][16dt + 4g + r] ----
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (myq >= Lp) return;
  const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;
  E* orow = out + (rb + myq) * ldo + hoff + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    V4 wv;
#pragma unroll
    for (int r = 0; r < 4; ++r) wv[r] = (E)(qvalid ? o[dt][r] * inv : 0.f);
    *reinterpret_cast<V4*>(orow + 16 * dt) = wv;
  }
}

// ------------------------------------------------------------------------------------
// Local branch, bf16, pipelined sliding window (k_band_attn_pipe): one workgroup walks a run
// of consecutive 64-query blocks of one (sequence, head). Keys are staged in 64-row chunks
// c = rows [64c-32, 64c+32): query block x needs chunks x and x+1, so each chunk is DMA'd
// once (not twice, as with one window per block) into a 3-slot ring, and Q blocks into a
// 2-slot ring. At the end of block x the slot it no longer needs receives chunk x+3 and
// Q(x+2), then O(x) is stored: loads run two blocks ahead and the stores, issued last, are
// never waited for by the next block's counted vmcnt. Key masks (valid & local, and valid)
// are 64-bit ballots per chunk computed once in the prologue. Needs gmax <= 32.
constexpr int AP_Q = 0;          // 2 x 64 rows x 128 B
constexpr int AP_KV = 16384;     // 3 x (K 64 x 128 B, V 64 x 128 B)
constexpr int AP_KG = 65536;     // 32 x 128 B
constexpr int AP_VG = 69632;     // 32 x 128 B
constexpr int AP_GP = 73728;     // 32 x int
constexpr int AP_MK = 73856;     // per chunk {local mask, valid mask} uint64

__device__ __forceinline__ void wait_vm_small(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__global__ void __launch_bounds__(256) k_band_attn_pipe(int Lp, int H, int qpb, const bf16* __restrict__ q,
                                                         const bf16* __restrict__ k,
                                                         const bf16* __restrict__ v, int ld,
                                                         const uint8_t* __restrict__ flags,
                                                         const int32_t* __restrict__ gidx, int gmax,
                                                         bf16* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = Lp >> 6;
  const int nparts = (nqb + qpb - 1) / qpb;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int part = wg % nparts, bh = wg / nparts;
  const int h = bh % H, b = bh / H;
  const int x0 = part * qpb, x1 = min(nqb, x0 + qpb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  int* gp = reinterpret_cast<int*>(smem + AP_GP);
  unsigned long long* mk = reinterpret_cast<unsigned long long*>(smem + AP_MK);

  // ---- prologue: chunk masks, global keys ----
  for (int c = x0 + wave; c <= x1; c += 4) {
    const int row = 64 * c - 32 + lane;
    const int f = (row >= 0 && row < Lp) ? flags[rb + row] : 0;
    const unsigned long long ml = __ballot(f == 1), mv = __ballot(f != 0);
    if (lane == 0) {
      mk[2 * (c - x0)] = ml;
      mk[2 * (c - x0) + 1] = mv;
    }
  }
  if (gmax > 0) {
    const int row = wave * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int p = row < gmax ? gidx[(int64_t)b * gmax + row] : -1;
    const int64_t off = (rb + (p >= 0 ? p : 0)) * ld + hoff + ch * 8;
    glds16(k + off, smem + AP_KG + wave * 1024);
    glds16(v + off, smem + AP_VG + wave * 1024);
    if (threadIdx.x < 32) gp[threadIdx.x] = (int)threadIdx.x < gmax ? gidx[(int64_t)b * gmax + threadIdx.x] : -1;
  }
  auto dma_chunk = [&](int c) {  // 4 DMAs per wave: K pieces 2w, 2w+1 and V pieces 2w, 2w+1
    char* base = smem + AP_KV + (c % 3) * 16384;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      const int row = pc * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (row & 7);
      const int kp = min(max(64 * c - 32 + row, 0), Lp - 1);
      const int64_t off = (rb + kp) * ld + hoff + ch * 8;
      glds16(k + off, base + pc * 1024);
      glds16(v + off, base + 8192 + pc * 1024);
    }
  };
  auto dma_q = [&](int x) {  // 2 DMAs per wave
    char* base = smem + AP_Q + (x & 1) * 8192;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      const int row = pc * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ (row & 7);
      const int64_t off = (rb + 64 * x + row) * ld + hoff + ch * 8;
      glds16(q + off, base + pc * 1024);
    }
  };
  dma_q(x0);
  dma_chunk(x0);
  dma_chunk(x0 + 1);  // x0 + 1 <= x1 always
  if (x0 + 1 < x1) dma_q(x0 + 1);
  if (x0 + 2 <= x1) dma_chunk(x0 + 2);

  const int ks = min(16 * wave, 32);  // first window row of the wave's 96-key span
  const int myw = 32 + 16 * wave + li;  // this lane's query row inside the 128-row window
  for (int x = x0; x < x1; ++x) {
    wait_vm_small((x + 2 <= x1 ? 4 : 0) + (x + 1 < x1 ? 2 : 0) + (x > x0 ? 2 : 0));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int i0 = 64 * x;
    const unsigned long long ml0 = mk[2 * (x - x0)], ml1 = mk[2 * (x - x0) + 2];
    const unsigned long long mv0 = mk[2 * (x - x0) + 1], mv1 = mk[2 * (x - x0) + 3];
#if defined(RF_BAND_DIAG) && (RF_BAND_DIAG & 1)
    float lsum = 1.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#else
    const char* qs = smem + AP_Q + (x & 1) * 8192;
    bf16x8 qf[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      qf[s2] = *reinterpret_cast<const bf16x8*>(qs + swz128(16 * wave + li, 4 * s2 + g));
    // LDS base of window row group starting at kr (16-aligned): chunk x + (kr >> 6)
    auto kslot = [&](int kr) { return smem + AP_KV + ((x + (kr >> 6)) % 3) * 16384; };

    // ---- window segment: 6 key tiles of 16 ----
    f32x4 st[6];
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int kr0 = ks + 16 * t;
      const char* kb = kslot(kr0);
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + swz128((kr0 & 63) + li, 4 * s2 + g));
        st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s2], st[t], 0, 0, 0);
      }
    }
    // allowed keys as three 32-bit words over the wave's 96-row span [ks, ks+96):
    // valid & local (chunk ballots, wave-uniform) & band |kr - myw| <= 32 (per lane), then
    // shifted right by 4g so element (t, r) is bit 16(t&1) + r of word t>>1.
    unsigned int aw[3];
    {
      const unsigned long long lo = ks ? ((ml0 >> ks) | (ml1 << (64 - ks))) : ml0;
      const unsigned long long hi = ml1 >> ks;
      const unsigned int kv[3] = {(unsigned int)lo, (unsigned int)(lo >> 32), (unsigned int)hi};
      const int blo = myw - 32 - ks;  // band = relative rows [blo, blo + 64]
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        const int a = blo - 32 * w, z = blo + 65 - 32 * w;  // band bits [a, z) of this word
        const unsigned int from = a <= 0 ? ~0u : (a >= 32 ? 0u : (~0u << a));
        const unsigned int below = z >= 32 ? ~0u : (z <= 0 ? 0u : ((1u << z) - 1u));
        aw[w] = (kv[w] & from & below) >> (4 * g);
      }
    }
    float mx = RF_NEG_INF;
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = (aw[t >> 1] >> (16 * (t & 1) + r)) & 1u;
        const float sv = ok ? st[t][r] : RF_NEG_INF;
        st[t][r] = sv;
        mx = fmaxf(mx, sv);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float m = mx;
    float lsum = 0.f;
    {
      const float mu = (m == RF_NEG_INF) ? 0.f : m;
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f((st[t][r] - mu) * LOG2E);
          st[t][r] = p;
          lsum += p;
        }
    }
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = (bf16)st[2 * s2 + (j >> 2)][j & 3];
      const int ga = ks + 32 * s2, gb = ga + 16;  // the two 16-row key groups of this k-step
      const char* va = kslot(ga) + 8192;
      const char* vb = kslot(gb) + 8192;
      const int rr = 4 * g + (li >> 2);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = 16 * dt + 4 * (li & 3);
        bf16x4 v0, v1;
        tr_read2(lds_addr(va + swz_el((ga & 63) + rr, col)), lds_addr(vb + swz_el((gb & 63) + rr, col)), v0, v1);
        bf16x8 vf;
        vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
        vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }

    // ---- global keys (local K/V at the global positions, staged once) ----
    if (gmax > 0) {
      f32x4 sg[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(smem + AP_KG + swz128(16 * t + li, 4 * s2 + g));
          sg[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s2], sg[t], 0, 0, 0);
        }
      }
      float cmx = RF_NEG_INF;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = gp[16 * t + 4 * g + r] >= 0;
          const float sv = ok ? sg[t][r] : RF_NEG_INF;
          sg[t][r] = sv;
          cmx = fmaxf(cmx, sv);
        }
      cmx = fmaxf(cmx, __shfl_xor(cmx, 16, 64));
      cmx = fmaxf(cmx, __shfl_xor(cmx, 32, 64));
      const float mn = fmaxf(m, cmx);
      const float mu = (mn == RF_NEG_INF) ? 0.f : mn;
      const float alpha = __builtin_amdgcn_exp2f((m - mu) * LOG2E);
      lsum *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f((sg[t][r] - mu) * LOG2E);
          sg[t][r] = p;
          lsum += p;
        }
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = (bf16)sg[j >> 2][j & 3];
      const int r0 = 4 * g + (li >> 2);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = 16 * dt + 4 * (li & 3);
        bf16x4 v0, v1;
        tr_read2(lds_addr(smem + AP_VG + swz_el(r0, col)), lds_addr(smem + AP_VG + swz_el(r0 + 16, col)), v0, v1);
        bf16x8 vf;
        vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
        vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }

#endif
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const unsigned long long qmw = (myw >> 6) ? mv1 : mv0;
    const bool qvalid = (qmw >> (myw & 63)) & 1ull;
    const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;

    // every wave is done with chunk slot x%3 and Q slot x&1: refill them two blocks ahead.
    // First the slot's K rows 16w..16w+15 (exactly what this wave's chunk DMA will overwrite)
    // stage the wave's 16 x 64 O tile, so it leaves as whole 128-B lines (8 rows x 128 B per
    // store instruction) instead of 16 rows x 32 B partial lines.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* ostg = smem + AP_KV + (x % 3) * 16384 + wave * 2048;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(qvalid ? o[dt][r] * inv : 0.f);
      *reinterpret_cast<bf16x4*>(ostg + li * 128 + (((2 * dt + (g >> 1)) ^ (li & 7)) << 4) + (g & 1) * 8) = w;
    }
    bf16x8 ov[2];
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      ov[p2] = *reinterpret_cast<const bf16x8*>(ostg + orow * 128 + (((lane & 7) ^ (orow & 7)) << 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staged O read back before the DMA lands
    if (x + 3 <= x1) dma_chunk(x + 3);
    if (x + 2 < x1) dma_q(x + 2);
#if !(defined(RF_BAND_DIAG) && (RF_BAND_DIAG & 2))
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      *reinterpret_cast<bf16x8*>(out + (rb + i0 + 16 * wave + orow) * ldo + hoff + (lane & 7) * 8) = ov[p2];
    }
#else
    if (ov[0][0] == (bf16)1234.5f && inv == 3.f) out[rb] = (bf16)1.f;
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------
// k_band_attn_pipe2: the pipelined kernel above with its per-block instruction count cut
// (it is issue-bound at two waves per SIMD, not HBM-bound):
//  - each wave scores exactly its band: keys [16w-32, 16w+48) of the block = 5 key tiles
//    (was 6), the PV tail step pairs tile 4 with zero probabilities;
//  - global keys are scored in the same pass (one max / exp / sum over local + global, no
//    online rescale of O); their K fragments and V^T fragments are loop-invariant registers;
//  - masks: one bit-extract + bit-select per score; ring-slot and DMA offsets are wave-uniform
//    or 24-bit products precomputed per lane; V^T reads are batched 8 per wait.
template <typename V4>
__device__ __forceinline__ void tr_read8(const uint32_t* a, V4* v) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\t"
      "ds_read_b64_tr_b16 %1, %9\n\t"
      "ds_read_b64_tr_b16 %2, %10\n\t"
      "ds_read_b64_tr_b16 %3, %11\n\t"
      "ds_read_b64_tr_b16 %4, %12\n\t"
      "ds_read_b64_tr_b16 %5, %13\n\t"
      "ds_read_b64_tr_b16 %6, %14\n\t"
      "ds_read_b64_tr_b16 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7])
      : "memory");
}

__device__ __forceinline__ float mask_score(unsigned int bits, int bit, float sv) {
  const int m = (int)(bits << (31 - bit)) >> 31;  // 0 or -1 (v_bfe_i32)
  return __int_as_float((m & __float_as_int(sv)) | (~m & (int)0xff800000u));  // v_bfi_b32
}

// Q / K / V chunks are read once per block walk: non-temporal DMA (with the LayerNorm's
// non-temporal loads, +1.2% per C2 step in an alternating whole-step A/B of library builds)
#if defined(RF_BAND_PLAIN_LOAD)
#define BAND_GLDS glds16
#else
#define BAND_GLDS glds16_nt
#endif
// DROP (training): attention-probability dropout (TF:585-586) on the probabilities that enter
// P.V; the normaliser is the undropped row sum, as softmax-then-dropout.
template <typename E, bool DROP>
__global__ void __launch_bounds__(256) k_band_attn_pipe2(int Lp, int H, int qpb, const E* __restrict__ q,
                                                          const E* __restrict__ k,
                                                          const E* __restrict__ v, int ld,
                                                          const uint8_t* __restrict__ flags,
                                                          const int32_t* __restrict__ gidx, int gmax,
                                                          E* __restrict__ out, int ldo, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = Lp >> 6;
  const int nparts = (nqb + qpb - 1) / qpb;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int part = wg % nparts, bh = wg / nparts;
  const int h = bh % H, b = bh / H;
  const int x0 = part * qpb, x1 = min(nqb, x0 + qpb);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const E* kb = k + rb * ld + h * 64;
  const E* vb = v + rb * ld + h * 64;
  const E* qb = q + rb * ld + h * 64;
  E* ob = out + rb * ldo + h * 64;
  int* gp = reinterpret_cast<int*>(smem + AP_GP);
  unsigned long long* mk = reinterpret_cast<unsigned long long*>(smem + AP_MK);
  const int gt = gmax > 16 ? 2 : (gmax > 0 ? 1 : 0);  // 16-key tiles of global keys

  // ---- prologue: chunk masks, global keys ----
  for (int c = x0 + wave; c <= x1; c += 4) {
    const int row = 64 * c - 32 + lane;
    const int f = (row >= 0 && row < Lp) ? flags[rb + row] : 0;
    const unsigned long long ml = __ballot(f == 1), mv = __ballot(f != 0);
    if (lane == 0) {
      mk[2 * (c - x0)] = ml;
      mk[2 * (c - x0) + 1] = mv;
    }
  }
  if (gmax > 0) {
    const int row = wave * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int p = row < gmax ? gidx[(int64_t)b * gmax + row] : -1;
    const uint32_t off = (__umul24(p >= 0 ? p : 0, ld) + ch * 8) * (uint32_t)sizeof(E);
    glds16(reinterpret_cast<const char*>(kb) + off, smem + AP_KG + wave * 1024);
    glds16(reinterpret_cast<const char*>(vb) + off, smem + AP_VG + wave * 1024);
    if (threadIdx.x < 32) gp[threadIdx.x] = (int)threadIdx.x < gmax ? gidx[(int64_t)b * gmax + threadIdx.x] : -1;
  }
  const int prow = 16 * wave + (lane >> 3);  // DMA piece rows prow, prow + 8 (pieces 2w, 2w+1)
  const int pch = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
  auto dma_chunk = [&](int c) {
    char* base = smem + AP_KV + (c % 3) * 16384 + wave * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kp = min(max(64 * c - 32 + prow + 8 * j, 0), Lp - 1);
      // byte offsets in 32 bits from the wave-uniform (b, h) bases: the SGPR-base load form, no
      // 64-bit address arithmetic per piece
      const uint32_t off = (__umul24(kp, ld) + pch) * (uint32_t)sizeof(E);
      BAND_GLDS(reinterpret_cast<const char*>(kb) + off, base + j * 1024);
      BAND_GLDS(reinterpret_cast<const char*>(vb) + off, base + 8192 + j * 1024);
    }
  };
  auto dma_q = [&](int x) {
    char* base = smem + AP_Q + (x & 1) * 8192 + wave * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      BAND_GLDS(reinterpret_cast<const char*>(qb) + (__umul24(64 * x + prow + 8 * j, ld) + pch) * (uint32_t)sizeof(E),
                base + j * 1024);
  };
  dma_q(x0);
  dma_chunk(x0);
  dma_chunk(x0 + 1);  // x0 + 1 <= x1 always
  if (x0 + 1 < x1) dma_q(x0 + 1);
  if (x0 + 2 <= x1) dma_chunk(x0 + 2);

  // per-lane LDS offsets: fragment reads of 16-row tiles (row li, 16-B chunk 4 s2 + g) and the
  // transposed V reads (rows rr, rr + 16 of a 32-row key step; columns 16 dt + 4 (li & 3))
  const int rr = 4 * g + (li >> 2);
  int koff[2], voff[4];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) koff[s2] = li * 128 + (((4 * s2 + g) ^ (li & 7)) << 4);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) voff[dt] = swz_el(rr, 16 * dt + 4 * (li & 3));
  const uint32_t lds0 = lds_addr(smem);
  const int myw = 32 + 16 * wave + li;  // this lane's query row in the 128-row window
  // band bits of the wave's 80-key span [16w, 16w + 80): relative rows [li, li + 64]
  const unsigned int band0 = ~0u << li, band2 = (2u << li) - 1u;

  V8 kgf[2][2], vgf[4];
  unsigned int gbits = 0;
  for (int x = x0; x < x1; ++x) {
    // retire chunks x, x+1 and Q(x); still in flight (issue order, newest last): the O stores of
    // block x-2, chunk x+2, Q(x+1), the O stores of block x-1
    wait_vm_small((x - 2 >= x0 ? 2 : 0) + (x + 2 <= x1 ? 4 : 0) + (x + 1 < x1 ? 2 : 0) + (x > x0 ? 2 : 0));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (x == x0 && gt > 0) {  // loop-invariant global-key operands (DMA'd first, so landed)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          kgf[t][s2] = *reinterpret_cast<const V8*>(smem + AP_KG + t * 2048 + koff[s2]);
      uint32_t a[8];
      V4 vv[8];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        a[2 * dt] = lds0 + AP_VG + voff[dt];
        a[2 * dt + 1] = lds0 + AP_VG + 16 * 128 + voff[dt];
      }
      tr_read8(a, vv);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        vgf[dt] = V8{vv[2 * dt][0], vv[2 * dt][1], vv[2 * dt][2], vv[2 * dt][3],
                         vv[2 * dt + 1][0], vv[2 * dt + 1][1], vv[2 * dt + 1][2], vv[2 * dt + 1][3]};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) gbits |= (gp[16 * t + 4 * g + r] >= 0 ? 1u : 0u) << (4 * t + r);
    }
    const int i0 = 64 * x;
    const int sb0 = AP_KV + (x % 3) * 16384, sb1 = AP_KV + ((x + 1) % 3) * 16384;
    const unsigned long long ml0 = mk[2 * (x - x0)], ml1 = mk[2 * (x - x0) + 2];
    const unsigned long long mv0 = mk[2 * (x - x0) + 1], mv1 = mk[2 * (x - x0) + 3];
    V8 qf[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      qf[s2] = *reinterpret_cast<const V8*>(smem + AP_Q + (x & 1) * 8192 + 16 * wave * 128 + koff[s2]);

    // ---- scores: 5 local key tiles (window rows 16w + 16t) + gt global tiles ----
    f32x4 st[5], sg[2];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int rt = 16 * wave + 16 * t;
      const char* kt = smem + (rt >= 64 ? sb1 : sb0) + (rt & 63) * 128;
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        st[t] = mfma16(*reinterpret_cast<const V8*>(kt + koff[s2]), qf[s2],
                                                        st[t]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < gt) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          sg[t] = mfma16(kgf[t][s2], qf[s2], sg[t]);
      }
    }
    // allowed local keys: valid & local (chunk ballots) & band, as 3 words over the span,
    // shifted right by 4g so score (t, r) is bit 16 (t & 1) + r of word t >> 1
    unsigned int aw[3];
    {
      const int ks = 16 * wave;
      const unsigned long long lo = ks ? ((ml0 >> ks) | (ml1 << (64 - ks))) : ml0;
      const unsigned long long hi = ml1 >> ks;
      aw[0] = ((unsigned int)lo & band0) >> (4 * g);
      aw[1] = (unsigned int)(lo >> 32) >> (4 * g);
      aw[2] = ((unsigned int)hi & band2) >> (4 * g);
    }
    float mx = RF_NEG_INF;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[t][r] = mask_score(aw[t >> 1], 16 * (t & 1) + r, st[t][r]);
        mx = fmaxf(mx, st[t][r]);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sg[t][r] = t < gt ? mask_score(gbits, 4 * t + r, sg[t][r]) : RF_NEG_INF;
        mx = fmaxf(mx, sg[t][r]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float nmu = (mx == RF_NEG_INF) ? 0.f : -mx * LOG2E;
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[t][r] = __builtin_amdgcn_exp2f(fmaf(st[t][r], LOG2E, nmu));
        lsum += st[t][r];
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sg[t][r] = __builtin_amdgcn_exp2f(fmaf(sg[t][r], LOG2E, nmu));
        lsum += sg[t][r];
      }

    // ---- O = P V: 3 key steps of 32 (the last pairs tile 4 with p = 0) + the global step ----
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // dropout mask row of this lane's query (b, h, i0 + 16 wave + li); keys are absolute positions
    const uint64_t drow = DROP ? ((uint64_t)bh * Lp + i0 + 16 * wave + li) : 0;
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      V8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = 2 * s2 + (j >> 2);
        float pv = t < 5 ? st[t < 5 ? t : 4][j & 3] : 0.f;
        if (DROP && t < 5) pv *= attn_keep_scale(dr, drow, Lp, i0 - 32 + 16 * wave + 16 * t + 4 * g + (j & 3));
        pf[j] = (E)pv;
      }
      const int ga = 16 * wave + 32 * s2, gb = s2 < 2 ? ga + 16 : ga;  // finite rows for p = 0
      const uint32_t va = lds0 + (ga >= 64 ? sb1 : sb0) + 8192 + (ga & 63) * 128;
      const uint32_t vb2 = lds0 + (gb >= 64 ? sb1 : sb0) + 8192 + (gb & 63) * 128;
      uint32_t a[8];
      V4 vv[8];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        a[2 * dt] = va + voff[dt];
        a[2 * dt + 1] = vb2 + voff[dt];
      }
      tr_read8(a, vv);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const V8 vf = V8{vv[2 * dt][0], vv[2 * dt][1], vv[2 * dt][2], vv[2 * dt][3],
                                 vv[2 * dt + 1][0], vv[2 * dt + 1][1], vv[2 * dt + 1][2], vv[2 * dt + 1][3]};
        o[dt] = mfma16(vf, pf, o[dt]);
      }
    }
    if (gt > 0) {
      V8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float pv = sg[j >> 2][j & 3];
        if (DROP) {
          const int gk = gp[16 * (j >> 2) + 4 * g + (j & 3)];
          pv *= gk >= 0 ? attn_keep_scale(dr, drow, Lp, gk) : 0.f;
        }
        pf[j] = (E)pv;
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(vgf[dt], pf, o[dt]);
    }

    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const unsigned long long qmw = (myw >> 6) ? mv1 : mv0;
    const bool qvalid = (qmw >> (myw & 63)) & 1ull;
    const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;

    // every wave is done with chunk slot x%3 and Q slot x&1: stage O in the slot's K rows
    // 16w..16w+15 (what this wave's chunk DMA overwrites next), then refill two blocks ahead
    // and store O as whole 128-B lines
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* ostg = smem + sb0 + wave * 2048;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      V4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (E)(o[dt][r] * inv);
      *reinterpret_cast<V4*>(ostg + li * 128 + (((2 * dt + (g >> 1)) ^ (li & 7)) << 4) + (g & 1) * 8) = w;
    }
    V8 ov[2];
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      ov[p2] = *reinterpret_cast<const V8*>(ostg + orow * 128 + (((lane & 7) ^ (orow & 7)) << 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (x + 3 <= x1) dma_chunk(x + 3);
    if (x + 2 < x1) dma_q(x + 2);
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      *reinterpret_cast<V8*>(reinterpret_cast<char*>(ob) +
                             (__umul24(i0 + 16 * wave + orow, ldo) + (lane & 7) * 8) * (uint32_t)sizeof(E)) = ov[p2];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------
// k_band_attn_pipe3: k_band_attn_pipe2 at three workgroups per CU. pipe2 holds 74 KB of LDS (the K/V
// ring, a two-slot Q ring and the global keys' K/V image), so only two 256-thread workgroups fit a
// CU: two waves per SIMD for a kernel that is issue- and latency-bound, not bandwidth-bound. Here
// the Q fragments go straight to registers (two 16-B loads per lane per block, issued one block
// ahead as inline asm so that hipcc's wait bookkeeping does not drain the K/V DMA queue, retired by
// the kernel's counted vmcnt and fenced with "+v" before use), and the loop-invariant global-key K
// and V^T fragments are loaded from global memory once per workgroup: 48.3 KB of LDS (the ring,
// the chunk masks, the global positions) -> three workgroups per CU (VGPR budget <= 168).
// (read-write operand: the load targets the registers the variable already lives in, so hipcc has
// no reason to copy it between the load and the fence that follows the counted wait)
// Non-temporal (the Q rows are read once, as pipe2's Q DMA: a temporal load left them in L2 / MALL
// in place of the attention output the next GEMM reads — pipe3 ran faster itself but the out-proj
// after it slower, round 3). RF_BAND_PLAIN_LOAD: the plain form, for A/B builds.
template <typename V8>
__device__ __forceinline__ void gload16(V8& dst, const void* p) {
#if defined(RF_BAND_PLAIN_LOAD)
  asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(dst) : "v"(p) : "memory");
#else
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "+v"(dst) : "v"(p) : "memory");
#endif
}

constexpr int AQ_KV = 0;          // 3 x (K 64 x 128 B, V 64 x 128 B)
constexpr int AQ_GP = 49152;      // 32 x int global positions
constexpr int AQ_MK = 49280;      // per chunk {local mask, valid mask} uint64

template <typename E, bool DROP>
__global__ void __launch_bounds__(256, 3) k_band_attn_pipe3(int Lp, int H, int qpb, const E* __restrict__ q,
                                                             const E* __restrict__ k,
                                                             const E* __restrict__ v, int ld,
                                                             const uint8_t* __restrict__ flags,
                                                             const int32_t* __restrict__ gidx, int gmax,
                                                             E* __restrict__ out, int ldo, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = Lp >> 6;
  const int nparts = (nqb + qpb - 1) / qpb;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int part = wg % nparts, bh = wg / nparts;
  const int h = bh % H, b = bh / H;
  const int x0 = part * qpb, x1 = min(nqb, x0 + qpb);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const E* kb = k + rb * ld + h * 64;
  const E* vb = v + rb * ld + h * 64;
  const E* qb = q + rb * ld + h * 64;
  E* ob = out + rb * ldo + h * 64;
  int* gp = reinterpret_cast<int*>(smem + AQ_GP);
  unsigned long long* mk = reinterpret_cast<unsigned long long*>(smem + AQ_MK);
  const int gt = gmax > 16 ? 2 : (gmax > 0 ? 1 : 0);  // 16-key tiles of global keys

  // ---- prologue: global positions, the global keys' K / V^T fragments (loop-invariant, ordinary
  // loads issued before anything else, so their wait never drains the DMA queue), Q(x0) into
  // registers, chunk masks, the first chunks ----
  if (gmax > 0 && threadIdx.x < 32) gp[threadIdx.x] = (int)threadIdx.x < gmax ? gidx[(int64_t)b * gmax + threadIdx.x] : -1;
  __syncthreads();  // gp (nothing in flight yet)
  V8 kgf[2][2], vgf[4];
  unsigned int gbits = 0;
  if (gt > 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int p = gp[16 * t + li];
      const E* kr = kb + (int64_t)(p >= 0 ? p : 0) * ld;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) kgf[t][s2] = *reinterpret_cast<const V8*>(kr + 8 * (4 * s2 + g));
    }
    // V^T fragment dt: lane (li, g) holds V[gp[key]][16 dt + li] for keys 4g..4g+3, 16+4g..16+4g+3 (the
    // MFMA K order of pipe2's transposed reads, matching the P fragment built from the S^T tiles)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = gp[(j < 4 ? 0 : 16) + 4 * g + (j & 3)];
      const E* vr = vb + (int64_t)(p >= 0 ? p : 0) * ld + li;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) vgf[dt][j] = vr[16 * dt];
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) gbits |= (gp[16 * t + 4 * g + r] >= 0 ? 1u : 0u) << (4 * t + r);
  }
  // this lane's Q fragment of block x: row 64 x + 16 wave + li, 16-B chunks 4 s2 + g
  const E* qlane = qb + (int64_t)(16 * wave + li) * ld + 8 * g;
  V8 qn[2];
  gload16(qn[0], qlane + (int64_t)64 * x0 * ld);
  gload16(qn[1], qlane + (int64_t)64 * x0 * ld + 32);
  for (int c = x0 + wave; c <= x1; c += 4) {
    const int row = 64 * c - 32 + lane;
    const int f = (row >= 0 && row < Lp) ? flags[rb + row] : 0;
    const unsigned long long ml = __ballot(f == 1), mv = __ballot(f != 0);
    if (lane == 0) {
      mk[2 * (c - x0)] = ml;
      mk[2 * (c - x0) + 1] = mv;
    }
  }
  const int prow = 16 * wave + (lane >> 3);  // DMA piece rows prow, prow + 8 (pieces 2w, 2w+1)
  const int pch = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
  auto dma_chunk = [&](int c) {
    char* base = smem + AQ_KV + (c % 3) * 16384 + wave * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kp = min(max(64 * c - 32 + prow + 8 * j, 0), Lp - 1);
      const uint32_t off = __umul24(kp, ld) + pch;
      BAND_GLDS(kb + off, base + j * 1024);
      BAND_GLDS(vb + off, base + 8192 + j * 1024);
    }
  };
  dma_chunk(x0);
  dma_chunk(x0 + 1);  // x0 + 1 <= x1 always
  if (x0 + 2 <= x1) dma_chunk(x0 + 2);

  // per-lane LDS offsets: fragment reads of 16-row tiles (row li, 16-B chunk 4 s2 + g) and the
  // transposed V reads (rows rr, rr + 16 of a 32-row key step; columns 16 dt + 4 (li & 3))
  const int rr = 4 * g + (li >> 2);
  int koff[2], voff[4];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) koff[s2] = li * 128 + (((4 * s2 + g) ^ (li & 7)) << 4);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) voff[dt] = swz_el(rr, 16 * dt + 4 * (li & 3));
  const uint32_t lds0 = lds_addr(smem);
  const int myw = 32 + 16 * wave + li;  // this lane's query row in the 128-row window
  // band bits of the wave's 80-key span [16w, 16w + 80): relative rows [li, li + 64]
  const unsigned int band0 = ~0u << li, band2 = (2u << li) - 1u;

  for (int x = x0; x < x1; ++x) {
    // retire chunks x, x+1 and Q(x); still in flight (issue order, newest last): chunk x+2 and the
    // O stores of block x-1 (x > x0), or chunk x0+2 (x = x0)
    if (x == x0) wait_vm_small(x0 + 2 <= x1 ? 4 : 0);
    else wait_vm_small((x + 2 <= x1 ? 4 : 0) + 2);
    asm volatile("" : "+v"(qn[0]), "+v"(qn[1]));  // Q(x) landed: no use of it above this point
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int i0 = 64 * x;
    const int sb0 = AQ_KV + (x % 3) * 16384, sb1 = AQ_KV + ((x + 1) % 3) * 16384;
    const unsigned long long ml0 = mk[2 * (x - x0)], ml1 = mk[2 * (x - x0) + 2];
    const unsigned long long mv0 = mk[2 * (x - x0) + 1], mv1 = mk[2 * (x - x0) + 3];

    // ---- scores: 5 local key tiles (window rows 16w + 16t) + gt global tiles ----
    f32x4 st[5], sg[2];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int rt = 16 * wave + 16 * t;
      const char* kt = smem + (rt >= 64 ? sb1 : sb0) + (rt & 63) * 128;
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        st[t] = mfma16(*reinterpret_cast<const V8*>(kt + koff[s2]), qn[s2], st[t]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < gt) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          sg[t] = mfma16(kgf[t][s2], qn[s2], sg[t]);
      }
    }
    if (x + 1 < x1) {  // Q(x+1) into the same registers, once this block's scores have read them
      gload16(qn[0], qlane + (int64_t)64 * (x + 1) * ld);
      gload16(qn[1], qlane + (int64_t)64 * (x + 1) * ld + 32);
    }
    unsigned int aw[3];
    {
      const int ks = 16 * wave;
      const unsigned long long lo = ks ? ((ml0 >> ks) | (ml1 << (64 - ks))) : ml0;
      const unsigned long long hi = ml1 >> ks;
      aw[0] = ((unsigned int)lo & band0) >> (4 * g);
      aw[1] = (unsigned int)(lo >> 32) >> (4 * g);
      aw[2] = ((unsigned int)hi & band2) >> (4 * g);
    }
    float mx = RF_NEG_INF;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[t][r] = mask_score(aw[t >> 1], 16 * (t & 1) + r, st[t][r]);
        mx = fmaxf(mx, st[t][r]);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sg[t][r] = t < gt ? mask_score(gbits, 4 * t + r, sg[t][r]) : RF_NEG_INF;
        mx = fmaxf(mx, sg[t][r]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float nmu = (mx == RF_NEG_INF) ? 0.f : -mx * LOG2E;
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st[t][r] = __builtin_amdgcn_exp2f(fmaf(st[t][r], LOG2E, nmu));
        lsum += st[t][r];
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sg[t][r] = __builtin_amdgcn_exp2f(fmaf(sg[t][r], LOG2E, nmu));
        lsum += sg[t][r];
      }

    // ---- O = P V: 3 key steps of 32 (the last pairs tile 4 with p = 0) + the global step ----
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint64_t drow = DROP ? ((uint64_t)bh * Lp + i0 + 16 * wave + li) : 0;
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      V8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = 2 * s2 + (j >> 2);
        float pv = t < 5 ? st[t < 5 ? t : 4][j & 3] : 0.f;
        if (DROP && t < 5) pv *= attn_keep_scale(dr, drow, Lp, i0 - 32 + 16 * wave + 16 * t + 4 * g + (j & 3));
        pf[j] = (E)pv;
      }
      const int ga = 16 * wave + 32 * s2, gb = s2 < 2 ? ga + 16 : ga;  // finite rows for p = 0
      const uint32_t va = lds0 + (ga >= 64 ? sb1 : sb0) + 8192 + (ga & 63) * 128;
      const uint32_t vb2 = lds0 + (gb >= 64 ? sb1 : sb0) + 8192 + (gb & 63) * 128;
      uint32_t a[8];
      V4 vv[8];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        a[2 * dt] = va + voff[dt];
        a[2 * dt + 1] = vb2 + voff[dt];
      }
      tr_read8(a, vv);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const V8 vf = V8{vv[2 * dt][0], vv[2 * dt][1], vv[2 * dt][2], vv[2 * dt][3],
                         vv[2 * dt + 1][0], vv[2 * dt + 1][1], vv[2 * dt + 1][2], vv[2 * dt + 1][3]};
        o[dt] = mfma16(vf, pf, o[dt]);
      }
    }
    if (gt > 0) {
      V8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float pv = sg[j >> 2][j & 3];
        if (DROP) {
          const int gk = gp[16 * (j >> 2) + 4 * g + (j & 3)];
          pv *= gk >= 0 ? attn_keep_scale(dr, drow, Lp, gk) : 0.f;
        }
        pf[j] = (E)pv;
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(vgf[dt], pf, o[dt]);
    }

    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const unsigned long long qmw = (myw >> 6) ? mv1 : mv0;
    const bool qvalid = (qmw >> (myw & 63)) & 1ull;
    const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;

    // every wave is done with chunk slot x%3: stage O in the slot's K rows 16w..16w+15 (what this
    // wave's chunk DMA overwrites next), then refill three blocks ahead and store O as whole lines
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* ostg = smem + sb0 + wave * 2048;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      V4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (E)(o[dt][r] * inv);
      *reinterpret_cast<V4*>(ostg + li * 128 + (((2 * dt + (g >> 1)) ^ (li & 7)) << 4) + (g & 1) * 8) = w;
    }
    V8 ov[2];
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      ov[p2] = *reinterpret_cast<const V8*>(ostg + orow * 128 + (((lane & 7) ^ (orow & 7)) << 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (x + 3 <= x1) dma_chunk(x + 3);
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int orow = 8 * p2 + (lane >> 3);
      *reinterpret_cast<V8*>(ob + __umul24(i0 + 16 * wave + orow, ldo) + (lane & 7) * 8) = ov[p2];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------
// Short sequences (Lp < 64, any length: catalog items of <s> + up to 63 tokens, unpadded instead of
// padded to the 64-token window; finetune.py:38-63): every key of the sequence
// is in one 64-row tile, so one workgroup per (sequence, head) scores all of them. Same contract
// as the band kernels: a local query i sees keys j with flag 1 and |i - j| <= 32, plus every global
// key (flag 2, local K/V); padded query rows are written as 0. Keys / values DMA'd to LDS, Q^T
// fragments straight from HBM; S^T = K Q^T and O^T = V^T P^T on MFMA.
constexpr int AS_K = 0, AS_V = 8192, AS_FL = 16384, AS_LDS = 16448;

template <typename E>
__global__ void __launch_bounds__(256) k_attn_short(int Lp, int H, const E* __restrict__ q, const E* __restrict__ k,
                                                    const E* __restrict__ v, int ld, const uint8_t* __restrict__ flags,
                                                    E* __restrict__ out, int ldo) {
  typedef typename H16<E>::x8 V8;
  typedef typename H16<E>::x4 V4;
  __shared__ __attribute__((aligned(16))) char smem[AS_LDS];
  const int bh = blockIdx.x, h = bh % H, b = bh / H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  uint8_t* fl = reinterpret_cast<uint8_t*>(smem + AS_FL);
  // K / V rows 0..63 (clamped into the sequence; rows >= Lp are masked): 2 pieces of 8 rows per wave
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 16 * wave + 8 * j + (lane >> 3);
    const int ch = (lane & 7) ^ (row & 7);
    const int64_t off = (rb + min(row, Lp - 1)) * ld + hoff + ch * 8;
    glds16(k + off, smem + AS_K + (16 * wave + 8 * j) * 128);
    glds16(v + off, smem + AS_V + (16 * wave + 8 * j) * 128);
  }
  if (threadIdx.x < 64) fl[threadIdx.x] = (int)threadIdx.x < Lp ? flags[rb + threadIdx.x] : 0;
  const int myq = 16 * wave + li;
  const int qr = min(myq, Lp - 1);
  V8 qf[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) qf[s2] = *reinterpret_cast<const V8*>(q + (rb + qr) * ld + hoff + 32 * s2 + 8 * g);
  wait_vmcnt0();
  __syncthreads();
  if (16 * wave >= Lp) return;  // whole wave past the sequence (after the barrier)
  f32x4 st[4];
  float mx = RF_NEG_INF;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      st[t] = mfma16(*reinterpret_cast<const V8*>(smem + AS_K + swz128(16 * t + li, 4 * s2 + g)), qf[s2], st[t]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kj = 16 * t + 4 * g + r;
      const int f = kj < Lp ? fl[kj] : 0;
      const bool ok = (f == 1 && abs(kj - myq) <= 32) || f == 2;
      st[t][r] = ok ? st[t][r] : RF_NEG_INF;
      mx = fmaxf(mx, st[t][r]);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float nmu = (mx == RF_NEG_INF) ? 0.f : -mx * LOG2E;
  float lsum = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      st[t][r] = __builtin_amdgcn_exp2f(fmaf(st[t][r], LOG2E, nmu));
      lsum += st[t][r];
    }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rr = 4 * g + (li >> 2);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    V8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (E)st[2 * s2 + (j >> 2)][j & 3];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const V4 v0 = tr_read<E>(smem + AS_V, swz_el(32 * s2 + rr, col));
      const V4 v1 = tr_read<E>(smem + AS_V, swz_el(32 * s2 + 16 + rr, col));
      const V8 vf = V8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      o[dt] = mfma16(vf, pf, o[dt]);
    }
  }
  if (myq >= Lp) return;
  const bool qvalid = fl[myq] != 0;
  const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;
  E* orow = out + (rb + myq) * ldo + hoff + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    V4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = (E)(o[dt][r] * inv);
    *reinterpret_cast<V4*>(orow + 16 * dt) = w;
  }
}

// ------------------------------------------------------------------------------------
// Local branch, generic element type, VALU (fp32 parity path; any even window).
// One wave per (query, head): lanes own keys; scores reduced with wave shuffles.
template <typename T>
__global__ void __launch_bounds__(256) k_band_attn_valu(int Lp, int half_w, const T* __restrict__ q,
                                                         const T* __restrict__ k,
                                                         const T* __restrict__ v, int ld,
                                                         const uint8_t* __restrict__ flags,
                                                         const int32_t* __restrict__ gidx,
                                                         int gmax, T* __restrict__ out, int ldo, AttnDrop dr) {
  drop_resolve(dr);  // device step counter (captured training steps)
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int h = blockIdx.y, b = blockIdx.z;
  const uint64_t drow = ((uint64_t)b * gridDim.y + h) * Lp + i;  // dropout mask row (TF:585-586)
  if (i >= Lp) return;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  const T* qr = q + (rb + i) * ld + hoff;
  const int nwin = 2 * half_w + 1;
  const int ntot = nwin + gmax;
  // pass 1: max
  float mx = RF_NEG_INF;
  for (int j0 = 0; j0 < ntot; j0 += 64) {
    const int j = j0 + lane;
    float sv = RF_NEG_INF;
    int kp = -1;
    if (j < nwin) {
      const int p = i - half_w + j;
      if (p >= 0 && p < Lp && flags[rb + p] == 1) kp = p;
    } else if (j < ntot) {
      kp = gidx[(int64_t)b * gmax + (j - nwin)];
    }
    if (kp >= 0) {
      const T* kr = k + (rb + kp) * ld + hoff;
      float acc = 0.f;
      for (int d = 0; d < 64; ++d) acc += to_f32(qr[d]) * to_f32(kr[d]);
      sv = acc;
    }
    mx = fmaxf(mx, wave_max(sv));
  }
  const float mu = (mx == RF_NEG_INF) ? 0.f : mx;
  // pass 2: probabilities and output (lane = head dim)
  float acc = 0.f, lsum = 0.f;
  for (int j0 = 0; j0 < ntot; j0 += 64) {
    const int j = j0 + lane;
    float p = 0.f;
    int kp = -1;
    if (j < nwin) {
      const int pp = i - half_w + j;
      if (pp >= 0 && pp < Lp && flags[rb + pp] == 1) kp = pp;
    } else if (j < ntot) {
      kp = gidx[(int64_t)b * gmax + (j - nwin)];
    }
    if (kp >= 0) {
      const T* kr = k + (rb + kp) * ld + hoff;
      float s = 0.f;
      for (int d = 0; d < 64; ++d) s += to_f32(qr[d]) * to_f32(kr[d]);
      p = expf(s - mu);
    }
    lsum += wave_sum(p);
    if (dr.thresh && kp >= 0) p *= attn_keep_scale(dr, drow, Lp, kp);  // after the normaliser's sum
    const int n = min(64, ntot - j0);
    for (int jj = 0; jj < n; ++jj) {
      const float pj = __shfl(p, jj, 64);
      const int kpj = __shfl(kp, jj, 64);
      if (kpj >= 0) acc += pj * to_f32(v[(rb + kpj) * ld + hoff + lane]);
    }
  }
  const bool qvalid = flags[rb + i] != 0;
  out[(rb + i) * ldo + hoff + lane] = from_f32<T>(qvalid && lsum > 0.f ? acc / lsum : 0.f);
}

// ------------------------------------------------------------------------------------
// Global query rows (A6). One 256-thread block per (global slot g, head, sequence).
template <typename T>
__global__ void __launch_bounds__(256) k_global_attn(int Lp, const T* __restrict__ qg, int ld_qg,
                                                      const T* __restrict__ kg,
                                                      const T* __restrict__ vg, int ld,
                                                      const uint8_t* __restrict__ flags,
                                                      const int32_t* __restrict__ gidx, int gmax,
                                                      T* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float sc[];  // Lp scores + 64 q + 256 partials
  float* qs = sc + Lp;
  float* part = qs + 64;
  __shared__ float red[8];
  const int gs = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int pos = gidx[(int64_t)b * gmax + gs];
  if (pos < 0) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t rb = (int64_t)b * Lp;
  const int hoff = h * 64;
  if (t < 64) qs[t] = to_f32(qg[((int64_t)b * gmax + gs) * ld_qg + hoff + t]);
  __syncthreads();
  float mx = RF_NEG_INF;
  for (int j = t; j < Lp; j += 256) {
    float s = RF_NEG_INF;
    if (flags[rb + j] != 0) {
      const T* kr = kg + (rb + j) * ld + hoff;
      float a = 0.f;
#pragma unroll 8
      for (int d = 0; d < 64; ++d) a += qs[d] * to_f32(kr[d]);
      s = a;
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float mu = (mx == RF_NEG_INF) ? 0.f : mx;
  float ls = 0.f;
  for (int j = t; j < Lp; j += 256) {
    const float p = expf(sc[j] - mu);
    sc[j] = p;
    ls += p;
  }
  ls = wave_sum(ls);
  __syncthreads();
  if (lane == 0) red[4 + wave] = ls;
  __syncthreads();
  const float lsum = red[4] + red[5] + red[6] + red[7];
  // out[d] = sum_j p_j vg[j][d]; thread = (part = wave, d = lane)
  float acc = 0.f;
  for (int j = wave; j < Lp; j += 4) {
    const float p = sc[j];
    if (p != 0.f) acc += p * to_f32(vg[(rb + j) * ld + hoff + lane]);
  }
  part[t] = acc;
  __syncthreads();
  if (t < 64) {
    const float s = part[t] + part[t + 64] + part[t + 128] + part[t + 192];
    out[(rb + pos) * ldo + hoff + t] = from_f32<T>(lsum > 0.f ? s / lsum : 0.f);
  }
}

}  // namespace rf

using namespace rf;

extern "C" int rf_band_attn_fwd_drop(int dtype, int B, int Lp, int H, int hd, int half_w,
                                     const void* q, const void* k, const void* v, int ld_qkv,
                                     const uint8_t* flags, const int32_t* gidx, int gmax, void* out,
                                     int ld_out, float p_drop, uint64_t seed, rf_stream_t stream);

extern "C" int rf_band_attn_fwd(int dtype, int B, int Lp, int H, int hd, int half_w,
                                const void* q, const void* k, const void* v, int ld_qkv,
                                const uint8_t* flags, const int32_t* gidx, int gmax, void* out,
                                int ld_out, rf_stream_t stream) {
  return rf_band_attn_fwd_drop(dtype, B, Lp, H, hd, half_w, q, k, v, ld_qkv, flags, gidx, gmax, out, ld_out, 0.f,
                               0, stream);
}

extern "C" int rf_band_attn_fwd_drop(int dtype, int B, int Lp, int H, int hd, int half_w,
                                     const void* q, const void* k, const void* v, int ld_qkv,
                                     const uint8_t* flags, const int32_t* gidx, int gmax, void* out,
                                     int ld_out, float p_drop, uint64_t seed, rf_stream_t stream) {
  RF_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "rf_band_attn_fwd: dropout p=%g outside [0, 1)", p_drop);
  const AttnDrop dr{seed, drop_thresh(p_drop), 1.0f / (1.0f - p_drop), g_seed_dev};
  RF_REQUIRE(hd == 64, "rf_band_attn_fwd: head_dim must be 64 (got %d)", hd);
  RF_REQUIRE(B >= 0 && H > 0 && Lp >= 0 && gmax >= 0, "rf_band_attn_fwd: bad shape");
  RF_REQUIRE(ld_qkv >= H * hd && ld_out >= H * hd, "rf_band_attn_fwd: bad leading dims");
  RF_REQUIRE((int64_t)Lp * (ld_qkv > ld_out ? ld_qkv : ld_out) * 4 < 0x7FFFFFFF,
             "rf_band_attn_fwd: one sequence's rows must span < 2 GiB (32-bit offsets from the sequence base)");
  RF_REQUIRE(gmax == 0 || gidx, "rf_band_attn_fwd: gidx required");
  if (B == 0 || Lp == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16 || dtype == RF_F16) {
    const bool h16 = dtype == RF_F16;
    if (half_w != 32) {
      // other windows: the chunked kernel (inference; the training path's other windows recompute
      // the local branch in fp32, train._local_torch)
      RF_REQUIRE(half_w > 0, "rf_band_attn_fwd: bad half window %d", half_w);
      RF_REQUIRE(dr.thresh == 0, "rf_band_attn_fwd(16-bit): window %d runs without dropout", 2 * half_w);
      RF_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0, "rf_band_attn_fwd(16-bit): alignment");
      const int grid = ((Lp + 63) / 64) * H * B;
      if (h16)
        k_band_attn_wide<f16><<<grid, 256, 0, s>>>(Lp, half_w, (const f16*)q, (const f16*)k, (const f16*)v, ld_qkv,
                                                   flags, gidx, gmax, (f16*)out, ld_out, H);
      else
        k_band_attn_wide<bf16><<<grid, 256, 0, s>>>(Lp, half_w, (const bf16*)q, (const bf16*)k, (const bf16*)v, ld_qkv,
                                                    flags, gidx, gmax, (bf16*)out, ld_out, H);
      RF_LAUNCH_CHECK("rf_band_attn_fwd");
    }
    RF_REQUIRE(Lp % 64 == 0 || (Lp < 64 && dr.thresh == 0),
               "rf_band_attn_fwd(16-bit): Lp=%d must be a multiple of 64, or < 64 (short sequences, any "
               "length; no dropout)", Lp);
    RF_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0, "rf_band_attn_fwd(bf16): alignment");
    RF_REQUIRE(dr.thresh == 0 || gmax <= 32, "rf_band_attn_fwd(bf16): dropout needs gmax <= 32 (got %d)", gmax);
    if (Lp < 64) {
      RF_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0, "rf_band_attn_fwd(short): alignment");
      if (h16)
        k_attn_short<f16><<<H * B, 256, 0, s>>>(Lp, H, (const f16*)q, (const f16*)k, (const f16*)v, ld_qkv, flags,
                                                 (f16*)out, ld_out);
      else
        k_attn_short<bf16><<<H * B, 256, 0, s>>>(Lp, H, (const bf16*)q, (const bf16*)k, (const bf16*)v, ld_qkv, flags,
                                                  (bf16*)out, ld_out);
    } else if (gmax <= 32 && (g_knob[KNOB_BAND_PATH] != 2 || dr.thresh)) {
      // pipelined: runs of qpb query blocks per workgroup, >= ~3 workgroups per CU slot
      const int nqb = Lp / 64;
      int qpb = nqb >= 16 ? (nqb + 1) / 2 : nqb;
      if (g_knob[KNOB_BAND_QPB] > 0) qpb = min(nqb, g_knob[KNOB_BAND_QPB]);  // A/B tools
      const int nparts = (nqb + qpb - 1) / qpb;
      const size_t lds = AP_MK + (size_t)(qpb + 1) * 16;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_band_attn_pipe, hipFuncAttributeMaxDynamicSharedMemorySize, 80000);
        attr = true;
      }
      RF_REQUIRE(lds <= 80000, "rf_band_attn_fwd(bf16): Lp=%d too long for the pipelined kernel", Lp);
      if (g_knob[KNOB_BAND_PATH] == 1 && dr.thresh == 0 && !h16) {
        k_band_attn_pipe<<<nparts * H * B, 256, lds, s>>>(Lp, H, qpb, (const bf16*)q, (const bf16*)k,
                                                           (const bf16*)v, ld_qkv, flags, gidx, gmax,
                                                           (bf16*)out, ld_out);
      } else {
        static bool attr2 = false;
        if (!attr2) {
          (void)hipFuncSetAttribute((const void*)k_band_attn_pipe2<bf16, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 80000);
          (void)hipFuncSetAttribute((const void*)k_band_attn_pipe2<bf16, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 80000);
          (void)hipFuncSetAttribute((const void*)k_band_attn_pipe2<f16, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 80000);
          (void)hipFuncSetAttribute((const void*)k_band_attn_pipe2<f16, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 80000);
          attr2 = true;
        }
#define P2_(E, D)                                                                                        \
  do {                                                                                                    \
    if (band_pipe3) {                                                                                     \
      k_band_attn_pipe3<E, D><<<nparts * H * B, 256, lds3, s>>>(Lp, H, qpb, (const E*)q, (const E*)k,       \
                                                               (const E*)v, ld_qkv, flags, gidx, gmax,     \
                                                               (E*)out, ld_out, dr);                       \
    } else {                                                                                              \
      k_band_attn_pipe2<E, D><<<nparts * H * B, 256, lds, s>>>(Lp, H, qpb, (const E*)q, (const E*)k,        \
                                                              (const E*)v, ld_qkv, flags, gidx, gmax,      \
                                                              (E*)out, ld_out, dr);                        \
    }                                                                                                     \
  } while (0)
        // pipe3 (three workgroups per CU; bit-identical to pipe2) by default (band_path 3; 0 = pipe2): round 6's
        // kernel traces of whole C2 steps, one setting per process in ABBA order (tools/gpu/band_trace.sh,
        // profiles/r06/band_trace_abba.txt): band 83.2 / 83.3 vs 86.7 / 87.1 us, every other kernel within
        // 0.5 us (no slower GEMM after it), kernel time per 50 steps 608.0 / 610.3 vs 611.7 / 611.7 ms,
        // 12.100 / 12.142 vs 12.149 / 12.163 ms per step (the earlier A/Bs, -0.2 .. +0.4%, were within noise)
        const bool band_pipe3 = g_knob[KNOB_BAND_PATH] == 3;
        const size_t lds3 = AQ_MK + (size_t)(qpb + 1) * 16;
        // training (dropout) keeps pipe2: pipe3's dropout form would spill at the 3-wave register budget
        if (h16) {
          if (dr.thresh) k_band_attn_pipe2<f16, true><<<nparts * H * B, 256, lds, s>>>(Lp, H, qpb, (const f16*)q,
              (const f16*)k, (const f16*)v, ld_qkv, flags, gidx, gmax, (f16*)out, ld_out, dr);
          else P2_(f16, false);
        } else {
          if (dr.thresh) k_band_attn_pipe2<bf16, true><<<nparts * H * B, 256, lds, s>>>(Lp, H, qpb, (const bf16*)q,
              (const bf16*)k, (const bf16*)v, ld_qkv, flags, gidx, gmax, (bf16*)out, ld_out, dr);
          else P2_(bf16, false);
        }
#undef P2_
      }
    } else {
      if (h16)
        k_band_attn_bf16<f16><<<(Lp / 64) * H * B, 256, 0, s>>>(Lp, (const f16*)q, (const f16*)k, (const f16*)v,
                                                                ld_qkv, flags, gidx, gmax, (f16*)out, ld_out, H);
      else
        k_band_attn_bf16<bf16><<<(Lp / 64) * H * B, 256, 0, s>>>(Lp, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                                                                 ld_qkv, flags, gidx, gmax, (bf16*)out, ld_out, H);
    }
  } else if (dtype == RF_F32) {
    RF_REQUIRE(half_w > 0, "rf_band_attn_fwd: bad half window");
    dim3 grid((Lp + 3) / 4, H, B);
    k_band_attn_valu<float><<<grid, 256, 0, s>>>(Lp, half_w, (const float*)q, (const float*)k,
                                                 (const float*)v, ld_qkv, flags, gidx, gmax,
                                                 (float*)out, ld_out, dr);
  } else {
    RF_REQUIRE(false, "rf_band_attn_fwd: bad dtype %d", dtype);
  }
  RF_LAUNCH_CHECK("rf_band_attn_fwd");
}

extern "C" int rf_global_attn_fwd(int dtype, int B, int Lp, int H, int hd, const void* qg,
                                  int ld_qg, const void* kg, const void* vg, int ld_kv,
                                  const uint8_t* flags, const int32_t* gidx, int gmax, void* out,
                                  int ld_out, rf_stream_t stream) {
  RF_REQUIRE(hd == 64, "rf_global_attn_fwd: head_dim must be 64 (got %d)", hd);
  RF_REQUIRE(B >= 0 && H > 0 && Lp >= 0 && gmax >= 0, "rf_global_attn_fwd: bad shape");
  RF_REQUIRE(Lp <= 16384, "rf_global_attn_fwd: Lp=%d too long for the LDS score row", Lp);
  if (B == 0 || Lp == 0 || gmax == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  dim3 grid(gmax, H, B);
  const size_t lds = (size_t)(Lp + 64 + 256) * sizeof(float);
  if (dtype == RF_BF16)
    k_global_attn<bf16><<<grid, 256, lds, s>>>(Lp, (const bf16*)qg, ld_qg, (const bf16*)kg,
                                               (const bf16*)vg, ld_kv, flags, gidx, gmax,
                                               (bf16*)out, ld_out);
  else if (dtype == RF_F16)
    k_global_attn<f16><<<grid, 256, lds, s>>>(Lp, (const f16*)qg, ld_qg, (const f16*)kg, (const f16*)vg, ld_kv, flags,
                                              gidx, gmax, (f16*)out, ld_out);
  else if (dtype == RF_F32)
    k_global_attn<float><<<grid, 256, lds, s>>>(Lp, (const float*)qg, ld_qg, (const float*)kg,
                                                (const float*)vg, ld_kv, flags, gidx, gmax,
                                                (float*)out, ld_out);
  else
    RF_REQUIRE(false, "rf_global_attn_fwd: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_global_attn_fwd");
}
