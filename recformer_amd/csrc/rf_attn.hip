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

__device__ __forceinline__ bf16x4 tr_read(const char* lds_base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds_base + off));
}

__global__ void __launch_bounds__(256) k_band_attn_bf16(int Lp, const bf16* __restrict__ q,
                                                         const bf16* __restrict__ k,
                                                         const bf16* __restrict__ v, int ld,
                                                         const uint8_t* __restrict__ flags,
                                                         const int32_t* __restrict__ gidx,
                                                         int gmax, bf16* __restrict__ out,
                                                         int ldo) {
  __shared__ __attribute__((aligned(16))) char smem[AT_LDS];
  const int i0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z;
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
  bf16x8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(q + (rb + myq) * ld + hoff + 32 * s + 8 * g);

  wait_vmcnt0();
  __syncthreads();

  // ---- window segment: 6 key tiles of 16 ----
  f32x4 st[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(smem + AT_KW + swz128(ks + 16 * t + li, 4 * s + g));
      st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], st[t], 0, 0, 0);
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
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (bf16)st[2 * s + (j >> 2)][j & 3];
    const int r0 = ks + 32 * s + 4 * g + (li >> 2);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const bf16x4 v0 = tr_read(smem + AT_VW, swz_el(r0, col));
      const bf16x4 v1 = tr_read(smem + AT_VW, swz_el(r0 + 16, col));
      bf16x8 vf;
      vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
      vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
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
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(smem + AT_KG + swz128(16 * t + li, 4 * s + g));
        sg[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sg[t], 0, 0, 0);
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
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 8; ++j) pf[j] = (bf16)sg[j >> 2][j & 3];
    const int r0 = 4 * g + (li >> 2);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = 16 * dt + 4 * (li & 3);
      const bf16x4 v0 = tr_read(smem + AT_VG, swz_el(r0, col));
      const bf16x4 v1 = tr_read(smem + AT_VG, swz_el(r0 + 16, col));
      bf16x8 vf;
      vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v0[2]; vf[3] = v0[3];
      vf[4] = v1[0]; vf[5] = v1[1]; vf[6] = v1[2]; vf[7] = v1[3];
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
    }
  }

  // ---- normalise and store O[q][16dt + 4g + r] ----
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  const bool qvalid = fl[32 + 16 * wave + li] != 0;
  const float inv = (qvalid && lsum > 0.f) ? 1.0f / lsum : 0.f;
  bf16* orow = out + (rb + myq) * ldo + hoff + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    bf16x4 w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = (bf16)(qvalid ? o[dt][r] * inv : 0.f);
    *reinterpret_cast<bf16x4*>(orow + 16 * dt) = w;
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
                                                         int gmax, T* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int h = blockIdx.y, b = blockIdx.z;
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

extern "C" int rf_band_attn_fwd(int dtype, int B, int Lp, int H, int hd, int half_w,
                                const void* q, const void* k, const void* v, int ld_qkv,
                                const uint8_t* flags, const int32_t* gidx, int gmax, void* out,
                                int ld_out, rf_stream_t stream) {
  RF_REQUIRE(hd == 64, "rf_band_attn_fwd: head_dim must be 64 (got %d)", hd);
  RF_REQUIRE(B >= 0 && H > 0 && Lp >= 0 && gmax >= 0, "rf_band_attn_fwd: bad shape");
  RF_REQUIRE(ld_qkv >= H * hd && ld_out >= H * hd, "rf_band_attn_fwd: bad leading dims");
  RF_REQUIRE(gmax == 0 || gidx, "rf_band_attn_fwd: gidx required");
  if (B == 0 || Lp == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16) {
    RF_REQUIRE(half_w == 32, "rf_band_attn_fwd(bf16): window must be 64 (half 32), got half %d", half_w);
    RF_REQUIRE(Lp % 64 == 0, "rf_band_attn_fwd(bf16): Lp=%d must be a multiple of 64", Lp);
    RF_REQUIRE(ld_qkv % 8 == 0 && ld_out % 4 == 0, "rf_band_attn_fwd(bf16): alignment");
    dim3 grid(Lp / 64, H, B);
    k_band_attn_bf16<<<grid, 256, 0, s>>>(Lp, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                                          ld_qkv, flags, gidx, gmax, (bf16*)out, ld_out);
  } else if (dtype == RF_F32) {
    RF_REQUIRE(half_w > 0, "rf_band_attn_fwd: bad half window");
    dim3 grid((Lp + 3) / 4, H, B);
    k_band_attn_valu<float><<<grid, 256, 0, s>>>(Lp, half_w, (const float*)q, (const float*)k,
                                                 (const float*)v, ld_qkv, flags, gidx, gmax,
                                                 (float*)out, ld_out);
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
  else if (dtype == RF_F32)
    k_global_attn<float><<<grid, 256, lds, s>>>(Lp, (const float*)qg, ld_qg, (const float*)kg,
                                                (const float*)vg, ld_kv, flags, gidx, gmax,
                                                (float*)out, ld_out);
  else
    RF_REQUIRE(false, "rf_global_attn_fwd: bad dtype %d", dtype);
  RF_LAUNCH_CHECK("rf_global_attn_fwd");
}
