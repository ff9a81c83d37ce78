// Backward of the fused 4-table embedding + LayerNorm (RecformerEmbeddings, models.py:108-138):
//   x = Ew[id] + Ep[pos] + Et[tt] + Ei[ip],  h = LN(x; gamma, beta, eps)
// gives dL/dgamma, dL/dbeta and, per table, dL/dE[v] = sum over the tokens t with index v of dL/dx_t
// (nn.Embedding's dense backward; rows at padding_idx receive none, as nn.Embedding(padding_idx=1)).
// Everything is deterministic: fixed-order sums, no atomics.
//
// k_embed_ln_bwd: one wave per token row (grid-stride over at most EB_BLOCKS x 4 waves): regathers the
//   four table rows (the pre-LN sum is not stored), recomputes the row statistics, writes
//   dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dh gamma, and sums dh xhat / dh per block
//   (the 4 waves combined in LDS in wave order) for gamma / beta; k_embed_affine_fin adds the block
//   partials in block order.
// Table gradients: the caller sorts a table's token indices (stable), giving keys (sorted) and perm;
//   the rows src[perm[j]] are then summed per run of equal keys in three fixed-order levels:
//   k_seg_partial  one wave per slice of 16 sorted positions: the sum of each run of equal keys inside
//                  the slice, stored at the run's first position (part, indexed by position);
//   k_seg_chain    one wave per 256 positions: the slice-start pieces that continue a segment
//                  (keys[b] == keys[b-1], b a multiple of 16) summed per chain of consecutive slices,
//                  stored at the chain's first slice (part2, indexed by slice);
//   k_seg_final    one wave per segment head h: part[h] + the chain starting at the first slice after h
//                  + one chain per 256-boundary inside the segment, written to dst[key].
//   Loads are issued in batches (indices broadcast from lanes, rows loaded 8 at a time) so a wave pays a
//   few memory latencies per slice, not one per row; long segments (type / item-position tables) cost
//   segment_length / 256 chain reads at the head (64 per ballot round).
#include "rf_common.h"

namespace rf {

constexpr int EB_SLICE = 16;     // sorted positions per k_seg_partial wave
constexpr int EB_SUPER = 256;    // positions per k_seg_chain wave (16 slices)
constexpr int EB_BLOCKS = 512;   // k_embed_ln_bwd blocks (4 waves each, grid-stride over the rows)

template <int NV>
__device__ __forceinline__ void row_load(float4 (&r)[NV / 4], const float* p, int lane, int D) {
#pragma unroll
  for (int j = 0; j < NV / 4; ++j) {
    const int c = 4 * lane + 256 * j;
    r[j] = c < D ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int NV>
__device__ __forceinline__ void row_add(float (&acc)[NV], const float4 (&r)[NV / 4]) {
#pragma unroll
  for (int j = 0; j < NV / 4; ++j) {
    acc[4 * j] += r[j].x;
    acc[4 * j + 1] += r[j].y;
    acc[4 * j + 2] += r[j].z;
    acc[4 * j + 3] += r[j].w;
  }
}

template <int NV>
__device__ __forceinline__ void row_store(float* p, const float (&acc)[NV], int lane, int D) {
#pragma unroll
  for (int j = 0; j < NV / 4; ++j) {
    const int c = 4 * lane + 256 * j;
    if (c < D) *reinterpret_cast<float4*>(p + c) = make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
  }
}

template <int NV>
__global__ void __launch_bounds__(256) k_embed_ln_bwd(int M, int D, const int32_t* __restrict__ ids,
                                                      const int32_t* __restrict__ pos, const int32_t* __restrict__ tt,
                                                      const int32_t* __restrict__ ip, const float* __restrict__ word,
                                                      const float* __restrict__ pe, const float* __restrict__ te,
                                                      const float* __restrict__ ie, const float* __restrict__ gamma,
                                                      float eps, const float* __restrict__ dh, float* __restrict__ dx,
                                                      float* __restrict__ part) {
  __shared__ float red[4][2][NV * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // lane owns columns 4 lane + 256 j, j < NV / 4
  float gw[NV], ag[NV], ab[NV];
  {
    float4 g4[NV / 4];
    row_load<NV>(g4, gamma, lane, D);
#pragma unroll
    for (int j = 0; j < NV / 4; ++j) {
      gw[4 * j] = g4[j].x; gw[4 * j + 1] = g4[j].y; gw[4 * j + 2] = g4[j].z; gw[4 * j + 3] = g4[j].w;
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) ag[k] = ab[k] = 0.f;
  const float invD = 1.0f / (float)D;
  for (int m = blockIdx.x * 4 + w; m < M; m += gridDim.x * 4) {
    float4 a[NV / 4], b[NV / 4], e[NV / 4], f[NV / 4], g[NV / 4];
    row_load<NV>(a, word + (int64_t)ids[m] * D, lane, D);
    row_load<NV>(b, pe + (int64_t)pos[m] * D, lane, D);
    row_load<NV>(e, te + (int64_t)tt[m] * D, lane, D);
    row_load<NV>(f, ie + (int64_t)ip[m] * D, lane, D);
    row_load<NV>(g, dh + (int64_t)m * D, lane, D);
    float x[NV], d[NV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV / 4; ++j) {
      // the forward's summation order (models.py:135): ((word + pos) + type) + item-pos
      x[4 * j] = ((a[j].x + b[j].x) + e[j].x) + f[j].x;
      x[4 * j + 1] = ((a[j].y + b[j].y) + e[j].y) + f[j].y;
      x[4 * j + 2] = ((a[j].z + b[j].z) + e[j].z) + f[j].z;
      x[4 * j + 3] = ((a[j].w + b[j].w) + e[j].w) + f[j].w;
      d[4 * j] = g[j].x; d[4 * j + 1] = g[j].y; d[4 * j + 2] = g[j].z; d[4 * j + 3] = g[j].w;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += x[4 * j + k];
    }
    const float mean = wave_sum(s) * invD;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < NV / 4; ++j)
      if (4 * lane + 256 * j < D) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float t = x[4 * j + k] - mean;
          v += t * t;
        }
      }
    const float rstd = rsqrtf(wave_sum(v) * invD + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      x[k] = (x[k] - mean) * rstd;  // xhat (d = 0 in the columns past D)
      const float gg = d[k] * gw[k];
      sg += gg;
      sgx += gg * x[k];
      ag[k] += d[k] * x[k];
      ab[k] += d[k];
    }
    const float mg = wave_sum(sg) * invD, mgx = wave_sum(sgx) * invD;
    float o[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) o[k] = rstd * (d[k] * gw[k] - mg - x[k] * mgx);
    row_store<NV>(dx + (int64_t)m * D, o, lane, D);
  }
  // block partial of gamma / beta: the 4 waves in wave order
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    red[w][0][k * 64 + lane] = ag[k];
    red[w][1][k * 64 + lane] = ab[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * NV * 64; i += 256) {
    const int which = i / (NV * 64), r = i - which * NV * 64;
    const int k = r / 64, l = r - k * 64;
    const int c = 4 * l + 256 * (k / 4) + (k & 3);
    if (c < D)
      part[((int64_t)blockIdx.x * 2 + which) * D + c] =
          ((red[0][which][r] + red[1][which][r]) + red[2][which][r]) + red[3][which][r];
  }
}

// gamma / beta: block partials summed in block order — 64 columns per workgroup of 16 waves, wave w
// summing a contiguous sixteenth of the partials, the 16 combined in wave order
__global__ void __launch_bounds__(1024) k_embed_affine_fin(int D, int nb, const float* __restrict__ part,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;  // over 2 D: gamma columns then beta columns
  const int which = c >= D ? 1 : 0, col = c - which * D;
  const int q = (nb + 15) / 16, b0 = w * q, b1 = min(nb, b0 + q);
  float s = 0.f;
  if (c < 2 * D) {
#pragma unroll 8
    for (int b = b0; b < b1; ++b) s += part[((int64_t)b * 2 + which) * D + col];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < 2 * D) {
    float t = red[0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][lane];
    (which ? dbeta : dgamma)[col] = t;
  }
}

// level 1: runs of equal keys inside each 16-position slice -> part[run start]
template <int NV>
__global__ void __launch_bounds__(256) k_seg_partial(int M, int D, const float* __restrict__ src,
                                                     const int32_t* __restrict__ perm, const int32_t* __restrict__ keys,
                                                     int pad, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int j0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * EB_SLICE;
  if (j0 >= M) return;
  const int n = min(EB_SLICE, M - j0);
  const int kl = lane < n ? keys[j0 + lane] : 0;
  const int pl = lane < n ? perm[j0 + lane] : 0;
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  int start = j0, key = __builtin_amdgcn_readfirstlane(kl);
#pragma unroll
  for (int g = 0; g < EB_SLICE / 8; ++g) {
    if (8 * g >= n) break;
    float4 r[8][NV / 4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = 8 * g + i;
      const int kj = __builtin_amdgcn_readlane(kl, j), pj = __builtin_amdgcn_readlane(pl, j);
      if (j < n && kj != pad) row_load<NV>(r[i], src + (int64_t)pj * D, lane, D);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = 8 * g + i;
      if (j >= n) break;
      const int kj = __builtin_amdgcn_readlane(kl, j);
      if (kj != key) {
        row_store<NV>(part + (int64_t)start * D, acc, lane, D);
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = 0.f;
        start = j0 + j;
        key = kj;
      }
      if (kj != pad) row_add<NV>(acc, r[i]);
    }
  }
  row_store<NV>(part + (int64_t)start * D, acc, lane, D);
}

// level 2: per 256 positions, the continuation pieces at slice starts summed per chain -> part2[slice]
template <int NV>
__global__ void __launch_bounds__(256) k_seg_chain(int M, int D, const int32_t* __restrict__ keys, int pad,
                                                   const float* __restrict__ part, float* __restrict__ part2) {
  const int lane = threadIdx.x & 63;
  const int s0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (EB_SUPER / EB_SLICE);  // first slice
  const int nsl = (M + EB_SLICE - 1) / EB_SLICE;
  if (s0 >= nsl) return;
  const int ns = min(EB_SUPER / EB_SLICE, nsl - s0);
  const int b = (s0 + lane) * EB_SLICE;
  int kl = 0, cont = 0;
  if (lane < ns && b > 0) {
    kl = keys[b];
    cont = (kl == keys[b - 1] && kl != pad) ? 1 : 0;
  }
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  int open = -1, key = 0;  // open chain: its first slice
#pragma unroll
  for (int g = 0; g < EB_SUPER / EB_SLICE / 8; ++g) {
    if (8 * g >= ns) break;
    float4 r[8][NV / 4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int l = 8 * g + i;
      if (l < ns && __builtin_amdgcn_readlane(cont, l))
        row_load<NV>(r[i], part + (int64_t)(s0 + l) * EB_SLICE * D, lane, D);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int l = 8 * g + i;
      if (l >= ns) break;
      const int c = __builtin_amdgcn_readlane(cont, l), kk = __builtin_amdgcn_readlane(kl, l);
      if (open >= 0 && (!c || kk != key)) {
        row_store<NV>(part2 + (int64_t)open * D, acc, lane, D);
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = 0.f;
        open = -1;
      }
      if (c) {
        if (open < 0) {
          open = s0 + l;
          key = kk;
        }
        row_add<NV>(acc, r[i]);
      }
    }
  }
  if (open >= 0) row_store<NV>(part2 + (int64_t)open * D, acc, lane, D);
}

// level 3: one wave per sorted position; segment heads write dst[key] (padding key skipped)
template <int NV>
__global__ void __launch_bounds__(256) k_seg_final(int M, int D, const int32_t* __restrict__ keys, int pad,
                                                   const float* __restrict__ part, const float* __restrict__ part2,
                                                   float* __restrict__ dst, int V) {
  const int lane = threadIdx.x & 63;
  const int h = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (h >= M) return;
  const int key = keys[h];
  if (h > 0 && keys[h - 1] == key) return;  // not the head of its segment
  if (key == pad || key < 0 || key >= V) return;
  float acc[NV];
  {
    float4 r[NV / 4];
    row_load<NV>(r, part + (int64_t)h * D, lane, D);
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.f;
    row_add<NV>(acc, r);
  }
  const int b1 = (h / EB_SLICE + 1) * EB_SLICE;
  if (b1 < M && keys[b1] == key) {
    {
      float4 r[NV / 4];
      row_load<NV>(r, part2 + (int64_t)(b1 / EB_SLICE) * D, lane, D);
      row_add<NV>(acc, r);
    }
    // chains starting at the 256-boundaries inside the segment, 64 boundaries per round
    for (int B0 = (b1 / EB_SUPER + 1) * EB_SUPER; B0 < M; B0 += 64 * EB_SUPER) {
      const int64_t Bl = (int64_t)B0 + (int64_t)lane * EB_SUPER;
      const bool in = Bl < M && keys[Bl] == key;
      const int cnt = __builtin_popcountll(__ballot(in));  // keys sorted: a prefix of the lanes
      for (int i = 0; i < cnt; i += 4) {
        float4 r[4][NV / 4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i + u < cnt) row_load<NV>(r[u], part2 + (int64_t)((B0 + (i + u) * EB_SUPER) / EB_SLICE) * D, lane, D);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i + u < cnt) row_add<NV>(acc, r[u]);
      }
      if (cnt < 64) break;
    }
  }
  row_store<NV>(dst + (int64_t)key * D, acc, lane, D);
}

inline int eb_blocks(int M) { return max(1, min(EB_BLOCKS, (M + 3) / 4)); }

}  // namespace rf

using namespace rf;

extern "C" size_t rf_embed_ln_bwd_workspace(int M, int D) { return (size_t)eb_blocks(M) * 2 * D * sizeof(float); }

extern "C" int rf_embed_ln_bwd(int M, int D, const int32_t* ids, const int32_t* pos, const int32_t* tt,
                               const int32_t* ip, const float* word, const float* pe, const float* te,
                               const float* ie, const float* ln_w, float eps, const float* dh, float* dx,
                               float* dgamma, float* dbeta, void* workspace, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && D > 0 && D <= 1024 && D % 4 == 0, "rf_embed_ln_bwd: bad shape M=%d D=%d", M, D);
  RF_REQUIRE(ids && pos && tt && ip && word && pe && te && ie && ln_w && dh && dx && dgamma && dbeta && workspace,
             "rf_embed_ln_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  float* part = reinterpret_cast<float*>(workspace);
  const int nb = eb_blocks(M);
#define ELB_(NV) k_embed_ln_bwd<NV><<<nb, 256, 0, s>>>(M, D, ids, pos, tt, ip, word, pe, te, ie, ln_w, eps, dh, dx, part)
  if (D <= 256)
    ELB_(4);
  else if (D <= 512)
    ELB_(8);
  else if (D <= 768)
    ELB_(12);
  else
    ELB_(16);
#undef ELB_
  k_embed_affine_fin<<<(2 * D + 63) / 64, 1024, 0, s>>>(D, nb, part, dgamma, dbeta);
  RF_LAUNCH_CHECK("rf_embed_ln_bwd");
}

extern "C" size_t rf_segment_rows_sum_workspace(int M, int D) {
  const size_t m = (size_t)(M > 0 ? M : 1);
  return (m + (m + EB_SLICE - 1) / EB_SLICE) * D * sizeof(float);
}

extern "C" int rf_segment_rows_sum(int M, int D, const float* src, const int32_t* perm, const int32_t* keys_sorted,
                                   int pad, float* dst, int V, void* workspace, rf_stream_t stream) {
  RF_REQUIRE(M >= 0 && D > 0 && D <= 1024 && D % 4 == 0 && V > 0, "rf_segment_rows_sum: bad shape M=%d D=%d V=%d",
             M, D, V);
  RF_REQUIRE(src && perm && keys_sorted && dst && workspace, "rf_segment_rows_sum: null pointer");
  if (M == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  float* part = reinterpret_cast<float*>(workspace);
  float* part2 = part + (size_t)M * D;
  const int nslice = (M + EB_SLICE - 1) / EB_SLICE;
  const int nsuper = (M + EB_SUPER - 1) / EB_SUPER;
#define SEG_(NV)                                                                               \
  k_seg_partial<NV><<<(nslice + 3) / 4, 256, 0, s>>>(M, D, src, perm, keys_sorted, pad, part); \
  k_seg_chain<NV><<<(nsuper + 3) / 4, 256, 0, s>>>(M, D, keys_sorted, pad, part, part2);       \
  k_seg_final<NV><<<(M + 3) / 4, 256, 0, s>>>(M, D, keys_sorted, pad, part, part2, dst, V);
  if (D <= 256) {
    SEG_(4)
  } else if (D <= 512) {
    SEG_(8)
  } else if (D <= 768) {
    SEG_(12)
  } else {
    SEG_(16)
  }
#undef SEG_
  RF_LAUNCH_CHECK("rf_segment_rows_sum");
}
