// Catalog retrieval with a fused ranking epilogue.
//
// Reference: Ranker (utils.py:76-108) over scores = Similarity(z, item_embeddings) / temp
// (models.py:358-369, evaluate / finetune.py:70-92, evaluate_seq.py:35-52) and the C5 target
// "score Q user queries against a 1M-item catalog sharded over 8 GPUs, output top-50 plus the
// rank of the label". The reference materialises the (B, N) score matrix; here it is never
// written. Per catalog shard:
//
//   k_label_score   s_label[b] = cos(q_b, E[label_b]) / temp for the labels in this shard, with
//                   the same MFMA chain (16x16x32, K ascending in 32-chunks) and the same epilogue
//                   expression as k_score_rank, so it is bit-identical to the score the ranking
//                   kernel computes for that column (strict ranks need exact equality).
//   k_score_rank    256x256 MFMA tiles (queries x items, K = d) with the Ranker epilogue: per row
//                   and tile, the strict-rank count #{s > s_label}, the valid count #{s > -MAX_VAL}
//                   and sum exp(s - shift) (the cross entropy's log-sum-exp with shift = 1/temp >=
//                   |s|) as deterministic per-tile partials, plus either the dense scores (MODE 0,
//                   the sample block that seeds the top-k threshold) or the top-k candidates
//                   s >= tau[row] appended to per-(tile, row) slots (MODE 1), or only the counts
//                   (MODE 2: metrics without a top-k).
//   k_rank_reduce   sums the per-tile partials per row in tile order (deterministic).
//   k_topk_dense / k_topk_merge
//                   exact top-k per row (value descending, ties by lower item index) by a radix
//                   select over order-preserving 32-bit keys in LDS; the merge reads the seed
//                   top-k and every tile's candidate slots and flags rows whose slots overflowed
//                   (the caller re-ranks those rows densely).
// Element types: bf16 and fp16 operands (v_mfma_f32_16x16x32_bf16 / _f16), fp32 scores.
#include "rf_common.h"

namespace rf {

template <typename T> struct RtElt;
template <> struct RtElt<bf16> {
  typedef bf16x8 V8;
  static __device__ __forceinline__ f32x4 mfma(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct RtElt<f16> {
  typedef f16x8 V8;
  static __device__ __forceinline__ f32x4 mfma(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

constexpr float RT_LOG2E = 1.4426950408889634f;

// the cosine score of one (query, item) pair from its fp32 dot product: one expression shared by
// every kernel of this file (and by rf_gemm's EPI_COS epilogue)
__device__ __forceinline__ float cos_score(float dot, float rq_scale, float rc) { return dot * rq_scale * rc; }

// ---- label scores ----------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(64) k_label_score(int B, int K, const T* __restrict__ q, int ldq,
                                                    const float* __restrict__ rq, const T* __restrict__ items,
                                                    int ldi, const float* __restrict__ ri, int nshard,
                                                    const int64_t* __restrict__ labels, int64_t label_base,
                                                    float scale, float* __restrict__ s_label) {
  typedef typename RtElt<T>::V8 V8;
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * 16;
  const int r = lane & 15, g = lane >> 4;
  const int qb = min(b0 + r, B - 1);
  const int64_t lr = labels[qb] - label_base;
  const bool mine = lr >= 0 && lr < nshard;
  const T* qa = q + (int64_t)qb * ldq + 8 * g;
  const T* ea = items + (mine ? lr : 0) * (int64_t)ldi + 8 * g;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32)
    acc = RtElt<T>::mfma(*reinterpret_cast<const V8*>(qa + k0), *reinterpret_cast<const V8*>(ea + k0), acc);
  // the diagonal C[i][i] sits in lane i + 16 (i >> 2), accumulator element i & 3
  const int i = r;
  if (g == (i >> 2)) {
    const int b = b0 + i;
    if (b < B) {
      const float v = acc[i & 3];
      s_label[b] = mine ? cos_score(v, rq[b] * scale, ri[lr]) : 0.f;
    }
  }
}

// ---- fused score + rank ----------------------------------------------------------------------
struct RankArgs {
  int B, ncols, col0;       // query rows; catalog rows [col0, col0 + ncols) of the shard
  const float* rq;          // query inverse norms (B)
  const float* rc;          // shard inverse norms
  float scale;              // 1 / temp
  const float* s_label;     // (B)
  float max_val, shift;
  const float* tau;         // MODE 1: candidate threshold per row
  float* dense;             // MODE 0: (B, ncols) scores
  int64_t ldd;
  float* cval;              // MODE 1: candidate slots [tn * B + row][cap] (tn: tile column of this launch)
  int32_t* cidx;
  int32_t* ccnt;            // MODE 1: [tn * B + row] candidates (> cap: overflow)
  int cap;
  int32_t idx_base;         // item id of shard row 0
  int32_t* part_cnt;        // [(tn0 + tn) * B + row] gt | valid << 16
  float* part_sexp;
  int tn0;
};

constexpr int RK_BM = 256, RK_BN = 256, RK_BK = 32, RK_NS = 4;
constexpr int RK_ROWB = 64;                        // 32 elements x 2 B
constexpr int RK_STAGE = (RK_BM + RK_BN) * RK_ROWB;  // 32 KiB
constexpr int RK_LDS = RK_NS * RK_STAGE;           // 128 KiB
constexpr int RK_EPI_LD = 68;                      // fp32 slab row stride
constexpr int RK_PART = 8 * 16 * RK_EPI_LD * 4;    // after the 8 waves' slabs
constexpr int RK_CNT = RK_PART + 256 * 4 * 12;     // per-row candidate counters

__device__ __forceinline__ int rk_slot(int r, int c) { return c ^ ((-(r >> 2)) & 3); }

template <typename T, int MODE>
__global__ void __launch_bounds__(512, 1) k_score_rank(int K, const T* __restrict__ Q, int ldq,
                                                       const T* __restrict__ E, int lde, RankArgs a, int nTm) {
  typedef typename RtElt<T>::V8 V8;
  constexpr int FM = 8, FN = 4, CPW = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // the nTm query tiles of one catalog tile are consecutive (same XCD): the catalog panel is read
  // from HBM once and served from that XCD's L2 to the other query tiles
  const int tn = wg / nTm, tm = wg - tn * nTm;
  const int m0 = tm * RK_BM, n0 = tn * RK_BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  const T* src[CPW];
  int dst[CPW];
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int c = wave * CPW + i;  // 1-KiB pieces of 16 rows: 0..15 queries, 16..31 items
    const bool isA = c < 16;
    const int row = (isA ? c : c - 16) * 16 + (lane >> 2);
    const int ch = rk_slot(row, lane & 3);
    if (isA)
      src[i] = Q + (int64_t)min(m0 + row, a.B - 1) * ldq + ch * 8;
    else
      src[i] = E + (int64_t)(a.col0 + min(n0 + row, a.ncols - 1)) * lde + ch * 8;
    dst[i] = c * 1024;
  }
  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * RK_STAGE;
#pragma unroll
    for (int i = 0; i < CPW; ++i) glds16(src[i] + kt * RK_BK, base + dst[i]);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / RK_BK;
  auto read_frags = [&](int kt, V8 (&fa)[FM], V8 (&fb)[FN]) {
    const char* as = smem + (kt & 3) * RK_STAGE;
    const char* ws = as + RK_BM * RK_ROWB;
    const int ch = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * 128 + i * 16 + (lane & 15);
      fa[i] = *reinterpret_cast<const V8*>(as + r * RK_ROWB + (rk_slot(r, ch) << 4));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int r = wn * 64 + j * 16 + (lane & 15);
      fb[j] = *reinterpret_cast<const V8*>(ws + r * RK_ROWB + (rk_slot(r, ch) << 4));
    }
  };
  auto mma = [&](const V8 (&fa)[FM], const V8 (&fb)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = RtElt<T>::mfma(fa[i], fb[j], acc[i][j]);
  };
  auto sync_tile = [&](int kt) {
    if (nk - 1 - kt >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // register-pipelined 4-slot ring: tile kt's MFMAs run while tile kt+1's fragments are read
  // and tile kt+3's DMA is in flight (the structure of rf_gemm.hip's BK = 32 ring)
  V8 a0[FM], b0[FN], a1[FM], b1[FN];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < nk) stage(i, i);
  if (nk >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (nk == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_frags(0, a0, b0);
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    sync_tile(kt + 1);
    if (kt + 3 < nk) stage(kt + 3, (kt + 3) & 3);
    read_frags(kt + 1, a1, b1);
    mma(a0, b0);
    if (kt + 2 < nk) {
      sync_tile(kt + 2);
      if (kt + 4 < nk) stage(kt + 4, (kt + 4) & 3);
      read_frags(kt + 2, a0, b0);
    }
    mma(a1, b1);
  }
  if (kt < nk) mma(a0, b0);
  __syncthreads();  // the ring becomes epilogue scratch

  int* cnt = reinterpret_cast<int*>(smem + RK_CNT);
  int* pc = reinterpret_cast<int*>(smem + RK_PART);             // [256 rows][4 wn] packed counts
  float* ps = reinterpret_cast<float*>(smem + RK_PART + 4096);  // [256 rows][4 wn] sexp
  if (threadIdx.x < 256) cnt[threadIdx.x] = 0;
  __syncthreads();

  float* scr = reinterpret_cast<float*>(smem) + wave * 16 * RK_EPI_LD;
  const int rr = lane >> 2, cc = (lane & 3) * 16;
  const int c0 = n0 + wn * 64 + cc;  // this lane's 16 columns within the launch's range
  float rcv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) rcv[k] = (c0 + k < a.ncols) ? a.rc[a.col0 + c0 + k] : 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[((lane >> 4) * 4 + r) * RK_EPI_LD + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    float v[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const float4 x = *reinterpret_cast<const float4*>(scr + rr * RK_EPI_LD + cc + 4 * q4);
      v[4 * q4] = x.x; v[4 * q4 + 1] = x.y; v[4 * q4 + 2] = x.z; v[4 * q4 + 3] = x.w;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const int rl = wm * 128 + i * 16 + rr;  // tile row
    const int row = m0 + rl;
    const bool rok = row < a.B;
    const int rowc = rok ? row : a.B - 1;
    const float rs = a.rq[rowc] * a.scale, sl = a.s_label[rowc];
    int gt = 0, valid = 0;
    float se = 0.f;
    unsigned int cmask = 0;
    const float tau = MODE == 1 ? a.tau[rowc] : 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const bool cok = c0 + k < a.ncols;
      const float s = cos_score(v[k], rs, rcv[k]);
      v[k] = s;
      gt += (cok && s > sl) ? 1 : 0;
      valid += (cok && s > -a.max_val) ? 1 : 0;
      se += cok ? __builtin_amdgcn_exp2f((s - a.shift) * RT_LOG2E) : 0.f;
      if (MODE == 1 && cok && s >= tau) cmask |= 1u << k;
    }
    if (MODE == 0 && rok) {
      float* d = a.dense + (int64_t)row * a.ldd + c0;
      if (c0 + 16 <= a.ncols) {
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4)
          *reinterpret_cast<float4*>(d + 4 * q4) = make_float4(v[4 * q4], v[4 * q4 + 1], v[4 * q4 + 2], v[4 * q4 + 3]);
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (c0 + k < a.ncols) d[k] = v[k];
      }
    }
    if (MODE == 1 && rok && cmask) {
      const int n = __builtin_popcount(cmask);
      const int base = atomicAdd(&cnt[rl], n);  // LDS atomic: slot order within (row, tile) is free
      const int64_t slot0 = ((int64_t)tn * a.B + row) * a.cap;
      int t = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (cmask & (1u << k)) {
          if (base + t < a.cap) {
            a.cval[slot0 + base + t] = v[k];
            a.cidx[slot0 + base + t] = a.idx_base + a.col0 + c0 + k;
          }
          ++t;
        }
      }
    }
    // the row's four lanes (16 columns each) -> one value per wave column group
    int pk = gt | (valid << 16);
    pk += __shfl_xor(pk, 1, 64);
    pk += __shfl_xor(pk, 2, 64);
    se += __shfl_xor(se, 1, 64);
    se += __shfl_xor(se, 2, 64);
    if ((lane & 3) == 0) {
      pc[rl * 4 + wn] = pk;
      ps[rl * 4 + wn] = se;
    }
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    const int rl = threadIdx.x, row = m0 + rl;
    if (row < a.B) {
      const int64_t o = (int64_t)(a.tn0 + tn) * a.B + row;
      a.part_cnt[o] = pc[rl * 4] + pc[rl * 4 + 1] + pc[rl * 4 + 2] + pc[rl * 4 + 3];
      a.part_sexp[o] = ((ps[rl * 4] + ps[rl * 4 + 1]) + ps[rl * 4 + 2]) + ps[rl * 4 + 3];
      if (MODE == 1) a.ccnt[(int64_t)tn * a.B + row] = cnt[rl];
    }
  }
}

__global__ void __launch_bounds__(256) k_rank_reduce(int B, int ntiles, const int32_t* __restrict__ part_cnt,
                                                     const float* __restrict__ part_sexp, int32_t* __restrict__ gt,
                                                     int32_t* __restrict__ valid, float* __restrict__ sexp) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  int g = 0, v = 0;
  float s = 0.f;
  for (int t = 0; t < ntiles; ++t) {
    const int p = part_cnt[(int64_t)t * B + row];
    g += p & 0xFFFF;
    v += p >> 16;
    s += part_sexp[(int64_t)t * B + row];
  }
  gt[row] = g;
  valid[row] = v;
  sexp[row] = s;
}

// ---- exact top-k per row --------------------------------------------------------------------
// order-preserving key: larger float -> larger unsigned key
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Top-k of the n (key, idx) pairs in LDS (n <= cap of the arrays), value descending, ties by
// lower idx; 256 threads. Writes k outputs (missing entries: -inf, -1). `tie` is scratch of n ints,
// `sel` of k ints.
__device__ void lds_topk(const uint32_t* keys, const int32_t* idx, int n, int k, int* tie, int* sel, float* out_v,
                         int32_t* out_i) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_need;
  __shared__ int s_nsel, s_ntie;
  const int t = threadIdx.x;
  const int kk = min(k, n);
  if (t == 0) {
    s_prefix = 0;
    s_need = kk;
    s_nsel = 0;
    s_ntie = 0;
  }
  uint32_t mask = 0;
  __syncthreads();
  if (kk > 0) {
    for (int shift = 24; shift >= 0; shift -= 8) {
      hist[t] = 0;
      __syncthreads();
      const uint32_t prefix = s_prefix;
      for (int e = t; e < n; e += 256) {
        const uint32_t key = keys[e];
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (t == 0) {
        uint32_t cum = 0, need = s_need;
        for (int b = 255; b >= 0; --b) {
          if (cum + hist[b] >= need) {
            s_prefix = prefix | ((uint32_t)b << shift);
            s_need = need - cum;
            break;
          }
          cum += hist[b];
        }
      }
      mask |= 255u << shift;
      __syncthreads();
    }
  }
  const uint32_t tau = s_prefix;
  const int need = (int)s_need;  // entries equal to tau to take
  // keys above tau, and the tie list
  for (int e = t; e < n && kk > 0; e += 256) {
    const uint32_t key = keys[e];
    if (key > tau) sel[atomicAdd(&s_nsel, 1)] = e;
    else if (key == tau) tie[atomicAdd(&s_ntie, 1)] = e;
  }
  __syncthreads();
  const int ngt = s_nsel, nt = s_ntie;
  // the `need` ties with the lowest idx (ranked among the ties)
  for (int a = t; a < nt; a += 256) {
    const int ea = tie[a];
    int r = 0;
    for (int b = 0; b < nt && r < need; ++b) r += idx[tie[b]] < idx[ea] ? 1 : 0;
    if (r < need) sel[ngt + r] = ea;
  }
  __syncthreads();
  // final order: key descending, idx ascending
  for (int a = t; a < kk; a += 256) {
    const int ea = sel[a];
    const uint32_t ka = keys[ea];
    const int ia = idx[ea];
    int r = 0;
    for (int b = 0; b < kk; ++b) {
      const int eb = sel[b];
      const uint32_t kb = keys[eb];
      r += (kb > ka || (kb == ka && idx[eb] < ia)) ? 1 : 0;
    }
    out_v[r] = kfloat(ka);
    out_i[r] = ia;
  }
  for (int a = kk + t; a < k; a += 256) {
    out_v[a] = -__builtin_inff();
    out_i[a] = -1;
  }
}

constexpr int TK_DENSE_MAX = 8192;
constexpr int TK_MERGE_MAX = 6144;
constexpr int TK_KMAX = 256;

__global__ void __launch_bounds__(256) k_topk_dense(int n, const float* __restrict__ vals, int64_t ldv,
                                                    const int32_t* __restrict__ idx, int64_t ldi, int32_t idx_base,
                                                    int k, float* __restrict__ out_v, int32_t* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* keys = reinterpret_cast<uint32_t*>(smem);
  int32_t* ids = reinterpret_cast<int32_t*>(smem + TK_DENSE_MAX * 4);
  int* tie = reinterpret_cast<int*>(smem + TK_DENSE_MAX * 8);
  int* sel = reinterpret_cast<int*>(smem + TK_DENSE_MAX * 12);
  const int row = blockIdx.x;
  for (int e = threadIdx.x; e < n; e += 256) {
    keys[e] = fkey(vals[(int64_t)row * ldv + e]);
    ids[e] = idx ? idx[(int64_t)row * ldi + e] : idx_base + e;
  }
  __syncthreads();
  lds_topk(keys, ids, n, k, tie, sel, out_v + (int64_t)row * k, out_i + (int64_t)row * k);
}

__global__ void __launch_bounds__(256) k_topk_merge(int B, int k0, const float* __restrict__ v0,
                                                    const int32_t* __restrict__ i0, int ntiles,
                                                    const float* __restrict__ cval, const int32_t* __restrict__ cidx,
                                                    const int32_t* __restrict__ ccnt, int cap, int k,
                                                    float* __restrict__ out_v, int32_t* __restrict__ out_i,
                                                    int32_t* __restrict__ overflow) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* keys = reinterpret_cast<uint32_t*>(smem);
  int32_t* ids = reinterpret_cast<int32_t*>(smem + TK_MERGE_MAX * 4);
  int* tie = reinterpret_cast<int*>(smem + TK_MERGE_MAX * 8);
  int* sel = reinterpret_cast<int*>(smem + TK_MERGE_MAX * 12);
  __shared__ int s_n, s_over;
  const int row = blockIdx.x, t = threadIdx.x;
  if (t == 0) {
    s_n = 0;
    s_over = 0;
  }
  __syncthreads();
  for (int e = t; e < k0; e += 256) {
    const int id = i0[(int64_t)row * k0 + e];
    if (id >= 0) {
      const int p = atomicAdd(&s_n, 1);
      keys[p] = fkey(v0[(int64_t)row * k0 + e]);
      ids[p] = id;
    }
  }
  for (int tt = t; tt < ntiles; tt += 256) {
    const int64_t o = (int64_t)tt * B + row;
    const int c = ccnt[o];
    if (c > cap) s_over = 1;
    const int m = min(c, cap);
    if (m > 0) {
      const int p = atomicAdd(&s_n, m);
      if (p + m <= TK_MERGE_MAX) {
        for (int j = 0; j < m; ++j) {
          keys[p + j] = fkey(cval[o * cap + j]);
          ids[p + j] = cidx[o * cap + j];
        }
      } else {
        s_over = 1;
      }
    }
  }
  __syncthreads();
  const int n = min(s_n, TK_MERGE_MAX);
  if (t == 0) overflow[row] = s_over;
  if (s_over) return;  // the caller re-ranks this row densely
  lds_topk(keys, ids, n, k, tie, sel, out_v + (int64_t)row * k, out_i + (int64_t)row * k);
}

}  // namespace rf

using namespace rf;

extern "C" int rf_label_scores(int dtype, int B, int D, const void* q, int ldq, const float* rq, const void* items,
                               int ldi, const float* ri, int nshard, const int64_t* labels, int64_t label_base,
                               float inv_temp, float* s_label, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && D > 0 && D % 32 == 0 && nshard >= 0, "rf_label_scores: bad shape (D %% 32 == 0)");
  RF_REQUIRE(ldq % 8 == 0 && ldi % 8 == 0, "rf_label_scores: leading dims must be multiples of 8");
  if (B == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  const int grid = (B + 15) / 16;
  if (dtype == RF_BF16)
    k_label_score<bf16><<<grid, 64, 0, s>>>(B, D, (const bf16*)q, ldq, rq, (const bf16*)items, ldi, ri, nshard,
                                            labels, label_base, inv_temp, s_label);
  else if (dtype == RF_F16)
    k_label_score<f16><<<grid, 64, 0, s>>>(B, D, (const f16*)q, ldq, rq, (const f16*)items, ldi, ri, nshard, labels,
                                           label_base, inv_temp, s_label);
  else
    RF_REQUIRE(false, "rf_label_scores: dtype must be bf16 or fp16");
  RF_LAUNCH_CHECK("rf_label_scores");
}

extern "C" int rf_score_rank(int dtype, int mode, int B, int D, const void* q, int ldq, const float* rq,
                             const void* items, int ldi, const float* ri, int col0, int ncols, float inv_temp,
                             const float* s_label, float max_val, float shift, const float* tau, float* dense,
                             int64_t ldd, float* cval, int32_t* cidx, int32_t* ccnt, int cap, int32_t idx_base,
                             int32_t* part_cnt, float* part_sexp, int tn0, rf_stream_t stream) {
  RF_REQUIRE(mode >= 0 && mode <= 2, "rf_score_rank: mode must be 0 (dense), 1 (candidates) or 2 (counts)");
  RF_REQUIRE(B >= 0 && ncols >= 0 && col0 >= 0 && D > 0 && D % 32 == 0, "rf_score_rank: bad shape (D %% 32 == 0)");
  RF_REQUIRE(ldq % 8 == 0 && ldi % 8 == 0, "rf_score_rank: leading dims must be multiples of 8");
  RF_REQUIRE(s_label && part_cnt && part_sexp && rq && ri, "rf_score_rank: null pointer");
  RF_REQUIRE(mode == 2 || (mode == 0 ? (dense && ldd >= ncols && ldd % 4 == 0) : (tau && cval && cidx && ccnt && cap > 0)),
             "rf_score_rank: mode %d outputs missing or misaligned", mode);
  if (B == 0 || ncols == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  RankArgs a{B, ncols, col0, rq, ri, inv_temp, s_label, max_val, shift, tau, dense, ldd,
             cval, cidx, ccnt, cap, idx_base, part_cnt, part_sexp, tn0};
  const int nTm = (B + RK_BM - 1) / RK_BM, nTn = (ncols + RK_BN - 1) / RK_BN;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_score_rank<bf16, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    (void)hipFuncSetAttribute((const void*)k_score_rank<bf16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    (void)hipFuncSetAttribute((const void*)k_score_rank<f16, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    (void)hipFuncSetAttribute((const void*)k_score_rank<f16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    (void)hipFuncSetAttribute((const void*)k_score_rank<bf16, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    (void)hipFuncSetAttribute((const void*)k_score_rank<f16, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, RK_LDS);
    attr = true;
  }
  const int grid = nTm * nTn;
#define RK_(T, M) k_score_rank<T, M><<<grid, 512, RK_LDS, s>>>(D, (const T*)q, ldq, (const T*)items, ldi, a, nTm)
  if (dtype == RF_BF16) {
    if (mode == 0) RK_(bf16, 0);
    else if (mode == 1) RK_(bf16, 1);
    else RK_(bf16, 2);
  } else if (dtype == RF_F16) {
    if (mode == 0) RK_(f16, 0);
    else if (mode == 1) RK_(f16, 1);
    else RK_(f16, 2);
  } else {
    RF_REQUIRE(false, "rf_score_rank: dtype must be bf16 or fp16");
  }
#undef RK_
  RF_LAUNCH_CHECK("rf_score_rank");
}

extern "C" int rf_score_rank_tiles(int ncols) { return (ncols + RK_BN - 1) / RK_BN; }

extern "C" int rf_rank_reduce(int B, int ntiles, const int32_t* part_cnt, const float* part_sexp, int32_t* gt,
                              int32_t* valid, float* sexp, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && ntiles >= 0, "rf_rank_reduce: bad shape");
  if (B == 0) return RF_OK;
  k_rank_reduce<<<(B + 255) / 256, 256, 0, as_stream(stream)>>>(B, ntiles, part_cnt, part_sexp, gt, valid, sexp);
  RF_LAUNCH_CHECK("rf_rank_reduce");
}

extern "C" int rf_topk_dense(int B, int n, const float* vals, int64_t ldv, const int32_t* idx, int64_t ldi,
                             int32_t idx_base, int k, float* out_v, int32_t* out_i, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && n >= 0 && n <= TK_DENSE_MAX && k > 0 && k <= TK_KMAX,
             "rf_topk_dense: n=%d must be <= %d and k=%d in [1, %d]", n, TK_DENSE_MAX, k, TK_KMAX);
  if (B == 0) return RF_OK;
  const size_t lds = (size_t)TK_DENSE_MAX * 12 + TK_KMAX * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_topk_dense, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  k_topk_dense<<<B, 256, lds, as_stream(stream)>>>(n, vals, ldv, idx, ldi, idx_base, k, out_v, out_i);
  RF_LAUNCH_CHECK("rf_topk_dense");
}

extern "C" int rf_topk_merge(int B, int k0, const float* v0, const int32_t* i0, int ntiles, const float* cval,
                             const int32_t* cidx, const int32_t* ccnt, int cap, int k, float* out_v, int32_t* out_i,
                             int32_t* overflow, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && k0 >= 0 && k0 <= TK_MERGE_MAX && ntiles >= 0 && cap > 0 && k > 0 && k <= TK_KMAX,
             "rf_topk_merge: bad arguments");
  if (B == 0) return RF_OK;
  const size_t lds = (size_t)TK_MERGE_MAX * 12 + TK_KMAX * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_topk_merge, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  k_topk_merge<<<B, 256, lds, as_stream(stream)>>>(B, k0, v0, i0, ntiles, cval, cidx, ccnt, cap, k, out_v, out_i,
                                                   overflow);
  RF_LAUNCH_CHECK("rf_topk_merge");
}
