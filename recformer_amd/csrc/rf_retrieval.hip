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
//                   exact top-k per row (value descending, ties by lower item index) by a ballot-
//                   counted binary search over order-preserving 32-bit keys held in registers (one
//                   wave per row); the merge reads the seed
//                   top-k and every tile's candidate slots and flags rows whose slots overflowed
//                   (the caller re-ranks those rows densely).
// Element types: bf16 and fp16 operands (v_mfma_f32_16x16x32_bf16 / _f16), fp32 scores.
#include "rf_common.h"
#include "rf_w32.h"

#include <algorithm>
#include <cstddef>

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

static int num_cus_rt() {
  static int n = 0;
  if (!n) {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    n = c > 0 ? c : 256;
  }
  return n;
}

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
  float* cval;              // MODE 1: per-row candidate lists [row][capr]
  int32_t* cidx;
  int32_t* rcnt;            // MODE 1: per-row candidate count (> capr: overflow)
  int capr;
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
constexpr int RK_TCAP = 32;                        // candidates per (row, tile) staged in LDS
constexpr int RK_CAND = RK_CNT + 1024;             // [256][RK_TCAP] values, then ids
static_assert(RK_CAND + 256 * RK_TCAP * 8 <= RK_LDS, "retrieval epilogue scratch");

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
  float* cv = reinterpret_cast<float*>(smem + RK_CAND);                      // [256 rows][RK_TCAP]
  int32_t* ci = reinterpret_cast<int32_t*>(smem + RK_CAND + 256 * RK_TCAP * 4);
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
      // stage in LDS per tile row (slot order within a (row, tile) is free: the merge sorts)
      const int n = __builtin_popcount(cmask);
      const int base = atomicAdd(&cnt[rl], n);
      int t = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (cmask & (1u << k)) {
          if (base + t < RK_TCAP) {
            cv[rl * RK_TCAP + base + t] = v[k];
            ci[rl * RK_TCAP + base + t] = a.idx_base + a.col0 + c0 + k;
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
      if (MODE == 1) {
        // the tile's candidates of this row appended to the row's list: one global atomic per
        // (row, tile) with candidates; a tile overflow poisons the row's count (> capr)
        const int c = cnt[rl];
        if (c > 0) {
          const int m = min(c, RK_TCAP);
          const int gbase = atomicAdd(a.rcnt + row, c > RK_TCAP ? a.capr + 1 : m);
          if (c <= RK_TCAP && gbase + m <= a.capr) {
            float* dv = a.cval + (int64_t)row * a.capr + gbase;
            int32_t* di = a.cidx + (int64_t)row * a.capr + gbase;
            for (int j = 0; j < m; ++j) {
              dv[j] = cv[rl * RK_TCAP + j];
              di[j] = ci[rl * RK_TCAP + j];
            }
          }
        }
      }
    }
  }
}

// ---- the same on the four-wave 32x32x16 main loop (rf_w32.h), catalog rows as the A operand ------
// k_rank_w32: A = the shard's item rows [col0, col0 + ncols) (M), W = the queries (N), so a lane holds
// 4 query columns x 64 item rows of every 256 x 256 tile: the per-query counts and exp-sums are
// in-lane sums over items, one shuffle across the lane halves and one LDS exchange between the two
// waves of a query half — no score matrix, no per-row cross-lane reductions. Candidates (MODE 1) are
// compacted per wave into LDS slots and appended to the queries' global lists after the tile (one
// atomic each, about k per row per column chunk); a row whose list overflows is flagged by the merge
// as before; MODE 0 also stores the dense scores.
// k_label_score32 computes the labels' own scores with the same MFMA (32x32x16, the same operand
// roles, K ascending in 16-chunks, the chain starting from zero) and the same epilogue expression, so
// the strict ranks compare bit-identical values. (The 16x16x32 kernels above are kept for D not a
// multiple of 64 and as the knob-selected A/B path; label and rank kernels are always chosen by the
// same predicate, rank_w32_ok.)
struct RankW32Args {
  int B, ncols, col0;
  const float* rq;
  const float* rc;
  float scale, max_val, shift;
  const float* s_label;
  const float* tau;
  float* dense;
  int64_t ldd;
  float* cval;
  int32_t* cidx;
  int32_t* rcnt;
  int capr;
  int32_t idx_base;
  int32_t* part_cnt;
  float* part_sexp;
  int tn0;
};

// k_rank_w32's parameter list as a struct: the kernarg segment lays the arguments out this way

struct RankKernArgs {
  int K;
  const void* items;
  int ldi;
  const void* Q;
  int ldq, nTm, nTn;
  RankW32Args a;
};
constexpr int RANK_KARG_OFF = (int)offsetof(RankKernArgs, a);

// k_rank_w32's epilogue scratch (W32_SCR_BYTES): [0, 8 KiB) the count / exp-sum exchange between the
// two waves of a query half, then MODE 1's per-wave candidate slots
constexpr int RW_CL = 8192;
constexpr int RW_CL_CAP = 543;  // candidates per wave and tile (about 3 per query in the densest chunk), + trash
constexpr int RW_CL_WAVE = (RW_CL_CAP + 1) * 8;
static_assert(RW_CL + 4 * RW_CL_WAVE <= W32_SCR_BYTES, "rank epilogue scratch");

template <int MODE>
struct RankW32Pol {
  static constexpr int S = 0;  // the epilogue's memory operations depend on the data: no relaxed wait
  // the arguments stay in the kernarg segment and are re-read (scalar loads) in each epilogue through
  // a laundered pointer: held in SGPRs across the K-loop they push the loop past the SGPR budget
  // (spills into VGPR lanes)
  typedef const __attribute__((address_space(4))) RankW32Args* KPtr;
  __device__ __forceinline__ RankW32Args args() const {
    // the kernel's `a` argument, read from the kernarg segment (its offset: RankKernArgs below)
    KPtr p = (KPtr)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
                    RANK_KARG_OFF);
    asm volatile("" : "+s"(p));
    RankW32Args r;  // field by field: scalar loads from the kernarg segment
    r.B = p->B; r.ncols = p->ncols; r.col0 = p->col0;
    r.rq = p->rq; r.rc = p->rc;
    r.scale = p->scale; r.max_val = p->max_val; r.shift = p->shift;
    r.s_label = p->s_label; r.tau = p->tau;
    r.dense = p->dense; r.ldd = p->ldd;
    r.cval = p->cval; r.cidx = p->cidx; r.rcnt = p->rcnt; r.capr = p->capr; r.idx_base = p->idx_base;
    r.part_cnt = p->part_cnt; r.part_sexp = p->part_sexp; r.tn0 = p->tn0;
    return r;
  }
  __device__ __forceinline__ void cols(char* slot, int wave, int lane, int tm0, int tn0) const {
    const RankW32Args a = args();
    // the tile's 256 item inverse norms, 4 B per lane (rows past ncols read as 0 by the range check)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.rc + a.col0), (short)0, a.ncols * 4, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + wave * 256), 4,
                                             (tm0 + 64 * wave + lane) * 4, 0, 0, 0);
  }
  __device__ __forceinline__ void epilogue(f32x16 (&acc)[4][4], const W32Tile& t) const {
    const RankW32Args a = args();
    int el = t.lane;
    asm volatile("" : "+v"(el));
    const int c = el & 31, g = el >> 5;
    const int q0 = t.n0 + t.wc * 128 + 4 * c;
    float rs[4], sl[4], tau[4];
    bool qok[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      qok[jb] = q0 + jb < a.B;
      const int qq = min(q0 + jb, a.B - 1);
      rs[jb] = a.rq[qq] * a.scale;
      sl[jb] = a.s_label[qq];
      tau[jb] = MODE == 1 ? a.tau[qq] : 0.f;
    }
    const int ib = t.wr * 128 + 4 * g;  // tile-relative item row of register 0 of block 0
    // MODE 1: this wave's candidates are staged in the epilogue scratch as (score, item << 8 | query)
    // by a ballot compaction (no atomics, LDS addresses only inside the unrolled loop: the direct
    // global appends of round 4 held 64-bit list addresses across it and spilled), then appended to
    // the queries' global lists after the loop; a query whose candidates miss the wave's slots is
    // poisoned (> capr) for the exact re-rank
    uint2* cl = reinterpret_cast<uint2*>(t.scr + RW_CL + t.wave * RW_CL_WAVE);
    int ncand = 0;
    uint32_t lost = 0;                                        // MODE 1: queries jb with candidates past the slots
    const uint32_t pkb = (uint32_t)((ib << 8) | (4 * c));     // + (pr << 8) + jb: item << 8 | query
    int gt[4] = {0, 0, 0, 0}, vc[4] = {0, 0, 0, 0};
    float se[4] = {0.f, 0.f, 0.f, 0.f};
    // MODE 0: dense scores through a buffer resource: a query past B is past num_records, an item past
    // ncols gets an offset >= 2^31 (branch-free stores)
    const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(MODE == 0 ? a.dense : nullptr), (short)0,
        MODE == 0 ? (int)min((int64_t)a.B * a.ldd * 4, (int64_t)0x7FFFFFFF) : 0, 0x00020000);
    const uint32_t lbD = (uint32_t)((q0 * (int)a.ldd + t.m0 + ib) * 4);
    static_for<64>([&](auto ir) {
      constexpr int i = decltype(ir)::value >> 4, r = decltype(ir)::value & 15;
      constexpr int pr = 32 * i + 8 * (r >> 2) + (r & 3);
      float v[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[jb]) : "a"(acc[i][jb][r]) : "memory");
      const int item = t.m0 + ib + pr;  // column of this launch's range [0, ncols)
      const bool iok = item < a.ncols;
      const float rcv = t.cb[ib + pr];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        // items past ncols score -inf: no count, exp2(-inf) = 0 — one select, no branch around the exp
        const float sv = iok ? cos_score(v[jb], rs[jb], rcv) : -__builtin_inff();
        gt[jb] += sv > sl[jb] ? 1 : 0;
        vc[jb] += sv > -a.max_val ? 1 : 0;
        se[jb] += __builtin_amdgcn_exp2f((sv - a.shift) * RT_LOG2E);
        if (MODE == 0) {
          // unconditional: the caller's row stride covers whole 256-column tiles (items past ncols land
          // in the row's padding), queries past B are past num_records
          uint32_t lb = lbD;
          asm volatile("" : "+v"(lb));
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sv), rsD, lb + (uint32_t)((jb * (int)a.ldd + pr) * 4),
                                                0, 0);
        }
        if (MODE == 1) {
          // a (query, item) pair is a candidate with probability ~k (grow - 1) / chunk (0.3-2.4%): the
          // ballot is taken per query column and the compaction runs only where some lane has one
          // (a wave-uniform branch); within it every lane stores, a lane without a candidate (or past
          // the slots) into the wave's trash slot, and the count advances by the ballot's popcount
          const bool cnd = qok[jb] && iok && sv >= tau[jb];
          const uint64_t m = __builtin_amdgcn_ballot_w64(cnd);
          if (m) {
            const int slot = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)ncand));
            const bool keep = cnd && slot < RW_CL_CAP;
            lost |= (cnd && !keep) ? (1u << jb) : 0u;
            cl[keep ? slot : RW_CL_CAP] = make_uint2(__float_as_uint(sv), pkb + (uint32_t)((pr << 8) + jb));
            ncand += (int)__popcll(m);
          }
          asm volatile("" : "+v"(lost));
        }
      }
      if (MODE == 1) {
        // the counts in place: the candidate branches would otherwise let their arithmetic sink to the
        // end of the loop, every score of the tile live until then (spills)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) asm volatile("" : "+v"(gt[jb]), "+v"(vc[jb]), "+v"(se[jb]));
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (MODE == 1) {  // the counts are complete here: otherwise their arithmetic sinks past the flush below
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) asm volatile("" : "+v"(gt[jb]), "+v"(vc[jb]), "+v"(se[jb]));
    }
    if (MODE == 1) {
      // append the staged candidates to the queries' lists: one global atomic each, predicated through
      // buffer offsets (>= 2^31: dropped) instead of divergent branches — a branch here costs the whole
      // kernel its registers (the allocator then spills the prologue's values across the K-loop)
      __builtin_amdgcn_wave_barrier();
      constexpr uint32_t OOR = 0x80000000u;
      const int nc = min(ncand, RW_CL_CAP);
      const int qb = t.n0 + t.wc * 128;
      const int lim = (int)min((int64_t)a.B * a.capr * 4, (int64_t)0x7FFFFFFF);
      const __amdgpu_buffer_rsrc_t rsN = __builtin_amdgcn_make_buffer_rsrc((void*)a.rcnt, (short)0, a.B * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)a.cval, (short)0, lim, 0x00020000);
      const __amdgpu_buffer_rsrc_t rsI = __builtin_amdgcn_make_buffer_rsrc((void*)a.cidx, (short)0, lim, 0x00020000);
      const int idb = a.idx_base + a.col0 + t.m0;
      for (int e0 = 0; e0 < nc; e0 += 64) {  // wave-uniform trip count
        const int e = e0 + el;
        const bool ok = e < nc;
        const uint2 x = cl[ok ? e : RW_CL_CAP];
        const int q = qb + (int)(x.y & 255u);
        const int pos = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rsN, ok ? q * 4 : (int)OOR, 0, 0);
        const uint32_t off = (ok && pos < a.capr) ? (uint32_t)((q * a.capr + pos) * 4) : OOR;
        __builtin_amdgcn_raw_buffer_store_b32(x.x, rsV, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(idb + (int)(x.y >> 8)), rsI, off, 0, 0);
      }
      if (ncand > RW_CL_CAP) {  // wave-uniform: poison the queries whose candidates missed the slots
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
          (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(a.capr + 1, rsN,
                                                               ((lost >> jb) & 1u) ? (q0 + jb) * 4 : (int)OOR, 0, 0);
      }
    }
    // lane halves (item rows 4g..), then the two waves (wr) of this query half through LDS
    int pk[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      pk[jb] = gt[jb] | (vc[jb] << 16);
      pk[jb] += __shfl_xor(pk[jb], 32, 64);
      se[jb] += __shfl_xor(se[jb], 32, 64);
    }
    int* xc = reinterpret_cast<int*>(t.scr) + t.wc * 512;      // [wc][4 c-quads][128]: counts
    float* xs = reinterpret_cast<float*>(t.scr + 4096) + t.wc * 512;
    if (t.wr == 1 && g == 0) {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        xc[4 * c + jb] = pk[jb];
        xs[4 * c + jb] = se[jb];
      }
    }
    __syncthreads();
    if (t.wr == 0 && g == 0) {
      const int64_t o = (int64_t)(a.tn0 + t.m0 / 256) * a.B;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        if (qok[jb]) {
          a.part_cnt[o + q0 + jb] = pk[jb] + xc[4 * c + jb];
          a.part_sexp[o + q0 + jb] = se[jb] + xs[4 * c + jb];
        }
      }
    }
  }
};

template <typename T, int MODE>
__global__ void __launch_bounds__(256, 1)
    k_rank_w32(int K, const T* __restrict__ items, int ldi, const T* __restrict__ Q, int ldq, int nTm, int nTn,
               RankW32Args a) {
  w32_run<T>(K, items, ldi, Q, ldq, a.ncols, a.B, nTn, 0, nTm, nTn, RankW32Pol<MODE>{});
}

template <typename T>
__global__ void __launch_bounds__(64) k_label_score32(int B, int K, const T* __restrict__ q, int ldq,
                                                      const float* __restrict__ rq, const T* __restrict__ items,
                                                      int ldi, const float* __restrict__ ri, int nshard,
                                                      const int64_t* __restrict__ labels, int64_t label_base,
                                                      float scale, float* __restrict__ s_label) {
  typedef typename RtElt<T>::V8 V8;
  const int lane = threadIdx.x;
  const int n = lane & 31, g = lane >> 5;
  const int qb = min((int)blockIdx.x * 32 + n, B - 1);
  const int64_t lr = labels[qb] - label_base;
  const bool mine = lr >= 0 && lr < nshard;
  const T* ea = items + (mine ? lr : 0) * (int64_t)ldi + 8 * g;  // A: the label items (rows)
  const T* qa = q + (int64_t)qb * ldq + 8 * g;                   // B: the queries (columns)
  f32x16 acc = f32x16{};
  for (int k0 = 0; k0 < K; k0 += 16)
    acc = mfma32(*reinterpret_cast<const V8*>(ea + k0), *reinterpret_cast<const V8*>(qa + k0), acc);
  // D[m][n] sits in lane n + 32 ((m >> 2) & 1), register 4 (m >> 3) + (m & 3): the diagonal m = n
  if (g == ((n >> 2) & 1)) {
    const int b = blockIdx.x * 32 + n;
    if (b < B) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r == 4 * (n >> 3) + (n & 3)) v = acc[r];
      s_label[b] = mine ? cos_score(v, rq[b] * scale, ri[lr]) : 0.f;
    }
  }
}

static bool rank_w32_ok(int D, int ldq, int ldi) {
  return g_knob[KNOB_RANK_W32] && D % 64 == 0 && D >= 128 && ldq % 8 == 0 && ldi % 8 == 0;
}

// 16 threads per row, each summing every 16th tile in order, then a fixed-order combine:
// deterministic, and enough threads to hide the partials' load latency
__global__ void __launch_bounds__(256) k_rank_reduce(int B, int ntiles, const int32_t* __restrict__ part_cnt,
                                                     const float* __restrict__ part_sexp, int32_t* __restrict__ gt,
                                                     int32_t* __restrict__ valid, float* __restrict__ sexp) {
  __shared__ int sc[16][17];
  __shared__ float ss[16][17];
  const int rl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int row = blockIdx.x * 16 + rl;
  int c = 0;
  float e = 0.f;
  if (row < B) {
    // 8 tiles' loads in flight per thread (the sums keep the tile order: the same result as one at a
    // time, which waited a memory round trip per tile: 111 us at 1M items x 4096 queries)
    int t = grp;
    for (; t + 7 * 16 < ntiles; t += 8 * 16) {
      int ci[8];
      float ei[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        ci[u] = part_cnt[(int64_t)(t + 16 * u) * B + row];
        ei[u] = part_sexp[(int64_t)(t + 16 * u) * B + row];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        c += ci[u];
        e += ei[u];
      }
    }
    for (; t < ntiles; t += 16) {
      c += part_cnt[(int64_t)t * B + row];
      e += part_sexp[(int64_t)t * B + row];
    }
  }
  sc[rl][grp] = c;
  ss[rl][grp] = e;
  __syncthreads();
  if (grp == 0 && row < B) {
    int g = 0, v = 0;
    float x = 0.f;
    for (int j = 0; j < 16; ++j) {
      g += sc[rl][j] & 0xFFFF;
      v += sc[rl][j] >> 16;
      x += ss[rl][j];
    }
    gt[row] = g;
    valid[row] = v;
    sexp[row] = x;
  }
}

// ---- exact top-k per row, one wave per row, keys in registers ---------------------------------
// order-preserving key: larger float -> larger unsigned key (0 only for a negative NaN: here the
// "missing entry" marker)
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
// lanes below this one in a ballot mask
__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

constexpr int TK_DENSE_MAX = 2048;  // entries per row of a dense block
constexpr int TK_MERGE_MAX = 2048;  // seed list + candidates per row
constexpr int TK_KMAX = 256;
constexpr int TK_WAVES = 4;         // rows per workgroup
// per-wave LDS: the selected keys and ids (TK_KMAX each), the ids of the entries tied at the threshold
constexpr int TK_WAVE_WORDS = 2 * TK_KMAX + TK_MERGE_MAX;

// final order of the kk selected entries: key descending, id ascending, as one 64-bit comparison key
// (key << 32 | ~id). Entry a = 64 t + lane is held by its lane (R registers, kk <= 64 R); every entry b
// is read from its lane (v_readlane into SGPRs: no LDS round trip per comparison)
template <int R>
__device__ __forceinline__ void rank_selected(const uint32_t* sk, const int32_t* si, int kk, float* out_v,
                                              int32_t* out_i) {
  const int lane = threadIdx.x & 63;
  uint64_t mc[R];
  int rank[R];
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int a = t * 64 + lane;
    mc[t] = a < kk ? ((uint64_t)sk[a] << 32) | (uint32_t)~si[a] : 0ull;
    rank[t] = 0;
  }
#pragma unroll
  for (int tb = 0; tb < R; ++tb) {
    const int nb = min(64, kk - tb * 64);
    const int lo = (int)(uint32_t)mc[tb], hi = (int)(uint32_t)(mc[tb] >> 32);
    for (int bl = 0; bl < nb; ++bl) {
      const uint64_t cb = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, bl) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane(lo, bl);
#pragma unroll
      for (int t = 0; t < R; ++t) rank[t] += cb > mc[t] ? 1 : 0;
    }
  }
#pragma unroll
  for (int t = 0; t < R; ++t) {
    if (t * 64 + lane < kk) {
      out_v[rank[t]] = kfloat((uint32_t)(mc[t] >> 32));
      out_i[rank[t]] = (int32_t)~(uint32_t)mc[t];
    }
  }
}

// The threshold search and the selection over keys held S per lane (entry j * 64 + lane; key 0 =
// missing), kk <= #valid keys, lo / hi bounds of the kk-th largest key (wave-uniform): tau = the largest
// t with #{key >= t} >= kk by a binary search whose counts are ballots (one compare and one popcount per
// register, no LDS, no atomics; it stops once exactly kk keys reach t), then the keys above tau and the
// lowest-id ties compacted into sk / si (ties' ids through tieb) and ranked. pos_of(j) is the entry's
// position in the row (its id through id_at).
template <int S, typename PosOf, typename IdAt>
__device__ __forceinline__ void search_select(const uint32_t (&key)[S], int kk, bool exact, uint32_t lo, uint32_t hi,
                                              PosOf pos_of, IdAt id_at, uint32_t* sk, int32_t* si, int32_t* tieb,
                                              float* out_v, int32_t* out_i) {
  const int lane = threadIdx.x & 63;
  while (!exact && lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1) + 1u;  // in (lo, hi]
    int c = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) c += __popcll(__ballot(key[j] >= mid));
    if (c >= kk) {
      lo = mid;
      exact = c == kk;
    } else {
      hi = mid - 1u;
    }
  }
  const uint32_t tau = lo;
  int ngt = 0, nt = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const bool g = key[j] != 0u && (exact ? key[j] >= tau : key[j] > tau);
    const bool q = !exact && key[j] == tau;
    const uint64_t mg = __ballot(g), mq = __ballot(q);
    if (g) {
      const int o = ngt + lanes_below(mg);
      sk[o] = key[j];
      si[o] = id_at(pos_of(j));
    }
    if (q) tieb[nt + lanes_below(mq)] = id_at(pos_of(j));
    ngt += __popcll(mg);
    nt += __popcll(mq);
  }
  __builtin_amdgcn_wave_barrier();
  const int need = kk - ngt;
  if (need > 0) {  // the `need` ties with the lowest ids (all of them when nt == need)
    for (int a = lane; a < nt; a += 64) {
      const int ia = tieb[a];
      int r = a;
      if (nt > need) {
        r = 0;
        for (int b = 0; b < nt && r < need; ++b) r += tieb[b] < ia ? 1 : 0;
      }
      if (r < need) {
        sk[ngt + r] = tau;
        si[ngt + r] = ia;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (kk <= 64) rank_selected<1>(sk, si, kk, out_v, out_i);
  else if (kk <= 128) rank_selected<2>(sk, si, kk, out_v, out_i);
  else rank_selected<4>(sk, si, kk, out_v, out_i);
}

constexpr int TK_CMAX = 256;  // compacted candidates of a long row (keys, then positions, in front of the ties)

// Top-k of one row's n entries (entry p at key_at(p), id_at(p); key 0 = missing): values descending,
// ties by lower id; missing outputs (-inf, -1). The n keys sit in registers, S per lane. Long rows
// (S >= 16) with kk <= 64 first narrow the range: the kk-th largest of the 64 lane maxima is a lower
// bound of the kk-th largest key (the lane maxima are a subset of the keys), found by the same search
// over one register; the keys at or above it — a few percent of a dense row — are compacted into LDS
// and the search and selection run on those, four registers per lane instead of S (rows with more than
// TK_CMAX of them keep the full form). Same tau, same selection: bit-identical either way.
template <int S, typename KeyAt, typename IdAt>
__device__ __forceinline__ void row_topk(int n, int k, KeyAt key_at, IdAt id_at, uint32_t* sk, int32_t* si,
                                         int32_t* tid, float* out_v, int32_t* out_i) {
  const int lane = threadIdx.x & 63;
  uint32_t key[S];
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
  int nv = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int p = j * 64 + lane;
    key[j] = p < n ? key_at(p) : 0u;
  }
#pragma unroll
  for (int j = 0; j < S; ++j) {
    if (key[j]) {
      lo = min(lo, key[j]);
      hi = max(hi, key[j]);
    }
    nv += __popcll(__ballot(key[j] != 0u));
  }
  const int kk = min(k, nv);
  if (kk > 0) {
    lo = __builtin_amdgcn_readfirstlane(wave_min_u(lo));
    hi = __builtin_amdgcn_readfirstlane(wave_max_u(hi));
    bool done = false;
    if (S >= 16 && kk <= 64 && nv > kk) {
      uint32_t lm = 0u;
#pragma unroll
      for (int j = 0; j < S; ++j) lm = max(lm, key[j]);
      uint32_t a = lo, b = hi;  // the kk-th largest lane maximum (a lane without keys holds 0 < lo)
      while (a < b) {
        const uint32_t mid = a + ((b - a) >> 1) + 1u;
        if (__popcll(__ballot(lm >= mid)) >= kk) a = mid;
        else b = mid - 1u;
      }
      int c0 = 0;
#pragma unroll
      for (int j = 0; j < S; ++j) c0 += __popcll(__ballot(key[j] >= a));
      if (c0 <= TK_CMAX) {
        uint32_t* ck = reinterpret_cast<uint32_t*>(tid);
        int32_t* cp = tid + TK_CMAX;
        int o = 0;
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const bool g = key[j] >= a;
          const uint64_t m = __ballot(g);
          if (g) {
            const int e = o + lanes_below(m);
            ck[e] = key[j];
            cp[e] = j * 64 + lane;
          }
          o += __popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t k2[TK_CMAX / 64];
#pragma unroll
        for (int t = 0; t < TK_CMAX / 64; ++t) {
          const int e = t * 64 + lane;
          k2[t] = e < c0 ? ck[e] : 0u;
        }
        search_select<TK_CMAX / 64>(
            k2, kk, c0 == kk, a, hi, [&](int t) { return cp[t * 64 + lane]; }, id_at, sk, si, tid + 2 * TK_CMAX,
            out_v, out_i);
        done = true;
      }
    }
    if (!done)
      search_select<S>(key, kk, nv == kk, lo, hi, [&](int j) { return j * 64 + lane; }, id_at, sk, si, tid, out_v,
                       out_i);
  }
  for (int a = kk + lane; a < k; a += 64) {
    out_v[a] = -__builtin_inff();
    out_i[a] = -1;
  }
}

// the register count per lane that holds n entries (one instantiation per size class)
template <typename KeyAt, typename IdAt>
__device__ __forceinline__ void row_topk_n(int n, int k, KeyAt key_at, IdAt id_at, int32_t* lds, float* out_v,
                                           int32_t* out_i) {
  uint32_t* sk = reinterpret_cast<uint32_t*>(lds);
  int32_t* si = lds + TK_KMAX;
  int32_t* tid = lds + 2 * TK_KMAX;
  if (n <= 512) row_topk<8>(n, k, key_at, id_at, sk, si, tid, out_v, out_i);
  else if (n <= 1024) row_topk<16>(n, k, key_at, id_at, sk, si, tid, out_v, out_i);
  else row_topk<32>(n, k, key_at, id_at, sk, si, tid, out_v, out_i);
}

__global__ void __launch_bounds__(64 * TK_WAVES) k_topk_dense(int B, int n, const float* __restrict__ vals,
                                                              int64_t ldv, const int32_t* __restrict__ idx,
                                                              int64_t ldi, int32_t idx_base, int k,
                                                              float* __restrict__ out_v, int32_t* __restrict__ out_i) {
  __shared__ int32_t lds[TK_WAVES * TK_WAVE_WORDS];
  const int wave = threadIdx.x >> 6;
  const int row = blockIdx.x * TK_WAVES + wave;
  if (row >= B) return;
  const float* vr = vals + (int64_t)row * ldv;
  const int32_t* ir = idx ? idx + (int64_t)row * ldi : nullptr;
  row_topk_n(
      n, k, [&](int p) { return fkey(vr[p]); }, [&](int p) { return ir ? ir[p] : idx_base + p; },
      lds + wave * TK_WAVE_WORDS, out_v + (int64_t)row * k, out_i + (int64_t)row * k);
}

__global__ void __launch_bounds__(64 * TK_WAVES) k_topk_merge(int B, int k0, const float* __restrict__ v0,
                                                              const int32_t* __restrict__ i0,
                                                              const float* __restrict__ cval,
                                                              const int32_t* __restrict__ cidx,
                                                              const int32_t* __restrict__ rcnt, int capr, int k,
                                                              float* __restrict__ out_v, int32_t* __restrict__ out_i,
                                                              int32_t* __restrict__ overflow) {
  __shared__ int32_t lds[TK_WAVES * TK_WAVE_WORDS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * TK_WAVES + wave;
  if (row >= B) return;
  const int c = rcnt[row];
  float* ov = out_v + (int64_t)row * k;
  int32_t* oi = out_i + (int64_t)row * k;
  const float* sv = v0 + (int64_t)row * k0;
  const int32_t* sd = i0 + (int64_t)row * k0;
  if (c > capr || k0 + c > TK_MERGE_MAX) {
    // overflowed: keep the previous list (a valid lower bound for the next threshold) and flag the
    // row for an exact dense re-rank
    for (int e = lane; e < k; e += 64) {
      ov[e] = e < k0 ? sv[e] : -__builtin_inff();
      oi[e] = e < k0 ? sd[e] : -1;
    }
    if (lane == 0) overflow[row] = 1;
    return;
  }
  // entries 0..k0-1: the running list (id < 0: empty slot, missing), then the c candidates
  const float* cv = cval + (int64_t)row * capr - k0;
  const int32_t* cd = cidx + (int64_t)row * capr - k0;
  row_topk_n(
      k0 + c, k, [&](int p) { return p < k0 ? (sd[p] >= 0 ? fkey(sv[p]) : 0u) : fkey(cv[p]); },
      [&](int p) { return p < k0 ? sd[p] : cd[p]; }, lds + wave * TK_WAVE_WORDS, ov, oi);
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
  if (rank_w32_ok(D, ldq, ldi)) {
    const int g32 = (B + 31) / 32;
    if (dtype == RF_BF16)
      k_label_score32<bf16><<<g32, 64, 0, s>>>(B, D, (const bf16*)q, ldq, rq, (const bf16*)items, ldi, ri, nshard,
                                               labels, label_base, inv_temp, s_label);
    else if (dtype == RF_F16)
      k_label_score32<f16><<<g32, 64, 0, s>>>(B, D, (const f16*)q, ldq, rq, (const f16*)items, ldi, ri, nshard,
                                              labels, label_base, inv_temp, s_label);
    else
      RF_REQUIRE(false, "rf_label_scores: dtype must be bf16 or fp16");
    RF_LAUNCH_CHECK("rf_label_scores");
  }
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
                             int64_t ldd, float* cval, int32_t* cidx, int32_t* rcnt, int capr, int32_t idx_base,
                             int32_t* part_cnt, float* part_sexp, int tn0, rf_stream_t stream) {
  RF_REQUIRE(mode >= 0 && mode <= 2, "rf_score_rank: mode must be 0 (dense), 1 (candidates) or 2 (counts)");
  RF_REQUIRE(B >= 0 && ncols >= 0 && col0 >= 0 && D > 0 && D % 32 == 0, "rf_score_rank: bad shape (D %% 32 == 0)");
  RF_REQUIRE(ldq % 8 == 0 && ldi % 8 == 0, "rf_score_rank: leading dims must be multiples of 8");
  RF_REQUIRE(s_label && part_cnt && part_sexp && rq && ri, "rf_score_rank: null pointer");
  RF_REQUIRE(mode == 2 || (mode == 0 ? (dense && ldd >= ncols && ldd % 4 == 0) : (tau && cval && cidx && rcnt && capr > 0)),
             "rf_score_rank: mode %d outputs missing or misaligned", mode);
  if (B == 0 || ncols == 0) return RF_OK;
  hipStream_t s = as_stream(stream);
  if (rank_w32_ok(D, ldq, ldi)) {
    static bool attr32 = false;
    if (!attr32) {
#define RK32_ATTR(T, M) \
  (void)hipFuncSetAttribute((const void*)k_rank_w32<T, M>, hipFuncAttributeMaxDynamicSharedMemorySize, W32_LDS)
      RK32_ATTR(bf16, 0); RK32_ATTR(bf16, 1); RK32_ATTR(bf16, 2);
      RK32_ATTR(f16, 0); RK32_ATTR(f16, 1); RK32_ATTR(f16, 2);
#undef RK32_ATTR
      attr32 = true;
    }
    // launches of at most 2^31 bytes of item rows (the loop's buffer resources), 256-column aligned
    const int64_t row_bytes = (int64_t)ldi * 2;
    const int cap_cols = (int)std::min<int64_t>(ncols, (0x7FFFFFFF / row_bytes) / 256 * 256);
    RF_REQUIRE(cap_cols > 0, "rf_score_rank: item rows too wide");
    RF_REQUIRE(mode != 0 || ldd >= (ncols + 255) / 256 * 256,
               "rf_score_rank: mode 0 needs ldd >= ncols rounded up to 256 (whole-tile rows)");
    const int nTn = (B + 255) / 256;
    for (int c0 = 0; c0 < ncols; c0 += cap_cols) {
      const int nc = std::min(cap_cols, ncols - c0);
      RankW32Args a{B, nc, col0 + c0, rq, ri, inv_temp, max_val, shift, s_label, tau,
                    dense ? dense + c0 : nullptr, ldd, cval, cidx, rcnt, capr, idx_base, part_cnt, part_sexp,
                    tn0 + c0 / 256};
      const int nTm = (nc + 255) / 256;
      const int grid = std::min(nTm * nTn, num_cus_rt());
      const void* it = (const char*)items + (int64_t)(col0 + c0) * row_bytes;
#define RK32_(T, M) \
  k_rank_w32<T, M><<<grid, 256, W32_LDS, s>>>(D, (const T*)it, ldi, (const T*)q, ldq, nTm, nTn, a)
      if (dtype == RF_BF16) {
        if (mode == 0) RK32_(bf16, 0);
        else if (mode == 1) RK32_(bf16, 1);
        else RK32_(bf16, 2);
      } else if (dtype == RF_F16) {
        if (mode == 0) RK32_(f16, 0);
        else if (mode == 1) RK32_(f16, 1);
        else RK32_(f16, 2);
      } else {
        RF_REQUIRE(false, "rf_score_rank: dtype must be bf16 or fp16");
      }
#undef RK32_
    }
    RF_LAUNCH_CHECK("rf_score_rank");
  }
  RankArgs a{B, ncols, col0, rq, ri, inv_temp, s_label, max_val, shift, tau, dense, ldd,
             cval, cidx, rcnt, capr, idx_base, part_cnt, part_sexp, tn0};
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
  k_rank_reduce<<<(B + 15) / 16, 256, 0, as_stream(stream)>>>(B, ntiles, part_cnt, part_sexp, gt, valid, sexp);
  RF_LAUNCH_CHECK("rf_rank_reduce");
}

extern "C" int rf_topk_dense(int B, int n, const float* vals, int64_t ldv, const int32_t* idx, int64_t ldi,
                             int32_t idx_base, int k, float* out_v, int32_t* out_i, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && n >= 0 && n <= TK_DENSE_MAX && k > 0 && k <= TK_KMAX,
             "rf_topk_dense: n=%d must be <= %d and k=%d in [1, %d]", n, TK_DENSE_MAX, k, TK_KMAX);
  if (B == 0) return RF_OK;
  k_topk_dense<<<(B + TK_WAVES - 1) / TK_WAVES, 64 * TK_WAVES, 0, as_stream(stream)>>>(
      B, n, vals, ldv, idx, ldi, idx_base, k, out_v, out_i);
  RF_LAUNCH_CHECK("rf_topk_dense");
}

extern "C" int rf_topk_merge(int B, int k0, const float* v0, const int32_t* i0, const float* cval,
                             const int32_t* cidx, const int32_t* rcnt, int capr, int k, float* out_v, int32_t* out_i,
                             int32_t* overflow, rf_stream_t stream) {
  RF_REQUIRE(B >= 0 && k0 >= 0 && k0 <= TK_KMAX && capr > 0 && k > 0 && k <= TK_KMAX,
             "rf_topk_merge: bad arguments");
  if (B == 0) return RF_OK;
  k_topk_merge<<<(B + TK_WAVES - 1) / TK_WAVES, 64 * TK_WAVES, 0, as_stream(stream)>>>(
      B, k0, v0, i0, cval, cidx, rcnt, capr, k, out_v, out_i, overflow);
  RF_LAUNCH_CHECK("rf_topk_merge");
}
