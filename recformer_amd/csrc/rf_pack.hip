// Per-step weight packing for the training path: every fp32 master weight the encoder's GEMMs read
// is rounded to the compute dtype (bf16 / fp16) ONCE per step, into the row-major copy the forward
// GEMMs take (C = A.W^T) and the transposed copy the backward's dA = dC.W takes (rf_gemm reads its
// second operand as N x K rows) — one launch for all layers instead of a cast + concatenation +
// transpose (+ scaled clone for the q rows) launch per weight per step (autocast's per-op casts in
// the reference's finetune.py:106-110 / TF:1064-1130 training).
//
// One descriptor per source matrix (rows x cols fp32, row-major, lda): written at row row_off of
// dst (ld_dst) and, if dstT, transposed at column row_off of dstT (ld_T), the first scale_n source
// rows of the transposed copy multiplied by t_scale after rounding (the attention's q-column scale
// folded into dA's operand). The fused q|k|v weight is three descriptors into one destination.
// Workgroup = one 64 x 64 tile: coalesced fp32 loads, coalesced 16-bit stores of the tile, and the
// transposed tile through LDS. block_entry[b] names the descriptor of workgroup b; a descriptor's
// tiles are consecutive from its first_tile (row-major over the tile grid).
#include "rf_common.h"

namespace rf {

template <typename E>
__global__ void __launch_bounds__(256) k_pack(const rf_pack_entry* __restrict__ ents,
                                              const int32_t* __restrict__ block_entry) {
  __shared__ uint16_t tile[64][66];
  const rf_pack_entry d = ents[block_entry[blockIdx.x]];
  const int tcols = (d.cols + 63) >> 6;
  const int tix = blockIdx.x - (int)d.first_tile;
  const int r0 = (tix / tcols) * 64, c0 = (tix % tcols) * 64;
  const int t = threadIdx.x;
  const int cq = (t & 15) * 4;
  const bool vec = (d.lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(d.src) & 15) == 0) && (d.ld_dst % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(d.dst) & 7) == 0) && c0 + 64 <= d.cols;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = (t >> 4) + 16 * i, r = r0 + rl;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < d.rows) {
      const float* s = d.src + (int64_t)r * d.lda + c0 + cq;
      if (vec) {
        const float4 x = *reinterpret_cast<const float4*>(s);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = c0 + cq + k < d.cols ? s[k] : 0.f;
      }
    }
    uint16_t hb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) hb[k] = __builtin_bit_cast(uint16_t, (E)v[k]);
    if (r < d.rows && d.dst) {
      E* o = reinterpret_cast<E*>(d.dst) + (int64_t)(d.row_off + r) * d.ld_dst + c0 + cq;
      if (vec) {
        *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)hb[0] | ((uint32_t)hb[1] << 16),
                                                  (uint32_t)hb[2] | ((uint32_t)hb[3] << 16));
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c0 + cq + k < d.cols) reinterpret_cast<uint16_t*>(o)[k] = hb[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rl][cq + k] = hb[k];
  }
  if (!d.dstT) return;
  __syncthreads();
  // transposed: dstT[c][row_off + r] = round(round(W[r][c]) * (r < scale_n ? t_scale : 1))
  const bool vecT = (d.ld_T % 4 == 0) && ((reinterpret_cast<uintptr_t>(d.dstT) & 7) == 0) && ((d.row_off & 3) == 0) &&
                    r0 + 64 <= d.rows;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl = (t >> 4) + 16 * i, c = c0 + cl;
    if (c >= d.cols) continue;
    uint16_t hb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t b = tile[cq + k][cl];
      if (r0 + cq + k < d.scale_n) b = __builtin_bit_cast(uint16_t, (E)((float)__builtin_bit_cast(E, b) * d.t_scale));
      hb[k] = b;
    }
    E* o = reinterpret_cast<E*>(d.dstT) + (int64_t)c * d.ld_T + d.row_off + r0 + cq;
    if (vecT) {
      *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)hb[0] | ((uint32_t)hb[1] << 16),
                                                (uint32_t)hb[2] | ((uint32_t)hb[3] << 16));
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (r0 + cq + k < d.rows) reinterpret_cast<uint16_t*>(o)[k] = hb[k];
    }
  }
}

}  // namespace rf

using namespace rf;

extern "C" int rf_pack_weights(int dtype, const rf_pack_entry* entries, int nentries, const int32_t* block_entry,
                               int nblocks, rf_stream_t stream) {
  RF_REQUIRE(dtype == RF_BF16 || dtype == RF_F16, "rf_pack_weights: dtype must be bf16 or fp16");
  RF_REQUIRE(nentries >= 0 && nblocks >= 0, "rf_pack_weights: bad counts");
  if (nblocks == 0) return RF_OK;
  RF_REQUIRE(entries && block_entry, "rf_pack_weights: null pointer");
  hipStream_t s = as_stream(stream);
  if (dtype == RF_BF16) k_pack<bf16><<<nblocks, 256, 0, s>>>(entries, block_entry);
  else k_pack<f16><<<nblocks, 256, 0, s>>>(entries, block_entry);
  RF_LAUNCH_CHECK("rf_pack_weights");
}
