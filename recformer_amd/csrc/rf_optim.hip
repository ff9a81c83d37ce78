// AdamW step over every parameter tensor of an optimizer in ONE launch (the reference trains with
// torch.optim.AdamW: optimization.py:28-32, litmodels.py:42-56, finetune.py:116-126). torch's
// multi-tensor AdamW makes ~8 passes over the state per step (mul, lerp, mul, addcmul, sqrt, div,
// add, addcdiv — each a foreach launch); here each element is read once and written once:
//   p  <- p (1 - lr wd)
//   m  <- lerp(m, g, 1 - beta1)                       (torch's lerp formula for weight < 0.5)
//   v  <- v beta2 + (1 - beta2) g g
//   p  <- p - step_size m / (sqrt(v) / sqrt(bc2) + eps),  step_size = lr / bc1
// The optimizer (recformer_amd/optim.py) keeps the step counts and bias corrections on the host,
// as torch's non-capturable AdamW (or, capturable, the step counts on the device and the bias
// corrections computed here), and hands one descriptor per tensor plus a block -> tensor table.
// 28 B of HBM traffic per fp32 element (read p g m v, write p m v): an HBM-bound stream.
#include "rf_common.h"

namespace rf {

constexpr int ADAM_CHUNK = 8192;  // elements per workgroup (256 threads x 8 float4)
static_assert(sizeof(rf_adamw_tensor) == 104, "rf_adamw_tensor layout (recformer_amd/optim.py _DESC)");

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const rf_adamw_tensor& d,
                                          float decay, float step_size, float bc2_sqrt, float inv_scale) {
  g = g * inv_scale;  // 1 unless a gradient scaler hands its scale (power of two: exact)
  if (d.maximize) g = -g;
  p = p * decay;
  const float w = d.w1;
  m = w < 0.5f ? m + w * (g - m) : g - (g - m) * (1.0f - w);
  v = v * d.beta2 + d.w2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + d.eps;
  p = p + (-step_size) * (m / denom);
}

// grad_scale / found_inf: device scalars of a gradient scaler (NULL: none). A step with an inf/NaN
// gradient (found_inf != 0) writes nothing — every workgroup returns before its first load.
template <bool NT>
__global__ void __launch_bounds__(256) k_adamw(const rf_adamw_tensor* __restrict__ descs,
                                               const int32_t* __restrict__ block_tensor,
                                               const float* __restrict__ grad_scale,
                                               const float* __restrict__ found_inf) {
  if (found_inf && *found_inf != 0.0f) return;
  const float inv_scale = grad_scale ? 1.0f / *grad_scale : 1.0f;
  const rf_adamw_tensor d = descs[block_tensor[blockIdx.x]];
  float step_size = d.step_size, bc2_sqrt = d.bias_correction2_sqrt, decay = d.decay, lr = d.lr;
  if (d.hyper) {  // capturable group: lr and 1 - lr wd from device memory the host updates between replays
    lr = d.hyper[0];
    decay = d.hyper[1];
  }
  if (d.step) {  // capturable: bias corrections from the device step count
    const float t = *d.step;
    step_size = lr / (1.0f - powf(d.beta1, t));
    bc2_sqrt = sqrtf(1.0f - powf(d.beta2, t));
  }
  const int64_t e0 = ((int64_t)blockIdx.x - d.first_block) * ADAM_CHUNK;
  const int64_t n = min((int64_t)ADAM_CHUNK, d.numel - e0);
  float* __restrict__ P = d.param + e0;
  const float* __restrict__ G = d.grad + e0;
  float* __restrict__ Mm = d.exp_avg + e0;
  float* __restrict__ Vv = d.exp_avg_sq + e0;
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(Mm) |
                     reinterpret_cast<uintptr_t>(Vv)) & 15) == 0;
  if (vec && n == ADAM_CHUNK) {
    // all loads of the thread's 8 float4 groups issued before the arithmetic
    float4 p[8], g[8], m[8], v[8];
    // NT: every operand is touched once per step: non-temporal loads and stores (no cache allocation)
    auto ld = [](const float* a) {
      if constexpr (NT) {
        const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a));
        return make_float4(x[0], x[1], x[2], x[3]);
      } else {
        return *reinterpret_cast<const float4*>(a);
      }
    };
    auto st = [](float* a, float4 x) {
      if constexpr (NT) __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w}, reinterpret_cast<f32x4*>(a));
      else *reinterpret_cast<float4*>(a) = x;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int o = 4 * (threadIdx.x + 256 * i);
      p[i] = ld(P + o);
      g[i] = ld(G + o);
      m[i] = ld(Mm + o);
      v[i] = ld(Vv + o);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      adam_elem(p[i].x, g[i].x, m[i].x, v[i].x, d, decay, step_size, bc2_sqrt, inv_scale);
      adam_elem(p[i].y, g[i].y, m[i].y, v[i].y, d, decay, step_size, bc2_sqrt, inv_scale);
      adam_elem(p[i].z, g[i].z, m[i].z, v[i].z, d, decay, step_size, bc2_sqrt, inv_scale);
      adam_elem(p[i].w, g[i].w, m[i].w, v[i].w, d, decay, step_size, bc2_sqrt, inv_scale);
      const int o = 4 * (threadIdx.x + 256 * i);
      st(P + o, p[i]);
      st(Mm + o, m[i]);
      st(Vv + o, v[i]);
    }
  } else {
    for (int64_t i = threadIdx.x; i < n; i += 256) {
      float p = P[i], m = Mm[i], v = Vv[i];
      adam_elem(p, G[i], m, v, d, decay, step_size, bc2_sqrt, inv_scale);
      P[i] = p;
      Mm[i] = m;
      Vv[i] = v;
    }
  }
}

}  // namespace rf

using namespace rf;

extern "C" int rf_adamw_chunk(void) { return ADAM_CHUNK; }

extern "C" int rf_adamw_step_amp(const rf_adamw_tensor* tensors, int ntensors, const int32_t* block_tensor,
                                 int nblocks, const float* grad_scale, const float* found_inf, rf_stream_t stream) {
  RF_REQUIRE(ntensors >= 0 && nblocks >= 0, "rf_adamw_step: bad counts %d %d", ntensors, nblocks);
  if (nblocks == 0) return RF_OK;
  RF_REQUIRE(tensors && block_tensor, "rf_adamw_step: null pointer");
  if (g_knob[KNOB_ADAM_NT]) k_adamw<true><<<nblocks, 256, 0, as_stream(stream)>>>(tensors, block_tensor, grad_scale, found_inf);
  else k_adamw<false><<<nblocks, 256, 0, as_stream(stream)>>>(tensors, block_tensor, grad_scale, found_inf);
  RF_LAUNCH_CHECK("rf_adamw_step");
}

extern "C" int rf_adamw_step(const rf_adamw_tensor* tensors, int ntensors, const int32_t* block_tensor, int nblocks,
                             rf_stream_t stream) {
  return rf_adamw_step_amp(tensors, ntensors, block_tensor, nblocks, nullptr, nullptr, stream);
}
