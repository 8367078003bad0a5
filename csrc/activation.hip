// K12 gated / plain activations: SiLU*mul (SwiGLU), GELU (erf and tanh forms,
// optional fused bias), ReLU.  All 16-byte vectorised and grid-strided
// (grid capped at ~8 blocks/CU worth of work so huge prefill batches do not
// launch millions of tiny blocks).
#include "common.h"
#include "kernels.h"

namespace {

LK_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }
LK_DEVICE float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
LK_DEVICE float gelu_tanh(float x) {
  const float k = 0.7978845608028654f;
  return 0.5f * x * (1.f + tanhf(k * (x + 0.044715f * x * x * x)));
}

// x: [rows, 2*I] (gate | up) with row stride xs; out: [rows, I] with row stride os
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16_t* __restrict__ out,
                                                       const bf16_t* __restrict__ x, long rows,
                                                       int I, long xs, long os) {
  const int vpr = I >> 3;
  const long total = rows * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / vpr;
    const int c = (int)(i - r * vpr) * 8;
    float g[8], u[8], y[8];
    load8(x + r * xs + c, g);
    load8(x + r * xs + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(silu(g[j]))) * u[j];
    store8(out + r * os + c, y);
  }
}

// in-place act(x + bias) on [rows, N] (row stride xs); kind 0 = gelu(erf), 1 = gelu(tanh), 2 = relu
template <int KIND>
__global__ __launch_bounds__(256) void act_kernel(bf16_t* __restrict__ x,
                                                  const bf16_t* __restrict__ bias, long rows,
                                                  int N, long xs) {
  const int vpr = N >> 3;
  const long total = rows * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / vpr;
    const int c = (int)(i - r * vpr) * 8;
    float v[8];
    load8(x + r * xs + c, v);
    if (bias) {
      float b[8];
      load8(bias + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] + b[j]));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (KIND == 0) v[j] = gelu_erf(v[j]);
      else if constexpr (KIND == 1) v[j] = gelu_tanh(v[j]);
      else v[j] = fmaxf(v[j], 0.f);
    }
    store8(x + r * xs + c, v);
  }
}

int grid_for(long work_items) {
  long g = (work_items + 255) / 256;
  const long cap = 256L * 8;  // 256 CUs x 8 blocks
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

int lk_silu_mul(bf16_t* out, const bf16_t* x, long rows, int I, long xs, long os, hipStream_t st) {
  if (I % 8 || rows < 0) return -1;
  if (rows == 0) return 0;
  silu_mul_kernel<<<grid_for(rows * (I / 8)), 256, 0, st>>>(out, x, rows, I, xs, os);
  return 0;
}

int lk_activation(bf16_t* x, const bf16_t* bias, long rows, int N, long xs, int kind,
                  hipStream_t st) {
  if (N % 8 || rows < 0) return -1;
  if (rows == 0) return 0;
  const int g = grid_for(rows * (N / 8));
  if (kind == 0) act_kernel<0><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else if (kind == 1) act_kernel<1><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else if (kind == 2) act_kernel<2><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else return -1;
  return 0;
}
