// K12 gated / plain activations: SiLU*mul (SwiGLU), GELU (erf and tanh forms,
// optional fused bias), ReLU.  All 16-byte vectorised on a 2-D (row segment, row)
// grid: no per-element 64-bit index divide, rows beyond 65535 are strided.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {

LK_DEVICE float silu(float x) { return lk_silu(x); }
LK_DEVICE float gelu_erf(float x) { return lk_gelu_erf(x); }
LK_DEVICE float gelu_tanh(float x) {
  const float k = 0.7978845608028654f;
  return 0.5f * x * (1.f + tanhf(k * (x + 0.044715f * x * x * x)));
}

// x: [rows, 2*I] (gate | up) with row stride xs; out: [rows, I] with row stride os.
// 2-D grid: blockIdx.x walks a row in 256-vector (16-byte) segments, blockIdx.y strides
// over rows, so there is no 64-bit divide per element.  One vector per thread (more per
// thread measured slower: benchmarks/silu_probe.hip).  NTL: non-temporal loads, used when
// the gate_up output is too big to still sit in the 256 MB MALL (5.7 -> 6.5 TB/s at 8k
// rows).  NTS: non-temporal stores speed this kernel up (5.9 -> 6.8 TB/s at 4k rows) but
// the down projection that reads the result loses more than that (silu+down pair 383 ->
// 388 us), so they are off by default.
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void silu_mul_kernel(bf16_t* __restrict__ out,
                                                       const bf16_t* __restrict__ x, long rows,
                                                       int I, long xs, long os) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= (I >> 3)) return;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
    const short8* gp = reinterpret_cast<const short8*>(x + r * xs + v * 8);
    const short8* up = reinterpret_cast<const short8*>(x + r * xs + I + v * 8);
    short8 g, u, y;
    if constexpr (NTL) {
      g = __builtin_nontemporal_load(gp);
      u = __builtin_nontemporal_load(up);
    } else {
      g = *gp;
      u = *up;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      y[j] = (short)f2bf(bf2f(f2bf(silu(bf2f((bf16_t)g[j])))) * bf2f((bf16_t)u[j]));
    short8* op = reinterpret_cast<short8*>(out + r * os + v * 8);
    if constexpr (NTS) __builtin_nontemporal_store(y, op);
    else *op = y;
  }
}

// in-place act(x + bias) on [rows, N] (row stride xs); kind 0 = gelu(erf), 1 = gelu(tanh), 2 = relu.
// Same 2-D (row segment, row) grid as silu_mul: one 16-byte vector per thread per row.
template <int KIND>
__global__ __launch_bounds__(256) void act_kernel(bf16_t* __restrict__ x,
                                                  const bf16_t* __restrict__ bias, long rows,
                                                  int N, long xs) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= (N >> 3)) return;
  const int c = v * 8;
  float b[8];
  if (bias) load8(bias + c, b);
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
    float e[8];
    load8(x + r * xs + c, e);
    if (bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = bf2f(f2bf(e[j] + b[j]));
    }
    if constexpr (KIND == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // pairs: packed fp32 math around the transcendentals
        const lk_f2 gv = lk_gelu_erf2(lk_f2{e[2 * j], e[2 * j + 1]});
        e[2 * j] = gv.x;
        e[2 * j + 1] = gv.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (KIND == 1) e[j] = gelu_tanh(e[j]);
        else e[j] = fmaxf(e[j], 0.f);
      }
    }
    store8(x + r * xs + c, e);
  }
}

dim3 row_grid(long rows, int n) {
  return dim3((unsigned)((n / 8 + 255) / 256), (unsigned)(rows < 65535 ? rows : 65535));
}


}  // namespace

int lk_silu_mul(bf16_t* out, const bf16_t* x, long rows, int I, long xs, long os, hipStream_t st) {
  if (I % 8 || rows < 0) return -1;
  if (rows == 0) return 0;
  // LK_SILU_NT: bit 0 = non-temporal stores, bit 1 = force non-temporal loads (A/B knob;
  // default: plain stores, NT loads once the [rows, 2I] input exceeds the 256 MB MALL)
  static const int nt_env = [] {
    const char* e = getenv("LK_SILU_NT");
    return e ? atoi(e) : -1;
  }();
  const bool nts = nt_env < 0 ? false : (nt_env & 1);
  const bool ntl = nt_env < 0 ? rows * (long)I * 4 > (256L << 20) : ((nt_env >> 1) & 1);
  const dim3 grid = row_grid(rows, I);
  if (ntl && nts) silu_mul_kernel<true, true><<<grid, 256, 0, st>>>(out, x, rows, I, xs, os);
  else if (ntl) silu_mul_kernel<true, false><<<grid, 256, 0, st>>>(out, x, rows, I, xs, os);
  else if (nts) silu_mul_kernel<false, true><<<grid, 256, 0, st>>>(out, x, rows, I, xs, os);
  else silu_mul_kernel<false, false><<<grid, 256, 0, st>>>(out, x, rows, I, xs, os);
  return 0;
}

int lk_activation(bf16_t* x, const bf16_t* bias, long rows, int N, long xs, int kind,
                  hipStream_t st) {
  if (N % 8 || rows < 0) return -1;
  if (rows == 0) return 0;
  const dim3 g = row_grid(rows, N);
  if (kind == 0) act_kernel<0><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else if (kind == 1) act_kernel<1><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else if (kind == 2) act_kernel<2><<<g, 256, 0, st>>>(x, bias, rows, N, xs);
  else return -1;
  return 0;
}
