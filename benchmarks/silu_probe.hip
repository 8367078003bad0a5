// Standalone probe of SwiGLU (silu(gate) * up) kernel variants at the engine's prefill
// shapes: vectors per thread (U), non-temporal loads/stores.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/silu_probe benchmarks/silu_probe.hip && /tmp/silu_probe
// Prints one line per (variant, shape): us and effective GB/s (read 2*T*I + write T*I bf16).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <vector>

typedef unsigned short bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7fff + ((u >> 16) & 1);
  return (bf16_t)(u >> 16);
}
__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

template <bool NT>
__device__ __forceinline__ short8 ld(const bf16_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const short8*>(p));
  else return *reinterpret_cast<const short8*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(bf16_t* p, short8 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<short8*>(p));
  else *reinterpret_cast<short8*>(p) = v;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k(bf16_t* __restrict__ out, const bf16_t* __restrict__ x, long rows,
                                         int I) {
  const int vpr = I >> 3;
  const int v0 = blockIdx.x * (256 * U) + threadIdx.x;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
    const bf16_t* xr = x + r * 2L * I;
    bf16_t* orow = out + r * (long)I;
    short8 g[U], u[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int v = v0 + j * 256;
      if (v < vpr) {
        g[j] = ld<NTL>(xr + v * 8);
        u[j] = ld<NTL>(xr + I + v * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int v = v0 + j * 256;
      if (v < vpr) {
        short8 y;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          y[e] = (short)f2bf(bf2f(f2bf(silu(bf2f((bf16_t)g[j][e])))) * bf2f((bf16_t)u[j][e]));
        st<NTS>(orow + v * 8, y);
      }
    }
  }
}

template <int U, bool NTL, bool NTS>
void run(const char* name, bf16_t* out, const bf16_t* x, long T, int I, int ymax) {
  const int vpr = I / 8;
  dim3 grid((vpr + 256 * U - 1) / (256 * U), (unsigned)(T < ymax ? T : ymax));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) k<U, NTL, NTS><<<grid, 256>>>(out, x, T, I);
  const int n = 50;
  hipEventRecord(a);
  for (int i = 0; i < n; ++i) k<U, NTL, NTS><<<grid, 256>>>(out, x, T, I);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / n;
  printf("%-22s ymax %6d T%5ld I%5d  %8.2f us  %7.0f GB/s\n", name, ymax, T, I, us, T * (double)I * 6 / us / 1e3);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const long Tmax = 8192;
  const int Imax = 14336;
  bf16_t *x, *out;
  hipMalloc(&x, Tmax * 2L * Imax * 2);
  hipMalloc(&out, Tmax * (long)Imax * 2);
  std::vector<bf16_t> h(Tmax * 2L * Imax);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (bf16_t)(0x3f00 + (i % 251));
  hipMemcpy(x, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep)
    for (long T : {3584L, 4096L, 8192L}) {
      run<1, false, false>("U1", out, x, T, Imax, 65535);
      run<1, false, true>("U1 ntstore", out, x, T, Imax, 65535);
      run<1, true, false>("U1 ntload", out, x, T, Imax, 65535);
      run<1, true, true>("U1 ntload+ntstore", out, x, T, Imax, 65535);
      run<2, false, true>("U2 ntstore", out, x, T, Imax, 65535);
      run<2, true, false>("U2 ntload", out, x, T, Imax, 65535);
      run<2, true, true>("U2 ntload+ntstore", out, x, T, Imax, 65535);
      run<4, true, true>("U4 ntload+ntstore", out, x, T, Imax, 65535);
    }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  hipFree(x);
  hipFree(out);
  return 0;
}
