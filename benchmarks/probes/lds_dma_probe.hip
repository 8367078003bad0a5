// Per-CU load throughput from an L2-resident operand: LDS-DMA (global_load_lds_dwordx4, the
// weight-streaming GEMM's X path) vs global_load_dwordx4 into VGPRs.  One 256-thread workgroup
// per CU (as the ws GEMM), every workgroup streams the SAME 1 MiB buffer (like the decode
// activations X, re-read by every column tile) `iters` times, `depth` 1-KiB wave-instructions in
// flight per wave.  Prints bytes per CU per ns and chip-wide TB/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_dma_probe benchmarks/probes/lds_dma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kBytes = 1 << 20;  // shared source buffer
constexpr int kThreads = 256;

template <int DEPTH>
__global__ __launch_bounds__(kThreads, 1) void dma_kernel(const unsigned char* src, int iters, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[4 * DEPTH * 1024];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = kBytes / 1024;  // 1-KiB wave pieces
  int c = (blockIdx.x * 4 + w) * 7 % nchunk;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + (long)c * 1024 + lane * 16),
                                       (lds_ptr_t)(lds + (w * DEPTH + d) * 1024), 16, 0, 0);
      c = c + 1 == nchunk ? 0 : c + 1;
    }
    __builtin_amdgcn_s_waitcnt((0) | (0x7 << 4) | (0xF << 8));  // vmcnt(0)
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[lane];
}

template <int DEPTH>
__global__ __launch_bounds__(kThreads, 1) void vgpr_kernel(const unsigned char* src, int iters, unsigned* sink) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nchunk = kBytes / 1024;
  int c = (blockIdx.x * 4 + w) * 7 % nchunk;
  uint4 acc = {0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
    uint4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      v[d] = *reinterpret_cast<const uint4*>(src + (long)c * 1024 + lane * 16);
      c = c + 1 == nchunk ? 0 : c + 1;
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc.x ^= v[d].x;
      acc.y ^= v[d].y;
      acc.z ^= v[d].z;
      acc.w ^= v[d].w;
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[blockIdx.x] = acc.x;
}

template <typename K>
static float run(K kern, int blocks, const unsigned char* src, int iters, unsigned* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<blocks, kThreads>>>(src, iters, sink);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a);
    kern<<<blocks, kThreads>>>(src, iters, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned char* src;
  unsigned* sink;
  hipMalloc(&src, kBytes);
  hipMemset(src, 1, kBytes);
  hipMalloc(&sink, 4096 * sizeof(unsigned));
  const int iters = 2000;
  auto report = [&](const char* name, int depth, float ms, int blocks) {
    const double bytes = (double)blocks * 4 * depth * 1024.0 * iters;
    printf("{\"probe\": \"%s\", \"depth\": %d, \"blocks\": %d, \"ms\": %.3f, \"GB_per_s_per_CU\": %.2f, \"TB_per_s\": %.2f}\n",
           name, depth, blocks, ms, bytes / blocks / (ms * 1e6), bytes / (ms * 1e9));
  };
  for (int blocks : {cus, cus / 8}) {
    report("lds_dma", 4, run(dma_kernel<4>, blocks, src, iters, sink), blocks);
    report("lds_dma", 8, run(dma_kernel<8>, blocks, src, iters, sink), blocks);
    report("lds_dma", 16, run(dma_kernel<16>, blocks, src, iters, sink), blocks);
    report("vgpr", 4, run(vgpr_kernel<4>, blocks, src, iters, sink), blocks);
    report("vgpr", 8, run(vgpr_kernel<8>, blocks, src, iters, sink), blocks);
    report("vgpr", 16, run(vgpr_kernel<16>, blocks, src, iters, sink), blocks);
  }
  hipFree(src);
  hipFree(sink);
  return 0;
}
