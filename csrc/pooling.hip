// K5 sentence-embedding pooling fused with L2 normalisation.
//   mode 0 = mean over the sequence's tokens (MiniLM, nomic-embed), 1 = CLS (bge)
// hidden: [T, H] packed varlen rows (cu_seqlens [B+1]); out: [B, H] rows of stride `os`, f32 or
// bf16 (the query path hands the bf16 rows straight to the kNN kernels: no cast pass).
// One workgroup per sequence; 16-byte loads along H, f32 accumulation.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

template <int MAXV, typename OutT>
__global__ __launch_bounds__(128) void pool_norm_kernel(const bf16_t* __restrict__ hidden, long hs,
                                                        const int* __restrict__ cu, int H, int mode,
                                                        int normalize, OutT* __restrict__ out, long os) {
  __shared__ float red[2];
  const int b = blockIdx.x;
  const int beg = cu[b], end = cu[b + 1];
  const int n = end - beg;
  const int nvec = H >> 3;
  float acc[MAXV][8];
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const int t_end = mode == 1 ? min(beg + 1, end) : end;
  for (int t = beg; t < t_end; ++t) {
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = threadIdx.x + i * 128;
      if (c < nvec) {
        float v[8];
        load8(hidden + (long)t * hs + c * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += v[j];
      }
    }
  }
  const float div = mode == 1 ? 1.f : (float)max(n, 1);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[i][j] /= div;
      ss += acc[i][j] * acc[i][j];
    }
  ss = block_sum<2>(ss, red);
  const float inv = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * 128;
    if (c < nvec) {
      if constexpr (std::is_same<OutT, float>::value) {
        float4* op = reinterpret_cast<float4*>(out + (long)b * os + c * 8);
        op[0] = make_float4(acc[i][0] * inv, acc[i][1] * inv, acc[i][2] * inv, acc[i][3] * inv);
        op[1] = make_float4(acc[i][4] * inv, acc[i][5] * inv, acc[i][6] * inv, acc[i][7] * inv);
      } else {
        uint4 pk;
        pk.x = pack_bf2(acc[i][0] * inv, acc[i][1] * inv);
        pk.y = pack_bf2(acc[i][2] * inv, acc[i][3] * inv);
        pk.z = pack_bf2(acc[i][4] * inv, acc[i][5] * inv);
        pk.w = pack_bf2(acc[i][6] * inv, acc[i][7] * inv);
        *reinterpret_cast<uint4*>(out + (long)b * os + c * 8) = pk;
      }
    }
  }
}

// row L2 norms of a bf16 matrix [N, D] -> f32 (corpus norms for the kNN index)
__global__ __launch_bounds__(256) void row_norm_kernel(const bf16_t* __restrict__ x, long N, int D,
                                                       float* __restrict__ out) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  float ss = 0.f;
  for (int c = lane; c < D / 8; c += 64) {
    float v[8];
    load8(x + row * D + c * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
  ss = wave_sum(ss);
  if (lane == 0) out[row] = sqrtf(ss);
}

}  // namespace

template <typename OutT>
static int launch_pool(const bf16_t* hidden, long hs, const int* cu, int B, int H, int mode, int normalize,
                       OutT* out, long os, hipStream_t st) {
  const int nvec = H / 8;
  if (nvec <= 128) pool_norm_kernel<1, OutT><<<B, 128, 0, st>>>(hidden, hs, cu, H, mode, normalize, out, os);
  else if (nvec <= 256) pool_norm_kernel<2, OutT><<<B, 128, 0, st>>>(hidden, hs, cu, H, mode, normalize, out, os);
  else if (nvec <= 512) pool_norm_kernel<4, OutT><<<B, 128, 0, st>>>(hidden, hs, cu, H, mode, normalize, out, os);
  else return -2;
  return 0;
}

int lk_pool_normalize(const bf16_t* hidden, long hs, const int* cu, int B, int H, int mode,
                      int normalize, void* out, long os, int out_bf16, hipStream_t st) {
  if (B <= 0) return 0;
  if (H % 8 || os < H || os % 8) return -1;
  return out_bf16 ? launch_pool(hidden, hs, cu, B, H, mode, normalize, reinterpret_cast<bf16_t*>(out), os, st)
                  : launch_pool(hidden, hs, cu, B, H, mode, normalize, reinterpret_cast<float*>(out), os, st);
}

int lk_row_norms(const bf16_t* x, long N, int D, float* out, hipStream_t st) {
  if (N <= 0) return 0;
  if (D % 8) return -1;
  row_norm_kernel<<<(unsigned)((N + 3) / 4), 256, 0, st>>>(x, N, D, out);
  return 0;
}
