// K11 paged decode attention (one query token per sequence, GQA, split-K).
//
// Workgroup = (split, kv_head, seq); 4 waves.  All G = Hq/Hkv query heads that
// share the kv head are processed together, so every K/V byte is read from HBM
// once per step (decode is bandwidth-bound: the KV stream IS the roofline).
//
//  QK^T : v_mfma_f32_16x16x32_bf16 with A = K (16 keys x 32 d, loaded straight
//         from the paged cache into VGPRs, 16 B/lane) and B = Q^T (the G query
//         rows padded to 16).  Scores land in LDS [G][P].
//  softmax: per query row over the split (max / exp / sum), exp'd in place.
//  PV   : each lane owns 8 contiguous d of one key row (16 B V loads), keeps
//         G x 8 f32 accumulators, then a butterfly + LDS reduction over rows.
//  Splits > 1 write (unnormalised O, max, sum) partials that lk_decode_reduce
//  combines (flash-decoding).  The grid is sized for the *maximum* context so the
//  launch shape is static and the whole step can be captured in a hipGraph;
//  splits beyond a sequence's length exit immediately.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int kSplit = 512;  // keys per workgroup

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    const bf16_t* __restrict__ q, long qs, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, bf16_t* __restrict__ out, long os,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hkv, int BS, int max_splits,
    float scale) {
  constexpr int P = kSplit;
  constexpr int KK = D / 32;   // MFMA k-steps over the head dim
  constexpr int LPR = D / 8;   // lanes per V row in the PV phase
  constexpr int RPW = 64 / LPR;
  const int s = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int ctx = ctx_lens[b];
  const int k_begin = s * P;
  if (k_begin >= ctx) return;  // uniform for the whole workgroup
  const int nkeys = min(P, ctx - k_begin);
  const int nsplit = min((ctx + P - 1) / P, max_splits);
  const int Hq = Hkv * G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;

  __shared__ float logits[G][P];
  __shared__ float red[4][G][D];
  __shared__ float stat[2][G];
  __shared__ int blk[P / 16];

  const int nblk = (nkeys + BS - 1) / BS;
  for (int i = threadIdx.x; i < nblk; i += 256)
    blk[i] = block_tables[(long)b * bt_stride + k_begin / BS + i];

  // Q^T fragments (B operand): lane holds Q[q = lane&15][32kk + 8(lane>>4) + j]
  const int qi = lane & 15, hq = lane >> 4;
  short8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    if (qi < G)
      qf[kk] = *reinterpret_cast<const short8*>(q + (long)b * qs + (long)(kvh * G + qi) * D +
                                                32 * kk + 8 * hq);
    else
      qf[kk] = short8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();

  // ---- QK^T over 16-key tiles, round-robin over the 4 waves
  const int ntile = (nkeys + 15) >> 4;
  for (int t = w; t < ntile; t += 4) {
    const int rel = min(16 * t + qi, nkeys - 1);  // clamp: rows past the end are masked below
    const int abs_k = k_begin + rel;
    const bf16_t* kp = kc + (((long)blk[rel / BS] * Hkv + kvh) * BS + (abs_k % BS)) * D + 8 * hq;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const short8 a = *reinterpret_cast<const short8*>(kp + 32 * kk);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[kk], acc, 0, 0, 0);
    }
    if (qi < G) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kr = 16 * t + 4 * hq + i;
        logits[qi][kr] = kr < nkeys ? acc[i] * scale : -INFINITY;
      }
    }
  }
  __syncthreads();

  // ---- softmax statistics per query row
  for (int g = w; g < G; g += 4) {
    float m = -INFINITY;
    for (int j = lane; j < nkeys; j += 64) m = fmaxf(m, logits[g][j]);
    m = wave_max(m);
    float sum = 0.f;
    for (int j = lane; j < nkeys; j += 64) {
      const float e = __expf(logits[g][j] - m);
      logits[g][j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    if (lane == 0) {
      stat[0][g] = m;
      stat[1][g] = sum;
    }
  }
  __syncthreads();

  // ---- P.V : lane owns d = (lane % LPR)*8 .. +7 of key row (lane / LPR)
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  const int dv = (lane % LPR) * 8;
  for (int kb = w * RPW; kb < nkeys; kb += 4 * RPW) {
    const int rel = kb + lane / LPR;
    if (rel < nkeys) {
      const int abs_k = k_begin + rel;
      float v[8];
      load8(vc + (((long)blk[rel / BS] * Hkv + kvh) * BS + (abs_k % BS)) * D + dv, v);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = logits[g][rel];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] += p * v[j];
      }
    }
  }
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] += __shfl_xor(acc[g][j], o, 64);
  if (lane < LPR) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[w][g][dv + j] = acc[g][j];
  }
  __syncthreads();

  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int g = i / D, d = i - g * D;
    const float o = red[0][g][d] + red[1][g][d] + red[2][g][d] + red[3][g][d];
    const int qh = kvh * G + g;
    if (nsplit == 1) {
      out[(long)b * os + (long)qh * D + d] = f2bf(o / stat[1][g]);
    } else {
      const long pi = ((long)b * Hq + qh) * max_splits + s;
      part_o[pi * D + d] = o;
      if (d == 0) {
        part_ml[pi * 2] = stat[0][g];
        part_ml[pi * 2 + 1] = stat[1][g];
      }
    }
  }
}

// combine split partials: grid (Hq, B), D threads
template <int D>
__global__ __launch_bounds__(D) void decode_reduce_kernel(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml,
                                                          const int* __restrict__ ctx_lens,
                                                          bf16_t* __restrict__ out, long os,
                                                          int Hq, int max_splits) {
  const int qh = blockIdx.x, b = blockIdx.y;
  const int ctx = ctx_lens[b];
  const int nsplit = min((ctx + kSplit - 1) / kSplit, max_splits);
  if (nsplit <= 1) return;  // written directly by the main kernel
  const long base = ((long)b * Hq + qh) * max_splits;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, part_ml[(base + s) * 2]);
  float den = 0.f, num = 0.f;
  const int d = threadIdx.x;
  for (int s = 0; s < nsplit; ++s) {
    const float f = __expf(part_ml[(base + s) * 2] - M);
    den += f * part_ml[(base + s) * 2 + 1];
    num += f * part_o[(base + s) * D + d];
  }
  out[(long)b * os + (long)qh * D + d] = f2bf(num / den);
}

}  // namespace

int lk_decode_splits(int max_context) { return (max_context + kSplit - 1) / kSplit; }

int lk_paged_decode(const bf16_t* q, long qs, const bf16_t* kc, const bf16_t* vc,
                    const int* block_tables, int bt_stride, const int* ctx_lens, bf16_t* out,
                    long os, float* part_o, float* part_ml, int B, int Hq, int Hkv, int D, int BS,
                    int max_splits, float scale, hipStream_t st) {
  if (B == 0) return 0;
  if (Hq % Hkv || BS % 16 || kSplit % BS) return -1;
  const int G = Hq / Hkv;
  dim3 grid(max_splits, Hkv, B);
#define LAUNCH(DD, GG)                                                                        \
  paged_decode_kernel<DD, GG><<<grid, 256, 0, st>>>(q, qs, kc, vc, block_tables, bt_stride,   \
                                                    ctx_lens, out, os, part_o, part_ml, Hkv, \
                                                    BS, max_splits, scale)
#define BY_G(DD)                          \
  switch (G) {                            \
    case 1: LAUNCH(DD, 1); break;         \
    case 2: LAUNCH(DD, 2); break;         \
    case 4: LAUNCH(DD, 4); break;         \
    case 8: LAUNCH(DD, 8); break;         \
    case 16: LAUNCH(DD, 16); break;       \
    default: return -2;                   \
  }
  if (D == 128) { BY_G(128) }
  else if (D == 64) { BY_G(64) }
  else return -3;
#undef BY_G
#undef LAUNCH
  if (max_splits > 1) {
    if (D == 128)
      decode_reduce_kernel<128><<<dim3(Hq, B), 128, 0, st>>>(part_o, part_ml, ctx_lens, out, os, Hq,
                                                             max_splits);
    else
      decode_reduce_kernel<64><<<dim3(Hq, B), 64, 0, st>>>(part_o, part_ml, ctx_lens, out, os, Hq,
                                                           max_splits);
  }
  return 0;
}
