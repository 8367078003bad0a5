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

constexpr int kMaxSplit = 2048;  // max keys per workgroup (LDS block-table slice)
#ifndef LK_DECODE_WG_PER_CU
#define LK_DECODE_WG_PER_CU 3
#endif
typedef short4_t __attribute__((address_space(3))) * lds_s4_ptr;

// The flash-decoding merge of one output element (seq b, query head qh, dim d) over nsplit
// split partials (+ the cascade prefix partial): the same arithmetic as decode_reduce_kernel.
// Partials are read past L1 / L2 (system-scope loads): other workgroups wrote them through.
template <int D>
LK_DEVICE void merge_splits(int b, int qh, int d, int Hq, int max_splits, int nsplit, const float* part_o,
                            const float* part_ml, const float* pp_o, const float* pp_ml, bf16_t* out, long os) {
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
  const long base = ((long)b * Hq + qh) * max_splits;
  const long pb = (long)b * Hq + qh;
  float M = pp_o ? pp_ml[pb * 2] : -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ld(part_ml + (base + s) * 2));
  if (M == -INFINITY) M = 0.f;  // no keys at all (padding row)
  float den = 0.f, num = 0.f;
  if (pp_o) {
    const float f = exp2f(pp_ml[pb * 2] - M);
    den = f * pp_ml[pb * 2 + 1];
    num = f * pp_o[pb * D + d];
  }
  for (int s = 0; s < nsplit; ++s) {
    const float f = exp2f(ld(part_ml + (base + s) * 2) - M);
    den += f * ld(part_ml + (base + s) * 2 + 1);
    num += f * ld(part_o + (base + s) * D + d);
  }
  out[(long)b * os + (long)qh * D + d] = f2bf(den > 0.f ? num / den : 0.f);
}

// v3 (streaming): workgroup = (split, kv_head, seq), 4 waves; each wave walks 32-key
// chunks (w, w+4, ...) of the split with its own online softmax, so there is no
// workgroup barrier inside the key loop and the next chunk's K/V loads are always
// in flight while the current chunk is computed.
//   QK^T: 2 x v_mfma_f32_16x16x32_bf16 tiles, A = K rows straight from the paged
//         cache, B = Q^T (G query heads of the GQA group padded to 16 columns).
//   PV:   v_mfma_f32_16x16x32_bf16, A = P taken from the S^T accumulators (k order
//         permuted to match), B = V^T via ds_read_b64_tr_b16 from a wave-private,
//         XOR-swizzled LDS image of the chunk.
// The 4 waves' (m, l, O) are merged through LDS at the end; splits > 1 emit
// partials for lk_decode_reduce (flash-decoding).
template <int D, int G>
__global__ __launch_bounds__(256, LK_DECODE_WG_PER_CU) void paged_decode_kernel(
    const bf16_t* __restrict__ q, long qs, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, bf16_t* __restrict__ out, long os,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hkv, int BS, int max_splits,
    int split, float scale_log2, const int* __restrict__ k_start, int has_prefix,
    const float* __restrict__ pp_o, const float* __restrict__ pp_ml, int* __restrict__ tickets) {
  constexpr int KK = D / 32;     // QK k-steps (16x16x32)
  constexpr int ND = D / 16;     // PV output tiles of 16 d
  constexpr int CPR = D / 8;     // 16-B chunks per V row
  constexpr int NVL = 32 * CPR / 64;  // V 16-B loads per lane per chunk
  constexpr int RPL = 64 / CPR;  // V rows per load instruction
  // grid (B*Hkv, max_splits): the flattened (seq, kv head) index varies fastest so the
  // active split-0 workgroups are dealt round-robin over all 8 XCDs (split-fastest
  // order put every active workgroup of a short-context batch on ONE XCD).
  const int s = blockIdx.y, kvh = blockIdx.x % Hkv, b = blockIdx.x / Hkv;
  const int ctx = ctx_lens[b];
  // cascade: keys [0, k0) are a prefix shared by the whole batch, attended by the flash
  // kernel once for all rows (its partial is merged by decode_reduce_kernel)
  const int k0 = k_start ? k_start[0] : 0;
  const int k_begin = k0 + s * split;
  const int Hq = Hkv * G;
  if (k_begin >= ctx) {  // uniform for the whole workgroup
    // fused reduce: split 0 of a row without keys past the prefix writes its output itself
    if (tickets != nullptr && s == 0)
      for (int i = threadIdx.x; i < G * D; i += 256)
        merge_splits<D>(b, kvh * G + i / D, i % D, Hq, max_splits, 0, part_o, part_ml, pp_o, pp_ml, out, os);
    return;
  }
  const int nkeys = min(split, ctx - k_begin);
  const int nsplit = min((ctx - k0 + split - 1) / split, max_splits);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, h4 = lane >> 4;

  __shared__ int blk[kMaxSplit / 16];
  __shared__ __attribute__((aligned(16))) bf16_t vlds[4][32 * D];
  __shared__ float mrg_ml[4][2][16];
  __shared__ float mrg_o[4][G][D];

  const int nblk = (nkeys + BS - 1) / BS;
  for (int i = threadIdx.x; i < nblk; i += 256) {
    blk[i] = block_tables[(long)b * bt_stride + k_begin / BS + i];
    LK_DASSERT(blk[i] >= 0);
  }
  __syncthreads();

  // A wave's 16 K rows (16t + r16) and the 4 V rows of one load (i * RPL + lane / CPR) lie in
  // one cache block (BS >= 16, splits and chunks block-aligned: checked on the host), so the
  // block lookup is wave-uniform -- a scalar read of the LDS slice -- and the lane part a
  // constant.  Rows past the split re-read its last key (block clamped here, slot by the
  // clamped row): never a stale slot, whose bytes could be NaN under a zero P.
  const int last_blk = (nkeys - 1) / BS;
  auto blk_base = [&](const bf16_t* cache, int rel0) {
    const int bi = __builtin_amdgcn_readfirstlane(min(rel0 / BS, last_blk));
    return cache + ((long)blk[bi] * Hkv + kvh) * BS * D;
  };

  // Q^T fragments (B of QK): lane holds Q[q = r16][32kk + 8*h4 + j]
  short8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk)
    qf[kk] = r16 < G ? *reinterpret_cast<const short8*>(q + (long)b * qs + (long)(kvh * G + r16) * D +
                                                        32 * kk + 8 * h4)
                     : short8{0, 0, 0, 0, 0, 0, 0, 0};

  const int nch = (nkeys + 31) >> 5;
  short8 kr[2][KK], vr[NVL];
  // k_begin is block-aligned (split % BS == 0, k_start a multiple of BS): row rel of the
  // split sits at slot rel % BS of its block
  auto load_chunk = [&](int c, short8 (&kd)[2][KK], short8 (&vd)[NVL]) {
    const int base = 32 * c;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16_t* kp = blk_base(kc, base + 16 * t) + (min(base + 16 * t + r16, nkeys - 1) % BS) * D + 8 * h4;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) kd[t][kk] = *reinterpret_cast<const short8*>(kp + 32 * kk);
    }
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int rel = min(base + i * RPL + lane / CPR, nkeys - 1);
      vd[i] = *reinterpret_cast<const short8*>(blk_base(vc, base + i * RPL) + (rel % BS) * D + (lane % CPR) * 8);
    }
  };

  floatx4 o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) o[n] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  bf16_t* vw = vlds[w];

  int c = w;
  if (c < nch) load_chunk(c, kr, vr);
  for (; c < nch; c += 4) {
    // stage this chunk's V into the wave-private LDS image (row-major, 16-B chunk
    // index XOR ((row & 7) << 1) so the transposed reads below are conflict-free)
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int row = i * RPL + lane / CPR, ch = lane % CPR;
      *reinterpret_cast<short8*>(vw + row * D + ((ch ^ ((row & 7) << 1)) & (CPR - 1)) * 8) = vr[i];
    }
    // S^T tiles: lane (q = r16) holds keys 16t + 4*h4 + i
    floatx4 sc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        sc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kr[t][kk], qf[kk], sc[t], 0, 0, 0);
    }
    // K consumed, V already in LDS: the next chunk's loads fly under softmax + PV (no
    // second register set: 32 VGPRs fewer, three workgroups per CU)
    if (c + 4 < nch) load_chunk(c + 4, kr, vr);
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rel = 32 * c + 16 * t + 4 * h4 + i;
        const float x = rel < nkeys ? sc[t][i] * scale_log2 : -INFINITY;
        sc[t][i] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);  // finite: every chunk has >= 1 valid key
    const float alpha = exp2f(m_run - m_new);
    float rs = 0.f;
    short8 pa;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = exp2f(sc[t][i] - m_new);
        rs += e;
        pa[4 * t + i] = (short)f2bf(e);
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
    // O rows are q = 4*h4 + reg: fetch alpha of those query rows (lanes 0..15 hold q = lane)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const float a = __shfl(alpha, 4 * h4 + rr, 64);
#pragma unroll
      for (int n = 0; n < ND; ++n) o[n][rr] *= a;
    }
    // PV: B = V^T fragment of k-step = keys {4*h4 + j} u {16 + 4*h4 + j}, column 16n + r16
    const int qq = r16 >> 2, pp = r16 & 3;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int col = 16 * n + 4 * pp;
      const int r0 = 4 * h4 + qq, r1 = 16 + 4 * h4 + qq;
      const bf16_t* a0 = vw + r0 * D + (((col >> 3) ^ ((r0 & 7) << 1)) & (CPR - 1)) * 8 + (col & 7);
      const bf16_t* a1 = vw + r1 * D + (((col >> 3) ^ ((r1 & 7) << 1)) & (CPR - 1)) * 8 + (col & 7);
      const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(a0));
      const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(a1));
      const short8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[n], 0, 0, 0);
    }
  }

  // ---- merge the 4 waves: (m, l) per query row (lanes 0..15 hold q = lane), O rows
  if (lane < 16) {
    mrg_ml[w][0][lane] = m_run;
    mrg_ml[w][1][lane] = l_run;
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int qrow = 4 * h4 + rr;
    if (qrow < G) {
#pragma unroll
      for (int n = 0; n < ND; ++n) mrg_o[w][qrow][16 * n + r16] = o[n][rr];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int g = i / D, d = i - g * D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, mrg_ml[ww][0][g]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = mrg_ml[ww][0][g] == -INFINITY ? 0.f : exp2f(mrg_ml[ww][0][g] - M);
      L += f * mrg_ml[ww][1][g];
      O += f * mrg_o[ww][g][d];
    }
    const int qh = kvh * G + g;
    if (nsplit == 1 && !has_prefix) {
      out[(long)b * os + (long)qh * D + d] = f2bf(O / L);
    } else if (tickets != nullptr) {
      // written through to memory: the workgroup that merges may sit on another XCD (own L2)
      const long pi = ((long)b * Hq + qh) * max_splits + s;
      __hip_atomic_store(part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (d == 0) {
        __hip_atomic_store(part_ml + pi * 2, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // log2 domain
        __hip_atomic_store(part_ml + pi * 2 + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    } else {
      const long pi = ((long)b * Hq + qh) * max_splits + s;
      part_o[pi * D + d] = O;
      if (d == 0) {
        part_ml[pi * 2] = M;  // log2 domain
        part_ml[pi * 2 + 1] = L;
      }
    }
  }
  if (tickets == nullptr || (nsplit == 1 && !has_prefix)) return;
  // Fused reduce (flash-decoding merge) by the LAST split workgroup of this (seq, kv head) to
  // finish: every split's partial stores are acknowledged before its ticket is taken, and the
  // last one reads them past L1 / L2 -- no decode_reduce launch (a ~5 us kernel per layer).
  // The ticket is reset by its last taker, ready for the next launch.
  __builtin_amdgcn_s_waitcnt(0);  // this thread's partial stores acknowledged
  __syncthreads();
  __shared__ int is_last;
  if (threadIdx.x == 0) {
    int* tk = tickets + (long)b * Hkv + kvh;
    const int old = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    is_last = old == nsplit - 1;
    if (is_last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (!is_last) return;
  for (int i = threadIdx.x; i < G * D; i += 256)
    merge_splits<D>(b, kvh * G + i / D, i % D, Hq, max_splits, nsplit, part_o, part_ml, pp_o, pp_ml, out, os);
}

// combine split partials (+ the shared-prefix partial of a cascade step): grid (Hq, B), D threads
template <int D>
__global__ __launch_bounds__(D) void decode_reduce_kernel(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml,
                                                          const int* __restrict__ ctx_lens,
                                                          bf16_t* __restrict__ out, long os,
                                                          int Hq, int max_splits, int split,
                                                          const int* __restrict__ k_start,
                                                          const float* __restrict__ pp_o,
                                                          const float* __restrict__ pp_ml) {
  const int qh = blockIdx.x, b = blockIdx.y;
  const int ctx = ctx_lens[b];
  const int k0 = k_start ? k_start[0] : 0;
  const int nsplit = max(0, min((ctx - k0 + split - 1) / split, max_splits));
  if (nsplit <= 1 && !pp_o) return;  // written directly by the main kernel
  const long base = ((long)b * Hq + qh) * max_splits;
  const long pb = (long)b * Hq + qh;
  float M = pp_o ? pp_ml[pb * 2] : -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, part_ml[(base + s) * 2]);
  if (M == -INFINITY) M = 0.f;  // no keys at all (padding row)
  float den = 0.f, num = 0.f;
  const int d = threadIdx.x;
  if (pp_o) {
    const float f = exp2f(pp_ml[pb * 2] - M);
    den = f * pp_ml[pb * 2 + 1];
    num = f * pp_o[pb * D + d];
  }
  for (int s = 0; s < nsplit; ++s) {
    const float f = exp2f(part_ml[(base + s) * 2] - M);
    den += f * part_ml[(base + s) * 2 + 1];
    num += f * part_o[(base + s) * D + d];
  }
  out[(long)b * os + (long)qh * D + d] = f2bf(den > 0.f ? num / den : 0.f);
}

}  // namespace

// keys per workgroup: enough workgroups to fill 256 CUs at small batch, long splits
// (few partials) at large batch; static per (B, Hkv) so hipGraph launches are fixed.
int lk_decode_split_size(int B, int Hkv) {
  const int bh = B * Hkv;
  // >= 2 workgroups per CU without splitting: the longest split (fewest launched-but-empty
  // split workgroups in the static graph grid, no partials below 2k keys)
  if (bh >= 512) return kMaxSplit;
  if (bh >= 128) return 512;
  if (bh >= 32) return 256;
  return 128;
}

int lk_decode_splits(int max_context, int split) { return (max_context + split - 1) / split; }

int lk_paged_decode(const bf16_t* q, long qs, const bf16_t* kc, const bf16_t* vc,
                    const int* block_tables, int bt_stride, const int* ctx_lens, bf16_t* out,
                    long os, float* part_o, float* part_ml, int B, int Hq, int Hkv, int D, int BS,
                    int max_splits, int split, float scale, const int* k_start, const float* pp_o,
                    const float* pp_ml, hipStream_t st, int* tickets, int reduce) {
  if (B == 0) return 0;
  if (Hq % Hkv || BS % 16 || split % 32 || split > kMaxSplit || split % BS) return -1;
  const int G = Hq / Hkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(B * Hkv, max_splits);
#define LAUNCH(DD, GG)                                                                        \
  paged_decode_kernel<DD, GG><<<grid, 256, 0, st>>>(q, qs, kc, vc, block_tables, bt_stride,   \
                                                    ctx_lens, out, os, part_o, part_ml, Hkv, \
                                                    BS, max_splits, split, scale_log2, k_start, \
                                                    pp_o != nullptr, pp_o, pp_ml, tickets)
#define BY_G(DD)                          \
  switch (G) {                            \
    case 1: LAUNCH(DD, 1); break;         \
    case 2: LAUNCH(DD, 2); break;         \
    case 4: LAUNCH(DD, 4); break;         \
    case 8: LAUNCH(DD, 8); break;         \
    default: return -2;                   \
  }
  if (D == 128) { BY_G(128) }
  else if (D == 64) { BY_G(64) }
  else return -3;
#undef BY_G
#undef LAUNCH
  LK_CHECK_LAUNCH();
  // (fused: the last split merges; reduce == 0: the consumer merges -- the O projection's
  // weight-streaming prologue, lk_wsgemm_pro kind 2)
  if ((max_splits > 1 || pp_o) && tickets == nullptr && reduce) {
    if (D == 128)
      decode_reduce_kernel<128><<<dim3(Hq, B), 128, 0, st>>>(part_o, part_ml, ctx_lens, out, os, Hq,
                                                             max_splits, split, k_start, pp_o, pp_ml);
    else
      decode_reduce_kernel<64><<<dim3(Hq, B), 64, 0, st>>>(part_o, part_ml, ctx_lens, out, os, Hq,
                                                           max_splits, split, k_start, pp_o, pp_ml);
  }
  LK_CHECK_LAUNCH();
  return 0;
}
