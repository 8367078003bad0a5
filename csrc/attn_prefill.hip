// K10 / K3: flash attention forward for prefill (causal, GQA, reading K/V from the
// paged cache) and for the encoder (bidirectional, K/V straight from the packed QKV
// buffer), varlen over a batch of sequences.
//
// Design (gfx950, wave64, v_mfma_f32_32x32x16_bf16):
//  * workgroup = 4 waves sharing ONE kv head; each wave owns 32 query rows of one
//    query head.  With G = Hq/Hkv >= 4 the block is 32 rows x 4 heads of the same
//    GQA group, so each K/V tile staged in LDS feeds 4 heads (4x fewer K/V bytes
//    than one block per head).  With G < 4 the block is (4/G)*32 rows x G heads.
//  * swapped product S^T = K . Q^T  (A = K tile rows from LDS, B = Q^T kept in
//    VGPRs for the whole loop), so each lane owns one query row's scores and the
//    softmax row reductions are in-register + one xor-32 shuffle.
//  * O^T = V^T . P^T: P^T is consumed straight out of the S^T accumulators
//    (pairwise bf16 packing; the MFMA k-order permutation is mirrored on the V
//    side), V^T fragments come from ds_read_b64_tr_b16 hardware transposed reads.
//  * LDS images are XOR-swizzled per head dim so that the row reads (K) and the
//    transposed reads (V) are bank-conflict free.
//  * K/V for tile t+1 are loaded into registers while tile t is computed and
//    written to LDS after the barrier (issue-early / write-late staging).
//  * online softmax in the exp2 domain with the scale folded into one multiply.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int KT = 64;  // keys per tile

typedef short4_t __attribute__((address_space(3))) * lds_short_ptr;

template <int D>
LK_DEVICE int k_swz(int row, int chunk) {
  if constexpr (D == 128) return chunk ^ (row & 15);
  else if constexpr (D == 64) return chunk ^ ((row >> 1) & 7);
  else return chunk ^ ((row >> 2) & 3);
}
template <int D>
LK_DEVICE int v_swz(int row, int chunk) {
  if constexpr (D == 128) return chunk ^ ((row & 3) << 2);
  else if constexpr (D == 64) return chunk ^ (((row >> 1) & 1) << 2);
  else return chunk;
}

struct PrefillParams {
  const bf16_t* q;
  long qs;
  const bf16_t* k;  // paged: k cache [NB,Hkv,BS,D]; dense: [T, Hkv, D] with token stride ks
  const bf16_t* v;
  long ks, vs;
  const int* block_tables;
  int bt_stride;
  const int* cu_q;      // [B+1] query row offsets
  const int* ctx_lens;  // [B] total keys (paged); dense: may be null -> q_len
  const int* tile_seq;
  const int* tile_q0;
  bf16_t* out;
  long os;
  int Hq, Hkv, BS, bs_shift;  // BS is a power of two (paged cache block size)
  float scale_log2;
  // partial mode (cascade decode over a shared prefix): instead of the normalised
  // bf16 `out`, write the unnormalised f32 O [row][Hq][D] and (max, sum) [row][Hq][2]
  // in the log2 domain of the split-K decode partials
  float* part_o;
  float* part_ml;
};

// NW waves per workgroup (4 or 8): WH of them share a row group (one head each), and
// NW / WH row groups of 32 queries sit on top of each other, all fed by the same staged
// K/V tile -- with NW = 8 each K/V byte brought into LDS serves 2x the MFMA work.
template <int D, bool CAUSAL, bool PAGED, int WH, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void flash_prefill_kernel(PrefillParams p) {
  constexpr int NT = 64 * NW;      // threads
  constexpr int KK = D / 16;       // QK k-steps
  constexpr int ND = D / 32;       // O^T d tiles
  constexpr int CPR = D / 8;       // 16-byte chunks per row
  constexpr int NCH = KT * CPR;    // chunks per tile
  constexpr int CPT = NCH / NT;    // chunks per thread per tile
  constexpr int WR = NW / WH;
  constexpr int QB = 32 * WR;
  static_assert(CPT >= 1 && NCH % NT == 0, "tile too small for the workgroup");

  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * KT * D];
  bf16_t* Ks = lds;
  bf16_t* Vs = lds + KT * D;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int G = p.Hq / p.Hkv;
  const int head = blockIdx.y * WH + (w % WH);
  const int kvh = head / G;
  const int rg = w / WH;

  const int b = p.tile_seq[blockIdx.x];
  const int q0 = p.tile_q0[blockIdx.x];
  const int qbeg = p.cu_q[b];
  const int qlen = p.cu_q[b + 1] - qbeg;
  const int ctx = p.ctx_lens ? p.ctx_lens[b] : qlen;
  const int past = ctx - qlen;
  const int kend = CAUSAL ? min(ctx, past + q0 + QB) : ctx;

  const int qrow = q0 + rg * 32 + r;  // query index within the sequence (this lane's column)
  const int qpos = past + qrow;        // absolute position
  const bool qvalid = qrow < qlen;

  // Paged K/V: the 64 / (D / 8) rows one wave stages lie in ONE cache block (BS >= 512 / D,
  // checked on the host), so the block-table lookup is wave-uniform: a scalar load and a
  // scalar base per chunk, the lane part (row within block, 16-byte chunk) a constant.
  // Rows past the context re-read the last valid key (block clamped here, slot by the
  // clamped key): never a stale slot, whose bytes could be NaN under a zero P.
  const int kvh_u = blockIdx.y * WH / G;  // == head / G for every wave of the workgroup
  auto paged_base = [&](int kt, int row) -> long {
    const int last = (ctx - 1) >> p.bs_shift;
    const int bi = __builtin_amdgcn_readfirstlane(min((kt + row) >> p.bs_shift, last));
    const long blk = p.block_tables[(long)b * p.bt_stride + bi];
    return ((blk * p.Hkv + kvh_u) << p.bs_shift) * D;
  };

  // Q^T fragments: lane holds Q[qrow][16kk + 8h + j]
  short8 qf[KK];
  {
    const bf16_t* qp = p.q + (long)(qbeg + (qvalid ? qrow : 0)) * p.qs + (long)head * D + 8 * h;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      qf[kk] = qvalid ? *reinterpret_cast<const short8*>(qp + 16 * kk)
                      : short8{0, 0, 0, 0, 0, 0, 0, 0};
  }

  floatx16 o[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[n][i] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // ---- staging helpers: chunk c of the tile = (row c / CPR, col chunk c % CPR)
  short8 kreg[CPT], vreg[CPT];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NT * i;
      const int row = c / CPR, ch = c % CPR;
      const int key = min(kt + row, ctx - 1);  // clamp: masked later
      const bf16_t *kp, *vp;
      if constexpr (PAGED) {
        const long base = paged_base(kt, row);
        const int loff = (key & (p.BS - 1)) * D + ch * 8;  // clamped key: a valid slot
        kp = p.k + base + loff;
        vp = p.v + base + loff;
      } else {
        kp = p.k + (long)(qbeg + key) * p.ks + (long)kvh * D + ch * 8;
        vp = p.v + (long)(qbeg + key) * p.vs + (long)kvh * D + ch * 8;
      }
      kreg[i] = *reinterpret_cast<const short8*>(kp);
      vreg[i] = *reinterpret_cast<const short8*>(vp);
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NT * i;
      const int row = c / CPR, ch = c % CPR;
      *reinterpret_cast<short8*>(Ks + row * D + k_swz<D>(row, ch) * 8) = kreg[i];
      *reinterpret_cast<short8*>(Vs + row * D + v_swz<D>(row, ch) * 8) = vreg[i];
    }
  };

  // loop-invariant LDS offsets (elements): the swizzle of K row 32m + r and of the
  // V^T rows 32m + 16s2 + 4h + qq (+8) depends only on the lane, so the tile loop
  // addresses LDS with per-lane bases plus compile-time row offsets.
  int koff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) koff[kk] = r * D + k_swz<D>(r, 2 * kk + h) * 8;
  const int g16 = lane >> 4, li = lane & 15;
  const int qq = li >> 2, pp = li & 3;  // this lane supplies row qq, cols 4pp..4pp+3
  int voff[ND];
#pragma unroll
  for (int n = 0; n < ND; ++n) {
    const int c0 = 32 * n + 16 * (g16 & 1) + 4 * pp;
    const int r0 = 4 * h + qq;
    voff[n] = r0 * D + v_swz<D>(r0, c0 >> 3) * 8 + (c0 & 7);
  }

  const int ntiles = (kend + KT - 1) / KT;
  if (ntiles > 0) gload(0);
  for (int t = 0; t < ntiles; ++t) {
    const int kt = t * KT;
    __syncthreads();  // everyone finished reading the previous tile
    swrite();
    __syncthreads();
    if (t + 1 < ntiles) gload(kt + KT);

    // ---- S^T = K . Q^T  for two 32-key halves
    floatx16 s[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[m][i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const short8 a = *reinterpret_cast<const short8*>(Ks + 32 * m * D + koff[kk]);
        s[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[kk], s[m], 0, 0, 0);
      }
    }

    // ---- mask + online softmax (this lane = query row qrow; 32 of the 64 keys).
    // One uniform branch for the (rare) boundary tiles; the row max is taken on the
    // raw scores and scaled once, the scale is folded into the exp2 argument (FMA).
    const bool need_mask = (kt + KT > ctx) || (CAUSAL && kt + KT - 1 > past + q0 + rg * 32);
    float mx = -INFINITY;
    if (need_mask) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kt + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * h;
          const bool ok = key < ctx && (!CAUSAL || key <= qpos);
          s[m][i] = ok ? s[m][i] : -INFINITY;
          mx = fmaxf(mx, s[m][i]);
        }
    } else {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[m][i]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * p.scale_log2;
    const float m_new = fmaxf(m_run, mx);
    const float base = m_new == -INFINITY ? 0.f : m_new;
    // bare v_exp_f32 (softmax tolerates flushed denormals)
    const float alpha = __builtin_amdgcn_exp2f(m_run - base);
    float rs = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[m][i], p.scale_log2, -base));
        s[m][i] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
    // rescale O only when some row's running max moved (wave-uniform branch; once the
    // early tiles have found each row's max this is skipped)
    if (!__all(alpha == 1.f)) {
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[n][i] *= alpha;
    }

    // ---- P^T fragments (B operand): k-step (m, s2) = regs 8*s2 .. 8*s2+7 of s[m]
    short8 pf[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint4_t pk;
#pragma unroll
        for (int j = 0; j < 4; ++j) pk[j] = pack_bf2(s[m][8 * s2 + 2 * j], s[m][8 * s2 + 2 * j + 1]);
        pf[m][s2] = __builtin_bit_cast(short8, pk);
      }

    // ---- O^T += V^T . P^T ; V^T fragments by transposed LDS reads.
    // element j of lane-half h in k-step (m,s2) is key 32m + 16s2 + 8(j>>2) + 4h + (j&3)
#pragma unroll
    for (int n = 0; n < ND; ++n) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16_t* a0 = Vs + (32 * m + 16 * s2) * D + voff[n];
          const bf16_t* a1 = a0 + 8 * D;
          const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short_ptr)(a0));
          const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short_ptr)(a1));
          const short8 a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          o[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pf[m][s2], o[n], 0, 0, 0);
        }
    }
  }

  // ---- epilogue: O^T lane layout: d = 32n + (i&3) + 8(i>>2) + 4h, query row = qrow
  if (qvalid && p.part_o) {
    const long pr = (long)(qbeg + qrow) * p.Hq + head;
    float* po = p.part_o + pr * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<floatx4*>(po + 32 * n + 8 * g4 + 4 * h) =
            floatx4{o[n][4 * g4 + 0], o[n][4 * g4 + 1], o[n][4 * g4 + 2], o[n][4 * g4 + 3]};
    if (h == 0) {
      p.part_ml[pr * 2] = m_run;
      p.part_ml[pr * 2 + 1] = l_run;
    }
  } else if (qvalid) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16_t* op = p.out + (long)(qbeg + qrow) * p.os + (long)head * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * n + 8 * g4 + 4 * h;
        uint2 pk;
        pk.x = pack_bf2(o[n][4 * g4 + 0] * inv, o[n][4 * g4 + 1] * inv);
        pk.y = pack_bf2(o[n][4 * g4 + 2] * inv, o[n][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d) = pk;
      }
  }
}


}  // namespace

// LK_PREFILL_WAVES=8: 8-wave workgroups (64 query rows x 4 heads of a GQA group) for
// G >= 4 at D >= 64.  Measured on MI355X (kernel_bench, 2 runs each): +3-5 % on long causal
// prefill (B8 L4096: 873-889 vs 849 TF/s), -2 % on the serving chunk shape (B6 q643 ctx930:
// 494 vs 503-507), so the 4-wave kernel is the default.
static int prefill_waves(int G, int D) {
  static const int env = [] {
    const char* e = getenv("LK_PREFILL_WAVES");
    return e ? atoi(e) : 4;
  }();
  return (G >= 4 && D >= 64 && env == 8) ? 8 : 4;
}

int lk_prefill_rows_per_tile(int G) { return G >= 4 ? 32 * (prefill_waves(G, 128) / 4) : 32 * (4 / G); }

int lk_flash_prefill(const bf16_t* q, long qs, const bf16_t* k, const bf16_t* v, long ks, long vs,
                     const int* block_tables, int bt_stride, const int* cu_q, const int* ctx_lens,
                     const int* tile_seq, const int* tile_q0, int ntiles, bf16_t* out, long os,
                     int Hq, int Hkv, int D, int BS, float scale, int causal, int paged,
                     float* part_o, float* part_ml, hipStream_t st) {
  if (ntiles == 0) return 0;
  if (Hq % Hkv) return -1;
  const int G = Hq / Hkv;
  if (!(G == 1 || G == 2 || G % 4 == 0)) return -2;
  if (paged && (BS <= 0)) return -4;
  if (paged && (BS & (BS - 1))) return -4;  // power-of-two cache blocks
  if (paged && BS < 512 / D) return -4;     // a wave's staged rows must share one block
  int bs_shift = 0;
  while ((1 << bs_shift) < BS) ++bs_shift;
  PrefillParams pr{q, qs, k, v, ks, vs, block_tables, bt_stride, cu_q, ctx_lens, tile_seq,
                   tile_q0, out, os, Hq, Hkv, BS, bs_shift, scale * 1.4426950408889634f, part_o, part_ml};
  const int WH = G >= 4 ? 4 : G;
  const int NW = prefill_waves(G, D);
  dim3 grid(ntiles, Hq / WH);
#define L(DD, C, PG, W, N) flash_prefill_kernel<DD, C, PG, W, N><<<grid, 64 * N, 0, st>>>(pr)
#define BY_W(DD, C, PG)                                 \
  if (WH == 4 && NW == 8) L(DD, C, PG, 4, (DD >= 64 ? 8 : 4));   \
  else if (WH == 4) L(DD, C, PG, 4, 4);                 \
  else if (WH == 2) L(DD, C, PG, 2, 4);                 \
  else L(DD, C, PG, 1, 4);
#define BY_MODE(DD)                                    \
  if (causal && paged) { BY_W(DD, true, true) }        \
  else if (causal && !paged) { BY_W(DD, true, false) } \
  else if (!causal && paged) { BY_W(DD, false, true) } \
  else { BY_W(DD, false, false) }
  if (D == 128) { BY_MODE(128) }
  else if (D == 64) { BY_MODE(64) }
  else if (D == 32) { BY_MODE(32) }
  else return -3;
#undef BY_MODE
#undef BY_W
#undef L
  return 0;
}
