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
//    written to LDS after the barrier (issue-early / write-late staging).  With PIPE the
//    loop is software-pipelined by one tile (PV(t-1) next to the exponentials of tile t).
//  * paged K/V come in through buffer loads whose descriptor is the cache block's
//    (wave-uniform) base: the per-lane offset is a loop constant, the block-table lookup
//    and the 64-bit base are scalar, so staging a tile costs no address VALU.
//  * online softmax in the exp2 domain with the scale folded into one multiply.
#include <cstdlib>
#include <type_traits>

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
  float defer;  // PIPE: move the running max only when it grows by more than this (log2 units)
  // context parallelism: position of sequence b's first query relative to its FIRST KEY (may be
  // negative or past the keys: this rank holds only a shard of the keys); null = ctx - q_len
  const int* q_past;
  int xcd;  // XCD-aware workgroup order (prefill_xcd())
  int btv;  // block-table entries preloaded per lane (LK_PREFILL_BTV, default 1)
};

// NW waves per workgroup (4 or 8): WH of them share a row group (one head each), and
// NW / WH row groups of 32 queries sit on top of each other, all fed by the same staged
// K/V tile -- with NW = 8 each K/V byte brought into LDS serves 2x the MFMA work.
template <int D, bool CAUSAL, bool PAGED, int WH, int NW, bool PIPE>
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

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int G = p.Hq / p.Hkv;
  // XCD-aware order: the hardware deals workgroups round-robin over the 8 XCDs (each with its own
  // L2); remapped, every XCD walks a contiguous range of (head group, query tile) -- the query
  // tiles of the same KV head and sequence, which read the same K / V tiles, share one L2, and
  // each XCD takes its tiles heaviest first (LK_PREFILL_XCD=0: the plain order)
  const int nx = gridDim.x;
  const int lin = p.xcd ? xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y) : blockIdx.y * nx + blockIdx.x;
  const int bx = lin % nx, by = lin / nx;
  const int head = by * WH + (w % WH);
  const int kvh = head / G;
  const int rg = w / WH;

  const int b = p.tile_seq[bx];
  const int q0 = p.tile_q0[bx];
  const int qbeg = p.cu_q[b];
  const int qlen = p.cu_q[b + 1] - qbeg;
  const int ctx = p.ctx_lens ? p.ctx_lens[b] : qlen;
  const int past = p.q_past ? p.q_past[b] : ctx - qlen;
  const int kend = CAUSAL ? min(ctx, past + q0 + QB) : ctx;

  const int qrow = q0 + rg * 32 + r;  // query index within the sequence (this lane's column)
  const int qpos = past + qrow;        // absolute position
  const bool qvalid = qrow < qlen;

  // Paged K/V: the 64 / (D / 8) rows one wave stages lie in ONE cache block (BS >= 512 / D,
  // checked on the host), so the block-table lookup is wave-uniform: a scalar load and a
  // scalar base per chunk, the lane part (row within block, 16-byte chunk) a constant.
  // Rows past the context re-read the last valid key (block clamped here, slot by the
  // clamped key): never a stale slot, whose bytes could be NaN under a zero P.
  const int kvh_u = by * WH / G;  // == head / G for every wave of the workgroup
  // The sequence's first 64 NBV block-table entries, one per lane, read once: a chunk's block
  // lookup is then a v_readlane instead of a scalar load whose lgkmcnt wait also drained the
  // wave's LDS reads (blocks past them: the scalar load)
  constexpr int NBV = 2;
  int btv[NBV];
  if (PAGED && p.btv) {
    const int nblk = (ctx + p.BS - 1) >> p.bs_shift;
#pragma unroll
    for (int j = 0; j < NBV; ++j) {
      const int bi = lane + 64 * j;
      btv[j] = bi < nblk ? p.block_tables[(long)b * p.bt_stride + bi] : 0;
    }
  }
  auto paged_base = [&](int kt, int row) __attribute__((always_inline)) -> long {
    const int last = (ctx - 1) >> p.bs_shift;
    const int bi = __builtin_amdgcn_readfirstlane(min((kt + row) >> p.bs_shift, last));
    long blk;
    if (p.btv && bi < 64) blk = __builtin_amdgcn_readlane(btv[0], bi);
    else if (p.btv && bi < 128) blk = __builtin_amdgcn_readlane(btv[1], bi - 64);
    else blk = p.block_tables[(long)b * p.bt_stride + bi];
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

  // ---- staging helpers: chunk c of the tile = (row c / CPR, col chunk c % CPR); CPR divides
  // NT, so a lane's column chunk is the same for every i and its row advances by NT / CPR
  short8 kreg[CPT], vreg[CPT];
  const int lch = tid % CPR, lrow = tid / CPR;
  // paged, full tile: slot of row r = (kt & (BS-1)) + (r & (BS-1)) (no carry: kt is a multiple
  // of KT, r < KT) -> a per-lane constant byte offset plus a scalar one
  unsigned poff[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) poff[i] = (unsigned)((((lrow + (NT / CPR) * i) & (p.BS - 1)) * D + lch * 8) * 2);
  const int wrow0 = __builtin_amdgcn_readfirstlane(w) * (64 / CPR);  // first tile row a wave stages
  auto paged_load = [&](const bf16_t* cache, long base, unsigned off, unsigned soff) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(cache + base), (short)0, p.BS * D * 2, 0x00020000);
    return __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, 0));
  };
  // rows of one tile of the K or V cache -> registers
  auto gload_one = [&](const bf16_t* cache, long dstride, int kt, short8* reg) __attribute__((always_inline)) {
    if constexpr (PAGED) {
      if (kt + KT <= ctx) {  // every row a valid key (uniform branch)
        const unsigned soff = (unsigned)((kt & (p.BS - 1)) * D * 2);
#pragma unroll
        for (int i = 0; i < CPT; ++i)
          reg[i] = paged_load(cache, paged_base(kt, wrow0 + (NT / CPR) * i), poff[i], soff);
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int row = lrow + (NT / CPR) * i;
      const int key = min(kt + row, ctx - 1);  // clamp: masked later
      if constexpr (PAGED) {
        const unsigned loff = (unsigned)(((key & (p.BS - 1)) * D + lch * 8) * 2);  // clamped key: a valid slot
        reg[i] = paged_load(cache, paged_base(kt, row), loff, 0);
      } else {
        reg[i] = *reinterpret_cast<const short8*>(cache + (long)(qbeg + key) * dstride + (long)kvh * D + lch * 8);
      }
    }
  };
  auto gload_k = [&](int kt) __attribute__((always_inline)) { gload_one(p.k, p.ks, kt, kreg); };
  auto gload_v = [&](int kt) __attribute__((always_inline)) { gload_one(p.v, p.vs, kt, vreg); };
  auto swrite_k = [&](bf16_t* Ks) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int row = lrow + (NT / CPR) * i;
      *reinterpret_cast<short8*>(Ks + row * D + k_swz<D>(row, lch) * 8) = kreg[i];
    }
  };
  auto swrite_v = [&](bf16_t* Vs) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int row = lrow + (NT / CPR) * i;
      *reinterpret_cast<short8*>(Vs + row * D + v_swz<D>(row, lch) * 8) = vreg[i];
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

  // ---- S^T = K . Q^T  for two 32-key halves
  auto qk = [&](const bf16_t* Ks, floatx16* s) __attribute__((always_inline)) {
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
  };
  // ---- mask + running max (this lane = query row qrow; 32 of the 64 keys).  One uniform
  // branch for the (rare) boundary tiles; the row max is taken on the raw scores and scaled
  // once.  Returns the rescale factor of the accumulated O / l; sets *base for exp_pack.
  // PIPE: the max is only moved when it grows by more than p.defer (LK_PREFILL_DEFER, log2
  // units: P <= 2^defer is as exact in bf16 and the f32 sums have the range), so after the
  // first tiles alpha == 1 and O is not rescaled at all.
  auto stats = [&](int kt, floatx16* s, float* base, auto may_mask) __attribute__((always_inline)) -> float {
    bool need_mask = false;
    if constexpr (decltype(may_mask)::value)
      need_mask = (kt + KT > ctx) || (CAUSAL && kt + KT - 1 > past + q0 + rg * 32);
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
    float m_new = fmaxf(m_run, mx);
    if constexpr (PIPE) m_new = m_new > m_run + p.defer ? m_new : m_run;
    *base = m_new == -INFINITY ? 0.f : m_new;
    // bare v_exp_f32 (softmax tolerates flushed denormals)
    const float alpha = __builtin_amdgcn_exp2f(m_run - *base);
    m_run = m_new;
    return alpha;
  };
  // ---- P = exp2(s * scale - base), row sums into l, P^T fragments (B operand): k-step
  // (m, s2) = regs 8*s2 .. 8*s2+7 of s[m]
  auto exp_pack = [&](floatx16* s, float base, float alpha, short8 (*pf)[2]) __attribute__((always_inline)) {
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
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint4_t pk;
#pragma unroll
        for (int j = 0; j < 4; ++j) pk[j] = pack_bf2(s[m][8 * s2 + 2 * j], s[m][8 * s2 + 2 * j + 1]);
        pf[m][s2] = __builtin_bit_cast(short8, pk);
      }
  };
  // rescale O only when some row's running max moved (wave-uniform branch)
  auto rescale = [&](float alpha) __attribute__((always_inline)) {
    if (!__all(alpha == 1.f)) {
#pragma unroll
      for (int n = 0; n < ND; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[n][i] *= alpha;
    }
  };
  // ---- O^T += V^T . P^T ; V^T fragments by transposed LDS reads.
  // element j of lane-half h in k-step (m,s2) is key 32m + 16s2 + 8(j>>2) + 4h + (j&3)
  auto pv = [&](const bf16_t* Vs, short8 (*pf)[2]) __attribute__((always_inline)) {
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
  };

  bf16_t* Ks = lds;
  bf16_t* Vs = lds + KT * D;
  const int ntiles = (kend + KT - 1) / KT;
  floatx16 s[2];
  short8 pf[2][2];
  if constexpr (!PIPE) {
    if (ntiles > 0) {
      gload_k(0);
      gload_v(0);
    }
    for (int t = 0; t < ntiles; ++t) {
      const int kt = t * KT;
      __syncthreads();  // everyone finished reading the previous tile
      swrite_k(Ks);
      swrite_v(Vs);
      __syncthreads();
      if (t + 1 < ntiles) {
        gload_k(kt + KT);
        gload_v(kt + KT);
      }
      qk(Ks, s);
      float base;
      const float alpha = stats(kt, s, &base, std::true_type{});
      exp_pack(s, base, alpha, pf);
      rescale(alpha);
      pv(Vs, pf);
    }
  } else if (ntiles > 0) {
    // Software-pipelined by one tile: iteration t runs QK(t), then PV(t-1) in the same basic
    // block as the exponentials of tile t (independent work the scheduler interleaves: MFMA
    // next to VALU within the wave), then O <- (O + P(t-1) V(t-1)) * alpha(t).  The LDS holds
    // K(t) and V(t-1); after each tile K(t+1) and V(t) are written and K(t+2) / V(t+1) issued.
    auto stage = [&](int t) __attribute__((always_inline)) {
      __syncthreads();  // K(t) and V(t-1) read by everyone
      if (t + 1 < ntiles) swrite_k(Ks);
      swrite_v(Vs);
      __syncthreads();
      if (t + 2 < ntiles) gload_k((t + 2) * KT);
      if (t + 1 < ntiles) gload_v((t + 1) * KT);
    };
    gload_k(0);
    gload_v(0);
    swrite_k(Ks);
    if (ntiles > 1) gload_k(KT);
    __syncthreads();
    short8 pfp[2][2];
    {
      qk(Ks, s);
      float base;
      const float alpha = stats(0, s, &base, std::true_type{});
      exp_pack(s, base, alpha, pfp);
      stage(0);
    }
    auto step = [&](int t, auto may_mask) __attribute__((always_inline)) {
      qk(Ks, s);
      float base;
      const float alpha = stats(t * KT, s, &base, may_mask);
      pv(Vs, pfp);
      exp_pack(s, base, alpha, pf);
      rescale(alpha);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) pfp[m][s2] = pf[m][s2];
      stage(t);
    };
    // leading tiles that no row of the workgroup masks: a branch-free body, so the row max
    // is scheduled next to PV(t-1) too.  (Unrolling by two to swap pf / pfp instead of
    // copying them takes the kernel to 256 VGPRs and spills.)
    const int nfree = min(ntiles, min(ctx / KT, CAUSAL ? (past + q0 + 1) / KT : ntiles));
    int t = 1;
    for (; t < nfree; ++t) step(t, std::false_type{});
    for (; t < ntiles; ++t) step(t, std::true_type{});
    pv(Vs, pfp);
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
  } else if (!p.part_o) {
    // lanes l and l+32 hold the two halves (4h) of each 8-column group of the same query row:
    // one v_permlane32_swap per dword gives lanes 0-31 group 2k whole and lanes 32-63 group
    // 2k+1 whole, so the row is written with 16-B stores (half the store instructions of the
    // issue-bound tail: CDNA playbook T21).  The swap runs on every lane (the pair shares qvalid).
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16_t* op = p.out + (long)(qbeg + qrow) * p.os + (long)head * D;
#pragma unroll
    for (int n = 0; n < ND; ++n)
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2) {
        unsigned a[2], b[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          a[j] = pack_bf2(o[n][8 * g2 + 2 * j] * inv, o[n][8 * g2 + 2 * j + 1] * inv);
          b[j] = pack_bf2(o[n][8 * g2 + 4 + 2 * j] * inv, o[n][8 * g2 + 4 + 2 * j + 1] * inv);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const auto r2 = __builtin_amdgcn_permlane32_swap(a[j], b[j], false, false);
          a[j] = r2[0];
          b[j] = r2[1];
        }
        if (qvalid) {
          uint4_t pk;
          pk.x = a[0];
          pk.y = a[1];
          pk.z = b[0];
          pk.w = b[1];
          *reinterpret_cast<uint4_t*>(op + 32 * n + 16 * g2 + 8 * h) = pk;
        }
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

// LK_PREFILL_PIPE=1: the software-pipelined tile loop (PV(t-1) beside the exponentials of t)
static bool prefill_pipe() {
  static const bool env = [] {
    const char* e = getenv("LK_PREFILL_PIPE");
    return e ? atoi(e) != 0 : true;
  }();
  return env;
}

static int prefill_btv() {
  static const int env = [] {
    const char* e = getenv("LK_PREFILL_BTV");
    return e ? atoi(e) : 1;
  }();
  return env;
}

static int prefill_xcd() {
  static const int env = [] {
    const char* e = getenv("LK_PREFILL_XCD");
    return e ? atoi(e) : 1;
  }();
  return env;
}

static float prefill_defer() {
  static const float env = [] {
    const char* e = getenv("LK_PREFILL_DEFER");
    return e ? (float)atof(e) : 8.f;
  }();
  return env;
}

// the query rows one workgroup covers: must use the launch's prefill_waves(G, D)
int lk_prefill_rows_per_tile(int G, int D) { return G >= 4 ? 32 * (prefill_waves(G, D) / 4) : 32 * (4 / G); }

int lk_flash_prefill(const bf16_t* q, long qs, const bf16_t* k, const bf16_t* v, long ks, long vs,
                     const int* block_tables, int bt_stride, const int* cu_q, const int* ctx_lens,
                     const int* tile_seq, const int* tile_q0, int ntiles, bf16_t* out, long os,
                     int Hq, int Hkv, int D, int BS, float scale, int causal, int paged,
                     float* part_o, float* part_ml, const int* q_past, hipStream_t st) {
  if (ntiles == 0) return 0;
  if (Hq % Hkv) return -1;
  // 16-B output stores (permlane-paired epilogue): 16-B aligned output rows
  if (part_o == nullptr && (os % 8 || reinterpret_cast<uintptr_t>(out) % 16)) return -5;
  const int G = Hq / Hkv;
  if (!(G == 1 || G == 2 || G % 4 == 0)) return -2;
  if (paged && (BS <= 0)) return -4;
  if (paged && (BS & (BS - 1))) return -4;  // power-of-two cache blocks
  if (paged && BS < 512 / D) return -4;     // a wave's staged rows must share one block
  int bs_shift = 0;
  while ((1 << bs_shift) < BS) ++bs_shift;
  PrefillParams pr{q, qs, k, v, ks, vs, block_tables, bt_stride, cu_q, ctx_lens, tile_seq,
                   tile_q0, out, os, Hq, Hkv, BS, bs_shift, scale * 1.4426950408889634f, part_o, part_ml,
                   part_o ? 0.f : prefill_defer(), q_past, 0, prefill_btv()};
  const int WH = G >= 4 ? 4 : G;
  const int NW = prefill_waves(G, D);
  dim3 grid(ntiles, Hq / WH);
  // XCD-aware order on grids of at most ~2 workgroups per CU slot (the serving chunk, B6 q643 over
  // 930 keys: 69.5 / 68.4 vs 75.5 / 76.1 us); the long-prefill grids of 8192 workgroups run
  // 2-6 % faster in the plain order (profiles/r5_flash_xcd/)
  pr.xcd = prefill_xcd() && (long)ntiles * (Hq / WH) <= 2048;
  const bool pipe = causal && prefill_pipe();
#define L(DD, C, PG, W, N)                                                        \
  if (pipe) flash_prefill_kernel<DD, C, PG, W, N, true><<<grid, 64 * N, 0, st>>>(pr); \
  else flash_prefill_kernel<DD, C, PG, W, N, false><<<grid, 64 * N, 0, st>>>(pr)
#define BY_W(DD, C, PG)                                 \
  if (WH == 4 && NW == 8) { L(DD, C, PG, 4, (DD >= 64 ? 8 : 4)); } \
  else if (WH == 4) { L(DD, C, PG, 4, 4); }                   \
  else if (WH == 2) { L(DD, C, PG, 2, 4); }                   \
  else { L(DD, C, PG, 1, 4); }
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
