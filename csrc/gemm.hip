// K2, prefill / encoder regime: Y[M, N] = epilogue(X[M, K] . W[N, K]^T) for M > 256 rows
// (chunked-prefill and mixed serving steps, encoder index-build batches).
//
// Epilogues (fused, so no second pass over Y):
//   NONE       y = acc
//   SWIGLU     y[:, c] = silu(X Wg^T) * (X Wu^T) for W = [Wg; Wu] (2I rows, out [M, I])
//   BIAS       y = acc + b
//   BIAS_GELU  y = gelu_erf(acc + b)          (BERT / bge / MiniLM FFN up-projection)
//   BIAS_RELU  y = relu(acc + b)              (OPT fc1)
// Each is rounded like the unfused library GEMM -> activation path (bf16 after the bias add,
// bf16 after the activation).
//
// gfx950 design (the 256x256 LDS-DMA / ping-pong GEMM of the CDNA4 playbook, re-derived for
// K-contiguous nn.Linear operands):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); the C tile is 256 x BN with BN = 64 * NF
//     (NF = 4: 256, NF = 3: 192 -- the 192-wide tile turns N = 6144 into 32 column tiles, so
//     an M = 4096 QKV projection is exactly 2 waves of 256 CUs instead of 1.5);
//     each wave owns 128 x 16NF outputs = 8 x NF v_mfma_f32_16x16x32_bf16 fragments;
//   * BK = 64; every K-tile is split into four LDS "slots" that are consumed at different
//     times: SA0 / SA1 = the A rows of the waves' first / second 64-row m-half, SB0 / SB1 =
//     the B rows of their first / second n-half.  Each phase is a READ segment (LDS ->
//     register fragments, LDS-DMA issue) and an MFMA segment closed by raw s_barriers, with
//     waves 4-7 one segment behind waves 0-3 so that on every SIMD one wave's MFMAs overlap
//     its partner's LDS reads.  Two schedules (per-shape choice, ops.tune_gemm):
//       sched 0: 4 phases per K-tile, one per C quadrant (m-half, n-half) in the order (0,0)
//         (0,1) (1,1) (1,0); both B halves stay in registers, so SA0/SB0 die after phase 1,
//         SB1 after 2, SA1 after 3, and each slot of K-tile t+2 is re-staged two phases after
//         its last read (SA0/SB0 in phase 3, SB1 in 4, SA1 in phase 1 of t+1): one counted
//         vmcnt(4 + SB1 loads) per K-tile, three slots (~1.75 K-tiles) in flight;
//       sched 1: 2 phases per K-tile, one per m-half (32 MFMAs per segment, half the
//         barriers); SA0/SB0/SB1 of K-tile t+1 are staged in phase 1 of t and SA1 in phase 2,
//         one K-tile of cover; waves 4-7 hold a static s_setprio 1 instead of per-cluster flips.
//     (PMC, profiles/r2_gemm.md: the barrier waits, not LDS or L2, separate the schedules.)
//   * staging is 16-byte buffer_load ... lds (LDS-DMA) through wave-uniform buffer
//     descriptors: per-lane 32-bit row offsets fixed for the whole K loop, the K offset in an
//     SGPR, rows past M read as zeros by the descriptor's range check (no clamping, no 64-bit
//     address VALU in the loop).  The LDS image is lane-linear with the (row >> 1) & 7 chunk
//     XOR applied on the SOURCE offset, which keeps every ds_read_b128 lane group of the
//     fragment reads on 16 distinct bank slots (SQ_LDS_BANK_CONFLICT = 0);
//   * operands are swapped in the MFMA (A <- W rows, B <- X rows): a lane ends with one
//     output row and 4 consecutive columns per fragment, and the B-slot row order pairs
//     fragments so that it holds 8 consecutive columns: epilogues are per-lane, the stores
//     16-byte packed (the store tail is issue-bound), and SwiGLU pairs the gate / up fragments
//     of the same columns in a lane;
//   * tiles are visited in an XCD-aware order (bijective remap, 4 row tiles x all column
//     tiles per group), so an XCD's ~32 concurrent tiles share their X / W K-slices in L2.
#include <cstdlib>
#include <map>
#include <mutex>

#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kBM = 256, kBK = 64;
constexpr int kSlotA = 128 * 128;  // an A slot: 128 rows x 128 B

enum { EPI_NONE = 0, EPI_SWIGLU = 1, EPI_BIAS = 2, EPI_BIAS_GELU = 3, EPI_BIAS_RELU = 4, EPI_PARTIAL = 5,
       EPI_RESID = 6, EPI_QKV = 7 };
// epilogues that can take the folded-RMSNorm row scale (LkEpi::ss_in)
constexpr bool scalable(int epi) { return epi == EPI_NONE || epi == EPI_SWIGLU || epi == EPI_QKV; }
// LDS layout after the K loop (the staging buffers are dead): [0, 64) stream-K give-up word,
// [64, 64 + 3 KB) row-scale partials (512) + scales (256), then the RESID reduction [4][256]
constexpr int kLdsScale = 64, kLdsResid = 64 + 768 * 4;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
LK_DEVICE __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)min(bytes, 0x7FFFFFF0L), 0x00020000);
}

LK_DEVICE int swz(int row) { return (row >> 1) & 7; }
template <int N>
LK_DEVICE void wait_vm() {  // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched
  static_assert(N >= 0 && N < 16, "vmcnt");
  __builtin_amdgcn_s_waitcnt(N | (0x7 << 4) | (0xF << 8));
}
LK_DEVICE void seg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }

template <int NF>
struct Geo {
  static_assert(NF == 3 || NF == 4, "NF");
  static constexpr int BN = 64 * NF;
  static constexpr int NF0 = 2, NF1 = NF - 2;          // fragments of n-half 0 / 1
  static constexpr int B1ROWS = 4 * 16 * NF1;           // 128 or 64
  static constexpr int OFF_A0 = 0, OFF_A1 = kSlotA, OFF_B0 = 2 * kSlotA, OFF_B1 = 3 * kSlotA;
  static constexpr int BUF = 3 * kSlotA + B1ROWS * 128;  // 64 KB / 56 KB
  static constexpr int G_B1 = B1ROWS / 64;               // LDS-DMA instructions per wave for SB1 (2 / 1)
};

// (kernel bodies are __device__ functions: the buffer-resource type exists for the device
// target only, and a __global__ whose body names it gets no host launch stub)
// stream-K (hybrid data-parallel + stream-K, persistent grid): the last `tiles` tiles of the
// tile order are cut into K-iteration units spread evenly over the grid, ipw units per
// workgroup; a tile's units owned by workgroups b+1, b+2, ... are summed into the fp32 slot of
// that workgroup (ws + slot * 256 * BN, one slot per workgroup: only its FIRST segment can
// start mid-tile) and published with a flag; workgroup b, which owns the tile's first units,
// adds them and runs the epilogue.  The waits only ever point at higher workgroups, which
// compute those segments first, so a resident finaliser never waits on work queued behind it.
struct SkArgs {
  int tiles;      // tiles in the stream-K region (0: every tile data-parallel)
  int split;      // max workgroups sharing one stream-K tile (per-XCD units derived in the kernel)
  float* ws;      // [gridDim.x][256 * BN] fp32 partial tiles
  int* flags;     // [gridDim.x] the launch epoch once the slot's partial is published
  int* err;       // set when a wait gives up (never expected: a bound instead of a hang)
  int epoch;      // this launch's publish value (per-stream counter, never 0): a flag left by
                  // a contributor that published after its finaliser gave up can never
                  // satisfy a later launch's wait
};
enum { SK_FULL = 0, SK_PARTIAL = 1, SK_FINAL = 2 };
constexpr int kSysCoherent = 1 | 16;  // buffer cache policy sc0 | sc1: past L1 and L2

// SC: this instantiation applies the folded-RMSNorm row scale (LkEpi::ss_in set): only those
// carry the partial-sum prefetch registers through the K loop
template <int NF, int EPI, int PH, int PRIO, bool SC>
__device__ __forceinline__ void gemm8_body(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                                           const bf16_t* __restrict__ bias, int M, int K, int I,
                                           bf16_t* __restrict__ out, long ldo, int TM, int TN, int group_m,
                                           int tile, int kt0, int nk, int kz, int mode, int fin_end,
                                           const SkArgs& sk, const LkEpi& ea) {
  using G = Geo<NF>;
  constexpr int BN = G::BN, NF0 = G::NF0, NF1 = G::NF1;
  static_assert(EPI != EPI_SWIGLU || NF == 4, "SwiGLU pairs fragments n and n+2");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // ---- tile of this block: XCD-contiguous logical ids, grouped 4 row tiles at a time
  const int nwg = TM * TN;
  const int L = xcd_remap(tile, nwg);
  const int per_group = group_m * TN;
  const int first = (L / per_group) * group_m;
  const int gm = min(TM - first, group_m);
  const int tm = first + (L % per_group) % gm;
  const int tn = (L % per_group) / gm;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases stay scalar
  const int wr = w >> 2, wc = w & 3;
  const int r = lane & 15, g = lane >> 4;

  // folded RMSNorm, consumer side: thread tid prefetches partials t = (tid >> 8) + 2 i of tile
  // row tid & 255 BEFORE the K loop (their latency hides under it; they are older than every
  // LDS-DMA, so the loop's counted vmcnt waits stay exact); the buffer range check returns 0
  // for t >= ss_nt -- no predicated loads
  constexpr bool has_scale = scalable(EPI) && SC;
  float ssp[16];
  if constexpr (has_scale) {
    {
      const __amdgpu_buffer_rsrc_t srs = rsrc_of(ea.ss_in, (long)ea.ss_nt * ea.ss_ld * 4);
      const unsigned base = (unsigned)(((tid >> 8) * ea.ss_ld + (long)tm * kBM + (tid & 255)) * 4);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        ssp[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               srs, base + (unsigned)(i * 2 * ea.ss_ld * 4), 0, 0));
    }
  }

  // W row feeding B-tile row j
  auto wrow = [&](int j) -> long {
    if constexpr (EPI == EPI_SWIGLU) {
      const int q = j >> 6, jj = j & 63;
      return (jj < 32 ? 0L : (long)I) + (long)tn * 128 + q * 32 + (jj & 31);
    } else {
      return (long)tn * BN + j;
    }
  };
  // slot row -> tile row
  auto a_row = [](int h, int s) { return (s & 63) + ((s >> 6) << 7) + 64 * h; };
  // B slot row -> tile column.  A fragment pair (n, n+1) of an n-half covers 32 columns, and
  // fragment-local column c of fragment n is tile column 8 (c >> 2) + 4 n + (c & 3), so lane
  // group g ends with 8 CONSECUTIVE output columns 8g .. 8g+7 (4 from each fragment): the
  // epilogue stores 16 B per lane (dwordx4) instead of 8 B.  Its store tail is issue-bound
  // (~7 B/cycle/CU with dwordx2: a ~9 us burst per wave of tiles, profiles/r2_gemm_tile_overhead.md),
  // so half the store instructions halve it.  NF = 3: the unpaired third fragment keeps c.
  auto pair_col = [](int rem) { return 8 * ((rem & 15) >> 2) + 4 * (rem >> 4) + (rem & 3); };  // rem < 32
  auto b0_row = [&](int s) { return (s >> 5) * (16 * NF) + pair_col(s & 31); };
  auto b1_row = [&](int s) {
    if constexpr (NF1 == 2) return (s >> 5) * (16 * NF) + 32 + pair_col(s & 31);
    else return (s / (16 * NF1)) * (16 * NF) + 32 + s % (16 * NF1);
  };

  // ---- LDS-DMA sources and per-wave destinations: a wave instruction moves 8 slot rows x
  // 128 B; lane l -> row l >> 3, 16-B chunk l & 7 (source chunk swizzled).  Sources are
  // buffer_load ... lds through wave-uniform descriptors: fixed 32-bit per-lane row offsets, the
  // K offset in an SGPR, rows past M read as zeros by the descriptor's range check.
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, (short)0, (int)min((long)M * ldx * 2, 0x7FFFFFF0L), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)min((long)(EPI == EPI_SWIGLU ? 2 * I : TN * BN) * K * 2, 0x7FFFFFF0L), 0x00020000);
  const int lr = lane >> 3, lc = lane & 7;
  // this workgroup's K-tiles [kt0, kt0 + nk) (split-K: gridDim.y ranges; stream-K: units)
  unsigned aoff[2][2], b0off[2], b1off[G::G_B1];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int s = 16 * w + 8 * i + lr;
      aoff[h][i] = (unsigned)(((long)tm * kBM + a_row(h, s)) * ldx * 2) + ((lc ^ swz(s)) << 4);
    }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = 16 * w + 8 * i + lr;
    b0off[i] = (unsigned)(wrow(b0_row(s)) * K * 2) + ((lc ^ swz(s)) << 4);
  }
#pragma unroll
  for (int i = 0; i < G::G_B1; ++i) {
    const int s = 8 * G::G_B1 * w + 8 * i + lr;
    b1off[i] = (unsigned)(wrow(b1_row(s)) * K * 2) + ((lc ^ swz(s)) << 4);
  }
  auto dma = [&](__amdgpu_buffer_rsrc_t rs, unsigned off, int kt, unsigned char* dst) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)dst, 16, off, (unsigned)(kt0 + kt) * kBK * 2, 0, 0);
  };
  auto issue_a = [&](int h, int kt) {
    unsigned char* d = smem + (kt & 1) * G::BUF + (h ? G::OFF_A1 : G::OFF_A0) + 16 * w * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(xrs, aoff[h][i], kt, d + i * 8 * 128);
  };
  auto issue_b0 = [&](int kt) {
    unsigned char* d = smem + (kt & 1) * G::BUF + G::OFF_B0 + 16 * w * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(wrs, b0off[i], kt, d + i * 8 * 128);
  };
  auto issue_b1 = [&](int kt) {
    unsigned char* d = smem + (kt & 1) * G::BUF + G::OFF_B1 + 8 * G::G_B1 * w * 128;
#pragma unroll
    for (int i = 0; i < G::G_B1; ++i) dma(wrs, b1off[i], kt, d + i * 8 * 128);
  };

  floatx4 acc[8][NF];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragments: lane reads slot row (16-row fragment base + r), k chunk 4 kk + g
  short8 fa[4][2], fb0[NF0][2], fb1[NF1][2];
  const int rsw = swz(r);  // the fragment bases are multiples of 16: swz(base + r) = swz(r)
  auto ld = [&](const unsigned char* slot, int s0, int kk) {
    return *reinterpret_cast<const short8*>(slot + (s0 + r) * 128 + (((4 * kk + g) ^ rsw) << 4));
  };
  auto read_a = [&](const unsigned char* buf, int h) {
    const unsigned char* slot = buf + (h ? G::OFF_A1 : G::OFF_A0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[m][kk] = ld(slot, wr * 64 + m * 16, kk);
  };
  auto read_b0 = [&](const unsigned char* buf) {
#pragma unroll
    for (int n = 0; n < NF0; ++n)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb0[n][kk] = ld(buf + G::OFF_B0, wc * 32 + n * 16, kk);
  };
  auto read_b1 = [&](const unsigned char* buf) {
#pragma unroll
    for (int n = 0; n < NF1; ++n)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb1[n][kk] = ld(buf + G::OFF_B1, wc * 16 * NF1 + n * 16, kk);
  };
  auto mma0 = [&](int mh) {  // quadrant (mh, n-half 0)
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < NF0; ++n)
          acc[mh * 4 + m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[n][kk], fa[m][kk], acc[mh * 4 + m][n], 0, 0, 0);
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
  };
  auto mma1 = [&](int mh) {  // quadrant (mh, n-half 1)
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < NF1; ++n)
          acc[mh * 4 + m][NF0 + n] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[n][kk], fa[m][kk], acc[mh * 4 + m][NF0 + n], 0, 0, 0);
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (PH == 2) {
    // 2 phases per K-tile: X = m-half 0 x both n-halves (32 MFMAs), Y = m-half 1.  SA0/SB0/SB1
    // of K-tile t+1 are staged in X(t) (their buffer's previous tile was last read in X(t-1)),
    // SA1 in Y(t); X(t+1) waits for the first three, Y(t+1) for SA1: one K-tile of cover.
    issue_a(0, 0);
    issue_b0(0);
    issue_b1(0);
    issue_a(1, 0);
    wait_vm<0>();
    seg_barrier();
    if (wr == 1) seg_barrier();
    if constexpr (PRIO == 1) {  // static priority for the lagging (younger) half, no per-cluster flips
      if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
    }
    for (int t = 0; t < nk; ++t) {
      const unsigned char* buf = smem + (t & 1) * G::BUF;
      read_a(buf, 0);
      read_b0(buf);
      read_b1(buf);
      if (t + 1 < nk) {
        issue_a(0, t + 1);
        issue_b0(t + 1);
        issue_b1(t + 1);
        wait_vm<4 + G::G_B1>();  // SA1(t) landed
      } else {
        wait_vm<0>();
      }
      seg_barrier();
      mma0(0);
      mma1(0);
      seg_barrier();
      read_a(buf, 1);
      if (t + 1 < nk) {
        issue_a(1, t + 1);
        wait_vm<2>();  // SA0 / SB0 / SB1 of t+1 landed
      }
      seg_barrier();
      mma1(1);
      mma0(1);
      seg_barrier();
    }
  } else {
  // prologue: K-tile 0 whole, K-tile 1 but its SA1 (issued in phase 1 of K-tile 0, as in
  // the steady state); the counted wait retires exactly K-tile 0
  issue_a(0, 0);
  issue_b0(0);
  issue_b1(0);
  issue_a(1, 0);
  if (nk > 1) {
    issue_a(0, 1);
    issue_b0(1);
    issue_b1(1);
    wait_vm<4 + G::G_B1>();
  } else {
    wait_vm<0>();
  }
  seg_barrier();
  if (wr == 1) seg_barrier();  // waves 4-7 run one segment behind
  if constexpr (PRIO == 1) {  // static priority for the lagging (younger) half instead of per-cluster flips
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  for (int t = 0; t < nk; ++t) {
    const unsigned char* buf = smem + (t & 1) * G::BUF;
    // phase 1: quadrant (0, 0)
    read_a(buf, 0);
    read_b0(buf);
    if (t + 1 < nk) issue_a(1, t + 1);
    seg_barrier();
    mma0(0);
    seg_barrier();
    // phase 2: quadrant (0, 1)
    read_b1(buf);
    seg_barrier();
    mma1(0);
    seg_barrier();
    // phase 3: quadrant (1, 1); SA0 / SB0 of this buffer are dead -> K-tile t+2
    read_a(buf, 1);
    if (t + 2 < nk) {
      issue_a(0, t + 2);
      issue_b0(t + 2);
    }
    seg_barrier();
    mma1(1);
    seg_barrier();
    // phase 4: quadrant (1, 0); SB1 is dead -> K-tile t+2, then K-tile t+1 must have
    // landed (every wave retires its own DMA here; the barrier publishes it)
    if (t + 2 < nk) {
      issue_b1(t + 2);
      wait_vm<4 + G::G_B1>();
    } else {
      wait_vm<0>();
    }
    seg_barrier();
    mma0(1);
    seg_barrier();
  }
  }
  if (wr == 0) seg_barrier();  // equal barrier counts for both halves

  if (mode != SK_FULL) {
    // fp32 tile image, fragment-major: element (f, thread) at f * 512 + tid -> coalesced 16-B rows
    // slot I/O through a buffer descriptor: one per-lane offset VGPR, the fragment offset in an
    // SGPR (raw pointers would hold a 64-bit address pair per fragment and spill the body)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    auto slot_rsrc = [&](int b) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(sk.ws + (long)b * kBM * BN), (short)0, kBM * BN * 4, 0x00020000);
    };
    const int voff = tid * 16;
    if (mode == SK_PARTIAL) {
      const __amdgpu_buffer_rsrc_t rs = slot_rsrc(blockIdx.x);
      // No release / acquire fences: an agent-scope pair costs an L2 write-back / invalidate of
      // the XCD (every XCD has its own L2), after which the whole grid's operands come from
      // beyond L2 again (measured: stream-K 0.45-0.9x of the plain tiling that way).  The
      // partials are written through to memory (sc0 sc1), the stores' acknowledgement awaited,
      // and the flag published with a relaxed system-scope store; the consumer reads flag and
      // partials past L1 and L2 -- no cache maintenance at all.
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[m][n]), rs, voff, (m * NF + n) * 8192,
                                                 kSysCoherent);
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt / lgkmcnt / expcnt 0: every partial store acknowledged
      __syncthreads();
      if (tid == 0) __hip_atomic_store(sk.flags + blockIdx.x, sk.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // no early return: the row loops below skip every store of a partial segment (a return
      // here costs the 8-wave body ~40 VGPRs and spills)
    }
    const int fin = mode == SK_FINAL ? blockIdx.x + 8 * (fin_end + 1) : 0;  // fin_end contributors, stride 8
    // a wait that gives up poisons the tile (NaN) instead of adding a slot that was never
    // published: wrong output must not pass silently (the engine also polls sk.err)
    int* bad = reinterpret_cast<int*>(smem);  // the staging LDS is dead after the K loop
    bool poisoned = false;
    for (int b = blockIdx.x + 8; b < fin; b += 8) {
      if (tid == 0) {
        int spins = 0, gave_up = 0;
        while (__hip_atomic_load(sk.flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != sk.epoch) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1 << 24)) {  // ~seconds: report instead of hanging the queue
            __hip_atomic_store(sk.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gave_up = 1;
            break;
          }
        }
        *reinterpret_cast<volatile int*>(bad) = gave_up;
      }
      __syncthreads();
      if (*reinterpret_cast<volatile int*>(bad)) poisoned = true;
      const __amdgpu_buffer_rsrc_t rs = slot_rsrc(b);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
#pragma unroll
        for (int n = 0; n < NF; ++n)
          acc[m][n] += __builtin_bit_cast(
              floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (m * NF + n) * 8192, kSysCoherent));
        __builtin_amdgcn_sched_barrier(0);  // NF loads in flight at a time: no register spike
      }
      __syncthreads();  // every wave read `bad` before the next contributor's wait rewrites it
    }
    if (poisoned) {
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n) acc[m][n] = floatx4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    }
  }

  // ---- row scales of the folded RMSNorm: s[row] = rsqrt(sum of the partials / H + eps), into LDS
  float* scl = reinterpret_cast<float*>(smem + kLdsScale);
  if constexpr (has_scale) {
    if (mode != SK_PARTIAL) {
      float part = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) part += ssp[i];
      __syncthreads();  // every wave is past its last staging read
      scl[tid] = part;
      __syncthreads();
      if (tid < 256) scl[512 + tid] = rsqrtf((scl[tid] + scl[tid + 256]) * ea.inv_h + ea.eps);
      __syncthreads();
    }
  }
  auto row_scale = [&](int lrow) -> float {
    if constexpr (has_scale) return scl[512 + lrow];
    else return 1.f;
  };

  // ---- epilogue: lane holds row (.. + r); fragment pair (2p, 2p+1) gives it the 8 consecutive
  // columns 32p + 8g .. +7 of its wave's 16NF (the pair_col layout); NF = 3's third fragment
  // the 4 columns 32 + 4g .. +3.  (An LDS-staged whole-row store variant measured 0.98-1.04x
  // and raised every instantiation's VGPRs; removed: profiles/r4_kernels/README.md.)
  constexpr int OW = EPI == EPI_SWIGLU ? 128 : BN;  // output columns of the tile
  auto emit8 = [&](int lrow, int lcol, const float (&y)[8]) {  // lcol: multiple of 8
    uint4_t pk;
    pk.x = pack_bf2(y[0], y[1]);
    pk.y = pack_bf2(y[2], y[3]);
    pk.z = pack_bf2(y[4], y[5]);
    pk.w = pack_bf2(y[6], y[7]);
    *reinterpret_cast<uint4_t*>(out + (long)(tm * kBM + lrow) * ldo + (long)tn * OW + lcol) = pk;
  };
  auto emit4 = [&](int lrow, int lcol, const float (&y)[4]) {  // lcol: multiple of 4
    uint2 pk;
    pk.x = pack_bf2(y[0], y[1]);
    pk.y = pack_bf2(y[2], y[3]);
    *reinterpret_cast<uint2*>(out + (long)(tm * kBM + lrow) * ldo + (long)tn * OW + lcol) = pk;
  };
  float scm[8];  // this lane's 8 row scales (1 unless the folded-norm scale applies)
#pragma unroll
  for (int m = 0; m < 8; ++m) scm[m] = row_scale(wr * 128 + m * 16 + r);

  if constexpr (EPI == EPI_PARTIAL) {  // fp32 partial sums of split kz: out is float [splits, M, ldo]
    float* part = reinterpret_cast<float*>(out) + (long)kz * M * ldo;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M || mode == SK_PARTIAL) continue;
      float* prow = part + (long)row * ldo + tn * BN + wc * 16 * NF;
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int col = (NF == 3 && n == 2) ? 32 + 4 * g : 32 * (n >> 1) + 8 * g + 4 * (n & 1);
        *reinterpret_cast<floatx4*>(prow + col) = acc[m][n];
      }
    }
  } else if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M || mode == SK_PARTIAL) continue;
      const float sc = scm[m];
      float y[8];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          y[4 * h + v] = rbf(lk_silu(rbf(acc[m][h][v] * sc))) * rbf(acc[m][h + 2][v] * sc);
      emit8(wr * 128 + m * 16 + r, wc * 32 + 8 * g, y);
    }
  } else if constexpr (EPI == EPI_RESID) {
    // producer side of the folded norm: r = bf16(r + bf16(acc)) in place, then the partial sum
    // of squares of the new r over this tile's BN columns (lanes r + 16 g, then the 4 wc waves)
    if (mode != SK_PARTIAL) {
      constexpr int NP = NF / 2;
      const __amdgpu_buffer_rsrc_t rrs = rsrc_of(ea.resid, (long)M * ea.ldr * 2);  // rows >= M: 0 / dropped
      float ssm[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const long row = (long)tm * kBM + wr * 128 + m * 16 + r;
        const long cb = (long)tn * BN + wc * 16 * NF;
        u32x4_t rv[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          rv[p] = __builtin_amdgcn_raw_buffer_load_b128(rrs, (unsigned)((row * ea.ldr + cb + 32 * p + 8 * g) * 2), 0, 0);
        u32x2_t rv3;
        if constexpr (NF == 3) rv3 = __builtin_amdgcn_raw_buffer_load_b64(rrs, (unsigned)((row * ea.ldr + cb + 32 + 4 * g) * 2), 0, 0);
        float ss = 0.f;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const unsigned rw[4] = {rv[p].x, rv[p].y, rv[p].z, rv[p].w};
          float y[8];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int j = 4 * h + v;
              const float res = bf2f((bf16_t)((rw[j >> 1] >> (16 * (j & 1))) & 0xFFFF));
              y[j] = rbf(rbf(acc[m][2 * p + h][v]) + res);
              ss += y[j] * y[j];
            }
          u32x4_t pk;
          pk.x = pack_bf2(y[0], y[1]);
          pk.y = pack_bf2(y[2], y[3]);
          pk.z = pack_bf2(y[4], y[5]);
          pk.w = pack_bf2(y[6], y[7]);
          __builtin_amdgcn_raw_buffer_store_b128(pk, rrs, (unsigned)((row * ea.ldr + cb + 32 * p + 8 * g) * 2), 0, 0);
        }
        if constexpr (NF == 3) {
          const unsigned rw[2] = {rv3.x, rv3.y};
          float y[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const float res = bf2f((bf16_t)((rw[v >> 1] >> (16 * (v & 1))) & 0xFFFF));
            y[v] = rbf(rbf(acc[m][2][v]) + res);
            ss += y[v] * y[v];
          }
          u32x2_t pk;
          pk.x = pack_bf2(y[0], y[1]);
          pk.y = pack_bf2(y[2], y[3]);
          __builtin_amdgcn_raw_buffer_store_b64(pk, rrs, (unsigned)((row * ea.ldr + cb + 32 + 4 * g) * 2), 0, 0);
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        ssm[m] = ss;
      }
      float* red = reinterpret_cast<float*>(smem + kLdsResid);  // [4 wc][256 tile rows]
      __syncthreads();  // every wave is past its last staging read
      if (g == 0) {
#pragma unroll
        for (int m = 0; m < 8; ++m) red[wc * 256 + wr * 128 + m * 16 + r] = ssm[m];
      }
      __syncthreads();
      if (tid < 256) {
        const int row = tm * kBM + tid;
        if (row < M) ea.ss_out[(long)tn * ea.ss_out_ld + row] = (red[tid] + red[256 + tid]) + (red[512 + tid] + red[768 + tid]);
      }
    }
  } else if constexpr (EPI == EPI_QKV) {
    // RoPE (interleaved pairs) on the q / k heads + the paged-KV scatter, on the bf16-rounded
    // (row-scaled) projection: the values "GEMM -> rope_kv_" would leave
    const int qcols = ea.hq * ea.hd, kcols = ea.hkv * ea.hd, half = ea.hd >> 1;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M || mode == SK_PARTIAL) continue;
      const float sc = scm[m];
      const int pos = ea.pos[row];
      const int slot = ea.slots ? ea.slots[row] : -1;
      const float* cs = ea.cos_sin + (long)pos * ea.hd;
      bf16_t* orow = out + (long)row * ldo;
      auto group = [&](int c, float* y, int n) {  // n = 8 or 4 consecutive columns c..c+n-1
        for (int j = 0; j < n; ++j) y[j] = rbf(y[j] * sc);
        if (c < qcols + kcols) {
          const int i0 = (c % ea.hd) >> 1;  // first rotation pair
          float cv[4], sv[4];
          if (n == 8) {
            const floatx4 c4 = *reinterpret_cast<const floatx4*>(cs + i0);
            const floatx4 s4 = *reinterpret_cast<const floatx4*>(cs + half + i0);
            for (int q = 0; q < 4; ++q) { cv[q] = c4[q]; sv[q] = s4[q]; }
          } else {
            const float2 c2 = *reinterpret_cast<const float2*>(cs + i0);
            const float2 s2 = *reinterpret_cast<const float2*>(cs + half + i0);
            cv[0] = c2.x; cv[1] = c2.y; sv[0] = s2.x; sv[1] = s2.y;
          }
          for (int q = 0; q < n / 2; ++q) {
            const float a = y[2 * q], b = y[2 * q + 1];
            y[2 * q] = a * cv[q] - b * sv[q];
            y[2 * q + 1] = b * cv[q] + a * sv[q];
          }
        }
        uint4_t pk;
        pk.x = pack_bf2(y[0], y[1]);
        pk.y = pack_bf2(y[2], y[3]);
        if (n == 8) {
          pk.z = pack_bf2(y[4], y[5]);
          pk.w = pack_bf2(y[6], y[7]);
          *reinterpret_cast<uint4_t*>(orow + c) = pk;
        } else {
          *reinterpret_cast<uint2*>(orow + c) = make_uint2(pk.x, pk.y);
        }
        if (c >= qcols && slot >= 0 && ea.kc != nullptr) {
          const bool isv = c >= qcols + kcols;
          const int cc = c - qcols - (isv ? kcols : 0);
          const int h = cc / ea.hd, d = cc - h * ea.hd;
          bf16_t* dst = (isv ? ea.vc : ea.kc) + (((long)(slot / ea.bs) * ea.hkv + h) * ea.bs + slot % ea.bs) * ea.hd + d;
          if (n == 8) *reinterpret_cast<uint4_t*>(dst) = pk;
          else *reinterpret_cast<uint2*>(dst) = make_uint2(pk.x, pk.y);
        }
      };
      const int cb = tn * BN + wc * 16 * NF;
#pragma unroll
      for (int p = 0; p < NF / 2; ++p) {
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v) y[4 * h + v] = acc[m][2 * p + h][v];
        group(cb + 32 * p + 8 * g, y, 8);
      }
      if constexpr (NF == 3) {
        float y[8];
#pragma unroll
        for (int v = 0; v < 4; ++v) y[v] = acc[m][2][v];
        group(cb + 32 + 4 * g, y, 4);
      }
    }
  } else {
    constexpr int NP = NF / 2;  // fragment pairs
    float bv[NF][4];
#pragma unroll
    for (int n = 0; n < NF; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) bv[n][v] = 0.f;
    if constexpr (EPI != EPI_NONE) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint4_t b = *reinterpret_cast<const uint4_t*>(bias + tn * BN + wc * 16 * NF + 32 * p + 8 * g);
        const unsigned bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bv[2 * p + (q >> 1)][2 * (q & 1)] = bf2f((bf16_t)(bw[q] & 0xFFFF));
          bv[2 * p + (q >> 1)][2 * (q & 1) + 1] = bf2f((bf16_t)(bw[q] >> 16));
        }
      }
      if constexpr (NF == 3) {
        const uint2 b = *reinterpret_cast<const uint2*>(bias + tn * BN + wc * 48 + 32 + 4 * g);
        bv[2][0] = bf2f((bf16_t)(b.x & 0xFFFF));
        bv[2][1] = bf2f((bf16_t)(b.x >> 16));
        bv[2][2] = bf2f((bf16_t)(b.y & 0xFFFF));
        bv[2][3] = bf2f((bf16_t)(b.y >> 16));
      }
    }
    auto act = [&](float e, float b) {
      if constexpr (EPI != EPI_NONE) e = rbf(e + b);
      if constexpr (EPI == EPI_BIAS_GELU) e = lk_gelu_erf(e);
      if constexpr (EPI == EPI_BIAS_RELU) e = fmaxf(e, 0.f);
      return e;
    };
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M || mode == SK_PARTIAL) continue;
      const int lrow = wr * 128 + m * 16 + r, lc = wc * 16 * NF;
      if constexpr (EPI == EPI_NONE && has_scale) {
#pragma unroll
        for (int n = 0; n < NF; ++n) acc[m][n] *= scm[m];
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v) y[4 * h + v] = act(acc[m][2 * p + h][v], bv[2 * p + h][v]);
        emit8(lrow, lc + 32 * p + 8 * g, y);
      }
      if constexpr (NF == 3) {
        float y[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) y[v] = act(acc[m][2][v], bv[2][v]);
        emit4(lrow, lc + 32 + 4 * g, y);
      }
    }
  }
  // the scale / RESID epilogues read LDS (scl, red) after the K loop; a persistent or stream-K
  // workgroup goes on to its next tile, whose first LDS-DMA would overwrite them under a slower
  // wave still reading: every wave is done with them before any wave leaves the tile
  if constexpr (has_scale || EPI == EPI_RESID) __syncthreads();
}

// split-K reduction: out[r, c..c+3] = epi(sum_z part[z, r, c..c+3] (+ bias)), rounded like the
// fused epilogues; one thread per 4 columns
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ out,
                                                            long ldo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nq = N / 4;
  if (i >= (long)M * nq) return;
  const int row = (int)(i / nq), col = (int)(i % nq) * 4;
  const long MN = (long)M * N;
  floatx4 a = *reinterpret_cast<const floatx4*>(part + (long)row * N + col);
  for (int z = 1; z < S; ++z) a += *reinterpret_cast<const floatx4*>(part + z * MN + (long)row * N + col);
  float y[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    float e = a[v];
    if constexpr (EPI != EPI_NONE) e = rbf(e + bf2f(bias[col + v]));
    if constexpr (EPI == EPI_BIAS_GELU) e = lk_gelu_erf(e);
    if constexpr (EPI == EPI_BIAS_RELU) e = fmaxf(e, 0.f);
    y[v] = e;
  }
  uint2 pk;
  pk.x = pack_bf2(y[0], y[1]);
  pk.y = pack_bf2(y[2], y[3]);
  *reinterpret_cast<uint2*>(out + (long)row * ldo + col) = pk;
}

// split-K reduction for the RESID epilogue: block (tile tn of 256 columns, row), 64 threads x 4
// columns: r = bf16(r + bf16(sum_z part)) in place, and the tile's partial sum of squares of the
// new r into ss_out[tn][row] -- the same planes the unsplit RESID epilogue writes
__global__ __launch_bounds__(64) void splitk_resid_kernel(const float* __restrict__ part, int S, int M, int N,
                                                          LkEpi ea) {
  const int tn = blockIdx.x, row = blockIdx.y, col = tn * 256 + 4 * threadIdx.x;
  const long MN = (long)M * N;
  floatx4 a = *reinterpret_cast<const floatx4*>(part + (long)row * N + col);
  for (int z = 1; z < S; ++z) a += *reinterpret_cast<const floatx4*>(part + z * MN + (long)row * N + col);
  bf16_t* rp = ea.resid + (long)row * ea.ldr + col;
  const uint2 rv = *reinterpret_cast<const uint2*>(rp);
  const unsigned rw[2] = {rv.x, rv.y};
  float y[4], ss = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    y[v] = rbf(rbf(a[v]) + bf2f((bf16_t)((rw[v >> 1] >> (16 * (v & 1))) & 0xFFFF)));
    ss += y[v] * y[v];
  }
  *reinterpret_cast<uint2*>(rp) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
  ss = wave_sum(ss);
  if (threadIdx.x == 0) ea.ss_out[(long)tn * ea.ss_out_ld + row] = ss;
}

template <int NF, int EPI, int PH, int PRIO, bool SC>
__global__ __launch_bounds__(512, 1) void gemm_kernel(const bf16_t* __restrict__ X, long ldx,
                                                      const bf16_t* __restrict__ W,
                                                      const bf16_t* __restrict__ bias, int M, int K, int I,
                                                      bf16_t* __restrict__ out, long ldo, int TM, int TN, int group_m,
                                                      SkArgs sk, LkEpi ea) {
  // gridDim.x == TM * TN: one tile per workgroup; fewer: persistent workgroups walking the
  // tiles b, b + grid, ... (same XCD: the grid is a multiple of 8), the epilogue stores of one
  // tile drained before the next tile's LDS-DMA prologue (vmcnt counts stores too)
  const int nwg = TM * TN, nkt = K / kBK;
  const int kz = blockIdx.y, ks = gridDim.y;
  const int kt0 = kz * nkt / ks, nk = (kz + 1) * nkt / ks - kt0;
  const int ndp = nwg - sk.tiles;
  // data-parallel tiles first, then this workgroup's stream-K units -- ONE body call site (two
  // inlined copies of the 8-wave body do not fit the register file).  The stream-K tiles stay
  // on the XCD their data-parallel neighbours run on: XCD x (= blockIdx.x % 8) owns the
  // region's tiles with hardware ids ndp + x + 8 j (the tail of its XCD-contiguous chunk of the
  // tile order, so they share X rows / W columns in its L2), and its gridDim.x / 8 workgroups
  // split those tiles' K units evenly; a finaliser's contributors are the next workgroups of
  // the same XCD (blockIdx.x + 8, + 16, ...).  (Spreading the units over the whole grid
  // without this ran 0.5-0.8x of the plain tiling: every tile's operands came from beyond L2.)
  constexpr int NX = 8;
  const int xcd = blockIdx.x % NX, li = blockIdx.x / NX, P = gridDim.x / NX;
  const int cx = sk.tiles > xcd ? (sk.tiles - xcd + NX - 1) / NX : 0;
  // at most sk.split workgroups per tile: a tile cut finer costs its finaliser more partial
  // reads than the balance gains (K 4096 remainders cut 16 ways ran 0.7x); the rest idle
  const int psk = min(P, cx * sk.split);
  const long units = (long)cx * nkt;
  const int ipw = cx ? (int)((units + psk - 1) / psk) : 0;
  int t = blockIdx.x;
  long u = (long)li * ipw;
  const long end = (cx && li < psk) ? min(units, u + ipw) : 0;
  while (true) {
    int tile, a0, n, mode, fin_end = 0;
    if (t < ndp) {
      tile = t;
      a0 = kt0;
      n = nk;
      mode = SK_FULL;
      t += gridDim.x;
    } else if (u < end) {
      const int j = (int)(u / nkt), k0 = (int)(u % nkt);
      const int k1 = (int)min((long)nkt, k0 + (end - u));
      mode = (k0 == 0 && k1 == nkt) ? SK_FULL : (k0 != 0 ? SK_PARTIAL : SK_FINAL);
      // a finaliser's contributors: this XCD's workgroups whose ranges start inside the tile's
      // tail: fin_end of them, local indices li + 1 .. li + fin_end
      const long tile_end = (long)(j + 1) * nkt;
      fin_end = (int)min((long)psk, (tile_end + ipw - 1) / ipw) - li - 1;
      tile = ndp + xcd + NX * j;
      a0 = k0;
      n = k1 - k0;
      u += n;
    } else {
      break;
    }
    gemm8_body<NF, EPI, PH, PRIO, SC>(X, ldx, W, bias, M, K, I, out, ldo, TM, TN, group_m, tile, a0, n, kz, mode,
                                      fin_end, sk, ea);
    wait_vm<0>();
  }
}

// persistent grid (LK_GEMM_PERSIST=1: one workgroup per CU walking the tiles) or one
// workgroup per tile (default)
int gemm_grid(int tiles) {
  static const bool persist = [] {
    const char* e = getenv("LK_GEMM_PERSIST");
    return e && atoi(e) != 0;
  }();
  if (!persist) return tiles;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return tiles < cus ? tiles : cus;
}

// row tiles per XCD group of the tile order (LK_GEMM_GROUP_M, default 4)
int group_rows() {
  static const int g = [] {
    const char* e = getenv("LK_GEMM_GROUP_M");
    const int v = e ? atoi(e) : 4;
    return v >= 1 ? v : 4;
  }();
  return g;
}

int cu_count() {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return cus;
}

// stream-K policy (LK_GEMM_STREAMK=0 disables): a grid whose last wave of tiles would leave
// CUs idle -- tiles % CUs in (0, 0.85 x CUs) -- runs persistent with that remainder spread as
// K units over every CU.  Not inside a hipGraph capture (the per-stream workspace is
// allocated and zeroed on first use, outside any capture).
int g_streamk = -1;
long g_sk_launches = 0;  // stream-K grids launched (tests: the policy really engaged)
struct SkWs {
  float* ws = nullptr;
  int* flags = nullptr;
  int* err = nullptr;
  long ws_floats = 0;
  int slots = 0;
  int epoch = 0;
};

std::mutex g_sk_mu;
std::map<hipStream_t, SkWs> g_sk_pool;

bool sk_plan(int M, int tiles, int nkt, int bn, hipStream_t st, SkArgs* sk, int* grid) {
  if (g_streamk < 0) {
    const char* e = getenv("LK_GEMM_STREAMK");
    g_streamk = e ? atoi(e) : 1;
  }
  // decoder prefill GEMMs only (M >= 1024, K >= 4096): the encoder GEMMs (K 768 / 3072) that
  // run on side streams (query encodes next to the engine's steps) never put a second
  // persistent stream-K grid on the CUs -- two such grids whose waiting workgroups filled an
  // XCD could each wait for a workgroup that cannot be dispatched
  if (!g_streamk || nkt < 64 || M < 1024) return false;
  static const int grid_cap = [] {  // LK_GEMM_SK_GRID: persistent grid size override (probes)
    const char* e = getenv("LK_GEMM_SK_GRID");
    return e ? atoi(e) : 0;
  }();
  const int G = grid_cap > 0 ? min(grid_cap, cu_count()) : cu_count();
  if (G % 8) return false;  // the kernel splits the grid into 8 XCD groups
  // only a short tail after at least one whole wave: a large remainder cut into K units breaks
  // the lockstep K walk that lets an XCD's tiles share K-slices in its L2 (measured: all-stream-K
  // grids of 144-208 tiles ran 0.55-0.7x of the plain partial wave, which is already ~0.95x
  // efficient per tile); a tail of <= half a wave after whole waves is what it fixes (K 14336
  // down projection at 272-336 tiles: 1.10-1.20x)
  const int rem = tiles % G;
  if (rem == 0 || tiles < G || 2 * rem > G) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  std::lock_guard<std::mutex> lock(g_sk_mu);
  SkWs& w = g_sk_pool[st];
  const long need = (long)G * kBM * bn;
  if (w.ws_floats < need || w.slots < G) {
    if (hipStreamSynchronize(st) != hipSuccess) return false;
    if (w.ws) (void)hipFree(w.ws);
    if (w.flags) (void)hipFree(w.flags);
    w = SkWs{};
    if (hipMalloc(&w.ws, need * sizeof(float)) != hipSuccess) return false;
    if (hipMalloc(&w.flags, (G + 1) * sizeof(int)) != hipSuccess) return false;
    if (hipMemset(w.flags, 0, (G + 1) * sizeof(int)) != hipSuccess) return false;
    w.err = w.flags + G;
    w.ws_floats = need;
    w.slots = G;
  }
  static const int split = [] {  // LK_GEMM_SK_SPLIT: max workgroups per stream-K tile
    const char* e = getenv("LK_GEMM_SK_SPLIT");
    const int v = e ? atoi(e) : 4;
    return v >= 1 ? v : 4;
  }();
  ++g_sk_launches;
  w.epoch = w.epoch >= 0x7FFFFFF0 ? 1 : w.epoch + 1;
  sk->epoch = w.epoch;
  sk->tiles = rem;
  sk->split = split;
  sk->ws = w.ws;
  sk->flags = w.flags;
  sk->err = w.err;
  *grid = G;
  return true;
}

template <int NF, int EPI, int PH, int PRIO, bool SC>
void launch_sc(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
               long ldo, int TM, int TN, int ks, hipStream_t st, const LkEpi& ea) {
  constexpr int lds = 2 * Geo<NF>::BUF;
  LK_SET_MAX_LDS((gemm_kernel<NF, EPI, PH, PRIO, SC>), lds);
  SkArgs sk{0, 0, nullptr, nullptr, nullptr, 0};
  int grid = gemm_grid(TM * TN);
  if (ks == 1 && EPI != EPI_PARTIAL) sk_plan(M, TM * TN, K / kBK, 64 * NF, st, &sk, &grid);
  gemm_kernel<NF, EPI, PH, PRIO, SC><<<dim3(grid, ks), 512, lds, st>>>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN,
                                                                       group_rows(), sk, ea);
}
template <int NF, int EPI, int PH, int PRIO = 0>
void launch_ph(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
               long ldo, int TM, int TN, int ks, hipStream_t st, const LkEpi& ea) {
  if constexpr (scalable(EPI)) {
    if (ea.ss_in != nullptr) {
      launch_sc<NF, EPI, PH, PRIO, true>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st, ea);
      return;
    }
  }
  launch_sc<NF, EPI, PH, PRIO, false>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st, ea);
}
// schedule: 0 = 4 phases per K-tile (per-cluster priority), 1 = 2 phases (static priority)
template <int NF, int EPI>
void launch(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
            long ldo, int TM, int TN, int sched, hipStream_t st, int ks = 1, const LkEpi& ea = LkEpi{}) {
  if (sched == 1) launch_ph<NF, EPI, 2, 1>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st, ea);
  else if (sched == 2) launch_ph<NF, EPI, 4, 1>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st, ea);
  else launch_ph<NF, EPI, 4, 0>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st, ea);
}

template <int NF>
int dispatch(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi,
             int sched, int ks, float* ws, bf16_t* out, long ldo, hipStream_t st, const LkEpi& ea) {
  const int TM = (M + kBM - 1) / kBM;
  constexpr int BN = 64 * NF;
  if (ks > 1) {  // fp32 partials of ks K-ranges into ws [ks, M, N], then the reduce applies the epilogue
    if (epi == EPI_SWIGLU || epi == EPI_QKV || N % BN || ws == nullptr || (epi >= EPI_BIAS && epi <= EPI_BIAS_RELU && bias == nullptr))
      return -1;
    launch<NF, EPI_PARTIAL>(x, ldx, w, nullptr, M, K, 0, reinterpret_cast<bf16_t*>(ws), N, TM, N / BN, sched, st, ks);
    if (epi == EPI_RESID) {
      splitk_resid_kernel<<<dim3(N / 256, M), 64, 0, st>>>(ws, ks, M, N, ea);
      return 0;
    }
    const long n = (long)M * (N / 4);
    const int blocks = (int)((n + 255) / 256);
    switch (epi) {
      case EPI_NONE: splitk_reduce_kernel<EPI_NONE><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS: splitk_reduce_kernel<EPI_BIAS><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS_GELU: splitk_reduce_kernel<EPI_BIAS_GELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS_RELU: splitk_reduce_kernel<EPI_BIAS_RELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      default: return -1;
    }
    return 0;
  }
  if (epi == EPI_SWIGLU) {
    if constexpr (NF != 4) {
      return -1;
    } else {
      if (N % 2 || (N / 2) % 128) return -1;
      launch<4, EPI_SWIGLU>(x, ldx, w, bias, M, K, N / 2, out, ldo, TM, N / 256, sched, st, 1, ea);
      return 0;
    }
  }
  if (N % BN) return -1;
  if (epi >= EPI_BIAS && epi <= EPI_BIAS_RELU && bias == nullptr) return -1;
  switch (epi) {
    case EPI_NONE: launch<NF, EPI_NONE>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / BN, sched, st, 1, ea); break;
    case EPI_BIAS: launch<NF, EPI_BIAS>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / BN, sched, st); break;
    case EPI_BIAS_GELU: launch<NF, EPI_BIAS_GELU>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / BN, sched, st); break;
    case EPI_BIAS_RELU: launch<NF, EPI_BIAS_RELU>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / BN, sched, st); break;
    case EPI_RESID:
      if constexpr (NF != 4) return -1;  // partial planes per 256 columns (same as the split-K reduce)
      else launch<4, EPI_RESID>(x, ldx, w, nullptr, M, K, 0, out, ldo, TM, N / BN, sched, st, 1, ea);
      break;
    case EPI_QKV: launch<NF, EPI_QKV>(x, ldx, w, nullptr, M, K, 0, out, ldo, TM, N / BN, sched, st, 1, ea); break;
    default: return -1;
  }
  return 0;
}

}  // namespace

// stream-K waits that gave up since the last call (0 expected), over every stream's workspace;
// mode >= 0 sets the policy (0 off, 1 on), -1 leaves it; -2 returns the stream-K launches so far
int lk_gemm_streamk(int mode) {
  if (mode == -2) return (int)g_sk_launches;
  if (mode >= 0) g_streamk = mode;
  std::lock_guard<std::mutex> lock(g_sk_mu);
  int errs = 0;
  for (auto& kv : g_sk_pool) {
    int e = 0;
    if (kv.second.err && hipMemcpy(&e, kv.second.err, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess && e) {
      errs += e;
      (void)hipMemset(kv.second.err, 0, sizeof(int));
    }
  }
  return errs;
}

int lk_gemm_supported(int M, int N, int K, int epi, int bn, int ks) {
  if (M < 1 || K < kBK || K % kBK || (bn != 192 && bn != 256)) return 0;
  if (ks < 1 || ks > 8 || K / kBK < 2 * ks || (ks > 1 && (epi == EPI_SWIGLU || epi == EPI_QKV || N % 4))) return 0;
  if (epi == EPI_SWIGLU) return bn == 256 && N % 2 == 0 && (N / 2) % 128 == 0;
  if (epi == EPI_RESID) return bn == 256 && N % 256 == 0;
  if (epi == EPI_QKV) return N % bn == 0;
  return epi >= EPI_NONE && epi <= EPI_BIAS_RELU && N % bn == 0;
}

// out = epi(X W^T (+ bias)): X [M, K] (row stride ldx), W [N, K] contiguous, out [M, N] (SwiGLU:
// [M, N/2]) with row stride ldo.  bn = 256 or 192 (column tile).  Requires K % 64 == 0,
// N % bn == 0 (SwiGLU: bn = 256 and I = N/2 % 128 == 0), 16-B aligned X / W rows and
// 8-B aligned output rows; any M >= 1.
int lk_gemm(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi, int bn,
            int variant, bf16_t* out, long ldo, hipStream_t st, int ks, float* ws, const LkEpi* ea_) {
  if (lk_gemm1w_bm(variant)) {  // the one-wave-per-SIMD kernel (csrc/gemm1w.hip): 256-wide column tiles
    if (bn != 256) return -1;
    return lk_gemm1w(x, ldx, w, bias, M, N, K, epi, out, ldo, st, ks, ws, ea_, 0, lk_gemm1w_bm(variant));
  }
  LkEpi ea = ea_ ? *ea_ : LkEpi{};
  // fused-chain epilogue arguments (checked here: a bad pointer / shape would fault the device)
  if (ea.ss_in && (ea.ss_nt < 1 || ea.ss_nt > 32 || ea.ss_ld < M || ea.inv_h <= 0.f)) return -1;
  // the split-K partial / reduce kernels carry no row scale: refuse instead of dropping it
  if (ea.ss_in && ks > 1) return -1;
  if (epi == EPI_RESID && (!ea.resid || !ea.ss_out || ea.ldr % 8 || ea.ss_out_ld < M)) return -1;
  if (epi == EPI_QKV && (!ea.pos || !ea.cos_sin || ea.hd % 16 || ea.hd <= 0 ||
                         N != (ea.hq + 2 * ea.hkv) * ea.hd || ((ea.kc || ea.vc) && (!ea.slots || ea.bs < 1))))
    return -1;
  // 16-B epilogue stores / bias loads: output rows and the bias 16-B aligned
  if (!lk_gemm_supported(M, N, K, epi, bn, ks) || ldx % 8 || ldo % 8 || reinterpret_cast<uintptr_t>(out) % 16 ||
      (bias != nullptr && reinterpret_cast<uintptr_t>(bias) % 16))
    return -1;
  // operands are addressed through 32-bit buffer offsets: W must fit, X is cut into row chunks
  if ((long)N * K * 2 >= 0x7FFFFFF0L) return -1;
  const long max_rows = (0x7FFFFFF0L / (ldx * 2)) / kBM * kBM;
  if (M > max_rows) {
    if (max_rows < kBM) return -1;
    for (long m0 = 0; m0 < M; m0 += max_rows) {
      const int mc = (int)min((long)M - m0, max_rows);
      if (ea_) return -1;  // the fused-chain epilogues index whole-M side buffers
      const int rc = lk_gemm(x + m0 * ldx, ldx, w, bias, mc, N, K, epi, bn, variant, out + m0 * ldo, ldo, st, 1, nullptr);
      if (rc) return rc;
    }
    return 0;
  }
  if (variant < 0 || variant > 2) return -1;
  const int rc = bn == 256 ? dispatch<4>(x, ldx, w, bias, M, N, K, epi, variant, ks, ws, out, ldo, st, ea)
                           : dispatch<3>(x, ldx, w, bias, M, N, K, epi, variant, ks, ws, out, ldo, st, ea);
  LK_CHECK_LAUNCH();
  return rc;
}
