// K2, prefill regime, one wave per SIMD: Y[M, N] = epilogue(X[M, K] . W[N, K]^T).
//
// The 256 x 256-tile schedule of hipBLASLt's gfx950 bf16 kernels
// (Cijk_..._MT256x256x64_MI16x16x1_..._DTLA1_DTLB1_PGR2_PLR1_..._WG32_8_1: its K loop read from
// the disassembly of the installed library), rebuilt in HIP for our K-contiguous operands and
// extended with the fused serving epilogues of gemm.hip and with 192 / 128-row tiles:
//   * 256 threads = 4 waves, ONE per SIMD, as 2 (M) x 2 (N); each wave owns (BM / 2) x 128 outputs =
//     MB x 8 v_mfma_f32_16x16x32_bf16 accumulators (MB = BM / 32: 8 / 6 / 4) pinned to AGPRs by
//     inline-asm MFMAs ("+a"); the first K-tile's MFMAs take an inline 0 as C (no zeroing pass);
//   * BK = 64, two LDS stages of (BM + 256) x 128 B (X rows | W rows, (row >> 1) & 7 chunk XOR
//     applied on the DMA SOURCE: lane-linear LDS image, conflict-free ds_read_b128);
//   * a full K-tile of fragments lives in registers (kk 0 and kk 1 sets); every LDS read, LDS-DMA
//     issue and wait is inline asm placed by hand among the NM = 16 MB MFMAs of a K-tile (BM 256:
//     positions below; 192 / 128: Tile<BM>):
//       top          : lgkmcnt(0) -- the (t, kk 0) fragments read at the end of K-tile t-1
//       MFMA  0..15  : the 16 fragment reads of (t, kk 1), one per MFMA
//       MFMA 26      : lgkmcnt(0) + s_barrier -- every wave is done with stage t & 1
//       MFMA 28..103 : the 16 LDS-DMA pieces (1 KB each) of K-tile t+2 into stage t & 1, one per
//                      5 MFMAs, M0 for the next piece written 2 MFMAs after each issue (no s_nop)
//       MFMA 108     : vmcnt(16) + s_barrier -- K-tile t+1 (issued one K-tile ago) has landed
//       MFMA 108..123: the 16 fragment reads of (t+1, kk 0)
//     (probe sweeps of these positions, the wait placement and the M0 lag:
//     benchmarks/gemm1w_probe.py, profiles/r5_gemm1w/);
//   * row tiles of 192 / 128 fill the 256 CUs where 256-row tiles leave most of a wave idle (the
//     serving bench's mixed steps: M = prefill chunk + ~105 decode rows); the dispatch picks the
//     row tile per M bucket from measurements (ops.tune_gemm, benchmarks/gemm_tiles.py);
//   * one tile per workgroup: the hardware starts the next workgroup on a CU while the finished
//     one's epilogue stores drain (a persistent walk with the next tile's first K-tiles DMA'd
//     during the last one measured 1-3 % slower);
//   * operands swapped in the MFMA (A <- W rows, B <- X rows) and the W rows of every 32-row
//     block permuted (pair_col) so a lane ends with one output row and 8 consecutive columns
//     per fragment pair: 16-B epilogue stores; SwiGLU pairs gate / up of the same columns;
//   * epilogues (same contracts and rounding as gemm.hip): NONE, SWIGLU, BIAS, BIAS_GELU,
//     BIAS_RELU, PARTIAL (split-K fp32 slabs), RESID (r += acc in place + per-row partial sums of
//     squares), QKV (RoPE + paged-KV scatter); NONE / SWIGLU / QKV take the folded-RMSNorm row
//     scale (LkEpi::ss_in); rows past M are dropped by the buffer descriptors' range checks.
#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));

constexpr int kBN = 256, kBK = 64;
constexpr int kRowB = kBK * 2;          // 128-B LDS rows
constexpr int kLdsEpi = 8192;           // epilogue scratch above the stages (row scales, RESID sums)

// Row-tile height BM (256, 192 or 128; the column tile is always 256): the 4 waves sit 2 (M) x 2 (N),
// each owning (BM / 2) x 128 outputs = MB x 8 accumulators of 16 x 16.  A K-tile is NM = 16 MB
// MFMAs, NR = MB + 8 fragment reads per kk set and NP = BM / 32 + 8 LDS-DMA pieces per wave.
// Smaller row tiles fill the 256 CUs where 256-row tiles leave most of a wave idle (M 2664,
// N 4096: 176 tiles of 256 rows, 224 of 192 rows -- the row tile hipBLASLt picks there).
template <int BM>
struct Tile {
  static constexpr int MB = BM / 32, NM = 16 * MB, NR = MB + 8, PX = BM / 32, NP = PX + 8;
  static constexpr int kOpX = BM * kRowB;                // X rows of one stage
  static constexpr int kStage = kOpX + 256 * kRowB;      // X rows then W rows
  static constexpr int kLdsStages = 2 * kStage;          // 128 / 112 / 96 KB
  static constexpr int kLds = kLdsStages + kLdsEpi;
  // K-loop schedule (MFMA indices within the NM of a K-tile): barrier 1, first DMA piece, DMA
  // spacing, M0 lag, barrier 2
  static constexpr int B1 = BM == 256 ? 26 : BM == 192 ? 24 : 14;
  static constexpr int D0 = B1 + 2;
  static constexpr int DS = BM == 256 ? 5 : BM == 192 ? 4 : 2;
  static constexpr int LAG = BM == 128 ? 1 : 2;
  static constexpr int B2 = BM == 256 ? 108 : BM == 192 ? 82 : 48;
  static_assert(NR - 1 < B1 && B1 < D0 && LAG < DS && D0 + DS * (NP - 1) + LAG < B2 && B2 + NR <= NM, "schedule");
};

enum { E_NONE = 0, E_SWIGLU = 1, E_BIAS = 2, E_BIAS_GELU = 3, E_BIAS_RELU = 4, E_PARTIAL = 5, E_RESID = 6,
       E_QKV = 7 };
constexpr bool scalable(int e) { return e == E_NONE || e == E_SWIGLU || e == E_QKV; }

template <class Fn, int... I>
LK_DEVICE void unroll_impl(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
LK_DEVICE void unroll(Fn&& f) {
  unroll_impl(f, std::make_integer_sequence<int, N>{});
}

template <int N>
LK_DEVICE void wait_vm() {  // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
LK_DEVICE void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
LK_DEVICE void barrier_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
LK_DEVICE void fence() { __builtin_amdgcn_sched_barrier(0); }
LK_DEVICE int swz(int row) { return (row >> 1) & 7; }
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }
LK_DEVICE unsigned rfl(unsigned v) { return (unsigned)__builtin_amdgcn_readfirstlane((int)v); }

// acc (+)= W-frag (16 x 32) . X-frag (32 x 16), acc pinned to AGPRs; volatile keeps issue order
LK_DEVICE void mfma(floatx4& acc, const short8& a, const short8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
LK_DEVICE void mfma0(floatx4& acc, const short8& a, const short8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}
LK_DEVICE void set_m0(unsigned v) { asm volatile("s_mov_b32 m0, %0" ::"s"(v) : "memory", "m0"); }
LK_DEVICE u32x4_t srd(const void* p, long bytes) {  // buffer descriptor words, wave-uniform
  const unsigned long a = reinterpret_cast<unsigned long>(p);
  return u32x4_t{rfl((unsigned)a), rfl((unsigned)(a >> 32)), (unsigned)min(bytes, 0x7FFFFFF0L), 0x00020000u};
}

// vector-memory operations per lane of the plain / bias epilogues (bias loads, then stores): the
// persistent walk's counted wait for the next tile's first K-tile skips them
template <int EPI, int MB>
constexpr int epi_vm_ops() { return (EPI == E_NONE ? 0 : 4) + 4 * MB; }
constexpr bool persistable(int e) { return e == E_NONE || e == E_BIAS || e == E_BIAS_GELU || e == E_BIAS_RELU; }

// SCP: partial-sum planes of the folded-RMSNorm row scale loaded per row (0: no row scale; 16 covers
// a 4096-wide producer, 32 an 8192-wide one).  PERSIST: one workgroup per CU walks the tiles
// blockIdx.x, + gridDim.x, ...; the next tile's first two K-tiles are DMA'd during the current
// tile's last two, so its load ramp hides behind the current epilogue (short-K shapes: the
// encoder's K = 768 projections, 12 K-tiles per tile)
template <int EPI, int SCP, int BM, bool PERSIST = false>
__global__ __launch_bounds__(256, 1) void gemm1w_kernel(const bf16_t* __restrict__ X, long ldx,
                                                        const bf16_t* __restrict__ W,
                                                        const bf16_t* __restrict__ bias, int M, int K, int I,
                                                        bf16_t* __restrict__ out, long ldo, int TM, int TN,
                                                        int tn0, int group_m, LkEpi ea) {
  constexpr bool SC = SCP > 0;
  static_assert(!SC || scalable(EPI), "row scale");
  static_assert(!PERSIST || (persistable(EPI) && !SC), "persistent walk: plain / bias epilogues");
  using TL = Tile<BM>;
  constexpr int MB = TL::MB, NM = TL::NM, NR = TL::NR, PX = TL::PX, NP = TL::NP, WM = BM / 2;
  constexpr int kOpX = TL::kOpX, kStage = TL::kStage, kLdsStages = TL::kLdsStages;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int r = lane & 15, g = lane >> 4;
  const int nwg = TM * TN;
  const int nkt = K / kBK, kz = blockIdx.y, ks = gridDim.y;
  const int kt0 = kz * nkt / ks, nk = (kz + 1) * nkt / ks - kt0;  // >= 3 (host check)

  auto coords = [&](int tile, int& tm, int& tn) {
    const int L = xcd_remap(tile, nwg);
    const int per_group = group_m * TN;
    const int first = (L / per_group) * group_m;
    const int gm = min(TM - first, group_m);
    tm = first + (L % per_group) % gm;
    tn = tn0 + (L % per_group) / gm;  // (tn0: a column-split launch's first column tile)
  };
  const u32x4_t xsrd = srd(X, (long)M * ldx * 2);
  const u32x4_t wsrd = srd(W, (long)(EPI == E_SWIGLU ? 2 * I : (tn0 + TN) * kBN) * K * 2);
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_ptr_t)smem));
  const unsigned ldsx = rfl(lds0 + (BM / 4) * w * kRowB), ldsw = rfl(lds0 + kOpX + 64 * w * kRowB);

  // ---- LDS-DMA piece i (0..NP-1) of a K-tile: rows BM/4 w + 8 i + (lane >> 3) of X (i < PX) or
  // 64 w + 8 (i - PX) + (lane >> 3) of W, 16-B chunk lane & 7 (source chunk swizzled); per-lane
  // row offsets of the tile
  const int lr8 = lane >> 3, lc8 = lane & 7;
  unsigned xo[PX], wo[8], xo2[PX], wo2[8];  // this tile's / (PERSIST) the next tile's
  int par = 0;  // stage of tile-relative K-tile t: (t + par) & 1 (a persistent walk carries it on)
  // (32-bit: the host keeps every operand under 2^31 bytes).  Closed forms with the piece index
  // i in immediates only -- per-i lane constants held across the tile loop spill:
  //   row = BM/4 w + 8 i + lr8;  swz(row) = (lr8 >> 1) ^ 4 (i & 1)  (BM/8 w is a multiple of 8);
  //   W row = lane part + 32 (i >> 2) + 16 (i & 1) + 4 ((i >> 1) & 1)   (pair_col of row & 31)
  const unsigned ldxb = (unsigned)ldx * 2, kb = (unsigned)K * 2;
  const unsigned ch0 = (unsigned)((lc8 ^ (lr8 >> 1)) << 4);
  auto offsets = [&](int tm, int tn, unsigned (&xo)[PX], unsigned (&wo)[8]) {
    const unsigned xb = (unsigned)(tm * BM + (BM / 4) * w + lr8) * ldxb;
    const int lanew = 8 * (lr8 >> 2) + (lr8 & 3);
    const unsigned wl = EPI == E_SWIGLU ? (unsigned)((w & 1) * I + tn * 128 + (w >> 1) * 64 + lanew)
                                        : (unsigned)(tn * kBN + 64 * w + lanew);
    const unsigned wb = wl * kb;
#pragma unroll
    for (int i = 0; i < PX; ++i) xo[i] = xb + (unsigned)(8 * i) * ldxb + (ch0 ^ (unsigned)((i & 1) << 6));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      wo[i] = wb + (unsigned)(32 * (i >> 2) + 16 * (i & 1) + 4 * ((i >> 1) & 1)) * kb + (ch0 ^ (unsigned)((i & 1) << 6));
  };
  auto piece_m0 = [&](int t, int i) -> unsigned {  // LDS base of piece i of (tile-relative) K-tile t
    return i < PX ? ldsx + (unsigned)(((t + par) & 1) * kStage + 8 * i * kRowB)
                  : ldsw + (unsigned)(((t + par) & 1) * kStage + 8 * (i - PX) * kRowB);
  };
  // issue piece i of K-tile t (M0 already holds its LDS base); NEXT: K-tile t - nk of the next tile
  auto dma = [&](bool NEXT, int t, int i) {  // (NEXT is a constant at every call: folded when inlined)
    const unsigned so = rfl((unsigned)(NEXT ? t - nk : kt0 + t) * (kBK * 2));
    const unsigned xv = NEXT ? xo2[i < PX ? i : 0] : xo[i < PX ? i : 0];
    const unsigned wv = NEXT ? wo2[i < PX ? 0 : i - PX] : wo[i < PX ? 0 : i - PX];
    if (i < PX) asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(xv), "s"(xsrd), "s"(so) : "memory");
    else asm volatile("buffer_load_dwordx4 %0, %1, %2 offen sc0 sc1 lds" ::"v"(wv), "s"(wsrd), "s"(so) : "memory");
  };

  // ---- fragments: lane reads stage row (16-row base + r), 16-B chunk 4 kk + g, from per-(kk,
  // operand) base VGPRs with the fragment offset as immediate
  const int rs = swz(r);
  unsigned bx[2], bw[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const unsigned b = lds0 + (((4 * kk + g) ^ rs) << 4) + r * kRowB;
    bx[kk] = b + wr * WM * kRowB;
    bw[kk] = b + kOpX + wc * 128 * kRowB;
  }
  short8 fx0[MB], fw0[8], fx1[MB], fw1[8];
  // read j in the consumption order of the MFMA loop: fw[0], fx[0..MB-1], fw[1..7]
  auto rd = [](unsigned bxv, unsigned bwv, auto j_t, short8(&fx)[MB], short8(&fw)[8]) {
    constexpr int j = decltype(j_t)::value;
    if constexpr (j == 0)
      asm volatile("ds_read_b128 %0, %1" : "=v"(fw[0]) : "v"(bwv));
    else if constexpr (j <= MB)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fx[j - 1]) : "v"(bxv), "i"((j - 1) * 16 * kRowB));
    else
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fw[j - MB]) : "v"(bwv), "i"((j - MB) * 16 * kRowB));
  };
  floatx4 acc[MB][8];
  using T = std::true_type;
  using F = std::false_type;

  // ---- folded RMSNorm, consumer side: thread tid sums the ss_nt partials of tile row tid.  The
  // loads are inline asm issued BEFORE the prologue's LDS-DMA, so the prologue's counted wait
  // retires them and they are summed right after it (hipcc would otherwise wait for them with
  // a vmcnt(0) in the middle of the K loop, draining the LDS-DMA pipeline)
  float* scl = reinterpret_cast<float*>(smem + kLdsStages);  // [256] row scales
  float ssp[SC ? SCP : 1];
  float ssum = 0.f;
  auto ss_issue = [&](int tm_) {
    if constexpr (SC) {
      const u32x4_t s = srd(ea.ss_in, (long)ea.ss_nt * ea.ss_ld * 4);
      const unsigned base = (unsigned)((tm_ * BM + tid) * 4);
#pragma unroll
      for (int p = 0; p < SCP; ++p)  // planes >= ss_nt read past the range: 0
        asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(ssp[p]) : "v"(base), "s"(s), "s"(rfl((unsigned)(p * ea.ss_ld * 4))) : "memory");
    }
  };

  // K-tile t: NM MFMAs (kk 0 set: n-major 0..NM/2-1, kk 1 set: the rest) with the reads / DMA /
  // barriers of the file comment (positions: Tile<BM>).  FIRST: C = 0.  DMA: K-tile t+2 exists
  // (NEXT: it is K-tile t+2-nk of the next tile of a persistent walk).  NXT: K-tile t+1 exists.
  auto ktile = [&](auto first_t, auto dma_t, auto nxt_t, auto next_t, int t) {
    constexpr bool FIRST = decltype(first_t)::value, DMA = decltype(dma_t)::value;
    constexpr bool NXT = decltype(nxt_t)::value;
    const unsigned so = (unsigned)((t + par) & 1) * kStage, sn = (unsigned)kStage - so;  // this / next stage
    unroll<NM>([&](auto i_t) {
      constexpr int i = decltype(i_t)::value;
      constexpr int B1 = TL::B1, D0 = TL::D0, DS = TL::DS, LAG = TL::LAG, B2 = TL::B2;
      if constexpr (i == 0) lgkm0();
      if constexpr (i < NR) rd(bx[1] + so, bw[1] + so, std::integral_constant<int, i>{}, fx1, fw1);
      if constexpr (i == B1) {
        lgkm0();
        barrier_raw();
      }
      if constexpr (DMA && i >= D0 && i < D0 + DS * NP && (i - D0) % DS == 0) {
        fence();
        dma(decltype(next_t)::value, t + 2, (i - D0) / DS);
        fence();
      }
      if constexpr (DMA && i >= D0 + LAG && i < D0 + LAG + DS * NP && (i - D0 - LAG) % DS == 0) {
        constexpr int k = (i - D0 - LAG) / DS;
        fence();
        set_m0(k < NP - 1 ? piece_m0(t + 2, k + 1) : piece_m0(t + 3, 0));
        fence();
      }
      if constexpr (NXT && i == B2) {
        if constexpr (DMA) wait_vm<NP>();
        else wait_vm<0>();
        barrier_raw();
      }
      if constexpr (NXT && i >= B2 && i < B2 + NR)
        rd(bx[0] + sn, bw[0] + sn, std::integral_constant<int, i - B2>{}, fx0, fw0);
      constexpr int kk = i / (NM / 2), n = (i % (NM / 2)) / MB, m = i % MB;
      if constexpr (kk == 0 && FIRST) mfma0(acc[m][n], fw0[n], fx0[m]);
      else if constexpr (kk == 0) mfma(acc[m][n], fw0[n], fx0[m]);
      else mfma(acc[m][n], fw1[n], fx1[m]);
    });
  };

  // ---- one tile per workgroup by default (for long K a persistent walk measured 1-3 % slower: the
  // hardware already starts the next workgroup on a CU while the finished one's stores drain --
  // profiles/r5_gemm1w/); PERSIST for short K, where the load ramp is a third of a tile
  int tile = blockIdx.x;
  int tm, tn;
  coords(tile, tm, tn);
  offsets(tm, tn, xo, wo);
  ss_issue(tm);
  // prologue: K-tiles 0 and 1 (the row-scale loads are older: retired with K-tile 0)
#pragma unroll
  for (int q = 0; q < 2 * NP; ++q) {
    set_m0(piece_m0(q / NP, q % NP));
    asm volatile("s_nop 0");
    dma(false, q / NP, q % NP);
  }
  set_m0(piece_m0(2, 0));
  wait_vm<NP>();
  for (;;) {
    int nxt = 0, tm2 = 0, tn2 = 0;
    bool has_next = false;
    if constexpr (PERSIST) {
      // opaque per tile: keeps hipcc from hoisting the unrolled K-tiles' per-piece / per-fragment
      // addresses out of the tile loop into hundreds of live registers (it spills them otherwise)
      asm volatile("" : "+v"(bx[0]), "+v"(bx[1]), "+v"(bw[0]), "+v"(bw[1]));
#pragma unroll
      for (int i = 0; i < PX; ++i) asm volatile("" : "+v"(xo[i]));
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(wo[i]));
      nxt = tile + (int)gridDim.x;
      has_next = nxt < nwg;
      // the last tile of the walk DMAs its own first K-tiles again (harmless, never read): one
      // straight-line tail instead of two
      coords(has_next ? nxt : tile, tm2, tn2);
      offsets(tm2, tn2, xo2, wo2);
    }
    barrier_raw();
    if constexpr (SC) {
#pragma unroll
      for (int p = 0; p < SCP; ++p) ssum += ssp[p];
    }
    {
      const unsigned s0 = (unsigned)(par & 1) * kStage;
      unroll<NR>([&](auto j_t) { rd(bx[0] + s0, bw[0] + s0, j_t, fx0, fw0); });
    }
    ktile(T{}, T{}, T{}, F{}, 0);
    int t = 1;
    for (; t + 2 < nk; ++t) ktile(F{}, T{}, T{}, F{}, t);
    if constexpr (PERSIST) {  // the next tile's K-tiles 0 and 1 into the stages these two free
      ktile(F{}, T{}, T{}, T{}, t);
      ktile(F{}, T{}, F{}, T{}, t + 1);
    } else {
      ktile(F{}, F{}, T{}, F{}, t);
      ktile(F{}, F{}, F{}, F{}, t + 1);
    }
    // the asm MFMAs are invisible to hipcc's hazard recognizer: wait out MFMA -> accumulator read,
    // and pin every accumulator behind that wait (hipcc otherwise schedules some v_accvgpr_read of
    // the final K-tile's results right after their MFMA is issued, before it has written them)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));

    // ================= epilogue of tile (tm, tn)
    // lane holds row tm*256 + wr*128 + 16m + r; fragment pair (2p, 2p+1) the 8 consecutive
    // columns 32p + 8g .. +7 of the wave's 128 (SwiGLU: gate pairs 0, 1 and up pairs 2, 3 of
    // each 64-row half ... the wave's 64 output columns)
    float scm[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) scm[m] = 1.f;
    if constexpr (SC) {
      scl[tid] = rsqrtf(ssum * ea.inv_h + ea.eps);
      lgkm0();
      barrier_raw();
#pragma unroll
      for (int m = 0; m < MB; ++m) scm[m] = scl[wr * WM + m * 16 + r];
    }
    auto pk8 = [](const float (&y)[8]) {
      return u32x4_t{pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]), pack_bf2(y[4], y[5]), pack_bf2(y[6], y[7])};
    };
    if constexpr (EPI == E_PARTIAL) {  // fp32 partial sums of split kz: out is float [splits, M, ldo]
      float* part = reinterpret_cast<float*>(out) + (long)kz * M * ldo;
      const auto ps = __builtin_amdgcn_make_buffer_rsrc(part, 0, (int)min((long)M * ldo * 4, 0x7FFFFFF0L), 0x00020000);
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const unsigned rb = (unsigned)(((long)tm * BM + wr * WM + m * 16 + r) * ldo + tn * kBN + wc * 128) * 4;
#pragma unroll
        for (int n = 0; n < 8; ++n)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[m][n]), ps,
                                                 rb + (unsigned)((32 * (n >> 1) + 8 * g + 4 * (n & 1)) * 4), 0, 0);
      }
    } else if constexpr (EPI == E_SWIGLU) {
      const auto os = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)min((long)M * ldo * 2, 0x7FFFFFF0L), 0x00020000);
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const unsigned rb = (unsigned)(((long)tm * BM + wr * WM + m * 16 + r) * ldo + tn * 128 + wc * 64 + 8 * g) * 2;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float y[8];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v)
              y[4 * h + v] = rbf(lk_silu(rbf(acc[m][2 * p + h][v] * scm[m]))) * rbf(acc[m][4 + 2 * p + h][v] * scm[m]);
          __builtin_amdgcn_raw_buffer_store_b128(pk8(y), os, rb + 64 * p, 0, 0);
        }
      }
    } else if constexpr (EPI == E_RESID) {
      // r = bf16(r + bf16(acc)) in place, then the partial sum of squares of the new r over the
      // tile's 256 columns (lanes g, then the two wc waves through LDS) into ss_out[tn][row]
      const auto rrs = __builtin_amdgcn_make_buffer_rsrc(ea.resid, 0, (int)min((long)M * ea.ldr * 2, 0x7FFFFFF0L), 0x00020000);
      float ssm[MB];
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const long row = (long)tm * BM + wr * WM + m * 16 + r;
        const unsigned rb = (unsigned)((row * ea.ldr + (long)tn * kBN + wc * 128 + 8 * g) * 2);
        u32x4_t rv[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) rv[p] = __builtin_amdgcn_raw_buffer_load_b128(rrs, rb + 64 * p, 0, 0);
        float ss = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
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
          __builtin_amdgcn_raw_buffer_store_b128(pk8(y), rrs, rb + 64 * p, 0, 0);
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        ssm[m] = ss;
      }
      float* red = reinterpret_cast<float*>(smem + kLdsStages + 1024);  // [2 wc][BM tile rows]
      if (g == 0) {
#pragma unroll
        for (int m = 0; m < MB; ++m) red[wc * BM + wr * WM + m * 16 + r] = ssm[m];
      }
      lgkm0();
      barrier_raw();
      const int row = tm * BM + tid;
      if (tid < BM && row < M) ea.ss_out[(long)tn * ea.ss_out_ld + row] = red[tid] + red[BM + tid];
    } else if constexpr (EPI == E_QKV) {
      // RoPE (interleaved pairs) on the q / k heads + the paged-KV scatter, on the bf16-rounded
      // (row-scaled) projection: the values "GEMM -> rope_kv_" would leave.  Everything that
      // depends only on the lane's columns is hoisted out of the row loop (no integer division
      // per row), the rows' positions / slots are loaded in one round before any store (a u32
      // store may alias the int metadata, so per-row loads would each wait behind the previous
      // row's stores), and the next row's cos / sin are in flight while this row is rotated.
      const int qcols = ea.hq * ea.hd, kcols = ea.hkv * ea.hd, half = ea.hd >> 1;
      const int cb = tn * kBN + wc * 128;
      int i0[4], coff[4];
      bool rot[4], kv[4], isv[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int c = cb + 32 * p + 8 * g;
        rot[p] = c < qcols + kcols;
        kv[p] = c >= qcols;
        isv[p] = c >= qcols + kcols;
        i0[p] = (c % ea.hd) >> 1;  // first rotation pair
        const int cc = c - qcols - (isv[p] ? kcols : 0);
        const int h = cc / ea.hd;
        coff[p] = h * ea.bs * ea.hd + (cc - h * ea.hd);  // head h, dim d within a cache block
      }
      const long blk_stride = (long)ea.hkv * ea.bs * ea.hd;
      int posv[MB], slotv[MB];
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const int row = tm * BM + wr * WM + m * 16 + r;
        const int rc = min(row, M - 1);  // unconditional loads: no branch per row around them
        posv[m] = ea.pos[rc];
        slotv[m] = ea.slots ? ea.slots[rc] : -1;
      }
      floatx4 c4[4], s4[4];
      auto load_cs = [&](int pos, floatx4 (&cv)[4], floatx4 (&sv)[4]) {
        const float* cs = ea.cos_sin + (long)pos * ea.hd;
#pragma unroll
        for (int p = 0; p < 4; ++p) {  // (loaded for v columns too: in range, and branch-free)
          cv[p] = *reinterpret_cast<const floatx4*>(cs + i0[p]);
          sv[p] = *reinterpret_cast<const floatx4*>(cs + half + i0[p]);
        }
      };
      load_cs(posv[0], c4, s4);
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        floatx4 c4n[4], s4n[4];
        if (m + 1 < MB) load_cs(posv[m + 1], c4n, s4n);
        const int row = tm * BM + wr * WM + m * 16 + r;
        if (row < M) {
          const float sc = scm[m];
          const int slot = slotv[m];
          const long kvb = slot >= 0 ? (long)(slot / ea.bs) * blk_stride + (long)(slot % ea.bs) * ea.hd : 0;
          bf16_t* orow = out + (long)row * ldo;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            float y[8];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int v = 0; v < 4; ++v) y[4 * h + v] = rbf(acc[m][2 * p + h][v] * sc);
            if (rot[p]) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float a = y[2 * q], b = y[2 * q + 1];
                y[2 * q] = a * c4[p][q] - b * s4[p][q];
                y[2 * q + 1] = b * c4[p][q] + a * s4[p][q];
              }
            }
            const u32x4_t pk = pk8(y);
            *reinterpret_cast<u32x4_t*>(orow + cb + 32 * p + 8 * g) = pk;
            if (kv[p] && slot >= 0 && ea.kc != nullptr)
              *reinterpret_cast<u32x4_t*>((isv[p] ? ea.vc : ea.kc) + kvb + coff[p]) = pk;
          }
        }
        // one row of cos / sin in flight, not all MB (hoisted, they would take MB x 32 VGPRs)
        asm volatile("" ::: "memory");
        if (m + 1 < MB) {
#pragma unroll
          for (int p = 0; p < 4; ++p) c4[p] = c4n[p], s4[p] = s4n[p];
        }
      }
    } else {  // NONE / BIAS / BIAS_GELU / BIAS_RELU
      const auto os = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)min((long)M * ldo * 2, 0x7FFFFFF0L), 0x00020000);
      float bv[8][4];
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int v = 0; v < 4; ++v) bv[n][v] = 0.f;
      if constexpr (EPI != E_NONE) {
        const auto bs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(bias), 0, (tn0 + TN) * kBN * 2, 0x00020000);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const u32x4_t b = __builtin_amdgcn_raw_buffer_load_b128(bs, (unsigned)((tn * kBN + wc * 128 + 32 * p + 8 * g) * 2), 0, 0);
          const unsigned bw4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            bv[2 * p + (q >> 1)][2 * (q & 1)] = bf2f((bf16_t)(bw4[q] & 0xFFFF));
            bv[2 * p + (q >> 1)][2 * (q & 1) + 1] = bf2f((bf16_t)(bw4[q] >> 16));
          }
        }
      }
      auto act = [&](float e, float b) {  // (GELU: applied pairwise below)
        if constexpr (EPI != E_NONE) e = rbf(e + b);
        if constexpr (EPI == E_BIAS_RELU) e = fmaxf(e, 0.f);
        return e;
      };
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const unsigned rb = (unsigned)(((long)tm * BM + wr * WM + m * 16 + r) * ldo + tn * kBN + wc * 128 + 8 * g) * 2;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float y[8];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) y[4 * h + v] = act(acc[m][2 * p + h][v] * scm[m], bv[2 * p + h][v]);
          if constexpr (EPI == E_BIAS_GELU) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const lk_f2 gv = lk_gelu_erf2(lk_f2{y[2 * j], y[2 * j + 1]});
              y[2 * j] = gv.x;
              y[2 * j + 1] = gv.y;
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(pk8(y), os, rb + 64 * p, 0, 0);
        }
      }
    }
    if constexpr (!PERSIST) {
      break;
    } else {
      if (!has_next) {
        wait_vm<0>();  // the walk's last (unread) DMAs land before the workgroup's LDS is released
        break;
      }
      tile = nxt;
      tm = tm2;
      tn = tn2;
#pragma unroll
      for (int i = 0; i < PX; ++i) xo[i] = xo2[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) wo[i] = wo2[i];
      par ^= nk & 1;
      // the next tile's K-tile 0 has landed: younger than it are K-tile 1's NP pieces and the
      // epilogue's bias loads and stores (the counter retires in issue order)
      wait_vm<NP + epi_vm_ops<EPI, MB>()>();
    }
  }
}

// split-K reduction: out[r, c..c+3] = epi(sum_z part[z, r, c..c+3] (+ bias)), rounded like the
// fused epilogues; one thread per 4 columns
template <int EPI>
__global__ __launch_bounds__(256) void reduce1w_kernel(const float* __restrict__ part, int S, int M, int N,
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
    if constexpr (EPI != E_NONE) e = rbf(e + bf2f(bias[col + v]));
    if constexpr (EPI == E_BIAS_GELU) e = lk_gelu_erf(e);
    if constexpr (EPI == E_BIAS_RELU) e = fmaxf(e, 0.f);
    y[v] = e;
  }
  *reinterpret_cast<uint2*>(out + (long)row * ldo + col) = make_uint2(pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]));
}

// split-K reduction for RESID (same planes as the unsplit epilogue: partial sums per 256 columns)
__global__ __launch_bounds__(64) void reduce1w_resid_kernel(const float* __restrict__ part, int S, int M, int N,
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

int group1w() {  // row tiles per XCD group of the tile order (LK_GEMM_GROUP_M, default 4)
  static const int g = [] {
    const char* e = getenv("LK_GEMM_GROUP_M");
    const int v = e ? atoi(e) : 4;
    return v >= 1 ? v : 4;
  }();
  return g;
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }();
  return n;
}

// persistent walk for short K (LK_GEMM1W_PERSIST_KT: the most K-tiles of 64 it is used for; 0: off)
int persist_kt() {
  static const int v = [] {
    const char* e = getenv("LK_GEMM1W_PERSIST_KT");
    return e ? atoi(e) : 16;
  }();
  return v;
}

template <int EPI, int SCP, int BM, bool PERSIST = false>
void launch1w_p(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
                long ldo, int TN, int tn0, int ks, int group_m, hipStream_t st, const LkEpi& ea) {
  constexpr int lds = Tile<BM>::kLds;
  LK_SET_MAX_LDS((gemm1w_kernel<EPI, SCP, BM, PERSIST>), lds);
  const int TM = (M + BM - 1) / BM;
  const int grid = PERSIST ? min(TM * TN, cu_count()) : TM * TN;
  gemm1w_kernel<EPI, SCP, BM, PERSIST><<<dim3(grid, ks), 256, lds, st>>>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN,
                                                                       tn0, group_m > 0 ? group_m : group1w(), ea);
}
template <int EPI, int SCP, int BM>
void launch1w(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
              long ldo, int TN, int tn0, int ks, int group_m, hipStream_t st, const LkEpi& ea) {
  if constexpr (persistable(EPI) && SCP == 0 && BM == 256) {
    const int tiles = ((M + BM - 1) / BM) * TN;
    if (ks == 1 && K / kBK <= persist_kt() && tiles > 2 * cu_count()) {
      launch1w_p<EPI, SCP, BM, true>(x, ldx, w, bias, M, K, I, out, ldo, TN, tn0, ks, group_m, st, ea);
      return;
    }
  }
  launch1w_p<EPI, SCP, BM, false>(x, ldx, w, bias, M, K, I, out, ldo, TN, tn0, ks, group_m, st, ea);
}
template <int EPI, int SCP>
void launch1w_bm(int bm, const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I,
                 bf16_t* out, long ldo, int TN, int tn0, int ks, int group_m, hipStream_t st, const LkEpi& ea) {
  if (bm == 192) launch1w<EPI, SCP, 192>(x, ldx, w, bias, M, K, I, out, ldo, TN, tn0, ks, group_m, st, ea);
  else if (bm == 128) launch1w<EPI, SCP, 128>(x, ldx, w, bias, M, K, I, out, ldo, TN, tn0, ks, group_m, st, ea);
  else launch1w<EPI, SCP, 256>(x, ldx, w, bias, M, K, I, out, ldo, TN, tn0, ks, group_m, st, ea);
}
template <int EPI, int SCP>
void launch1w_tiles(int bm, const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I,
                    bf16_t* out, long ldo, int TN, int ks, int group_m, hipStream_t st, const LkEpi& ea) {
  if (bm == LK_GEMM1W_SPLIT128 || bm == LK_GEMM1W_SPLIT192) {
    // column split: the column tiles that fill whole waves of the CUs with 256-row tiles, then
    // the rest -- less than one wave of 256-row tiles -- on smaller row tiles that fill one.
    // The QKV projection at M 4096 (16 x 24 tiles = 1.5 waves of 256 CUs) runs 16 x 16 256-row
    // tiles, then 32 x 8 128-row tiles: 1 + ~0.6 tile times instead of 2.
    const int ca = lk_gemm1w_split_cols(M, TN, cu_count());
    if (ca > 0 && ca < TN) {
      launch1w_bm<EPI, SCP>(256, x, ldx, w, bias, M, K, I, out, ldo, ca, 0, ks, group_m, st, ea);
      launch1w_bm<EPI, SCP>(bm == LK_GEMM1W_SPLIT128 ? 128 : 192, x, ldx, w, bias, M, K, I, out, ldo, TN - ca, ca, ks,
                            group_m, st, ea);
      return;
    }
    bm = 256;
  }
  launch1w_bm<EPI, SCP>(bm, x, ldx, w, bias, M, K, I, out, ldo, TN, 0, ks, group_m, st, ea);
}
template <int EPI>
void launch1w_sc(int bm, const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I,
                 bf16_t* out, long ldo, int TN, int ks, int group_m, hipStream_t st, const LkEpi& ea) {
  if constexpr (scalable(EPI)) {
    if (ea.ss_in != nullptr) {
      if (ea.ss_nt <= 16) launch1w_tiles<EPI, 16>(bm, x, ldx, w, bias, M, K, I, out, ldo, TN, ks, group_m, st, ea);
      else launch1w_tiles<EPI, 32>(bm, x, ldx, w, bias, M, K, I, out, ldo, TN, ks, group_m, st, ea);
      return;
    }
  }
  launch1w_tiles<EPI, 0>(bm, x, ldx, w, bias, M, K, I, out, ldo, TN, ks, group_m, st, ea);
}

}  // namespace

int lk_gemm1w_split_cols(int M, int TN, int cus) {
  const int tm = (M + 255) / 256;
  const int waves = tm * TN / cus;  // whole waves of 256-row tiles
  return min(TN, waves * cus / tm);
}

int lk_gemm1w_supported(int M, int N, int K, int epi, int ks, int bm) {
  if (bm != 256 && bm != 192 && bm != 128 && bm != LK_GEMM1W_SPLIT128 && bm != LK_GEMM1W_SPLIT192) return 0;
  if (M < 1 || K % kBK || ks < 1 || ks > 8 || K / kBK < 3 * ks) return 0;  // >= 3 K-tiles per split
  if (ks > 1 && (epi == E_SWIGLU || epi == E_QKV || N % 256)) return 0;
  if (epi == E_SWIGLU) return N % 2 == 0 && (N / 2) % 128 == 0;
  if (epi == E_RESID || epi == E_QKV) return N % kBN == 0;
  return epi >= E_NONE && epi <= E_BIAS_RELU && N % kBN == 0;
}

// out = epi(X W^T (+ bias)): the contract of lk_gemm with a bm x 256 tile, bm = 256 / 192 / 128
// (ea: the fused chain arguments, see kernels.h).  group_m <= 0: LK_GEMM_GROUP_M / 4.
int lk_gemm1w(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi,
              bf16_t* out, long ldo, hipStream_t st, int ks, float* ws, const LkEpi* ea_, int group_m, int bm) {
  LkEpi ea = ea_ ? *ea_ : LkEpi{};
  if (ea.ss_in && (ea.ss_nt < 1 || ea.ss_nt > 32 || ea.ss_ld < M || ea.inv_h <= 0.f || ks > 1)) return -1;
  if (epi == E_RESID && (!ea.resid || !ea.ss_out || ea.ldr % 8 || ea.ss_out_ld < M)) return -1;
  if (epi == E_QKV && (!ea.pos || !ea.cos_sin || ea.hd % 16 || ea.hd <= 0 || N != (ea.hq + 2 * ea.hkv) * ea.hd ||
                       ((ea.kc || ea.vc) && (!ea.slots || ea.bs < 1))))
    return -1;
  if (!lk_gemm1w_supported(M, N, K, epi, ks, bm) || ldx % 8 || ldo % 8 || reinterpret_cast<uintptr_t>(out) % 16 ||
      (bias != nullptr && reinterpret_cast<uintptr_t>(bias) % 16))
    return -1;
  if (epi >= E_BIAS && epi <= E_BIAS_RELU && bias == nullptr) return -1;
  if ((long)N * K * 2 >= 0x7FFFFFF0L) return -1;
  // 32-bit buffer offsets: X, the output (fp32 partials for split-K) and the residual in row chunks
  const int bmx = bm < 128 ? 256 : bm;  // (a column split's largest row tile)
  const int TMall = (M + bmx - 1) / bmx;
  const long rows_pad = (long)TMall * bmx;
  const long xb = rows_pad * ldx * 2, ob = rows_pad * ldo * (ks > 1 ? 4 * ks : 2), rb = epi == E_RESID ? rows_pad * ea.ldr * 2 : 0;
  if (xb >= 0x7FFFFFF0L || ob >= 0x7FFFFFF0L || rb >= 0x7FFFFFF0L) {
    if (ea_ || ks > 1) return -1;  // (the fused chain indexes whole-M side buffers)
    const long per = max(ldx, ldo) * 2;
    const long max_rows = (0x7FFFFFF0L / per) / bmx * bmx - bmx;
    if (max_rows < bmx) return -1;
    for (long m0 = 0; m0 < M; m0 += max_rows) {
      const int mc = (int)min((long)M - m0, max_rows);
      const int rc = lk_gemm1w(x + m0 * ldx, ldx, w, bias, mc, N, K, epi, out + m0 * ldo, ldo, st, 1, nullptr, nullptr,
                               group_m, bm);
      if (rc) return rc;
    }
    return 0;
  }
  if (ks > 1) {  // fp32 partials of ks K-ranges into ws [ks, M, N], then the reduce applies the epilogue
    if (ws == nullptr) return -1;
    launch1w_sc<E_PARTIAL>(bm, x, ldx, w, nullptr, M, K, 0, reinterpret_cast<bf16_t*>(ws), N, N / kBN, ks, group_m, st,
                           ea);
    if (epi == E_RESID) {
      reduce1w_resid_kernel<<<dim3(N / 256, M), 64, 0, st>>>(ws, ks, M, N, ea);
    } else {
      const long n = (long)M * (N / 4);
      const int blocks = (int)((n + 255) / 256);
      switch (epi) {
        case E_NONE: reduce1w_kernel<E_NONE><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
        case E_BIAS: reduce1w_kernel<E_BIAS><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
        case E_BIAS_GELU: reduce1w_kernel<E_BIAS_GELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
        case E_BIAS_RELU: reduce1w_kernel<E_BIAS_RELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
        default: return -1;
      }
    }
    LK_CHECK_LAUNCH();
    return 0;
  }
  switch (epi) {
    case E_NONE: launch1w_sc<E_NONE>(bm, x, ldx, w, bias, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    case E_SWIGLU: launch1w_sc<E_SWIGLU>(bm, x, ldx, w, bias, M, K, N / 2, out, ldo, N / 256, 1, group_m, st, ea); break;
    case E_BIAS: launch1w_tiles<E_BIAS, 0>(bm, x, ldx, w, bias, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    case E_BIAS_GELU: launch1w_tiles<E_BIAS_GELU, 0>(bm, x, ldx, w, bias, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    case E_BIAS_RELU: launch1w_tiles<E_BIAS_RELU, 0>(bm, x, ldx, w, bias, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    case E_RESID: launch1w_tiles<E_RESID, 0>(bm, x, ldx, w, nullptr, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    case E_QKV: launch1w_sc<E_QKV>(bm, x, ldx, w, nullptr, M, K, 0, out, ldo, N / kBN, 1, group_m, st, ea); break;
    default: return -1;
  }
  LK_CHECK_LAUNCH();
  return 0;
}

// probes (benchmarks/gemm1w_probe.py): plain / SwiGLU / bias epilogues through ctypes
extern "C" int lk_gemm1w_c(const void* x, long ldx, const void* w, const void* bias, int M, int N, int K, int epi,
                           void* out, long ldo, void* stream, int group_m, int bm) {
  return lk_gemm1w((const bf16_t*)x, ldx, (const bf16_t*)w, (const bf16_t*)bias, M, N, K, epi, (bf16_t*)out, ldo,
                   (hipStream_t)stream, 1, nullptr, nullptr, group_m, bm);
}
