// K2, prefill / encoder regime, one-wave-per-SIMD variant: Y[M, N] = epilogue(X[M, K] . W[N, K]^T).
// NOT BUILT: the round-3 one-wave-per-SIMD prefill GEMM, kept as a measured probe (it lost
// 6-12 % to csrc/gemm.hip on the served shapes, profiles/r3_gemm_4wave/README.md).  Moved out of
// the _C extension in round 4; build it by hand next to csrc/common.h for loop ablations.
//
// Why a second prefill kernel: the 8-wave ping-pong of gemm.hip keeps two waves per SIMD and
// pays for it in barrier waits (PMC, profiles/r2_gemm.md: SQ_WAIT_ANY 176.7 M vs the library's
// 12.2 M at the same MFMA work and the same L2 / HBM traffic).  This kernel is the other design
// point of CDNA4's playbook:
//   * 256 threads = 4 waves, ONE per SIMD, as 2 (M) x 2 (N); the C tile is 256 x 256 and each
//     wave owns 128 x 128 outputs = 8 x 8 v_mfma_f32_16x16x32_bf16 accumulators (256 floats per
//     lane) that live in AGPRs for the whole K loop: the MFMAs are issued from inline asm with
//     "+a" accumulator operands, so hipcc never moves an accumulator through VGPRs, and an asm
//     statement is a scheduling boundary, so the LDS reads / LDS-DMA issues placed between them
//     in the source stay interleaved with the matrix work in that order;
//   * LDS per wave-fragment byte: 256 B per MFMA (128 x 128 per wave) instead of 384 B (the
//     8-wave kernel's 128 x 64), a third fewer LDS reads per FLOP -- less energy per MFMA on a
//     chip that holds its clock down under MFMA load;
//   * K is staged in 32-deep slices (64-B LDS rows, 32 KB per slice: 256 X rows + 256 W rows)
//     through a 4-slot LDS-DMA ring (128 KB).  ONE barrier per slice: before it every wave has
//     its fragments of slice t in registers (lgkmcnt(0)) and its DMA of slice t+1 landed
//     (counted vmcnt, never 0 in the loop); after it slice t+1 is readable and slot t % 4 is
//     free, so the DMA of slice t+4 goes straight into it: three slices (~3 x 1024 MFMA
//     cycles) of cover for every load.  Fragments are double-buffered in VGPRs: the 64 MFMAs of
//     slice t run while the 16 ds_read_b128 of slice t+1 and the 8 DMA issues of t+4 go out;
//   * 64-B rows: the 16-B chunk index is XORed with ((row >> 3) & 1) << 1 on the DMA SOURCE
//     address (lane-linear LDS image) and on the read, which keeps each ds_read_b128 lane group
//     on 16 distinct bank slots;
//   * operands are swapped in the MFMA (A <- W rows, B <- X rows) and the W rows of every
//     32-row block are permuted (pair_col) so a lane ends with one output row and 8 consecutive
//     columns per fragment pair: 16-B epilogue stores, SwiGLU gate / up of the same columns in
//     one lane, bias / GELU / ReLU fused as in gemm.hip;
//   * tiles in the same XCD-aware grouped order as gemm.hip; split-K by fp32 partials.
#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kBM = 256, kBN = 256;
constexpr int kBKS = 32;                  // K per ring slice
constexpr int kRow = kBKS * 2;            // 64-B LDS rows
constexpr int kRegion = 256 * kRow;       // 16 KB: 256 rows of one operand
constexpr int kSlice = 2 * kRegion;       // 32 KB: X rows then W rows
constexpr int kSlots = 4;
constexpr int kLds = kSlots * kSlice;     // 128 KB
constexpr int kDmaPerWave = 8;            // 1-KB LDS-DMA issues per wave per slice (4 X + 4 W)

enum { EPI_NONE = 0, EPI_SWIGLU = 1, EPI_BIAS = 2, EPI_BIAS_GELU = 3, EPI_BIAS_RELU = 4, EPI_PARTIAL = 5 };

LK_DEVICE int fsw(int row) { return ((row >> 3) & 1) << 1; }  // 64-B row chunk swizzle
template <int N>
LK_DEVICE void wait_vm() {  // s_waitcnt vmcnt(N); lgkmcnt / expcnt untouched
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
LK_DEVICE void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0x3F | (0x7 << 4) | (0x3 << 14) | (0x0 << 8)); }
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }
// raw s_barrier: no vmcnt(0) drain of the in-flight LDS-DMA ring (unlike __syncthreads); the
// empty "memory" asm keeps the compiler from moving LDS loads across it
LK_DEVICE void barrier_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): a compile-time loop
template <class Fn, int... I>
LK_DEVICE void unroll_impl(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
LK_DEVICE void unroll(Fn&& f) {
  unroll_impl(f, std::make_integer_sequence<int, N>{});
}

// acc += A(16x32) . B(32x16), acc pinned to AGPRs; volatile keeps the issue order
LK_DEVICE void mfma(floatx4& acc, const short8& a, const short8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// MODE 0: LDS-DMA ring (4 slots of 32-deep slices, DMA issued 4 slices ahead);
// MODE 1: register staging (buffer_load_dwordx4 to VGPRs 4 slices ahead, two staging sets,
//         ds_write_b128 into a 2-slot ring two slices ahead): no LDS-DMA issue on the MFMA waves
template <int EPI, int MODE>
__device__ __forceinline__ void gemm4w_body(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                                            const bf16_t* __restrict__ bias, int M, int K, int I,
                                            bf16_t* __restrict__ out, long ldo, int TM, int TN, int group_m,
                                            int tile) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // ---- tile of this block: XCD-contiguous logical ids, grouped group_m row tiles at a time
  const int nwg = TM * TN;
  const int L = xcd_remap(tile, nwg);
  const int per_group = group_m * TN;
  const int first = (L / per_group) * group_m;
  const int gm = min(TM - first, group_m);
  const int tm = first + (L % per_group) % gm;
  const int tn = (L % per_group) / gm;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int r = lane & 15, g = lane >> 4;

  // LDS W-row j -> output column: fragment pair (2p, 2p+1) of a 32-row block gives lane group g
  // the 8 consecutive columns 8g .. 8g+7 (see the file comment)
  auto pair_col = [](int rem) { return 8 * ((rem & 15) >> 2) + 4 * (rem >> 4) + (rem & 3); };
  auto wrow = [&](int j) -> long {
    if constexpr (EPI == EPI_SWIGLU) {  // per wave: 64 gate rows then the 64 up rows of its 64 columns
      const int wv = j >> 7, h = (j >> 6) & 1, s = j & 63;
      return (long)h * I + (long)tn * 128 + wv * 64 + (s >> 5) * 32 + pair_col(s & 31);
    } else {
      return (long)tn * kBN + (j >> 5) * 32 + pair_col(j & 31);
    }
  };

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, (short)0, (int)min((long)M * ldx * 2, 0x7FFFFFF0L), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)W, (short)0, (int)min((long)(EPI == EPI_SWIGLU ? 2 * I : TN * kBN) * K * 2, 0x7FFFFFF0L), 0x00020000);

  // split-K (gridDim.y): this workgroup's 64-deep K-tiles [kt0, kt0 + nk) = slices [2 kt0, 2 kt0 + ns)
  const int nkt = K / 64, kz = blockIdx.y, ks = gridDim.y;
  const int kt0 = kz * nkt / ks, nk = (kz + 1) * nkt / ks - kt0;
  const int ns = 2 * nk, s0 = 2 * kt0;

  // ---- LDS-DMA: instruction i of wave w moves LDS rows 16 (4w + i) .. +15 of one operand;
  // lane -> row lane >> 2, 16-B chunk lane & 3 (source chunk swizzled)
  const int lrow = lane >> 2, lc = lane & 3;
  unsigned xoff[4], woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 16 * (4 * w + i) + lrow;
    const unsigned ch = (unsigned)((lc ^ fsw(row)) << 4);
    xoff[i] = (unsigned)(((long)tm * kBM + row) * ldx * 2) + ch;
    woff[i] = (unsigned)(wrow(row) * K * 2) + ch;
  }
  // ring slots of the LDS-DMA mode (a 5-slot / 160 KB ring measured 2-3 % slower)
  constexpr int RS = kSlots;
  auto issue = [&](int s) {  // slice s -> ring slot s % RS
    unsigned char* base = smem + (s % RS) * kSlice + 16 * 4 * w * kRow;
    const unsigned so = (unsigned)(s0 + s) * (kBKS * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(base + i * 16 * kRow), 16, xoff[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(base + kRegion + i * 16 * kRow), 16, woff[i], so, 0,
                                               0);
  };

  floatx4 acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: lane reads row (16-row fragment base + r), 16-B chunk g (k 8g .. 8g+7)
  const int fofs = r * kRow + ((g ^ fsw(r)) << 4);
  short8 fx0[8], fw0[8], fx1[8], fw1[8];

  // one slice: the 64 MFMAs of fragments (fx, fw) with the next slice's 16 fragment reads (RD)
  // and the 8 DMA issues of slice s + 4 (DMA) spread over them, 8 MFMAs per row m.  The flags
  // are template parameters: a runtime condition would put a branch around every issue.
  auto step = [&](auto rd_t, auto dma_t, short8(&fx)[8], short8(&fw)[8], short8(&nx)[8], short8(&nw)[8], int s) {
    constexpr bool RD = decltype(rd_t)::value, DMA = decltype(dma_t)::value;
    const unsigned char* nb = smem + ((s + 1) % RS) * kSlice + fofs;
    unsigned char* db = smem + ((s + RS) % RS) * kSlice + 16 * 4 * w * kRow;
    const unsigned so = (unsigned)(s0 + s + RS) * (kBKS * 2);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (RD && MODE != 2 && MODE != 4) {
        nx[m] = *reinterpret_cast<const short8*>(nb + (wr * 128 + m * 16) * kRow);
        nw[m] = *reinterpret_cast<const short8*>(nb + kRegion + (wc * 128 + m * 16) * kRow);
      }
      if constexpr (DMA && MODE != 3 && MODE != 4) {
        if (m < 4)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(db + m * 16 * kRow), 16, xoff[m & 3], so, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(db + kRegion + (m - 4) * 16 * kRow), 16,
                                                   woff[m & 3], so, 0, 0);
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) mfma(acc[m][n], fw[n], fx[m]);
    }
  };
  // before the barrier of slice s: own fragments of s in registers, own DMA of s + 1 landed
  // (VM = DMA issues still allowed in flight: those of the slices after s + 1)
  auto sync = [&](auto vm_t) {
    wait_vm<decltype(vm_t)::value>();
    wait_lgkm0();
    barrier_raw();
  };
  using T = std::true_type;
  using F = std::false_type;
  using V0 = std::integral_constant<int, 0>;
  using V1 = std::integral_constant<int, kDmaPerWave>;
  using V2 = std::integral_constant<int, 2 * kDmaPerWave>;

  if constexpr (MODE == 5) {
  // ---- 64-deep K-tiles, 128-B LDS rows (every DMA issue moves 8 rows x one full 128-B line:
  // the 32-deep slices' half-line pieces measured 31 % of the loop in the ablations), a 2-slot
  // ring (2 x 64 KB).  Fragments go per 32-deep half (kk); K-tile t:
  //   half (t,0): MFMAs of frags (t,0) | read frags (t,1)
  //   vmcnt(0) (own DMA of t+1 landed), lgkmcnt(0), barrier: t+1 readable, slot t%2 free
  //   half (t,1): MFMAs of frags (t,1) | read frags (t+1,0), 16 DMA issues of tile t+2 -> slot t%2
  constexpr int R2 = 128, REG2 = 256 * R2, SL2 = 2 * REG2;
  const int lr8 = lane >> 3, lc8 = lane & 7;
  auto swz2 = [](int row) { return (row >> 1) & 7; };
  unsigned xo2[8], wo2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // instruction i of wave w: rows 64w + 8i .. +7 of each operand
    const int row = 64 * w + 8 * i + lr8;
    const unsigned ch = (unsigned)((lc8 ^ swz2(row)) << 4);
    xo2[i] = (unsigned)(((long)tm * kBM + row) * ldx * 2) + ch;
    wo2[i] = (unsigned)(wrow(row) * K * 2) + ch;
  }
  const int rs2 = swz2(r);
  auto frag = [&](const unsigned char* slot, int row0, int kk) {
    return *reinterpret_cast<const short8*>(slot + (row0 + r) * R2 + (((4 * kk + g) ^ rs2) << 4));
  };
  auto rd_half = [&](int t, int kk, short8(&fx)[8], short8(&fw)[8], int m) {
    const unsigned char* sl = smem + (t & 1) * SL2;
    fx[m] = frag(sl, wr * 128 + m * 16, kk);
    fw[m] = frag(sl + REG2, wc * 128 + m * 16, kk);
  };
  auto dma2 = [&](int t, int i) {  // i < 8: X rows, else W rows
    unsigned char* d = smem + (t & 1) * SL2 + (i < 8 ? 0 : REG2) + (64 * w + 8 * (i & 7)) * R2;
    const unsigned so = (unsigned)(kt0 + t) * 128;
    if (i < 8) __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)d, 16, xo2[i & 7], so, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)d, 16, wo2[i & 7], so, 0, 0);
  };
  // the 64 MFMAs of one half (fx, fw), with the fragment reads of the next half (RD: tile nt,
  // half nkk) and 16 DMA issues of tile t+2 (DMA) interleaved, 8 MFMAs per row m
  auto half = [&](auto rd_t, auto dma_t, short8(&fx)[8], short8(&fw)[8], short8(&nx)[8], short8(&nw)[8], int nt,
                  int nkk, int t) {
    constexpr bool RD = decltype(rd_t)::value, DMA = decltype(dma_t)::value;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (RD) rd_half(nt, nkk, nx, nw, m);
      if constexpr (DMA) {
        dma2(t + 2, 2 * m);
        dma2(t + 2, 2 * m + 1);
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) mfma(acc[m][n], fw[n], fx[m]);
    }
  };
  auto ktile = [&](auto rd_t, auto dma_t, int t) {
    half(T{}, F{}, fx0, fw0, fx1, fw1, t, 1, t);
    wait_vm<0>();
    wait_lgkm0();
    barrier_raw();
    half(rd_t, dma_t, fx1, fw1, fx0, fw0, t + 1, 0, t);
  };
  // prologue: tiles 0 and 1 in flight, tile 0 landed, frags (0,0) read
#pragma unroll
  for (int i = 0; i < 16; ++i) dma2(0, (i & 1) ? 8 + (i >> 1) : (i >> 1));
#pragma unroll
  for (int i = 0; i < 16; ++i) dma2(1, (i & 1) ? 8 + (i >> 1) : (i >> 1));
  wait_vm<16>();
  barrier_raw();
#pragma unroll
  for (int m = 0; m < 8; ++m) rd_half(0, 0, fx0, fw0, m);
  int t = 0;
  for (; t + 2 < nk; ++t) ktile(T{}, T{}, t);
  ktile(T{}, F{}, t);        // nk - 2
  ktile(F{}, F{}, t + 1);    // nk - 1
  } else if constexpr (MODE != 1) {  // MODE 0 (+ the timing-only ablations 2-4 of its loop)
  // prologue: slices 0 .. RS-1 in flight, slice 0 landed and read (ns >= RS + (RS & 1))
#pragma unroll
  for (int s = 0; s < RS; ++s) issue(s);
  wait_vm<(RS - 1) * kDmaPerWave>();
  barrier_raw();
  {
    const unsigned char* b0 = smem + fofs;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      fx0[m] = *reinterpret_cast<const short8*>(b0 + (wr * 128 + m * 16) * kRow);
      fw0[m] = *reinterpret_cast<const short8*>(b0 + kRegion + (wc * 128 + m * 16) * kRow);
    }
  }
  // steady state: every slice reads the next one's fragments and issues the DMA of s + RS
  using VS = std::integral_constant<int, (RS - 2) * kDmaPerWave>;
  int s = 0;
  for (; s + RS + 2 <= ns; s += 2) {
    sync(VS{});
    step(T{}, T{}, fx0, fw0, fx1, fw1, s);
    sync(VS{});
    step(T{}, T{}, fx1, fw1, fx0, fw0, s + 1);
  }
  // drain: the last TL = RS + (RS & 1) slices; tail slice i issues a DMA while i < TL - RS and
  // may leave min(TL - 2 - i, RS - 2) later slices in flight at its barrier
  constexpr int TL = RS + (RS & 1);
  auto tail = [&](auto i_t) {
    constexpr int i = decltype(i_t)::value;
    constexpr int left = (TL - 2 - i) < (RS - 2) ? (TL - 2 - i) : (RS - 2);
    sync(std::integral_constant<int, (left > 0 ? left : 0) * kDmaPerWave>{});
    using RDT = std::integral_constant<bool, (i < TL - 1)>;
    using DMT = std::integral_constant<bool, (i < TL - RS)>;
    if constexpr (i % 2 == 0) step(RDT{}, DMT{}, fx0, fw0, fx1, fw1, s + i);
    else step(RDT{}, DMT{}, fx1, fw1, fx0, fw0, s + i);
  };
  unroll<TL>(tail);
  } else {
  // ---- register staging.  Slice t is loaded (8 x 16 B per lane: 4 X, 4 W row groups) into
  // staging set t & 1 at step t - 4, written to LDS slot t & 1 at step t - 2 (that slot's
  // previous slice, t - 2, was read during step t - 3, before barrier t - 2), published by
  // barrier t - 1 and read during step t - 1.  hipcc counts these plain loads itself (vmcnt
  // before each ds_write), so no wait here is hand-placed.
  uint4_t st0[8], st1[8];
  const unsigned wofs = (unsigned)((16 * 4 * w + lrow) * kRow + ((lc ^ fsw(lrow)) << 4));
  unsigned xo[4], wo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // source offsets without the chunk swizzle (applied on the write)
    const int row = 16 * (4 * w + i) + lrow;
    xo[i] = (unsigned)(((long)tm * kBM + row) * ldx * 2) + (unsigned)(lc << 4);
    wo[i] = (unsigned)(wrow(row) * K * 2) + (unsigned)(lc << 4);
  }
  auto gload = [&](uint4_t(&st)[8], int t, int i) {
    const int so = (s0 + t) * (kBKS * 2);
    if (i < 4) st[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo[i & 3], so, 0));
    else st[i] = __builtin_bit_cast(uint4_t, __builtin_amdgcn_raw_buffer_load_b128(wrs, wo[i & 3], so, 0));
  };
  auto lwrite = [&](const uint4_t(&st)[8], int t, int i) {
    unsigned char* b = smem + (t & 1) * kSlice + wofs + (i < 4 ? 0 : kRegion) + (i & 3) * 16 * kRow;
    *reinterpret_cast<uint4_t*>(b) = st[i];
  };
  // slice s: 64 MFMAs of (fx, fw) with the 16 fragment reads of s + 1 (RD), the 8 LDS writes of
  // s + 2 (WR, staging set (s + 2) & 1 = s & 1) and the 8 loads of s + 4 into that set (LD)
  auto rstep = [&](auto rd_t, auto wr_t, auto ld_t, short8(&fx)[8], short8(&fw)[8], short8(&nx)[8],
                   short8(&nw)[8], uint4_t(&st)[8], int s) {
    constexpr bool RD = decltype(rd_t)::value, WR = decltype(wr_t)::value, LD = decltype(ld_t)::value;
    const unsigned char* nb = smem + ((s + 1) & 1) * kSlice + fofs;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (RD) {
        nx[m] = *reinterpret_cast<const short8*>(nb + (wr * 128 + m * 16) * kRow);
        nw[m] = *reinterpret_cast<const short8*>(nb + kRegion + (wc * 128 + m * 16) * kRow);
      }
      if constexpr (WR) lwrite(st, s + 2, m);
      if constexpr (LD) gload(st, s + 4, m);
#pragma unroll
      for (int n = 0; n < 8; ++n) mfma(acc[m][n], fw[n], fx[m]);
    }
  };
  auto rsync = [&]() {
    wait_lgkm0();
    barrier_raw();
  };
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(st0, 0, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(st1, 1, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) lwrite(st0, 0, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) lwrite(st1, 1, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(st0, 2, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(st1, 3, i);
  rsync();
  {
    const unsigned char* b0 = smem + fofs;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      fx0[m] = *reinterpret_cast<const short8*>(b0 + (wr * 128 + m * 16) * kRow);
      fw0[m] = *reinterpret_cast<const short8*>(b0 + kRegion + (wc * 128 + m * 16) * kRow);
    }
  }
  int s = 0;
  for (; s + 6 <= ns; s += 2) {
    rsync();
    rstep(T{}, T{}, T{}, fx0, fw0, fx1, fw1, st0, s);
    rsync();
    rstep(T{}, T{}, T{}, fx1, fw1, fx0, fw0, st1, s + 1);
  }
  rsync();
  rstep(T{}, T{}, F{}, fx0, fw0, fx1, fw1, st0, s);
  rsync();
  rstep(T{}, T{}, F{}, fx1, fw1, fx0, fw0, st1, s + 1);
  rsync();
  rstep(T{}, F{}, F{}, fx0, fw0, fx1, fw1, st0, s + 2);
  rsync();
  rstep(F{}, F{}, F{}, fx1, fw1, fx0, fw0, st1, s + 3);
  }
  // MFMA results -> VALU reads of the accumulators: the asm MFMAs are invisible to hipcc's
  // hazard recognizer, so wait out the longest MFMA -> read latency here
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

  // ---- epilogue: lane holds row tm*256 + wr*128 + 16m + r; fragment pair (2p, 2p+1) the 8
  // consecutive columns 32p + 8g .. +7 of the wave's 128 (SwiGLU: gate pairs 0, 1 and up
  // pairs 2, 3 over the wave's 64 output columns)
  auto put8 = [](bf16_t* dst, const float (&y)[8]) {
    uint4_t pk;
    pk.x = pack_bf2(y[0], y[1]);
    pk.y = pack_bf2(y[2], y[3]);
    pk.z = pack_bf2(y[4], y[5]);
    pk.w = pack_bf2(y[6], y[7]);
    *reinterpret_cast<uint4_t*>(dst) = pk;
  };
  if constexpr (EPI == EPI_PARTIAL) {
    float* part = reinterpret_cast<float*>(out) + (long)kz * M * ldo;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M) continue;
      float* prow = part + (long)row * ldo + tn * kBN + wc * 128;
#pragma unroll
      for (int n = 0; n < 8; ++n) *reinterpret_cast<floatx4*>(prow + 32 * (n >> 1) + 8 * g + 4 * (n & 1)) = acc[m][n];
    }
  } else if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * kBM + wr * 128 + m * 16 + r;
      if (row >= M) continue;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            y[4 * h + v] = rbf(lk_silu(rbf(acc[m][2 * p + h][v]))) * rbf(acc[m][4 + 2 * p + h][v]);
        put8(out + (long)row * ldo + tn * 128 + wc * 64 + 32 * p + 8 * g, y);
      }
    }
  } else {
    float bv[8][4];
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) bv[n][v] = 0.f;
    if constexpr (EPI != EPI_NONE) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint4_t b = *reinterpret_cast<const uint4_t*>(bias + tn * kBN + wc * 128 + 32 * p + 8 * g);
        const unsigned bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bv[2 * p + (q >> 1)][2 * (q & 1)] = bf2f((bf16_t)(bw[q] & 0xFFFF));
          bv[2 * p + (q >> 1)][2 * (q & 1) + 1] = bf2f((bf16_t)(bw[q] >> 16));
        }
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
      if (row >= M) continue;
      bf16_t* orow = out + (long)row * ldo + tn * kBN + wc * 128;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int v = 0; v < 4; ++v) y[4 * h + v] = act(acc[m][2 * p + h][v], bv[2 * p + h][v]);
        put8(orow + 32 * p + 8 * g, y);
      }
    }
  }
}

template <int EPI, int MODE>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(const bf16_t* __restrict__ X, long ldx,
                                                        const bf16_t* __restrict__ W,
                                                        const bf16_t* __restrict__ bias, int M, int K, int I,
                                                        bf16_t* __restrict__ out, long ldo, int TM, int TN,
                                                        int group_m) {
  gemm4w_body<EPI, MODE>(X, ldx, W, bias, M, K, I, out, ldo, TM, TN, group_m, blockIdx.x);
}

int group_rows4() {
  static const int g = [] {
    const char* e = getenv("LK_GEMM_GROUP_M");
    const int v = e ? atoi(e) : 4;
    return v >= 1 ? v : 4;
  }();
  return g;
}

template <int EPI, int MODE>
void launch4m(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
              long ldo, int TM, int TN, int ks, hipStream_t st) {
  constexpr int lds = MODE == 5 ? 2 * 2 * 256 * 128 : MODE != 1 ? kLds : 2 * kSlice;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm4w_kernel<EPI, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  gemm4w_kernel<EPI, MODE><<<dim3(TM * TN, ks), 256, lds, st>>>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN,
                                                               group_rows4());
}
int g_mode4 = 0;  // kernel variant of this call (lk_gemm4w's `variant`)
template <int EPI>
void launch4(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int K, int I, bf16_t* out,
             long ldo, int TM, int TN, int ks, hipStream_t st) {
  if (g_mode4 == 1) launch4m<EPI, 1>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
  else if (g_mode4 == 2) launch4m<EPI, 2>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
  else if (g_mode4 == 3) launch4m<EPI, 3>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
  else if (g_mode4 == 4) launch4m<EPI, 4>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
  else if (g_mode4 == 5) launch4m<EPI, 5>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
  else launch4m<EPI, 0>(x, ldx, w, bias, M, K, I, out, ldo, TM, TN, ks, st);
}

// split-K reduction (same rounding as the fused epilogues)
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* __restrict__ part, int S, int M, int N,
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

}  // namespace

int lk_gemm4w_supported(int M, int N, int K, int epi, int ks) {
  if (M < 1 || K < 64 || K % 64 || ks < 1 || ks > 8 || K / 64 < 2 * ks) return 0;
  if (epi == EPI_SWIGLU) return ks == 1 && N % 2 == 0 && (N / 2) % 128 == 0;
  return epi >= EPI_NONE && epi <= EPI_BIAS_RELU && N % kBN == 0;
}

// Same contract as lk_gemm with a fixed 256 x 256 tile (bn = 256).
int lk_gemm4w(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi,
              bf16_t* out, long ldo, hipStream_t st, int ks, float* ws, int variant) {
  // variants 2-4: timing-only ablations of variant 0's loop (2: no fragment reads, 3: no
  // LDS-DMA, 4: neither) -- WRONG results by construction, for the PMC / microbench only
  if (variant < 0 || variant > 5) return -1;
  g_mode4 = variant;
  if (!lk_gemm4w_supported(M, N, K, epi, ks) || ldx % 8 || ldo % 8 || reinterpret_cast<uintptr_t>(out) % 16 ||
      (bias != nullptr && reinterpret_cast<uintptr_t>(bias) % 16))
    return -1;
  if ((long)N * K * 2 >= 0x7FFFFFF0L) return -1;
  const long max_rows = (0x7FFFFFF0L / (ldx * 2)) / kBM * kBM;
  if (M > max_rows) {
    if (max_rows < kBM) return -1;
    for (long m0 = 0; m0 < M; m0 += max_rows) {
      const int mc = (int)min((long)M - m0, max_rows);
      const int rc = lk_gemm4w(x + m0 * ldx, ldx, w, bias, mc, N, K, epi, out + m0 * ldo, ldo, st, 1, nullptr, variant);
      if (rc) return rc;
    }
    return 0;
  }
  const int TM = (M + kBM - 1) / kBM;
  if (ks > 1) {
    if (ws == nullptr || (epi != EPI_NONE && bias == nullptr)) return -1;
    launch4<EPI_PARTIAL>(x, ldx, w, nullptr, M, K, 0, reinterpret_cast<bf16_t*>(ws), N, TM, N / kBN, ks, st);
    const long n = (long)M * (N / 4);
    const int blocks = (int)((n + 255) / 256);
    switch (epi) {
      case EPI_NONE: splitk_reduce4_kernel<EPI_NONE><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS: splitk_reduce4_kernel<EPI_BIAS><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS_GELU: splitk_reduce4_kernel<EPI_BIAS_GELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      case EPI_BIAS_RELU: splitk_reduce4_kernel<EPI_BIAS_RELU><<<blocks, 256, 0, st>>>(ws, ks, M, N, bias, out, ldo); break;
      default: return -1;
    }
    LK_CHECK_LAUNCH();
    return 0;
  }
  switch (epi) {
    case EPI_NONE: launch4<EPI_NONE>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / kBN, 1, st); break;
    case EPI_SWIGLU: launch4<EPI_SWIGLU>(x, ldx, w, bias, M, K, N / 2, out, ldo, TM, N / 256, 1, st); break;
    case EPI_BIAS: launch4<EPI_BIAS>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / kBN, 1, st); break;
    case EPI_BIAS_GELU: launch4<EPI_BIAS_GELU>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / kBN, 1, st); break;
    case EPI_BIAS_RELU: launch4<EPI_BIAS_RELU>(x, ldx, w, bias, M, K, 0, out, ldo, TM, N / kBN, 1, st); break;
    default: return -1;
  }
  LK_CHECK_LAUNCH();
  return 0;
}
