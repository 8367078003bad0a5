// K2, prefill regime: Y[M,N] = X[M,K] . W[N,K]^T for M > 256 rows (chunked-prefill
// steps, encoder batches), optionally with the SwiGLU epilogue fused:
//   out[M, I] = silu(X Wg^T) * (X Wu^T) for W = [Wg; Wu] (2I rows).
//
// gfx950 design (CDNA4 playbook, "256^2 tile" GEMM):
//   * block = 8 waves (512 threads), C tile 256 x 256, waves 2 (M) x 4 (N), each
//     wave 128 x 64 = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (128 acc VGPRs);
//   * BK = 64; both operands are K-contiguous (nn.Linear layout), staged global ->
//     LDS with 16-B LDS-DMA (global_load_lds_dwordx4): each wave instruction moves
//     8 rows x one 128-B line, lane-linear in LDS, with the (row>>1)&7 XOR chunk
//     swizzle applied on the SOURCE address, so the ds_read_b128 fragment reads are
//     bank-conflict free;
//   * 2 LDS stages (2 x 64 KB): the DMA of K-step k+1 is in flight under the MFMAs
//     of step k; one vmcnt(0) + barrier per step;
//   * operands swapped in the MFMA (A <- W rows, B <- X rows): each lane ends with
//     one output row and 4 consecutive columns, so the epilogue is 8-byte packed
//     stores straight from the accumulators (and SwiGLU pairs the gate / up
//     fragments of the same columns inside one lane);
//   * grid = (M/256) x (N/256) tiles in an XCD-aware order: consecutive logical
//     tiles run on one XCD (bijective remap), grouped 4 row tiles x N column tiles so
//     the ~32 concurrent tiles of an XCD share their X and W K-slices in its L2.
// SwiGLU: column tile t covers output columns [128t, 128t+128); wave wn's 64 B rows
// are 32 gate rows and the 32 matching up rows, so fragments n and n+2 hold gate and
// up of the same columns.  Rounded like the unfused linear -> silu_mul path.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kStageBytes = (kBM + kBN) * kBK * 2;  // 64 KB
constexpr int kGroupM = 4;

LK_DEVICE int swz(int row) { return (row >> 1) & 7; }
// s_waitcnt vmcnt(0) only (lgkmcnt / expcnt left at their maxima)
LK_DEVICE void wait_vmcnt0() { __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8)); }
LK_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }

template <bool SWIGLU>
__global__ __launch_bounds__(512, 1) void big_gemm_kernel(const bf16_t* __restrict__ X, long ldx,
                                                          const bf16_t* __restrict__ W, int M, int K, int I,
                                                          bf16_t* __restrict__ out, long ldo, int TM, int TN) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // ---- tile of this block: XCD-contiguous logical ids, grouped along M
  const int nwg = TM * TN;
  const int L = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupM * TN;
  const int first = (L / per_group) * kGroupM;
  const int gm = min(TM - first, kGroupM);
  const int tm = first + (L % per_group) % gm;
  const int tn = (L % per_group) / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int r = lane & 15, g = lane >> 4;

  // W row (output column of the plain GEMM) of B-tile row j
  auto wrow = [&](int j) -> long {
    if constexpr (SWIGLU) {
      const int q = j >> 6, jj = j & 63;
      return (jj < 32 ? 0L : (long)I) + (long)tn * 128 + q * 32 + (jj & 31);
    } else {
      return (long)tn * kBN + j;
    }
  };

  // ---- LDS-DMA sources: wave w stages rows [32w, 32w + 32) of both tiles, 8 per instruction
  const int lrow = lane >> 3, lch = lane & 7;
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = w * 32 + i * 8 + lrow;
    const long xr = min(tm * kBM + row, M - 1);  // tail rows re-read the last row; stores are masked
    asrc[i] = X + xr * ldx + (lch ^ swz(row)) * 8;
    bsrc[i] = W + wrow(row) * K + (lch ^ swz(row)) * 8;
  }
  auto issue = [&](int kt) {
    unsigned char* base = smem + (kt & 1) * kStageBytes;
    const int k = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k), (lds_ptr_t)(base + (w * 32 + i * 8) * 128), 16, 0,
                                       0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k),
                                       (lds_ptr_t)(base + kBM * 128 + (w * 32 + i * 8) * 128), 16, 0, 0);
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int kt) {
    const unsigned char* base = smem + (kt & 1) * kStageBytes;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + g;
      short8 xa[8], wb[4];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int row = wm * 128 + m * 16 + r;
        xa[m] = *reinterpret_cast<const short8*>(base + row * 128 + ((c ^ swz(row)) << 4));
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + r;
        wb[n] = *reinterpret_cast<const short8*>(base + kBM * 128 + row * 128 + ((c ^ swz(row)) << 4));
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[n], xa[m], acc[m][n], 0, 0, 0);
    }
  };

  const int nk = K / kBK;
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // vmcnt(0): stage kt landed (every wave); stage kt-1's buffer is free
    if (kt + 1 < nk) issue(kt + 1);
    compute(kt);
  }

  // ---- epilogue: lane holds row (.. + r), columns (.. + 4g + v), v = 0..3
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int row = tm * kBM + wm * 128 + m * 16 + r;
    if (row >= M) continue;
    bf16_t* orow = out + (long)row * ldo;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = tn * 128 + wn * 32 + n * 16 + 4 * g;
        float y[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) y[v] = rbf(silu_f(rbf(acc[m][n][v]))) * rbf(acc[m][n + 2][v]);
        uint2 pk;
        pk.x = pack_bf2(y[0], y[1]);
        pk.y = pack_bf2(y[2], y[3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = tn * kBN + wn * 64 + n * 16 + 4 * g;
        uint2 pk;
        pk.x = pack_bf2(acc[m][n][0], acc[m][n][1]);
        pk.y = pack_bf2(acc[m][n][2], acc[m][n][3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    }
  }
}


LK_DEVICE void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }  // no vmcnt drain, compiler fence

// Ping-pong schedule (v2): each K-step is 4 phases, one per C quadrant of the wave's
// 128 x 64 tile (4 m x 2 n fragments x K = 64 = 16 MFMAs).  A phase is a READ segment
// (its register subtile from LDS, plus LDS-DMA pieces of the next K-step) and an MFMA
// segment, each closed by a raw s_barrier.  Waves 4-7 start one barrier late, so on
// every SIMD one wave's MFMA segment runs while its partner's LDS reads run.  The DMA
// for step t+1 goes out in phases 1-2 of step t (>= 2 segments after the partner
// group's last read of that buffer), and each wave retires it with vmcnt(0) at the end
// of its phase-3 READ segment: for the lagging group that boundary is the barrier after
// which the leading group reads step t+1.
template <bool SWIGLU>
__global__ __launch_bounds__(512, 1) void big_gemm_pp_kernel(const bf16_t* __restrict__ X, long ldx,
                                                             const bf16_t* __restrict__ W, int M, int K, int I,
                                                             bf16_t* __restrict__ out, long ldo, int TM, int TN) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = TM * TN;
  const int L = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupM * TN;
  const int first = (L / per_group) * kGroupM;
  const int gm = min(TM - first, kGroupM);
  const int tm = first + (L % per_group) % gm;
  const int tn = (L % per_group) / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int r = lane & 15, g = lane >> 4;

  auto wrow = [&](int j) -> long {
    if constexpr (SWIGLU) {
      const int q = j >> 6, jj = j & 63;
      return (jj < 32 ? 0L : (long)I) + (long)tn * 128 + q * 32 + (jj & 31);
    } else {
      return (long)tn * kBN + j;
    }
  };

  const int lrow = lane >> 3, lch = lane & 7;
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = w * 32 + i * 8 + lrow;
    const long xr = min(tm * kBM + row, M - 1);
    asrc[i] = X + xr * ldx + (lch ^ swz(row)) * 8;
    bsrc[i] = W + wrow(row) * K + (lch ^ swz(row)) * 8;
  }
  auto issue_a = [&](int kt) {
    unsigned char* base = smem + (kt & 1) * kStageBytes;
    const int k = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k), (lds_ptr_t)(base + (w * 32 + i * 8) * 128), 16, 0,
                                       0);
  };
  auto issue_b = [&](int kt) {
    unsigned char* base = smem + (kt & 1) * kStageBytes + kBM * 128;
    const int k = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k), (lds_ptr_t)(base + (w * 32 + i * 8) * 128), 16, 0,
                                       0);
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  short8 xa[4][2], wb[2][2];
  auto read_a = [&](const unsigned char* base, int qm) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row = wm * 128 + (qm * 4 + m) * 16 + r;
        xa[m][h] = *reinterpret_cast<const short8*>(base + row * 128 + (((4 * h + g) ^ swz(row)) << 4));
      }
  };
  auto read_b = [&](const unsigned char* base, int qn) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int row = wn * 64 + (qn * 2 + n) * 16 + r;
        wb[n][h] = *reinterpret_cast<const short8*>(base + kBM * 128 + row * 128 + (((4 * h + g) ^ swz(row)) << 4));
      }
  };
  auto mfma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[qm * 4 + m][qn * 2 + n] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[n][h], xa[m][h], acc[qm * 4 + m][qn * 2 + n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = K / kBK;
  issue_a(0);
  issue_b(0);
  wait_vmcnt0();
  lds_barrier();
  if (wm == 1) lds_barrier();  // stagger: group 1 runs one segment behind group 0
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* base = smem + (kt & 1) * kStageBytes;
    const bool more = kt + 1 < nk;
    // phase 0: quadrant (0,0)
    read_a(base, 0);
    read_b(base, 0);
    lds_barrier();
    mfma(0, 0);
    lds_barrier();
    // phase 1: quadrant (0,1)
    read_b(base, 1);
    if (more) issue_a(kt + 1);
    lds_barrier();
    mfma(0, 1);
    lds_barrier();
    // phase 2: quadrant (1,1)
    read_a(base, 1);
    if (more) issue_b(kt + 1);
    lds_barrier();
    mfma(1, 1);
    lds_barrier();
    // phase 3: quadrant (1,0)
    read_b(base, 0);
    // this wave's DMA for step kt+1 landed.  Retired in the READ segment: the lagging
    // group's segment boundary here is the barrier after which the leading group
    // reads step kt+1.
    wait_vmcnt0();
    lds_barrier();
    mfma(1, 0);
    lds_barrier();
  }
  if (wm == 0) lds_barrier();  // equal barrier counts for both groups

#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int row = tm * kBM + wm * 128 + m * 16 + r;
    if (row >= M) continue;
    bf16_t* orow = out + (long)row * ldo;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = tn * 128 + wn * 32 + n * 16 + 4 * g;
        float y[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) y[v] = rbf(silu_f(rbf(acc[m][n][v]))) * rbf(acc[m][n + 2][v]);
        uint2 pk;
        pk.x = pack_bf2(y[0], y[1]);
        pk.y = pack_bf2(y[2], y[3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = tn * kBN + wn * 64 + n * 16 + 4 * g;
        uint2 pk;
        pk.x = pack_bf2(acc[m][n][0], acc[m][n][1]);
        pk.y = pack_bf2(acc[m][n][2], acc[m][n][3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    }
  }
}

// Variant 2: BK = 32 with a 4-stage LDS ring (4 x 32 KB).  The ping-pong structure of
// variant 1 (READ / MFMA segments, waves 4-7 one barrier behind) at 2 phases per
// 32-deep K-step -- phase p: the 4 m fragments of half p x all 4 n fragments, 16 MFMAs
// -- but the LDS-DMA runs 3 steps ahead (issued in phase 1 of step t for step t+3,
// two segments after the partner group's last read of that buffer; counted vmcnt
// retires only step t+1), so the loads see ~1.5 K=64 steps of latency cover instead
// of ~0.5.  LDS rows are 64 B: chunk c of row r lives at chunk c ^ f(r),
// f(r) = (-(r >> 2)) & 3, which keeps every ds_read_b128 lane group of the fragment
// reads (rows 0-3/12-15 at chunk c, rows 4-11 at chunk c+1) on 16 distinct bank slots.
constexpr int kBK2 = 32, kStages2 = 4;
constexpr int kStage2Bytes = (kBM + kBN) * kBK2 * 2;  // 32 KB

LK_DEVICE int swz2(int row) { return (4 - ((row >> 2) & 3)) & 3; }

template <int N>
LK_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt");
  __builtin_amdgcn_s_waitcnt(N | (0x7 << 4) | (0xF << 8));
}

template <bool SWIGLU>
__global__ __launch_bounds__(512, 1) void big_gemm_r4_kernel(const bf16_t* __restrict__ X, long ldx,
                                                             const bf16_t* __restrict__ W, int M, int K, int I,
                                                             bf16_t* __restrict__ out, long ldo, int TM, int TN) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = TM * TN;
  const int L = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupM * TN;
  const int first = (L / per_group) * kGroupM;
  const int gm = min(TM - first, kGroupM);
  const int tm = first + (L % per_group) % gm;
  const int tn = (L % per_group) / gm;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int r = lane & 15, g = lane >> 4;

  auto wrow = [&](int j) -> long {
    if constexpr (SWIGLU) {
      const int q = j >> 6, jj = j & 63;
      return (jj < 32 ? 0L : (long)I) + (long)tn * 128 + q * 32 + (jj & 31);
    } else {
      return (long)tn * kBN + j;
    }
  };

  // DMA: a wave instruction moves 16 rows x 64 B; wave w stages rows [32w, 32w+32) of each tile
  const int lrow = lane >> 2, lch = lane & 3;
  const bf16_t* asrc[2];
  const bf16_t* bsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = w * 32 + i * 16 + lrow;
    const long xr = min(tm * kBM + row, M - 1);
    asrc[i] = X + xr * ldx + (lch ^ swz2(row)) * 8;
    bsrc[i] = W + wrow(row) * K + (lch ^ swz2(row)) * 8;
  }
  auto issue = [&](int kt) {
    unsigned char* base = smem + (kt & (kStages2 - 1)) * kStage2Bytes;
    const int k = kt * kBK2;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[i] + k), (lds_ptr_t)(base + (w * 32 + i * 16) * 64), 16, 0,
                                       0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + k),
                                       (lds_ptr_t)(base + kBM * 64 + (w * 32 + i * 16) * 64), 16, 0, 0);
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  short8 xa[4], wb[4];
  auto read_a = [&](const unsigned char* base, int half) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = wm * 128 + (half * 4 + m) * 16 + r;
      xa[m] = *reinterpret_cast<const short8*>(base + row * 64 + ((g ^ swz2(row)) << 4));
    }
  };
  auto read_b = [&](const unsigned char* base) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = wn * 64 + n * 16 + r;
      wb[n] = *reinterpret_cast<const short8*>(base + kBM * 64 + row * 64 + ((g ^ swz2(row)) << 4));
    }
  };
  auto mfma = [&](int half) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[half * 4 + m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[n], xa[m], acc[half * 4 + m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = K / kBK2;  // >= 2 (K >= 64)
  issue(0);
  issue(1);
  if (nk > 2) {
    issue(2);
    wait_vm<8>();
  } else {
    wait_vm<4>();
  }
  lds_barrier();
  if (wm == 1) lds_barrier();  // stagger
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* base = smem + (kt & (kStages2 - 1)) * kStage2Bytes;
    // phase 0
    read_a(base, 0);
    read_b(base);
    lds_barrier();
    mfma(0);
    lds_barrier();
    // phase 1: DMA for step kt+3, then retire step kt+1 (read after this segment's barrier)
    read_a(base, 1);
    if (kt + 3 < nk) {
      issue(kt + 3);
      wait_vm<8>();
    } else if (kt + 2 < nk) {
      wait_vm<4>();
    } else {
      wait_vm<0>();
    }
    lds_barrier();
    mfma(1);
    lds_barrier();
  }
  if (wm == 0) lds_barrier();

#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int row = tm * kBM + wm * 128 + m * 16 + r;
    if (row >= M) continue;
    bf16_t* orow = out + (long)row * ldo;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = tn * 128 + wn * 32 + n * 16 + 4 * g;
        float y[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) y[v] = rbf(silu_f(rbf(acc[m][n][v]))) * rbf(acc[m][n + 2][v]);
        uint2 pk;
        pk.x = pack_bf2(y[0], y[1]);
        pk.y = pack_bf2(y[2], y[3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = tn * kBN + wn * 64 + n * 16 + 4 * g;
        uint2 pk;
        pk.x = pack_bf2(acc[m][n][0], acc[m][n][1]);
        pk.y = pack_bf2(acc[m][n][2], acc[m][n][3]);
        *reinterpret_cast<uint2*>(orow + col) = pk;
      }
    }
  }
}

template <bool SWIGLU>
void launch_big(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int I, bf16_t* out, long ldo, int TM,
                int TN, int variant, hipStream_t st) {
  auto kern = variant == 0 ? big_gemm_kernel<SWIGLU> : variant == 1 ? big_gemm_pp_kernel<SWIGLU>
                                                                      : big_gemm_r4_kernel<SWIGLU>;
  static bool attr[3] = {false, false, false};
  if (!attr[variant]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * kStageBytes);
    attr[variant] = true;
  }
  kern<<<TM * TN, 512, 2 * kStageBytes, st>>>(x, ldx, w, M, K, I, out, ldo, TM, TN);
}

}  // namespace

// out = X W^T (swiglu=0: W [N, K], out [M, N]) or silu(X Wg^T) * (X Wu^T) (swiglu=1: W = [Wg; Wu]
// of N = 2I rows, out [M, I]).  Requires K % 64 == 0, N % 256 == 0 (plain) / I % 128 == 0 (SwiGLU),
// 16-B aligned rows; any M >= 1.
int lk_big_gemm(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int swiglu, bf16_t* out,
                long ldo, int variant, hipStream_t st) {
  if (M < 1 || K < kBK || K % kBK || ldx % 8 || ldo % 4 || variant < 0 || variant > 2) return -1;
  const int TM = (M + kBM - 1) / kBM;
  if (swiglu) {
    if (N % 2 || (N / 2) % 128) return -1;
    const int I = N / 2;
    launch_big<true>(x, ldx, w, M, K, I, out, ldo, TM, I / 128, variant, st);
  } else {
    if (N % kBN) return -1;
    launch_big<false>(x, ldx, w, M, K, 0, out, ldo, TM, N / kBN, variant, st);
  }
  LK_CHECK_LAUNCH();
  return 0;
}
