// K2, decode regime: Y[M,N] = X[M,K] . W[N,K]^T for M <= 128 rows (one decode
// token per running sequence), optionally with the SwiGLU epilogue fused.
//
// At M <= 128 every Llama linear is HBM-bound on the weight stream (O-proj at
// M=64: 32 MiB of W vs 2 GFLOP), so the kernel is built to keep all 256 CUs
// pulling W at full rate rather than to maximise MFMA reuse:
//   * block = 4 waves owning BN = 16*NTW output columns and ALL M rows; the
//     4 waves split the block's K range (intra-block split-K), so every W and
//     X element a block needs is loaded exactly once, straight to VGPRs in the
//     MFMA fragment layout (no LDS round trip on the way in: the "GEMV / M<=16"
//     rule of the CDNA4 playbook, extended to M<=128 because X is tiny and
//     L2-resident).
//   * blocks split K further (S-way) when N/BN alone would leave CUs idle
//     (QKV/O/down at 64-96 column tiles); S partial slabs go to an f32
//     workspace and a 16-B-vectorised reduce kernel sums them (with the SwiGLU
//     epilogue when fused).  gate_up (448 tiles) and the LM head run S=1 with
//     the epilogue in the GEMM itself.
//   * W is read with non-temporal loads (streamed once; keeps X in L2), one
//     64-deep K step of fragments in flight under the current step's MFMAs.
//   * v_mfma_f32_16x16x32_bf16: lane l holds A = X[16m + (l&15)][k0 + 8(l>>4) + j]
//     and B = W[n0 + (l&15)][k0 + 8(l>>4) + j]: both are 16-B row-contiguous
//     loads, two K sub-steps cover each 128-B line of W exactly.
//   * the 4 waves' f32 tiles are summed through LDS (rows padded by 4 floats so
//     the 4 lane groups hit different banks) and stored coalesced.
// SwiGLU fusion: block t owns gate columns [t*BN/2, (t+1)*BN/2) and the matching
// up columns I + [...]; out[m][j] = bf16(silu(bf16(g)) ) * bf16(u), rounded like
// the unfused linear -> silu_mul path (bit-identical to it).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int kSkW = 4;  // waves per block

LK_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }

template <int MT, int NTW, bool SWIGLU>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(
    const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W, int M, int K, int ks,
    int n_tiles, int swiglu_I, bf16_t* __restrict__ out, long ldo, float* __restrict__ part,
    long part_ld) {
  constexpr int BN = 16 * NTW;
  constexpr int ROWS = 16 * MT;
  constexpr int LDR = BN + 4;
  extern __shared__ float red[];  // [kSkW][ROWS][LDR]

  const int t = blockIdx.x % n_tiles, s = blockIdx.x / n_tiles;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int kw = ks / kSkW;
  const long kbase = (long)s * ks + (long)w * kw + 8 * g;

  auto ncol = [&](int c) -> long {  // global W row (output column) of column tile c, lane r
    if constexpr (SWIGLU) {
      constexpr int H = NTW / 2;
      return c < H ? (long)t * (BN / 2) + 16 * c + r : (long)swiglu_I + (long)t * (BN / 2) + 16 * (c - H) + r;
    } else {
      return (long)t * BN + 16 * c + r;
    }
  };

  const bf16_t* wp[NTW];
#pragma unroll
  for (int c = 0; c < NTW; ++c) wp[c] = W + ncol(c) * K + kbase;
  const bf16_t* xp[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int row = min(16 * m + r, M - 1);
    xp[m] = X + (long)row * ldx + kbase;
  }

  floatx4 acc[MT][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int c = 0; c < NTW; ++c) acc[m][c] = floatx4{0.f, 0.f, 0.f, 0.f};

  short8 wa[NTW][2], xa[MT][2], wb[NTW][2], xb[MT][2];
  auto load = [&](short8 (&wf)[NTW][2], short8 (&xf)[MT][2], int k) {
#pragma unroll
    for (int c = 0; c < NTW; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        wf[c][h] = __builtin_nontemporal_load(reinterpret_cast<const short8*>(wp[c] + k + 32 * h));
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h) xf[m][h] = *reinterpret_cast<const short8*>(xp[m] + k + 32 * h);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issued ahead of the MFMAs below
  };
  auto compute = [&](const short8 (&wf)[NTW][2], const short8 (&xf)[MT][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int c = 0; c < NTW; ++c)
          acc[m][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[m][h], wf[c][h], acc[m][c], 0, 0, 0);
  };

  // ping-pong register sets, no copies (a copy of a just-loaded register makes the
  // compiler wait for that load and serialises the stream): step i+1 is in flight
  // under step i's MFMAs.
  const int nsteps = kw / 64;
  load(wa, xa, 0);
  int i = 0;
  for (; i + 2 < nsteps; i += 2) {
    load(wb, xb, (i + 1) * 64);
    compute(wa, xa);
    load(wa, xa, (i + 2) * 64);
    compute(wb, xb);
  }
  if (nsteps - i == 2) {
    load(wb, xb, (i + 1) * 64);
    compute(wa, xa);
    compute(wb, xb);
  } else {
    compute(wa, xa);
  }

  // ---- intra-block split-K reduction through LDS
  float* mine = red + w * ROWS * LDR;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int c = 0; c < NTW; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) mine[(16 * m + 4 * g + i) * LDR + 16 * c + r] = acc[m][c][i];
  __syncthreads();

  auto sum4 = [&](int row, int col) -> floatx4 {
    floatx4 v = *reinterpret_cast<const floatx4*>(red + row * LDR + col);
#pragma unroll
    for (int ww = 1; ww < kSkW; ++ww) {
      const floatx4 u = *reinterpret_cast<const floatx4*>(red + ww * ROWS * LDR + row * LDR + col);
      v += u;
    }
    return v;
  };

  const bool split = part != nullptr;
  if (SWIGLU && !split) {
    constexpr int HB = BN / 2, Q = HB / 4;
    for (int idx = threadIdx.x; idx < ROWS * Q; idx += 256) {
      const int row = idx / Q, c4 = (idx % Q) * 4;
      if (row >= M) continue;
      const floatx4 gv = sum4(row, c4), uv = sum4(row, HB + c4);
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = rbf(silu_f(rbf(gv[i]))) * rbf(uv[i]);
      uint2 pk;
      pk.x = pack_bf2(y[0], y[1]);
      pk.y = pack_bf2(y[2], y[3]);
      *reinterpret_cast<uint2*>(out + (long)row * ldo + (long)t * HB + c4) = pk;
    }
  } else {
    constexpr int Q = BN / 4;
    for (int idx = threadIdx.x; idx < ROWS * Q; idx += 256) {
      const int row = idx / Q, c4 = (idx % Q) * 4;
      if (row >= M) continue;
      const floatx4 v = sum4(row, c4);
      if (split) {
        long n;
        if constexpr (SWIGLU) {
          n = c4 < BN / 2 ? (long)t * (BN / 2) + c4 : (long)swiglu_I + (long)t * (BN / 2) + c4 - BN / 2;
        } else {
          n = (long)t * BN + c4;
        }
        *reinterpret_cast<floatx4*>(part + (long)s * M * part_ld + (long)row * part_ld + n) = v;
      } else {
        uint2 pk;
        pk.x = pack_bf2(v[0], v[1]);
        pk.y = pack_bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(out + (long)row * ldo + (long)t * BN + c4) = pk;
      }
    }
  }
}

// sum S f32 slabs [S][M][ld] -> bf16 out (optionally SwiGLU over [gate | up])
template <bool SWIGLU>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int M,
                                                            long ld, int n_out, int swiglu_I,
                                                            bf16_t* __restrict__ out, long ldo) {
  const int q = n_out / 4;
  const long total = (long)M * q;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int row = (int)(i / q), c4 = (int)(i % q) * 4;
    const float* p = part + (long)row * ld + c4;
    floatx4 v = *reinterpret_cast<const floatx4*>(p);
    for (int s = 1; s < S; ++s) v += *reinterpret_cast<const floatx4*>(p + (long)s * M * ld);
    float y[4];
    if constexpr (SWIGLU) {
      floatx4 u = *reinterpret_cast<const floatx4*>(p + swiglu_I);
      for (int s = 1; s < S; ++s) u += *reinterpret_cast<const floatx4*>(p + (long)s * M * ld + swiglu_I);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = rbf(silu_f(rbf(v[j]))) * rbf(u[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = v[j];
    }
    uint2 pk;
    pk.x = pack_bf2(y[0], y[1]);
    pk.y = pack_bf2(y[2], y[3]);
    *reinterpret_cast<uint2*>(out + (long)row * ldo + c4) = pk;
  }
}

template <int MT, int NTW, bool SWIGLU>
void launch_skinny(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S, int n_tiles,
                   int I, bf16_t* out, long ldo, float* part, long part_ld, hipStream_t st) {
  const size_t lds = sizeof(float) * kSkW * 16 * MT * (16 * NTW + 4);
  auto kern = skinny_gemm_kernel<MT, NTW, SWIGLU>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr = true;
  }
  kern<<<n_tiles * S, 256, lds, st>>>(x, ldx, w, M, K, ks, n_tiles, I, out, ldo, part, part_ld);
}

template <bool SWIGLU>
int dispatch_mt(int MT, const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S, int n_tiles,
                int I, bf16_t* out, long ldo, float* part, long part_ld, hipStream_t st) {
  switch (MT) {
    case 1: launch_skinny<1, 4, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, st); break;
    case 2: launch_skinny<2, 4, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, st); break;
    case 4: launch_skinny<4, 4, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, st); break;
    case 8: launch_skinny<8, 4, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, st); break;
    default: return -2;
  }
  return 0;
}

}  // namespace

int lk_skinny_splits(int M, int N, int K, int swiglu) {
  (void)M;
  const int BN = 64;
  const int cols = swiglu ? N / 2 : N;
  const int n_tiles = cols / (swiglu ? BN / 2 : BN);
  int S = 1;
  while (n_tiles * S < 256 && S < 8 && K % (2 * S * kSkW * 64) == 0 && K / (2 * S) >= 512) S *= 2;
  return S;
}

// out = X W^T (swiglu=0, out [M,N]) or silu(X Wg^T) * (X Wu^T) (swiglu=1, W = [Wg; Wu]
// of 2I rows, out [M,I]).  part: f32 workspace of S*M*N floats when S > 1.
int lk_skinny_gemm(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int S, int swiglu,
                   bf16_t* out, long ldo, float* part, hipStream_t st) {
  if (M < 1 || M > 128 || S < 1 || K % (S * kSkW * 64)) return -1;
  const int BN = 64;
  if (swiglu ? (N % 2 || (N / 2) % (BN / 2)) : N % BN) return -1;
  if (S > 1 && part == nullptr) return -1;
  const int I = swiglu ? N / 2 : 0;
  const int n_tiles = swiglu ? I / (BN / 2) : N / BN;
  const int MT = M <= 16 ? 1 : M <= 32 ? 2 : M <= 64 ? 4 : 8;
  const int ks = K / S;
  float* p = S > 1 ? part : nullptr;
  const int rc = swiglu ? dispatch_mt<true>(MT, x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, p, N, st)
                        : dispatch_mt<false>(MT, x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, p, N, st);
  if (rc) return rc;
  if (S > 1) {
    const int n_out = swiglu ? I : N;
    const long work = (long)M * (n_out / 4);
    int grid = (int)((work + 255) / 256);
    if (grid > 2048) grid = 2048;
    if (swiglu)
      splitk_reduce_kernel<true><<<grid, 256, 0, st>>>(part, S, M, N, n_out, I, out, ldo);
    else
      splitk_reduce_kernel<false><<<grid, 256, 0, st>>>(part, S, M, N, n_out, 0, out, ldo);
  }
  LK_CHECK_LAUNCH();
  return 0;
}
