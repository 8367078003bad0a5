// Decode-step GEMV for one or two rows (batch-1 / batch-2 decode), with the neighbouring
// elementwise work of a Llama block folded into its prologue and epilogue.
//
// At M <= 2 a projection is a pure weight stream (16 GB per Llama-3-8B step), so the MFMA tile
// machinery of the weight-streaming GEMM (skinny_gemm.hip: 16-row padded tiles, split-K slabs
// reduced by a second kernel) buys nothing, while the kernels around it (split-K reduce,
// residual add + RMSNorm, RoPE + KV write) each cost a dependent ~5 us launch.  Here:
//   * one wave owns a PAIR of W rows at a time and splits K over its 64 lanes in 16-B chunks
//     (lane l: chunks l, l + 64, ...: every wave load is one contiguous 1-KB segment of a row),
//     U chunks of both rows in flight per lane; fp32 FMAs, 64-lane butterfly at the end -- no
//     split-K, no partial slabs;
//   * long-K projections (an even number >= 2 of U-chunk blocks per row: down at K 14,336) give
//     each pair two waves, a K half each, joined in LDS (KW = 2);
//   * X (the M input rows) is staged once per workgroup in LDS by LDS-DMA; the NORM prologue
//     computes RMSNorm(res) * gamma there itself (the rmsnorm kernel's exact arithmetic), so the
//     producer of res never launches a norm; PRO 2 (the O projection, opt-in: measured slower)
//     merges the paged-decode split partials there instead of a decode_reduce launch;
//   * epilogues on the pair's two dot products: 0 plain bf16 out, 1 res += out (the residual
//     stream updated in place, each element owned by one wave), 2 SwiGLU (pair = gate row p,
//     up row I + p: the splitk_reduce_kernel<true> arithmetic), 3 RoPE + paged-KV write (pair =
//     the two rows one rotation mixes: (2i, 2i+1) for weights permuted by fold_norms, (i,
//     i + D/2) rotate-half otherwise; q rotated into out, k rotated into the cache and kept
//     unrotated in out, v copied -- the rope_kv_kernel contract).
// A Llama block's decode step becomes QKV(norm, rope/kv) -> paged decode -> O(+res) ->
// gate_up(norm, swiglu) -> down(+res): no reduce, norm or RoPE launches
// (models/llama.py _forward_decode_gemv; the block it computes is the reference's generate
// call, Minimal_RAG/Helpers/Helpers.cs:116, served by Ollama).
#include "common.h"
#include "kernels.h"

namespace {

struct GemvArgs {
  const bf16_t* x = nullptr;  // [M, K] input rows (NORM: the residual rows to normalise)
  long ldx = 0;
  const bf16_t* gamma = nullptr;  // NORM weights [K]
  float eps = 0.f;
  const bf16_t* w = nullptr;  // [N, K] row-major
  int M = 0, N = 0, K = 0;
  int npairs = 0;
  bf16_t* out = nullptr;  // modes 0 / 2 / 3
  long ldo = 0;
  bf16_t* res = nullptr;  // mode 1
  long ldr = 0;
  int I = 0;  // mode 2: gate rows [0, I), up rows [I, 2I)
  // mode 3
  const int* positions = nullptr;
  const float* cos_sin = nullptr;
  int Hq = 0, Hkv = 0, D = 0, BS = 0, neox = 0;
  bf16_t* kc = nullptr;
  bf16_t* vc = nullptr;
  const int* slots = nullptr;
  // PRO 2 (O projection): the paged-decode split partials of X's rows, merged in the prologue
  const float* po = nullptr;   // [(row * Hq + h) * max_splits + s][D]
  const float* pml = nullptr;  // [(row * Hq + h) * max_splits + s][2] (max in the log2 domain, sum)
  const int* ctx = nullptr;
  int max_splits = 0, split = 0;
};

typedef __attribute__((address_space(3))) void* gemv_lptr;
typedef const __attribute__((address_space(1))) void* gemv_gptr;

LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }
LK_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }

// 8 bf16 (one 16-B chunk, as 4 dwords) -> fp32 pairs: lo = w << 16, hi = w & 0xffff0000
LK_DEVICE void dot8(const uint4_t wv, const uint4_t xv, float& acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned a = wv[j], b = xv[j];
    acc = fmaf(__uint_as_float(a << 16), __uint_as_float(b << 16), acc);
    acc = fmaf(__uint_as_float(a & 0xffff0000u), __uint_as_float(b & 0xffff0000u), acc);
  }
}

template <int MR, int PRO, int MODE, int U, int KW>
__global__ __launch_bounds__(256) void gemv_decode_kernel(GemvArgs g) {
  constexpr bool NORM = PRO == 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);  // [MR][K]
  __shared__ float red[4 * MR];
  const int K = g.K;
  const int nch = K >> 3;  // 16-B chunks per row
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;

  // rows of pair p (see the header)
  auto pair_rows = [&](int p, long& ra, long& rb, int& hd, int& head, int& ip) {
    if constexpr (MODE == 2) {
      ra = p;
      rb = (long)g.I + p;
    } else if constexpr (MODE == 3) {
      hd = g.D >> 1;
      head = p / hd;
      ip = p - head * hd;
      if (g.neox && head < g.Hq + g.Hkv) {
        ra = (long)head * g.D + ip;
        rb = ra + hd;
      } else {
        ra = (long)head * g.D + 2 * ip;
        rb = ra + 1;
      }
    } else {
      ra = 2L * p;
      rb = ra + 1;
    }
  };
  const int kc_lane = nch >> 6;  // chunks per lane (K % 512 == 0)

  // ---- stage X (with the RMSNorm prologue) into LDS.  The rows (and gamma) come in by LDS-DMA
  // (global_load_lds: no registers, every chunk's load in flight at once, one memory round trip
  // for the whole prologue -- a load -> store loop serialised K / 2048 of them); chunk c of row m
  // lands at xs + m * K + 8 c (64 consecutive chunks per wave instruction: nch % 64 == 0)
  bf16_t* gs = xs + MR * K;  // NORM: gamma [K]
  // PRO 2: rows whose attention ran in more than one split are merged below (flash-decoding merge,
  // decode_reduce_kernel's arithmetic); the attention kernel wrote the others into x itself
  int nsp[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
    nsp[m] = PRO == 2 ? max(0, min((g.ctx[m] + g.split - 1) / g.split, g.max_splits)) : 1;
  for (int c0 = wv * 64; c0 < nch; c0 += 256) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (nsp[m] <= 1)
        __builtin_amdgcn_global_load_lds((gemv_gptr)(g.x + (long)m * g.ldx + (c0 + lane) * 8),
                                         (gemv_lptr)(xs + m * K + c0 * 8), 16, 0, 0);
    if constexpr (NORM)
      __builtin_amdgcn_global_load_lds((gemv_gptr)(g.gamma + (c0 + lane) * 8), (gemv_lptr)(gs + c0 * 8), 16, 0, 0);
  }
  if constexpr (PRO == 2) {
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int ns = nsp[m];
      if (ns <= 1) continue;
      for (int c = threadIdx.x; c < nch; c += 256) {
        const int e0 = c * 8, h = e0 / g.D, d0 = e0 - h * g.D;
        const long base = ((long)m * g.Hq + h) * g.max_splits;
        float Mx = -INFINITY;
        for (int q = 0; q < ns; ++q) Mx = fmaxf(Mx, g.pml[(base + q) * 2]);
        if (Mx == -INFINITY) Mx = 0.f;
        float den = 0.f, num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int q = 0; q < ns; ++q) {
          const float f = exp2f(g.pml[(base + q) * 2] - Mx);
          den += f * g.pml[(base + q) * 2 + 1];
          const floatx4 a = *reinterpret_cast<const floatx4*>(g.po + (base + q) * g.D + d0);
          const floatx4 b = *reinterpret_cast<const floatx4*>(g.po + (base + q) * g.D + d0 + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            num[j] += f * a[j];
            num[j + 4] += f * b[j];
          }
        }
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = den > 0.f ? num[j] / den : 0.f;
        store8(xs + m * K + e0, y);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (lgkmcnt / expcnt untouched)
  __syncthreads();
  if constexpr (NORM) {
    // RMSNorm with rmsnorm_kernel's rounding: y = bf16(bf16(v * inv) * g), in place in LDS
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      float ss = 0.f;
      for (int c = threadIdx.x; c < nch; c += 256) {
        const uint4_t v = *reinterpret_cast<const uint4_t*>(xs + m * K + c * 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float lo = __uint_as_float(v[j] << 16), hi = __uint_as_float(v[j] & 0xffff0000u);
          ss += lo * lo + hi * hi;
        }
      }
      ss = wave_sum(ss);
      if (lane == 0) red[m * 4 + wv] = ss;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float tot = red[m * 4] + red[m * 4 + 1] + red[m * 4 + 2] + red[m * 4 + 3];
      const float inv = rsqrtf(tot / (float)K + g.eps);
      for (int c = threadIdx.x; c < nch; c += 256) {
        const uint4_t v = *reinterpret_cast<const uint4_t*>(xs + m * K + c * 8);
        const uint4_t gv = *reinterpret_cast<const uint4_t*>(gs + c * 8);
        uint4_t o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float y0 = rbf(__uint_as_float(v[j] << 16) * inv) * __uint_as_float(gv[j] << 16);
          const float y1 = rbf(__uint_as_float(v[j] & 0xffff0000u) * inv) * __uint_as_float(gv[j] & 0xffff0000u);
          o[j] = pack_bf2(y0, y1);
        }
        *reinterpret_cast<uint4_t*>(xs + m * K + c * 8) = o;
      }
    }
    __syncthreads();
  }

  // ---- stream W: one pair of rows per KW waves at a time (KW = 2: the two waves take one half of
  // K each and their sums meet in LDS -- twice the loads in flight for the long-K projections).
  // The round loop is uniform over the workgroup (its barriers), a wave past the last pair idles.
  constexpr int PPW = 4 / KW;  // pairs per workgroup per round
  const int ps = wv / KW, kh = wv % KW;
  const int kc_w = kc_lane / KW;  // chunks per lane of this wave's part of K
  const int jb = kh * kc_w;
  __shared__ float red2[KW > 1 ? PPW : 1][MR][2];
  for (int pb = blockIdx.x * PPW; pb < g.npairs; pb += gridDim.x * PPW) {
    const int p = pb + ps;
    const bool valid = p < g.npairs;
    long ra = 0, rb = 0;
    int hd = 0, head = 0, ip = 0;
    float acc_a[MR], acc_b[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) acc_a[m] = acc_b[m] = 0.f;
    if (valid) {
      pair_rows(p, ra, rb, hd, head, ip);
      const uint4_t* wa = reinterpret_cast<const uint4_t*>(g.w + ra * K) + lane;
      const uint4_t* wb = reinterpret_cast<const uint4_t*>(g.w + rb * K) + lane;
      const uint4_t* xl = reinterpret_cast<const uint4_t*>(xs) + lane;
      for (int j0 = jb; j0 < jb + kc_w; j0 += U) {
        uint4_t va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          va[u] = __builtin_nontemporal_load(wa + (j0 + u) * 64);
          vb[u] = __builtin_nontemporal_load(wb + (j0 + u) * 64);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const uint4_t xv = xl[m * nch + (j0 + u) * 64];
            dot8(va[u], xv, acc_a[m]);
            dot8(vb[u], xv, acc_b[m]);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      acc_a[m] = wave_sum(acc_a[m]);
      acc_b[m] = wave_sum(acc_b[m]);
    }
    if constexpr (KW > 1) {
      static_assert(KW == 2, "two K halves");
      if (kh == 1 && lane == 0)
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          red2[ps][m][0] = acc_a[m];
          red2[ps][m][1] = acc_b[m];
        }
      __syncthreads();
      if (kh == 0)
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          acc_a[m] += red2[ps][m][0];
          acc_b[m] += red2[ps][m][1];
        }
      __syncthreads();  // (red2 is rewritten next round)
      if (kh != 0) continue;
    }
    if (!valid) continue;
    if (lane != 0) continue;
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float da = acc_a[m], db = acc_b[m];
      if constexpr (MODE == 0) {
        g.out[(long)m * g.ldo + ra] = f2bf(da);
        g.out[(long)m * g.ldo + rb] = f2bf(db);
      } else if constexpr (MODE == 1) {
        bf16_t* rr = g.res + (long)m * g.ldr;
        const unsigned old = *reinterpret_cast<const unsigned*>(rr + ra);  // (ra even: rb = ra + 1)
        const float va = rbf(rbf(da) + __uint_as_float(old << 16));
        const float vb = rbf(rbf(db) + __uint_as_float(old & 0xffff0000u));
        *reinterpret_cast<unsigned*>(rr + ra) = pack_bf2(va, vb);
      } else if constexpr (MODE == 2) {
        g.out[(long)m * g.ldo + p] = f2bf(rbf(silu_f(rbf(da))) * rbf(db));
      } else {
        bf16_t* orow = g.out + (long)m * g.ldo;
        const float x1 = rbf(da), x2 = rbf(db);
        const int slot = g.slots ? g.slots[m] : -1;
        const long blk = slot >= 0 ? slot / g.BS : 0;
        const int off = slot >= 0 ? slot % g.BS : 0;
        const int d0 = (int)(ra - (long)head * g.D), d1 = (int)(rb - (long)head * g.D);
        if (head >= g.Hq + g.Hkv) {  // V: copied (into the row and the cache)
          const int h = head - g.Hq - g.Hkv;
          orow[ra] = f2bf(x1);
          orow[rb] = f2bf(x2);
          if (g.vc && slot >= 0) {
            bf16_t* vd = g.vc + ((blk * g.Hkv + h) * g.BS + off) * g.D;
            vd[d0] = f2bf(x1);
            vd[d1] = f2bf(x2);
          }
        } else {
          const float* cs = g.cos_sin + (long)g.positions[m] * g.D;  // [cos(D/2) | sin(D/2)]
          const float c = cs[ip], s = cs[hd + ip];
          const float y1 = x1 * c - x2 * s, y2 = x2 * c + x1 * s;
          if (head < g.Hq) {
            orow[ra] = f2bf(y1);
            orow[rb] = f2bf(y2);
          } else {  // K: unrotated in the row, rotated in the cache
            orow[ra] = f2bf(x1);
            orow[rb] = f2bf(x2);
            if (g.kc && slot >= 0) {
              bf16_t* kd = g.kc + ((blk * g.Hkv + (head - g.Hq)) * g.BS + off) * g.D;
              kd[d0] = f2bf(y1);
              kd[d1] = f2bf(y2);
            }
          }
        }
      }
    }
  }
}

// Infinity-Cache (L3) prefetch: default-policy 16-B loads over [p, p + bytes) whose values are
// folded into one word that is stored only if it equals a value no sum of these loads takes in
// practice (the loads cannot be dropped).  Launched on a side stream while the latency-bound
// attention kernels leave HBM idle, so the next projection's weights are read from the 256 MiB L3.
__global__ __launch_bounds__(256) void l3_prefetch_kernel(const uint4_t* __restrict__ p, long n16,
                                                          unsigned* __restrict__ sink) {
  unsigned acc = 0;
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    uint4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  for (; i < n16; i += stride) {
    const uint4_t v = p[i];
    acc ^= v[0] ^ v[3];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

constexpr int kGemvMaxLds = 163840 - 1024;  // dynamic LDS opt-in (the static `red` stays below)
int g_gemv_wgs = 0;  // target workgroup count (0: the default below)
int g_gemv_ksplit = 1;  // two waves per pair on the long-K projections (ops.GEMV_KSPLIT)

template <int MR, int PRO, int MODE>
int launch_u(const GemvArgs& a, int U, hipStream_t st) {
  constexpr bool NORM = PRO == 1;
  int target = g_gemv_wgs > 0 ? g_gemv_wgs : 512;
  int wgs = (a.npairs + 3) / 4;
  if (wgs > target) wgs = target;
  const size_t lds = (size_t)(MR + (NORM ? 1 : 0)) * a.K * 2;  // X rows (+ gamma)
  if (lds > kGemvMaxLds) return -3;
  // two waves per pair (a K half each) where a pair's K walk is an even number >= 2 of U-blocks
  const int blocks = a.K / 512 / U;
  const bool ks2 = g_gemv_ksplit && blocks >= 2 && blocks % 2 == 0;
  if (ks2) {
    wgs = (a.npairs + 1) / 2;
    if (wgs > 2 * target) wgs = 2 * target;
  }
#define LK_GEMV_U(UU)                                                                  \
  if (U == UU) {                                                                       \
    if (ks2) {                                                                         \
      LK_SET_MAX_LDS((gemv_decode_kernel<MR, PRO, MODE, UU, 2>), kGemvMaxLds);        \
      gemv_decode_kernel<MR, PRO, MODE, UU, 2><<<wgs, 256, lds, st>>>(a);             \
    } else {                                                                           \
      LK_SET_MAX_LDS((gemv_decode_kernel<MR, PRO, MODE, UU, 1>), kGemvMaxLds);        \
      gemv_decode_kernel<MR, PRO, MODE, UU, 1><<<wgs, 256, lds, st>>>(a);             \
    }                                                                                  \
  } else
  LK_GEMV_U(8) LK_GEMV_U(7) LK_GEMV_U(4) return -4;
#undef LK_GEMV_U
  LK_CHECK_LAUNCH();
  return 0;
}

int pick_u(int K) {
  const int kc = K / 512;
  if (kc % 8 == 0) return 8;
  if (kc % 7 == 0) return 7;
  if (kc % 4 == 0) return 4;
  return 0;
}

template <int PRO, int MODE>
int launch_m(const GemvArgs& a, hipStream_t st) {
  const int U = pick_u(a.K);
  if (!U || a.K % 512) return -2;
  if (a.M == 1) return launch_u<1, PRO, MODE>(a, U, st);
  if (a.M == 2) return launch_u<2, PRO, MODE>(a, U, st);
  return -2;
}

}  // namespace

int lk_gemv_supported(int M, int N, int K, int mode) {
  // (K <= 16384: the prologue's SCH = 8 staging chunks per thread)
  // (X rows and, for the RMSNorm prologue, gamma in LDS)
  if (M < 1 || M > 2 || K % 512 || !pick_u(K) || (long)(M + 1) * K * 2 > kGemvMaxLds) return 0;
  if (mode == 2) return N % 2 == 0;
  return N % 2 == 0;
}

void lk_gemv_set_wgs(int wgs) { g_gemv_wgs = wgs; }

int lk_l3_prefetch(const void* p, long bytes, int wgs, unsigned* sink, hipStream_t st) {
  if (!p || bytes < 16 || ((uintptr_t)p & 15) || !sink || wgs < 1) return bytes < 16 ? 0 : -1;
  l3_prefetch_kernel<<<wgs, 256, 0, st>>>(reinterpret_cast<const uint4_t*>(p), bytes / 16, sink);
  LK_CHECK_LAUNCH();
  return 0;
}
void lk_gemv_set_ksplit(int on) { g_gemv_ksplit = on ? 1 : 0; }

int lk_gemv_decode(int mode, const bf16_t* x, long ldx, const bf16_t* gamma, float eps, const bf16_t* w, int M, int N,
                   int K, bf16_t* out, long ldo, bf16_t* res, long ldr, const int* positions, const float* cos_sin,
                   int Hq, int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                   const float* po, const float* pml, const int* ctx, int max_splits, int split, hipStream_t st) {
  if (!lk_gemv_supported(M, N, K, mode) || !x || !w || ldx % 8) return -1;
  GemvArgs a;
  a.x = x;
  a.ldx = ldx;
  a.gamma = gamma;
  a.eps = eps;
  a.w = w;
  a.M = M;
  a.N = N;
  a.K = K;
  a.out = out;
  a.ldo = ldo;
  a.res = res;
  a.ldr = ldr;
  switch (mode) {
    case 0:
      if (!out) return -1;
      a.npairs = N / 2;
      break;
    case 1:
      if (!res || ldr % 2) return -1;
      a.npairs = N / 2;
      break;
    case 2:
      if (!out) return -1;
      a.I = N / 2;
      a.npairs = N / 2;
      break;
    case 3:
      if (!out || !positions || !cos_sin || D % 2 || D <= 0 || N != (Hq + 2 * Hkv) * D || (kc && BS <= 0))
        return -1;
      a.positions = positions;
      a.cos_sin = cos_sin;
      a.Hq = Hq;
      a.Hkv = Hkv;
      a.D = D;
      a.BS = BS;
      a.neox = neox;
      a.kc = kc;
      a.vc = vc;
      a.slots = slots;
      a.npairs = N / 2;
      break;
    default:
      return -1;
  }
  const bool norm = gamma != nullptr;
  if (po) {  // the split merge prologue: the O projection (mode 1) only, no norm
    if (mode != 1 || norm || !pml || !ctx || Hq <= 0 || D <= 0 || D % 8 || Hq * D != K || max_splits < 1 ||
        split < 1)
      return -1;
    a.po = po;
    a.pml = pml;
    a.ctx = ctx;
    a.Hq = Hq;
    a.D = D;
    a.max_splits = max_splits;
    a.split = split;
    return launch_m<2, 1>(a, st);
  }
#define LK_GEMV_MODE(MD)                                             \
  if (mode == MD) return norm ? launch_m<1, MD>(a, st) : launch_m<0, MD>(a, st);
  LK_GEMV_MODE(0) LK_GEMV_MODE(1) LK_GEMV_MODE(2) LK_GEMV_MODE(3)
#undef LK_GEMV_MODE
  return -1;
}
