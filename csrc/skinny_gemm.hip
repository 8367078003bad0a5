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
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int kSkW = 4;  // waves per block

LK_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }
LK_DEVICE float rbf(float x) { return bf2f(f2bf(x)); }

constexpr int kSysCoherent = 1 | 16;  // buffer cache policy sc0 | sc1: past L1 and L2

// Fused split-K tail of the weight-streaming GEMM (kind != 0).  Every split workgroup writes its
// f32 partial through to memory and takes a ticket; the LAST one to finish reduces the slabs
// itself, so no reduce kernel is launched after the GEMM (at decode sizes a reduce launch is a
// ~5 us step of the critical path per projection):
//   kind 1: RoPE + paged-KV write, one ticket per column tile = one head (BN == D): the qkv rows
//           exactly as lk_splitk_rope_kv leaves them (q rotated, k rotated in the cache and in
//           the row only with write_k_inplace, v copied);
//   kind 2: residual add + RMSNorm, one ticket for the whole grid (few rows: the last workgroup
//           normalises every row), exactly as lk_splitk_rmsnorm.
// Tickets are zero-initialised int32 counters reset by their last taker.
struct WsTail {
  int kind = 0;
  int* tickets = nullptr;
  bf16_t* out = nullptr;  // 1: qkv rows; 2: normed rows
  long os = 0;
  const int* positions = nullptr;
  const float* cos_sin = nullptr;
  int Hq = 0, Hkv = 0, D = 0;
  bf16_t* kc = nullptr;
  bf16_t* vc = nullptr;
  const int* slots = nullptr;
  int BS = 1, neox = 0, write_k_inplace = 0;
  bf16_t* residual = nullptr;
  long rs = 0;
  const bf16_t* norm_w = nullptr;
  float eps = 0.f;
};

// Consumer-side prologue of the weight-streaming GEMM (kind != 0, <= 64 rows): before its K walk
// every workgroup computes the X rows of its K slice itself and stages them from the scratch
// rows `x` it wrote, so the launch that would have produced X disappears from the decode step
// (its W prefetch is issued before the prologue and flies under it):
//   kind 1: x = RMSNorm(bf16(sum of the producer's split-K slabs) + res) * gamma -- exactly the
//           rmsnorm_kernel<_, 4, S> arithmetic (256 threads slicing the row the same way, same
//           block_sum), so the values are bit-identical to lk_splitk_rmsnorm; workgroup 0 also
//           writes the summed residual row(s) to res_out (a buffer other than res: the other
//           workgroups still read res);
//   kind 2: the flash-decoding merge of a split-K paged-decode step's partials, exactly as
//           decode_reduce_kernel, for the rows with more than one split (the others the
//           attention kernel wrote into x itself).
struct WsPro {
  int kind = 0;
  bf16_t* x = nullptr;  // [M, K] scratch rows (row stride K): written here, then staged as X
  const float* part = nullptr;  // 1: producer slabs [S][M][K]
  int S = 0;
  long slab = 0;
  const bf16_t* res = nullptr;
  bf16_t* res_out = nullptr;
  long rs = 0;  // row stride of res and res_out
  const bf16_t* gamma = nullptr;
  float eps = 0.f;
  const float* po = nullptr;   // 2: [(row * Hq + qh) * max_splits + s][D]
  const float* pml = nullptr;  // 2: [(row * Hq + qh) * max_splits + s][2]
  const int* ctx = nullptr;
  int Hq = 0, D = 0, max_splits = 0, split = 0;
};

template <int KIND>
LK_DEVICE void ws_prologue(const WsPro& pr, int M, int K, long kbase, int ks) {
  if constexpr (KIND == 1) {
    __shared__ float red[4];
    const int nvec = K >> 3;
    for (int m = 0; m < M; ++m) {
      float v[4][8];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = threadIdx.x + i * 256;
        if (c < nvec) {
          const float* pp = pr.part + (long)m * K + c * 8;
          floatx4 a = *reinterpret_cast<const floatx4*>(pp), b = *reinterpret_cast<const floatx4*>(pp + 4);
          for (int q = 1; q < pr.S; ++q) {
            a += *reinterpret_cast<const floatx4*>(pp + q * pr.slab);
            b += *reinterpret_cast<const floatx4*>(pp + q * pr.slab + 4);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[i][j] = bf2f(f2bf(a[j]));
            v[i][j + 4] = bf2f(f2bf(b[j]));
          }
          float r[8];
          load8(pr.res + (long)m * pr.rs + c * 8, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + r[j]));
          if (blockIdx.x == 0) store8(pr.res_out + (long)m * pr.rs + c * 8, v[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
        }
      }
      ss = block_sum<4>(ss, red);
      const float inv = rsqrtf(ss / (float)K + pr.eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = threadIdx.x + i * 256;
        if (c < nvec && c * 8 >= kbase && c * 8 < kbase + ks) {
          float g[8], y[8];
          load8(pr.gamma + c * 8, g);
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(v[i][j] * inv)) * g[j];
          store8(pr.x + (long)m * K + c * 8, y);
        }
      }
    }
  } else if constexpr (KIND == 2) {
    for (int m = 0; m < M; ++m) {
      const int nsplit = max(0, min((pr.ctx[m] + pr.split - 1) / pr.split, pr.max_splits));
      if (nsplit <= 1) continue;  // (uniform) the attention kernel wrote this row into x
      for (int e = threadIdx.x; e < ks; e += 256) {
        const long col = kbase + e;
        const int qh = (int)(col / pr.D), d = (int)(col - (long)qh * pr.D);
        const long base = ((long)m * pr.Hq + qh) * pr.max_splits;
        float Mx = -INFINITY;
        for (int q = 0; q < nsplit; ++q) Mx = fmaxf(Mx, pr.pml[(base + q) * 2]);
        if (Mx == -INFINITY) Mx = 0.f;
        float den = 0.f, num = 0.f;
        for (int q = 0; q < nsplit; ++q) {
          const float f = exp2f(pr.pml[(base + q) * 2] - Mx);
          den += f * pr.pml[(base + q) * 2 + 1];
          num += f * pr.po[(base + q) * pr.D + d];
        }
        pr.x[(long)m * K + col] = f2bf(den > 0.f ? num / den : 0.f);
      }
    }
  }
}

// 8 consecutive columns of one row: the S slabs summed in slab order, rounded to bf16 (the values
// the unfused reduce stores); partials read past L1 / L2 (other workgroups wrote them through)
LK_DEVICE void tail_ld8(__amdgpu_buffer_rsrc_t prs, int S, long slab, long off, float* f) {
  floatx4 a = floatx4{0.f, 0.f, 0.f, 0.f}, b = a;
  for (int q0 = 0; q0 < S; q0 += 4) {  // 4 slabs in flight at a time (registers: the tail shares the kernel's)
    floatx4 pa[4], pb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q0 + q < S) {
        const unsigned o = (unsigned)((off + (q0 + q) * slab) * 4);
        pa[q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(prs, o, 0, kSysCoherent));
        pb[q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(prs, o + 16, 0, kSysCoherent));
      }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q0 + q < S) {
        a += pa[q];
        b += pb[q];
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = bf2f(f2bf(a[j]));
    f[j + 4] = bf2f(f2bf(b[j]));
  }
}

// kind 1: head = column tile t of the fused [(Hq + 2 Hkv) * D] projection, all M rows
LK_DEVICE void tail_rope_kv(const WsTail& tl, __amdgpu_buffer_rsrc_t prs, int S, int M, long ld, int head) {
  const int D = tl.D, half = D >> 1;
  const long slab = (long)M * ld;
  const bool rot = head < tl.Hq + tl.Hkv;
  const int ipr = rot ? (tl.neox ? (D >> 4) : (D >> 3)) : (D >> 3);
  const bool is_k = head >= tl.Hq && rot;
  const bool store_src = !is_k || tl.write_k_inplace;
  for (int it = threadIdx.x; it < M * ipr; it += blockDim.x) {
    const int row = it / ipr, v = it - row * ipr;
    bf16_t* hp = tl.out + (long)row * tl.os + (long)head * D;
    const long pbase = (long)row * ld + (long)head * D;
    const int slot = tl.slots ? tl.slots[row] : -1;
    const long blk = slot >= 0 ? slot / tl.BS : 0;
    const int off = slot >= 0 ? slot % tl.BS : 0;
    if (!rot) {  // V: copy into the row and the cache
      const int c = v * 8, h = head - tl.Hq - tl.Hkv;
      float f[8];
      tail_ld8(prs, S, slab, pbase + c, f);
      store8(hp + c, f);
      if (tl.vc && slot >= 0) store8(tl.vc + ((blk * tl.Hkv + h) * tl.BS + off) * D + c, f);
      continue;
    }
    const float* cs = tl.cos_sin + (long)tl.positions[row] * D;  // [cos(D/2) | sin(D/2)]
    bf16_t* kdst = (is_k && tl.kc && slot >= 0) ? tl.kc + ((blk * tl.Hkv + (head - tl.Hq)) * tl.BS + off) * D : nullptr;
    if (tl.neox) {
      const int i0 = v * 8;
      float x1[8], x2[8], y1[8], y2[8];
      tail_ld8(prs, S, slab, pbase + i0, x1);
      tail_ld8(prs, S, slab, pbase + half + i0, x2);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cs[i0 + j], sn = cs[half + i0 + j];
        y1[j] = x1[j] * c - x2[j] * sn;
        y2[j] = x2[j] * c + x1[j] * sn;
      }
      store8(hp + i0, store_src ? y1 : x1);
      store8(hp + half + i0, store_src ? y2 : x2);
      if (kdst) {
        store8(kdst + i0, y1);
        store8(kdst + half + i0, y2);
      }
    } else {
      const int e0 = v * 8;  // elements e0..e0+7 = pairs e0/2 .. e0/2+3
      float x[8], y[8];
      tail_ld8(prs, S, slab, pbase + e0, x);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float c = cs[(e0 >> 1) + p], sn = cs[half + (e0 >> 1) + p];
        y[2 * p] = x[2 * p] * c - x[2 * p + 1] * sn;
        y[2 * p + 1] = x[2 * p + 1] * c + x[2 * p] * sn;
      }
      store8(hp + e0, store_src ? y : x);
      if (kdst) store8(kdst + e0, y);
    }
  }
}

// kind 2: rows 0..M-1 of N = ld columns: residual += bf16(sum of slabs); out = RMSNorm(residual) * w
LK_DEVICE void tail_rmsnorm(const WsTail& tl, __amdgpu_buffer_rsrc_t prs, int S, int M, long ld, float* red) {
  const int nvec = (int)(ld >> 3);
  const long slab = (long)M * ld;
  const int nw = blockDim.x >> 6, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int row = 0; row < M; ++row) {
    float ss = 0.f;
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      float v[8], r[8];
      tail_ld8(prs, S, slab, (long)row * ld + c * 8, v);
      bf16_t* rr = tl.residual + (long)row * tl.rs + c * 8;
      load8(rr, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = bf2f(f2bf(v[j] + r[j]));  // the new residual stream: the bf16-rounded sum
        ss += v[j] * v[j];
      }
      store8(rr, v);
    }
    ss = wave_sum(ss);
    __syncthreads();  // (the previous row's reads of red are done)
    if (lane == 0) red[wv] = ss;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < nw; ++i) tot += red[i];
    const float inv = rsqrtf(tot / (float)ld + tl.eps);
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      float v[8], g[8], y[8];
      load8(tl.residual + (long)row * tl.rs + c * 8, v);  // (this thread's own stores above)
      load8(tl.norm_w + c * 8, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = v[j] * inv * g[j];
      store8(tl.out + (long)row * tl.os + c * 8, y);
    }
  }
}

// after the epilogue, by ALL threads of the workgroup (uniform control flow: it has barriers).
// lds: the kernel's dynamic LDS, dead once the K loop is done (no static LDS here: the ring
// already fills the 160 KB)
__attribute__((noinline)) __device__ void ws_tail(const WsTail& tl, float* part, int M, long ld, int S, int t, int n_tiles, unsigned char* lds) {
  int* is_last = reinterpret_cast<int*>(lds);
  float* red = reinterpret_cast<float*>(lds + 64);
  __builtin_amdgcn_s_waitcnt(0);  // this thread's write-through partial stores acknowledged
  __syncthreads();                // (and every wave is done with the LDS ring)
  if (threadIdx.x == 0) {
    int* tk = tl.tickets + (tl.kind == 1 ? t : 0);
    const int need = tl.kind == 1 ? S : S * n_tiles;
    const int old = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int last = old == need - 1;
    if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *is_last = last;
  }
  __syncthreads();
  if (!*is_last) return;
  const long bytes = (long)S * M * ld * 4;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)part, (short)0, (int)min(bytes, 0x7FFFFFF0L), 0x00020000);
  if (tl.kind == 1) tail_rope_kv(tl, prs, S, M, ld, t);
  else tail_rmsnorm(tl, prs, S, M, ld, red);
}

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

// ---------------------------------------------------------------------------------
// Weight-streaming GEMM for 64 < M <= 256 rows ("wsgemm").  The fragment-shaped loads
// of skinny_gemm_kernel touch 16 rows x 64 B per wave instruction, which caps the
// per-CU load rate once X (re-read by every column block) grows with M.  Here both
// operands are staged through LDS with 16-B global_load_lds (LDS-DMA): every wave
// instruction moves 8 rows x one full 128-B line, lane-linear into LDS, with the
// (row>>1)&7 XOR chunk swizzle applied on the SOURCE address so the MFMA fragment
// reads (ds_read_b128, 16 rows x 16 B per lane group) are bank-conflict free.
//   * block = 4 waves, tile = all M rows (16*MT) x BN columns, BK = 64 per stage,
//     3-stage LDS ring, ONE raw s_barrier per stage, counted vmcnt (the DMA of the
//     next stage stays in flight across the barrier and under the MFMAs);
//   * waves split M (each 4*MT rows x BN columns: acc = MT/4 x BN/16 tiles);
//   * W rows are streamed once with the non-temporal policy (aux = 2);
//   * split-K over blocks (S) when N/BN leaves CUs idle; partial slabs -> the same
//     reduce / SwiGLU kernel as skinny_gemm; S = 1 writes bf16 (or SwiGLU) directly.
template <int N>
LK_DEVICE void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* gbl_void_ptr;

LK_DEVICE int wsz(int row) { return (row >> 1) & 7; }

// ring depth: the in-flight DMA bytes per CU set the per-CU load rate (latency-bound
// at one block per CU), so fill the 160 KB LDS
constexpr int ws_stages(int MT, int BN) {
  const int sb = (16 * MT + BN) * 128;
  const int n = 163840 / sb;
  return n > 8 ? 8 : (n < 3 ? 3 : n);
}

template <int L, int NS>
LK_DEVICE void wait_ahead(int ahead) {  // vmcnt(ahead * L), ahead in [0, NS-2]
  if constexpr (NS > 2) {
    if (ahead >= NS - 2) {
      wait_vmcnt<L * (NS - 2)>();
      return;
    }
    wait_ahead<L, NS - 1>(ahead);
  } else {
    wait_vmcnt<0>();
  }
}

// (PRO: a WsPro prologue computes X first -- the LDS ring leaves room for its static scratch)
constexpr int ws_stages_pro(int MT, int BN, int PRO) {
  const int sb = (16 * MT + BN) * 128;
  const int n = (163840 - (PRO ? 1024 : 0)) / sb;
  return n > 8 ? 8 : (n < 3 ? 3 : n);
}

template <int MT, int BN, bool SWIGLU, bool TAIL, int PRO = 0>
__global__ __launch_bounds__(256, 1) void wsgemm_kernel(const bf16_t* __restrict__ X, long ldx,
                                                        const bf16_t* __restrict__ W, int M, int K, int ks,
                                                        int n_tiles, int swiglu_I, bf16_t* __restrict__ out,
                                                        long ldo, float* __restrict__ part, long part_ld,
                                                        long n_rows, int rot_mul, WsTail tl, WsPro pr) {
  // n_rows: valid W rows (the last column tile may be partial: kNN over a corpus of
  // any size); loads clamp to the last row, stores are masked
  constexpr int ROWS = 16 * MT;          // padded M
  constexpr int MTW = MT / 4;            // row tiles per wave
  constexpr int NT = BN / 16;            // column tiles per wave
  constexpr int XB = ROWS * 128;         // X stage bytes
  constexpr int WB = BN * 128;           // W stage bytes
  constexpr int SB = XB + WB;            // stage bytes
  constexpr int NS = ws_stages_pro(MT, BN, PRO);  // ring depth: as many stages as 160 KB of LDS holds
  constexpr int LX = ROWS / 32;          // X glds per wave per stage (8 rows each, 4 waves)
  constexpr int LW = BN / 32;            // W glds per wave per stage
  constexpr int L = LX + LW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int t = blockIdx.x % n_tiles, s = blockIdx.x / n_tiles;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const long kbase = (long)s * ks;
  const int nst = ks / 64;
  // K-step rotation: column tile t starts its K walk at step (t * rot_mul) % nst, so the
  // blocks streaming at the same moment read different 128-B columns of X (every block
  // reads all of X: in lockstep they would all hit the same few L2 channels)
  const int rot = rot_mul ? (int)(((long)t * rot_mul) % nst) : 0;

  auto wrow = [&](int row) -> long {  // tile row -> global W row (output column)
    if constexpr (SWIGLU) {
      return row < BN / 2 ? (long)t * (BN / 2) + row : (long)swiglu_I + (long)t * (BN / 2) + row - BN / 2;
    } else {
      return (long)t * BN + row;
    }
  };

  // per-lane source pointers of this wave's glds instructions (k offset added per stage)
  const bf16_t* xsrc[LX];
  const bf16_t* wsrc[LW];
  const int lrow = lane >> 3, lch = lane & 7;
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (w * LX + i) * 8 + lrow;
    xsrc[i] = X + (long)min(row, M - 1) * ldx + kbase + ((lch ^ wsz(row)) * 8);
  }
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int row = (w * LW + i) * 8 + lrow;
    wsrc[i] = W + min(wrow(row), n_rows - 1) * K + kbase + ((lch ^ wsz(row)) * 8);
  }
  auto issue_x = [&](int st) {
    unsigned char* base = smem + (st % NS) * SB;
    const int k = (st + rot < nst ? st + rot : st + rot - nst) * 64;
#pragma unroll
    for (int i = 0; i < LX; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(xsrc[i] + k),
                                       (lds_void_ptr)(base + (w * LX + i) * 8 * 128), 16, 0, 0);
  };
  auto issue_w = [&](int st) {
    unsigned char* base = smem + (st % NS) * SB;
    const int k = (st + rot < nst ? st + rot : st + rot - nst) * 64;
#pragma unroll
    for (int i = 0; i < LW; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(wsrc[i] + k),
                                       (lds_void_ptr)(base + XB + (w * LW + i) * 8 * 128), 16, 0, 2);
  };
  auto issue = [&](int st) {
    issue_x(st);
    issue_w(st);
  };

  floatx4 acc[MTW][NT];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int st) {
    const unsigned char* base = smem + (st % NS) * SB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + g;
      short8 a[MTW], b[NT];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const int row = w * (4 * MT) + 16 * m + r;
        a[m] = *reinterpret_cast<const short8*>(base + row * 128 + ((c ^ wsz(row)) << 4));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int row = 16 * n + r;
        b[n] = *reinterpret_cast<const short8*>(base + XB + row * 128 + ((c ^ wsz(row)) << 4));
      }
      // W fragment as the MFMA's A operand: the lane ends with ONE output row and 4
      // consecutive columns, so the epilogue writes 16 B (f32 partials) / 8 B (bf16) per lane
      // -- a quarter of the store instructions of a column-per-lane image (the store tail
      // of a short weight-streaming kernel is issue-bound)
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[n], a[m], acc[m][n], 0, 0, 0);
    }
  };

  if constexpr (PRO != 0) {
    // W of the first stages streams in while the workgroup computes its X slice; then X's
    // first stages come from the rows just written (every wave waits for its own DMAs, the
    // loop's barrier for everyone's)
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < nst) issue_w(p);
    ws_prologue<PRO>(pr, M, K, kbase, ks);
    wait_vmcnt<0>();
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < nst) issue_x(p);
    wait_vmcnt<0>();
  } else {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < nst) issue(p);
  }
  for (int st = 0; st < nst; ++st) {
    // stage st landed (this wave's DMAs); later stages may stay in flight
    wait_ahead<L, NS>(min(NS - 2, nst - 1 - st));
    __builtin_amdgcn_s_barrier();  // ... for every wave; and buffer (st-1)%NS is free
    __builtin_amdgcn_sched_barrier(0);
    if (st + NS - 1 < nst) issue(st + NS - 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(st);
  }

  // ---- epilogue straight from the accumulators: lane holds row 16m + r of its wave's rows,
  // tile columns 16n + 4g .. +3
  const bool split = part != nullptr;
  const bool part_vec = split && part_ld % 4 == 0 && reinterpret_cast<uintptr_t>(part) % 16 == 0;
  // (fused tail: the partial slabs through a buffer resource, written past L1 / L2)
  const __amdgpu_buffer_rsrc_t tprs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)part, (short)0, (int)min((long)(K / ks) * M * part_ld * 4, 0x7FFFFFF0L), 0x00020000);
  const bool out_vec = ldo % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 8 == 0;
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    const int row = w * (4 * MT) + 16 * m + r;
    if (row >= M) continue;
    if (SWIGLU && !split) {
#pragma unroll
      for (int n = 0; n < NT / 2; ++n) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = rbf(silu_f(rbf(acc[m][n][i]))) * rbf(acc[m][n + NT / 2][i]);
        bf16_t* dst = out + (long)row * ldo + (long)t * (BN / 2) + 16 * n + 4 * g;
        if (out_vec) {
          uint2 pk;
          pk.x = pack_bf2(y[0], y[1]);
          pk.y = pack_bf2(y[2], y[3]);
          *reinterpret_cast<uint2*>(dst) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) dst[i] = f2bf(y[i]);
        }
      }
    } else if (split) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        // 4 consecutive tile rows stay inside one half of a SwiGLU tile: contiguous W rows
        const long col = wrow(16 * n + 4 * g);
        float* dst = part + (long)s * M * part_ld + (long)row * part_ld + col;
        if (TAIL) {  // fused tail: through to memory (full 16-B tiles: checked on the host)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, acc[m][n]), tprs,
                                                 (unsigned)(((long)s * M + row) * part_ld + col) * 4u, 0, kSysCoherent);
        } else if (part_vec && col + 3 < n_rows) {
          *reinterpret_cast<floatx4*>(dst) = acc[m][n];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (col + i < n_rows) dst[i] = acc[m][n][i];
        }
      }
    } else {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const long col = (long)t * BN + 16 * n + 4 * g;
        bf16_t* dst = out + (long)row * ldo + col;
        if (out_vec && col + 3 < n_rows) {
          uint2 pk;
          pk.x = pack_bf2(acc[m][n][0], acc[m][n][1]);
          pk.y = pack_bf2(acc[m][n][2], acc[m][n][3]);
          *reinterpret_cast<uint2*>(dst) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (col + i < n_rows) dst[i] = f2bf(acc[m][n][i]);
        }
      }
    }
  }
  if constexpr (TAIL) ws_tail(tl, part, M, part_ld, K / ks, t, n_tiles, smem);
}

// ---------------------------------------------------------------------------------
// Loader-wave variant of the weight-streaming GEMM ("lw").  s_waitcnt vmcnt retires a wave's
// vector-memory ops in issue order, so in wsgemm_kernel -- X and W of a stage issued together by
// the same waves -- the W prefetch can run only as far ahead as the shared ring, and at M 192-256
// (X stages twice the W stages) that is 1-2 stages: the W stream ran 3.0-3.9 TB/s, in proportion
// to the W bytes in flight per CU.  Here the W stream has waves of its own (2 loader waves, their
// own vmcnt): 4 compute waves stage X through a short ring (L2-resident, 2-3 stages) and compute;
// the loader waves keep NSW - 1 W stages (all the remaining LDS) in flight; one s_barrier per
// stage joins them.  Same tile, swizzles, K rotation and epilogue as wsgemm_kernel.
constexpr int lw_nsx(int MT) { return MT <= 8 ? 3 : 2; }
constexpr int lw_nsw(int MT, int BN) {
  const int n = (163840 - lw_nsx(MT) * 16 * MT * 128) / (BN * 128);
  return n > 12 ? 12 : n;
}

template <int MT, int BN, bool SWIGLU, bool TAIL>
__global__ __launch_bounds__(384, 1) void wsgemm_lw_kernel(const bf16_t* __restrict__ X, long ldx,
                                                           const bf16_t* __restrict__ W, int M, int K, int ks,
                                                           int n_tiles, int swiglu_I, bf16_t* __restrict__ out,
                                                           long ldo, float* __restrict__ part, long part_ld,
                                                           long n_rows, int rot_mul, WsTail tl) {
  constexpr int ROWS = 16 * MT;
  constexpr int MTW = MT / 4;
  constexpr int NT = BN / 16;
  constexpr int XB = ROWS * 128;
  constexpr int WB = BN * 128;
  constexpr int NSX = lw_nsx(MT);
  constexpr int NSW = lw_nsw(MT, BN);
  constexpr int LX = ROWS / 32;  // X glds per compute wave per stage (4 waves x 8 rows)
  constexpr int LW = BN / 16;    // W glds per loader wave per stage (2 waves x 8 rows)
  static_assert(NSW >= 3, "W ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xring = smem;
  unsigned char* wring = smem + NSX * XB;

  const int t = blockIdx.x % n_tiles, s = blockIdx.x / n_tiles;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = w >= 4;
  const int r = lane & 15, g = lane >> 4;
  const long kbase = (long)s * ks;
  const int nst = ks / 64;
  const int rot = rot_mul ? (int)(((long)t * rot_mul) % nst) : 0;
  auto kof = [&](int st) { return (st + rot < nst ? st + rot : st + rot - nst) * 64; };

  auto wrow = [&](int row) -> long {
    if constexpr (SWIGLU) {
      return row < BN / 2 ? (long)t * (BN / 2) + row : (long)swiglu_I + (long)t * (BN / 2) + row - BN / 2;
    } else {
      return (long)t * BN + row;
    }
  };
  const int lrow = lane >> 3, lch = lane & 7;

  floatx4 acc[MTW][NT];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (loader) {
    const int lw = w - 4;
    const bf16_t* wsrc[LW];
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int row = (lw * LW + i) * 8 + lrow;
      wsrc[i] = W + min(wrow(row), n_rows - 1) * K + kbase + ((lch ^ wsz(row)) * 8);
    }
    auto issue_w = [&](int st) {
      unsigned char* base = wring + (st % NSW) * WB;
#pragma unroll
      for (int i = 0; i < LW; ++i)
        __builtin_amdgcn_global_load_lds((gbl_void_ptr)(wsrc[i] + kof(st)),
                                         (lds_void_ptr)(base + (lw * LW + i) * 8 * 128), 16, 0, 2);
    };
#pragma unroll
    for (int p = 0; p < NSW - 1; ++p)
      if (p < nst) issue_w(p);
    for (int st = 0; st < nst; ++st) {
      wait_ahead<LW, NSW>(min(NSW - 2, nst - 1 - st));  // W(st) landed, later stages in flight
      __builtin_amdgcn_s_barrier();                      // ... and ring slot (st - 1) % NSW is free
      __builtin_amdgcn_sched_barrier(0);
      if (st + NSW - 1 < nst) issue_w(st + NSW - 1);
    }
    // the epilogue is the compute waves' (no barrier after the loop); a fused tail needs
    // every wave again
  } else {

  const bf16_t* xsrc[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (w * LX + i) * 8 + lrow;
    xsrc[i] = X + (long)min(row, M - 1) * ldx + kbase + ((lch ^ wsz(row)) * 8);
  }
  auto issue_x = [&](int st) {
    unsigned char* base = xring + (st % NSX) * XB;
#pragma unroll
    for (int i = 0; i < LX; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(xsrc[i] + kof(st)),
                                       (lds_void_ptr)(base + (w * LX + i) * 8 * 128), 16, 0, 0);
  };
  auto compute = [&](int st) {
    const unsigned char* xb = xring + (st % NSX) * XB;
    const unsigned char* wb = wring + (st % NSW) * WB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + g;
      short8 a[MTW], b[NT];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const int row = w * (4 * MT) + 16 * m + r;
        a[m] = *reinterpret_cast<const short8*>(xb + row * 128 + ((c ^ wsz(row)) << 4));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int row = 16 * n + r;
        b[n] = *reinterpret_cast<const short8*>(wb + row * 128 + ((c ^ wsz(row)) << 4));
      }
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[n], a[m], acc[m][n], 0, 0, 0);
    }
  };
#pragma unroll
  for (int p = 0; p < NSX - 1; ++p)
    if (p < nst) issue_x(p);
  for (int st = 0; st < nst; ++st) {
    wait_ahead<LX, NSX>(min(NSX - 2, nst - 1 - st));  // X(st) landed (the W side waits in the loaders)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (st + NSX - 1 < nst) issue_x(st + NSX - 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(st);
  }

  // ---- epilogue (as wsgemm_kernel): lane holds row 16m + r of its wave's rows, tile columns
  // 16n + 4g .. +3
  const bool split = part != nullptr;
  const bool part_vec = split && part_ld % 4 == 0 && reinterpret_cast<uintptr_t>(part) % 16 == 0;
  // (fused tail: the partial slabs through a buffer resource, written past L1 / L2)
  const __amdgpu_buffer_rsrc_t tprs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)part, (short)0, (int)min((long)(K / ks) * M * part_ld * 4, 0x7FFFFFF0L), 0x00020000);
  const bool out_vec = ldo % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 8 == 0;
#pragma unroll
  for (int m = 0; m < MTW; ++m) {
    const int row = w * (4 * MT) + 16 * m + r;
    if (row >= M) continue;
    if (SWIGLU && !split) {
#pragma unroll
      for (int n = 0; n < NT / 2; ++n) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = rbf(silu_f(rbf(acc[m][n][i]))) * rbf(acc[m][n + NT / 2][i]);
        bf16_t* dst = out + (long)row * ldo + (long)t * (BN / 2) + 16 * n + 4 * g;
        if (out_vec) {
          uint2 pk;
          pk.x = pack_bf2(y[0], y[1]);
          pk.y = pack_bf2(y[2], y[3]);
          *reinterpret_cast<uint2*>(dst) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) dst[i] = f2bf(y[i]);
        }
      }
    } else if (split) {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const long col = wrow(16 * n + 4 * g);
        float* dst = part + (long)s * M * part_ld + (long)row * part_ld + col;
        if (TAIL) {  // fused tail: through to memory
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, acc[m][n]), tprs,
                                                 (unsigned)(((long)s * M + row) * part_ld + col) * 4u, 0, kSysCoherent);
        } else if (part_vec && col + 3 < n_rows) {
          *reinterpret_cast<floatx4*>(dst) = acc[m][n];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (col + i < n_rows) dst[i] = acc[m][n][i];
        }
      }
    } else {
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const long col = (long)t * BN + 16 * n + 4 * g;
        bf16_t* dst = out + (long)row * ldo + col;
        if (out_vec && col + 3 < n_rows) {
          uint2 pk;
          pk.x = pack_bf2(acc[m][n][0], acc[m][n][1]);
          pk.y = pack_bf2(acc[m][n][2], acc[m][n][3]);
          *reinterpret_cast<uint2*>(dst) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (col + i < n_rows) dst[i] = f2bf(acc[m][n][i]);
        }
      }
    }
  }
  }  // (compute waves)
  if constexpr (TAIL) ws_tail(tl, part, M, part_ld, K / ks, t, n_tiles, smem);  // every wave: it has barriers
}

// K-step rotation multiplier: -1 = policy (5 for unsplit-K grids -- the long-K gate_up
// + SwiGLU and LM-head shapes, 4-8 % faster on MI355X; off for split-K grids, where it
// measured neutral to 30 % slower: benchmarks/ws_rot_probe.py), >= 0 forces it
int g_ws_rot_mul = -1;

template <int MT, int BN, bool SWIGLU>
void launch_ws(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S, int n_tiles, int I,
               bf16_t* out, long ldo, float* part, long part_ld, long n_rows, hipStream_t st, const WsTail& tl) {
  constexpr size_t lds = (size_t)ws_stages(MT, BN) * (16 * MT * 128 + BN * 128);
  // (the fused-tail instantiation only where a tail runs: the plain kernel keeps its registers)
  auto kern = tl.kind ? wsgemm_kernel<MT, BN, SWIGLU, true> : wsgemm_kernel<MT, BN, SWIGLU, false>;
  if (tl.kind) LK_SET_MAX_LDS((wsgemm_kernel<MT, BN, SWIGLU, true>), (int)lds);
  else LK_SET_MAX_LDS((wsgemm_kernel<MT, BN, SWIGLU, false>), (int)lds);
  // kNN scores (n_rows given: a corpus, not a weight) walk K in one order in every tile, so
  // equal corpus rows score bit-identically and ties keep the stable id order
  const int rot_mul = n_rows < (1L << 40) ? 0 : g_ws_rot_mul >= 0 ? g_ws_rot_mul : (S == 1 ? 5 : 0);
  kern<<<n_tiles * S, 256, lds, st>>>(x, ldx, w, M, K, ks, n_tiles, I, out, ldo, part, part_ld, n_rows, rot_mul, tl,
                                      WsPro{});
}

// the prologue instantiations (one LDS ring, 16-row tiles: M <= 64)
template <int BN, bool SWIGLU, int PRO>
void launch_ws_pro(const bf16_t* x, const bf16_t* w, int M, int K, int ks, int S, int n_tiles, int I, bf16_t* out,
                   long ldo, float* part, long part_ld, hipStream_t st, const WsPro& pr) {
  constexpr int MT = 4;
  constexpr size_t lds = (size_t)ws_stages_pro(MT, BN, PRO) * (16 * MT * 128 + BN * 128);
  LK_SET_MAX_LDS((wsgemm_kernel<MT, BN, SWIGLU, false, PRO>), (int)lds);
  const int rot_mul = g_ws_rot_mul >= 0 ? g_ws_rot_mul : (S == 1 ? 5 : 0);
  wsgemm_kernel<MT, BN, SWIGLU, false, PRO><<<n_tiles * S, 256, lds, st>>>(
      x, K, w, M, K, ks, n_tiles, I, out, ldo, part, part_ld, 1L << 40, rot_mul, WsTail{}, pr);
}

template <int MT, int BN, bool SWIGLU>
void launch_ws_lw(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S, int n_tiles, int I,
                  bf16_t* out, long ldo, float* part, long part_ld, long n_rows, hipStream_t st, const WsTail& tl) {
  constexpr size_t lds = (size_t)lw_nsx(MT) * 16 * MT * 128 + (size_t)lw_nsw(MT, BN) * BN * 128;
  auto kern = tl.kind ? wsgemm_lw_kernel<MT, BN, SWIGLU, true> : wsgemm_lw_kernel<MT, BN, SWIGLU, false>;
  if (tl.kind) LK_SET_MAX_LDS((wsgemm_lw_kernel<MT, BN, SWIGLU, true>), (int)lds);
  else LK_SET_MAX_LDS((wsgemm_lw_kernel<MT, BN, SWIGLU, false>), (int)lds);
  const int rot_mul = n_rows < (1L << 40) ? 0 : g_ws_rot_mul >= 0 ? g_ws_rot_mul : (S == 1 ? 5 : 0);
  kern<<<n_tiles * S, 384, lds, st>>>(x, ldx, w, M, K, ks, n_tiles, I, out, ldo, part, part_ld, n_rows, rot_mul, tl);
}

template <bool SWIGLU>
int dispatch_ws(int MT, int BN, const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S,
                int n_tiles, int I, bf16_t* out, long ldo, float* part, long part_ld, hipStream_t st,
                long n_rows = 1L << 40, int variant = 0, const WsTail& tl = WsTail{}) {
#define LK_WS(mt, bn)                                                                                          \
  if (MT == mt && BN == bn) {                                                                                  \
    if (variant == 1)                                                                                          \
      launch_ws_lw<mt, bn, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, n_rows, st, tl); \
    else                                                                                                       \
      launch_ws<mt, bn, SWIGLU>(x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, part, part_ld, n_rows, st, tl);    \
    return 0;                                                                                                  \
  }
  LK_WS(4, 64) LK_WS(4, 128) LK_WS(8, 64) LK_WS(8, 128) LK_WS(12, 64) LK_WS(12, 128) LK_WS(16, 64) LK_WS(16, 128)
  if constexpr (!SWIGLU) {  // 96-column tiles: projections whose N / 128 tiles leave CUs idle
    LK_WS(4, 96) LK_WS(8, 96) LK_WS(12, 96) LK_WS(16, 96)
  }
#undef LK_WS
  return -2;
}

template <int MT, int NTW, bool SWIGLU>
void launch_skinny(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int ks, int S, int n_tiles,
                   int I, bf16_t* out, long ldo, float* part, long part_ld, hipStream_t st) {
  const size_t lds = sizeof(float) * kSkW * 16 * MT * (16 * NTW + 4);
  auto kern = skinny_gemm_kernel<MT, NTW, SWIGLU>;
  LK_SET_MAX_LDS(kern, (int)lds);
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

// padded row tiles of the weight-streaming GEMM: 16-row MFMA tiles, 4 waves splitting M
// (the X bytes every column block stages grow with the padding: 192 rows for M 129-192
// instead of 256)
static int ws_mt(int M) { return M <= 64 ? 4 : M <= 128 ? 8 : M <= 192 ? 12 : 16; }

// wsgemm launch plan for (M, N, K): BN (64/128) and split S maximising CU occupancy
// (1 block per CU: its LDS ring is 72-144 KB), fewest partial slabs on ties.
void lk_wsgemm_plan(int M, int N, int K, int swiglu, int* bn_out, int* s_out) {
  // Rule fitted to the exhaustive (BN, S) sweep on MI355X (profiles/r1_ws_sweep.md):
  // one block per CU, so fill <= 256 CUs in ONE round; prefer BN = 128 (half the X
  // re-reads through L2) and split K only while every block keeps >= 16 stages;
  // fall back to BN = 64 when BN = 128 leaves more than 30 % of the CUs idle.
  (void)M;
  auto plan = [&](int BN, int* S_out) -> double {
    const int cols = swiglu ? N / 2 : N, per = swiglu ? BN / 2 : BN;
    if (cols % per) return -1.0;
    const int tiles = cols / per;
    int S = 1;
    while (tiles * S * 2 <= 256 && K % (S * 2 * 64) == 0 && K / (S * 2) >= 1024) S *= 2;
    *S_out = S;
    const int blocks = tiles * S, rounds = (blocks + 255) / 256;
    return (double)blocks / (rounds * 256.0);
  };
  int s128 = 1, s64 = 1;
  const double o128 = plan(128, &s128), o64 = plan(64, &s64);
  double occ;
  if (o128 >= 0.7 || (o128 >= 0 && o64 <= o128)) {
    *bn_out = 128;
    *s_out = s128;
    occ = o128;
  } else {
    *bn_out = 64;
    *s_out = o64 >= 0 ? s64 : 1;
    occ = o64;
  }
  // 96-column tiles where they fill the CUs better: the Llama-3-8B QKV projection (N 6144) is
  // 48 x 128-column tiles x 4 K-splits = 192 blocks for 256 CUs, 64 x 96-column tiles x 4 = 256
  // (LK_WS_BN96=0: off)
  static const int bn96 = [] {
    const char* e = getenv("LK_WS_BN96");
    return e ? atoi(e) : 1;
  }();
  if (bn96 && !swiglu) {
    int s96 = 1;
    const double o96 = plan(96, &s96);
    if (o96 > occ + 1e-9) {
      *bn_out = 96;
      *s_out = s96;
    }
  }
}

// per-shape kernel variant of the weight-streaming GEMM: 0 = one LDS ring (wsgemm_kernel),
// 1 = loader waves (wsgemm_lw_kernel); keyed by (row tile MT, N, K, swiglu), set by the decode
// tuner's measurement (ops.tune_decode), default LK_WS_LOADER (0)
static std::mutex g_ws_var_mu;
static std::map<long, int> g_ws_var;
static long ws_var_key(int MT, int N, int K, int swiglu) {
  return (((long)MT * 1000003L + N) * 1000003L + K) * 2 + (swiglu ? 1 : 0);
}
static int ws_variant(int M, int N, int K, int swiglu) {
  static const int dflt = [] {
    const char* e = getenv("LK_WS_LOADER");
    return e ? (atoi(e) != 0) : 0;
  }();
  std::lock_guard<std::mutex> lock(g_ws_var_mu);
  auto it = g_ws_var.find(ws_var_key(ws_mt(M), N, K, swiglu));
  return it != g_ws_var.end() ? it->second : dflt;
}
int lk_wsgemm_set_variant(int M, int N, int K, int swiglu, int variant) {
  if (variant < -1 || variant > 1) return -1;
  std::lock_guard<std::mutex> lock(g_ws_var_mu);
  const long key = ws_var_key(ws_mt(M), N, K, swiglu);
  if (variant < 0) g_ws_var.erase(key);
  else g_ws_var[key] = variant;
  return 0;
}

int lk_wsgemm(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, int swiglu,
              bf16_t* out, long ldo, float* part, hipStream_t st) {
  if (M < 1 || M > 256 || S < 1 || K % (S * 64) || (BN != 64 && BN != 128 && (BN != 96 || swiglu))) return -1;
  const int per = swiglu ? BN / 2 : BN;
  if (swiglu ? (N % 2 || (N / 2) % per) : N % BN) return -1;
  if (S > 1 && part == nullptr) return -1;
  const int I = swiglu ? N / 2 : 0;
  const int n_tiles = (swiglu ? I : N) / per;
  const int MT = ws_mt(M);
  const int ks = K / S;
  float* p = S > 1 ? part : nullptr;
  const int var = ws_variant(M, N, K, swiglu);
  const int rc = swiglu ? dispatch_ws<true>(MT, BN, x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, p, N, st,
                                            1L << 40, var)
                        : dispatch_ws<false>(MT, BN, x, ldx, w, M, K, ks, S, n_tiles, I, out, ldo, p, N, st,
                                             1L << 40, var);
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

void lk_wsgemm_set_rot(int rot_mul) { g_ws_rot_mul = rot_mul < 0 ? -1 : rot_mul; }

// Weight-streaming GEMM with a consumer-side X prologue (WsPro, one LDS ring, M <= 64): kind 1 =
// residual add + RMSNorm of the producer's split-K slabs, kind 2 = flash-decoding merge of a
// paged-decode step's split partials.  x: [M, K] bf16 rows (kind 1: written; kind 2: the
// attention output, merged rows written).  S > 1: partial slabs into part, and with out also the
// reduce (SwiGLU) into out; S == 1: out directly.
int lk_wsgemm_pro(int kind, bf16_t* x, const bf16_t* w, int M, int N, int K, int BN, int S, int swiglu,
                  bf16_t* out, long ldo, float* part, const float* pp, int pS, const bf16_t* res, bf16_t* res_out,
                  long rs, const bf16_t* gamma, float eps, const float* po, const float* pml, const int* ctx, int Hq,
                  int D, int max_splits, int split, hipStream_t st) {
  if (M < 1 || M > 64 || S < 1 || K % (S * 64) || !x || (BN != 64 && BN != 128 && (BN != 96 || swiglu))) return -1;
  const int per = swiglu ? BN / 2 : BN;
  if (swiglu ? (N % 2 || (N / 2) % per) : N % BN) return -1;
  if ((S > 1 && !part) || (S == 1 && !out)) return -1;
  WsPro pr;
  pr.kind = kind;
  pr.x = x;
  if (kind == 1) {
    if (K % 8 || K > 8192 || !pp || pS < 1 || !res || !res_out || res == res_out || !gamma || rs % 8) return -1;
    pr.part = pp;
    pr.S = pS;
    pr.slab = (long)M * K;
    pr.res = res;
    pr.res_out = res_out;
    pr.rs = rs;
    pr.gamma = gamma;
    pr.eps = eps;
  } else if (kind == 2) {
    if (!po || !pml || !ctx || D <= 0 || Hq * D != K || max_splits < 1 || split < 1) return -1;
    pr.po = po;
    pr.pml = pml;
    pr.ctx = ctx;
    pr.Hq = Hq;
    pr.D = D;
    pr.max_splits = max_splits;
    pr.split = split;
  } else {
    return -1;
  }
  const int I = swiglu ? N / 2 : 0;
  const int n_tiles = (swiglu ? I : N) / per;
  const int ks = K / S;
  float* p = S > 1 ? part : nullptr;
#define LK_PRO(bn, sw, kd) \
  if (BN == bn && (swiglu != 0) == sw && kind == kd) launch_ws_pro<bn, sw, kd>(x, w, M, K, ks, S, n_tiles, I, out, ldo, p, N, st, pr); else
  LK_PRO(64, false, 1) LK_PRO(96, false, 1) LK_PRO(128, false, 1) LK_PRO(64, true, 1) LK_PRO(128, true, 1)
  LK_PRO(64, false, 2) LK_PRO(96, false, 2) LK_PRO(128, false, 2) return -2;
#undef LK_PRO
  LK_CHECK_LAUNCH();
  if (S > 1 && out) {
    const int n_out = swiglu ? I : N;
    const long work = (long)M * (n_out / 4);
    int grid = (int)((work + 255) / 256);
    if (grid > 2048) grid = 2048;
    if (swiglu)
      splitk_reduce_kernel<true><<<grid, 256, 0, st>>>(part, S, M, N, n_out, I, out, ldo);
    else
      splitk_reduce_kernel<false><<<grid, 256, 0, st>>>(part, S, M, N, n_out, 0, out, ldo);
    LK_CHECK_LAUNCH();
  }
  return 0;
}

int lk_wsgemm_part(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, float* part,
                   hipStream_t st) {
  if (M < 1 || M > 256 || S < 2 || K % (S * 64) || (BN != 64 && BN != 96 && BN != 128) || N % BN ||
      part == nullptr)
    return -1;
  const int MT = ws_mt(M);
  const int rc = dispatch_ws<false>(MT, BN, x, ldx, w, M, K, K / S, S, N / BN, 0, nullptr, 0, part, N, st,
                                    1L << 40, ws_variant(M, N, K, 0));
  LK_CHECK_LAUNCH();
  return rc;
}

// split-K GEMM whose last split workgroup per head applies RoPE and writes the paged KV (WsTail
// kind 1): the rows lk_splitk_rope_kv would leave, without its launch.  Needs one column tile per
// head (BN == D) and S in {2, 4, 8}; tickets: >= (Hq + 2 Hkv) zeroed int32.
int lk_ws_rope_kv_fused(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int BN, int S, float* part,
                        int* tickets, bf16_t* qkv, long qs, const int* positions, const float* cos_sin, int Hq,
                        int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                        int write_k_inplace, hipStream_t st) {
  const int N = (Hq + 2 * Hkv) * D;
  if (M < 1 || M > 256 || !(S == 2 || S == 4 || S == 8) || K % (S * 64) || BN != D || BN != 128 || !part ||
      !tickets || !qkv || qs % 8 || D % 16 || (long)S * M * N * 4 >= 0x7FFFFFF0L)
    return -1;
  WsTail tl;
  tl.kind = 1;
  tl.tickets = tickets;
  tl.out = qkv;
  tl.os = qs;
  tl.positions = positions;
  tl.cos_sin = cos_sin;
  tl.Hq = Hq;
  tl.Hkv = Hkv;
  tl.D = D;
  tl.kc = kc;
  tl.vc = vc;
  tl.slots = slots;
  tl.BS = BS;
  tl.neox = neox;
  tl.write_k_inplace = write_k_inplace;
  const int rc = dispatch_ws<false>(ws_mt(M), BN, x, ldx, w, M, K, K / S, S, N / BN, 0, nullptr, 0, part, N, st,
                                    1L << 40, ws_variant(M, N, K, 0), tl);
  LK_CHECK_LAUNCH();
  return rc;
}

// split-K GEMM + residual add + RMSNorm by the grid's last workgroup (WsTail kind 2), for a few
// rows (M <= 4: one workgroup normalises them all); tickets: >= 1 zeroed int32
int lk_ws_rmsnorm_fused(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, float* part,
                        int* tickets, bf16_t* out, long os, bf16_t* residual, long rs, const bf16_t* norm_w, float eps,
                        hipStream_t st) {
  if (M < 1 || M > 4 || !(S == 2 || S == 4 || S == 8) || K % (S * 64) || (BN != 64 && BN != 128) || N % BN ||
      !part || !tickets || !out || !residual || os % 8 || rs % 8 || (long)S * M * N * 4 >= 0x7FFFFFF0L)
    return -1;
  WsTail tl;
  tl.kind = 2;
  tl.tickets = tickets;
  tl.out = out;
  tl.os = os;
  tl.residual = residual;
  tl.rs = rs;
  tl.norm_w = norm_w;
  tl.eps = eps;
  const int rc = dispatch_ws<false>(ws_mt(M), BN, x, ldx, w, M, K, K / S, S, N / BN, 0, nullptr, 0, part, N, st,
                                    1L << 40, ws_variant(M, N, K, 0), tl);
  LK_CHECK_LAUNCH();
  return rc;
}

// f32 X W^T for a W of any row count (kNN scores: X = queries, W = corpus rows):
// out[M, N] with row stride ldo; one pass over W, no split-K.
int lk_ws_scores_f32(const bf16_t* x, long ldx, const bf16_t* w, int M, long N, int K, float* out, long ldo,
                     hipStream_t st) {
  if (M < 1 || M > 256 || N < 1 || K % 64 || K < 64) return -1;
  const int BN = 128;
  const long tiles = (N + BN - 1) / BN;
  if (tiles > (1L << 30)) return -1;
  const int MT = ws_mt(M);
  const int rc = dispatch_ws<false>(MT, BN, x, ldx, w, M, K, K, 1, (int)tiles, 0, nullptr, 0, out, ldo, st, N);
  LK_CHECK_LAUNCH();
  return rc;
}

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
