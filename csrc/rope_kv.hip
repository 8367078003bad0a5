// K9 rotary embedding fused with the paged KV-cache write.
//
// Input is the packed output of the fused QKV projection, [T, (Hq + 2*Hkv) * D].
// Q (and optionally K) are rotated in place; rotated K and raw V are scattered
// into the paged cache [num_blocks, Hkv, BS, D] at slot_mapping[t] (slot = block*BS
// + offset; negative slot = padding token, skipped).  One workgroup per token;
// each work item moves 16 bytes per half (8 rotation pairs), so the op is a single
// HBM-bound pass over Q, K, V and the cos/sin table row.
#include "common.h"
#include "kernels.h"

namespace {

// grid (T, ceil(items / 64)), 64 threads: one 16-B rotation item (or V chunk) per
// thread, so a decode step (T ~ 128 tokens) still puts ~900 single-wave workgroups
// on the 256 CUs instead of 128 workgroups each looping over 3 dependent items.
//
// SP > 0: the QKV projection left SP f32 split-K partial slabs (part[s][t][ld], slab floats
// apart) instead of its bf16 output.  Each item sums its 8 columns in slab order and
// rounds to bf16 (the values splitk_reduce_kernel would have stored), writes the qkv row
// exactly as "reduce, then rope_kv" leaves it (q rotated, k unrotated unless
// write_k_inplace, v copied) and scatters K/V into the cache: one launch instead of two.
template <bool NEOX, int SP>
__global__ __launch_bounds__(64) void rope_kv_kernel(
    bf16_t* __restrict__ qkv, long qs, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int Hq, int Hkv, int D, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, const int* __restrict__ slots, int BS, int write_k_inplace,
    const float* __restrict__ part, long slab, long ld) {
  constexpr bool PART = SP > 0;
  const long t = blockIdx.x;
  // 8 consecutive elements of this token's qkv row at column col, as f32 (all SP slab
  // loads issued before the first add)
  auto ld8 = [&](int col, float* f) {
    if constexpr (PART) {
      const float* pp = part + t * ld + col;
      floatx4 pa[SP], pb[SP];
#pragma unroll
      for (int s = 0; s < SP; ++s) {
        pa[s] = *reinterpret_cast<const floatx4*>(pp + s * slab);
        pb[s] = *reinterpret_cast<const floatx4*>(pp + s * slab + 4);
      }
      floatx4 a = pa[0], b = pb[0];
#pragma unroll
      for (int s = 1; s < SP; ++s) {
        a += pa[s];
        b += pb[s];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = bf2f(f2bf(a[j]));
        f[j + 4] = bf2f(f2bf(b[j]));
      }
    } else {
      load8(qkv + t * qs + col, f);
    }
  };
  const int it = blockIdx.y * 64 + threadIdx.x;
  const int half = D >> 1;
  const int ipr = NEOX ? (D >> 4) : (D >> 3);  // rotation items per head
  const int nrot = (Hq + Hkv) * ipr;
  const int vpr = D >> 3;
  if (it >= nrot + Hkv * vpr) return;
  bf16_t* row = qkv + t * qs;
  const int slot = slots ? slots[t] : -1;
  LK_DASSERT(slot >= -1);
  const long blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  if (it >= nrot) {  // V: plain copy into the cache
    const int i = it - nrot, h = i / vpr, c = (i - h * vpr) * 8;
    if constexpr (PART) {
      float f[8];
      ld8((Hq + Hkv + h) * D + c, f);
      store8(row + (long)(Hq + Hkv + h) * D + c, f);
      if (vc && slot >= 0) store8(vc + ((blk * Hkv + h) * BS + off) * D + c, f);
    } else if (vc && slot >= 0) {
      *reinterpret_cast<short8*>(vc + ((blk * Hkv + h) * BS + off) * D + c) =
          *reinterpret_cast<const short8*>(row + (long)(Hq + Hkv + h) * D + c);
    }
    return;
  }
  const float* cs = cos_sin + (long)positions[t] * D;  // [cos(D/2) | sin(D/2)]
  const int head = it / ipr;
  const int v = it - head * ipr;
  bf16_t* hp = row + head * D;
  const bool is_k = head >= Hq;
  const int kvh = head - Hq;
  bf16_t* kdst = (is_k && kc && slot >= 0) ? kc + ((blk * Hkv + kvh) * BS + off) * D : nullptr;
  const bool store_src = !is_k || write_k_inplace;
  if constexpr (NEOX) {
    const int i0 = v * 8;
    float x1[8], x2[8], y1[8], y2[8];
    ld8(head * D + i0, x1);
    ld8(head * D + half + i0, x2);
    if (PART && !store_src) {  // k kept unrotated in the qkv row
      store8(hp + i0, x1);
      store8(hp + half + i0, x2);
    }
    const floatx4 c0 = *reinterpret_cast<const floatx4*>(cs + i0);
    const floatx4 c1 = *reinterpret_cast<const floatx4*>(cs + i0 + 4);
    const floatx4 s0 = *reinterpret_cast<const floatx4*>(cs + half + i0);
    const floatx4 s1 = *reinterpret_cast<const floatx4*>(cs + half + i0 + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4], s = j < 4 ? s0[j] : s1[j - 4];
      y1[j] = x1[j] * c - x2[j] * s;
      y2[j] = x2[j] * c + x1[j] * s;
    }
    if (store_src) {
      store8(hp + i0, y1);
      store8(hp + half + i0, y2);
    }
    if (kdst) {
      store8(kdst + i0, y1);
      store8(kdst + half + i0, y2);
    }
  } else {
    const int e0 = v * 8;  // elements e0..e0+7 = pairs e0/2 .. e0/2+3
    float x[8], y[8];
    ld8(head * D + e0, x);
    if (PART && !store_src) store8(hp + e0, x);
    const floatx4 c4 = *reinterpret_cast<const floatx4*>(cs + (e0 >> 1));
    const floatx4 s4 = *reinterpret_cast<const floatx4*>(cs + half + (e0 >> 1));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      y[2 * p] = x[2 * p] * c4[p] - x[2 * p + 1] * s4[p];
      y[2 * p + 1] = x[2 * p + 1] * c4[p] + x[2 * p] * s4[p];
    }
    if (store_src) store8(hp + e0, y);
    if (kdst) store8(kdst + e0, y);
  }
}

// plain paged write of K/V (no rotation): k,v [T, Hkv, D] with token strides ks/vs
__global__ __launch_bounds__(128) void kv_write_kernel(const bf16_t* __restrict__ k, long ks,
                                                       const bf16_t* __restrict__ v, long vs,
                                                       bf16_t* __restrict__ kc,
                                                       bf16_t* __restrict__ vc,
                                                       const int* __restrict__ slots, int Hkv,
                                                       int D, int BS) {
  const long t = blockIdx.x;
  const int slot = slots[t];
  if (slot < 0) return;
  const long blk = slot / BS;
  const int off = slot % BS;
  const int vpr = D >> 3;
  for (int it = threadIdx.x; it < Hkv * vpr; it += blockDim.x) {
    const int h = it / vpr, c = (it - h * vpr) * 8;
    const long dst = ((blk * Hkv + h) * BS + off) * D + c;
    *reinterpret_cast<short8*>(kc + dst) = *reinterpret_cast<const short8*>(k + t * ks + h * D + c);
    *reinterpret_cast<short8*>(vc + dst) = *reinterpret_cast<const short8*>(v + t * vs + h * D + c);
  }
}

}  // namespace

int lk_rope_kv(bf16_t* qkv, long qs, const int* positions, const float* cos_sin, long T, int Hq,
               int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
               int write_k_inplace, hipStream_t st) {
  if (D % 16 || T < 0) return -1;
  if (T == 0) return 0;
  const int items = (Hq + Hkv) * (neox ? D / 16 : D / 8) + Hkv * (D / 8);
  const dim3 grid((unsigned)T, (items + 63) / 64);
  if (neox)
    rope_kv_kernel<true, 0><<<grid, 64, 0, st>>>(qkv, qs, positions, cos_sin, Hq, Hkv, D, kc, vc, slots, BS,
                                                 write_k_inplace, nullptr, 0, 0);
  else
    rope_kv_kernel<false, 0><<<grid, 64, 0, st>>>(qkv, qs, positions, cos_sin, Hq, Hkv, D, kc, vc, slots, BS,
                                                  write_k_inplace, nullptr, 0, 0);
  return 0;
}

int lk_splitk_rope_kv(const float* part, int S, bf16_t* qkv, long qs, const int* positions, const float* cos_sin,
                      long T, int Hq, int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                      int write_k_inplace, hipStream_t st) {
  if (D % 16 || T < 0 || !(S == 2 || S == 4 || S == 8)) return -1;
  if (T == 0) return 0;
  const long ld = (long)(Hq + 2 * Hkv) * D;  // partial row = the whole projection output
  const long slab = T * ld;
  const int items = (Hq + Hkv) * (neox ? D / 16 : D / 8) + Hkv * (D / 8);
  const dim3 grid((unsigned)T, (items + 63) / 64);
#define LK_ROPE_SP(SPC)                                                                                        \
  if (neox)                                                                                                    \
    rope_kv_kernel<true, SPC><<<grid, 64, 0, st>>>(qkv, qs, positions, cos_sin, Hq, Hkv, D, kc, vc, slots, BS,   \
                                                   write_k_inplace, part, slab, ld);                           \
  else                                                                                                         \
    rope_kv_kernel<false, SPC><<<grid, 64, 0, st>>>(qkv, qs, positions, cos_sin, Hq, Hkv, D, kc, vc, slots, BS,  \
                                                    write_k_inplace, part, slab, ld);
  if (S == 2) { LK_ROPE_SP(2) }
  else if (S == 4) { LK_ROPE_SP(4) }
  else { LK_ROPE_SP(8) }
#undef LK_ROPE_SP
  return 0;
}

int lk_kv_write(const bf16_t* k, long ks, const bf16_t* v, long vs, bf16_t* kc, bf16_t* vc,
                const int* slots, long T, int Hkv, int D, int BS, hipStream_t st) {
  if (D % 8 || T < 0) return -1;
  if (T == 0) return 0;
  kv_write_kernel<<<dim3(T), 128, 0, st>>>(k, ks, v, vs, kc, vc, slots, Hkv, D, BS);
  return 0;
}
