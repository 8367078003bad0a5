// K7 RMSNorm (+fused residual add), K8/K4 LayerNorm (+bias, +residual),
// K1 BERT embedding gather fused with LayerNorm.
//
// One workgroup per row; every thread keeps its slice of the row in registers
// (MAXV x 16-byte vectors), so the row is read from HBM exactly once and the
// residual sum is written back in the same pass (the vLLM-style fused
// "add + norm" that replaces two separate elementwise passes).
#include "common.h"
#include "kernels.h"
#include "rowcfg.h"

namespace {

// SP > 0: x is not a bf16 tensor but the SP f32 split-K partial slabs of the producing
// weight-streaming GEMM (part[s][row][H], slab = rows * H floats apart): they are summed
// in slab order and rounded to bf16 -- exactly the values splitk_reduce_kernel would have
// stored -- so "GEMM partials -> reduce -> add + norm" becomes one launch with
// bit-identical results (the decode step's o / down projections).
// (SP is a template constant so all SP x MAXV slab loads of a thread are issued before the
// first add: a runtime slab loop serialised one L2 round trip per slab)
template <int MAXV, int NW, int SP>
__global__ __launch_bounds__(NW * 64) void rmsnorm_kernel(
    bf16_t* __restrict__ out, bf16_t* __restrict__ residual, const bf16_t* __restrict__ x,
    const bf16_t* __restrict__ w, int H, float eps, long xs, long os, long rs,
    const float* __restrict__ part, long slab) {
  __shared__ float red[NW];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16_t* xr = x + row * xs;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      if constexpr (SP > 0) {
        const float* pp = part + row * H + c * 8;
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
          v[i][j] = bf2f(f2bf(a[j]));
          v[i][j + 4] = bf2f(f2bf(b[j]));
        }
      } else {
        load8(xr + c * 8, v[i]);
      }
      if (residual) {
        float r[8];
        bf16_t* rr = residual + row * rs + c * 8;
        load8(rr, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // the new residual stream is the bf16-rounded sum (same as eager bf16 add)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j]));
        store8(rr, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum<NW>(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      float g[8], y[8];
      load8(w + c * 8, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(v[i][j] * inv)) * g[j];
      store8(out + row * os + c * 8, y);
    }
  }
}

// LayerNorm over (x [+ res]); optionally writes x+res back into `res_out`.
template <int MAXV, int NW>
__global__ __launch_bounds__(NW * 64) void layernorm_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
    bf16_t* __restrict__ res_out, const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
    int H, float eps, long xs, long os, long rs) {
  __shared__ float red[NW];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      load8(x + row * xs + c * 8, v[i]);
      if (res) {
        float r[8];
        load8(res + row * rs + c * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + r[j]));
        if (res_out) store8(res_out + row * rs + c * 8, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum<NW>(s, red) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NW>(q, red) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      float g[8], bb[8], y[8];
      load8(w + c * 8, g);
      if (b) load8(b + c * 8, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (v[i][j] - mean) * inv * g[j] + (b ? bb[j] : 0.f);
      store8(out + row * os + c * 8, y);
    }
  }
}

// out[t] = LN(tok[ids[t]] + pos[pos_ids[t]] + type[type_ids[t]])   (pos/type optional)
template <int MAXV, int NW>
__global__ __launch_bounds__(NW * 64) void embed_ln_kernel(
    bf16_t* __restrict__ out, const int* __restrict__ ids, const int* __restrict__ pos_ids,
    const int* __restrict__ type_ids, const bf16_t* __restrict__ tok, const bf16_t* __restrict__ pos,
    const bf16_t* __restrict__ typ, const bf16_t* __restrict__ w, const bf16_t* __restrict__ b, int H,
    float eps) {
  __shared__ float red[NW];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  const long tid = ids[row];
  const long pid = pos ? (long)pos_ids[row] : 0;
  const long yid = (typ && type_ids) ? (long)type_ids[row] : 0;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      float t[8];
      load8(tok + tid * H + c * 8, v[i]);
      if (pos) {
        load8(pos + pid * H + c * 8, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
      if (typ) {
        load8(typ + yid * H + c * 8, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum<NW>(s, red) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NW>(q, red) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NW * 64;
    if (c < nvec) {
      float g[8], bb[8], y[8];
      load8(w + c * 8, g);
      load8(b + c * 8, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (v[i][j] - mean) * inv * g[j] + bb[j];
      store8(out + row * (long)H + c * 8, y);
    }
  }
}

}  // namespace

int lk_rmsnorm(bf16_t* out, bf16_t* residual, const bf16_t* x, const bf16_t* w, long rows, int H,
               float eps, long xs, long os, long rs, hipStream_t st) {
  if (H % 8 || rows <= 0) return rows == 0 ? 0 : -1;
#define CALL(MV, NW)                                                                                   \
  rmsnorm_kernel<MV, NW, 0><<<dim3(rows), dim3(NW * 64), 0, st>>>(out, residual, x, w, H, eps, xs, os, rs, \
                                                                 nullptr, 0)
  ROW_DISPATCH(H, CALL);
#undef CALL
  return 0;
}

// out = RMSNorm(bf16(sum of S partial slabs) + residual) * w, residual updated in place;
// part: [S][rows][H] f32 (the layout lk_wsgemm_part writes)
int lk_splitk_rmsnorm(bf16_t* out, bf16_t* residual, const float* part, int S, const bf16_t* w, long rows, int H,
                      float eps, long os, long rs, hipStream_t st) {
  if (H % 8 || !residual || rows <= 0) return rows == 0 ? 0 : -1;
  const long slab = rows * H;
#define CALL_SP(MV, NW, SPC)                                                                         \
  rmsnorm_kernel<MV, NW, SPC><<<dim3(rows), dim3(NW * 64), 0, st>>>(out, residual, nullptr, w, H, eps, 0, os, \
                                                                   rs, part, slab)
#define CALL2(MV, NW) CALL_SP(MV, NW, 2)
#define CALL4(MV, NW) CALL_SP(MV, NW, 4)
#define CALL8(MV, NW) CALL_SP(MV, NW, 8)
  if (S == 2) ROW_DISPATCH(H, CALL2);
  else if (S == 4) ROW_DISPATCH(H, CALL4);
  else if (S == 8) ROW_DISPATCH(H, CALL8);
  else return -1;
#undef CALL2
#undef CALL4
#undef CALL8
#undef CALL_SP
  return 0;
}

int lk_layernorm(bf16_t* out, const bf16_t* x, const bf16_t* res, bf16_t* res_out, const bf16_t* w,
                 const bf16_t* b, long rows, int H, float eps, long xs, long os, long rs,
                 hipStream_t st) {
  if (H % 8 || rows <= 0) return rows == 0 ? 0 : -1;
#define CALL(MV, NW)                                                                          \
  layernorm_kernel<MV, NW><<<dim3(rows), dim3(NW * 64), 0, st>>>(out, x, res, res_out, w, b, H, \
                                                                eps, xs, os, rs)
  ROW_DISPATCH(H, CALL);
#undef CALL
  return 0;
}

int lk_embed_layernorm(bf16_t* out, const int* ids, const int* pos_ids, const int* type_ids,
                       const bf16_t* tok, const bf16_t* pos, const bf16_t* typ, const bf16_t* w,
                       const bf16_t* b, long rows, int H, float eps, hipStream_t st) {
  if (H % 8 || rows <= 0) return rows == 0 ? 0 : -1;
#define CALL(MV, NW)                                                                      \
  embed_ln_kernel<MV, NW><<<dim3(rows), dim3(NW * 64), 0, st>>>(out, ids, pos_ids, type_ids, \
                                                               tok, pos, typ, w, b, H, eps)
  ROW_DISPATCH(H, CALL);
#undef CALL
  return 0;
}
