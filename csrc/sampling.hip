// K13 token selection over the vocabulary: greedy argmax, temperature sampling via
// the Gumbel-max trick (one pass, no sort: argmax(l/T + G), G = -log(-log U)) and
// Ollama/llama.cpp-style repetition penalty.  One workgroup per row, 16-byte logits
// loads, (value, lowest index) wave reductions — argmax ties resolve to the first
// index, like torch.argmax.
#include "common.h"
#include "kernels.h"

namespace {

LK_DEVICE bool gt(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

LK_DEVICE unsigned hash3(unsigned a, unsigned b, unsigned c) {
  // splitmix-style avalanche over three words
  unsigned long long x = ((unsigned long long)a << 32) ^ ((unsigned long long)b * 0x9E3779B97F4A7C15ull) ^ c;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (unsigned)(x >> 32);
}

// ALLOWED: grammar-constrained rows consider only their allowed ids (plan = [B flags |
// B+1 row offsets | ids]; flags[row] = 0 -> the whole vocabulary).  Same values, same
// Gumbel noise per (row, step, id) and the same tie order as scanning the row with every
// other id masked to -inf -- without materialising the [B, V] mask (3 full passes over
// the logits) or scanning 128k entries per row.
template <bool BF16, bool SAMPLE, bool ALLOWED = false>
__global__ __launch_bounds__(256) void select_kernel(const void* __restrict__ logits, long ls, int V,
                                                     const float* __restrict__ temps,
                                                     unsigned long long seed, int step,
                                                     int* __restrict__ out, const int* __restrict__ plan = nullptr) {
  __shared__ float rs[4];
  __shared__ int ri[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float temp = SAMPLE ? temps[row] : 1.f;
  const bool greedy = !SAMPLE || temp <= 0.f;
  const float invt = greedy ? 1.f : 1.f / temp;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int nv = V / 8;
  const int B = gridDim.x;
  const bool sparse = ALLOWED && plan[row] != 0;
  auto consider = [&](float x, int idx) {
    if (!greedy) {
      const unsigned hsh = hash3((unsigned)(seed ^ (seed >> 32)) + row, (unsigned)step, (unsigned)idx);
      const float u = ((float)(hsh >> 8) + 0.5f) * (1.f / 16777216.f);
      x = x * invt - __logf(-__logf(u));
    }
    if (gt(x, idx, best, bi)) {
      best = x;
      bi = idx;
    }
  };
  if (sparse) {
    const int* ids = plan + 2 * B + 1;
    const int a0 = plan[B + row], a1 = plan[B + row + 1];
    for (int j = a0 + tid; j < a1; j += 256) {
      const int id = ids[j];
      if constexpr (BF16) consider(bf2f(reinterpret_cast<const bf16_t*>(logits)[(long)row * ls + id]), id);
      else consider(reinterpret_cast<const float*>(logits)[(long)row * ls + id], id);
    }
  } else if constexpr (BF16) {
    const bf16_t* lp = reinterpret_cast<const bf16_t*>(logits) + (long)row * ls;
    for (int c = tid; c < nv; c += 256) {
      float v[8];
      load8(lp + c * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) consider(v[j], c * 8 + j);
    }
    for (int i = nv * 8 + tid; i < V; i += 256) consider(bf2f(lp[i]), i);
  } else {
    const float* lp = reinterpret_cast<const float*>(logits) + (long)row * ls;
    for (int c = tid; c < nv; c += 256) {
      const float4 a = *reinterpret_cast<const float4*>(lp + c * 8);
      const float4 b = *reinterpret_cast<const float4*>(lp + c * 8 + 4);
      consider(a.x, c * 8 + 0); consider(a.y, c * 8 + 1); consider(a.z, c * 8 + 2); consider(a.w, c * 8 + 3);
      consider(b.x, c * 8 + 4); consider(b.y, c * 8 + 5); consider(b.z, c * 8 + 6); consider(b.w, c * 8 + 7);
    }
    for (int i = nv * 8 + tid; i < V; i += 256) consider(lp[i], i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (gt(b2, i2, best, bi)) {
      best = b2;
      bi = i2;
    }
  }
  if (lane == 0) {
    rs[w] = best;
    ri[w] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int j = 1; j < 4; ++j)
      if (gt(rs[j], ri[j], best, bi)) {
        best = rs[j];
        bi = ri[j];
      }
    if (bi == 0x7fffffff) bi = 0;  // all -inf / NaN row: fall back to token 0
    out[row] = bi;
  }
}

// logits[row, tok] = l > 0 ? l / p : l * p for each UNIQUE token of the row's window
template <bool BF16>
__global__ void repeat_penalty_kernel(void* __restrict__ logits, long ls,
                                      const int* __restrict__ window, int W,
                                      const float* __restrict__ penalty) {
  const int row = blockIdx.x;
  const float p = penalty[row];
  const int* win = window + (long)row * W;
  for (int j = threadIdx.x; j < W; j += blockDim.x) {
    const int tok = win[j];
    if (tok < 0) continue;
    bool dup = false;
    for (int i = 0; i < j; ++i) dup |= (win[i] == tok);
    if (dup) continue;
    if constexpr (BF16) {
      bf16_t* lp = reinterpret_cast<bf16_t*>(logits) + (long)row * ls + tok;
      const float l = bf2f(*lp);
      *lp = f2bf(l > 0.f ? l / p : l * p);
    } else {
      float* lp = reinterpret_cast<float*>(logits) + (long)row * ls + tok;
      const float l = *lp;
      *lp = l > 0.f ? l / p : l * p;
    }
  }
}

}  // namespace

int lk_select_tokens(const void* logits, int is_bf16, long ls, int B, int V, const float* temps,
                     unsigned long long seed, int step, int* out, hipStream_t st) {
  if (B <= 0) return 0;
  if (ls % 8 && is_bf16) return -1;
  if (is_bf16) {
    if (temps) select_kernel<true, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out);
    else select_kernel<true, false><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out);
  } else {
    if (temps) select_kernel<false, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out);
    else select_kernel<false, false><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out);
  }
  return 0;
}

int lk_select_allowed(const void* logits, int is_bf16, long ls, int B, int V, const float* temps,
                      unsigned long long seed, int step, const int* plan, int* out, hipStream_t st) {
  if (B <= 0) return 0;
  if ((ls % 8 && is_bf16) || !plan) return -1;
  if (is_bf16) {
    if (temps) select_kernel<true, true, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out, plan);
    else select_kernel<true, false, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out, plan);
  } else {
    if (temps) select_kernel<false, true, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out, plan);
    else select_kernel<false, false, true><<<B, 256, 0, st>>>(logits, ls, V, temps, seed, step, out, plan);
  }
  return 0;
}

int lk_repeat_penalty(void* logits, int is_bf16, long ls, int B, const int* window, int W,
                      const float* penalty, hipStream_t st) {
  if (B <= 0 || W <= 0) return 0;
  if (is_bf16) repeat_penalty_kernel<true><<<B, 64, 0, st>>>(logits, ls, window, W, penalty);
  else repeat_penalty_kernel<false><<<B, 64, 0, st>>>(logits, ls, window, W, penalty);
  return 0;
}
