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
// KEY: greedy only; instead of the id, write the row's order-preserving int64 (value, id) key
// (ops.argmax_key: vocab-parallel greedy = ONE all-gather of these + a max) to key_out
template <bool BF16, bool SAMPLE, bool ALLOWED = false, bool KEY = false>
__global__ __launch_bounds__(256) void select_kernel(const void* __restrict__ logits, long ls, int V,
                                                     const float* __restrict__ temps,
                                                     unsigned long long seed, int step,
                                                     int* __restrict__ out, const int* __restrict__ plan = nullptr,
                                                     long long* __restrict__ key_out = nullptr, int key_lo = 0) {
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
    if constexpr (KEY) {
      // high word: the max's float bits made order-preserving and signed; low word: ~global id
      // (the larger key is the larger value, then the lower id -- torch.argmax's tie order)
      const unsigned fb = __float_as_uint(best == best ? best : -INFINITY);
      const unsigned u = (fb & 0x80000000u) ? ~fb : (fb | 0x80000000u);
      key_out[row] = (long long)(((unsigned long long)(u ^ 0x80000000u) << 32) | (unsigned)(~(unsigned)(bi + key_lo)));
    } else {
      out[row] = bi;
    }
  }
}

// ids[r] = the id of max_w keys[w, r] (the gathered per-rank argmax keys)
__global__ void keys_to_ids_kernel(const long long* __restrict__ keys, int W, int R, int* __restrict__ ids) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  long long k = keys[r];
  for (int w = 1; w < W; ++w) k = max(k, keys[(long)w * R + r]);
  ids[r] = (int)(~(unsigned)(k & 0xFFFFFFFFll));
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

int lk_argmax_key(const void* logits, int is_bf16, long ls, int B, int V, int vocab_lo, long long* keys, hipStream_t st) {
  if (B <= 0) return 0;
  if (ls % 8 && is_bf16) return -1;
  if (is_bf16) select_kernel<true, false, false, true><<<B, 256, 0, st>>>(logits, ls, V, nullptr, 0, 0, nullptr, nullptr, keys, vocab_lo);
  else select_kernel<false, false, false, true><<<B, 256, 0, st>>>(logits, ls, V, nullptr, 0, 0, nullptr, nullptr, keys, vocab_lo);
  return 0;
}

int lk_keys_to_ids(const long long* keys, int W, int R, int* ids, hipStream_t st) {
  if (R <= 0) return 0;
  if (W < 1) return -1;
  keys_to_ids_kernel<<<(R + 255) / 256, 256, 0, st>>>(keys, W, R, ids);
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

// ---------------------------------------------------------------------------------------
// Ollama-default sampling on the device (temperature 0.8, top-k 40, top-p 0.9, repeat
// penalty 1.1 over the last 64 generated tokens): two launches per step, no host work
// beyond one per-row parameter row.
//
//   sample_penalty_kernel: per row, the window of the sequence's device history ring
//     (hist[slot][*], the last min(len, last_n) tokens) is de-duplicated and applied to
//     the f32 logits in place (l > 0 ? l / p : l * p).
//   sample_topkp_kernel (1024 threads per row):
//     1. each thread's max over its strided slice of the row; the K-th largest of the 1024
//        maxima (bitonic sort in LDS) is a lower bound T0 of the row's K-th largest value;
//     2. every element >= T0 is appended to an LDS candidate list (typically ~K of them;
//        more than kCand -> exact radix select over the row in LDS histograms instead);
//     3. bitonic sort of the candidates by (value desc, index asc) -> the top K;
//     4. p_i = exp((v_i - v_0) / T), inclusive scan; keep i while the mass before it is
//        <= top_p * total (so the token crossing top_p is kept); draw u from a counter-based
//        hash of (request seed, generated-token position) and pick the first kept i with
//        prefix > u * kept_total;
//     5. the token goes to out[row] and is appended to the ring (len + 1).
//   Greedy rows (T <= 0) take K = 1: the argmax with the lowest index among ties.
// Row parameters (8 x 32-bit): temperature, top_p, repeat_penalty (f32), top_k, last_n,
// slot, reset (1 = new sequence: its ring restarts empty), seed (i32).
constexpr int kSampThreads = 1024, kSampKMax = 1024, kCand = 4096;

LK_DEVICE unsigned fkey(float f) {  // order-preserving float -> uint
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
constexpr unsigned kNegInfKey = 0x007FFFFFu;  // fkey(-inf); NaN with the sign bit below it
LK_DEVICE float keyf(unsigned k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }

// One workgroup per row.  The window's tokens are de-duplicated through a V-bit "seen" bitmap
// in LDS (one atomicOr per entry; the thread that sets a token's bit penalises it): O(window)
// for any repeat_last_n, including -1 (= the whole ring, sized to max_model_len by the engine).
__global__ __launch_bounds__(256) void sample_penalty_kernel(float* __restrict__ logits, long ls, int V,
                                                             const int* __restrict__ prm,
                                                             const int* __restrict__ hist,
                                                             const int* __restrict__ hist_len, int W) {
  extern __shared__ unsigned seen[];
  const int row = blockIdx.x;
  const int* p = prm + row * 8;
  const float pen = __int_as_float(p[2]);
  const int last_n = p[4], slot = p[5], reset = p[6];
  if (pen == 1.f || last_n == 0) return;  // uniform per workgroup
  const int hl = reset ? 0 : hist_len[slot];
  const int n = min(min(hl, last_n > 0 ? last_n : W), W);
  if (n == 0) return;
  const int words = (V + 31) >> 5;
  for (int i = threadIdx.x; i < words; i += blockDim.x) seen[i] = 0u;
  __syncthreads();
  const int* h = hist + (long)slot * W;
  float* lp = logits + (long)row * ls;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int tok = h[(hl - 1 - j) % W];
    if (tok < 0 || tok >= V) continue;
    const unsigned bit = 1u << (tok & 31);
    if (atomicOr(&seen[tok >> 5], bit) & bit) continue;  // another entry of the window owns it
    const float l = lp[tok];
    lp[tok] = l > 0.f ? l / pen : l * pen;
  }
}

// block-wide inclusive scan (1024 threads = 16 waves)
LK_DEVICE float block_scan(float v, float* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  __syncthreads();
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  float add = 0.f;
  for (int i = 0; i < w; ++i) add += wsum[i];
  return v + add;
}

// bitonic sort of n (power of two <= 4 * 1024) (key desc, idx asc) pairs in LDS
LK_DEVICE bool before(unsigned ka, int ia, unsigned kb, int ib) { return ka > kb || (ka == kb && ia < ib); }
LK_DEVICE void bitonic(unsigned* key, int* idx, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += kSampThreads) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;  // this run sorted "before"-first
          const bool swap = up ? before(key[l], idx[l], key[i], idx[i]) : before(key[i], idx[i], key[l], idx[l]);
          if (swap) {
            const unsigned tk = key[i];
            key[i] = key[l];
            key[l] = tk;
            const int ti = idx[i];
            idx[i] = idx[l];
            idx[l] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(kSampThreads) void sample_topkp_kernel(const float* __restrict__ logits, long ls, int V,
                                                                   const int* __restrict__ prm,
                                                                   int* __restrict__ hist,
                                                                   int* __restrict__ hist_len, int W,
                                                                   unsigned long long seed, int* __restrict__ out) {
  __shared__ unsigned ckey[kCand];
  __shared__ int cidx[kCand];
  __shared__ float wsum[16];
  __shared__ int ncand_s, thr_s, above_s;
  const int row = blockIdx.x, tid = threadIdx.x;
  const int* p = prm + row * 8;
  const float temp = __int_as_float(p[0]), top_p = __int_as_float(p[1]);
  const int top_k = p[3], slot = p[5], reset = p[6], rseed = p[7];
  const bool greedy = temp <= 0.f;
  const int K = greedy ? 1 : min(top_k > 0 ? top_k : kSampKMax, min(V, kSampKMax));
  const float* lp = logits + (long)row * ls;

  // 1. per-thread maxima -> lower bound of the K-th largest
  unsigned tmax = 0;
  for (int i = tid; i < V; i += kSampThreads) tmax = max(tmax, fkey(lp[i]));
  ckey[tid] = tmax;
  cidx[tid] = tid;
  if (tid == 0) ncand_s = 0;
  __syncthreads();
  bitonic(ckey, cidx, kSampThreads);
  // -inf entries (a grammar mask) are never candidates: with fewer finite entries than K the
  // bound would otherwise be -inf and every masked entry would flood the candidate list and
  // the radix fallback's histograms (same-bin atomics).  k_eff below = min(K, finite ones).
  const unsigned t0 = max(ckey[K - 1], kNegInfKey + 1u);
  __syncthreads();
  // 2. gather every element >= t0
  for (int i = tid; i < V; i += kSampThreads) {
    const unsigned k = fkey(lp[i]);
    if (k >= t0) {
      const int s = atomicAdd(&ncand_s, 1);
      if (s < kCand) {
        ckey[s] = k;
        cidx[s] = i;
      }
    }
  }
  __syncthreads();
  int nc = ncand_s;
  if (nc > kCand) {
    // adversarial row (huge tie / plateau above t0): exact K-th key by a 3-digit MSB radix
    // select with LDS histograms, then gather > threshold plus the lowest-index ties
    unsigned* hst = ckey;  // reuse the candidate buffer as a 2048-bin histogram
    unsigned prefix = 0, mask = 0;
    int kr = K;
    const int shifts[3] = {21, 10, 0}, bits[3] = {11, 11, 10};
    for (int d = 0; d < 3; ++d) {
      const int nb = 1 << bits[d];
      for (int b = tid; b < 2048; b += kSampThreads) hst[b] = 0;
      __syncthreads();
      for (int i = tid; i < V; i += kSampThreads) {
        const unsigned k = fkey(lp[i]);
        if (k > kNegInfKey && (k & mask) == prefix) atomicAdd(&hst[(k >> shifts[d]) & (nb - 1)], 1u);
      }
      __syncthreads();
      // thread t owns bins 2t', 2t'+1 counted from the top (t' = 1023 - t)
      const int hi = 2047 - 2 * tid;
      const float mine = (hi < nb ? (float)hst[hi] : 0.f) + (hi - 1 < nb && hi >= 1 ? (float)hst[hi - 1] : 0.f);
      const float incl = block_scan(mine, wsum);
      const float excl = incl - mine;
      if (excl < kr && incl >= kr) {
        const float c_hi = hi < nb ? (float)hst[hi] : 0.f;
        const int b = (excl + c_hi >= kr) ? hi : hi - 1;
        thr_s = b;
        above_s = (int)(excl + (b == hi ? 0.f : c_hi));  // elements strictly above bin b
      }
      __syncthreads();
      kr -= above_s;
      prefix |= (unsigned)thr_s << shifts[d];
      mask |= (unsigned)(nb - 1) << shifts[d];
      __syncthreads();
    }
    // gather: key > prefix (K - kr of them), then the first kr ties in index order
    if (tid == 0) ncand_s = 0;
    __syncthreads();
    for (int i = tid; i < V; i += kSampThreads) {
      const unsigned k = fkey(lp[i]);
      if (k > prefix) {
        const int s = atomicAdd(&ncand_s, 1);
        ckey[s] = k;
        cidx[s] = i;
      }
    }
    __syncthreads();
    int base = ncand_s, need = kr;
    for (int c0 = 0; c0 < V && need > 0; c0 += kSampThreads) {
      const int i = c0 + tid;
      const bool tie = i < V && fkey(lp[i]) == prefix;
      const int pos = (int)block_scan(tie ? 1.f : 0.f, wsum);  // ties up to and including this lane
      if (tie && pos <= need) {
        ckey[base + pos - 1] = prefix;
        cidx[base + pos - 1] = i;
      }
      if (tid == kSampThreads - 1) thr_s = pos;  // ties in this chunk
      __syncthreads();
      const int taken = min(need, thr_s);
      base += taken;
      need -= taken;
      __syncthreads();
    }
    nc = base;
  }
  // 3. sort the candidates; the first K are the top K
  int n2 = 1;
  while (n2 < nc) n2 <<= 1;
  for (int i = nc + tid; i < n2; i += kSampThreads) {
    ckey[i] = 0;
    cidx[i] = 0x7fffffff;
  }
  __syncthreads();
  bitonic(ckey, cidx, n2);
  const int k_eff = min(K, nc);
  // 4. temperature softmax over the top K, top-p cut, inverse-CDF draw
  int tok;
  if (greedy || k_eff <= 1) {
    tok = k_eff == 0 ? 0 : cidx[0];  // a fully masked row (all -inf) yields id 0
  } else {
    const float v0 = keyf(ckey[0]);
    const float invt = 1.f / temp;
    const float e = tid < k_eff ? __expf((keyf(ckey[tid]) - v0) * invt) : 0.f;
    const float incl = block_scan(e, wsum);
    __shared__ float tot_s, keep_s;
    __shared__ int nkeep_s;
    if (tid == k_eff - 1) tot_s = incl;
    if (tid == 0) nkeep_s = 0;
    __syncthreads();
    const bool keep = tid < k_eff && (incl - e) <= top_p * tot_s;
    if (keep) atomicMax(&nkeep_s, tid + 1);
    __syncthreads();
    if (tid == nkeep_s - 1) keep_s = incl;
    __syncthreads();
    const int hl = reset ? 0 : hist_len[slot];
    // one draw per (request seed, generated-token position): reproducible per request, independent
    // of which batch row or engine step the sequence lands in
    const unsigned hsh = hash3((unsigned)(seed ^ (seed >> 32)), (unsigned)rseed, (unsigned)hl);
    const float u = ((float)(hsh >> 8) + 0.5f) * (1.f / 16777216.f) * keep_s;
    // the first kept i whose inclusive prefix exceeds u
    __shared__ int pick_s;
    if (tid == 0) pick_s = nkeep_s - 1;
    __syncthreads();
    if (tid < nkeep_s && incl > u && (tid == 0 || incl - e <= u)) atomicMin(&pick_s, tid);
    __syncthreads();
    tok = cidx[pick_s];
  }
  // 5. emit + append to the history ring
  if (tid == 0) {
    const int hl = reset ? 0 : hist_len[slot];
    out[row] = tok;
    hist[(long)slot * W + hl % W] = tok;
    hist_len[slot] = hl + 1;
  }
}

int lk_sample(float* logits, long ls, int B, int V, const int* prm, int* hist, int* hist_len, int W,
              unsigned long long seed, int* out, hipStream_t st) {
  if (B <= 0) return 0;
  if (V < 1 || W < 1) return -1;
  const size_t seen_bytes = (size_t)((V + 31) >> 5) * 4;
  if (seen_bytes > 160 * 1024) return -1;  // the LDS "seen" bitmap: V <= 1.3M
  if (seen_bytes > 64 * 1024) {
    LK_SET_MAX_LDS(sample_penalty_kernel, 160 * 1024);
  }
  sample_penalty_kernel<<<B, 256, seen_bytes, st>>>(logits, ls, V, prm, hist, hist_len, W);
  sample_topkp_kernel<<<B, kSampThreads, 0, st>>>(logits, ls, V, prm, hist, hist_len, W, seed, out);
  return 0;
}
