// K6 brute-force cosine kNN with fused top-k over a corpus resident in HBM.
//
// Semantics follow RagIndex.Cosine / QueryAsync (reference
// Minimal_RAG/Helpers/RagIndex.cs:59-67,124-135): score = dot / (|q|*|c| + 1e-9),
// dimension mismatch is rejected on the host, results ordered by descending score
// with ties kept in corpus (insertion) order — i.e. a stable sort.
//
// Pass 1 (lk_knn_partial): workgroup = 256 corpus rows x 32 queries.  Each wave
// computes two 32x32 score tiles with v_mfma_f32_32x32x16_bf16 (A = corpus rows
// read straight from HBM, B = Q^T from a swizzled LDS image).  The MFMA k-order is
// permuted so every lane streams 64 contiguous bytes of its corpus row per group of
// 4 k-steps (the reduction order of a dot product is free).  Scores are staged in
// LDS and each wave extracts the block-local top-k of 8 queries by k rounds of
// wave-wide (score, index) argmax.
// Pass 2 (lk_knn_merge): one workgroup per query merges nblocks*k candidates with
// the same tie rule.  Sharded (multi-GPU) search reuses pass 2 on all-gathered
// candidates.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int ROWS = 256;  // corpus rows per workgroup
constexpr int QT = 32;     // queries per workgroup

// (score desc, index asc) ordering
LK_DEVICE bool better(float s1, int i1, float s2, int i2) {
  return s1 > s2 || (s1 == s2 && (unsigned)i1 < (unsigned)i2);
}

LK_DEVICE void wave_argmax(float& s, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float s2 = __shfl_xor(s, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (better(s2, i2, s, i)) {
      s = s2;
      i = i2;
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void knn_partial_kernel(
    const bf16_t* __restrict__ corpus, const float* __restrict__ cnorm, long N,
    const bf16_t* __restrict__ queries, const float* __restrict__ qnorm, int nq, int K,
    float* __restrict__ part_s, int* __restrict__ part_i, int nblocks) {
  constexpr int CPR = D / 8;  // 16-B chunks per row
  constexpr int NG = D / 64;  // groups of 4 k-steps
  // one LDS buffer: the Q tile during the MFMA phase, then (after a barrier) the score
  // tile for the top-k phase -- max(QT*D*2, QT*(ROWS+1)*4) bytes instead of the sum,
  // so 2-3 workgroups fit per CU
  constexpr int QBYTES = QT * D * 2, SBYTES = QT * (ROWS + 1) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[QBYTES > SBYTES ? QBYTES : SBYTES];
  bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);
  float(*sc)[ROWS + 1] = reinterpret_cast<float(*)[ROWS + 1]>(smem);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int qbase = blockIdx.y * QT;
  const long row0 = (long)blockIdx.x * ROWS;

  // stage Q tile (zero-padded) with chunk swizzle c ^ (row & 15)
  for (int c = tid; c < QT * CPR; c += 256) {
    const int qr = c / CPR, ch = c % CPR;
    short8 v = short8{0, 0, 0, 0, 0, 0, 0, 0};
    if (qbase + qr < nq) v = *reinterpret_cast<const short8*>(queries + (long)(qbase + qr) * D + ch * 8);
    *reinterpret_cast<short8*>(Qs + qr * D + (ch ^ (qr & 15)) * 8) = v;
  }
  __syncthreads();

  // k-step (4g+u), element j  <->  d = 64g + 32h + 8u + j
  floatx16 acc2[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const long doc = row0 + w * 64 + m * 32 + r;
    const long docc = doc < N ? doc : N - 1;
    const bf16_t* cp = corpus + docc * D + 32 * h;
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll 2
    for (int g = 0; g < NG; ++g) {
      short8 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const short8*>(cp + 64 * g + 8 * u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ch = 8 * g + 4 * h + u;
        const short8 bq = *reinterpret_cast<const short8*>(Qs + r * D + (ch ^ (r & 15)) * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], bq, acc, 0, 0, 0);
      }
    }
    acc2[m] = acc;
  }
  __syncthreads();  // every wave done with Qs: the buffer becomes the score tile
  // C[row = doc (i&3)+8(i>>2)+4h][col = query r]
  const float qn = (qbase + r < nq) ? qnorm[qbase + r] : 1.f;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int lr = w * 64 + m * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      const long d = row0 + lr;
      sc[r][lr] = d < N ? acc2[m][i] / (qn * cnorm[d] + 1e-9f) : -INFINITY;
    }
  }
  __syncthreads();

  // block-local top-k: wave w handles queries w, w+4, ...
  for (int qq = w; qq < QT; qq += 4) {
    if (qbase + qq >= nq) break;
    float v[ROWS / 64];
#pragma unroll
    for (int j = 0; j < ROWS / 64; ++j) v[j] = sc[qq][lane + 64 * j];
    float* ps = part_s + ((long)(qbase + qq) * nblocks + blockIdx.x) * K;
    int* pi = part_i + ((long)(qbase + qq) * nblocks + blockIdx.x) * K;
    for (int kk = 0; kk < K; ++kk) {
      float bs = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < ROWS / 64; ++j) {
        const int idx = (int)(row0 + lane + 64 * j);
        if (better(v[j], idx, bs, bi)) {
          bs = v[j];
          bi = idx;
        }
      }
      wave_argmax(bs, bi);
      if (lane == 0) {
        ps[kk] = bs;
        pi[kk] = bs == -INFINITY ? -1 : bi;
      }
#pragma unroll
      for (int j = 0; j < ROWS / 64; ++j)
        if ((int)(row0 + lane + 64 * j) == bi) v[j] = -INFINITY;
    }
  }
}

// Top-k over precomputed dot products (scores [nq, ld] from the weight-streaming GEMM,
// csrc/skinny_gemm.hip lk_ws_scores_f32): one workgroup per (chunk of 4096 rows, query)
// normalises dot / (|q| |c| + 1e-9) and extracts the chunk's top-k (score desc, index
// asc) by k rounds of block-wide argmax.
constexpr int SCH = 4096;

__global__ __launch_bounds__(256) void score_topk_kernel(const float* __restrict__ scores, long ld,
                                                         const float* __restrict__ cnorm,
                                                         const float* __restrict__ qnorm, long N, int K,
                                                         float* __restrict__ part_s, int* __restrict__ part_i,
                                                         int nchunks) {
  __shared__ float rs[4];
  __shared__ int ri[4];
  const int q = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int PER = SCH / 256;
  const long base = (long)c * SCH;
  const float qn = qnorm[q];
  float v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const long d = base + j * 256 + tid;
    v[j] = d < N ? scores[(long)q * ld + d] / (qn * cnorm[d] + 1e-9f) : -INFINITY;
  }
  float* ps = part_s + ((long)q * nchunks + c) * K;
  int* pi = part_i + ((long)q * nchunks + c) * K;
  for (int kk = 0; kk < K; ++kk) {
    float bs = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = (int)(base + j * 256 + tid);
      if (better(v[j], idx, bs, bi)) {
        bs = v[j];
        bi = idx;
      }
    }
    wave_argmax(bs, bi);
    if (lane == 0) {
      rs[w] = bs;
      ri[w] = bi;
    }
    __syncthreads();
    float fs = rs[0];
    int fi = ri[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (better(rs[j], ri[j], fs, fi)) {
        fs = rs[j];
        fi = ri[j];
      }
    if (tid == 0) {
      ps[kk] = fs;
      pi[kk] = fs == -INFINITY ? -1 : fi;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if ((int)(base + j * 256 + tid) == fi) v[j] = -INFINITY;
    __syncthreads();
  }
}

// merge: one workgroup per query over `ncand` (score, idx) candidates
__global__ __launch_bounds__(256) void knn_merge_kernel(const float* __restrict__ cs,
                                                        const int* __restrict__ ci, int ncand,
                                                        int K, float* __restrict__ out_s,
                                                        int* __restrict__ out_i) {
  __shared__ float rs[4];
  __shared__ int ri[4];
  __shared__ int last;
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* s = cs + (long)q * ncand;
  const int* ix = ci + (long)q * ncand;
  float prev_s = INFINITY;
  int prev_i = -1;
  for (int kk = 0; kk < K; ++kk) {
    // best candidate strictly "worse" than the previous winner
    float bs = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = tid; c < ncand; c += 256) {
      const float v = s[c];
      const int id = ix[c];
      if (id < 0) continue;
      if (kk > 0 && !better(prev_s, prev_i, v, id)) continue;
      if (better(v, id, bs, bi)) {
        bs = v;
        bi = id;
      }
    }
    wave_argmax(bs, bi);
    if (lane == 0) {
      rs[w] = bs;
      ri[w] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      float fs = rs[0];
      int fi = ri[0];
      for (int j = 1; j < 4; ++j)
        if (better(rs[j], ri[j], fs, fi)) {
          fs = rs[j];
          fi = ri[j];
        }
      out_s[(long)q * K + kk] = fs;
      out_i[(long)q * K + kk] = fi == 0x7fffffff ? -1 : fi;
      rs[0] = fs;
      ri[0] = fi;
    }
    __syncthreads();
    prev_s = rs[0];
    prev_i = ri[0];
    __syncthreads();
  }
  (void)last;
}

}  // namespace

int lk_knn_nblocks(long N) { return (int)((N + ROWS - 1) / ROWS); }

int lk_knn_partial(const bf16_t* corpus, const float* cnorm, long N, int D, const bf16_t* queries,
                   const float* qnorm, int nq, int K, float* part_s, int* part_i,
                   hipStream_t st) {
  if (N <= 0 || nq <= 0) return 0;
  if (K < 1 || K > 64) return -1;
  const int nb = lk_knn_nblocks(N);
  dim3 grid(nb, (nq + QT - 1) / QT);
  switch (D) {
    case 128: knn_partial_kernel<128><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    case 256: knn_partial_kernel<256><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    case 512: knn_partial_kernel<512><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    case 384: knn_partial_kernel<384><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    case 768: knn_partial_kernel<768><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    case 1024: knn_partial_kernel<1024><<<grid, 256, 0, st>>>(corpus, cnorm, N, queries, qnorm, nq, K, part_s, part_i, nb); break;
    default: return -2;
  }
  return 0;
}

int lk_knn_score_chunks(long N) { return (int)((N + SCH - 1) / SCH); }

int lk_knn_score_topk(const float* scores, long ld, const float* cnorm, const float* qnorm, long N, int nq, int K,
                      float* part_s, int* part_i, hipStream_t st) {
  if (N <= 0 || nq <= 0) return 0;
  if (K < 1 || K > 64) return -1;
  const int nc = lk_knn_score_chunks(N);
  score_topk_kernel<<<dim3(nc, nq), 256, 0, st>>>(scores, ld, cnorm, qnorm, N, K, part_s, part_i, nc);
  return 0;
}

int lk_knn_merge(const float* cand_s, const int* cand_i, int nq, int ncand, int K, float* out_s,
                 int* out_i, hipStream_t st) {
  if (nq <= 0) return 0;
  knn_merge_kernel<<<nq, 256, 0, st>>>(cand_s, cand_i, ncand, K, out_s, out_i);
  return 0;
}
