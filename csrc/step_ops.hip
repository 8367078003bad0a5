// Small per-step data movement of the engine's forward, so a steady-state step runs no
// framework (at::native) kernels: the embedding gather from int32 token ids (vocab-parallel
// masked form included), the in-flight decode-id gather of pipelined steps, and the row gather
// of the hidden states that feed the LM head.  Each is one launch of 16-B vector copies.
#include "common.h"
#include "kernels.h"

// token ids outside a whole (non-sharded) table since the last lk_embed_errors() read: a bad id
// must not pass as a silent zero embedding (the engine polls this with the GEMM health check)
__device__ int g_embed_bad_ids = 0;

namespace {

// out[t, :] = table[ids[t] - lo, :] if lo <= ids[t] < lo + n_local else 0   (row of H bf16);
// strict (the whole table, no vocab shard): an id outside it is also counted in g_embed_bad_ids
__global__ __launch_bounds__(256) void embed_rows_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ table,
                                                         const int* __restrict__ ids, long T, int H, long lo,
                                                         long n_local, int strict) {
  const int vpr = H >> 3;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= T * vpr) return;
  const long t = i / vpr;
  const int c = (int)(i - t * vpr);
  const long id = (long)ids[t] - lo;
  uint4_t v = {0u, 0u, 0u, 0u};
  if (id >= 0 && id < n_local) v = *reinterpret_cast<const uint4_t*>(table + id * H + c * 8);
  else if (strict && c == 0) atomicAdd(&g_embed_bad_ids, 1);
  *reinterpret_cast<uint4_t*>(out + t * H + c * 8) = v;
}

// ids[dst[i]] = prev[src[i]]
__global__ __launch_bounds__(256) void scatter_ids_kernel(int* __restrict__ ids, const long* __restrict__ dst,
                                                          const int* __restrict__ prev, const long* __restrict__ src,
                                                          int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) ids[dst[i]] = prev[src[i]];
}

// out[r, :] = x[idx[r], :]  (rows of H bf16, x row stride xs)
__global__ __launch_bounds__(256) void gather_rows_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                          long xs, const long* __restrict__ idx, long R, int H) {
  const int vpr = H >> 3;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * vpr) return;
  const long r = i / vpr;
  const int c = (int)(i - r * vpr);
  *reinterpret_cast<uint4_t*>(out + r * H + c * 8) = *reinterpret_cast<const uint4_t*>(x + idx[r] * xs + c * 8);
}

}  // namespace

int lk_embed_rows(bf16_t* out, const bf16_t* table, const int* ids, long T, int H, long lo, long n_local,
                  hipStream_t st, int strict) {
  if (H % 8 || T < 0) return -1;
  if (T == 0) return 0;
  const long n = T * (H / 8);
  embed_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(out, table, ids, T, H, lo, n_local, strict);
  return 0;
}

// ids outside the table counted by strict embed_rows launches on the CURRENT device since the
// last call for that device.  The device counter only grows (no read-then-reset race with a
// kernel incrementing it in between); the host keeps the last value it saw per device.
int lk_embed_errors() {
  static int last[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
  int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_embed_bad_ids), sizeof(int)) != hipSuccess) return -1;
  const int d = v - last[dev];  // (wraps only after 2^31 bad ids)
  last[dev] = v;
  return d;
}

int lk_scatter_ids(int* ids, const long* dst, const int* prev, const long* src, int n, hipStream_t st) {
  if (n < 0) return -1;
  if (n == 0) return 0;
  scatter_ids_kernel<<<(n + 255) / 256, 256, 0, st>>>(ids, dst, prev, src, n);
  return 0;
}

int lk_gather_rows(bf16_t* out, const bf16_t* x, long xs, const long* idx, long R, int H, hipStream_t st) {
  if (H % 8 || xs % 8 || R < 0) return -1;
  if (R == 0) return 0;
  const long n = R * (H / 8);
  gather_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(out, x, xs, idx, R, H);
  return 0;
}
