// K14: one-shot all-reduce over xGMI peer memory (HIP IPC), for the latency-bound
// tensor-parallel decode all-reduces (B x hidden bf16, ~16 KiB per token row).
//
// RCCL's ring is per-link bound and pays several protocol hops per call; at decode
// sizes (<= a few MB) one pass that reads every peer's buffer directly over its own
// xGMI link (7 links per MI355X, full mesh) is latency-optimal:
//   1. every rank copies its input slice into its own IPC-exported staging buffer;
//   2. barrier-in: each workgroup publishes its slice (system-scope release, then a
//      relaxed system-scope flag store into EVERY peer's signal buffer) and polls its
//      own signal buffer until every peer's matching workgroup has published;
//   3. system-scope acquire, then each workgroup sums its slice over all ranks' staging
//      buffers (f32 accumulation in rank order -> bitwise identical on every rank) and
//      writes the bf16 result (in place is fine: a slice is read before it is written);
//   4. barrier-out: the same handshake on a second flag set, so no rank overwrites its
//      staging buffer (next call) while a peer may still be reading it.
// The TP decode layer's fused form (xgmi_ar_rmsnorm_kernel): the row-parallel o / down
// partial sums are all-reduced, added to the residual stream and RMS-normalised in the SAME
// kernel -- each workgroup owns whole rows, so after the handshake it sums its rows over the
// ranks, rounds them to bf16 (the plain all-reduce's output), adds the residual, writes the
// new residual and the normed row: bit-identical to all-reduce -> rmsnorm(x, residual) with
// one launch and one pass over the rows instead of three.
// Two-shot form (xgmi_ar2_kernel, prefill-sized messages): one-shot reads the WHOLE message
// from every peer, i.e. S bytes over each of the 7 links; two-shot is a reduce-scatter then an
// all-gather through the same peer mappings -- rank r sums only its 1/world row slice over
// the ranks (S/world per link), publishes the bf16 slice in its second IPC region, and after a
// second handshake every rank reads each owner's reduced slice (S/world per link again):
// 2S/world per link in total, 4x less than one-shot on 8 ranks.  The residual + RMSNorm tail
// runs on the gathered rows in the same kernel, and the sums are rounded exactly where the
// one-shot kernel rounds them (bf16 after the rank-order f32 sum), so the two forms are
// bit-identical.  Every cross-rank read of a row is between workgroups of the SAME index
// (workgroup b stages, reduces and gathers rows o*n + [j0(b), j1(b)) of every owner o), so the
// per-workgroup handshakes order everything.
// Flags are per-workgroup monotonic epochs kept in device memory (one counter per
// workgroup, advanced by the kernel itself), so a captured hipGraph replays correctly
// with no host-side state.  Every spin is bounded: a peer that never arrives sets the
// error word and the kernel exits instead of hanging the device.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "rowcfg.h"

namespace {

constexpr int kMaxRanks = 8;
constexpr int kArBlocks = 256;   // max workgroups per call (the plain all-reduce uses <= 32 slices; the fused
                                 // all-reduce + RMSNorm one row per workgroup up to 256 rows)
constexpr int kArSlices = 32;    // workgroups of the plain all-reduce
constexpr int kArThreads = 512;
// signal buffer (uncached): [3 phases][kArBlocks][kMaxRanks] flags + [kArBlocks] epoch counters
// (one-shot kernels use phases 0 / 1, the two-shot kernel 0 / 1 / 2)
constexpr int kPhases = 3;
constexpr int kSigWords = kPhases * kArBlocks * kMaxRanks + kArBlocks;
constexpr unsigned kSpinLimit = 1u << 22;  // ~4 s of polling: a decode all-reduce waits us, not s

struct ArPeers {
  bf16_t* data[kMaxRanks];
  unsigned* sig[kMaxRanks];
};

LK_DEVICE unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
LK_DEVICE void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane t < world: signal peer t's slot [phase][blk][rank], then wait for our own slot
// [phase][blk][t] to reach this call's epoch; false on timeout (error word set)
LK_DEVICE bool handshake(const ArPeers& p, int rank, int world, int phase, unsigned epoch, int* err) {
  const int t = threadIdx.x;
  int ok = 1;
  if (t < world) {
    st_sys(p.sig[t] + (phase * kArBlocks + blockIdx.x) * kMaxRanks + rank, epoch);
    const unsigned* mine = p.sig[rank] + (phase * kArBlocks + blockIdx.x) * kMaxRanks + t;
    unsigned spins = 0;
    while ((int)(ld_sys(mine) - epoch) < 0) {
      if (++spins > kSpinLimit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return __syncthreads_and(ok) != 0;
}

__global__ __launch_bounds__(kArThreads) void xgmi_allreduce_kernel(ArPeers p, int rank, int world,
                                                                    const bf16_t* __restrict__ in,
                                                                    bf16_t* __restrict__ out, long n, int* err) {
  const long nv = n >> 3;  // 16-B vectors
  const long per = (nv + gridDim.x - 1) / gridDim.x;
  const long v0 = (long)blockIdx.x * per, v1 = min(nv, v0 + per);
  unsigned* ctr = p.sig[rank] + kPhases * kArBlocks * kMaxRanks + blockIdx.x;
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) {
    s_epoch = *ctr + 1;  // only this workgroup of this rank touches its counter
    *ctr = s_epoch;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;

  // 1. stage this slice
  bf16_t* mine = p.data[rank];
  for (long v = v0 + threadIdx.x; v < v1; v += kArThreads)
    *reinterpret_cast<short8*>(mine + v * 8) = *reinterpret_cast<const short8*>(in + v * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: staged bytes reach memory
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 2. barrier-in
  if (!handshake(p, rank, world, 0, epoch, err)) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 3. reduce the slice over all ranks, same order everywhere
  for (long v = v0 + threadIdx.x; v < v1; v += kArThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      float x[8];
      load8(p.data[r] + v * 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    store8(out + v * 8, acc);
  }
  __syncthreads();
  // 4. barrier-out: every peer finished reading our staging buffer
  handshake(p, rank, world, 1, epoch, err);
}

// Stage the block's rows, handshake, then per row: x = bf16(sum over ranks in rank order),
// res = bf16(x + res) (written back), out = bf16(bf16(res * rsqrt(mean(res^2) + eps)) * w).
// The thread -> column slicing and the reduction order are rmsnorm_kernel's (rowcfg.h).
template <int MAXV, int NW>
__global__ __launch_bounds__(NW * 64) void xgmi_ar_rmsnorm_kernel(ArPeers p, int rank, int world,
                                                                   const bf16_t* __restrict__ in,
                                                                   bf16_t* __restrict__ residual,
                                                                   const bf16_t* __restrict__ w,
                                                                   bf16_t* __restrict__ out, int T, int H, float eps,
                                                                   int* err) {
  __shared__ float red[NW];
  __shared__ unsigned s_epoch;
  const int nb = gridDim.x;
  const int r0 = (int)((long)blockIdx.x * T / nb), r1 = (int)((long)(blockIdx.x + 1) * T / nb);
  unsigned* ctr = p.sig[rank] + kPhases * kArBlocks * kMaxRanks + blockIdx.x;
  if (threadIdx.x == 0) {
    s_epoch = *ctr + 1;
    *ctr = s_epoch;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const int nvec = H >> 3;
  // 1. stage this block's rows
  bf16_t* mine = p.data[rank];
  for (long v = (long)r0 * nvec + threadIdx.x; v < (long)r1 * nvec; v += NW * 64)
    *reinterpret_cast<short8*>(mine + v * 8) = *reinterpret_cast<const short8*>(in + v * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 2. barrier-in: every peer staged the same rows
  if (!handshake(p, rank, world, 0, epoch, err)) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 3. reduce + residual + RMSNorm, row by row
  for (int row = r0; row < r1; ++row) {
    float v[MAXV][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = threadIdx.x + i * NW * 64;
      if (c < nvec) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < world; ++r) {
          float x[8];
          load8(p.data[r] + (long)row * H + c * 8, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += x[j];
        }
        float rr[8];
        bf16_t* rp = residual + (long)row * H + c * 8;
        load8(rp, rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(acc[j])) + rr[j];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j]));
        store8(rp, v[i]);
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
        store8(out + (long)row * H + c * 8, y);
      }
    }
  }
  __syncthreads();
  // 4. barrier-out: every peer finished reading this block's rows of our staging buffer
  handshake(p, rank, world, 1, epoch, err);
}

// system-scope publish / acquire around a handshake (staged or reduced bytes of this
// workgroup visible to the peers; theirs visible here)
LK_DEVICE void publish() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
LK_DEVICE void acquire() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// Two-shot all-reduce (NORM = false: out = allreduce(in)) or all-reduce + residual + RMSNorm
// (NORM = true: residual += allreduce(in) rounded to bf16, out = RMSNorm(residual) * w).
// red_off: element offset of the reduced-slice region inside every rank's staging buffer.
template <int MAXV, int NW, bool NORM>
__global__ __launch_bounds__(NW * 64) void xgmi_ar2_kernel(ArPeers p, long red_off, int rank, int world,
                                                           const bf16_t* __restrict__ in,
                                                           bf16_t* __restrict__ residual,
                                                           const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
                                                           int T, int H, float eps, int* err) {
  __shared__ float red[NW];
  __shared__ unsigned s_epoch;
  constexpr int NT = NW * 64;
  const int n = (T + world - 1) / world;  // rows per owner slice
  const int j0 = (int)((long)blockIdx.x * n / gridDim.x), j1 = (int)((long)(blockIdx.x + 1) * n / gridDim.x);
  unsigned* ctr = p.sig[rank] + kPhases * kArBlocks * kMaxRanks + blockIdx.x;
  if (threadIdx.x == 0) {
    s_epoch = *ctr + 1;
    *ctr = s_epoch;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const int nvec = H >> 3;
  bf16_t* mine = p.data[rank];
  auto rows_of = [&](int o, int* ra, int* rb) {
    *ra = min(T, o * n + j0);
    *rb = min(T, o * n + j1);
  };
  // 1. stage this workgroup's rows of every owner slice
  for (int o = 0; o < world; ++o) {
    int ra, rb;
    rows_of(o, &ra, &rb);
    for (long v = (long)ra * nvec + threadIdx.x; v < (long)rb * nvec; v += NT)
      *reinterpret_cast<short8*>(mine + v * 8) = *reinterpret_cast<const short8*>(in + v * 8);
  }
  publish();
  if (!handshake(p, rank, world, 0, epoch, err)) return;
  acquire();
  // 2. reduce-scatter: this rank's slice rows, f32 sum in rank order -> bf16 into the reduced region
  {
    int ra, rb;
    rows_of(rank, &ra, &rb);
    for (long v = (long)ra * nvec + threadIdx.x; v < (long)rb * nvec; v += NT) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < world; ++r) {
        float x[8];
        load8(p.data[r] + v * 8, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      }
      store8(mine + red_off + v * 8, acc);
    }
  }
  publish();
  if (!handshake(p, rank, world, 1, epoch, err)) return;
  acquire();
  // 3. all-gather each owner's reduced rows (+ residual + RMSNorm)
  for (int o = 0; o < world; ++o) {
    int ra, rb;
    rows_of(o, &ra, &rb);
    const bf16_t* src = p.data[o] + red_off;
    if constexpr (!NORM) {
      for (long v = (long)ra * nvec + threadIdx.x; v < (long)rb * nvec; v += NT)
        *reinterpret_cast<short8*>(out + v * 8) = *reinterpret_cast<const short8*>(src + v * 8);
    } else {
      for (int row = ra; row < rb; ++row) {
        float v[MAXV][8];
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
          const int c = threadIdx.x + i * NT;
          if (c < nvec) {
            float x[8], rr[8];
            load8(src + (long)row * H + c * 8, x);
            bf16_t* rp = residual + (long)row * H + c * 8;
            load8(rp, rr);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(x[j] + rr[j]));
            store8(rp, v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
          }
        }
        ss = block_sum<NW>(ss, red);
        const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
          const int c = threadIdx.x + i * NT;
          if (c < nvec) {
            float g[8], y[8];
            load8(w + c * 8, g);
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = bf2f(f2bf(v[i][j] * inv)) * g[j];
            store8(out + (long)row * H + c * 8, y);
          }
        }
      }
    }
  }
  __syncthreads();
  // 4. barrier-out: every peer finished reading this workgroup's staged and reduced rows
  handshake(p, rank, world, 2, epoch, err);
}

// All-gather / broadcast of raw bytes through the same peer mappings (a TP group that runs every
// collective on the IPC path -- e.g. several ranks on one device, where RCCL refuses a
// communicator): root < 0: every rank stages its nv 16-B vectors, handshake, each workgroup copies
// its slice of EVERY rank's part into out[r * nv ..], barrier-out; root >= 0: broadcast -- only
// root stages, every rank copies root's part into out (root's own out may alias in).
__global__ __launch_bounds__(kArThreads) void xgmi_gather_kernel(ArPeers p, int rank, int world, int root,
                                                                 const uint4_t* __restrict__ in, uint4_t* out, long nv,
                                                                 int* err) {
  const long per = (nv + gridDim.x - 1) / gridDim.x;
  const long v0 = (long)blockIdx.x * per, v1 = min(nv, v0 + per);
  unsigned* ctr = p.sig[rank] + kPhases * kArBlocks * kMaxRanks + blockIdx.x;
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) {
    s_epoch = *ctr + 1;
    *ctr = s_epoch;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  uint4_t* mine = reinterpret_cast<uint4_t*>(p.data[rank]);
  if (root < 0 || rank == root)
    for (long v = v0 + threadIdx.x; v < v1; v += kArThreads) mine[v] = in[v];
  publish();
  if (!handshake(p, rank, world, 0, epoch, err)) return;
  acquire();
  if (root < 0) {
    for (int r = 0; r < world; ++r) {
      const uint4_t* src = reinterpret_cast<const uint4_t*>(p.data[r]);
      for (long v = v0 + threadIdx.x; v < v1; v += kArThreads) out[r * nv + v] = src[v];
    }
  } else if (rank != root || out != in) {
    const uint4_t* src = reinterpret_cast<const uint4_t*>(p.data[root]);
    for (long v = v0 + threadIdx.x; v < v1; v += kArThreads) out[v] = src[v];
  }
  __syncthreads();
  handshake(p, rank, world, 1, epoch, err);  // every peer finished reading our staged part
}

// workgroups per call cap (LK_XGMI_AR_BLOCKS, default kArBlocks): several ranks sharing ONE
// device (the single-GPU multi-rank tests) need every rank's spinning workgroups co-resident;
// every rank must use the same value (the per-workgroup epochs are indexed by block)
int block_cap() {
  static const int cap = [] {
    const char* e = getenv("LK_XGMI_AR_BLOCKS");
    const int v = e ? atoi(e) : kArBlocks;
    return v < 1 ? 1 : (v > kArBlocks ? kArBlocks : v);
  }();
  return cap;
}

}  // namespace

// out = RMSNorm(allreduce(in) + residual) * w, residual updated in place; in / residual / out
// [T, H] contiguous, T * H * 2 <= staging bytes (checked by the caller).  Same launch on every
// rank (block count depends on T only), so the per-block epochs stay in step with the plain
// all-reduce's.
int lk_xgmi_allreduce_rmsnorm(bf16_t* const* data, unsigned* const* sig, int rank, int world, const bf16_t* in,
                              bf16_t* residual, const bf16_t* w, bf16_t* out, int T, int H, float eps, int* err,
                              hipStream_t st) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || H % 8 || T < 0) return -1;
  if (T == 0) return 0;
  ArPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.sig[r] = sig[r];
  }
  const int blocks = std::min(block_cap(), T);
#define CALL(MV, NW) \
  xgmi_ar_rmsnorm_kernel<MV, NW><<<blocks, NW * 64, 0, st>>>(p, rank, world, in, residual, w, out, T, H, eps, err)
  ROW_DISPATCH(H, CALL);
#undef CALL
  LK_CHECK_LAUNCH();
  return 0;
}

// Two-shot forms (reduce-scatter + all-gather through the peer mappings): in / out [T, H]
// bf16 contiguous; norm != 0 also applies residual += sum, out = RMSNorm(residual) * w.
// red_off: element offset of the reduced region in every staging buffer (T * H <= red_off and
// the region as large, checked by the caller).  Same launch on every rank (depends on T, world).
int lk_xgmi_allreduce2(bf16_t* const* data, unsigned* const* sig, long red_off, int rank, int world,
                       const bf16_t* in, bf16_t* residual, const bf16_t* w, bf16_t* out, int T, int H, float eps,
                       int norm, int* err, hipStream_t st) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || H % 8 || T < 0) return -1;
  if (norm && (residual == nullptr || w == nullptr)) return -1;
  if (T == 0) return 0;
  ArPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.sig[r] = sig[r];
  }
  const int n = (T + world - 1) / world;
  const int blocks = std::min(block_cap(), n);
#define CALL(MV, NW)                                                                                              \
  if (norm)                                                                                                       \
    xgmi_ar2_kernel<MV, NW, true><<<blocks, NW * 64, 0, st>>>(p, red_off, rank, world, in, residual, w, out, T, H, \
                                                             eps, err);                                          \
  else                                                                                                            \
    xgmi_ar2_kernel<MV, NW, false><<<blocks, NW * 64, 0, st>>>(p, red_off, rank, world, in, residual, w, out, T, \
                                                              H, eps, err)
  ROW_DISPATCH(H, CALL);
#undef CALL
  LK_CHECK_LAUNCH();
  return 0;
}

int lk_xgmi_ar_sig_words() { return kSigWords; }
int lk_xgmi_ar_max_ranks() { return kMaxRanks; }

// data[r] / sig[r]: rank r's staging and signal buffers as mapped in THIS process (own ones
// included).  n bf16 elements, n % 8 == 0, n * 2 <= staging bytes (checked by the caller).
int lk_xgmi_allreduce(bf16_t* const* data, unsigned* const* sig, int rank, int world, const bf16_t* in,
                      bf16_t* out, long n, int* err, hipStream_t st) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || n % 8) return -1;
  if (n == 0) return 0;
  ArPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.sig[r] = sig[r];
  }
  const long nv = n / 8;
  const int blocks = (int)std::min<long>(std::min(kArSlices, block_cap()), std::max<long>(1, (nv + kArThreads - 1) / kArThreads));
  xgmi_allreduce_kernel<<<blocks, kArThreads, 0, st>>>(p, rank, world, in, out, n, err);
  LK_CHECK_LAUNCH();
  return 0;
}

// nbytes % 16 == 0, nbytes <= staging bytes (checked by the caller); out holds world * nbytes
// (all-gather, root < 0) or nbytes (broadcast from root).  Same launch on every rank.
int lk_xgmi_gather(bf16_t* const* data, unsigned* const* sig, int rank, int world, int root, const void* in,
                   void* out, long nbytes, int* err, hipStream_t st) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || root >= world || nbytes % 16) return -1;
  if (nbytes == 0) return 0;
  ArPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.sig[r] = sig[r];
  }
  const long nv = nbytes / 16;
  const int blocks = (int)std::min<long>(std::min(kArSlices, block_cap()), std::max<long>(1, (nv + kArThreads - 1) / kArThreads));
  xgmi_gather_kernel<<<blocks, kArThreads, 0, st>>>(p, rank, world, root, reinterpret_cast<const uint4_t*>(in),
                                                     reinterpret_cast<uint4_t*>(out), nv, err);
  LK_CHECK_LAUNCH();
  return 0;
}
