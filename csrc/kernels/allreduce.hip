// Custom all-reduce over xGMI peer memory for tensor-parallel decode collectives.
//
// vLLM runs 2L+1 NCCL all-reduces of [T, hidden] bf16 per
// forward under TP (reference bcg/vllm_agent.py:131,139-142 only sets the TP
// degree).  At decode sizes (100 KiB - 2 MiB) those are latency-bound; RCCL's
// ring is also per-link bound on the fully connected xGMI mesh.  Here every
// rank maps its peers' buffers (hipIpc, dmabuf) and:
//
//   one-shot  : copy input -> own buffer, barrier, each rank reads the full
//               message from every peer over its direct link and reduces
//               locally (ideal for <= ~1 MiB: one hop, n-1 links in parallel);
//   two-shot  : reduce-scatter (rank r reduces slice r from every peer) +
//               all-gather (read the other reduced slices from their owners):
//               2(n-1)/n of the message per rank, spread over all n-1 links;
//   addnorm   : the all-reduce fused with the residual update + RMSNorm that follows
//               the row-parallel o/down projections (one kernel, rows per block), in a
//               one-shot and a two-shot (rows split over the ranks) form.
//
// Hand-off protocol (MI355X_MICROARCH.md "inter-workgroup visibility", at
// system instead of agent scope because the consumer is another GPU):
//   producer: plain stores -> every wave s_waitcnt vmcnt(0) -> barrier ->
//             wave 0: release fence (L2 write-back) -> vmcnt(0) -> relaxed
//             system-scope flag store into each peer's signal buffer;
//   consumer: relaxed system-scope polls of its own flags -> ONE acquire fence
//             (L1/L2 invalidate) -> vmcnt(0) -> barrier -> plain loads.
// Flags are per (phase, block, sender) and carry an epoch kept in device
// memory (advanced by the last block of each call), so the kernels replay
// correctly inside captured HIP graphs.  Data buffers are double-buffered on
// the epoch's parity: a peer can be at most one call ahead, so one barrier
// per phase suffices.  Sums run in fp32 in a fixed rank order -- every rank
// gets bitwise-identical activations.  Every wait has a wall-clock timeout: a
// rank that never arrives sets the error word and the grid still drains.

#include <string.h>

#include "common.h"

namespace {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 128;
constexpr int AR_THREADS = 512;

struct ArSignal {
  uint32_t flags[2][AR_MAX_BLOCKS][AR_MAX_RANKS];  // [phase][block][sender], written by peers
  uint32_t epoch;                                  // calls completed by this rank
  uint32_t done;                                   // blocks finished in the current call
  uint32_t error;                                  // 1 = a barrier timed out
  uint32_t pad[61];
};

struct ArPeers {
  u16x8* data[AR_MAX_RANKS];  // each rank's data buffer, as mapped in this process
  ArSignal* sig[AR_MAX_RANKS];
};

__device__ __forceinline__ uint32_t ar_begin(ArSignal* me) {
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&me->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  return s_epoch;
}

// Every thread calls this after its own stores to the buffer the peers read.
__device__ __forceinline__ void ar_signal(const ArPeers& P, int rank, int world, int phase, uint32_t epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < world && t != rank) {  // lanes of wave 0
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: XCD L2 -> HBM
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&P.sig[t]->flags[phase][blockIdx.x][rank], epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void ar_wait(const ArPeers& P, int rank, int world, int phase, uint32_t epoch,
                                        uint64_t timeout_ticks) {
  const int t = threadIdx.x;
  if (t < WAVE) {
    // once any barrier of this rank timed out the group is broken: do not wait again
    // (the grid drains at once; the host reads the error word after the burst and raises)
    const bool broken = __hip_atomic_load(&P.sig[rank]->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    if (t < world && t != rank && !broken) {
      uint32_t* f = &P.sig[rank]->flags[phase][blockIdx.x][t];
      const uint64_t t0 = wall_clock64();
      // a peer may already be one call ahead: accept any epoch >= ours (wrap-safe)
      while (static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > timeout_ticks) {
          __hip_atomic_store(&P.sig[rank]->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale peer lines (L1 + L2)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__device__ __forceinline__ void ar_end(ArSignal* me) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(&me->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // last block of this call: advance the epoch for the next launch
      __hip_atomic_store(&me->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&me->epoch, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int W>
__device__ __forceinline__ u16x8 ar_sum(const ArPeers& P, int64_t off, int64_t i) {
  u16x8 v[W];
#pragma unroll
  for (int r = 0; r < W; ++r) v[r] = P.data[r][off + i];  // W loads in flight (n-1 links)
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int r = 0; r < W; ++r)  // fixed rank order -> identical bits on every rank
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[r][j]);
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
  return o;
}

// Buffer of every rank: [parity 0: input copy | result][parity 1: input copy | result], cap_vec each.
template <int W>
__global__ __launch_bounds__(AR_THREADS) void ar_oneshot_kernel(ArPeers P, int rank, const u16x8* __restrict__ in,
                                                                u16x8* out, int64_t nvec, int64_t cap_vec,
                                                                uint64_t timeout_ticks) {
  ArSignal* me = P.sig[rank];
  const uint32_t epoch = ar_begin(me);
  const int64_t off = static_cast<int64_t>(epoch & 1u) * 2 * cap_vec;
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per;
  const int64_t hi = lo + per < nvec ? lo + per : nvec;
  u16x8* mine = P.data[rank] + off;
  for (int64_t i = lo + threadIdx.x; i < hi; i += AR_THREADS) mine[i] = in[i];
  ar_signal(P, rank, W, 0, epoch);
  ar_wait(P, rank, W, 0, epoch, timeout_ticks);
  for (int64_t i = lo + threadIdx.x; i < hi; i += AR_THREADS) out[i] = ar_sum<W>(P, off, i);
  ar_end(me);
}

template <int W>
__global__ __launch_bounds__(AR_THREADS) void ar_twoshot_kernel(ArPeers P, int rank, const u16x8* __restrict__ in,
                                                                u16x8* out, int64_t nvec, int64_t cap_vec,
                                                                uint64_t timeout_ticks) {
  ArSignal* me = P.sig[rank];
  const uint32_t epoch = ar_begin(me);
  const int64_t off = static_cast<int64_t>(epoch & 1u) * 2 * cap_vec;
  const int64_t S = (nvec + W - 1) / W;                 // slice (vectors) owned by each rank
  const int64_t per = (S + gridDim.x - 1) / gridDim.x;  // this block's part of every slice
  const int64_t b0 = blockIdx.x * per;
  u16x8* mine = P.data[rank] + off;
  // 1. stage this block's part of every slice
  for (int s = 0; s < W; ++s) {
    const int64_t lo = s * S + b0;
    const int64_t hi = min(min(lo + per, (s + 1) * S), nvec);
    for (int64_t i = lo + threadIdx.x; i < hi; i += AR_THREADS) mine[i] = in[i];
  }
  ar_signal(P, rank, W, 0, epoch);
  ar_wait(P, rank, W, 0, epoch, timeout_ticks);
  // 2. reduce-scatter: my slice from every rank -> my result region (+ my output)
  {
    const int64_t lo = rank * S + b0;
    const int64_t hi = min(min(lo + per, (rank + 1) * S), nvec);
    for (int64_t i = lo + threadIdx.x; i < hi; i += AR_THREADS) {
      const u16x8 o = ar_sum<W>(P, off, i);
      mine[cap_vec + i] = o;
      out[i] = o;
    }
  }
  ar_signal(P, rank, W, 1, epoch);
  ar_wait(P, rank, W, 1, epoch, timeout_ticks);
  // 3. all-gather: the other slices from their owners' result regions
  for (int s = 0; s < W; ++s) {
    if (s == rank) continue;
    const u16x8* src = P.data[s] + off + cap_vec;
    const int64_t lo = s * S + b0;
    const int64_t hi = min(min(lo + per, (s + 1) * S), nvec);
    for (int64_t i = lo + threadIdx.x; i < hi; i += AR_THREADS) out[i] = src[i];
  }
  ar_end(me);
}

// One-shot all-reduce fused with the residual update and RMSNorm of the rows (TP decode:
// the o_proj / down_proj partials of every rank -> residual += sum; h = rmsnorm(residual)).
// A block owns whole rows (rows b, b + nblk, ...), so the row statistics never leave it.
// Roundings follow the unfused pair exactly: sum -> bf16, residual + bf16(sum) -> bf16,
// normalise the stored residual -- bitwise identical to all-reduce + add_rmsnorm.
constexpr int AR_ROW_VECS = 2;  // H <= AR_THREADS * 8 * AR_ROW_VECS = 8192

template <int W>
__global__ __launch_bounds__(AR_THREADS) void ar_oneshot_addnorm_kernel(
    ArPeers P, int rank, const u16x8* __restrict__ in, u16x8* residual, const u16x8* __restrict__ w,
    u16x8* __restrict__ h_out, int rows, int hv /* H / 8 */, float eps, int64_t cap_vec, uint64_t timeout_ticks) {
  __shared__ float s_part[AR_THREADS / WAVE];
  ArSignal* me = P.sig[rank];
  const uint32_t epoch = ar_begin(me);
  const int64_t off = static_cast<int64_t>(epoch & 1u) * 2 * cap_vec;
  u16x8* mine = P.data[rank] + off;
  for (int r = blockIdx.x; r < rows; r += gridDim.x)
    for (int i = threadIdx.x; i < hv; i += AR_THREADS) mine[static_cast<int64_t>(r) * hv + i] = in[static_cast<int64_t>(r) * hv + i];
  ar_signal(P, rank, W, 0, epoch);
  ar_wait(P, rank, W, 0, epoch, timeout_ticks);
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    float v[AR_ROW_VECS][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < AR_ROW_VECS; ++c) {
      const int i = threadIdx.x + c * AR_THREADS;
      if (i < hv) {
        const int64_t e = static_cast<int64_t>(r) * hv + i;
        const u16x8 sum = ar_sum<W>(P, off, e);
        const u16x8 res = residual[e];
        u16x8 nr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nr[j] = f2bf(bf2f(res[j]) + bf2f(sum[j]));
          v[c][j] = bf2f(nr[j]);
          ss += v[c][j] * v[c][j];
        }
        residual[e] = nr;
      }
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < AR_THREADS / WAVE; ++k) tot += s_part[k];
    const float inv = rsqrtf(tot / (hv * 8) + eps);
#pragma unroll
    for (int c = 0; c < AR_ROW_VECS; ++c) {
      const int i = threadIdx.x + c * AR_THREADS;
      if (i < hv) {
        const u16x8 wv = w[i];
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c][j] * inv * bf2f(wv[j]));
        h_out[static_cast<int64_t>(r) * hv + i] = o;
      }
    }
    __syncthreads();  // s_part reused by the next row
  }
  ar_end(me);
}

// Two-shot form of the fused all-reduce + add + RMSNorm (prefill-sized messages): rank r owns
// rows [r S, (r+1) S), S = ceil(rows / W).
//   1. every rank stages its whole partial (block b: rows s S + b + k nblk of every slice s);
//   2. reduce-scatter: the owner sums its rows over every rank (fixed rank order), updates the
//      residual, writes the new residual rows to its result region and normalises them;
//   3. all-gather: every other row's new residual comes from its owner's result region and is
//      normalised locally -- the same bf16 inputs and the same arithmetic as the owner's, so h is
//      bitwise identical on every rank and to the one-shot kernel.
// Link bytes per rank 2 (W-1)/W of the message (one-shot: W-1), spread over all W-1 links.
template <int W>
__device__ __forceinline__ void ar_norm_row(const float (&v)[AR_ROW_VECS][8], float ss, const u16x8* __restrict__ w,
                                            u16x8* __restrict__ h_row, int hv, float eps, float* s_part) {
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < AR_THREADS / WAVE; ++k) tot += s_part[k];
  const float inv = rsqrtf(tot / (hv * 8) + eps);
#pragma unroll
  for (int c = 0; c < AR_ROW_VECS; ++c) {
    const int i = threadIdx.x + c * AR_THREADS;
    if (i < hv) {
      const u16x8 wv = w[i];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c][j] * inv * bf2f(wv[j]));
      h_row[i] = o;
    }
  }
  __syncthreads();  // s_part reused by the next row
}

template <int W>
__global__ __launch_bounds__(AR_THREADS) void ar_twoshot_addnorm_kernel(
    ArPeers P, int rank, const u16x8* __restrict__ in, u16x8* residual, const u16x8* __restrict__ w,
    u16x8* __restrict__ h_out, int rows, int hv /* H / 8 */, float eps, int64_t cap_vec, uint64_t timeout_ticks) {
  __shared__ float s_part[AR_THREADS / WAVE];
  ArSignal* me = P.sig[rank];
  const uint32_t epoch = ar_begin(me);
  const int64_t off = static_cast<int64_t>(epoch & 1u) * 2 * cap_vec;
  u16x8* mine = P.data[rank] + off;
  const int S = (rows + W - 1) / W;
  // 1. stage this block's rows of every slice
  for (int s = 0; s < W; ++s)
    for (int r = s * S + blockIdx.x; r < min((s + 1) * S, rows); r += gridDim.x)
      for (int i = threadIdx.x; i < hv; i += AR_THREADS)
        mine[static_cast<int64_t>(r) * hv + i] = in[static_cast<int64_t>(r) * hv + i];
  ar_signal(P, rank, W, 0, epoch);
  ar_wait(P, rank, W, 0, epoch, timeout_ticks);
  // 2. reduce-scatter + residual update + norm of the owned rows
  for (int r = rank * S + blockIdx.x; r < min((rank + 1) * S, rows); r += gridDim.x) {
    float v[AR_ROW_VECS][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < AR_ROW_VECS; ++c) {
      const int i = threadIdx.x + c * AR_THREADS;
      if (i < hv) {
        const int64_t e = static_cast<int64_t>(r) * hv + i;
        const u16x8 sum = ar_sum<W>(P, off, e);
        const u16x8 res = residual[e];
        u16x8 nr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nr[j] = f2bf(bf2f(res[j]) + bf2f(sum[j]));
          v[c][j] = bf2f(nr[j]);
          ss += v[c][j] * v[c][j];
        }
        residual[e] = nr;
        mine[cap_vec + e] = nr;
      }
    }
    ar_norm_row<W>(v, ss, w, h_out + static_cast<int64_t>(r) * hv, hv, eps, s_part);
  }
  ar_signal(P, rank, W, 1, epoch);
  ar_wait(P, rank, W, 1, epoch, timeout_ticks);
  // 3. all-gather the other slices' new residual rows, normalise them here
  for (int s = 0; s < W; ++s) {
    if (s == rank) continue;
    const u16x8* src = P.data[s] + off + cap_vec;
    for (int r = s * S + blockIdx.x; r < min((s + 1) * S, rows); r += gridDim.x) {
      float v[AR_ROW_VECS][8];
      float ss = 0.f;
#pragma unroll
      for (int c = 0; c < AR_ROW_VECS; ++c) {
        const int i = threadIdx.x + c * AR_THREADS;
        if (i < hv) {
          const int64_t e = static_cast<int64_t>(r) * hv + i;
          const u16x8 nr = src[e];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v[c][j] = bf2f(nr[j]);
            ss += v[c][j] * v[c][j];
          }
          residual[e] = nr;
        }
      }
      ar_norm_row<W>(v, ss, w, h_out + static_cast<int64_t>(r) * hv, hv, eps, s_part);
    }
  }
  ar_end(me);
}

template <int W>
int launch_ar(const ArPeers& P, int rank, const void* in, void* out, int64_t nvec, int64_t cap_vec, int mode,
              int blocks, uint64_t ticks, hipStream_t stream) {
  const u16x8* src = static_cast<const u16x8*>(in);
  u16x8* dst = static_cast<u16x8*>(out);
  if (mode == 1)
    hipLaunchKernelGGL(ar_oneshot_kernel<W>, dim3(blocks), dim3(AR_THREADS), 0, stream, P, rank, src, dst, nvec,
                       cap_vec, ticks);
  else
    hipLaunchKernelGGL(ar_twoshot_kernel<W>, dim3(blocks), dim3(AR_THREADS), 0, stream, P, rank, src, dst, nvec,
                       cap_vec, ticks);
  return BCG_CHECK_LAUNCH();
}

}  // namespace

BCG_API int bcg_ar_limits(int* max_ranks, int* max_blocks, int* signal_bytes) {
  *max_ranks = AR_MAX_RANKS;
  *max_blocks = AR_MAX_BLOCKS;
  *signal_bytes = static_cast<int>(sizeof(ArSignal));
  return 0;
}

// Zeroed data buffer (4 * cap_bytes: two parities x {input copy, result}) + signal block.
BCG_API int bcg_ar_alloc(int64_t cap_bytes, void** data, void** sig) {
  *data = nullptr;
  *sig = nullptr;
  if (cap_bytes <= 0 || cap_bytes % 16) return -2;
  if (hipMalloc(data, 4 * cap_bytes) != hipSuccess) return -1;
  if (hipExtMallocWithFlags(sig, sizeof(ArSignal), hipDeviceMallocUncached) != hipSuccess &&
      hipMalloc(sig, sizeof(ArSignal)) != hipSuccess) {
    (void)hipFree(*data);
    *data = nullptr;
    return -1;
  }
  if (hipMemset(*data, 0, 4 * cap_bytes) != hipSuccess || hipMemset(*sig, 0, sizeof(ArSignal)) != hipSuccess)
    return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

BCG_API int bcg_ar_free(void* p) { return p && hipFree(p) != hipSuccess ? -1 : 0; }

BCG_API int bcg_ar_ipc_handle_size() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

BCG_API int bcg_ar_ipc_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return -1;
  memcpy(out, &h, sizeof(h));
  return 0;
}

BCG_API int bcg_ar_ipc_open(const void* handle, void** p) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : -1;
}

BCG_API int bcg_ar_ipc_close(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : -1; }

// Synchronous read of a rank's error word (1 = some barrier timed out); clears it.
BCG_API int bcg_ar_take_error(void* sig) {
  ArSignal* s = static_cast<ArSignal*>(sig);
  uint32_t err = 0;
  if (hipMemcpy(&err, &s->error, sizeof(err), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (err) {
    const uint32_t zero = 0;
    if (hipMemcpy(&s->error, &zero, sizeof(zero), hipMemcpyHostToDevice) != hipSuccess) return -1;
  }
  return static_cast<int>(err);
}

// Asynchronous copy of a rank's error word into (pinned) host memory on `stream`
// -- queued after a decode burst, read by the host once the burst's event fired.
BCG_API int bcg_ar_error_async(void* sig, void* host, hipStream_t stream) {
  ArSignal* s = static_cast<ArSignal*>(sig);
  return hipMemcpyAsync(host, &s->error, sizeof(uint32_t), hipMemcpyDeviceToHost, stream) == hipSuccess ? 0 : -1;
}

// Sets a rank's error word (tests: the forced-timeout path).
BCG_API int bcg_ar_set_error(void* sig) {
  ArSignal* s = static_cast<ArSignal*>(sig);
  const uint32_t one = 1;
  return hipMemcpy(&s->error, &one, sizeof(one), hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

// Fused all-reduce + residual add + RMSNorm over [rows, H] bf16 (see the kernels): mode 1 =
// one-shot, 2 = two-shot (rows split over the ranks).  Identical bits either way.
BCG_API int bcg_ar_allreduce_addnorm(void* const* data, void* const* sig, int rank, int world, const void* in,
                                     void* residual, const void* weight, void* h_out, int rows, int H, float eps,
                                     int64_t cap_bytes, int blocks, double timeout_s, int mode, hipStream_t stream) {
  if (world < 2 || world > AR_MAX_RANKS || (world & (world - 1)) || rank < 0 || rank >= world) return -2;
  if (rows <= 0 || H % 8 || H > AR_THREADS * 8 * AR_ROW_VECS || static_cast<int64_t>(rows) * H * 2 > cap_bytes)
    return -2;
  if (blocks < 1 || blocks > AR_MAX_BLOCKS || cap_bytes % 16 || (mode != 1 && mode != 2)) return -2;
  ArPeers P{};
  for (int r = 0; r < world; ++r) {
    if (!data[r] || !sig[r]) return -2;
    P.data[r] = static_cast<u16x8*>(data[r]);
    P.sig[r] = static_cast<ArSignal*>(sig[r]);
  }
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  const uint64_t ticks = static_cast<uint64_t>(timeout_s * 1e3 * khz);
  const int64_t cap_vec = cap_bytes / 16;
  const u16x8* src = static_cast<const u16x8*>(in);
  u16x8* res = static_cast<u16x8*>(residual);
  const u16x8* wv = static_cast<const u16x8*>(weight);
  u16x8* ho = static_cast<u16x8*>(h_out);
  const int hv = H / 8;
#define BCG_AR_ADDNORM(WW)                                                                                        \
  if (mode == 1)                                                                                                  \
    hipLaunchKernelGGL(ar_oneshot_addnorm_kernel<WW>, dim3(blocks), dim3(AR_THREADS), 0, stream, P, rank, src, res, \
                       wv, ho, rows, hv, eps, cap_vec, ticks);                                                   \
  else                                                                                                            \
    hipLaunchKernelGGL(ar_twoshot_addnorm_kernel<WW>, dim3(blocks), dim3(AR_THREADS), 0, stream, P, rank, src, res, \
                       wv, ho, rows, hv, eps, cap_vec, ticks);
  switch (world) {
    case 2: BCG_AR_ADDNORM(2) break;
    case 4: BCG_AR_ADDNORM(4) break;
    default: BCG_AR_ADDNORM(8)
  }
#undef BCG_AR_ADDNORM
  return BCG_CHECK_LAUNCH();
}

// n: bf16 elements (multiple of 8); mode 1 = one-shot, 2 = two-shot.
// data/sig: `world` pointers (peer buffers as mapped in this process, own at [rank]).
BCG_API int bcg_ar_allreduce(void* const* data, void* const* sig, int rank, int world, const void* in, void* out,
                             int64_t n, int64_t cap_bytes, int mode, int blocks, double timeout_s,
                             hipStream_t stream) {
  if (world < 2 || world > AR_MAX_RANKS || (world & (world - 1)) || rank < 0 || rank >= world) return -2;
  if (n <= 0 || n % 8 || n * 2 > cap_bytes || cap_bytes % 16) return -2;
  if (blocks < 1 || blocks > AR_MAX_BLOCKS || (mode != 1 && mode != 2)) return -2;
  ArPeers P{};
  for (int r = 0; r < world; ++r) {
    if (!data[r] || !sig[r]) return -2;
    P.data[r] = static_cast<u16x8*>(data[r]);
    P.sig[r] = static_cast<ArSignal*>(sig[r]);
  }
  static int khz = 0;
  if (khz <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  }
  const uint64_t ticks = static_cast<uint64_t>(timeout_s * 1e3 * khz);
  const int64_t nvec = n / 8, cap_vec = cap_bytes / 16;
  switch (world) {
    case 2: return launch_ar<2>(P, rank, in, out, nvec, cap_vec, mode, blocks, ticks, stream);
    case 4: return launch_ar<4>(P, rank, in, out, nvec, cap_vec, mode, blocks, ticks, stream);
    default: return launch_ar<8>(P, rank, in, out, nvec, cap_vec, mode, blocks, ticks, stream);
  }
}
