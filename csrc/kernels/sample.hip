// Fused guided-decoding step: JSON-FSM mask + temperature + Gumbel-max sampling
// + FSM advance + per-row bookkeeping, one workgroup (1024 threads) per row.
//
// For row b (skipped when done[b]):
//   allowed(t) = fsm_next[fsm_base+state][t] >= 0            (guided rows)
//              = t < n_text || t in {eos, eos2}                (free-text rows)
//   budget mode: also require dist[base+next(t)] <= remaining-1 whenever some
//   allowed token satisfies it (the JSON can always be closed in time).
//   token = argmax_allowed( logit/T + Gumbel(hash(seed, row_key, step, t)) ),
//   greedy when T <= 0.  The hash is ops/reference.py:gumbel_hash bit for bit.
// The int16 FSM row and the bf16 logits are read once with 16-byte loads.
// Two argmax candidates (budget-tight / any-allowed) are reduced per wave by
// shuffles and across the 16 waves through LDS.

#include "common.h"

namespace {

constexpr int SAMPLE_THREADS = 1024;

struct Cand {
  float score;
  int idx;
};

__device__ __forceinline__ void better(Cand& a, float s, int i) {
  if (s > a.score || (s == a.score && i < a.idx)) {
    a.score = s;
    a.idx = i;
  }
}

__device__ __forceinline__ Cand wave_argmax(Cand c) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float s = __shfl_xor(c.score, o, WAVE);
    const int i = __shfl_xor(c.idx, o, WAVE);
    better(c, s, i);
  }
  return c;
}

__global__ __launch_bounds__(SAMPLE_THREADS) void guided_sample_kernel(
    const bf16_t* __restrict__ logits, int V, const int16_t* __restrict__ fsm_next,
    const int16_t* __restrict__ fsm_dist, const int* __restrict__ fsm_base, int* __restrict__ fsm_state,
    int* __restrict__ gen_count, const int* __restrict__ max_new, const float* __restrict__ temperature,
    const int* __restrict__ row_keys, int* __restrict__ done, int* __restrict__ seq_lens,
    int* __restrict__ out_tokens, int out_stride, int* __restrict__ next_tokens, uint32_t seed,
    int budget_aware, int n_text, int eos, int eos2) {
  const int b = blockIdx.x;
  if (done[b]) return;
  const int tid = threadIdx.x;
  const int base = fsm_base[b];
  const int step = gen_count[b];
  const int remaining = max_new[b] - step;
  const float temp = temperature[b];
  const bool greedy = !(temp > 0.f);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const uint32_t a = fmix32(static_cast<uint32_t>(row_keys[b]) * 0x9E3779B9u + static_cast<uint32_t>(step) * 0x632BE5ABu + seed);
  const bf16_t* lrow = logits + static_cast<size_t>(b) * V;
  const int state = fsm_state[b];
  const int16_t* frow = base >= 0 ? fsm_next + static_cast<size_t>(base + state) * V : nullptr;

  Cand tight{-INFINITY, 0x7fffffff}, any{-INFINITY, 0x7fffffff};
  const int nvec = V / 8;
  for (int vi = tid; vi < nvec; vi += SAMPLE_THREADS) {
    const int t0 = vi * 8;
    u16x8 lv = *reinterpret_cast<const u16x8*>(lrow + t0);
    int16_t nx[8];
    if (frow) {
      *reinterpret_cast<u16x8*>(nx) = *reinterpret_cast<const u16x8*>(frow + t0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + j;
      bool ok;
      int nxt = -1;
      if (frow) {
        nxt = nx[j];
        ok = nxt >= 0;
      } else {
        ok = t < n_text || t == eos || t == eos2;
      }
      if (!ok) continue;
      float s = bf2f(lv[j]);
      if (!greedy) {
        const uint32_t h = fmix32(a ^ (static_cast<uint32_t>(t) * 0x27D4EB2Fu));
        const float u = (static_cast<float>(h >> 8) + 0.5f) * (1.f / 16777216.f);
        s = s * inv_t - __logf(-__logf(u));
      }
      better(any, s, t);
      if (budget_aware && frow && static_cast<int>(fsm_dist[base + nxt]) <= remaining - 1) better(tight, s, t);
    }
  }
  // tail (V not a multiple of 8)
  for (int t = nvec * 8 + tid; t < V; t += SAMPLE_THREADS) {
    int nxt = frow ? frow[t] : -1;
    const bool ok = frow ? nxt >= 0 : (t < n_text || t == eos || t == eos2);
    if (!ok) continue;
    float s = bf2f(lrow[t]);
    if (!greedy) {
      const uint32_t h = fmix32(a ^ (static_cast<uint32_t>(t) * 0x27D4EB2Fu));
      const float u = (static_cast<float>(h >> 8) + 0.5f) * (1.f / 16777216.f);
      s = s * inv_t - __logf(-__logf(u));
    }
    better(any, s, t);
    if (budget_aware && frow && static_cast<int>(fsm_dist[base + nxt]) <= remaining - 1) better(tight, s, t);
  }

  __shared__ Cand s_any[SAMPLE_THREADS / WAVE], s_tight[SAMPLE_THREADS / WAVE];
  any = wave_argmax(any);
  tight = wave_argmax(tight);
  if ((tid & 63) == 0) {
    s_any[tid >> 6] = any;
    s_tight[tid >> 6] = tight;
  }
  __syncthreads();
  if (tid != 0) return;
  for (int w = 1; w < SAMPLE_THREADS / WAVE; ++w) {
    better(any, s_any[w].score, s_any[w].idx);
    better(tight, s_tight[w].score, s_tight[w].idx);
  }
  const Cand pick = (budget_aware && tight.idx != 0x7fffffff) ? tight : any;
  if (pick.idx == 0x7fffffff) {  // nothing allowed: dead state
    done[b] = 1;
    return;
  }
  const int tok = pick.idx;
  out_tokens[static_cast<size_t>(b) * out_stride + step] = tok;
  next_tokens[b] = tok;
  gen_count[b] = step + 1;
  seq_lens[b] += 1;
  bool finished = remaining - 1 <= 0;
  if (frow) {
    const int ns = frow[tok];
    fsm_state[b] = ns;
    finished = finished || fsm_dist[base + ns] == 0;
  } else {
    finished = finished || tok == eos || tok == eos2;
  }
  if (finished) done[b] = 1;
}

}  // namespace

BCG_API int bcg_guided_sample(const void* logits, int B, int V, const int16_t* fsm_next, const int16_t* fsm_dist,
                              const int* fsm_base, int* fsm_state, int* gen_count, const int* max_new,
                              const float* temperature, const int* row_keys, int* done, int* seq_lens,
                              int* out_tokens, int out_stride, int* next_tokens, uint32_t seed, int budget_aware,
                              int n_text, int eos, int eos2, hipStream_t stream) {
  if (B <= 0 || V <= 0) return -2;
  hipLaunchKernelGGL(guided_sample_kernel, dim3(B), dim3(SAMPLE_THREADS), 0, stream,
                     static_cast<const bf16_t*>(logits), V, fsm_next, fsm_dist, fsm_base, fsm_state, gen_count,
                     max_new, temperature, row_keys, done, seq_lens, out_tokens, out_stride, next_tokens, seed,
                     budget_aware, n_text, eos, eos2);
  return BCG_CHECK_LAUNCH();
}
