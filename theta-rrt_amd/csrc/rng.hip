// The np.random gaussian stream on the device: rand_conf's three legacy gaussians per iteration
// (rrt.py:58,66), bit for bit what numpy's RandomState.standard_normal returns from the same state
// (legacy_gauss.hpp restates the arithmetic; tests/test_rng.py pins it).
//
// Layout.  The MT19937 word stream is independent of how it is consumed, so it is produced ahead
// into a ring of raw (untempered) state words, one 624-word block per twist: word w of the stream
// lives at ring[w mod RS] (RS a multiple of 624); gen_end[0] = words generated, gen_end[1] = the
// oldest word the ring is known to hold (0 after a seed; moved up when the ring is regrown).  Block 0 is the key of the state the stream was
// seeded from; a stream position is the index of the next word to consume plus numpy's cached
// gaussian (has_gauss, gauss).
//
// Kernels per chunk of n gaussians (one or more batches of `blen` each):
//   k_mt_gen     one workgroup: twists blocks until the ring holds the chunk's worst-case words
//                (227 threads each advance a chain key[t] -> key[t+227] -> key[t+454]; one LDS
//                barrier pair per 624 words).  The recurrence is serial from block to block, so
//                chunks of more than MT_PAR_MIN words are generated in super-steps instead:
//   k_mt_jump    the state blocks MT_SEG, 2 MT_SEG, ... words ahead of the ring's end by MT19937
//                jump-ahead (mt_jump.hpp: each is the XOR of windows of the last MT_HIST words
//                at the set bits of a fixed polynomial), one block per (seed, 64 output words),
//                the window staged in LDS
//   k_mt_gen_par MT_NSEG workgroups each twist MT_SEG_BLOCKS blocks from their seed: MT_SUPER
//                words per super-step in the time one workgroup twists MT_SEG_BLOCKS blocks
//   k_gauss_count  polar-method attempts (4 words each) from the chunk's start, accepted per block
//   k_gauss_emit   prefix of the block counts, each accepted attempt's pair index, f = sqrt(-2 log
//                r2 / r2), outputs in stream order; the stream position after every batch boundary
//                (so a run can rewind the stream to the last batch it used)
#pragma clang fp contract(off)
#include "thetarrt_internal.hpp"
#include "legacy_gauss.hpp"
#include "mt_jump.hpp"
#include "diaglog.hpp"
TR_DLOG_EXPORT(tr_diag_log_rng)

namespace tr {

constexpr int MT_N = 624, MT_SHIFT = 227;   // N - M
constexpr int RG_T = 256, RG_APT = 4, RG_APB = RG_T * RG_APT;   // attempts per thread / block

constexpr int64_t MT_SEG = (int64_t)MT_SEG_BLOCKS * MT_N;   // words per generator workgroup
constexpr int64_t MT_SUPER = MT_SEG * MT_NSEG;              // words per super-step
// generated words before the first jump: its window [end - MT_HIST, end) must start at a word
// >= 1 (word 0 is a seed key's first word, whose low 31 bits are not part of the state)
constexpr int64_t MT_HIST_MIN = ((MT_HIST + MT_N) / MT_N) * MT_N;
constexpr int64_t MT_PAR_MIN = 256 * MT_N;   // chunks below this stay serial: one workgroup busy
                                             // for ~0.1 ms on its own stream is off every critical
                                             // path (a super-step only pays from a few hundred
                                             // blocks per chunk, i.e. global batches >= 16384)

// One twist of the 624-word state in LDS (all RG_T threads of the block).
__device__ __forceinline__ void mt_twist(uint32_t* s, int t) {
  uint32_t n0 = 0, n1 = 0, n2 = 0;
  if (t < MT_SHIFT) {
    n0 = mt_mix(s[t], s[t + 1], s[t + 397]);
    n1 = mt_mix(s[t + 227], s[t + 228], n0);
    if (t < 169) {
      n2 = mt_mix(s[t + 454], s[t + 455], n1);
    } else if (t == 169) {                     // key[623] from the new key[0] and key[396]
      const uint32_t k0 = mt_mix(s[0], s[1], s[397]);
      n2 = mt_mix(s[623], k0, n1);
    }
  }
  __syncthreads();
  if (t < MT_SHIFT) {
    s[t] = n0;
    s[t + 227] = n1;
    if (t <= 169) s[t + 454] = n2;
  }
  __syncthreads();
}

// Serial generation: until the ring holds `need` words past the chunk's start, or `limit` words
// in all (the history the first jump needs), whichever comes first.
__global__ __launch_bounds__(RG_T) void k_mt_gen(uint32_t* __restrict__ ring, int64_t rs,
                                                 int64_t* __restrict__ gen_end,
                                                 const RngPos* __restrict__ start, int64_t need,
                                                 int64_t limit) {
  __shared__ uint32_t s[MT_N];
  const int t = threadIdx.x;
  TR_DLOG_T0;
  int64_t ge = *gen_end;
  // limit: words of valid history (gen_end[1] = the oldest word the ring still holds) a jump needs
  const int64_t target = min(start->wpos + need, limit == INT64_MAX ? limit : gen_end[1] + limit);
  if (ge >= target) return;
  for (int i = t; i < MT_N; i += RG_T) s[i] = ring[(ge - MT_N) % rs + i];
  __syncthreads();
  while (ge < target) {
    mt_twist(s, t);
    uint32_t* dst = ring + ge % rs;
    for (int i = t; i < MT_N; i += RG_T) dst[i] = s[i];
    ge += MT_N;
  }
  if (t == 0) *gen_end = ge;
  TR_DLOG(6);
}

// A super-step runs when the chunk still lacks words and the ring holds the jump's history; both
// of its kernels read the same gen_end (the generator's last workgroup advances it at its end).
__device__ __forceinline__ bool mt_super_due(const int64_t* gen_end, const RngPos* start,
                                             int64_t need, int64_t& ge) {
  ge = gen_end[0];
  return ge < start->wpos + need && ge >= gen_end[1] + MT_HIST_MIN;
}

// seeds[(w - 1) * 624 + k] = stream word end + w MT_SEG - 624 + k, w = 1 .. MT_NSEG - 1: the state
// block each generator workgroup starts from.  Block (kt, w - 1): output words [64 kt, 64 kt + 64).
constexpr int JT = 1024, JW = JT / 64;         // threads / waves per jump block
constexpr int J_WIN = MT_HIST - MT_N + 64;     // window words a block's 64 outputs read (20000)
constexpr int J_LIST = 8192;                   // >= the heaviest polynomial's weight (checked)
__global__ __launch_bounds__(JT) void k_mt_jump(const uint32_t* __restrict__ ring, int64_t rs,
                                                const int64_t* __restrict__ gen_end,
                                                const RngPos* __restrict__ start, int64_t need,
                                                uint32_t* __restrict__ seeds,
                                                int32_t* __restrict__ err) {
  extern __shared__ uint32_t jsm[];
  uint32_t* win = jsm;                                         // J_WIN words
  uint16_t* list = reinterpret_cast<uint16_t*>(jsm + J_WIN);   // set bits of the polynomial
  uint32_t* part = jsm + J_WIN + J_LIST / 2;                   // JW x 64 partial XORs
  __shared__ int32_t s_wsum[JW];
  int64_t ge;
  TR_DLOG_T0;
  if (!mt_super_due(gen_end, start, need, ge)) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int w = blockIdx.y, k0 = blockIdx.x * 64;
  const int64_t base = ge - MT_HIST + k0;
  for (int q = t; q < J_WIN; q += JT) win[q] = ring[(base + q) % rs];
  // ordered list of the polynomial's set bits: a block scan of the words' weights
  const uint32_t pw = t < MT_JW ? MT_JUMP[w][t] : 0u;
  const int c = __popc(pw);
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  if (lane == 63) s_wsum[wv] = inc;
  __syncthreads();
  int off = inc - c, total = 0;
#pragma unroll
  for (int q = 0; q < JW; ++q) {
    off += q < wv ? s_wsum[q] : 0;
    total += s_wsum[q];
  }
  if (total > J_LIST) {                        // cannot happen with the generated table
    if (t == 0) atomicOr(err, 2);
    return;
  }
  for (uint32_t m = pw; m; m &= m - 1) list[off++] = (uint16_t)(32 * t + __builtin_ctz(m));
  __syncthreads();
  uint32_t acc = 0;
  for (int e = wv * 8; e < total; e += JW * 8) {
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = e + q < total ? win[list[e + q] + lane] : 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) acc ^= v[q];
  }
  part[wv * 64 + lane] = acc;
  __syncthreads();
  if (t < 64 && k0 + t < MT_N) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < JW; ++q) r ^= part[q * 64 + t];
    seeds[(int64_t)w * MT_N + k0 + t] = r;
  }
  TR_DLOG(7);
}

// Workgroup w twists MT_SEG_BLOCKS blocks from its seed (w = 0: the ring's last block) into ring
// words [end + w MT_SEG, end + (w + 1) MT_SEG); the last workgroup to finish advances gen_end.
__global__ __launch_bounds__(RG_T) void k_mt_gen_par(uint32_t* __restrict__ ring, int64_t rs,
                                                     int64_t* __restrict__ gen_end,
                                                     const RngPos* __restrict__ start,
                                                     int64_t need,
                                                     const uint32_t* __restrict__ seeds,
                                                     int32_t* __restrict__ done) {
  __shared__ uint32_t s[MT_N];
  int64_t ge;
  TR_DLOG_T0;
  if (!mt_super_due(gen_end, start, need, ge)) return;
  const int t = threadIdx.x, w = blockIdx.x;
  const uint32_t* src = w == 0 ? ring + (ge - MT_N) % rs : seeds + (int64_t)(w - 1) * MT_N;
  for (int i = t; i < MT_N; i += RG_T) s[i] = src[i];
  __syncthreads();
  int64_t at = ge + (int64_t)w * MT_SEG;
  for (int b = 0; b < MT_SEG_BLOCKS; ++b, at += MT_N) {
    mt_twist(s, t);
    uint32_t* dst = ring + at % rs;
    for (int i = t; i < MT_N; i += RG_T) dst[i] = s[i];
  }
  // every workgroup read gen_end before it arrives here; the last one publishes the new end
  wave_stores_done();
  __syncthreads();
  if (t == 0) {
    release_l2();
    if (atomicAdd(done, 1) == (int32_t)gridDim.x - 1) {
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *gen_end = ge + MT_SUPER;
    }
  }
  TR_DLOG(8);
}

__device__ __forceinline__ bool rg_attempt(const uint32_t* __restrict__ ring, int64_t rs, int64_t w,
                                           double* a, double* b) {
  return legacy_attempt(mt_temper(ring[w % rs]), mt_temper(ring[(w + 1) % rs]),
                        mt_temper(ring[(w + 2) % rs]), mt_temper(ring[(w + 3) % rs]), a, b);
}

// attempts available from the chunk start: the generated words, capped by the launch's bound
__device__ __forceinline__ int64_t rg_avail(const int64_t* gen_end, const RngPos* start, int64_t cap) {
  const int64_t a = (*gen_end - start->wpos) / 4;
  return a < cap ? a : cap;
}

__device__ __forceinline__ bool rg_accept(const uint32_t* __restrict__ ring, int64_t rs, int64_t w) {
  const uint32_t w0 = mt_temper(ring[w % rs]), w1 = mt_temper(ring[(w + 1) % rs]);
  const uint32_t w2 = mt_temper(ring[(w + 2) % rs]), w3 = mt_temper(ring[(w + 3) % rs]);
  const double d1 = ((double)(int32_t)(w0 >> 5) * 67108864.0 + (double)(int32_t)(w1 >> 6)) / 9007199254740992.0;
  const double d2 = ((double)(int32_t)(w2 >> 5) * 67108864.0 + (double)(int32_t)(w3 >> 6)) / 9007199254740992.0;
  const double x1 = 2.0 * d1 - 1.0, x2 = 2.0 * d2 - 1.0;
  const double r2 = x1 * x1 + x2 * x2;
  return !(r2 >= 1.0 || r2 == 0.0);
}

__global__ __launch_bounds__(RG_T) void k_gauss_count(const uint32_t* __restrict__ ring, int64_t rs,
                                                      const int64_t* __restrict__ gen_end,
                                                      const RngPos* __restrict__ start, int64_t cap,
                                                      int32_t* __restrict__ counts) {
  __shared__ int32_t s_n;
  const int t = threadIdx.x;
  TR_DLOG_T0;
  if (t == 0) s_n = 0;
  __syncthreads();
  const int64_t A = rg_avail(gen_end, start, cap), w0 = start->wpos;
  int32_t n = 0;
#pragma unroll
  for (int k = 0; k < RG_APT; ++k) {
    const int64_t a = (int64_t)blockIdx.x * RG_APB + k * RG_T + t;
    if (a < A) n += rg_accept(ring, rs, w0 + 4 * a);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
  if ((t & 63) == 0) atomicAdd(&s_n, n);
  __syncthreads();
  if (t == 0) counts[blockIdx.x] = s_n;
  TR_DLOG(9);
}

// out[0 .. n): the chunk's gaussians; bstate[b] = stream position after out[0 .. (b + 1) blen).
__global__ __launch_bounds__(RG_T) void k_gauss_emit(const uint32_t* __restrict__ ring, int64_t rs,
                                                     const int64_t* __restrict__ gen_end,
                                                     const RngPos* __restrict__ start, int64_t cap,
                                                     const int32_t* __restrict__ counts, int64_t n,
                                                     int64_t blen, double* __restrict__ out,
                                                     RngPos* __restrict__ bstate,
                                                     int32_t* __restrict__ err) {
  __shared__ int64_t s_pre;
  __shared__ int32_t s_w[RG_T / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  TR_DLOG_T0;
  const RngPos st0 = *start;
  const int64_t A = rg_avail(gen_end, start, cap);
  const int64_t has0 = st0.has, P = (n - has0 + 1) / 2;   // pairs this chunk consumes
  // pairs before this block
  int64_t pre = 0;
  for (int q = t; q < (int)blockIdx.x; q += RG_T) pre += counts[q];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o);
  if (t == 0) s_pre = 0;
  __syncthreads();
  if (lane == 0) atomicAdd((unsigned long long*)&s_pre, (unsigned long long)pre);
  __syncthreads();
  int64_t base = s_pre;
  if (blockIdx.x == 0 && t == 0) {
    if (has0 && n > 0) out[0] = st0.gauss;
    if (P == 0) bstate[n / blen - 1] = RngPos{st0.wpos, 0, 0, 0.0};   // only the cached value
  }
  if (blockIdx.x == gridDim.x - 1 && t == 0) {
    if (base + counts[blockIdx.x] < P) atomicOr(err, 1);          // ring too short (bound broken)
  }
#pragma unroll 1
  for (int k = 0; k < RG_APT; ++k) {
    const int64_t a = (int64_t)blockIdx.x * RG_APB + k * RG_T + t;
    double g1 = 0.0, g2 = 0.0;
    const bool acc = a < A && rg_attempt(ring, rs, st0.wpos + 4 * a, &g1, &g2);
    const uint64_t m = __ballot(acc);
    const int32_t r = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[wv] = __popcll(m);
    __syncthreads();
    int32_t off = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < RG_T / 64; ++q) {
      off += q < wv ? s_w[q] : 0;
      tot += s_w[q];
    }
    const int64_t pair = base + off + r;
    if (acc && pair < P) {
      const int64_t o = has0 + 2 * pair;
      out[o] = g1;
      if (o + 1 < n) out[o + 1] = g2;
      const int64_t wnext = st0.wpos + 4 * (a + 1);
      if ((o + 1) % blen == 0) bstate[(o + 1) / blen - 1] = RngPos{wnext, 1, 0, g2};
      if ((o + 2) % blen == 0 && o + 2 <= n) bstate[(o + 2) / blen - 1] = RngPos{wnext, 0, 0, 0.0};
    }
    base += tot;
    __syncthreads();
  }
  TR_DLOG(10);
}

// The key block holding a stream position (numpy's (key, 624) and (next key, 0) are the same
// position; the former is used) and the position within it.
__device__ __forceinline__ int64_t rg_block(int64_t w) { return w > 0 && w % MT_N == 0 ? w / MT_N - 1 : w / MT_N; }

// keys[b] = the key block of batch b's end position bstate[b] (a later rewind re-seeds from it).
__global__ __launch_bounds__(RG_T) void k_rng_keep(const uint32_t* __restrict__ ring, int64_t rs,
                                                   const RngPos* __restrict__ bstate,
                                                   uint32_t* __restrict__ keys) {
  const int64_t blk = rg_block(bstate[blockIdx.x].wpos);
  const uint32_t* src = ring + (MT_N * blk) % rs;
  for (int i = threadIdx.x; i < MT_N; i += RG_T) keys[(int64_t)blockIdx.x * MT_N + i] = src[i];
}

// Re-seed the stream at a kept position: ring block 0 = its key, generation restarts after it.
__global__ __launch_bounds__(RG_T) void k_rng_rebase(uint32_t* __restrict__ ring,
                                                     int64_t* __restrict__ gen_end,
                                                     RngPos* __restrict__ pos0,
                                                     const RngPos* __restrict__ src,
                                                     const uint32_t* __restrict__ key) {
  const RngPos p = *src;
  for (int i = threadIdx.x; i < MT_N; i += RG_T) ring[i] = key[i];
  if (threadIdx.x == 0) {
    gen_end[0] = MT_N;
    gen_end[1] = 0;
    *pos0 = RngPos{p.wpos - MT_N * rg_block(p.wpos), p.has, 0, p.gauss};
  }
}

void rng_keep(hipStream_t st, const uint32_t* ring, int64_t rs, const RngPos* bstate, int64_t nb,
              uint32_t* keys) {
  if (nb > 0) hipLaunchKernelGGL(k_rng_keep, dim3((unsigned)nb), dim3(RG_T), 0, st, ring, rs, bstate, keys);
}

void rng_rebase(hipStream_t st, uint32_t* ring, int64_t* gen_end, RngPos* pos0, const RngPos* src,
                const uint32_t* key) {
  hipLaunchKernelGGL(k_rng_rebase, dim3(1), dim3(RG_T), 0, st, ring, gen_end, pos0, src, key);
}

int64_t rng_attempts_ub(int64_t n) {         // worst-case attempts for n gaussians (> 12 sigma)
  const double P = (double)((n + 1) / 2);
  return (int64_t)ceil(P * 1.27324 + 12.0 * sqrt(P) + 64.0);
}

int64_t rng_ring_extra(int64_t n) {           // ring words beyond the chunk's own (super-steps)
  return 4 * rng_attempts_ub(n) >= MT_PAR_MIN ? 2 * MT_SUPER + MT_HIST + MT_N : 0;
}

void rng_chunk(hipStream_t st, uint32_t* ring, int64_t rs, int64_t* gen_end, const RngPos* start,
               int64_t n, int64_t blen, double* out, RngPos* bstate, int32_t* counts, int32_t* err,
               uint32_t* seeds, int32_t* done) {
  if (n <= 0) return;
  const int64_t cap = rng_attempts_ub(n);
  const unsigned g = (unsigned)((cap + RG_APB - 1) / RG_APB);
  const int64_t need = 4 * cap;
  if (need < MT_PAR_MIN) {
    hipLaunchKernelGGL(k_mt_gen, dim3(1), dim3(RG_T), 0, st, ring, rs, gen_end, start, need,
                       INT64_MAX);
  } else {
    // the history the first jump reads (a no-op once the ring holds it), then super-steps: each
    // adds MT_SUPER words while the chunk still lacks some
    constexpr size_t jlds = sizeof(uint32_t) * (J_WIN + J_LIST / 2 + JW * 64);
    static const bool big_lds = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mt_jump),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)jlds) == hipSuccess;
    (void)big_lds;
    hipLaunchKernelGGL(k_mt_gen, dim3(1), dim3(RG_T), 0, st, ring, rs, gen_end, start, need,
                       MT_HIST_MIN);
    for (int64_t q = 0; q < (need + MT_SUPER - 1) / MT_SUPER; ++q) {
      hipLaunchKernelGGL(k_mt_jump, dim3((MT_N + 63) / 64, MT_NSEG - 1), dim3(JT), jlds, st, ring,
                         rs, gen_end, start, need, seeds, err);
      hipLaunchKernelGGL(k_mt_gen_par, dim3(MT_NSEG), dim3(RG_T), 0, st, ring, rs, gen_end, start,
                         need, seeds, done);
    }
  }
  hipLaunchKernelGGL(k_gauss_count, dim3(g), dim3(RG_T), 0, st, ring, rs, gen_end, start, cap, counts);
  hipLaunchKernelGGL(k_gauss_emit, dim3(g), dim3(RG_T), 0, st, ring, rs, gen_end, start, cap, counts,
                     n, blen, out, bstate, err);
}

int64_t rng_counts_len(int64_t n) { return (rng_attempts_ub(n) + RG_APB - 1) / RG_APB; }

}  // namespace tr
