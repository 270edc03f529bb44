// qkv projection (+ RMSNorm prologue, RoPE / paged-KV-write epilogue) AND the decode attention of
// the same token in ONE launch, for one-row engines (the tensor-parallel ranks' shards with 1-2 kv
// heads, where it measured faster; the engine decides per shape). Host: llmc_qkv_attn.
//
// Why (profiles/r4_tp8_shard_kernel_stats.md, a Llama-3-8B TP=8 rank at 2k keys): the qkv GEMV
// (4.8 us) and the attention (9.0 us for ~1 MB of K/V) are both latency chains; as two launches
// the attention's own round trips (length and page id, then the K/V stream) start only after the
// GEMV's boundary. Here they run under the GEMV: the K/V of the cached keys do not depend on this
// token, so the attention blocks request them at once and only wait for the rotated q.
//
// Grid: the GEMV blocks (gemv_core.h gemv_block: 4 waves x 1 row, 8 x 16-B loads per lane in
// flight; every row's dot product in the same order as the qkv_rope launch, whose geometry for
// outputs under 2048 rows this is, so there q / k / v are the same bits; wider outputs group the
// RMS norm's sum of squares differently, last bits), then gc fused-form attention chunks per kv
// head (attn_core.h SubTile, 4 waves x 32 / 64 keys of one page). An attention block only waits on
// GEMV blocks, which have lower indices and are dispatched first: no wait is on a block that has
// not started.
//
// Hand-off: the GEMV epilogue publishes every rotated q / k pair and v pair as an 8-B {bf16x2, tag}
// granule (RopeEpi::granules: one single-copy-atomic write-through store, the data IS the flag,
// MI355X_MICROARCH.md handoff-1to1). An attention block requests its K/V (keys < L - 1: already
// in the cache), then gathers its kv head's q granules into LDS, polling tags; the block holding
// key L - 1 (this token's, still being written to the cache) also gathers its k / v granules and
// folds that key into wave 0's softmax state. Then the usual publish + last-arriver merge.
// The hand-off tag = a per-launch epoch in hctr: every attention block counts its exit, the last
// one advances the epoch (by then every GEMV block has published, so every block of the launch
// has read it). Bounded spins: a lost granule sets fault = 4.
#include "attn_core.h"
#include "gemv_core.h"
#include "car_proto.h"

namespace llmc {

constexpr int kQaThreads = 256, kQaWaves = 4;

template <int G, int D, bool SC1OUT = false>
__device__ __forceinline__ void qa_attention(int c, int kvh, char* smem, const int32_t* __restrict__ block_table,
                                             int bt_len, int L, const bf16_t* __restrict__ k_cache,
                                             const bf16_t* __restrict__ v_cache, float* __restrict__ part,
                                             int* __restrict__ counters, bf16_t* __restrict__ out, int nh, int nkv,
                                             int bs, int nblocks, int chunk, int max_chunks, int gsize, int max_groups,
                                             float scale_log2, int* __restrict__ fault,
                                             const uint64_t* __restrict__ granules, uint32_t htag) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  constexpr int HALF = D / 2;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  int* ctr = counters + kvh * (2 + max_groups) * kCtrPitch;  // row 0: {ticket, epoch, group tickets}
  const uint32_t tag = static_cast<uint32_t>(__hip_atomic_load(ctr + kCtrPitch, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const int per_wave = chunk / kQaWaves;  // 32 or 64 keys, inside one page (host-checked)
  const int key0 = c * chunk + wave * per_wave;
  const int pidx = __builtin_amdgcn_readfirstlane(min(key0 / bs, bt_len - 1));
  const int page = min(max(ld_scalar(block_table + pidx), 0), nblocks - 1);  // clamped into the cache
  const int Lc = L - 1;  // keys already in the cache; key L - 1 is this launch's
  const int nchunks = (L + chunk - 1) / chunk;
  const bool last = c == (L - 1) / chunk;  // block-uniform: this block folds in the new key
  const int end = min(Lc, key0 + per_wave);
  const bool wk = key0 < end;  // wave-uniform

  char* vbuf = smem + wave * 32 * kVRowBytes;
  float* red = reinterpret_cast<float*>(smem + kQaWaves * 32 * kVRowBytes);
  int* flag = reinterpret_cast<int*>(red + kQaWaves * G * (D + 2));
  bf16_t* qn = reinterpret_cast<bf16_t*>(flag + 4);  // [G][D] this kv head's rotated q
  bf16_t* kn = qn + G * D;                           // [D] the new key
  bf16_t* vn = kn + D;                               // [D] its value

  // 1. the cached keys' K / V first: in flight while the projection still runs
  ST st;
  bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
  u32x4 vsA[ST::NV], vsB[ST::NV];
  const int64_t base = (static_cast<int64_t>(page) * nkv + kvh) * bs * D;
  auto row = [&](const bf16_t* cache, int key) { return cache + base + static_cast<int64_t>(key % bs) * D; };
  if (wk) {
    st.issue(key0, end, lane, row, k_cache, v_cache, kfA, vsA);
    if (key0 + 32 < end) st.issue(key0 + 32, end, lane, row, k_cache, v_cache, kfB, vsB);
  }
  // 2. this kv head's q (and in the last block the new key's k / v) granules -> LDS. One thread
  // polls a sentinel (this head group's last q granule) until it lands, the block then reads them
  // all (re-polling any that lags): every thread polling its own granule flooded the memory path
  // the projection's weights stream through (MI355X_MICROARCH.md polling-cost)
  const int nq = G * HALF, total = nq + (last ? 2 * HALF : 0);
  if (tid == 0) {
    for (unsigned spins = 0; spins < kSpinLimit; ++spins) {
      const uint64_t v = __hip_atomic_load(granules + (kvh * G + G - 1) * HALF + HALF - 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (static_cast<uint32_t>(v >> 32) == htag) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  for (int t = tid; t < total; t += kQaThreads) {
    const int gi = t < nq ? kvh * G * HALF + t
                          : (t < nq + HALF ? (nh + kvh) * HALF + (t - nq) : (nh + nkv + kvh) * HALF + (t - nq - HALF));
    uint64_t v = 0;
    for (unsigned spins = 0;; ++spins) {
      v = __hip_atomic_load(granules + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (static_cast<uint32_t>(v >> 32) == htag) break;
      if (spins >= kSpinLimit) {
        if (fault != nullptr) __hip_atomic_store(fault, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bf16_t lo = static_cast<bf16_t>(v & 0xffffu), hi = static_cast<bf16_t>((v >> 16) & 0xffffu);
    if (t < nq) {  // q head g pair i = dims (i, i + D/2)
      const int g = t / HALF, i = t % HALF;
      qn[g * D + i] = lo;
      qn[g * D + i + HALF] = hi;
    } else if (t < nq + HALF) {  // k pair i = dims (i, i + D/2)
      const int i = t - nq;
      kn[i] = lo;
      kn[i + HALF] = hi;
    } else {  // v pair j = dims (2j, 2j + 1)
      const int j = t - nq - HALF;
      vn[2 * j] = lo;
      vn[2 * j + 1] = hi;
    }
  }
  __syncthreads();
  st.init(qn, lane);
  if (wk) {
    st.compute(key0, end, lane, vbuf, scale_log2, kfA, vsA);
    if (key0 + 32 < end) st.compute(key0 + 32, end, lane, vbuf, scale_log2, kfB, vsB);
  }
  // 3. the new key into wave 0's online-softmax state (head h = lane & 15; columns >= G copy head 0)
  if (last && wave == 0) {
    const int h = lane & 15, g4 = lane >> 4;
    const bf16_t* qh = qn + (h < G ? h : 0) * D;
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < D / 4; ++e) {
      const int d = g4 * (D / 4) + e;
      s += bf16_to_f32(qh[d]) * bf16_to_f32(kn[d]);
    }
    s = xor16_add(s);
    s = xor32_add(s);
    s *= scale_log2;
    const float m_new = fmaxf(st.m_run, s);
    const float alpha = exp2f(st.m_run - m_new), p = exp2f(s - m_new);
    st.l_run = st.l_run * alpha + p;
    st.m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < ST::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) st.acc[dt][i] = st.acc[dt][i] * alpha + p * bf16_to_f32(vn[dt * 16 + 4 * g4 + i]);
  }
  st.to_lds(red, wave, lane);
  __syncthreads();
  bf16_t* out_row = out + kvh * G * D;
  if (nchunks == 1) {
    if constexpr (SC1OUT) store_direct_sc1<G, D, kQaWaves>(red, out_row, tid);
    else store_direct<G, D, kQaWaves>(red, out_row, tid);
    return;
  }
  publish_and_merge<G, D, kQaWaves, SC1OUT>(red, part, ctr, 0, nkv, kvh, c, nchunks, gsize, max_chunks, max_groups, tag,
                                            out_row, smem, flag, tid, fault);
}

// ---- o-role (round 6): the decode o_proj of the same token in the same launch -------------------
// Blocks after the attention blocks, 4 waves x kOrRows rows each. A block requests its W_o rows at
// once (they do not depend on the token) and its residual, then waits until every attention block
// of the launch has written its head output (an arrival counter the attention blocks bump after
// draining their write-through stores), reads the attention output with write-through-coherent
// loads, and finishes its rows: h = resid + W_o . attn (TP=1, or TP rank 0 without the fused
// all-reduce), h = W_o . attn (another rank: its all-reduce follows as its own launch), or the
// all-reduce in this epilogue (car_proto.h push protocol, gemv_core.h EPI_AR's exchange: the block's
// 16 rows as 8 granules of its virtual block bo, the same epoch words as the row-parallel GEMVs'
// EPI_AR). Replaces the o GEMV launch after the one-launch qkv + attention on TP ranks.
constexpr int kOrRpw = 4, kOrRows = kOrRpw * kQaWaves, kOrMaxCpl = 4;
static_assert(kOrMaxCpl == 4, "the CPL dispatch below covers 1..4");  // rows per wave / block; 16-B chunks per lane per row

struct OArgs {
  const bf16_t* w_o;  // [n_o, k_o]
  bf16_t* h;          // [n_o] (one row)
  int n_o, k_o;
  int mode;           // 0 = no o-role; 1 = h += W_o . attn; 2 = h = W_o . attn; 3 = all-reduce (ar), rank 0 adds h
  CarArgs ar;
};

template <int CPL>
__device__ __forceinline__ void qa_oproj_block(int bo, char* smem, const bf16_t* __restrict__ attn, const OArgs& o,
                                               int* __restrict__ adone, int n_attn, int* __restrict__ fault) {
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int r0 = bo * kOrRows + wave * kOrRpw;
  // 1. weights (nt: read once) and the residual, before the wait
  u32x4 wv[kOrRpw][CPL];
#pragma unroll
  for (int j = 0; j < kOrRpw; ++j) {
    const int n = min(r0 + j, o.n_o - 1);
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc)
      wv[j][cc] = load16<true>(reinterpret_cast<const u32x4*>(o.w_o + static_cast<int64_t>(n) * o.k_o) + lane + cc * kWave);
  }
  const bool resid = o.mode == 1 || (o.mode == 3 && o.ar.rank == 0);
  float rv[kOrRpw];
#pragma unroll
  for (int j = 0; j < kOrRpw; ++j) rv[j] = resid && r0 + j < o.n_o ? bf16_to_f32(o.h[r0 + j]) : 0.f;
  uint32_t ar_epoch = 0;
  if (o.mode == 3 && tid == 0)
    ar_epoch = __hip_atomic_load(car_ctr(o.ar.P.base[o.ar.rank]) + bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  // 2. every attention block has drained its output stores and counted in (the wait is on
  // lower-index blocks only: they were dispatched first, so it always ends)
  if (tid == 0) {
    for (unsigned spins = 0;; ++spins) {
      if (__hip_atomic_load(adone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n_attn) break;
      if (spins >= kSpinLimit) {
        if (fault != nullptr) __hip_atomic_store(fault, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  // 3. the attention output through write-through-coherent (sc1) loads, the dot products
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(attn), 0, o.k_o * 2, 0x00020000);
  u32x4 xv[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) xv[cc] = ld16_sc1(ra, (lane + cc * kWave) * 16);
  float acc[kOrRpw];
#pragma unroll
  for (int j = 0; j < kOrRpw; ++j) {
    float a = 0.f;
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) a = dot8_bf16(wv[j][cc], xv[cc], a);
    acc[j] = wave_sum(a) + rv[j];
  }
  if (o.mode != 3) {
    if (lane < kOrRpw) {
#pragma unroll
      for (int j = 0; j < kOrRpw; ++j)
        if (lane == j && r0 + j < o.n_o) o.h[r0 + j] = f32_to_bf16(acc[j]);
    }
    return;
  }
  // 4. the all-reduce of the block's rows (pairs of rows = granules of virtual block bo)
  float* rowv = reinterpret_cast<float*>(smem);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < kOrRpw; ++j) rowv[wave * kOrRpw + j] = acc[j];
  }
  __syncthreads();
  if (wave != 0) return;
  constexpr int NG = kOrRows / 2;
  const CarArgs& ar = o.ar;
  const uint32_t epoch = __shfl(ar_epoch, 0, 64);
  const int pairs = max(0, min(kOrRows, o.n_o - bo * kOrRows)) / 2;
  const long gbase = static_cast<long>(bo) * kArGranulesPerBlock;
  const int gi = lane % NG;
  const uint32_t mine = pack_bf16x2(rowv[2 * gi], rowv[2 * gi + 1]);
  for (int base = 0; base < ar.world * NG; base += kWave) {  // push: (peer, granule); uniform trip count
    const int idx = base + lane;
    const bool live = idx < ar.world * NG;
    const int p = idx / NG, g2 = idx % NG;
    const uint32_t pay = __shfl(mine, g2, 64);
    if (live && p != ar.rank && g2 < pairs) car_put(ar.P.base[p] + car_granule_off(epoch, ar.cap, ar.rank, gbase + g2), pay, epoch);
  }
  if (lane < NG && lane < pairs) {  // collect my granule of every peer, sum in rank order
    const long g[1] = {gbase + lane};
    uint32_t in[kMaxRanks][1];
    car_collect<1>(ar.P, ar.rank, ar.world, ar.cap, epoch, g, in);
    in[ar.rank][0] = mine;
    float lo = 0.f, hi = 0.f;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < ar.world) {
        lo += bf16_lo(in[r][0]);
        hi += bf16_hi(in[r][0]);
      }
    }
    *reinterpret_cast<uint32_t*>(o.h + bo * kOrRows + 2 * lane) = pack_bf16x2(lo, hi);
  }
  if (lane == 0)
    __hip_atomic_store(car_ctr(ar.P.base[ar.rank]) + bo, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int G, int D>
__global__ __launch_bounds__(kQaThreads) void qkv_attn_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ norm_w, float eps, const bf16_t* __restrict__ W, int N,
    int K, RopeEpi rope, const int32_t* __restrict__ block_table, int bt_len,
    const int32_t* __restrict__ seq_len, float* __restrict__ part, int* __restrict__ counters, bf16_t* __restrict__ out,
    int bs, int nblocks, int chunk, int gc, int max_chunks, int gsize, int max_groups, float scale_log2,
    int* __restrict__ fault, uint64_t* __restrict__ granules, int* __restrict__ hctr, OArgs o) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // Block order: every GEMV block (4 rows each, natural row order), then the gc attention blocks
  // of each kv head; an attention block only waits on lower-index blocks. (Per-head segments —
  // a head's GEMV blocks, then its attention blocks — measured the same on one kv head and 3 %
  // slower at 17k keys on two: profiles/r4_qkv_attn.md.)
  const int nq = N / kQaWaves;
  const uint32_t htag =
      static_cast<uint32_t>(__hip_atomic_load(hctr + kCtrPitch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  if (static_cast<int>(blockIdx.x) < nq) {  // block-uniform: the projection of 4 rows
    RopeEpi re = rope;
    re.granules = granules;
    re.gtag = htag;
    gemv_block<1, kQaThreads, 1, 8, PRO_NORM, EPI_ROPE, false>(blockIdx.x, 0, smem, x, K, norm_w, eps, W, nullptr, 0, N,
                                                               K, nullptr, 1, re, CarArgs{});
    return;
  }
  const int A = gc * rope.nkv;
  int* adone = hctr + 2 * kCtrPitch;  // o-role: attention blocks whose head output is written
  const int no = o.mode != 0 ? (o.n_o + kOrRows - 1) / kOrRows : 0;
  if (static_cast<int>(blockIdx.x) >= nq + A) {  // block-uniform: the o-role
    const int bo = blockIdx.x - nq - A;
    // exactly k_o / 512 chunks per lane per row (host: k_o a multiple of 512, <= kOrMaxCpl x 512):
    // a wider instantiation would read past the row (and past W_o at its last row)
    switch (o.k_o / (kWave * 8)) {
      case 1: qa_oproj_block<1>(bo, smem, out, o, adone, A, fault); break;
      case 2: qa_oproj_block<2>(bo, smem, out, o, adone, A, fault); break;
      case 3: qa_oproj_block<3>(bo, smem, out, o, adone, A, fault); break;
      default: qa_oproj_block<kOrMaxCpl>(bo, smem, out, o, adone, A, fault); break;
    }
  } else {
    const int g = (blockIdx.x - nq) / gc, c = (blockIdx.x - nq) % gc;
    const int L = ld_scalar(seq_len);
    if (no == 0) {
      if (c * chunk < L)
        qa_attention<G, D>(c, g, smem, block_table, bt_len, L, rope.k_cache, rope.v_cache, part, counters, out,
                           rope.nh, rope.nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale_log2, fault,
                           granules, htag);
    } else {
      // the head output goes out write-through (sc1): the o-role reads it inside this launch
      if (c * chunk < L)
        qa_attention<G, D, true>(c, g, smem, block_table, bt_len, L, rope.k_cache, rope.v_cache, part, counters, out,
                                 rope.nh, rope.nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale_log2,
                                 fault, granules, htag);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's output stores have left
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(adone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // every attention (and o-role) block counts its exit; the last advances the hand-off epoch and
  // re-arms the o-role's arrival counter (every GEMV block has published by now: each one's
  // granules were waited for, so each one read the epoch; every o-role block is past its wait)
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(hctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A + no - 1) {
      __hip_atomic_store(hctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (no) __hip_atomic_store(adone, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(hctr + kCtrPitch, static_cast<int>(htag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_attn_decode_groups(int max_chunks);

// 0 when (nh, nkv, D, K) is covered: G = nh / nkv in {1, 2, 4, 8}, D in {64, 96, 128} (whole
// 4-row GEMV blocks per head, pairs inside a block), x of K <= 32 Ki bf16 in LDS.
extern "C" int llmc_qkv_attn_check(int nh, int nkv, int D, int K) {
  if (nkv < 1 || nh % nkv != 0 || K % 8 != 0 || K <= 0) return -1;
  const int G = nh / nkv;
  if (!(G == 1 || G == 2 || G == 4 || G == 8) || !(D == 64 || D == 96 || D == 128)) return -3;
  if (static_cast<size_t>(K) * 2 + 64 > 64 * 1024) return -4;
  return 0;
}

// One decode row: q/k/v = rope(W . rmsnorm(x)) (k / v written to the paged cache at slots[0]) and
// out = attention(q, cache keys < L - 1 and this token's key) in the fused form: grid_chunks
// blocks of `chunk` (128 / 256) keys per kv head, bs % (chunk / 4) == 0. part / counters: the
// decode-attention workspace (max_chunks >= grid_chunks, its row 0). granules: u64 [(nh + 2 nkv)
// D / 2]; hctr: int32 [2 kCtrPitch]; both zeroed once.
//
// o-role (o_mode != 0; hctr then int32 [3 kCtrPitch]): the token's o_proj in the same launch, on
// kOrRows-row blocks after the attention blocks: h (o_n rows) += / = w_o [o_n, nh D] . out (o_mode 1 /
// 2), or the tensor-parallel all-reduce in its epilogue (o_mode 3 over `bases`, cap bytes per data
// parity, host status page `host`; rank 0 adds the residual). nh D <= 2048.
extern "C" int llmc_qkv_attn(const void* x, const void* norm_w, float eps, const void* W, int K, void* q_out,
                             void* k_cache, void* v_cache, const void* positions, const void* slots, const void* cos_t,
                             const void* sin_t, const void* block_table, int bt_len, const void* seq_len, void* part,
                             void* counters, void* out, int nh, int nkv, int D, int bs, int nblocks, int chunk,
                             int grid_chunks, int max_chunks, float scale, void* fault, void* granules, void* hctr,
                             int o_mode, const void* w_o, void* h, int o_n, const void* const* bases, void* host,
                             int rank, int world, size_t cap, hipStream_t s) {
  if (llmc_qkv_attn_check(nh, nkv, D, K) != 0) return -1;
  OArgs o{};
  if (o_mode != 0) {
    const int k_o = nh * D;
    if (o_mode < 1 || o_mode > 3 || w_o == nullptr || h == nullptr || o_n < 2 || o_n % 2 != 0 || k_o % 512 != 0 ||
        k_o > kOrMaxCpl * kWave * 8)
      return -1;
    o.w_o = static_cast<const bf16_t*>(w_o);
    o.h = static_cast<bf16_t*>(h);
    o.n_o = o_n;
    o.k_o = k_o;
    o.mode = o_mode;
    if (o_mode == 3) {
      const int no = (o_n + kOrRows - 1) / kOrRows;
      if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || bases == nullptr || no > kMaxBlocks ||
          static_cast<size_t>(no) * kArGranulesPerBlock * 8 > cap / kMaxRanks)
        return -6;
      for (int r = 0; r < kMaxRanks; ++r)
        o.ar.P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
      o.ar.P.host = static_cast<uint32_t*>(host);
      o.ar.rank = rank;
      o.ar.world = world;
      o.ar.cap = static_cast<long>(cap);
    }
  }
  if ((chunk != 128 && chunk != 256) || bs % (chunk / 4) != 0 || grid_chunks < 1 || grid_chunks > max_chunks ||
      bt_len < 1 || nblocks < 1 || counters == nullptr || granules == nullptr || hctr == nullptr)
    return -1;
  const int G = nh / nkv, N = (nh + 2 * nkv) * D;
  const int max_groups = llmc_attn_decode_groups(max_chunks);
  const int gsize = grid_chunks > kAttnOneLevel ? kAttnGroup : grid_chunks;
  const size_t lds_gemv = static_cast<size_t>(K) * 2 + 2 * kQaWaves * sizeof(float);
  const size_t lds_attn = kQaWaves * 32 * kVRowBytes + static_cast<size_t>(kQaWaves) * G * (D + 2) * sizeof(float) +
                          16 + static_cast<size_t>(G * D + 2 * D) * sizeof(bf16_t);
  size_t lds = lds_gemv > lds_attn ? lds_gemv : lds_attn;
  if (lds < kOrRows * sizeof(float)) lds = kOrRows * sizeof(float);
  if (lds > 64 * 1024) return -4;
  RopeEpi rope{(bf16_t*)q_out, nh * D, (bf16_t*)k_cache, (bf16_t*)v_cache, (const int32_t*)positions,
               (const int32_t*)slots, (const float*)cos_t, (const float*)sin_t, nh, nkv, D, bs};
  const dim3 grid(N / kQaWaves + grid_chunks * nkv + (o_mode != 0 ? (o_n + kOrRows - 1) / kOrRows : 0));
  const float sl2 = scale * 1.4426950408889634f;
#define LLMC_QA(GG, DD)                                                                                         \
  qkv_attn_kernel<GG, DD><<<grid, kQaThreads, lds, s>>>(                                                        \
      (const bf16_t*)x, (const bf16_t*)norm_w, eps, (const bf16_t*)W, N, K, rope,                                \
      (const int32_t*)block_table, bt_len, (const int32_t*)seq_len, (float*)part, (int*)counters, (bf16_t*)out,   \
      bs, nblocks, chunk, grid_chunks, max_chunks, gsize, max_groups, sl2, (int*)fault, (uint64_t*)granules,      \
      (int*)hctr, o)
#define LLMC_QA_D(GG)                     \
  if (D == 64) LLMC_QA(GG, 64);           \
  else if (D == 96) LLMC_QA(GG, 96);      \
  else LLMC_QA(GG, 128)
  switch (G) {
    case 1: LLMC_QA_D(1); break;
    case 2: LLMC_QA_D(2); break;
    case 4: LLMC_QA_D(4); break;
    default: LLMC_QA_D(8); break;
  }
#undef LLMC_QA_D
#undef LLMC_QA
  return static_cast<int>(hipGetLastError());
}
