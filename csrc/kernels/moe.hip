// K9 router top-k, K10 permute/align, K12 combine for Mixtral-style MoE.
// The expert GEMMs themselves are K11: gemm_kernel<.., GATHER> (prefill) and
// gemv_kernel<.., EXPERT> (decode) — same MFMA / weight-streaming cores as the dense layers.
//
// Data flow (prefill, T tokens, top-k):
//   router logits [T, E] f32 --moe_route--> w [T, k] f32, ids [T, k] i32
//   ids --moe_align--> sorted_rows [cap] (pair index t*k+j grouped by expert, each expert padded
//                      to 128- or 256-row tiles, -1 = pad), tile_expert [max_tiles], tile_count [1]
//   x [T, H] --gemm<GATHER, EPI_SILU>(a_row_div = k)--> act [T*k, I]   (SiLU-mul in the epilogue)
//   act --gemm<GATHER>(a_row_div = 1)--> y [T*k, H] --moe_combine--> h[t] += sum_j w[t,j] y[t*k+j]
// The combine is a fixed-order sum in f32 (no float atomics: bitwise reproducible,
// MI355X_MICROARCH.md "Global float atomics" pitfall). Expert parallel: moe_ep_localize maps the
// router's global ids to this rank's experts (-1, weight 0 elsewhere); expert GEMV blocks of a -1
// pair exit and the combine skips zero-weight pairs.
#include <algorithm>

#include "common.h"

namespace llmc {

// one thread per token; E <= 64, k <= 8. Mixtral: softmax over all experts, top-k, renormalise.
// The token's logits are loaded ONCE into registers (every loop has a compile-time bound, guarded
// by E / k): re-reading l[e] in each of the (2 + k) passes made every pass a chain of dependent
// global loads (~144 us for 2048 tokens x 8 experts in the round-6 EP prefill trace).
__global__ void moe_route_kernel(const float* __restrict__ logits, int T, int E, int k, float* __restrict__ w,
                                 int32_t* __restrict__ ids) {
  constexpr int kMaxE = 64, kMaxK = 8;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const float* l = logits + static_cast<int64_t>(t) * E;
  float v[kMaxE];
#pragma unroll
  for (int e = 0; e < kMaxE; ++e) v[e] = e < E ? l[e] : -INFINITY;
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < kMaxE; ++e) mx = fmaxf(mx, v[e]);
  float z = 0.f;
#pragma unroll
  for (int e = 0; e < kMaxE; ++e)
    if (e < E) z += __expf(v[e] - mx);
  uint64_t taken = 0;
  float sel[kMaxK];
  int pick[kMaxK];
  float ssum = 0.f;
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) {
    sel[j] = 0.f;
    pick[j] = -1;
    if (j < k) {
      int best = -1;
      float bv = -INFINITY;
#pragma unroll
      for (int e = 0; e < kMaxE; ++e) {
        const bool ok = e < E && !((taken >> e) & 1ull) && (best < 0 || v[e] > bv);  // first max wins ties
        bv = ok ? v[e] : bv;
        best = ok ? e : best;
      }
      taken |= 1ull << best;
      sel[j] = __expf(bv - mx) / z;
      pick[j] = best;
      ssum += sel[j];
    }
  }
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) {
    if (j < k) {
      ids[static_cast<int64_t>(t) * k + j] = pick[j];
      w[static_cast<int64_t>(t) * k + j] = sel[j] / ssum;
    }
  }
}

// Prefill router, fused (replaces the router-logits GEMM + moe_route_kernel pair of the prefill
// path: the GEMM ran as a narrow-N tile grid of M / 128 blocks for N = 8 outputs, ~125 us per
// 2048-token layer, latency-bound): logits = x . Wr^T in f32, softmax, top-k, renormalise, ONE
// launch. Each block stages the E x H router weights in LDS once (64 KB for Mixtral), then every
// wave takes whole tokens: all of the token's 16-B x chunks in flight at once, E dot products per
// lane against the LDS rows (lane-consecutive chunks: conflict-free), E wave sums, and lane 0 picks
// the top-k (first max wins ties, as moe_route_kernel). x = the normalised rows the expert GEMMs
// also read.
constexpr int kRouteFusedMaxE = 16, kRouteFusedPre = 16;  // experts; x chunks per lane (H <= 8192)

constexpr int kRouteFusedThreads = 512;

__global__ __launch_bounds__(kRouteFusedThreads) void moe_route_fused_kernel(const bf16_t* __restrict__ x, int x_stride,
                                                              const bf16_t* __restrict__ Wr, int T, int E, int H,
                                                              int k, float* __restrict__ w_out,
                                                              int32_t* __restrict__ ids_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u32x4* wl = reinterpret_cast<u32x4*>(smem);  // [E][H / 8]
  const int nch = H / 8;
  for (int i = threadIdx.x; i < E * nch; i += kRouteFusedThreads) wl[i] = reinterpret_cast<const u32x4*>(Wr)[i];
  __syncthreads();
  constexpr int kW = kRouteFusedThreads / kWave;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  for (int t = blockIdx.x * kW + wave; t < T; t += gridDim.x * kW) {  // wave-uniform
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(t) * x_stride);
    u32x4 xv[kRouteFusedPre];
#pragma unroll
    for (int i = 0; i < kRouteFusedPre; ++i) {
      const int c = lane + i * kWave;
      if (c < nch) xv[i] = xr[c];
    }
    float acc[kRouteFusedMaxE];
#pragma unroll
    for (int e = 0; e < kRouteFusedMaxE; ++e) {
      acc[e] = 0.f;
      if (e < E) {
#pragma unroll
        for (int i = 0; i < kRouteFusedPre; ++i) {
          const int c = lane + i * kWave;
          if (c < nch) acc[e] = dot8_bf16(wl[e * nch + c], xv[i], acc[e]);
        }
        acc[e] = wave_sum(acc[e]);
      }
    }
    if (lane == 0) {
      float mx = -INFINITY;
#pragma unroll
      for (int e = 0; e < kRouteFusedMaxE; ++e)
        if (e < E) mx = fmaxf(mx, acc[e]);
      float z = 0.f;
#pragma unroll
      for (int e = 0; e < kRouteFusedMaxE; ++e)
        if (e < E) z += __expf(acc[e] - mx);
      uint32_t taken = 0;
      float sel[8];
      int pick[8];
      float ssum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sel[j] = 0.f;
        pick[j] = -1;
        if (j < k) {
          int best = -1;
          float bv = -INFINITY;
#pragma unroll
          for (int e = 0; e < kRouteFusedMaxE; ++e) {
            const bool ok = e < E && !((taken >> e) & 1u) && (best < 0 || acc[e] > bv);
            bv = ok ? acc[e] : bv;
            best = ok ? e : best;
          }
          taken |= 1u << best;
          sel[j] = __expf(bv - mx) / z;
          pick[j] = best;
          ssum += sel[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < k) {
          ids_out[static_cast<int64_t>(t) * k + j] = pick[j];
          w_out[static_cast<int64_t>(t) * k + j] = sel[j] / ssum;
        }
      }
    }
  }
}

// Decode router, fused: RMSNorm of the token's hidden row -> router GEMV (one wave per expert,
// the E x H router weights streamed once) -> softmax / top-k / renormalise, in ONE launch of one
// block per token (replaces rmsnorm + router GEMV + moe_route: three latency-bound launches per
// MoE layer). The expert GEMVs normalise x again in their own prologue (PRO_NORM), so the normed
// row is never written to memory. H <= 8 * 512 * 2 (two 16-B chunks per thread).
constexpr int kRouterThreads = 512;

__global__ __launch_bounds__(kRouterThreads) void moe_router_kernel(
    const bf16_t* __restrict__ x, int x_stride, const bf16_t* __restrict__ norm_w, float eps,
    const bf16_t* __restrict__ Wr, int E, int H, int k, float* __restrict__ w_out, int32_t* __restrict__ ids_out) {
  constexpr int WAVES = kRouterThreads / kWave;
  __shared__ __attribute__((aligned(16))) bf16_t xs[8192];
  __shared__ float red[WAVES];
  __shared__ float logit[64];
  const int t = blockIdx.x, tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int nchunk = H / 8;
  const bf16_t* xr = x + static_cast<int64_t>(t) * x_stride;
  // The router weights do not depend on x: with one expert per wave (E <= 8 waves) the wave's whole
  // row is requested FIRST, so its HBM round trip overlaps the x load and the norm instead of
  // following them (one memory round trip on the launch's chain instead of two; Mixtral: E = 8,
  // H = 4096 -> 8 chunks per lane). x and the norm weights are issued right behind.
  constexpr int kPre = 16;  // chunks per lane preloaded (H <= 8192)
  const bool pre = E <= WAVES && nchunk <= kPre * kWave;  // block-uniform
  u32x4 wpre[kPre];
  if (pre && wave < E) {
    const u32x4* wr = reinterpret_cast<const u32x4*>(Wr + static_cast<int64_t>(wave) * H);
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
      const int c = lane + i * kWave;
      if (c < nchunk) wpre[i] = load16<true>(wr + c);
    }
  }
  u32x4 xv[2], gv[2];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = tid + j * kRouterThreads;
    if (c < nchunk) {
      xv[j] = reinterpret_cast<const u32x4*>(xr)[c];
      gv[j] = reinterpret_cast<const u32x4*>(norm_w)[c];
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (tid + j * kRouterThreads < nchunk) {
      float f[8];
      unpack8(xv[j], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
    }
  }
  const float tot = block_sum<kRouterThreads>(ss, red);
  const float inv = rsqrtf(tot / H + eps);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = tid + j * kRouterThreads;
    if (c < nchunk) {
      float f[8], g[8];
      unpack8(xv[j], f);
      unpack8(gv[j], g);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] * inv * g[e];
      reinterpret_cast<u32x4*>(xs)[c] = pack8(f);  // bf16, as the standalone rmsnorm would store it
    }
  }
  __syncthreads();
  const u32x4* xsv = reinterpret_cast<const u32x4*>(xs);
  if (pre) {
    if (wave < E) {
      float acc = 0.f;  // same chunk order as the loop below: bit-identical logits
#pragma unroll
      for (int i = 0; i < kPre; ++i) {
        const int c = lane + i * kWave;
        if (c < nchunk) acc = dot8_bf16(wpre[i], xsv[c], acc);
      }
      acc = wave_sum(acc);
      if (lane == 0) logit[wave] = acc;
    }
  } else {
    for (int e = wave; e < E; e += WAVES) {
    const u32x4* wr = reinterpret_cast<const u32x4*>(Wr + static_cast<int64_t>(e) * H);
    float acc = 0.f;
    for (int c = lane; c < nchunk; c += kWave) acc = dot8_bf16(load16<true>(wr + c), xsv[c], acc);
    acc = wave_sum(acc);
    if (lane == 0) logit[e] = acc;
    }
  }
  __syncthreads();
  if (tid == 0) {
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) mx = fmaxf(mx, logit[e]);
    float z = 0.f;
    for (int e = 0; e < E; ++e) z += __expf(logit[e] - mx);
    uint64_t taken = 0;
    float sel[8];
    float ssum = 0.f;
    for (int j = 0; j < k; ++j) {
      int best = -1;
      float bv = -INFINITY;
      for (int e = 0; e < E; ++e) {
        if ((taken >> e) & 1ull) continue;
        if (logit[e] > bv) {
          bv = logit[e];
          best = e;
        }
      }
      taken |= 1ull << best;
      sel[j] = __expf(bv - mx) / z;
      ssum += sel[j];
      ids_out[static_cast<int64_t>(t) * k + j] = best;
    }
    for (int j = 0; j < k; ++j) w_out[static_cast<int64_t>(t) * k + j] = sel[j] / ssum;
  }
}

constexpr int kAlignThreads = 1024;
constexpr int kMaxEpRanks = 8;  // expert-parallel group size (one node)

__global__ __launch_bounds__(kAlignThreads) void moe_align_kernel(const int32_t* __restrict__ ids, int npairs, int E,
                                                                  int cap, int max_tiles, int tile,
                                                                  int32_t* __restrict__ sorted_rows,
                                                                  int32_t* __restrict__ tile_expert,
                                                                  int32_t* __restrict__ tile_count,
                                                                  int32_t* __restrict__ counts_out) {
  __shared__ int cnt[64];
  __shared__ int off[65];
  __shared__ int cur[64];
  for (int e = threadIdx.x; e < E; e += kAlignThreads) {
    cnt[e] = 0;
    cur[e] = 0;
  }
  for (int i = threadIdx.x; i < cap; i += kAlignThreads) sorted_rows[i] = -1;
  __syncthreads();
  // ids < 0: a pair of another rank's expert (expert parallel) or an all-to-all padding slot —
  // not placed in any tile, so the grouped GEMM never reads or writes its row
  for (int i = threadIdx.x; i < npairs; i += kAlignThreads)
    if (ids[i] >= 0) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int o = 0;
    for (int e = 0; e < E; ++e) {
      off[e] = o;
      const int nt = (cnt[e] + tile - 1) / tile;
      for (int tt = 0; tt < nt; ++tt) tile_expert[o / tile + tt] = e;
      o += nt * tile;
      if (counts_out) counts_out[e] = cnt[e];
    }
    off[E] = o;
    tile_count[0] = o / tile;
    for (int tt = o / tile; tt < max_tiles; ++tt) tile_expert[tt] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < npairs; i += kAlignThreads) {
    const int e = ids[i];
    if (e < 0) continue;
    const int pos = off[e] + atomicAdd(&cur[e], 1);
    sorted_rows[pos] = i;
  }
}

// Expert-parallel dispatch plan of the sequence-parallel prefill (C4): pair i = t * k + j of this
// rank's token shard goes to rank d = ids[i] / El. Its slot in the send buffer is d * cap + r, r =
// its rank among the pairs bound for d in pair order (stable, so the plan is deterministic). All
// outputs stay on the device (no host sync in the layer loop; the all-to-all moves cap rows per
// peer): send_pair [n * cap] pair index or -1 (padding), send_e [n * cap] the expert id local to
// rank d or -1, pair_slot [npairs] = the slot (the un-permute map of the rows coming back),
// counts [n]. One block of 16 waves: each wave owns a contiguous run of pairs; pass 1 counts its
// pairs per destination with ballots, a prefix over the waves gives every wave its first slot per
// destination, pass 2 places each pair at that offset plus its rank within the 64-pair ballot.
constexpr int kDispatchWaves = 16;

__global__ __launch_bounds__(kDispatchWaves * kWave) void moe_ep_dispatch_kernel(
    const int32_t* __restrict__ ids, int npairs, int El, int n, int cap, int32_t* __restrict__ send_pair,
    int32_t* __restrict__ send_e, int32_t* __restrict__ pair_slot, int32_t* __restrict__ counts) {
  __shared__ int wcnt[kDispatchWaves][kMaxEpRanks];
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  for (int i = tid; i < n * cap; i += kDispatchWaves * kWave) {
    send_pair[i] = -1;
    send_e[i] = -1;
  }
  const int seg = (npairs + kDispatchWaves * kWave - 1) / (kDispatchWaves * kWave) * kWave;
  const int lo = wave * seg, hi = min(npairs, lo + seg);
  int c[kMaxEpRanks];
#pragma unroll
  for (int d = 0; d < kMaxEpRanks; ++d) c[d] = 0;
  for (int base = lo; base < hi; base += kWave) {
    const int i = base + lane;
    const int dst = i < hi ? ids[i] / El : -1;
#pragma unroll
    for (int d = 0; d < kMaxEpRanks; ++d)
      if (d < n) c[d] += __popcll(__ballot(dst == d));
  }
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < kMaxEpRanks; ++d) wcnt[wave][d] = c[d];
  }
  __syncthreads();  // also orders the padding fill above before the placement below
  int run[kMaxEpRanks];
#pragma unroll
  for (int d = 0; d < kMaxEpRanks; ++d) {
    int o = 0;
    for (int w = 0; w < wave; ++w) o += wcnt[w][d];
    run[d] = o;
  }
  if (tid < n) {
    int o = 0;
    for (int w = 0; w < kDispatchWaves; ++w) o += wcnt[w][tid];
    counts[tid] = o;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  for (int base = lo; base < hi; base += kWave) {
    const int i = base + lane;
    const int e = i < hi ? ids[i] : -1;
    const int dst = e >= 0 ? e / El : -1;
    int slot = -1;
#pragma unroll
    for (int d = 0; d < kMaxEpRanks; ++d) {
      if (d >= n) break;
      const uint64_t b = __ballot(dst == d);
      if (dst == d) slot = d * cap + run[d] + __popcll(b & below);
      run[d] += __popcll(b);
    }
    if (slot >= 0) {
      send_pair[slot] = i;
      send_e[slot] = e - dst * El;
      pair_slot[i] = slot;
    }
  }
}

// out[j] = x[rows[j] / div] (bf16 rows of H), zeros where rows[j] < 0: the send buffer of the
// expert-parallel all-to-all (row j = slot j of moe_ep_dispatch's plan, div = top-k).
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16_t* __restrict__ x, int x_stride,
                                                          const int32_t* __restrict__ rows, int div, int H,
                                                          bf16_t* __restrict__ out, int out_stride) {
  const int j = blockIdx.x;
  const int r = rows[j];
  u32x4* o = reinterpret_cast<u32x4*>(out + static_cast<int64_t>(j) * out_stride);
  if (r < 0) {
    for (int c = threadIdx.x; c < H / 8; c += 256) o[c] = u32x4{0u, 0u, 0u, 0u};
    return;
  }
  const u32x4* src = reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(r / div) * x_stride);
  for (int c = threadIdx.x; c < H / 8; c += 256) o[c] = src[c];
}

// h[t] (bf16, in place) += sum_j w[t, j] * y[row(t*k + j)], row = rows[.] when given (the expert-
// parallel all-to-all's returned slots, moe_ep_dispatch pair_slot), else the pair index itself
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16_t* __restrict__ y, const float* __restrict__ w,
                                                          bf16_t* __restrict__ h, int k, int H,
                                                          const int32_t* __restrict__ rows) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float acc[8];
    unpack8(reinterpret_cast<const u32x4*>(h + static_cast<int64_t>(t) * H)[c], acc);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = w[static_cast<int64_t>(t) * k + j];
      if (wj == 0.f) continue;  // another rank's expert (expert parallel): its y row is not written
      float f[8];
      const int64_t yr = rows != nullptr ? rows[static_cast<int64_t>(t) * k + j] : static_cast<int64_t>(t) * k + j;
      unpack8(reinterpret_cast<const u32x4*>(y + yr * H)[c], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += wj * f[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += s[q];
    reinterpret_cast<u32x4*>(h + static_cast<int64_t>(t) * H)[c] = pack8(acc);
  }
}

// expert parallel: global expert id -> local id on this rank (-1 + weight 0 for other ranks')
__global__ void moe_ep_localize_kernel(const int32_t* __restrict__ ids, const float* __restrict__ w, int n, int e0,
                                       int n_local, int32_t* __restrict__ lids, float* __restrict__ lw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = ids[i] - e0;
  const bool mine = e >= 0 && e < n_local;
  lids[i] = mine ? e : -1;
  lw[i] = mine ? w[i] : 0.f;
}

}  // namespace llmc

using namespace llmc;

extern "C" {

int llmc_moe_route(const void* logits, int T, int E, int k, void* w, void* ids, hipStream_t s) {
  if (E > 64 || k > 8 || k > E) return -1;
  moe_route_kernel<<<(T + 255) / 256, 256, 0, s>>>((const float*)logits, T, E, k, (float*)w, (int32_t*)ids);
  return static_cast<int>(hipGetLastError());
}

// Prefill router in one launch (moe_route_fused_kernel): E <= 16, k <= min(8, E), H % 8 == 0,
// H <= 8192 (x chunks per lane), E * H * 2 bytes of LDS.
int llmc_moe_route_fused(const void* x, int x_stride, const void* Wr, int T, int E, int H, int k, void* w, void* ids,
                         hipStream_t s) {
  if (E < 1 || E > kRouteFusedMaxE || k < 1 || k > 8 || k > E || H % 8 != 0 || H > kRouteFusedPre * kWave * 8 ||
      x_stride % 8 != 0)
    return -1;
  if (T <= 0) return 0;
  const size_t lds = static_cast<size_t>(E) * H * 2;
  if (lds > 160 * 1024) return -1;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(moe_route_fused_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  // 8-wave blocks, up to two per CU (64 KB of router weights each for Mixtral): 16 waves per CU,
  // one token per wave up to 4096 tokens (measured 4-wave blocks at <= 256 per grid: 19.6 us at 2048
  // tokens, 67.9 at 8192)
  const int grid = std::min(512, (T + kRouteFusedThreads / kWave - 1) / (kRouteFusedThreads / kWave));
  moe_route_fused_kernel<<<grid, kRouteFusedThreads, lds, s>>>((const bf16_t*)x, x_stride, (const bf16_t*)Wr, T, E, H, k, (float*)w,
                                                (int32_t*)ids);
  return static_cast<int>(hipGetLastError());
}

int llmc_moe_router(const void* x, int x_stride, const void* norm_w, float eps, const void* Wr, int T, int E, int H,
                    int k, void* w, void* ids, hipStream_t s) {
  if (E > 64 || k > 8 || k > E || H % 8 != 0 || H > 8192) return -1;
  moe_router_kernel<<<T, kRouterThreads, 0, s>>>((const bf16_t*)x, x_stride, (const bf16_t*)norm_w, eps,
                                                 (const bf16_t*)Wr, E, H, k, (float*)w, (int32_t*)ids);
  return static_cast<int>(hipGetLastError());
}

// tile must be 128 (the grouped GEMM's M tile); max_tiles = ceil(npairs/128) + E
int llmc_moe_align(const void* ids, int T, int k, int E, int tile, void* sorted_rows, void* tile_expert,
                   void* tile_count, void* counts, hipStream_t s) {
  if ((tile != 128 && tile != 256) || E > 64) return -1;
  const int npairs = T * k;
  const int max_tiles = (npairs + tile - 1) / tile + E;
  moe_align_kernel<<<1, kAlignThreads, 0, s>>>((const int32_t*)ids, npairs, E, max_tiles * tile, max_tiles, tile,
                                               (int32_t*)sorted_rows, (int32_t*)tile_expert, (int32_t*)tile_count,
                                               (int32_t*)counts);
  return static_cast<int>(hipGetLastError());
}

// rows: nullptr = y row t*k + j for pair (t, j); else y row rows[t*k + j] (expert-parallel return slots)
int llmc_moe_combine(const void* y, const void* w, const void* rows, void* h, int T, int k, int H, hipStream_t s) {
  if (H % 8 != 0) return -1;
  if (T <= 0) return 0;
  moe_combine_kernel<<<T, 256, 0, s>>>((const bf16_t*)y, (const float*)w, (bf16_t*)h, k, H, (const int32_t*)rows);
  return static_cast<int>(hipGetLastError());
}

int llmc_moe_ep_dispatch(const void* ids, int npairs, int El, int n, int cap, void* send_pair, void* send_e,
                         void* pair_slot, void* counts, hipStream_t s) {
  if (n < 1 || n > kMaxEpRanks || El < 1 || npairs < 0 || cap < npairs || cap < 1) return -1;
  moe_ep_dispatch_kernel<<<1, kDispatchWaves * kWave, 0, s>>>((const int32_t*)ids, npairs, El, n, cap,
                                                               (int32_t*)send_pair, (int32_t*)send_e,
                                                               (int32_t*)pair_slot, (int32_t*)counts);
  return static_cast<int>(hipGetLastError());
}

int llmc_gather_rows(const void* x, int x_stride, const void* rows, int M, int div, int H, void* out, int out_stride,
                     hipStream_t s) {
  if (H % 8 != 0 || x_stride % 8 != 0 || out_stride % 8 != 0 || div < 1) return -1;
  if (M <= 0) return 0;
  gather_rows_kernel<<<M, 256, 0, s>>>((const bf16_t*)x, x_stride, (const int32_t*)rows, div, H, (bf16_t*)out,
                                       out_stride);
  return static_cast<int>(hipGetLastError());
}

int llmc_moe_ep_localize(const void* ids, const void* w, int n, int e0, int n_local, void* lids, void* lw,
                         hipStream_t s) {
  if (n <= 0) return 0;
  moe_ep_localize_kernel<<<(n + 255) / 256, 256, 0, s>>>((const int32_t*)ids, (const float*)w, n, e0, n_local,
                                                         (int32_t*)lids, (float*)lw);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
