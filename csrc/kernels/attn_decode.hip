// K5: paged decode attention with the GQA group on the matrix cores (one query token per
// sequence), ONE launch per step in both of its forms (host: llmc_attn_decode).
//
// Shared sub-tile step (a wave and 32 keys), mfma_f32_16x16x32_bf16:
//   S^T[key][h] = K . Q^T     A = K (16 keys x 32 dims: one 16-B global load per lane, no LDS),
//                             B = Q^T (32 dims x 16 heads; the G real heads, rest zero) in VGPRs.
//                             C puts head h = lane & 15 on the lane and 4 keys per 16x16 tile in
//                             registers -> per head, 8 of the 32 keys are lane-local and the
//                             row max / row sum need only 2 xor-shuffles (offsets 16, 32).
//   O^T[d][h] += V^T . P^T    B = P^T straight from the S^T accumulators (cvt to bf16; the
//                             k-order is permuted to match, guide §3 "accumulator tile as the next
//                             MFMA's operand"); A = V^T via ds_read_b64_tr_b16 (T10) from a per-wave
//                             LDS image of the 32 V rows, chunk-swizzled c ^ ((row & 7) << 1) so a
//                             half-wave's 8 rows x 32 B hit 64 distinct banks. O^T keeps the head on
//                             the lane, so the online-softmax rescale uses lane-local alpha.
//
// FUSED form (short contexts, <= 4k keys: responders): a block = 4 waves = one kv head x a FIXED
// 128- or 256-key chunk. The chunk does not depend on L, so a wave's page id (its 32/64 keys share
// a page), the length, the merge epoch and Q are loaded together in ONE round trip, then K/V.
// SPLIT form (long contexts: the judge): a block = 8 waves (4 without GQA) = one kv head x one balanced key range
// (the L keys split evenly, in 32-key units, over min(grid_chunks, L / min_chunk) blocks:
// common.h decode_nsplit / decode_range), so a graph captured for a bucket keeps every block
// equally busy whatever the actual L; the block's page ids are staged in LDS once; 8 waves put
// 2 x 16 KB of K/V per wave in flight (the 4-wave form of round 1 left the HBM queue half empty
// and needed a second, reduce launch).
//
// Cross-block merge, both forms, in the same launch, with no fence and no drain: every chunk block
// publishes its normalised partial (O/l per dim in bf16, lambda = m + log2 l per head in f32) as
// 8-byte {value, tag} granules (two per 16-B write-through store; MI355X_MICROARCH.md
// § visibility R2: the data IS the flag) and takes a ticket; the LAST arriver merges every
// partial with an online log-sum-exp, re-polling any granule whose tag is not yet this launch's
// (a store still in flight from a block that has already arrived — never a block that is not yet
// running, so nothing waits on scheduling and no CU is held while co-located engines need it;
// polling mergers that waited on unscheduled producers cost the 3-engine bench 8-20 %). The tag is
// a per-(row, kv head) epoch in device memory the merger advances (tag = epoch + 1: never 0,
// never reused), so a granule left by any earlier launch can never match. Spins are bounded.
#include "attn_core.h"

namespace llmc {

// ---------------------------------------------------------------------------------------------
// One block of the split form: chunk c (of a grid of `gridc` per head) of kv head kvh, row b.
template <int G, int D, int NW>
__device__ __forceinline__ void attn_split_block(
    int c, int kvh, int b, int gridc, const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters, bf16_t* __restrict__ out,
    int out_stride, int nkv, int bs, int nblocks, int min_chunk, int max_chunks, int gsize, int max_groups,
    float scale_log2, int* __restrict__ fault, char* smem) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  constexpr int NT = NW * 64;
  int* ctr = counters + (b * nkv + kvh) * (2 + max_groups) * kCtrPitch;  // {ticket, epoch, group tickets}
  const uint32_t tag = static_cast<uint32_t>(__hip_atomic_load(ctr + kCtrPitch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const int L = seq_lens[b];
  const int nchunks = decode_nsplit(L, gridc, -min_chunk);
  if (c >= nchunks) return;
  int start, end;
  decode_range(L, nchunks, c, -min_chunk, start, end);

  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  char* vbuf = smem + wave * 32 * kVRowBytes;  // per-wave V image [32][256 B]
  float* red = reinterpret_cast<float*>(smem + NW * 32 * kVRowBytes);
  int* pages = reinterpret_cast<int*>(red + NW * G * (D + 2));  // this block's page ids

  ST st;
  st.init(q + static_cast<int64_t>(b) * q_stride + kvh * G * D, lane);
  // stage the block's page ids once (no dependent block-table load per key)
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int p0 = start / bs;
  const int npages = (end - 1) / bs - p0 + 1;
  // page ids clamped into the cache: a corrupt block table reads a wrong page, never a wild address
  for (int i = tid; i < npages; i += NT) pages[i] = min(max(bt[min(p0 + i, bt_stride - 1)], 0), nblocks - 1);
  __syncthreads();
  const int64_t head_stride = static_cast<int64_t>(bs) * D;
  auto row = [&](const bf16_t* cache, int key) {
    const int64_t page = pages[key / bs - p0];
    return cache + (page * nkv + kvh) * head_stride + static_cast<int64_t>(key % bs) * D;
  };

  const int per_wave = (((end - start + NW - 1) / NW) + 31) & ~31;  // 32-key sub-tiles per wave
  const int wbase = start + wave * per_wave;
  bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
  u32x4 vsA[ST::NV], vsB[ST::NV];
  auto valid = [&](int k) { return k - wbase < per_wave && k < end; };  // wave-uniform
  // two named register sets, hand-unrolled (no runtime-indexed register arrays, guide rule 20):
  // the next sub-tile's loads are in flight while the current one computes
  if (valid(wbase)) st.issue(wbase, end, lane, row, k_cache, v_cache, kfA, vsA);
  for (int k0 = wbase;; k0 += 64) {
    if (!valid(k0)) break;
    if (valid(k0 + 32)) st.issue(k0 + 32, end, lane, row, k_cache, v_cache, kfB, vsB);
    st.compute(k0, end, lane, vbuf, scale_log2, kfA, vsA);
    if (!valid(k0 + 32)) break;
    if (valid(k0 + 64)) st.issue(k0 + 64, end, lane, row, k_cache, v_cache, kfA, vsA);
    st.compute(k0 + 32, end, lane, vbuf, scale_log2, kfB, vsB);
  }
  st.to_lds(red, wave, lane);
  __syncthreads();
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  if (nchunks == 1) {
    store_direct<G, D, NW>(red, out_row, tid);
    return;
  }
  publish_and_merge<G, D, NW>(red, part, ctr, b, nkv, kvh, c, nchunks, gsize, max_chunks, max_groups, tag, out_row, smem,
                              reinterpret_cast<int*>(pages), tid, fault);
}

template <int G, int D, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode_split_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters, bf16_t* __restrict__ out,
    int out_stride, int nkv, int bs, int nblocks, int min_chunk, int max_chunks, int gsize, int max_groups,
    float scale_log2, int* __restrict__ fault) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  attn_split_block<G, D, NW>(blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, q, q_stride, k_cache, v_cache, block_tables,
                             bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, min_chunk, max_chunks,
                             gsize, max_groups, scale_log2, fault, smem);
}

// ---------------------------------------------------------------------------------------------
template <int G, int D>
__global__ __launch_bounds__(256) void attn_decode_fused_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters,
    bf16_t* __restrict__ out, int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
    int max_groups, float scale_log2, int* __restrict__ fault) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int per_wave = chunk / 4;  // keys per wave (32 or 64): inside one page (host-checked)
  // ONE round trip for everything that does not depend on the sequence length: the length, this
  // wave's page id (wave-uniform: scalar cache), the merge epoch and Q (vector)
  const int key0 = c * chunk + wave * per_wave;
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int pidx = __builtin_amdgcn_readfirstlane(min(key0 / bs, bt_stride - 1));
  const int page = min(max(ld_scalar(bt + pidx), 0), nblocks - 1);  // clamped into the cache
  const int L = ld_scalar(seq_lens + b);
  int* ctr = counters + (b * nkv + kvh) * (2 + max_groups) * kCtrPitch;  // {ticket, epoch, group tickets}
  const uint32_t tag = static_cast<uint32_t>(__hip_atomic_load(ctr + kCtrPitch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  ST st;
  st.init(q + static_cast<int64_t>(b) * q_stride + kvh * G * D, lane);
  if (c * chunk >= L) return;  // block-uniform
  const int nchunks = (L + chunk - 1) / chunk;
  const int end = min(L, key0 + per_wave);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;
  float* red = reinterpret_cast<float*>(smem + 4 * 32 * kVRowBytes);
  if (key0 < L) {  // wave-uniform
    const int64_t base = (static_cast<int64_t>(page) * nkv + kvh) * bs * D;
    auto row = [&](const bf16_t* cache, int key) { return cache + base + static_cast<int64_t>(key % bs) * D; };
    bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
    u32x4 vsA[ST::NV], vsB[ST::NV];
    st.issue(key0, end, lane, row, k_cache, v_cache, kfA, vsA);
    if (key0 + 32 < end) st.issue(key0 + 32, end, lane, row, k_cache, v_cache, kfB, vsB);
    st.compute(key0, end, lane, vbuf, scale_log2, kfA, vsA);
    if (key0 + 32 < end) st.compute(key0 + 32, end, lane, vbuf, scale_log2, kfB, vsB);
  }
  st.to_lds(red, wave, lane);
  __syncthreads();
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  if (nchunks == 1) {
    store_direct<G, D, 4>(red, out_row, tid);
    return;
  }
  publish_and_merge<G, D, 4>(red, part, ctr, b, nkv, kvh, c, nchunks, gsize, max_chunks, max_groups, tag, out_row, smem,
                             reinterpret_cast<int*>(red + 4 * G * (D + 2)), tid, fault);
}

// Split blocks: 8 waves when a block's balanced range at the table's full length is >= 512 keys
// (2 x 16 KB of K/V in flight per wave), 4 otherwise (wide TP grids: a TP=8 rank's one kv head
// over 256 blocks has ~130 keys per block) and always without GQA (G = 1: Phi-3's 32 kv heads
// already give 512 blocks, and 8-wave blocks at 212 VGPRs would halve the blocks resident per CU).
template <int G, int D, int NW>
static int launch_split_nw(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                           const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                           int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
                           int max_groups, int max_chunk_keys, float scale, int* fault) {
  const size_t lds = NW * 32 * kVRowBytes + static_cast<size_t>(NW) * G * (D + 2) * sizeof(float) +
                     static_cast<size_t>((max_chunk_keys + bs - 1) / bs + 2) * sizeof(int);
  if (lds > 160 * 1024) return -4;
  auto kern = attn_decode_split_kernel<G, D, NW>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  kern<<<grid, NW * 64, lds, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc,
                                  (const int32_t*)bt, bt_stride, (const int32_t*)sl, (float*)part, (int*)ctr,
                                  (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups,
                                  scale * 1.4426950408889634f, fault);
  return static_cast<int>(hipGetLastError());
}

template <int G, int D>
static int launch_split(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                        int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize, int max_groups,
                        float scale, int* fault) {
  // page-id staging sized for the largest balanced range any sequence of this table can get
  const int grid_chunks = static_cast<int>(grid.x);
  const int units = (bt_stride * bs + 31) / 32;
  const int bal = 32 * ((units + grid_chunks - 1) / grid_chunks) + 32;
  const int max_chunk = bal > 2 * chunk ? bal : 2 * chunk;
  // a minimum block range of >= 512 keys (the length-only split of batching engines) always takes
  // 8 waves, so a row's per-wave key partition never depends on the bucket its batch selected
  if (G > 1 && (bal >= 512 || chunk >= 512))
    return launch_split_nw<G, D, 8>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv,
                                    bs, nblocks, chunk, max_chunks, gsize, max_groups, max_chunk, scale, fault);
  return launch_split_nw<G, D, 4>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv, bs,
                                  nblocks, chunk, max_chunks, gsize, max_groups, max_chunk, scale, fault);
}

template <int G, int D>
static int launch_fused(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                        int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize, int max_groups,
                        float scale, int* fault) {
  const size_t lds = 4 * 32 * kVRowBytes + static_cast<size_t>(4) * G * (D + 2) * sizeof(float) + 16;  // + flag
  if (lds > 64 * 1024) return -4;
  attn_decode_fused_kernel<G, D><<<grid, 256, lds, s>>>(
      (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt, bt_stride,
      (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize,
      max_groups, scale * 1.4426950408889634f, fault);
  return static_cast<int>(hipGetLastError());
}

template <int G>
static int launch_g(bool fused, int D, dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc,
                    const void* vc, const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                    int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
                    int max_groups, float scale, int* fault) {
#define LLMC_ATTN_D(DD)                                                                                          \
  case DD:                                                                                                       \
    return fused ? launch_fused<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, \
                                       nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, fault)     \
                 : launch_split<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, \
                                       nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, fault);
  switch (D) {
    LLMC_ATTN_D(64)
    LLMC_ATTN_D(96)
    LLMC_ATTN_D(128)
    default: return -2;
  }
#undef LLMC_ATTN_D
}

}  // namespace llmc

using namespace llmc;

// Attention of one decode step for rows 0..B-1, one launch.
// part: f32 [B, nkv, max_chunks + max_groups, G, D + 4] partial granules (zeroed once); counters:
// int32 [B, nkv, 2 + max_groups, kCtrPitch] {top ticket, epoch, group tickets}, one 128-B line per
// word (zeroed once; the kernel re-arms
// the tickets and advances the epoch); max_groups = attn_decode_groups(max_chunks).
// fused = 1 (short contexts): grid_chunks fixed chunk-key blocks (chunk 128 or 256; bs % (chunk/4) == 0).
// fused = 0 (long contexts): balanced split over <= grid_chunks blocks of >= chunk keys (multiple of 128).
// Chunk partials are merged in one level up to kAttnOneLevel chunks, else in groups of kAttnGroup.
// fault (nullable int32): set to 1 when a merger gave up waiting for a partial (bounded spin): the
// step's attention output is then invalid and the caller must fail the request.

extern "C" int llmc_attn_decode_groups(int max_chunks) {
  return max_chunks > kAttnOneLevel ? (max_chunks + kAttnGroup - 1) / kAttnGroup : 0;
}

extern "C" int llmc_attn_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                int nblocks, int chunk, int grid_chunks, int max_chunks, float scale, int fused,
                                void* fault, hipStream_t s) {
  if (nh % nkv != 0 || grid_chunks > max_chunks || grid_chunks < 1 || nblocks < 1 || counters == nullptr ||
      bt_stride < 1)
    return -1;
  if (fused ? ((chunk != 128 && chunk != 256) || bs % (chunk / 4) != 0) : (chunk % 128 != 0)) return -1;
  const int G = nh / nkv;
  const int max_groups = llmc_attn_decode_groups(max_chunks);
  const int gsize = grid_chunks > kAttnOneLevel ? kAttnGroup : grid_chunks;
  if (static_cast<int64_t>(max_chunks + max_groups) * G * (D / 4 + 1) * 16 >= (1ll << 31)) return -4;
  dim3 grid(grid_chunks, nkv, B);
  const bool f = fused != 0;
  switch (G) {
    case 1: return launch_g<1>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 2: return launch_g<2>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 4: return launch_g<4>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 8: return launch_g<8>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    default: return -3;
  }
}
