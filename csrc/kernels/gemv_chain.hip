// A batch-1 decode layer's MLP and the next layer's qkv projection as ONE launch of three GEMV
// phases (hand-off protocol: gemv_core.h ChainWait):
//
//   phase A  gate_up_l   act  = silu(g) * u  of  W_gu . rmsnorm(h) * ln2        (PRO_NORM, EPI_SILU)
//   phase B  down_l      h   += W_down . act                                    (EPI_RESADD)
//   phase C  qkv_{l+1}   q, k/v cache <- RoPE(W_qkv . rmsnorm(h) * ln1_{l+1})   (PRO_NORM, EPI_ROPE)
//
// Without the chain these are three launches, each paying a boundary plus its own ramp and tail
// (~3.8 us per GEMV launch on Llama-3-8B shapes: profiles/r4_dec9k_kernel_stats_final.md fits
// t = 3.8 us + bytes / 7.4 TB/s over qkv, down and gate_up). In one grid the next phase's blocks
// are dispatched as the previous phase's last blocks drain, issue their first weight batch at once
// and only then wait for the hand-off, so the weight stream does not stop at the phase edge.
// Phase C is optional (the last layer: the chain ends at down and lm_head follows).
//
// Numerics: every phase is gemv_block with one row per wave, so each dot product is summed in the
// same order as in the separate launches (a lane's chunks in order, then the wave sum: independent
// of the waves per block and the loads in flight). gate_up and down are bit-identical to their
// launches; qkv's RMS norm sums its squares over 16 waves here against 12 in its own launch, so its
// outputs may differ by a bf16 rounding of the normalised input (tests/test_gemv_chain_gpu.py).
#include "gemv_core.h"

namespace llmc {

struct ChainPhase {
  const bf16_t* x;       // [K] this phase's input row
  const bf16_t* norm_w;  // [K] (PRO_NORM phases)
  const bf16_t* W;       // [N, K]
  void* out;             // output row (phase C: unused, RoPE epilogue)
  int N, K, blocks;
};

constexpr int kChainNT = 1024;  // 16 waves: 16 rows per block in every phase

template <int UB, bool QKV>
__global__ __launch_bounds__(kChainNT) void gemv_chain_kernel(ChainPhase a, ChainPhase b, ChainPhase c, RopeEpi rope,
                                                              float eps, ChainWait wab, ChainWait wbc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int bx = blockIdx.x;
  if (bx < a.blocks) {
    gemv_block<1, kChainNT, 1, 4, PRO_NORM, EPI_SILU, false, CH_COHERENT>(
        bx, 0, smem, a.x, 0, a.norm_w, eps, a.W, a.out, 0, a.N, a.K, nullptr, 1, RopeEpi{}, CarArgs{});
    chain_signal(wab.ctr);
    return;
  }
  bx -= a.blocks;
  if (!QKV || bx < b.blocks) {
    gemv_block<1, kChainNT, 1, UB, PRO_NONE, EPI_RESADD, false, CH_WAIT | (QKV ? CH_COHERENT : 0)>(
        bx, 0, smem, b.x, 0, nullptr, eps, b.W, b.out, 0, b.N, b.K, nullptr, 1, RopeEpi{}, CarArgs{}, &wab);
    if constexpr (QKV) chain_signal(wbc.ctr);
    return;
  }
  if constexpr (QKV) {
    bx -= b.blocks;
    gemv_block<1, kChainNT, 1, 4, PRO_NORM, EPI_ROPE, false, CH_WAIT>(bx, 0, smem, c.x, 0, c.norm_w, eps, c.W, nullptr,
                                                                     0, c.N, c.K, nullptr, 1, rope, CarArgs{}, &wbc);
  }
}

static ChainWait chain_wait_for(int* ctr, int first, int producers, int consumers, int* fault, int flags) {
  ChainWait w{};
  w.probe_nowait = flags & 1;
  w.poll_sleep = 1 + ((flags >> 4) & 0xff);
  w.ctr = ctr;
  for (int s = 0; s < kChainShards; ++s) w.expect[s] = 0;
  for (int i = first; i < first + producers; ++i) ++w.expect[i % kChainShards];
  w.consumers = consumers;
  w.fault = fault;
  return w;
}

}  // namespace llmc

using namespace llmc;

// Counter words of the chain workspace (int32, zeroed once, re-armed by the kernel itself).
extern "C" int llmc_gemv_chain_ws_words() { return 2 * (kChainShards + 1) * kChainPitch; }

// h: [H] bf16 residual row (phase A input, phase B output, phase C input); act: [I] bf16;
// W_gu [2I, H] (interleaved gate/up rows), W_down [H, I]; qkv (W_qkv != nullptr): W_qkv [Nq, H] with
// the RoPE / paged-KV-write epilogue as llmc_gemv_qkv_rope. ws: llmc_gemv_chain_ws_words() int32.
// down_unroll: 16-B loads per lane in flight in phase B (4 or 8). flags (microbenchmarks): bit 0
// consumers skip the wait (wrong results: the overlap bound), bits 4-11 extra poll sleeps.
extern "C" int llmc_gemv_chain(void* h, const void* ln2, const void* W_gu, void* act, const void* W_down, int H, int I,
                               const void* ln1_next, const void* W_qkv, int Nq, void* q_out, void* k_cache,
                               void* v_cache, const void* positions, const void* slots, const void* cos_t,
                               const void* sin_t, int nh, int nkv, int D, int bs, float eps, void* ws, void* fault,
                               int down_unroll, int flags, hipStream_t s) {
  constexpr int WAVES = kChainNT / kWave;
  const bool qkv = W_qkv != nullptr;
  // every phase stages its x in registers (x_fast: K <= 2 x 1024 chunks of 8) and tiles its rows
  // by whole blocks (paired epilogues: 16 rows = 8 pairs per block)
  if (H % 8 != 0 || I % 8 != 0 || H / 8 > 2 * kChainNT || I / 8 > 2 * kChainNT) return -1;
  if ((2 * I) % (2 * WAVES) != 0 || H % WAVES != 0) return -1;
  if (qkv && (Nq != (nh + 2 * nkv) * D || Nq % (2 * WAVES) != 0 || D % 2 != 0)) return -1;
  if (down_unroll != 4 && down_unroll != 8) return -1;
  ChainPhase a{static_cast<const bf16_t*>(h), static_cast<const bf16_t*>(ln2), static_cast<const bf16_t*>(W_gu), act,
               2 * I, H, 2 * I / WAVES};
  ChainPhase b{static_cast<const bf16_t*>(act), nullptr, static_cast<const bf16_t*>(W_down), h, H, I, H / WAVES};
  ChainPhase c{static_cast<const bf16_t*>(h), static_cast<const bf16_t*>(ln1_next), static_cast<const bf16_t*>(W_qkv),
               nullptr, Nq, H, qkv ? Nq / WAVES : 0};
  RopeEpi rope{};
  if (qkv)
    rope = RopeEpi{(bf16_t*)q_out, nh * D, (bf16_t*)k_cache, (bf16_t*)v_cache, (const int32_t*)positions,
                   (const int32_t*)slots, (const float*)cos_t, (const float*)sin_t, nh, nkv, D, bs};
  int* ctr = static_cast<int*>(ws);
  const ChainWait wab = chain_wait_for(ctr, 0, a.blocks, b.blocks, static_cast<int*>(fault), flags);
  const ChainWait wbc = chain_wait_for(ctr + (kChainShards + 1) * kChainPitch, a.blocks, b.blocks, c.blocks,
                                       static_cast<int*>(fault), flags);
  // x [K] bf16 | norm partials [WAVES] f32 | pair exchange [WAVES / 2] f32, for the widest phase
  const size_t lds = static_cast<size_t>(H > I ? H : I) * sizeof(bf16_t) + 2 * WAVES * sizeof(float);
  const int grid = a.blocks + b.blocks + c.blocks;
#define LLMC_CHAIN(UB, Q)                                                                                    \
  do {                                                                                                        \
    auto kern = gemv_chain_kernel<UB, Q>;                                                                     \
    if (lds > 64 * 1024)                                                                                      \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                160 * 1024);                                                                  \
    kern<<<grid, kChainNT, lds, s>>>(a, b, c, rope, eps, wab, wbc);                                           \
  } while (0)
  if (down_unroll == 8) {
    if (qkv) LLMC_CHAIN(8, true); else LLMC_CHAIN(8, false);
  } else {
    if (qkv) LLMC_CHAIN(4, true); else LLMC_CHAIN(4, false);
  }
#undef LLMC_CHAIN
  return static_cast<int>(hipGetLastError());
}
