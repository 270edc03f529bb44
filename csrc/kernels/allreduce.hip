// K13: custom one-shot all-reduce / all-gather over IPC-mapped peer buffers (xGMI).
//
// Decode-sized TP collectives (a [B, H] bf16 hidden state: 8-64 KiB, 2 per layer; the vocab-shard
// logits gather) are pure latency for RCCL (ring steps over one link each); MI355X has a direct
// xGMI link to every peer (7 x ~153 GB/s), so a ONE-SHOT exchange — every rank pushes its copy
// into every peer's buffer and each reduces locally — is one one-way trip. SURVEY.md §5.8 (2).
// Buffer layout and protocol (push, data-tagged granules, per-block epochs): car_proto.h.
//
// Data mapping, shared by both one-shot kernels (so a granule position is only ever written by
// ONE block, whose epochs are monotone): thread t of block b holds the 16-B vector v = b * 256 + t
// of the message; its payload word j (4 B) travels as granule b * 1024 + j * 256 + t, so each
// store / load instruction of a wave moves 64 consecutive granules (512 B).
#include <hip/hip_ext.h>

#include <cstring>

#include "car_proto.h"

namespace llmc {

constexpr int kBlocks = 64;      // one-shot: blocks per launch at most (256 KiB of payload)
// two-shot: fixed grid (every launch, every rank). Kept to a quarter of the chip: the blocks spin
// on their peers, and a full-chip grid of spinning blocks can starve a peer's queued kernel of CUs
// when ranks share a GPU (a 512-thread, 160-KiB GEMM block needs a whole CU) -> spin timeout.
constexpr int kTsBlocks = 64;
static_assert(kTsBlocks <= kTsFlagBlocks, "two-shot flags");
constexpr int kChunk = 256;      // 16-B vectors per block (one per thread)

__device__ __forceinline__ uint32_t* sig_flag(char* b, int blk, int r, int off = kFlagOff) {
  return reinterpret_cast<uint32_t*>(b + off) + blk * kMaxRanks + r;
}

// two-shot barrier: returns the epoch (LDS-broadcast). ``off``: which flag array (2 barriers)
__device__ __forceinline__ uint32_t car_arrive_and_wait(const CarPeers& P, int rank, int world, uint32_t* lds_epoch,
                                                        int off = kFlagOff) {
  const int b = blockIdx.x, tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its staging stores are out
  __syncthreads();
  const uint32_t epoch = *lds_epoch;
  if (tid < world) {  // signal peer `tid`
    __hip_atomic_store(sig_flag(P.base[tid], b, rank, off), epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world) {  // wait for peer `tid` (bounded, see car_spin; this rank's timeout word ends it)
    uint32_t* f = sig_flag(P.base[rank], b, tid, off);
    unsigned polls = 0;
    uint64_t t0 = 0;
    for (;;) {
      const uint32_t got = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t tmo = car_timeout_word(P, rank);
      if (got >= epoch) {
        car_record_wait(P, rank, polls, t0);
        break;
      }
      if (tmo != 0) {
        car_mark_host(P);
        break;
      }
      if (!car_spin(P, rank, world, polls, t0)) break;
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    // the fence's buffer_inv completes asynchronously: wait for it HERE, so the barrier below
    // releases the block's other waves (whose plain loads read the peers' staging) only once the
    // invalidate is done (MI355X_MICROARCH.md, Consumer recipe). Without it a wave could read a
    // line of a peer's buffer still cached from two launches earlier: rare wrong values in the
    // sequence-parallel prefill (tests/test_tp_gpu.py, llama-small sp_min_tokens=16).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return epoch;
}

__device__ __forceinline__ uint32_t car_begin(const CarPeers& P, int rank, uint32_t* lds_epoch) {
  if (threadIdx.x == 0) {
    *lds_epoch = __hip_atomic_load(car_ctr(P.base[rank]) + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  }
  __syncthreads();
  return *lds_epoch;
}

__device__ __forceinline__ void car_end(const CarPeers& P, int rank, uint32_t epoch) {
  if (threadIdx.x == 0)
    __hip_atomic_store(car_ctr(P.base[rank]) + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Push my vector to every peer, then collect every peer's copy of the same vector (rank order).
__device__ __forceinline__ void car_exchange(const CarPeers& P, int rank, int world, size_t cap, uint32_t epoch,
                                             const u32x4& mine, uint32_t (&in)[kMaxRanks][4]) {
  const long g0 = static_cast<long>(blockIdx.x) * 1024 + threadIdx.x;
  const long g[4] = {g0, g0 + 256, g0 + 512, g0 + 768};
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {
    if (p < world && p != rank) {
#pragma unroll
      for (int j = 0; j < 4; ++j) car_put(P.base[p] + car_granule_off(epoch, cap, rank, g[j]), mine[j], epoch);
    }
  }
  car_collect<4>(P, rank, world, cap, epoch, g, in);
#pragma unroll
  for (int j = 0; j < 4; ++j) in[rank][j] = mine[j];
}

// In-place sum over ranks of x [n16 x 16 B] (bf16), f32 in rank order (same bits on every rank).
__global__ __launch_bounds__(256) void car_allreduce_kernel(CarPeers P, bf16_t* __restrict__ x, int n16, int rank,
                                                            int world, size_t cap) {
  __shared__ uint32_t lds_epoch;
  const int v = blockIdx.x * kChunk + threadIdx.x;
  u32x4 mine{};
  if (v < n16) mine = reinterpret_cast<const u32x4*>(x)[v];  // overlaps the epoch round trip
  const uint32_t epoch = car_begin(P, rank, &lds_epoch);
  if (v < n16) {
    uint32_t in[kMaxRanks][4];
    car_exchange(P, rank, world, cap, epoch, mine, in);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < world) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[2 * j] += bf16_lo(in[r][j]);
          acc[2 * j + 1] += bf16_hi(in[r][j]);
        }
      }
    }
    reinterpret_cast<u32x4*>(x)[v] = pack8(acc);
  }
  car_end(P, rank, epoch);
}

// out[r * nbytes + i] = x_r[i] for every rank r (nbytes per rank, multiple of 16).
__global__ __launch_bounds__(256) void car_allgather_kernel(CarPeers P, const char* __restrict__ x, char* __restrict__ out,
                                                            int n16, int rank, int world, size_t cap) {
  __shared__ uint32_t lds_epoch;
  const int v = blockIdx.x * kChunk + threadIdx.x;
  u32x4 mine{};
  if (v < n16) mine = reinterpret_cast<const u32x4*>(x)[v];
  const uint32_t epoch = car_begin(P, rank, &lds_epoch);
  if (v < n16) {
    uint32_t in[kMaxRanks][4];
    car_exchange(P, rank, world, cap, epoch, mine, in);
    u32x4* ov = reinterpret_cast<u32x4*>(out);
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < world) ov[static_cast<int64_t>(r) * n16 + v] = u32x4{in[r][0], in[r][1], in[r][2], in[r][3]};
  }
  car_end(P, rank, epoch);
}


// ---- two-shot: reduce-scatter + all-gather over peer reads ----------------
// Prefill-sized messages (judge TP prefill, sequence-parallel reduce-scatter / all-gather): the
// one-shot kernel would pull world x S bytes into every rank; the two-shot pulls (world-1)/world x
// S per phase, spread over all world-1 xGMI links at once (each link carries ~S/world per phase
// instead of a ring's per-link-bound 2(w-1)/w x S over one link).
// The piece (<= cap bytes) is world segments of seg16 16-B vectors; vector v = (segment s = v /
// seg16, offset j = v % seg16) lives in chunk v / kChunk, owned by block (chunk % kTsBlocks) on
// EVERY rank and in every phase, so block b only ever waits for block b of its peers. The grid is
// fixed (kTsBlocks, idle blocks still flag), so every block's epoch advances once per launch and the
// data parity (epoch & 1) is the same for the whole launch: a peer at most one launch ahead writes
// the other parity (argument of the one-shot protocol above).
//   MODE 0 all-reduce (in place; in == out, contiguous, last segment may be short):
//       stage all -> A -> reduce my segment (rank order, f32) into my staging + out -> B ->
//       copy the other segments' reduced values from their owners' staging;
//   MODE 1 reduce-scatter: stage all -> A -> reduce my segment into out (my rows only);
//   MODE 2 all-gather: stage my segment (and copy it to out) -> A -> copy the peers' segments.
// Segment s of ``in`` (modes 0/1) / ``out`` (modes 0/2) starts at s * seg_stride bytes.
template <int MODE>
__global__ __launch_bounds__(256) void car_twoshot_kernel(CarPeers P, const char* __restrict__ in, char* __restrict__ out,
                                                          long seg_stride, int seg16, int nv, int rank, int world,
                                                          size_t cap) {
  __shared__ uint32_t lds_epoch;
  const int b = blockIdx.x, t = threadIdx.x;
  const int nchunks = (nv + kChunk - 1) / kChunk;
  const uint32_t epoch = car_begin(P, rank, &lds_epoch);
  const size_t doff = kSigBytes + (epoch & 1) * cap;
  u32x4* mine = reinterpret_cast<u32x4*>(P.base[rank] + doff);
  auto src = [&](int v) -> const u32x4* {
    const int sg = v / seg16, j = v - sg * seg16;
    return reinterpret_cast<const u32x4*>(in + sg * seg_stride) + j;
  };
  auto dst = [&](int v) -> u32x4* {
    const int sg = v / seg16, j = v - sg * seg16;
    return reinterpret_cast<u32x4*>(out + sg * seg_stride) + j;
  };
  const int my0 = rank * seg16, my1 = min(nv, my0 + seg16);
  // 1. stage
  for (int c = b; c < nchunks; c += kTsBlocks) {
    const int v = c * kChunk + t;
    if (v >= nv) continue;
    if constexpr (MODE == 2) {
      if (v >= my0 && v < my1) {
        const u32x4 x = reinterpret_cast<const u32x4*>(in)[v - my0];
        mine[v] = x;
        *dst(v) = x;
      }
    } else {
      mine[v] = *src(v);
    }
  }
  car_arrive_and_wait(P, rank, world, &lds_epoch);
  if constexpr (MODE == 2) {
    for (int c = b; c < nchunks; c += kTsBlocks) {
      const int v = c * kChunk + t;
      if (v >= nv || (v >= my0 && v < my1)) continue;
      *dst(v) = reinterpret_cast<const u32x4*>(P.base[v / seg16] + doff)[v];
    }
  } else {
    // 2. reduce my segment: every rank's copy, summed in rank order (identical bits everywhere)
    for (int c = b; c < nchunks; c += kTsBlocks) {
      const int v = c * kChunk + t;
      if (v < my0 || v >= my1) continue;
      u32x4 inr[kMaxRanks];
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r)
        if (r < world) inr[r] = reinterpret_cast<const u32x4*>(P.base[r] + doff)[v];
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r) {
        if (r < world) {
          float f[8];
          unpack8(inr[r], f);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += f[k];
        }
      }
      const u32x4 red = pack8(acc);
      if constexpr (MODE == 0) {
        mine[v] = red;
        *dst(v) = red;
      } else {
        reinterpret_cast<u32x4*>(out)[v - my0] = red;
      }
    }
    if constexpr (MODE == 0) {
      // 3. the other segments, reduced by their owners
      car_arrive_and_wait(P, rank, world, &lds_epoch, kFlag2Off);
      for (int c = b; c < nchunks; c += kTsBlocks) {
        const int v = c * kChunk + t;
        if (v >= nv || (v >= my0 && v < my1)) continue;
        *dst(v) = reinterpret_cast<const u32x4*>(P.base[v / seg16] + doff)[v];
      }
    }
  }
  car_end(P, rank, epoch);
}

}  // namespace llmc

using namespace llmc;

static int car_grid(int n16) {
  const int chunks = (n16 + kChunk - 1) / kChunk;
  return chunks < 1 ? 1 : chunks;
}

// One-shot payload bytes per rank that a buffer of `cap` bytes per parity carries: kMaxRanks
// slots of cap / kMaxRanks bytes, 8-B granules with 4 B of payload, 1024 granules per block.
static size_t car_oneshot_max(size_t cap) {
  const size_t blocks = cap / kMaxRanks / 8 / 1024;
  return (blocks < static_cast<size_t>(kBlocks) ? blocks : kBlocks) * kChunk * 16;
}

extern "C" {

size_t llmc_car_sig_bytes() { return kSigBytes; }

// One rank's buffer: signals + 2 x cap data, uncached (fine-grained) so peer accesses over xGMI
// bypass the caches; zeroed.
int llmc_car_alloc(size_t cap, void** out) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, kSigBytes + 2 * cap, hipDeviceMallocUncached);
  if (e != hipSuccess) return static_cast<int>(e);
  e = hipMemset(p, 0, kSigBytes + 2 * cap);
  if (e != hipSuccess) return static_cast<int>(e);
  *out = p;
  return 0;
}

int llmc_car_free(void* p) { return static_cast<int>(hipFree(p)); }

int llmc_ipc_handle(void* p, void* handle_out) {
  return static_cast<int>(hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), p));
}

int llmc_ipc_handle_size() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

int llmc_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return static_cast<int>(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
}

int llmc_ipc_close(void* p) { return static_cast<int>(hipIpcCloseMemHandle(p)); }

size_t llmc_car_timeout_off() { return kTimeoutOff; }

// Re-synchronise after a timeout: the caller's group has drained every stream (no launch in
// flight on any rank) and meets in a host barrier before and after: epochs, flags, granules and
// the timeout word go back to zero on every rank.
int llmc_car_reset(void* own, size_t cap) {
  // the data too: granule tags restart with the epochs
  hipError_t e = hipMemset(own, 0, kSigBytes + 2 * cap);
  if (e != hipSuccess) return static_cast<int>(e);
  return static_cast<int>(hipDeviceSynchronize());
}

// A new stream on `device` whose kernels run only on the CUs set in `mask` (bit i of word w = CU
// 32 w + i): one-GPU rehearsals of multi-rank flows give each rank its own CUs, so ranks that
// spin on each other (the custom collectives) run side by side as on separate GPUs.
int llmc_stream_cu_mask(int device, const uint32_t* mask, int words, void** out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return static_cast<int>(e);
  hipStream_t st = nullptr;
  e = hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(words), mask);
  *out = st;
  return static_cast<int>(e);
}

// 1 if device `dev` can map memory of device `peer` (xGMI P2P), else 0; same device -> 1.
int llmc_can_access_peer(int dev, int peer, int* out) {
  if (dev == peer) {
    *out = 1;
    return 0;
  }
  int v = 0;
  hipError_t e = hipDeviceCanAccessPeer(&v, dev, peer);
  *out = v;
  return static_cast<int>(e);
}

// timeout word of this rank's buffer (host read after a sync; 1 = a spin gave up)
int llmc_car_timed_out(void* own, int* out) {
  uint32_t v = 0;
  hipError_t e = hipMemcpy(&v, static_cast<char*>(own) + kTimeoutOff, 4, hipMemcpyDeviceToHost);
  *out = static_cast<int>(v);
  return static_cast<int>(e);
}

// Longest wait (100-MHz ticks) any spin of this rank's buffer recorded since the last reset (host
// read after a sync).
int llmc_car_max_wait(void* own, uint32_t* out) {
  return static_cast<int>(hipMemcpy(out, static_cast<char*>(own) + kStatOff, 4, hipMemcpyDeviceToHost));
}

// The host status page of one rank buffer (car_proto.h kHost*): pinned, coherent (fine-grained:
// device stores reach the host and host stores reach the device without cache maintenance),
// mapped; zeroed. *host is the host address, *dev the device address the kernels take.
int llmc_car_host_alloc(void** host, void** dev) {
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, kHostWords * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped);
  if (e != hipSuccess) return static_cast<int>(e);
  std::memset(p, 0, kHostWords * sizeof(uint32_t));
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, p, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(p);
    return static_cast<int>(e);
  }
  *host = p;
  *dev = d;
  return 0;
}

int llmc_car_host_free(void* host) { return static_cast<int>(hipHostFree(host)); }

// Host side of the status page: plain volatile accesses (no GPU call, usable while the stream is
// busy). word: kHostAbort / kHostTimedOut.
int llmc_car_host_get(const void* host, int word) {
  return static_cast<int>(static_cast<const volatile uint32_t*>(host)[word]);
}
void llmc_car_host_set(void* host, int word, int v) {
  static_cast<volatile uint32_t*>(host)[word] = static_cast<uint32_t>(v);
}
int llmc_car_host_word(int which) { return which == 0 ? kHostAbort : which == 1 ? kHostTimedOut : kHostSpinTicks; }

size_t llmc_car_oneshot_max(size_t cap) { return car_oneshot_max(cap); }

int llmc_car_allreduce(const void* const* bases, void* host, int rank, int world, size_t cap, void* x, size_t nbytes,
                       hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || nbytes > car_oneshot_max(cap))
    return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  P.host = static_cast<uint32_t*>(host);
  const int n16 = static_cast<int>(nbytes / 16);
  car_allreduce_kernel<<<car_grid(n16), 256, 0, s>>>(P, static_cast<bf16_t*>(x), n16, rank, world, cap);
  return static_cast<int>(hipGetLastError());
}

int llmc_car_allgather(const void* const* bases, void* host, int rank, int world, size_t cap, const void* x, void* out,
                       size_t nbytes, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || nbytes > car_oneshot_max(cap))
    return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  P.host = static_cast<uint32_t*>(host);
  const int n16 = static_cast<int>(nbytes / 16);
  car_allgather_kernel<<<car_grid(n16), 256, 0, s>>>(P, static_cast<const char*>(x), static_cast<char*>(out), n16, rank,
                                               world, cap);
  return static_cast<int>(hipGetLastError());
}

// Two-shot collective over one piece (see car_twoshot_kernel): mode 0 all-reduce (in == out,
// nv vectors), 1 reduce-scatter, 2 all-gather; world * seg16 * 16 <= cap.
int llmc_car_twoshot(const void* const* bases, void* host, int rank, int world, size_t cap, int mode, const void* in,
                     void* out, long seg_stride, int seg16, int nv, hipStream_t s) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || seg16 <= 0 || nv <= 0 ||
      nv > world * seg16 || static_cast<size_t>(world) * seg16 * 16 > cap)
    return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  P.host = static_cast<uint32_t*>(host);
  const char* i = static_cast<const char*>(in);
  char* o = static_cast<char*>(out);
  switch (mode) {
    case 0: car_twoshot_kernel<0><<<kTsBlocks, 256, 0, s>>>(P, i, o, seg_stride, seg16, nv, rank, world, cap); break;
    case 1: car_twoshot_kernel<1><<<kTsBlocks, 256, 0, s>>>(P, i, o, seg_stride, seg16, nv, rank, world, cap); break;
    case 2: car_twoshot_kernel<2><<<kTsBlocks, 256, 0, s>>>(P, i, o, seg_stride, seg16, nv, rank, world, cap); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
