// K13: custom one-shot all-reduce / all-gather over IPC-mapped peer buffers (xGMI).
//
// Decode-sized TP collectives (a [B, H] bf16 hidden state: 8-64 KiB, 2 per layer) are pure
// latency for RCCL (ring steps over one link each); MI355X has a direct xGMI link to every peer
// (7 x ~153 GB/s), so a ONE-SHOT exchange — every rank reads every peer's copy directly and
// reduces locally — is one link round trip. SURVEY.md §5.8 (2).
//
// Buffers: each rank owns ONE uncached (fine-grained) allocation, exported with hipIpc and
// mapped by every peer:   [ signals 64 KiB | data parity 0 (cap) | data parity 1 (cap) ]
//   signals: ctr[kBlocks] (per-block launch epoch, persists across graph replays),
//            flag[kMaxBlocks][kMaxRanks] (epoch of the last arrival of rank r for block b),
//            timeout word (set when a bounded spin gives up).
// Block b always owns the same 4 KiB chunks (c % kBlocks == b) whatever the message size, so
// block b's epochs and data slices line up across ranks and across calls of different sizes. A
// launch runs only the blocks that own data (min(kBlocks, chunks)): every rank issues the same
// sequence of sizes, so an idle block's epoch simply stays put on every rank, and a decode-sized
// [1, 4096] bf16 message costs 2 blocks' flag exchanges over xGMI instead of 32. Protocol per
// launch, per block b:
//   1. epoch = ctr[b] + 1; stage my slice into my data[epoch & 1] (uncached stores);
//   2. every wave drains its stores (s_waitcnt vmcnt(0)), barrier, then ONE lane per peer
//      stores `epoch` into peer.flag[b][me] (system-scope release);
//   3. one lane per peer polls my flag[b][peer] >= epoch (relaxed, s_sleep, BOUNDED), then one
//      system-scope acquire;
//   4. read every rank's slice from data[epoch & 1] (fixed rank order -> bitwise-identical
//      results on every rank), sum in f32, write the local output;
//   5. ctr[b] = epoch.
// Double-buffered data (by epoch parity) + monotone ">= epoch" flags make a second barrier
// unnecessary: a peer can be at most one launch ahead (it cannot pass launch k+1's step 3 before
// I signal k+1), so it writes the other parity while I still read this one.
// The whole launch is graph-capturable: peers and sizes are fixed, epochs live in device memory.
#include <cstring>

#include "common.h"

namespace llmc {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;  // signal slots (two-shot launches use all of them)
constexpr int kBlocks = 32;      // one-shot: blocks per launch (at most; see car_grid)
// two-shot: fixed grid (every launch, every rank). Kept to a quarter of the chip: the blocks spin
// on their peers, and a full-chip grid of spinning blocks can starve a peer's queued kernel of CUs
// when ranks share a GPU (a 512-thread, 160-KiB GEMM block needs a whole CU) -> spin timeout.
constexpr int kTsBlocks = 64;
constexpr int kChunk = 256;      // 16-B vectors per chunk (one per thread)
constexpr size_t kSigBytes = 64 * 1024;
constexpr int kFlagOff = 1024;                              // bytes: after ctr[kMaxBlocks]
constexpr int kFlag2Off = kFlagOff + kMaxBlocks * kMaxRanks * 4;  // two-shot's second barrier
constexpr int kTimeoutOff = kFlag2Off + kMaxBlocks * kMaxRanks * 4;
static_assert(kTimeoutOff + 4 <= static_cast<int>(kSigBytes), "signal layout");

struct CarPeers {
  char* base[kMaxRanks];  // each rank's buffer (own one included), mapped in this process
};

__device__ __forceinline__ uint32_t* sig_ctr(char* b) { return reinterpret_cast<uint32_t*>(b); }
__device__ __forceinline__ uint32_t* sig_flag(char* b, int blk, int r, int off = kFlagOff) {
  return reinterpret_cast<uint32_t*>(b + off) + blk * kMaxRanks + r;
}

// steps 1-3: returns the epoch (LDS-broadcast). ``off``: which flag array (two-shot: 2 barriers)
__device__ __forceinline__ uint32_t car_arrive_and_wait(const CarPeers& P, int rank, int world, uint32_t* lds_epoch,
                                                        int off = kFlagOff) {
  const int b = blockIdx.x, tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its staging stores are out
  __syncthreads();
  const uint32_t epoch = *lds_epoch;
  if (tid < world) {  // signal peer `tid`
    __hip_atomic_store(sig_flag(P.base[tid], b, rank, off), epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world) {  // wait for peer `tid`
    uint32_t* f = sig_flag(P.base[rank], b, tid, off);
    unsigned spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {  // ~seconds: give up instead of hanging the GPU
        __hip_atomic_store(reinterpret_cast<uint32_t*>(P.base[rank] + kTimeoutOff), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  return epoch;
}

__device__ __forceinline__ uint32_t car_begin(const CarPeers& P, int rank, uint32_t* lds_epoch) {
  if (threadIdx.x == 0) {
    *lds_epoch = __hip_atomic_load(sig_ctr(P.base[rank]) + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  }
  __syncthreads();
  return *lds_epoch;
}

__device__ __forceinline__ void car_end(const CarPeers& P, int rank, uint32_t epoch) {
  if (threadIdx.x == 0)
    __hip_atomic_store(sig_ctr(P.base[rank]) + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// In-place sum over ranks of x [n16 x 16 B] (bf16).
__global__ __launch_bounds__(256) void car_allreduce_kernel(CarPeers P, bf16_t* __restrict__ x, int n16, int rank,
                                                            int world, size_t cap) {
  __shared__ uint32_t lds_epoch;
  const int v0 = blockIdx.x * kChunk + threadIdx.x, vstep = kBlocks * kChunk;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  // this thread's first vector is loaded before the epoch: the two memory round trips overlap
  // (a decode-sized message is one vector per thread)
  u32x4 first{};
  if (v0 < n16) first = xv[v0];
  const uint32_t epoch = car_begin(P, rank, &lds_epoch);
  const size_t doff = kSigBytes + (epoch & 1) * cap;
  u32x4* mine = reinterpret_cast<u32x4*>(P.base[rank] + doff);
  if (v0 < n16) mine[v0] = first;
  for (int v = v0 + vstep; v < n16; v += vstep) mine[v] = xv[v];
  car_arrive_and_wait(P, rank, world, &lds_epoch);
  for (int v = v0; v < n16; v += vstep) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    u32x4 in[kMaxRanks];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)  // all peer loads in flight before the sums
      if (r < world) in[r] = reinterpret_cast<const u32x4*>(P.base[r] + doff)[v];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < world) {
        float f[8];
        unpack8(in[r], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
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
  const int v0 = blockIdx.x * kChunk + threadIdx.x, vstep = kBlocks * kChunk;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x4 first{};
  if (v0 < n16) first = xv[v0];  // overlaps the epoch load (see car_allreduce_kernel)
  const uint32_t epoch = car_begin(P, rank, &lds_epoch);
  const size_t doff = kSigBytes + (epoch & 1) * cap;
  u32x4* mine = reinterpret_cast<u32x4*>(P.base[rank] + doff);
  if (v0 < n16) mine[v0] = first;
  for (int v = v0 + vstep; v < n16; v += vstep) mine[v] = xv[v];
  car_arrive_and_wait(P, rank, world, &lds_epoch);
  u32x4* ov = reinterpret_cast<u32x4*>(out);
  for (int v = v0; v < n16; v += vstep) {
    u32x4 in[kMaxRanks];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < world) in[r] = reinterpret_cast<const u32x4*>(P.base[r] + doff)[v];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < world) ov[static_cast<int64_t>(r) * n16 + v] = in[r];
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
  return chunks < 1 ? 1 : (chunks < kBlocks ? chunks : kBlocks);
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
// flight on any rank) and meets in a host barrier before and after: epochs, flags and the
// timeout word go back to zero on every rank.
int llmc_car_reset(void* own) {
  hipError_t e = hipMemset(own, 0, kSigBytes);
  if (e != hipSuccess) return static_cast<int>(e);
  return static_cast<int>(hipDeviceSynchronize());
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

int llmc_car_allreduce(const void* const* bases, int rank, int world, size_t cap, void* x, size_t nbytes,
                       hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || nbytes > cap) return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  const int n16 = static_cast<int>(nbytes / 16);
  car_allreduce_kernel<<<car_grid(n16), 256, 0, s>>>(P, static_cast<bf16_t*>(x), n16, rank, world, cap);
  return static_cast<int>(hipGetLastError());
}

int llmc_car_allgather(const void* const* bases, int rank, int world, size_t cap, const void* x, void* out,
                       size_t nbytes, hipStream_t s) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || nbytes > cap) return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  const int n16 = static_cast<int>(nbytes / 16);
  car_allgather_kernel<<<car_grid(n16), 256, 0, s>>>(P, static_cast<const char*>(x), static_cast<char*>(out), n16, rank,
                                               world, cap);
  return static_cast<int>(hipGetLastError());
}

// Two-shot collective over one piece (see car_twoshot_kernel): mode 0 all-reduce (in == out,
// nv vectors), 1 reduce-scatter, 2 all-gather; world * seg16 * 16 <= cap.
int llmc_car_twoshot(const void* const* bases, int rank, int world, size_t cap, int mode, const void* in, void* out,
                     long seg_stride, int seg16, int nv, hipStream_t s) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || seg16 <= 0 || nv <= 0 ||
      nv > world * seg16 || static_cast<size_t>(world) * seg16 * 16 > cap)
    return -1;
  CarPeers P;
  for (int r = 0; r < kMaxRanks; ++r) P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
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
