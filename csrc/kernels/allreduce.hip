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
constexpr int kMaxBlocks = 64;  // signal slots
constexpr int kBlocks = 32;     // blocks per launch (at most; see car_grid)
constexpr int kChunk = 256;     // 16-B vectors per chunk (one per thread)
constexpr size_t kSigBytes = 64 * 1024;
constexpr int kFlagOff = 1024;                             // bytes: after ctr[]
constexpr int kTimeoutOff = kFlagOff + kMaxBlocks * kMaxRanks * 4;

struct CarPeers {
  char* base[kMaxRanks];  // each rank's buffer (own one included), mapped in this process
};

__device__ __forceinline__ uint32_t* sig_ctr(char* b) { return reinterpret_cast<uint32_t*>(b); }
__device__ __forceinline__ uint32_t* sig_flag(char* b, int blk, int r) {
  return reinterpret_cast<uint32_t*>(b + kFlagOff) + blk * kMaxRanks + r;
}

// steps 1-3: returns the epoch (LDS-broadcast)
__device__ __forceinline__ uint32_t car_arrive_and_wait(const CarPeers& P, int rank, int world, uint32_t* lds_epoch) {
  const int b = blockIdx.x, tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its staging stores are out
  __syncthreads();
  const uint32_t epoch = *lds_epoch;
  if (tid < world) {  // signal peer `tid`
    __hip_atomic_store(sig_flag(P.base[tid], b, rank), epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < world) {  // wait for peer `tid`
    uint32_t* f = sig_flag(P.base[rank], b, tid);
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

}  // extern "C"
