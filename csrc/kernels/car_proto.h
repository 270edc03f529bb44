// K13 custom-collective protocol shared by the standalone one-shot kernels (allreduce.hip) and the
// row-parallel GEMV's fused all-reduce epilogue (gemv_core.h, EPI_AR).
//
// Each rank owns ONE uncached (fine-grained) allocation, exported with hipIpc and mapped by every
// peer:   [ signals kSigBytes | data parity 0 (cap) | data parity 1 (cap) ]
//   signals: ctr[kMaxBlocks]   per-block launch epoch (persists across graph replays),
//            two-shot flags    (allreduce.hip, car_twoshot_kernel),
//            timeout word      (set when a bounded spin gives up).
//   data parity p: kMaxRanks slots of cap / kMaxRanks bytes; slot r receives rank r's pushes.
//
// One-shot protocol (push, data-tagged granules; MI355X_MICROARCH.md "handoff-1to1": the price of
// a hand-off is in the consumer's queue, and a granule that carries its own tag needs no flag):
//   1. epoch = ctr[b] + 1 (block b owns the same data on every rank and every launch);
//   2. every rank STORES its contribution straight into every peer's slot [parity][rank] as 8-byte
//      granules {4-B payload, 4-B tag = epoch}, one 64-bit atomic store each (single-copy atomic
//      by the memory model, also across xGMI), fire and forget: no fence, no flag, no drain;
//   3. it polls its OWN buffer (local memory) until every peer's granules carry this epoch
//      (bounded spin), and combines them in rank order (bitwise-identical results on all ranks);
//   4. ctr[b] = epoch.
// A peer can be at most one participation of block b ahead (it cannot finish its launch k+1
// before my launch-(k+1) pushes, which follow my launch k), so it writes the other parity while I
// still read this one; tags never repeat (epochs only grow; a resync zeroes the whole buffer).
// Against the pull protocol it replaces (stage locally, release-flag each peer, poll, acquire,
// read the peers' copies over xGMI) this is one one-way trip instead of a flag trip plus a remote
// read round trip, and no system-scope fences.
#pragma once
#include "common.h"

namespace llmc {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 1024;     // epoch counters: blocks of any one-shot / EPI_AR launch
constexpr int kTsFlagBlocks = 256;   // two-shot flag slots (its grid is kTsBlocks <= this)
constexpr size_t kSigBytes = 128 * 1024;
constexpr int kFlagOff = 4 * kMaxBlocks;                              // bytes: after ctr[kMaxBlocks]
constexpr int kFlag2Off = kFlagOff + kTsFlagBlocks * kMaxRanks * 4;   // two-shot's second barrier
constexpr int kTimeoutOff = kFlag2Off + kTsFlagBlocks * kMaxRanks * 4;
constexpr int kStatOff = kTimeoutOff + 128;  // u32: longest wait seen by a spin of this rank (ticks)
static_assert(kStatOff + 4 <= static_cast<int>(kSigBytes), "signal layout");
// Bounded waits: a spin gives up after kCarSpinTicks of the 100-MHz constant clock (s_memrealtime),
// i.e. 1 s whatever the poll latency (local uncached load, xGMI, contention). Every kCarCheckPolls
// polls it also reads the host abort word. A peer that is merely slow never waits this long in a
// decode (the ranks are in lockstep through their collectives; host skew is milliseconds).
constexpr uint64_t kCarSpinTicks = 100ull * 1000 * 1000;
constexpr unsigned kCarCheckPolls = 64;
// Host status page (pinned, coherent, mapped into the device; one per rank buffer), u32 words:
//   [kHostAbort]    the host sets it (a replay overran its deadline): every spin gives up at its
//                   next check instead of polling to the limit;
//   [kHostTimedOut] a spin of this rank gave up or returned without its data: the host reads it
//                   with a plain load, no GPU call (the stream may still be busy).
//   [kHostSpinTicks] the spin bound in ticks when non-zero (LLMC_CAR_SPIN_S, <= 21 s: ranks
//                    time-sharing one GPU without CU partitions can be starved past kCarSpinTicks)
constexpr int kHostAbort = 0, kHostTimedOut = 16, kHostSpinTicks = 32, kHostWords = 64;
// fused-all-reduce buffer (gemv_core.h EPI_AR): block b of a launch owns granules [16 b, 16 b + 16)
// of every slot and epoch ctr[b]
constexpr int kArGranulesPerBlock = 16;

struct CarPeers {
  char* base[kMaxRanks];  // each rank's buffer (own one included), mapped in this process
  uint32_t* host;         // this rank's host status page (device pointer), or nullptr
};

// What a fused epilogue needs besides the buffers: who I am and the data parity size.
struct CarArgs {
  CarPeers P;
  int rank, world;
  long cap;  // bytes per data parity
};

__device__ __forceinline__ uint32_t* car_ctr(char* b) { return reinterpret_cast<uint32_t*>(b); }

// Byte offset of granule g of slot r in parity (epoch & 1).
__device__ __forceinline__ size_t car_granule_off(uint32_t epoch, size_t cap, int r, long g) {
  return kSigBytes + (epoch & 1) * cap + static_cast<size_t>(r) * (cap / kMaxRanks) + static_cast<size_t>(g) * 8;
}

__device__ __forceinline__ void car_put(char* p, uint32_t payload, uint32_t tag) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (static_cast<uint64_t>(tag) << 32) | payload, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t car_get(const char* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t car_timeout_word(const CarPeers& P, int rank) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(P.base[rank] + kTimeoutOff), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// This rank's collective results since the last resync are invalid: tell the host (its page).
__device__ __forceinline__ void car_mark_host(const CarPeers& P) {
  if (P.host != nullptr)
    __hip_atomic_store(P.host + kHostTimedOut, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A spin gave up: set the timeout word of EVERY rank's buffer (mine: every later spin of this rank
// returns at once; the peers': their spins on this exchange and the later ones end too, so a stalled
// exchange fails on every rank within one check instead of each rank polling to its own limit) and
// mark the host page.
__device__ __forceinline__ void car_give_up(const CarPeers& P, int rank, int world) {
  for (int r = 0; r < world && r < kMaxRanks; ++r)
    __hip_atomic_store(reinterpret_cast<uint32_t*>(P.base[r] + kTimeoutOff), 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  car_mark_host(P);
  (void)rank;
}

// Slow-path bookkeeping after a failed poll (`polls` failed polls so far, `t0` the clock at the
// first): sleeps and returns true to poll again, or gives up (deadline passed or the host set its
// abort word) and returns false.
__device__ __forceinline__ bool car_spin(const CarPeers& P, int rank, int world, unsigned& polls, uint64_t& t0) {
  if (polls == 0) t0 = __builtin_amdgcn_s_memrealtime();
  ++polls;
  if (polls % kCarCheckPolls == 0) {
    uint64_t bound = kCarSpinTicks;
    bool stop = false;
    if (P.host != nullptr) {
      const uint32_t b = __hip_atomic_load(P.host + kHostSpinTicks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (b != 0) bound = b;
      stop = __hip_atomic_load(P.host + kHostAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    }
    stop = stop || __builtin_amdgcn_s_memrealtime() - t0 > bound;
    if (stop) {
      car_give_up(P, rank, world);
      return false;
    }
  }
  __builtin_amdgcn_s_sleep(2);
  return true;
}

// A wait that ended with its data after `polls` failed polls: lane 0 records its length (ticks) in
// this rank's longest-wait word (bench.py reports it per collective buffer).
__device__ __forceinline__ void car_record_wait(const CarPeers& P, int rank, unsigned polls, uint64_t t0) {
  if (polls != 0 && (threadIdx.x % kWave) == 0) {
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
    __hip_atomic_fetch_max(reinterpret_cast<uint32_t*>(P.base[rank] + kStatOff),
                           static_cast<uint32_t>(dt > 0xffffffffull ? 0xffffffffull : dt), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wait until granules g[0..NG) of every peer's slot (not mine) carry `epoch`; payloads out in
// v[r][i] (v[rank][*] untouched). Every load in flight at once, re-polled together, with this
// rank's timeout word in the same batch: once any spin of the group has given up, the wait returns
// at once (the results are invalid and the host is told). Bounded: car_spin.
template <int NG>
__device__ __forceinline__ void car_collect(const CarPeers& P, int rank, int world, size_t cap, uint32_t epoch,
                                            const long (&g)[NG], uint32_t (&v)[kMaxRanks][NG]) {
  const char* own = P.base[rank];
  unsigned polls = 0;
  uint64_t t0 = 0;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < world && r != rank) {
#pragma unroll
        for (int i = 0; i < NG; ++i) {
          const uint64_t x = car_get(own + car_granule_off(epoch, cap, r, g[i]));
          v[r][i] = static_cast<uint32_t>(x);
          ok = ok && static_cast<uint32_t>(x >> 32) == epoch;
        }
      }
    }
    const uint32_t tmo = car_timeout_word(P, rank);
    if (ok) {
      car_record_wait(P, rank, polls, t0);
      return;
    }
    if (tmo != 0) {
      car_mark_host(P);
      return;
    }
    if (!car_spin(P, rank, world, polls, t0)) return;
  }
}

}  // namespace llmc
