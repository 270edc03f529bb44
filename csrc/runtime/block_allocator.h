// Paged-KV block allocator (SURVEY.md §2.6 "Runtime components").
//
// One allocator per engine KV pool. Blocks are ref-counted so a prefix (e.g. the judge's
// template header) can be shared between sequences; allocation is all-or-nothing so an OOM
// surfaces as one engine-level error instead of a half-built block table.
// Host-only and O(1) per block: it runs between decode steps, never inside a HIP graph (the
// decode graph reads block tables that were filled before capture/replay).
#pragma once
#include <cstdint>
#include <mutex>
#include <vector>

namespace llmc {

class BlockAllocator {
 public:
  BlockAllocator(int64_t num_blocks, int64_t block_size);
  // Returns block ids, or an empty vector when fewer than n blocks are free.
  std::vector<int32_t> allocate(int64_t n);
  void free(const std::vector<int32_t>& blocks);
  void incref(const std::vector<int32_t>& blocks);
  int64_t num_free() const;
  int64_t num_blocks() const { return num_blocks_; }
  int64_t block_size() const { return block_size_; }
  int32_t refcount(int32_t block) const;
  // Blocks needed to hold `tokens` tokens.
  int64_t blocks_for(int64_t tokens) const { return (tokens + block_size_ - 1) / block_size_; }

 private:
  int64_t num_blocks_;
  int64_t block_size_;
  std::vector<int32_t> free_list_;
  std::vector<int32_t> refs_;
  mutable std::mutex mu_;
};

}  // namespace llmc
