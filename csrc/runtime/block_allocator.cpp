#include "block_allocator.h"

#include <stdexcept>
#include <string>

namespace llmc {

BlockAllocator::BlockAllocator(int64_t num_blocks, int64_t block_size)
    : num_blocks_(num_blocks), block_size_(block_size), refs_(static_cast<size_t>(num_blocks), 0) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad allocator geometry");
  free_list_.reserve(static_cast<size_t>(num_blocks));
  // Hand out low ids first (stack pops from the back).
  for (int64_t b = num_blocks - 1; b >= 0; --b) free_list_.push_back(static_cast<int32_t>(b));
}

std::vector<int32_t> BlockAllocator::allocate(int64_t n) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int32_t> out;
  if (n < 0 || static_cast<size_t>(n) > free_list_.size()) return out;
  out.reserve(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    int32_t b = free_list_.back();
    free_list_.pop_back();
    refs_[static_cast<size_t>(b)] = 1;
    out.push_back(b);
  }
  return out;
}

void BlockAllocator::free(const std::vector<int32_t>& blocks) {
  std::lock_guard<std::mutex> g(mu_);
  for (int32_t b : blocks) {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id " + std::to_string(b));
    int32_t& r = refs_[static_cast<size_t>(b)];
    if (r <= 0) throw std::logic_error("double free of block " + std::to_string(b));
    if (--r == 0) free_list_.push_back(b);
  }
}

void BlockAllocator::incref(const std::vector<int32_t>& blocks) {
  std::lock_guard<std::mutex> g(mu_);
  for (int32_t b : blocks) {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id " + std::to_string(b));
    if (refs_[static_cast<size_t>(b)] <= 0) throw std::logic_error("incref of free block");
    ++refs_[static_cast<size_t>(b)];
  }
}

int64_t BlockAllocator::num_free() const {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int64_t>(free_list_.size());
}

int32_t BlockAllocator::refcount(int32_t block) const {
  std::lock_guard<std::mutex> g(mu_);
  if (block < 0 || block >= num_blocks_) throw std::out_of_range("block id");
  return refs_[static_cast<size_t>(block)];
}

}  // namespace llmc
