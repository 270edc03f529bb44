#include "tokenizer.h"

#include <stdexcept>

namespace llmc {

static const char kAlphabet[] =
    "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
static constexpr int kSyms = 62;
static constexpr int kBytes = 256;
static constexpr int kSpecial = 2;

SyntheticTokenizer::SyntheticTokenizer(int64_t vocab_size) : vocab_(vocab_size) {
  if (vocab_size < kBytes + kSpecial + 1) throw std::invalid_argument("vocab too small");
  int64_t max_pieces = static_cast<int64_t>(kSyms) * kSyms * kSyms;
  n_pieces_ = vocab_size - kBytes - kSpecial;
  if (n_pieces_ > max_pieces) n_pieces_ = max_pieces;
  for (int i = 0; i < 256; ++i) sym_index_[i] = -1;
  for (int i = 0; i < kSyms; ++i) sym_index_[static_cast<unsigned char>(kAlphabet[i])] = static_cast<int8_t>(i);
}

std::vector<int32_t> SyntheticTokenizer::encode(const std::string& text) const {
  std::vector<int32_t> out;
  out.reserve(text.size() / 4 + 8);
  const unsigned char* s = reinterpret_cast<const unsigned char*>(text.data());
  const size_t n = text.size();
  size_t i = 0;
  while (i < n) {
    if (s[i] == ' ' && i + 3 < n) {
      const int a = sym_index_[s[i + 1]], b = sym_index_[s[i + 2]], c = sym_index_[s[i + 3]];
      if (a >= 0 && b >= 0 && c >= 0) {
        const int64_t p = (static_cast<int64_t>(a) * kSyms + b) * kSyms + c;
        if (p < n_pieces_) {
          out.push_back(static_cast<int32_t>(kBytes + p));
          i += 4;
          continue;
        }
      }
    }
    out.push_back(static_cast<int32_t>(s[i]));
    ++i;
  }
  return out;
}

std::string SyntheticTokenizer::piece(int32_t id) const {
  if (id < 0 || id >= vocab_) return std::string();
  if (id < kBytes) return std::string(1, static_cast<char>(id));
  const int64_t p = static_cast<int64_t>(id) - kBytes;
  if (p >= n_pieces_) return std::string();  // specials and unused ids decode to ""
  char buf[4] = {' ', kAlphabet[(p / (kSyms * kSyms)) % kSyms], kAlphabet[(p / kSyms) % kSyms],
                 kAlphabet[p % kSyms]};
  return std::string(buf, 4);
}

std::string SyntheticTokenizer::decode(const int32_t* ids, int64_t n) const {
  std::string out;
  out.reserve(static_cast<size_t>(n) * 4);
  for (int64_t i = 0; i < n; ++i) out += piece(ids[i]);
  return out;
}

}  // namespace llmc
