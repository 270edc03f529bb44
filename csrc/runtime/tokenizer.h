// Synthetic, segment-stable tokenizer.
//
// There is no network and weights are random, so a real BPE vocabulary buys nothing. This
// tokenizer maps every id to a printable piece so that (a) the reference UI's chars/4 token
// estimate (internal/ui/ui.go:142) stays meaningful, (b) decoded text is valid UTF-8 for the
// Go-compatible JSON encoder, and (c) encode() is segment-stable at the judge-template block
// boundaries (internal/consensus/judge.go:20-25), which lets the judge prefill incrementally.
//
// Vocabulary of size V:
//   [0, 256)            byte tokens (raw bytes; used for any text that is not a piece)
//   [256, V - 2)        pieces: " " + 3 chars of a 62-symbol alphabet (base-62 index)
//   V - 2, V - 1        BOS, EOS (decode to "")
// A piece can only start at a space followed by three alphanumerics, so no piece can span a
// '\n' boundary: encode(a + b) == encode(a) + encode(b) whenever a ends with '\n'.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace llmc {

class SyntheticTokenizer {
 public:
  explicit SyntheticTokenizer(int64_t vocab_size);
  std::vector<int32_t> encode(const std::string& text) const;
  // Raw bytes (may be invalid UTF-8 when byte tokens split a sequence).
  std::string decode(const int32_t* ids, int64_t n) const;
  std::string piece(int32_t id) const;
  int64_t vocab_size() const { return vocab_; }
  int32_t bos_id() const { return static_cast<int32_t>(vocab_ - 2); }
  int32_t eos_id() const { return static_cast<int32_t>(vocab_ - 1); }
  int64_t num_pieces() const { return n_pieces_; }

 private:
  int64_t vocab_;
  int64_t n_pieces_;
  int8_t sym_index_[256];
};

}  // namespace llmc
