// Native chat tokenizer (see tokenizer.h).
#include "tokenizer.h"

#include <stdexcept>

namespace drtc {
namespace {

enum : uint8_t { kOther = 0, kWord = 1, kSpace = 2 };

struct CharClass {
  uint8_t c[256];
  CharClass() {
    for (int i = 0; i < 256; ++i) c[i] = kOther;
    for (int i = 'a'; i <= 'z'; ++i) c[i] = kWord;
    for (int i = 'A'; i <= 'Z'; ++i) c[i] = kWord;
    for (int i = '0'; i <= '9'; ++i) c[i] = kWord;
    c[(int)'_'] = kWord;
    c[(int)'\''] = kWord;
    for (int i : {9, 10, 11, 12, 13, 28, 29, 30, 31, 32}) c[i] = kSpace;
  }
};
const CharClass kClass;

inline uint8_t cls(char ch) { return kClass.c[(uint8_t)ch]; }

}  // namespace

WordTokenizer::WordTokenizer(std::vector<std::string> vocab, int32_t byte_base, int32_t bos_id,
                             std::vector<int32_t> skip_ids)
    : vocab_(std::move(vocab)), byte_base_(byte_base), bos_id_(bos_id) {
  if (byte_base_ < 0 || byte_base_ + 256 > (int32_t)vocab_.size())
    throw std::invalid_argument("byte tokens out of the vocabulary");
  ids_.reserve(vocab_.size() * 2);
  for (int32_t i = 0; i < (int32_t)vocab_.size(); ++i) {
    if (i >= byte_base_ && i < byte_base_ + 256) continue;  // "<0xNN>" names: not text pieces
    ids_.emplace(std::string_view(vocab_[i]), i);           // first id of a string wins
  }
  space_id_ = lookup(" ");
  skip_.assign(vocab_.size(), 0);
  for (int32_t s : skip_ids)
    if (s >= 0 && s < (int32_t)vocab_.size()) skip_[s] = 1;
}

int32_t WordTokenizer::lookup(std::string_view piece) const {
  auto it = ids_.find(piece);
  return it == ids_.end() ? -1 : it->second;
}

std::vector<int32_t> WordTokenizer::encode(std::string_view text, bool add_bos) const {
  std::vector<int32_t> out;
  out.reserve(text.size() / 3 + 2);
  if (add_bos) out.push_back(bos_id_);
  const size_t n = text.size();
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    const bool sp = text[i] == ' ';
    const uint8_t next = sp && i + 1 < n ? cls(text[i + 1]) : kSpace;
    if (cls(text[i]) == kWord || (sp && next == kWord)) {
      j = sp ? i + 1 : i;
      while (j < n && cls(text[j]) == kWord) ++j;
    } else if (cls(text[i]) == kOther || (sp && next == kOther)) {
      j = sp ? i + 1 : i;
      while (j < n && cls(text[j]) == kOther) ++j;
    } else {  // whitespace run
      while (j < n && cls(text[j]) == kSpace) ++j;
    }
    const std::string_view piece = text.substr(i, j - i);
    int32_t t = lookup(piece);
    if (t >= 0) {
      out.push_back(t);
    } else if (piece.size() > 1 && piece[0] == ' ' && space_id_ >= 0 &&
               (t = lookup(piece.substr(1))) >= 0) {
      out.push_back(space_id_);
      out.push_back(t);
    } else {
      for (char ch : piece) out.push_back(byte_base_ + (uint8_t)ch);
    }
    i = j;
  }
  return out;
}

std::string WordTokenizer::decode(const std::vector<int64_t>& ids, bool skip_special) const {
  std::string out;
  out.reserve(ids.size() * 6);
  const int64_t nv = (int64_t)vocab_.size();
  for (int64_t i : ids) {
    if (i >= byte_base_ && i < byte_base_ + 256) {
      out.push_back((char)(i - byte_base_));
    } else if (i >= 0 && i < nv) {
      if (skip_[i] && skip_special) continue;
      out += vocab_[i];
    }
  }
  return out;
}

}  // namespace drtc
