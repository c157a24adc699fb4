// Word-level chat tokenizer, native form of engine/tokenizer.py ChatTokenizer for ASCII text
// (the Python class keeps the vocabulary construction and handles non-ASCII input itself).
//
// The serving path tokenizes every prompt and detokenizes every reply in the engine's worker
// process, beside the engine thread (llm/backends.py _worker_main): in Python the regex
// pre-split alone is ~93 us per smart-reply prompt, all of it holding the GIL the engine
// thread needs to launch its kernels.  Here the split, the vocabulary lookup and the byte
// fallback run without the GIL.
//
// Pre-split (the same pieces as the Python pattern  ` ?[A-Za-z0-9_']+| ?[^\sA-Za-z0-9_']+|\s+`
// over ASCII, whitespace as Python's str.isspace(): \t \n \v \f \r, 0x1c-0x1f, space):
//   * an optional single space followed by a run of word characters, else
//   * an optional single space followed by a run of other non-space characters, else
//   * a run of whitespace (greedy: it also takes a last space before a word).
// A piece missing from the vocabulary becomes " " + the rest when the rest is a token, else its
// bytes (ids byte_base + b).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace drtc {

class WordTokenizer {
 public:
  WordTokenizer(std::vector<std::string> vocab, int32_t byte_base, int32_t bos_id,
                std::vector<int32_t> skip_ids);

  // ids of ASCII `text` (callers check text.isascii()), BOS first when add_bos
  std::vector<int32_t> encode(std::string_view text, bool add_bos) const;
  // UTF-8 bytes of `ids` (special / skip ids dropped when skip_special)
  std::string decode(const std::vector<int64_t>& ids, bool skip_special) const;

  int32_t vocab_size() const { return (int32_t)vocab_.size(); }

 private:
  int32_t lookup(std::string_view piece) const;  // -1 when absent

  std::vector<std::string> vocab_;
  std::unordered_map<std::string_view, int32_t> ids_;  // views into vocab_
  int32_t byte_base_, bos_id_, space_id_;
  std::vector<uint8_t> skip_;  // per id: dropped by decode(skip_special = true)
};

}  // namespace drtc
