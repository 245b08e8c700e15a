// Incremental, UTF-8-safe detokenizer (SURVEY.md §7.5 hard part 9).
//
// Byte-level BPE / Unigram pieces can end in the middle of a multi-byte UTF-8
// character, so each `token` WebSocket frame must carry only complete
// characters.  Each stream keeps its pending bytes; push() appends the bytes of
// one id and returns the longest valid UTF-8 prefix (invalid bytes become
// U+FFFD so a stream can never stall), flush() drains the rest.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ftrt {

class Detokenizer {
 public:
  explicit Detokenizer(std::vector<std::string> id_bytes);

  int new_stream();
  void release(int sid);
  std::string push(int sid, int32_t token);
  std::vector<std::string> push_many(const std::vector<int>& sids,
                                     const std::vector<int32_t>& tokens);
  std::string flush(int sid);
  int vocab_size() const { return (int)id_bytes_.size(); }

  // decode a complete token list (replacement chars for invalid bytes)
  std::string decode(const std::vector<int32_t>& tokens) const;

 private:
  static size_t take_valid(const std::string& buf, std::string& out, bool final);
  std::vector<std::string> id_bytes_;
  std::vector<std::string> pending_;
  std::vector<uint8_t> live_;
  std::vector<int> free_ids_;
};

}  // namespace ftrt
