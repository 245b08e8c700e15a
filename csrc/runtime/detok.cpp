#include "detok.h"

#include <stdexcept>

namespace ftrt {

static const char kRepl[] = "\xEF\xBF\xBD";  // U+FFFD

Detokenizer::Detokenizer(std::vector<std::string> id_bytes) : id_bytes_(std::move(id_bytes)) {}

int Detokenizer::new_stream() {
  if (!free_ids_.empty()) {
    const int s = free_ids_.back();
    free_ids_.pop_back();
    pending_[s].clear();
    live_[s] = 1;
    return s;
  }
  pending_.emplace_back();
  live_.push_back(1);
  return (int)pending_.size() - 1;
}

void Detokenizer::release(int sid) {
  if (sid < 0 || sid >= (int)pending_.size() || !live_[sid]) return;
  live_[sid] = 0;
  pending_[sid].clear();
  free_ids_.push_back(sid);
}

// Move the longest decodable prefix of `buf` to `out`; returns bytes consumed.
size_t Detokenizer::take_valid(const std::string& buf, std::string& out, bool final) {
  const size_t n = buf.size();
  size_t i = 0;
  while (i < n) {
    const unsigned char c = (unsigned char)buf[i];
    size_t len;
    if (c < 0x80) {
      out.push_back((char)c);
      ++i;
      continue;
    } else if ((c & 0xE0) == 0xC0 && c >= 0xC2) {
      len = 2;
    } else if ((c & 0xF0) == 0xE0) {
      len = 3;
    } else if ((c & 0xF8) == 0xF0 && c <= 0xF4) {
      len = 4;
    } else {
      out.append(kRepl);
      ++i;
      continue;
    }
    // check the continuation bytes that are present
    size_t k = 1;
    bool bad = false;
    for (; k < len && i + k < n; ++k) {
      const unsigned char cc = (unsigned char)buf[i + k];
      if ((cc & 0xC0) != 0x80) { bad = true; break; }
      if (k == 1) {  // overlong / surrogate / range checks on the second byte
        if (c == 0xE0 && cc < 0xA0) { bad = true; break; }
        if (c == 0xED && cc > 0x9F) { bad = true; break; }
        if (c == 0xF0 && cc < 0x90) { bad = true; break; }
        if (c == 0xF4 && cc > 0x8F) { bad = true; break; }
      }
    }
    if (bad) {
      out.append(kRepl);
      ++i;
      continue;
    }
    if (i + len > n) {  // incomplete character at the end
      if (final) {
        out.append(kRepl);
        return n;
      }
      return i;
    }
    out.append(buf, i, len);
    i += len;
  }
  return n;
}

std::string Detokenizer::push(int sid, int32_t token) {
  if (sid < 0 || sid >= (int)pending_.size() || !live_[sid]) throw std::out_of_range("stream");
  std::string& p = pending_[sid];
  if (token >= 0 && token < (int32_t)id_bytes_.size()) p += id_bytes_[token];
  std::string out;
  const size_t used = take_valid(p, out, false);
  p.erase(0, used);
  return out;
}

std::vector<std::string> Detokenizer::push_many(const std::vector<int>& sids,
                                                const std::vector<int32_t>& tokens) {
  if (sids.size() != tokens.size()) throw std::invalid_argument("length mismatch");
  std::vector<std::string> out;
  out.reserve(sids.size());
  for (size_t i = 0; i < sids.size(); ++i) out.push_back(push(sids[i], tokens[i]));
  return out;
}

std::string Detokenizer::flush(int sid) {
  if (sid < 0 || sid >= (int)pending_.size() || !live_[sid]) return std::string();
  std::string out;
  take_valid(pending_[sid], out, true);
  pending_[sid].clear();
  return out;
}

std::string Detokenizer::decode(const std::vector<int32_t>& tokens) const {
  std::string all;
  for (int32_t t : tokens)
    if (t >= 0 && t < (int32_t)id_bytes_.size()) all += id_bytes_[t];
  std::string out;
  take_valid(all, out, true);
  return out;
}

}  // namespace ftrt
