#include "gojson.h"

#include <cstdint>

namespace llmc {

// Length of the valid UTF-8 sequence at s[i], or 0 if invalid (Go utf8.DecodeRune semantics).
static size_t valid_utf8_len(const unsigned char* s, size_t n, size_t i, uint32_t* cp) {
  const unsigned char c0 = s[i];
  if (c0 < 0x80) { *cp = c0; return 1; }
  if (c0 < 0xC2) return 0;  // continuation byte or overlong 2-byte lead
  auto cont = [&](size_t k) { return i + k < n && (s[i + k] & 0xC0) == 0x80; };
  if (c0 < 0xE0) {
    if (!cont(1)) return 0;
    *cp = ((c0 & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu);
    return 2;
  }
  if (c0 < 0xF0) {
    if (!cont(1) || !cont(2)) return 0;
    const unsigned char c1 = s[i + 1];
    if (c0 == 0xE0 && c1 < 0xA0) return 0;   // overlong
    if (c0 == 0xED && c1 >= 0xA0) return 0;  // surrogate
    *cp = ((c0 & 0x0Fu) << 12) | ((c1 & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
    return 3;
  }
  if (c0 < 0xF5) {
    if (!cont(1) || !cont(2) || !cont(3)) return 0;
    const unsigned char c1 = s[i + 1];
    if (c0 == 0xF0 && c1 < 0x90) return 0;   // overlong
    if (c0 == 0xF4 && c1 >= 0x90) return 0;  // > U+10FFFF
    *cp = ((c0 & 0x07u) << 18) | ((c1 & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
    return 4;
  }
  return 0;
}

std::string go_json_string(const std::string& in) {
  static const char hex[] = "0123456789abcdef";
  const unsigned char* s = reinterpret_cast<const unsigned char*>(in.data());
  const size_t n = in.size();
  std::string out;
  out.reserve(n + 2 + n / 8);
  out.push_back('"');
  size_t i = 0;
  while (i < n) {
    const unsigned char b = s[i];
    if (b < 0x80) {
      switch (b) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '<': case '>': case '&':
          out += "\\u00"; out.push_back(hex[b >> 4]); out.push_back(hex[b & 0xF]); break;
        default:
          if (b < 0x20) {
            out += "\\u00"; out.push_back(hex[b >> 4]); out.push_back(hex[b & 0xF]);
          } else {
            out.push_back(static_cast<char>(b));
          }
      }
      ++i;
      continue;
    }
    uint32_t cp = 0;
    const size_t len = valid_utf8_len(s, n, i, &cp);
    if (len == 0) {
      out += "\\ufffd";
      ++i;
      continue;
    }
    if (cp == 0x2028 || cp == 0x2029) {
      out += (cp == 0x2028) ? "\\u2028" : "\\u2029";
    } else {
      out.append(in, i, len);
    }
    i += len;
  }
  out.push_back('"');
  return out;
}

}  // namespace llmc
