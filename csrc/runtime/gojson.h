// Go encoding/json string-literal encoder (reference output: cmd/llm-consensus/main.go:227-228
// uses json.NewEncoder with default HTML escaping). Reproduced byte-for-byte:
//   '"' and '\\' backslash-escaped; \b \f \n \r \t short escapes; other bytes < 0x20 as \u00xx;
//   '<' '>' '&' as < > &; U+2028/U+2029 as  / ; each byte of an
//   invalid UTF-8 sequence (Go's DecodeRune rules: overlong, surrogate, > U+10FFFF, truncated)
//   as �; everything else copied raw.
#pragma once
#include <string>

namespace llmc {
std::string go_json_string(const std::string& utf8);
}
