// Minimal JSON DOM for the host side: non-file actions (protocol / metaData / txn lines, a few per
// commit) and record materialisation at export. The bulk of the log never goes through here.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace dr {

struct JVal {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  std::string s;        // STR value (unescaped) or NUM text
  std::vector<JVal> a;
  std::vector<std::pair<std::string, JVal>> o;  // insertion order; duplicate keys: last wins on get
  const JVal* get(const std::string& k) const {
    const JVal* r = nullptr;
    for (auto& kv : o) if (kv.first == k) r = &kv.second;
    return r;
  }
  bool is_int() const;
  int64_t as_int() const;
};

// Parses one JSON text; returns false (and leaves `err`) on malformed input.
bool json_parse(const char* p, size_t n, JVal* out, std::string* err = nullptr);
// Serialises compactly (Jackson-like: no spaces).
std::string json_dump(const JVal& v);
std::string json_quote(const std::string& s);

}  // namespace dr
