// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product (pixie_amd/).
//
// Minimal JSON reader used by the CPU Carnot restatement to read plans handed over by the
// Python test harness (protobuf JSON mapping of px.carnot.planpb.Plan, produced with
// google.protobuf.json_format from the same message the product receives as binary planpb).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oracle {

struct Json {
  enum Kind { kNull, kBool, kNumber, kString, kArray, kObject } kind = kNull;
  bool b = false;
  std::string num;  // numbers kept as text so int64 values stay exact
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;

  bool has(const std::string& k) const { return kind == kObject && obj.count(k) > 0; }
  const Json& operator[](const std::string& k) const {
    static const Json null_json;
    if (kind != kObject) return null_json;
    auto it = obj.find(k);
    return it == obj.end() ? null_json : it->second;
  }
  size_t size() const { return kind == kArray ? arr.size() : 0; }
  const Json& at(size_t i) const { return arr.at(i); }

  // protobuf JSON mapping renders int64/uint64 as strings and int32/enums as numbers or names.
  int64_t as_i64(int64_t dflt = 0) const {
    if (kind == kNumber) return static_cast<int64_t>(std::strtoll(num.c_str(), nullptr, 10));
    if (kind == kString) return static_cast<int64_t>(std::strtoll(str.c_str(), nullptr, 10));
    if (kind == kBool) return b ? 1 : 0;
    return dflt;
  }
  uint64_t as_u64(uint64_t dflt = 0) const {
    if (kind == kNumber) return std::strtoull(num.c_str(), nullptr, 10);
    if (kind == kString) return std::strtoull(str.c_str(), nullptr, 10);
    return dflt;
  }
  double as_f64(double dflt = 0) const {
    if (kind == kNumber) return std::strtod(num.c_str(), nullptr);
    if (kind == kString) {
      if (str == "NaN") return std::strtod("nan", nullptr);
      if (str == "Infinity") return std::strtod("inf", nullptr);
      if (str == "-Infinity") return std::strtod("-inf", nullptr);
      return std::strtod(str.c_str(), nullptr);
    }
    return dflt;
  }
  bool as_bool(bool dflt = false) const { return kind == kBool ? b : dflt; }
  const std::string& as_str() const { return str; }
};

class JsonParser {
 public:
  explicit JsonParser(const std::string& s) : s_(s) {}
  Json Parse() {
    Json j = Value();
    Ws();
    if (i_ != s_.size()) throw std::runtime_error("json: trailing characters");
    return j;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;

  void Ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) ++i_;
  }
  char Peek() {
    Ws();
    if (i_ >= s_.size()) throw std::runtime_error("json: unexpected end");
    return s_[i_];
  }
  void Expect(char c) {
    if (Peek() != c) throw std::runtime_error(std::string("json: expected ") + c);
    ++i_;
  }
  Json Value() {
    char c = Peek();
    Json j;
    if (c == '{') {
      j.kind = Json::kObject;
      ++i_;
      if (Peek() == '}') { ++i_; return j; }
      while (true) {
        std::string k = String();
        Expect(':');
        j.obj[k] = Value();
        char d = Peek();
        ++i_;
        if (d == '}') break;
        if (d != ',') throw std::runtime_error("json: bad object");
      }
    } else if (c == '[') {
      j.kind = Json::kArray;
      ++i_;
      if (Peek() == ']') { ++i_; return j; }
      while (true) {
        j.arr.push_back(Value());
        char d = Peek();
        ++i_;
        if (d == ']') break;
        if (d != ',') throw std::runtime_error("json: bad array");
      }
    } else if (c == '"') {
      j.kind = Json::kString;
      j.str = String();
    } else if (c == 't' || c == 'f') {
      j.kind = Json::kBool;
      j.b = (c == 't');
      i_ += j.b ? 4 : 5;
    } else if (c == 'n') {
      i_ += 4;
    } else {
      j.kind = Json::kNumber;
      size_t st = i_;
      while (i_ < s_.size() && (isdigit(static_cast<unsigned char>(s_[i_])) || s_[i_] == '-' ||
                                s_[i_] == '+' || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E'))
        ++i_;
      j.num = s_.substr(st, i_ - st);
    }
    return j;
  }
  static void PutUtf8(std::string* out, uint32_t cp) {
    if (cp < 0x80) {
      out->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  std::string String() {
    Expect('"');
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c != '\\') { out.push_back(c); continue; }
      char e = s_[i_++];
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'u': {
          uint32_t cp = std::strtoul(s_.substr(i_, 4).c_str(), nullptr, 16);
          i_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
            uint32_t lo = std::strtoul(s_.substr(i_ + 2, 4).c_str(), nullptr, 16);
            i_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          PutUtf8(&out, cp);
          break;
        }
        default: out.push_back(e);
      }
    }
    ++i_;
    return out;
  }
};

inline Json ParseJson(const std::string& s) { return JsonParser(s).Parse(); }

}  // namespace oracle
