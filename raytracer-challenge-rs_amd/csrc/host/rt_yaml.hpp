// rt_yaml.hpp — the YAML subset the reference's scene files use, with
// yaml-rust 0.4.5's scalar resolution (the reference's scene-parser loads
// scenes with `YamlLoader::load_from_str`, scene-parser/src/lib.rs:92-95;
// Cargo.lock pins yaml-rust 0.4.5).
//
// Supported: comments, block mappings, block sequences (nested, and a
// sequence at the same indent as its parent key), flow sequences / mappings
// ([a, [b, c]], {k: v}), plain / single- / double-quoted scalars, the first
// document of a stream. Not supported (rejected with an error): anchors,
// aliases, tags, block scalars (| and >), multi-line flow collections.
//
// Plain scalars resolve like yaml-rust's `Yaml::from_str`: "~" / "null" ->
// Null, "true" / "false" -> Boolean, 0x.. / 0o.. / [+-]digits -> Integer
// (i64), anything Rust's f64 parser accepts (plus .inf / .nan) -> Real
// (the source text is kept, as yaml-rust does), everything else -> String.
#pragma once
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace rt {
namespace yaml {

struct Node {
  enum Kind { Null, Boolean, Integer, Real, String, Array, Hash };
  Kind kind = Null;
  bool b = false;
  int64_t i = 0;
  std::string s;  // String value, or the source text of a Real
  std::vector<Node> seq;
  std::vector<std::pair<Node, Node>> map;  // insertion order

  bool is(Kind k) const { return kind == k; }
  // yaml::Hash::get with a String key
  const Node* get(const std::string& key) const {
    for (const auto& kv : map)
      if (kv.first.kind == String && kv.first.s == key) return &kv.second;
    return nullptr;
  }
  bool contains(const std::string& key) const { return get(key) != nullptr; }
  // Yaml::as_f64: only Real converts (yaml-rust parses the kept text)
  bool as_f64(double* out) const;
  bool as_i64(int64_t* out) const {
    if (kind != Integer) return false;
    *out = i;
    return true;
  }
};

class ParseError : public std::runtime_error {
 public:
  ParseError(const std::string& m, int line) : std::runtime_error("yaml line " + std::to_string(line) + ": " + m) {}
};

namespace detail {

inline bool parse_rust_f64(const std::string& v, double* out) {
  // yaml-rust parse_f64: the YAML infinities / NaN, else str::parse::<f64>
  if (v == ".inf" || v == ".Inf" || v == ".INF" || v == "+.inf" || v == "+.Inf" || v == "+.INF") {
    *out = INFINITY;
    return true;
  }
  if (v == "-.inf" || v == "-.Inf" || v == "-.INF") {
    *out = -INFINITY;
    return true;
  }
  if (v == ".nan" || v == ".NaN" || v == ".NAN") {
    *out = NAN;
    return true;
  }
  if (v.empty()) return false;
  // Rust accepts [+-] (digits [. digits?] | . digits) ([eE] [+-]? digits)?, and inf / infinity / nan
  size_t p = 0;
  if (v[p] == '+' || v[p] == '-') ++p;
  std::string rest = v.substr(p);
  std::string low;
  for (char c : rest) low += (char)std::tolower((unsigned char)c);
  if (low == "inf" || low == "infinity" || low == "nan") {
    *out = std::strtod(v.c_str(), nullptr);
    return true;
  }
  size_t q = p, digits = 0;
  while (q < v.size() && std::isdigit((unsigned char)v[q])) ++q, ++digits;
  if (q < v.size() && v[q] == '.') {
    ++q;
    while (q < v.size() && std::isdigit((unsigned char)v[q])) ++q, ++digits;
  }
  if (digits == 0) return false;
  if (q < v.size() && (v[q] == 'e' || v[q] == 'E')) {
    ++q;
    if (q < v.size() && (v[q] == '+' || v[q] == '-')) ++q;
    size_t e0 = q;
    while (q < v.size() && std::isdigit((unsigned char)v[q])) ++q;
    if (q == e0) return false;
  }
  if (q != v.size()) return false;
  *out = std::strtod(v.c_str(), nullptr);  // correctly rounded, like Rust's parser
  return true;
}

inline bool parse_i64(const std::string& v, int base, int64_t* out) {
  if (v.empty()) return false;
  errno = 0;
  char* end = nullptr;
  long long x = std::strtoll(v.c_str(), &end, base);
  if (errno != 0 || end != v.c_str() + v.size()) return false;
  for (char c : v)
    if (std::isspace((unsigned char)c)) return false;
  *out = (int64_t)x;
  return true;
}

// yaml-rust Yaml::from_str (plain scalars)
inline Node resolve_plain(const std::string& v) {
  Node n;
  int64_t iv;
  double dv;
  if (v.rfind("0x", 0) == 0 && v.size() > 2 && parse_i64(v.substr(2), 16, &iv) && v[2] != '-' && v[2] != '+') {
    n.kind = Node::Integer; n.i = iv; return n;
  }
  if (v.rfind("0o", 0) == 0 && v.size() > 2 && parse_i64(v.substr(2), 8, &iv) && v[2] != '-' && v[2] != '+') {
    n.kind = Node::Integer; n.i = iv; return n;
  }
  if (v == "~" || v == "null") { n.kind = Node::Null; return n; }
  if (v == "true") { n.kind = Node::Boolean; n.b = true; return n; }
  if (v == "false") { n.kind = Node::Boolean; n.b = false; return n; }
  if (parse_i64(v, 10, &iv)) { n.kind = Node::Integer; n.i = iv; return n; }
  if (parse_rust_f64(v, &dv)) { n.kind = Node::Real; n.s = v; return n; }
  n.kind = Node::String; n.s = v;
  return n;
}

struct Line {
  int indent;
  std::string text;  // comment-stripped, right-trimmed, non-empty
  int no;            // 1-based source line
};

// Strip a comment (# at line start or after whitespace, outside quotes).
inline std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
  }
  return s;
}
inline std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}
inline std::string trim(const std::string& s) {
  size_t a = 0;
  while (a < s.size() && (s[a] == ' ' || s[a] == '\t')) ++a;
  return rtrim(s.substr(a));
}

class Parser {
 public:
  explicit Parser(const std::string& text) {
    int no = 0;
    size_t pos = 0;
    bool started = false;
    while (pos <= text.size()) {
      size_t nl = text.find('\n', pos);
      if (nl == std::string::npos) nl = text.size();
      std::string raw = text.substr(pos, nl - pos);
      pos = nl + 1;
      ++no;
      std::string t = rtrim(strip_comment(raw));
      if (t.empty()) continue;
      if (t == "---") {
        if (started) break;  // first document only
        continue;
      }
      if (t == "...") break;
      int ind = 0;
      while (ind < (int)t.size() && t[ind] == ' ') ++ind;
      if (ind < (int)t.size() && t[ind] == '\t') throw ParseError("tab indentation", no);
      lines_.push_back({ind, t.substr(ind), no});
      started = true;
      if (nl == text.size()) break;
    }
  }
  Node parse() {
    if (lines_.empty()) return Node{};
    Node n = parse_node(lines_[0].indent);
    if (cur_ < lines_.size()) throw ParseError("unexpected content", lines_[cur_].no);
    return n;
  }

 private:
  std::vector<Line> lines_;
  size_t cur_ = 0;

  static bool is_seq_entry(const std::string& t) { return t == "-" || t.rfind("- ", 0) == 0; }

  // position of the ':' of a block-mapping key ("key:" or "key: value"), or npos
  static size_t key_colon(const std::string& t) {
    if (t.empty() || t[0] == '[' || t[0] == '{') return std::string::npos;
    bool sq = false, dq = false;
    for (size_t i = 0; i < t.size(); ++i) {
      const char c = t[i];
      if (c == '\'' && !dq) sq = !sq;
      else if (c == '"' && !sq) dq = !dq;
      else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    }
    return std::string::npos;
  }

  Node parse_node(int indent) {
    const Line& l = lines_[cur_];
    if (is_seq_entry(l.text)) return parse_seq(l.indent);
    if (key_colon(l.text) != std::string::npos) return parse_map(l.indent);
    ++cur_;
    return parse_inline(l.text, l.no);
    (void)indent;
  }

  Node parse_seq(int indent) {
    Node n;
    n.kind = Node::Array;
    while (cur_ < lines_.size() && lines_[cur_].indent == indent && is_seq_entry(lines_[cur_].text)) {
      Line& l = lines_[cur_];
      if (l.text == "-") {
        ++cur_;
        if (cur_ < lines_.size() && lines_[cur_].indent > indent) n.seq.push_back(parse_node(lines_[cur_].indent));
        else n.seq.push_back(Node{});
        continue;
      }
      // "- rest": the rest is a node whose first line sits at indent + 2 (+ extra spaces)
      size_t k = 2;
      while (k < l.text.size() && l.text[k] == ' ') ++k;
      l.indent = indent + (int)k;
      l.text = l.text.substr(k);
      n.seq.push_back(parse_node(l.indent));
    }
    if (cur_ < lines_.size() && lines_[cur_].indent > indent)
      throw ParseError("bad indentation in sequence", lines_[cur_].no);
    return n;
  }

  Node parse_map(int indent) {
    Node n;
    n.kind = Node::Hash;
    while (cur_ < lines_.size() && lines_[cur_].indent == indent && !is_seq_entry(lines_[cur_].text)) {
      const Line l = lines_[cur_];
      const size_t c = key_colon(l.text);
      if (c == std::string::npos) throw ParseError("expected 'key: value'", l.no);
      Node key = parse_inline(trim(l.text.substr(0, c)), l.no);
      const std::string rest = trim(l.text.substr(c + 1));
      ++cur_;
      Node val;
      if (!rest.empty()) {
        if (rest[0] == '|' || rest[0] == '>') throw ParseError("block scalars are not supported", l.no);
        val = parse_inline(rest, l.no);
      } else if (cur_ < lines_.size() && lines_[cur_].indent > indent) {
        val = parse_node(lines_[cur_].indent);
      } else if (cur_ < lines_.size() && lines_[cur_].indent == indent && is_seq_entry(lines_[cur_].text)) {
        val = parse_seq(indent);  // "key:\n- item" at the key's indent
      }
      for (const auto& kv : n.map)
        if (kv.first.kind == key.kind && kv.first.s == key.s && kv.first.i == key.i && key.kind == Node::String)
          throw ParseError("duplicate key '" + key.s + "'", l.no);
      n.map.emplace_back(std::move(key), std::move(val));
    }
    if (cur_ < lines_.size() && lines_[cur_].indent > indent)
      throw ParseError("bad indentation in mapping", lines_[cur_].no);
    return n;
  }

  // a scalar or a flow collection on one line
  Node parse_inline(const std::string& t, int no) {
    size_t p = 0;
    Node n = parse_flow(t, p, no, false);
    while (p < t.size() && t[p] == ' ') ++p;
    if (p != t.size()) throw ParseError("trailing characters '" + t.substr(p) + "'", no);
    return n;
  }

  static void skip_ws(const std::string& t, size_t& p) {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t')) ++p;
  }

  Node parse_flow(const std::string& t, size_t& p, int no, bool in_flow) {
    skip_ws(t, p);
    if (p >= t.size()) return Node{};
    const char c = t[p];
    if (c == '&' || c == '*' || c == '!') throw ParseError("anchors, aliases and tags are not supported", no);
    if (c == '[') {
      Node n;
      n.kind = Node::Array;
      ++p;
      skip_ws(t, p);
      if (p < t.size() && t[p] == ']') { ++p; return n; }
      while (true) {
        n.seq.push_back(parse_flow(t, p, no, true));
        skip_ws(t, p);
        if (p >= t.size()) throw ParseError("unterminated flow sequence", no);
        if (t[p] == ',') { ++p; skip_ws(t, p); if (p < t.size() && t[p] == ']') { ++p; return n; } continue; }
        if (t[p] == ']') { ++p; return n; }
        throw ParseError("expected ',' or ']'", no);
      }
    }
    if (c == '{') {
      Node n;
      n.kind = Node::Hash;
      ++p;
      skip_ws(t, p);
      if (p < t.size() && t[p] == '}') { ++p; return n; }
      while (true) {
        Node k = parse_flow(t, p, no, true);
        skip_ws(t, p);
        Node v;
        if (p < t.size() && t[p] == ':') { ++p; v = parse_flow(t, p, no, true); }
        n.map.emplace_back(std::move(k), std::move(v));
        skip_ws(t, p);
        if (p >= t.size()) throw ParseError("unterminated flow mapping", no);
        if (t[p] == ',') { ++p; continue; }
        if (t[p] == '}') { ++p; return n; }
        throw ParseError("expected ',' or '}'", no);
      }
    }
    if (c == '"' || c == '\'') {
      Node n;
      n.kind = Node::String;
      ++p;
      while (true) {
        if (p >= t.size()) throw ParseError("unterminated quoted scalar", no);
        const char d = t[p++];
        if (d == c) {
          if (c == '\'' && p < t.size() && t[p] == '\'') { n.s += '\''; ++p; continue; }
          break;
        }
        if (c == '"' && d == '\\' && p < t.size()) {
          const char e = t[p++];
          switch (e) {
            case 'n': n.s += '\n'; break;
            case 't': n.s += '\t'; break;
            case '\\': n.s += '\\'; break;
            case '"': n.s += '"'; break;
            case '/': n.s += '/'; break;
            default: throw ParseError(std::string("unsupported escape \\") + e, no);
          }
          continue;
        }
        n.s += d;
      }
      return n;
    }
    // plain scalar: up to ',' ']' '}' (in flow) or ': ' (flow mapping key)
    size_t q = p;
    while (q < t.size()) {
      const char d = t[q];
      if (in_flow && (d == ',' || d == ']' || d == '}')) break;
      if (in_flow && d == ':' && (q + 1 == t.size() || t[q + 1] == ' ')) break;
      ++q;
    }
    const std::string v = rtrim(t.substr(p, q - p));
    p = q;
    return resolve_plain(v);
  }
};

}  // namespace detail

inline bool Node::as_f64(double* out) const {
  if (kind != Real) return false;
  return detail::parse_rust_f64(s, out);
}

// YamlLoader::load_from_str(..)[0]
inline Node load(const std::string& text) { return detail::Parser(text).parse(); }

}  // namespace yaml
}  // namespace rt
