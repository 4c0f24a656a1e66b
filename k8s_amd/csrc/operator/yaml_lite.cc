#include "yaml_lite.h"

#include <cctype>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace tfop {

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

namespace {

struct Line {
  int indent;
  std::string text;  // without indentation, comments stripped (outside quotes)
  int lineno;
};

std::string rstrip(const std::string& s) {
  size_t e = s.size();
  while (e > 0 && isspace((unsigned char)s[e - 1])) --e;
  return s.substr(0, e);
}

std::string strip(const std::string& s) {
  size_t b = 0;
  while (b < s.size() && isspace((unsigned char)s[b])) ++b;
  return rstrip(s.substr(b));
}

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || isspace((unsigned char)s[i - 1]))) return s.substr(0, i);
  }
  return s;
}

// unclosed '[' / '{' outside quotes (> 0: the flow collection continues on the next line)
int flow_depth(const std::string& s) {
  bool sq = false, dq = false;
  int d = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (dq && c == '\\') { ++i; continue; }
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (!sq && !dq && (c == '[' || c == '{')) ++d;
    else if (!sq && !dq && (c == ']' || c == '}')) --d;
  }
  return d;
}

Json scalar(const std::string& raw) {
  std::string s = strip(raw);
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Json();
  if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
    // reuse the JSON string decoder for escapes
    return Json::parse(s);
  }
  if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
        out += '\'';
        ++i;
      } else {
        out += s[i];
      }
    }
    return Json(out);
  }
  if (s == "true" || s == "True" || s == "TRUE") return Json(true);
  if (s == "false" || s == "False" || s == "FALSE") return Json(false);
  // integer
  {
    size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
    bool digits = i < s.size();
    for (size_t k = i; k < s.size(); ++k)
      if (!isdigit((unsigned char)s[k])) digits = false;
    if (digits) {
      try {
        return Json((long long)std::stoll(s));
      } catch (...) {
      }
    }
  }
  // float
  {
    char* end = nullptr;
    double d = strtod(s.c_str(), &end);
    bool numchars = true;
    for (char c : s)
      if (!(isdigit((unsigned char)c) || c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+')) numchars = false;
    if (numchars && end && *end == '\0' && s.find_first_of("0123456789") != std::string::npos) return Json(d);
  }
  return Json(s);
}

// flow collections: [a, b, {c: d}] / {a: 1, b: [x]}
Json flow_parse(const std::string& s);

Json flow_map(const std::string& s, size_t& i);
Json flow_seq(const std::string& s, size_t& i);

void fws(const std::string& s, size_t& i) {
  while (i < s.size() && isspace((unsigned char)s[i])) ++i;
}

std::string flow_token(const std::string& s, size_t& i, bool key) {
  fws(s, i);
  if (i < s.size() && (s[i] == '"' || s[i] == '\'')) {
    char q = s[i];
    size_t st = i++;
    while (i < s.size() && s[i] != q) {
      if (s[i] == '\\' && q == '"') ++i;
      ++i;
    }
    ++i;
    return s.substr(st, i - st);
  }
  size_t st = i;
  while (i < s.size() && s[i] != ',' && s[i] != ']' && s[i] != '}') {
    if (key && s[i] == ':') break;
    ++i;
  }
  return s.substr(st, i - st);
}

Json flow_value(const std::string& s, size_t& i) {
  fws(s, i);
  if (i < s.size() && s[i] == '[') return flow_seq(s, i);
  if (i < s.size() && s[i] == '{') return flow_map(s, i);
  return scalar(flow_token(s, i, false));
}

Json flow_seq(const std::string& s, size_t& i) {
  ++i;  // [
  Json a = Json::array();
  fws(s, i);
  if (i < s.size() && s[i] == ']') {
    ++i;
    return a;
  }
  while (i < s.size()) {
    a.push_back(flow_value(s, i));
    fws(s, i);
    if (i < s.size() && s[i] == ',') {
      ++i;
      continue;
    }
    if (i < s.size() && s[i] == ']') {
      ++i;
      return a;
    }
    break;
  }
  throw std::runtime_error("yaml: bad flow sequence: " + s);
}

Json flow_map(const std::string& s, size_t& i) {
  ++i;  // {
  Json o = Json::object();
  fws(s, i);
  if (i < s.size() && s[i] == '}') {
    ++i;
    return o;
  }
  while (i < s.size()) {
    Json k = scalar(flow_token(s, i, true));
    fws(s, i);
    if (i >= s.size() || s[i] != ':') throw std::runtime_error("yaml: bad flow map: " + s);
    ++i;
    o[k.is_string() ? k.as_string() : k.dump()] = flow_value(s, i);
    fws(s, i);
    if (i < s.size() && s[i] == ',') {
      ++i;
      continue;
    }
    if (i < s.size() && s[i] == '}') {
      ++i;
      return o;
    }
    break;
  }
  throw std::runtime_error("yaml: bad flow map: " + s);
}

Json flow_parse(const std::string& s) {
  size_t i = 0;
  return flow_value(s, i);
}

Json value_of(const std::string& v) {
  std::string t = strip(v);
  if (!t.empty() && (t[0] == '[' || t[0] == '{')) return flow_parse(t);
  return scalar(t);
}

// find "key: value" split point (colon followed by space or end, outside quotes)
bool split_key(const std::string& t, std::string& key, std::string& rest) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < t.size(); ++i) {
    char c = t[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) {
      Json k = scalar(t.substr(0, i));
      key = k.is_string() ? k.as_string() : k.dump();
      rest = i + 1 < t.size() ? t.substr(i + 1) : "";
      return true;
    }
    if ((c == '[' || c == '{') && i == 0) return false;
  }
  return false;
}

class Parser {
 public:
  Parser(std::vector<Line> lines, std::vector<std::string> raw) : L(std::move(lines)), raw_(std::move(raw)) {}
  Json parse() {
    if (L.empty()) return Json();
    return block(L[0].indent);
  }

 private:
  std::vector<Line> L;
  std::vector<std::string> raw_;
  size_t p = 0;

  Json block(int indent) {
    if (p >= L.size()) return Json();
    if (L[p].text.rfind("- ", 0) == 0 || L[p].text == "-") return seq(L[p].indent);
    return map(indent);
  }

  Json block_scalar(const std::string& style, int parent_indent) {
    // collect raw lines with indentation > parent_indent
    std::string out;
    bool fold = style[0] == '>';
    int bi = -1;
    while (p < L.size() && L[p].indent > parent_indent) {
      const std::string& r = raw_[L[p].lineno];
      if (bi < 0) bi = L[p].indent;
      std::string content = r.size() > (size_t)bi ? r.substr(bi) : "";
      if (!out.empty()) out += fold ? " " : "\n";
      out += rstrip(content);
      ++p;
    }
    if (style.find('-') == std::string::npos) out += "\n";
    return Json(out);
  }

  Json after_key(const std::string& rest, int indent) {
    std::string r = strip(rest);
    if (r == "|" || r == "|-" || r == ">" || r == ">-" || r == "|+" || r == ">+") return block_scalar(r, indent);
    if (!r.empty()) return value_of(r);
    if (p < L.size() && (L[p].indent > indent || (L[p].indent == indent && L[p].text.rfind("-", 0) == 0 &&
                                                  (L[p].text.size() == 1 || L[p].text[1] == ' '))))
      return block(L[p].indent);
    return Json();
  }

  Json map(int indent) {
    Json o = Json::object();
    while (p < L.size() && L[p].indent == indent) {
      const std::string t = L[p].text;
      if (t.rfind("- ", 0) == 0 || t == "-") break;
      std::string key, rest;
      if (!split_key(t, key, rest)) throw std::runtime_error("yaml: expected 'key: value' at line " +
                                                             std::to_string(L[p].lineno + 1) + ": " + t);
      ++p;
      o[key] = after_key(rest, indent);
    }
    return o;
  }

  Json seq(int indent) {
    Json a = Json::array();
    while (p < L.size() && L[p].indent == indent && (L[p].text.rfind("- ", 0) == 0 || L[p].text == "-")) {
      std::string item = L[p].text == "-" ? "" : L[p].text.substr(2);
      std::string itrim = strip(item);
      size_t lead = 0;
      while (lead < item.size() && item[lead] == ' ') ++lead;
      const int child_indent = indent + 2 + (int)lead;
      if (itrim.empty()) {
        ++p;
        if (p < L.size() && L[p].indent > indent) a.push_back(block(L[p].indent));
        else a.push_back(Json());
        continue;
      }
      std::string key, rest;
      if ((itrim[0] != '[' && itrim[0] != '{' && itrim[0] != '"' && itrim[0] != '\'') && split_key(itrim, key, rest)) {
        // a mapping starting on the dash line: rewrite this line as a map entry at child_indent
        L[p].indent = child_indent;
        L[p].text = itrim;
        a.push_back(map(child_indent));
      } else if (itrim.rfind("- ", 0) == 0) {
        L[p].indent = child_indent;
        L[p].text = itrim;
        a.push_back(seq(child_indent));
      } else {
        ++p;
        a.push_back(value_of(itrim));
      }
    }
    return a;
  }
};

std::vector<std::vector<std::string>> split_docs(const std::string& text) {
  std::vector<std::vector<std::string>> docs(1);
  std::stringstream ss(text);
  std::string line;
  while (std::getline(ss, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.rfind("---", 0) == 0 && strip(line.substr(3)).empty()) {
      docs.emplace_back();
      continue;
    }
    if (line.rfind("...", 0) == 0 && strip(line.substr(3)).empty()) continue;
    docs.back().push_back(line);
  }
  return docs;
}

Json parse_doc(const std::vector<std::string>& raw) {
  // a document that is one flow collection (JSON is a YAML subset)
  std::string all;
  for (auto& r : raw) all += strip_comment(r) + "\n";
  std::string t = strip(all);
  if (!t.empty() && (t[0] == '{' || t[0] == '[')) {
    try {
      return Json::parse(t);
    } catch (const JsonError&) {
      std::string flat;
      for (char c : t) flat += (c == '\n' ? ' ' : c);
      return flow_parse(flat);
    }
  }
  std::vector<Line> lines;
  for (size_t i = 0; i < raw.size(); ++i) {
    std::string s = strip_comment(raw[i]);
    if (strip(s).empty()) continue;
    // a flow collection continued over several lines: join until the brackets balance
    const size_t first = i;
    while (flow_depth(s) > 0 && i + 1 < raw.size()) s = rstrip(s) + " " + strip(strip_comment(raw[++i]));
    if (s.find('\t') != std::string::npos && s.find_first_not_of(" \t") > s.find('\t'))
      throw std::runtime_error("yaml: tabs are not allowed for indentation");
    int ind = 0;
    while (ind < (int)s.size() && s[ind] == ' ') ++ind;
    lines.push_back({ind, rstrip(s.substr(ind)), (int)first});
  }
  // block scalars need raw (comment-preserving) text; Parser reads raw_ for them
  Parser p(std::move(lines), raw);
  return p.parse();
}

}  // namespace

Json yaml_parse(const std::string& text) {
  for (auto& d : split_docs(text)) {
    Json j = parse_doc(d);
    if (!j.is_null()) return j;
  }
  return Json();
}

std::vector<Json> yaml_parse_all(const std::string& text) {
  std::vector<Json> out;
  for (auto& d : split_docs(text)) {
    Json j = parse_doc(d);
    if (!j.is_null()) out.push_back(j);
  }
  return out;
}

}  // namespace tfop
