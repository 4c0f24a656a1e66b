#include "flags.h"

#include <cstdlib>

namespace tfop {

// version/version.go: Version = "0.3.0+git"; ours marks the MI355X-native build.
const char* kVersion = "0.3.0+amd";
const char* kGitSHA = "Not provided.";

void Flags::def(const std::string& name, const std::string& d, const std::string& help, bool is_bool) {
  f_[name] = F{d, help, is_bool};
}

std::string Flags::parse(int argc, char** argv) {
  static const char* glog_bool[] = {"alsologtostderr", "logtostderr"};
  static const char* glog_val[] = {"stderrthreshold", "log_dir", "vmodule", "log_backtrace_at"};
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") {
      for (++i; i < argc; ++i) args_.push_back(argv[i]);
      break;
    }
    if (a.size() < 2 || a[0] != '-') {
      args_.push_back(a);
      continue;
    }
    std::string s = a.substr(a[1] == '-' ? 2 : 1);
    std::string name = s, val;
    bool has_val = false;
    size_t eq = s.find('=');
    if (eq != std::string::npos) {
      name = s.substr(0, eq);
      val = s.substr(eq + 1);
      has_val = true;
    }
    auto it = f_.find(name);
    if (it == f_.end()) {
      bool known = false;
      for (auto g : glog_bool)
        if (name == g) known = true;
      for (auto g : glog_val)
        if (name == g) {
          known = true;
          if (!has_val && i + 1 < argc) ++i;
        }
      if (name == "v") {
        known = true;
        if (!has_val && i + 1 < argc) val = argv[++i];
        f_["v"] = F{val, "log verbosity", false};
      }
      if (!known) return "flag provided but not defined: -" + name;
      continue;
    }
    if (it->second.is_bool) {
      it->second.value = has_val ? val : "true";
    } else {
      if (!has_val) {
        if (i + 1 >= argc) return "flag needs an argument: -" + name;
        val = argv[++i];
      }
      it->second.value = val;
    }
  }
  return "";
}

std::string Flags::str(const std::string& n) const {
  auto it = f_.find(n);
  return it == f_.end() ? "" : it->second.value;
}
int Flags::num(const std::string& n) const { return atoi(str(n).c_str()); }
bool Flags::on(const std::string& n) const {
  std::string v = str(n);
  return v == "true" || v == "1" || v == "True" || v == "TRUE";
}

std::string Flags::usage() const {
  std::string u;
  for (auto& kv : f_) u += "  -" + kv.first + (kv.second.is_bool ? "" : " value") + "\n    \t" + kv.second.help + "\n";
  return u;
}

}  // namespace tfop
