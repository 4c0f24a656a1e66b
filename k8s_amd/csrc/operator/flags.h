// Go-`flag`-compatible command line parsing: -name=value, --name=value,
// -name value, boolean -name. Unknown glog flags (-alsologtostderr, -v,
// -logtostderr, -stderrthreshold) are accepted.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace tfop {

class Flags {
 public:
  void def(const std::string& name, const std::string& def, const std::string& help, bool is_bool = false);
  // returns error text ("" ok); positional args collected in args()
  std::string parse(int argc, char** argv);
  std::string str(const std::string& n) const;
  int num(const std::string& n) const;
  bool on(const std::string& n) const;
  const std::vector<std::string>& args() const { return args_; }
  std::string usage() const;

 private:
  struct F {
    std::string value, help;
    bool is_bool;
  };
  std::map<std::string, F> f_;
  std::vector<std::string> args_;
};

extern const char* kVersion;
extern const char* kGitSHA;

}  // namespace tfop
