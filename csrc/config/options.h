// Typed option registry with the gpgpusim.config grammar.
//
// Grammar (compatible with the reference OptionParser, option_parser.cc:201-322):
//   * a config file is a stream of whitespace separated tokens; '#' starts a
//     comment that runs to the end of the line;
//   * "double quoted" values may span several tokens / lines (joined by ' ');
//   * `-config <file>` includes another file (paths relative to the CWD);
//   * boolean flags take an optional 0/1 value;
//   * an unknown option is a fatal error; the last occurrence wins.
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace asim {

class OptionError : public std::runtime_error {
 public:
  explicit OptionError(const std::string& m) : std::runtime_error(m) {}
};

enum class OptType { Bool, Int32, UInt32, Int64, UInt64, Float, Double, Str };

class OptionRegistry {
 public:
  struct Opt {
    std::string name;
    OptType type;
    void* dst;
    std::string help;
    std::string deflt;
    std::string value;  // textual value last assigned
    bool parsed = false;
    // internal storage when dst == nullptr
    long long iv = 0;
    unsigned long long uv = 0;
    double dv = 0;
    std::string sv;
  };

  void reg(const std::string& name, OptType t, void* dst, const std::string& help, const std::string& deflt);
  // convenience overloads
  void reg(const std::string& n, bool* d, const std::string& h, const std::string& df) { reg(n, OptType::Bool, d, h, df); }
  void reg(const std::string& n, int32_t* d, const std::string& h, const std::string& df) { reg(n, OptType::Int32, d, h, df); }
  void reg(const std::string& n, uint32_t* d, const std::string& h, const std::string& df) { reg(n, OptType::UInt32, d, h, df); }
  void reg(const std::string& n, int64_t* d, const std::string& h, const std::string& df) { reg(n, OptType::Int64, d, h, df); }
  void reg(const std::string& n, uint64_t* d, const std::string& h, const std::string& df) { reg(n, OptType::UInt64, d, h, df); }
  void reg(const std::string& n, float* d, const std::string& h, const std::string& df) { reg(n, OptType::Float, d, h, df); }
  void reg(const std::string& n, double* d, const std::string& h, const std::string& df) { reg(n, OptType::Double, d, h, df); }
  void reg(const std::string& n, std::string* d, const std::string& h, const std::string& df) { reg(n, OptType::Str, d, h, df); }

  // internally stored option (table driven registration)
  void reg(const std::string& n, OptType t, const std::string& h, const std::string& df) { reg(n, t, nullptr, h, df); }
  // typed getters (work for internal and external storage)
  long long geti(const std::string& n) const;
  unsigned long long getu(const std::string& n) const;
  bool getb(const std::string& n) const { return geti(n) != 0; }
  double getd(const std::string& n) const;
  std::string gets(const std::string& n) const;

  // argv[0] is skipped like a program name
  void parse_cmdline(const std::vector<std::string>& argv, bool skip_first = true);
  void parse_file(const std::string& path);
  // directories of the -config files read so far (relative file options such
  // as -inter_config_file are looked up there, like run directories expect)
  const std::vector<std::string>& config_dirs() const { return config_dirs_; }
  // parse a string of tokens; characters in `delims` act as whitespace
  void parse_string(const std::string& s, const std::string& delims = " ;");
  void set(const std::string& name, const std::string& value);
  bool has(const std::string& name) const { return map_.count(name) != 0; }
  const Opt* find(const std::string& name) const;
  void print(FILE* f) const;
  std::vector<std::string> names() const;
  // options explicitly set by the user (not defaults)
  std::vector<std::pair<std::string, std::string>> user_values() const;

 private:
  void tokens_to_cmdline(const std::string& buffer);
  bool assign(Opt& o, const std::string& v);
  std::vector<std::unique_ptr<Opt>> opts_;
  std::map<std::string, Opt*> map_;
  int include_depth_ = 0;
  std::vector<std::string> config_dirs_;
};

// split helpers shared by config derivation
std::vector<std::string> split(const std::string& s, char d);
std::string trim(const std::string& s);
std::string strip_ws(const std::string& s);

}  // namespace asim
