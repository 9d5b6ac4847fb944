#include "options.h"

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace asim {

std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == d) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(" \t\r\n");
  return s.substr(b, e - b + 1);
}

std::string strip_ws(const std::string& s) {
  std::string o;
  for (char c : s)
    if (c != ' ' && c != '\t' && c != '\n' && c != '\r') o.push_back(c);
  return o;
}

void OptionRegistry::reg(const std::string& name, OptType t, void* dst, const std::string& help,
                         const std::string& deflt) {
  if (map_.count(name)) {
    // re-registration (the reference registers -gpgpu_shmem_warp_parts twice):
    // keep the first destination, update the default
    return;
  }
  auto o = std::make_unique<Opt>();
  o->name = name;
  o->type = t;
  o->dst = dst;
  o->help = help;
  o->deflt = deflt;
  Opt* p = o.get();
  opts_.push_back(std::move(o));
  map_[name] = p;
  if (!assign(*p, deflt)) throw OptionError("bad default '" + deflt + "' for option " + name);
  p->parsed = false;
}

static bool parse_int64(const std::string& v, long long& out) {
  std::string s = trim(v);
  if (s.empty()) return false;
  errno = 0;
  char* end = nullptr;
  long long x = strtoll(s.c_str(), &end, 0);
  if (errno || end == s.c_str() || *end) return false;
  out = x;
  return true;
}
static bool parse_uint64(const std::string& v, unsigned long long& out) {
  std::string s = trim(v);
  if (s.empty() || s[0] == '-') return false;
  errno = 0;
  char* end = nullptr;
  unsigned long long x = strtoull(s.c_str(), &end, 0);
  if (errno || end == s.c_str() || *end) return false;
  out = x;
  return true;
}

bool OptionRegistry::assign(Opt& o, const std::string& v) {
  if (!o.dst) {
    switch (o.type) {
      case OptType::Bool:
      case OptType::Int32:
      case OptType::Int64: {
        long long x;
        if (!parse_int64(v, x)) return false;
        if (o.type == OptType::Bool && x != 0 && x != 1) return false;
        o.iv = x;
        o.uv = (unsigned long long)x;
        o.dv = (double)x;
        break;
      }
      case OptType::UInt32:
      case OptType::UInt64: {
        unsigned long long x;
        if (!parse_uint64(v, x)) return false;
        o.uv = x;
        o.iv = (long long)x;
        o.dv = (double)x;
        break;
      }
      case OptType::Float:
      case OptType::Double: {
        std::string s = trim(v);
        char* end = nullptr;
        if (s.empty()) return false;
        double x = strtod(s.c_str(), &end);
        if (end == s.c_str() || *end) return false;
        o.dv = x;
        o.iv = (long long)x;
        break;
      }
      case OptType::Str:
        o.sv = v;
        break;
    }
    o.value = v;
    o.parsed = true;
    return true;
  }
  switch (o.type) {
    case OptType::Bool: {
      long long x;
      if (!parse_int64(v, x) || (x != 0 && x != 1)) return false;
      *static_cast<bool*>(o.dst) = x != 0;
      break;
    }
    case OptType::Int32: {
      long long x;
      if (!parse_int64(v, x)) return false;
      *static_cast<int32_t*>(o.dst) = (int32_t)x;
      break;
    }
    case OptType::UInt32: {
      unsigned long long x;
      if (!parse_uint64(v, x)) return false;
      *static_cast<uint32_t*>(o.dst) = (uint32_t)x;
      break;
    }
    case OptType::Int64: {
      long long x;
      if (!parse_int64(v, x)) return false;
      *static_cast<int64_t*>(o.dst) = (int64_t)x;
      break;
    }
    case OptType::UInt64: {
      unsigned long long x;
      if (!parse_uint64(v, x)) return false;
      *static_cast<uint64_t*>(o.dst) = (uint64_t)x;
      break;
    }
    case OptType::Float:
    case OptType::Double: {
      std::string s = trim(v);
      if (s.empty()) return false;
      char* end = nullptr;
      double x = strtod(s.c_str(), &end);
      if (end == s.c_str() || *end) return false;
      if (o.type == OptType::Float)
        *static_cast<float*>(o.dst) = (float)x;
      else
        *static_cast<double*>(o.dst) = x;
      break;
    }
    case OptType::Str:
      *static_cast<std::string*>(o.dst) = v;
      break;
  }
  o.value = v;
  o.parsed = true;
  return true;
}

void OptionRegistry::set(const std::string& name, const std::string& value) {
  auto it = map_.find(name);
  if (it == map_.end()) throw OptionError("Unknown Option: '" + name + "'");
  if (!assign(*it->second, value))
    throw OptionError("Cannot parse value '" + value + "' for option '" + name + "'");
}

static const OptionRegistry::Opt& must(const std::map<std::string, OptionRegistry::Opt*>& m,
                                      const std::string& n) {
  auto it = m.find(n);
  if (it == m.end()) throw OptionError("option not registered: " + n);
  return *it->second;
}
long long OptionRegistry::geti(const std::string& n) const {
  const Opt& o = must(map_, n);
  if (!o.dst) return o.iv;
  switch (o.type) {
    case OptType::Bool: return *static_cast<bool*>(o.dst);
    case OptType::Int32: return *static_cast<int32_t*>(o.dst);
    case OptType::UInt32: return *static_cast<uint32_t*>(o.dst);
    case OptType::Int64: return *static_cast<int64_t*>(o.dst);
    case OptType::UInt64: return (long long)*static_cast<uint64_t*>(o.dst);
    case OptType::Float: return (long long)*static_cast<float*>(o.dst);
    case OptType::Double: return (long long)*static_cast<double*>(o.dst);
    default: throw OptionError("option is a string: " + n);
  }
}
unsigned long long OptionRegistry::getu(const std::string& n) const {
  const Opt& o = must(map_, n);
  if (!o.dst) return o.uv;
  return (unsigned long long)geti(n);
}
double OptionRegistry::getd(const std::string& n) const {
  const Opt& o = must(map_, n);
  if (!o.dst) return o.dv;
  if (o.type == OptType::Float) return *static_cast<float*>(o.dst);
  if (o.type == OptType::Double) return *static_cast<double*>(o.dst);
  return (double)geti(n);
}
std::string OptionRegistry::gets(const std::string& n) const {
  const Opt& o = must(map_, n);
  if (!o.dst) return o.type == OptType::Str ? o.sv : o.value;
  if (o.type == OptType::Str) return *static_cast<std::string*>(o.dst);
  return o.value;
}

const OptionRegistry::Opt* OptionRegistry::find(const std::string& name) const {
  auto it = map_.find(name);
  return it == map_.end() ? nullptr : it->second;
}

void OptionRegistry::parse_cmdline(const std::vector<std::string>& argv, bool skip_first) {
  for (size_t i = skip_first ? 1 : 0; i < argv.size(); ++i) {
    const std::string& a = argv[i];
    auto it = map_.find(a);
    if (it != map_.end()) {
      Opt& o = *it->second;
      std::string next = (i + 1 < argv.size()) ? argv[i + 1] : "";
      if (o.type == OptType::Bool) {
        // optional value
        long long x;
        if (parse_int64(next, x) && (x == 0 || x == 1)) {
          assign(o, next);
          ++i;
        } else {
          assign(o, "1");
        }
      } else {
        if (i + 1 >= argv.size()) throw OptionError("Missing value for option '" + a + "'");
        if (!assign(o, next)) throw OptionError("Cannot parse value '" + next + "' for option '" + a + "'");
        ++i;
      }
    } else if (a == "-config") {
      if (i + 1 >= argv.size()) throw OptionError("Missing filename for option '-config'");
      parse_file(argv[i + 1]);
      ++i;
    } else {
      throw OptionError("Unknown Option: '" + a + "'");
    }
  }
}

void OptionRegistry::tokens_to_cmdline(const std::string& buffer) {
  std::istringstream in(buffer);
  std::vector<std::string> argv;
  std::string tok;
  while (in >> tok) {
    if (!tok.empty() && tok[0] == '"') {
      std::string acc = tok;
      while ((acc.size() < 2 || acc.back() != '"') && (in >> tok)) acc += " " + tok;
      if (acc.size() >= 2 && acc.back() == '"')
        acc = acc.substr(1, acc.size() - 2);
      else
        acc = acc.substr(1);
      argv.push_back(acc);
    } else {
      argv.push_back(tok);
    }
  }
  parse_cmdline(argv, false);
}

void OptionRegistry::parse_file(const std::string& path) {
  std::ifstream f(path);
  if (!f.good()) throw OptionError("Cannot open config file '" + path + "'");
  if (++include_depth_ > 32) throw OptionError("-config include depth exceeded at '" + path + "'");
  {
    const size_t sl = path.find_last_of('/');
    config_dirs_.push_back(sl == std::string::npos ? std::string(".") : path.substr(0, sl));
  }
  std::string line, buf;
  while (std::getline(f, line)) {
    size_t h = line.find('#');
    if (h != std::string::npos) line.erase(h);
    buf += line;
    buf += ' ';
  }
  tokens_to_cmdline(buf);
  --include_depth_;
}

void OptionRegistry::parse_string(const std::string& s, const std::string& delims) {
  std::string t = s;
  for (auto& ch : t)
    if (delims.find(ch) != std::string::npos) ch = ' ';
  tokens_to_cmdline(t);
}

void OptionRegistry::print(FILE* f) const {
  for (auto& o : opts_) fprintf(f, "%-50s %-20s # %s\n", o->name.c_str(), o->value.c_str(), o->help.c_str());
}

std::vector<std::string> OptionRegistry::names() const {
  std::vector<std::string> n;
  for (auto& o : opts_) n.push_back(o->name);
  return n;
}

std::vector<std::pair<std::string, std::string>> OptionRegistry::user_values() const {
  std::vector<std::pair<std::string, std::string>> v;
  for (auto& o : opts_)
    if (o->parsed) v.emplace_back(o->name, o->value);
  return v;
}

}  // namespace asim
