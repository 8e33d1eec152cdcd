#include "common.h"

#include <ctime>
#include <iostream>

namespace dmlc {
namespace ctl {

std::string format_time_us(int64_t us) {
  time_t secs = (time_t)(us / 1000000);
  struct tm tmv;
  localtime_r(&secs, &tmv);
  char buf[64];
  strftime(buf, sizeof(buf), "%Y-%m-%d %H:%M:%S", &tmv);
  char out[96];
  snprintf(out, sizeof(out), "%s.%06lld", buf, (long long)(us % 1000000));
  return out;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> out;
  std::istringstream is(s);
  std::string t;
  while (is >> t) out.push_back(t);
  return out;
}

std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(" \t\r\n");
  return s.substr(b, e - b + 1);
}

bool starts_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(0, p.size(), p) == 0;
}

Logger& Logger::get() {
  static Logger l;
  return l;
}

void Logger::open(const std::string& path) {
  std::lock_guard<std::mutex> g(mu_);
  if (f_) fclose(f_);
  f_ = fopen(path.c_str(), "a");
}

void Logger::log(const char* level, const std::string& msg) {
  std::lock_guard<std::mutex> g(mu_);
  if (!f_) return;
  fprintf(f_, "%s [%s] %s\n", format_time_us(wall_us()).c_str(), level, msg.c_str());
  fflush(f_);
}

void Logger::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (f_) fclose(f_);
  f_ = nullptr;
}

static std::mutex g_out_mu;

void out_line(const std::string& s) {
  std::lock_guard<std::mutex> g(g_out_mu);
  std::cout << s << std::endl;
}

}  // namespace ctl
}  // namespace dmlc
