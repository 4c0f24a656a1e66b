// glog-style logging for the operator binaries (stderr, level + timestamp + file-less).
#pragma once

#include <cstdarg>
#include <string>

namespace tfop {

extern int g_verbosity;  // -v=N

void log_at(char level, const char* fmt, va_list ap);
inline void log_info(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
inline void log_warn(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
inline void log_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
inline void log_v(int v, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

inline void log_info(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  log_at('I', fmt, ap);
  va_end(ap);
}
inline void log_warn(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  log_at('W', fmt, ap);
  va_end(ap);
}
inline void log_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  log_at('E', fmt, ap);
  va_end(ap);
}
inline void log_v(int v, const char* fmt, ...) {
  if (g_verbosity < v) return;
  va_list ap;
  va_start(ap, fmt);
  log_at('I', fmt, ap);
  va_end(ap);
}

}  // namespace tfop
