#include "log.h"

#include <sys/time.h>
#include <unistd.h>

#include <cstdio>
#include <ctime>
#include <mutex>

namespace tfop {

int g_verbosity = 0;
bool g_quiet = false;
static std::mutex g_log_mu;

void log_at(char level, const char* fmt, va_list ap) {
  if (g_quiet && level == 'I') return;
  char msg[4096];
  vsnprintf(msg, sizeof msg, fmt, ap);
  timeval tv;
  gettimeofday(&tv, nullptr);
  std::tm tm;
  localtime_r(&tv.tv_sec, &tm);
  std::lock_guard<std::mutex> g(g_log_mu);
  fprintf(stderr, "%c%02d%02d %02d:%02d:%02d.%06ld %d] %s\n", level, tm.tm_mon + 1, tm.tm_mday, tm.tm_hour, tm.tm_min,
          tm.tm_sec, (long)tv.tv_usec, (int)getpid(), msg);
}

}  // namespace tfop
