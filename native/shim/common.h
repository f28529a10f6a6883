// Shared helpers for the in-container enforcement library (libvgpu.so):
// logging, environment parsing and clocks.
//
// Reference parity: the closed-source libvgpu.so logs with the prefix
// "[4pdvGPU Debug/Info/Msg/Warn/ERROR (pid:tid:file:line)]" gated by
// LIBCUDA_LOG_LEVEL.  Ours is VGPU_LOG_LEVEL with the
// same five levels (0 error .. 4 debug); LIBCUDA_LOG_LEVEL is honoured as an alias.
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <string>

namespace vgpu {

enum LogLevel { kError = 0, kWarn = 1, kMsg = 2, kInfo = 3, kDebug = 4 };

int log_level();
void log_write(int level, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 4, 5)));

#define VGPU_LOG(level, ...)                                                 \
  do {                                                                       \
    if ((level) <= ::vgpu::log_level()) ::vgpu::log_write((level), __FILE__, \
                                                           __LINE__, __VA_ARGS__); \
  } while (0)
#define VLOG_ERR(...) VGPU_LOG(::vgpu::kError, __VA_ARGS__)
#define VLOG_WARN(...) VGPU_LOG(::vgpu::kWarn, __VA_ARGS__)
#define VLOG_MSG(...) VGPU_LOG(::vgpu::kMsg, __VA_ARGS__)
#define VLOG_INFO(...) VGPU_LOG(::vgpu::kInfo, __VA_ARGS__)
#define VLOG_DEBUG(...) VGPU_LOG(::vgpu::kDebug, __VA_ARGS__)

inline uint64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
inline uint64_t real_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
inline void sleep_ns(uint64_t ns) {
  struct timespec ts;
  ts.tv_sec = (time_t)(ns / 1000000000ull);
  ts.tv_nsec = (long)(ns % 1000000000ull);
  nanosleep(&ts, nullptr);
}

// Environment lookups. `names` are tried in order; the first one set wins.
const char* env_first(const char* a, const char* b = nullptr, const char* c = nullptr);
bool env_bool(const char* v, bool dflt);

// Parse a memory quantity.  Accepts "<n>", "<n>b", "<n>k", "<n>m", "<n>g"
// (binary multiples; the reference's device-plugin writes "<MiB>m",
// pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:339).
// Returns 0 on empty/invalid input.
uint64_t parse_mem(const char* s);

// Parse a hex CU mask ("0xffff0000..." or "ffff,0000"-style 64-bit words,
// least-significant word LAST as in HSA_CU_MASK / sysfs masks) into
// `words` little-endian 64-bit words. Returns number of set bits, -1 on error.
int parse_cu_mask(const char* s, uint64_t* out, int words);
std::string format_cu_mask(const uint64_t* in, int words);

}  // namespace vgpu
