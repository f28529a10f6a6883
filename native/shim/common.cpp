#include "common.h"

#include <ctype.h>
#include <pthread.h>
#include <stdarg.h>

namespace vgpu {

static int g_log_level = -1;

int log_level() {
  int lv = __atomic_load_n(&g_log_level, __ATOMIC_RELAXED);
  if (lv >= 0) return lv;
  const char* v = env_first("VGPU_LOG_LEVEL", "LIBCUDA_LOG_LEVEL");
  lv = v ? atoi(v) : kMsg;
  if (lv < 0) lv = 0;
  __atomic_store_n(&g_log_level, lv, __ATOMIC_RELAXED);
  return lv;
}

void log_write(int level, const char* file, int line, const char* fmt, ...) {
  static const char* names[] = {"ERROR", "Warn", "Msg", "Info", "Debug"};
  if (level < 0) level = 0;
  if (level > 4) level = 4;
  const char* base = strrchr(file, '/');
  base = base ? base + 1 : file;
  char buf[1024];
  int n = snprintf(buf, sizeof(buf), "[vgpu %s (pid:%d tid:%ld %s:%d)]: ", names[level],
                   (int)getpid(), (long)syscall(SYS_gettid), base, line);
  va_list ap;
  va_start(ap, fmt);
  if (n < (int)sizeof(buf)) n += vsnprintf(buf + n, sizeof(buf) - n, fmt, ap);
  va_end(ap);
  if (n >= (int)sizeof(buf) - 1) n = (int)sizeof(buf) - 2;
  if (n > 0 && buf[n - 1] != '\n') buf[n++] = '\n';
  ssize_t w = write(2, buf, (size_t)n);
  (void)w;
}

const char* env_first(const char* a, const char* b, const char* c) {
  const char* names[3] = {a, b, c};
  for (const char* n : names) {
    if (!n) continue;
    const char* v = getenv(n);
    if (v && *v) return v;
  }
  return nullptr;
}

bool env_bool(const char* v, bool dflt) {
  if (!v) return dflt;
  if (!strcasecmp(v, "1") || !strcasecmp(v, "true") || !strcasecmp(v, "yes") ||
      !strcasecmp(v, "on"))
    return true;
  if (!strcasecmp(v, "0") || !strcasecmp(v, "false") || !strcasecmp(v, "no") ||
      !strcasecmp(v, "off"))
    return false;
  return dflt;
}

uint64_t parse_mem(const char* s) {
  if (!s) return 0;
  while (isspace((unsigned char)*s)) ++s;
  if (!*s) return 0;
  char* end = nullptr;
  double v = strtod(s, &end);
  if (end == s || v < 0) return 0;
  while (end && isspace((unsigned char)*end)) ++end;
  uint64_t mul = 1;
  if (end && *end) {
    switch (tolower((unsigned char)*end)) {
      case 'b': mul = 1; break;
      case 'k': mul = 1ull << 10; break;
      case 'm': mul = 1ull << 20; break;
      case 'g': mul = 1ull << 30; break;
      case 't': mul = 1ull << 40; break;
      default: return 0;
    }
  }
  return (uint64_t)(v * (double)mul);
}

int parse_cu_mask(const char* s, uint64_t* out, int words) {
  for (int i = 0; i < words; ++i) out[i] = 0;
  if (!s) return -1;
  while (isspace((unsigned char)*s)) ++s;
  if (s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) s += 2;
  // Collect hex digits (separators ',' '_' ':' ignored); last digit = bits 0..3.
  size_t len = strlen(s);
  int bit = 0;
  for (size_t k = len; k-- > 0;) {
    char ch = s[k];
    if (ch == ',' || ch == '_' || ch == ':' || isspace((unsigned char)ch)) continue;
    int d;
    if (ch >= '0' && ch <= '9') d = ch - '0';
    else if (ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
    else if (ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
    else return -1;
    for (int b = 0; b < 4; ++b, ++bit) {
      if ((d >> b) & 1) {
        if (bit >= words * 64) return -1;
        out[bit / 64] |= 1ull << (bit % 64);
      }
    }
  }
  int n = 0;
  for (int i = 0; i < words; ++i) n += __builtin_popcountll(out[i]);
  return n;
}

std::string format_cu_mask(const uint64_t* in, int words) {
  std::string s = "0x";
  bool lead = true;
  for (int i = words - 1; i >= 0; --i) {
    char buf[17];
    snprintf(buf, sizeof(buf), "%016llx", (unsigned long long)in[i]);
    if (lead) {
      if (in[i] == 0 && i > 0) continue;
      // trim leading zeros of the most significant printed word
      const char* p = buf;
      while (*p == '0' && p[1]) ++p;
      s += p;
      lead = false;
    } else {
      s += buf;
    }
  }
  return s;
}

}  // namespace vgpu
