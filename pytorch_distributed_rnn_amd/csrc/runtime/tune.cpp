// PDRNN_TUNE: the one environment variable that carries every kernel-map /
// tiling override used for A/B sweeps and for the tests that force a path
// ("key=value,key=value", e.g. PDRNN_TUNE=sw_mode=2,sw_bwd_mode=3).  Read on
// every call (tests flip it in-process); keys are documented in README.md
// (tuning overrides).  Unknown keys are ignored.
#include "pdrnn/api.h"

#include <cstdlib>
#include <cstring>

extern "C" int pdrnn_tune_str(const char* key, char* out, int out_len) {
  const char* e = std::getenv("PDRNN_TUNE");
  if (!e || !*e || !key || !*key) return 0;
  const size_t kl = std::strlen(key);
  for (const char* p = e; *p;) {
    while (*p == ',' || *p == ' ') ++p;
    const char* end = p;
    while (*end && *end != ',') ++end;
    const char* eq = static_cast<const char*>(std::memchr(p, '=', (size_t)(end - p)));
    if (eq && (size_t)(eq - p) == kl && std::strncmp(p, key, kl) == 0) {
      const int n = (int)(end - eq - 1);
      if (out && out_len > 0) {
        const int c = n < out_len - 1 ? n : out_len - 1;
        std::memcpy(out, eq + 1, (size_t)c);
        out[c] = 0;
      }
      return 1;
    }
    p = end;
  }
  return 0;
}

extern "C" int pdrnn_tune_int(const char* key, int dflt) {
  char buf[32];
  if (!pdrnn_tune_str(key, buf, (int)sizeof(buf)) || !buf[0]) return dflt;
  char* endp = nullptr;
  const long v = std::strtol(buf, &endp, 10);
  return (endp && *endp == 0) ? (int)v : dflt;
}
