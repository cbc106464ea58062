// mythgpu_jitd: the JIT compiler in its own process (jit.cpp, "The compiler in its own process").
// Reads compile requests on fd 0 and answers on fd 1 (both ends of one socket), until end of
// input.  Each request carries the caller's AMD_COMGR_* / MYTHGPU_JIT* environment of the moment,
// applied here before compiling, so per-call settings (AMD_COMGR_CACHE, MYTHGPU_JIT_DUMP, …) behave
// as they did in-process.  An LLVM fatal error aborts this process only; the engine sees the
// socket close and keeps searching on the interpreter.
//
// MYTHGPU_JITD_FAULT=abort in a request's environment makes this process abort() on it: the
// test hook for that path (tests/test_gpu_jit_isolation.py).
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "jit.hpp"

namespace {

bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = read(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

extern "C" char** environ;

// make this process's AMD_COMGR_* / MYTHGPU_JIT* variables exactly the caller's
void apply_env(const std::string& env) {
  std::vector<std::string> mine;
  for (char** e = environ; e && *e; e++)
    if (!std::strncmp(*e, "AMD_COMGR_", 10) || !std::strncmp(*e, "MYTHGPU_JIT", 11)) {
      const char* eq = std::strchr(*e, '=');
      if (eq) mine.emplace_back(*e, eq - *e);
    }
  for (const auto& n : mine) unsetenv(n.c_str());
  size_t i = 0;
  while (i < env.size()) {
    const size_t end = env.find('\0', i);
    const std::string kv = env.substr(i, end == std::string::npos ? std::string::npos : end - i);
    const size_t eq = kv.find('=');
    if (eq != std::string::npos) setenv(kv.substr(0, eq).c_str(), kv.c_str() + eq + 1, 1);
    if (end == std::string::npos) break;
    i = end + 1;
  }
}

}  // namespace

int main() {
  for (;;) {
    uint64_t el = 0, sl = 0;
    if (!read_all(0, &el, 8) || el > (1u << 20)) return 0;
    std::string env(el, '\0');
    if (!read_all(0, &env[0], el) || !read_all(0, &sl, 8) || sl > (1ull << 30)) return 0;
    std::string src(sl, '\0');
    if (!read_all(0, &src[0], sl)) return 0;
    apply_env(env);
    // the first tier's assembly: comgr's on-disk cache costs more than the assembler it would skip
    // (the first write of an entry ~10 ms on the box against ~4 ms of assembly); off for it
    if (src.compare(0, std::strlen(mg::kAsmMarker), mg::kAsmMarker) == 0) setenv("AMD_COMGR_CACHE", "0", 1);
    if (const char* f = getenv("MYTHGPU_JITD_FAULT"))
      if (!std::strcmp(f, "abort")) abort();
    std::vector<char> code;
    std::string log;
    const int32_t rc = mg::jit_compile_local(src, code, log);
    const uint64_t cl = rc == 0 ? code.size() : 0, ll = log.size();
    if (!write_all(1, &rc, 4) || !write_all(1, &cl, 8) || !write_all(1, code.data(), cl) || !write_all(1, &ll, 8) ||
        !write_all(1, log.data(), ll))
      return 0;
  }
}
