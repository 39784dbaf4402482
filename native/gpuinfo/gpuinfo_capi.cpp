// C ABI over the gpuinfo core (ctypes fallback for Python, and for non-Python
// consumers). Returns the number of bytes needed (excluding NUL); writes at
// most `len` bytes.
#include <cstring>

#include "gpuinfo.h"

extern "C" __attribute__((visibility("default"))) long kgs_gpuinfo_discover_json(const char* root, int use_amdsmi,
                                                                                  char* buf, long len) {
  auto t = kgs::gpuinfo::discover(root ? root : "/", use_amdsmi != 0);
  std::string s = kgs::gpuinfo::to_json(t);
  if (buf && len > 0) {
    long n = (long)s.size() < len - 1 ? (long)s.size() : len - 1;
    std::memcpy(buf, s.data(), (size_t)n);
    buf[n] = '\0';
  }
  return (long)s.size();
}
