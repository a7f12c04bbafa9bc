// hostcopy.hpp — host-side copy of JPEG byte ranges into the pinned staging buffer.
//
// The staging buffer is written once and then only read by the DMA engine, so a
// streaming (non-temporal) store is the right kind: it skips the read-for-ownership
// of every destination line that a cached store pays (~1/3 of the host memory traffic
// of a plain memcpy of lines not in cache) and keeps the copy from evicting the
// source ranges' neighbours.  Copies shorter than kStreamMin take memcpy.
#pragma once

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

namespace dino {

constexpr int64_t kStreamMin = 4096;

inline bool stream_copy_enabled() {
  static const bool on = [] {
    const char* e = getenv("DINO_GATHER_NT");
    return !(e && e[0] == '0');
  }();
  return on;
}

inline void stream_copy(uint8_t* dst, const uint8_t* src, int64_t n) {
  if (n < kStreamMin || !stream_copy_enabled()) {
    memcpy(dst, src, (size_t)n);
    return;
  }
  typedef long long v2i __attribute__((vector_size(16)));
  const int64_t head = (int64_t)((16 - ((uintptr_t)dst & 15)) & 15);
  memcpy(dst, src, (size_t)head);
  dst += head;
  src += head;
  n -= head;
  const int64_t nv = n >> 4;
  v2i* d = (v2i*)dst;
  int64_t k = 0;
  for (; k + 4 <= nv; k += 4) {
    v2i a, b, c, e;
    memcpy(&a, src + 16 * k, 16);
    memcpy(&b, src + 16 * k + 16, 16);
    memcpy(&c, src + 16 * k + 32, 16);
    memcpy(&e, src + 16 * k + 48, 16);
    __builtin_nontemporal_store(a, d + k);
    __builtin_nontemporal_store(b, d + k + 1);
    __builtin_nontemporal_store(c, d + k + 2);
    __builtin_nontemporal_store(e, d + k + 3);
  }
  for (; k < nv; ++k) {
    v2i a;
    memcpy(&a, src + 16 * k, 16);
    __builtin_nontemporal_store(a, d + k);
  }
  memcpy(dst + 16 * nv, src + 16 * nv, (size_t)(n & 15));
}

// Streaming stores are weakly ordered: fence before another thread (or the DMA
// engine, through a later runtime call) reads the buffer.
inline void stream_fence() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }

}  // namespace dino
