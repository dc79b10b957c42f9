// Test harness (CPU, g++): the device gaussian stream's arithmetic (legacy_gauss.hpp) compiled for
// the host, so tests/test_rng.py can pin it against np.log / np.random.RandomState bit for bit
// without a GPU.  Sequential MT19937 (numpy's mt19937_gen / mt19937_next order).  Not product code.
#include <stdint.h>

#include "../../theta-rrt_amd/csrc/legacy_gauss.hpp"

extern "C" {

void gc_log(const double* x, int64_t n, double* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = tr::legacy_log(x[i]);
}

// numpy state (key[624], pos, has_gauss, gauss) -> n gaussians; the state is advanced in place.
void gc_stream(uint32_t* key, int32_t* pos, int32_t* has, double* gauss, int64_t n, double* out) {
  auto next = [&]() -> uint32_t {
    if (*pos >= 624) {
      uint32_t nk[624];
      for (int i = 0; i < 624; ++i) {
        const uint32_t cur = key[i];
        const uint32_t nxt = i < 623 ? key[i + 1] : nk[0];
        const uint32_t far = i < 227 ? key[i + 397] : nk[i - 227];
        nk[i] = tr::mt_mix(cur, nxt, far);
      }
      for (int i = 0; i < 624; ++i) key[i] = nk[i];
      *pos = 0;
    }
    return tr::mt_temper(key[(*pos)++]);
  };
  for (int64_t j = 0; j < n; ++j) {
    if (*has) {
      out[j] = *gauss;
      *has = 0;
      *gauss = 0.0;
      continue;
    }
    double a, b;
    for (;;) {
      const uint32_t w0 = next(), w1 = next(), w2 = next(), w3 = next();
      if (tr::legacy_attempt(w0, w1, w2, w3, &a, &b)) break;
    }
    out[j] = a;
    *gauss = b;
    *has = 1;
  }
}
}
