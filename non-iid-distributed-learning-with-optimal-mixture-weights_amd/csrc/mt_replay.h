// Bit-exact replay of torch.randperm(n, generator=g) after g.manual_seed(seed) on the CPU
// (torch 2.10): MT19937 seeded with (uint32)seed, then a forward Fisher-Yates taking
// z = mt() % (n - k).  This is the permutation of every shuffled
// DataLoader pass of the reference (/root/reference/functions/tools.py:179, 220;
// /root/reference/exp.py:99).  Host code (g++ / hipcc host side).
#pragma once

#include <cstdint>
#include <utility>

namespace fs {

struct MT19937 {
  uint32_t s[624];
  int i;
  explicit MT19937(uint32_t x) {
    s[0] = x;
    for (int k = 1; k < 624; ++k) {
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)k;
      s[k] = x;
    }
    i = 624;
  }
  void twist() {
    int k = 0;
    for (; k < 227; ++k) {
      const uint32_t y = (s[k] & 0x80000000u) | (s[k + 1] & 0x7fffffffu);
      s[k] = s[k + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    for (; k < 623; ++k) {
      const uint32_t y = (s[k] & 0x80000000u) | (s[k + 1] & 0x7fffffffu);
      s[k] = s[k - 227] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    const uint32_t y = (s[623] & 0x80000000u) | (s[0] & 0x7fffffffu);
    s[623] = s[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    i = 0;
  }
  inline uint32_t operator()() {
    if (i >= 624) twist();
    uint32_t y = s[i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
};

// r % m for 32-bit r, m >= 1, via a double quotient and a one-step correction (exact)
inline uint32_t mod_u32(uint32_t r, uint32_t m) {
  const int64_t q = (int64_t)((double)r / (double)m);
  int64_t rem = (int64_t)r - q * (int64_t)m;
  rem += rem < 0 ? (int64_t)m : 0;
  rem -= rem >= (int64_t)m ? (int64_t)m : 0;
  return (uint32_t)rem;
}

inline void replay_randperm(uint64_t seed, int64_t n, int32_t* out) {
  for (int64_t k = 0; k < n; ++k) out[k] = (int32_t)k;
  MT19937 g((uint32_t)seed);
  for (int64_t k = 0; k + 1 < n; ++k) {
    const int64_t z = (int64_t)mod_u32(g(), (uint32_t)(n - k));
    std::swap(out[k], out[k + z]);
  }
}

}  // namespace fs
