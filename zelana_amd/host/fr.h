// fr.h — host BN254 scalar field Fr (4 x 64-bit Montgomery, R = 2^256) for the
// C++ host mirror of the reference's prover (circuit synthesis, StdRng
// sampling).  ark-ff 0.5 semantics where they are observable: canonical
// little-endian limbs, from_le_bytes_mod_order, Fp::rand's Montgomery-limb
// sampling (std_rng.h).
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>

namespace zp {

typedef unsigned __int128 u128;

struct Fr {
  uint64_t l[4] = {0, 0, 0, 0};  // Montgomery form

  static constexpr uint64_t P[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                    0x30644e72e131a029ULL};
  static constexpr uint64_t INV = 0xc2e1f593efffffffULL;  // -r^-1 mod 2^64
  static constexpr uint64_t R2[4] = {0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL, 0x8c49833d53bb8085ULL,
                                     0x0216d0b17f4e44a5ULL};

  static bool geq_p(const uint64_t a[4]) {
    for (int i = 3; i >= 0; i--)
      if (a[i] != P[i]) return a[i] > P[i];
    return true;
  }
  static void sub_p(uint64_t a[4]) {
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
      u128 d = (u128)a[i] - P[i] - br;
      a[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
  }
  // Montgomery product (CIOS; r < 2^254 leaves room for the running value)
  static Fr mont(const uint64_t a[4], const uint64_t b[4]) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
      uint64_t c = 0;
      for (int j = 0; j < 4; j++) {
        u128 x = (u128)a[j] * b[i] + t[j] + c;
        t[j] = (uint64_t)x;
        c = (uint64_t)(x >> 64);
      }
      u128 s = (u128)t[4] + c;
      t[4] = (uint64_t)s;
      t[5] = (uint64_t)(s >> 64);
      uint64_t m = t[0] * INV;
      u128 x = (u128)m * P[0] + t[0];
      c = (uint64_t)(x >> 64);
      for (int j = 1; j < 4; j++) {
        x = (u128)m * P[j] + t[j] + c;
        t[j - 1] = (uint64_t)x;
        c = (uint64_t)(x >> 64);
      }
      s = (u128)t[4] + c;
      t[3] = (uint64_t)s;
      t[4] = t[5] + (uint64_t)(s >> 64);
    }
    Fr r;
    memcpy(r.l, t, 32);
    if (t[4] || geq_p(r.l)) sub_p(r.l);
    return r;
  }

  static Fr zero() { return Fr(); }
  static Fr one() { return from_u64(1); }
  static Fr from_canon(const uint64_t c[4]) {  // c < r
    return mont(c, R2);
  }
  static Fr from_u64(uint64_t v) {
    const uint64_t c[4] = {v, 0, 0, 0};
    return from_canon(c);
  }
  // Fr::from_le_bytes_mod_order (any length): sum of 31-byte chunks * 2^(248 k)
  static Fr from_le_bytes_mod_order(const uint8_t* b, size_t n) {
    Fr acc = zero(), mult = one();
    const Fr base = pow2_248();
    for (size_t lo = 0; lo < n; lo += 31) {
      const size_t hi = lo + 31 < n ? lo + 31 : n;
      uint64_t c[4] = {0, 0, 0, 0};
      for (size_t k = lo; k < hi; k++) c[(k - lo) / 8] |= (uint64_t)b[k] << (8 * ((k - lo) % 8));
      acc = acc + from_canon(c) * mult;
      mult = mult * base;
    }
    return acc;
  }
  static Fr pow2_248() {
    const uint64_t c[4] = {0, 0, 0, 1ULL << 56};
    return from_canon(c);
  }
  void to_canon(uint64_t out[4]) const {
    const uint64_t one_[4] = {1, 0, 0, 0};
    Fr c = mont(l, one_);
    memcpy(out, c.l, 32);
  }
  bool is_zero() const { return (l[0] | l[1] | l[2] | l[3]) == 0; }
  bool operator==(const Fr& o) const { return memcmp(l, o.l, 32) == 0; }
  bool operator!=(const Fr& o) const { return !(*this == o); }
  Fr operator+(const Fr& o) const {
    Fr r;
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)l[i] + o.l[i] + c;
      r.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    if (c || geq_p(r.l)) sub_p(r.l);
    return r;
  }
  Fr operator-() const {
    if (is_zero()) return *this;
    Fr r;
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
      u128 d = (u128)P[i] - l[i] - br;
      r.l[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
    return r;
  }
  Fr operator-(const Fr& o) const { return *this + (-o); }
  Fr operator*(const Fr& o) const { return mont(l, o.l); }
  Fr pow(const uint64_t e[4]) const {
    Fr r = one(), b = *this;
    for (int i = 0; i < 256; i++) {
      if ((e[i / 64] >> (i % 64)) & 1) r = r * b;
      b = b * b;
    }
    return r;
  }
  Fr pow_u64(uint64_t e) const {
    const uint64_t x[4] = {e, 0, 0, 0};
    return pow(x);
  }
  Fr inverse() const {  // a^(r-2); zero maps to zero
    const uint64_t e[4] = {P[0] - 2, P[1], P[2], P[3]};
    return pow(e);
  }
  // bit i of the canonical value
  bool bit(int i) const {
    uint64_t c[4];
    to_canon(c);
    return (c[i / 64] >> (i % 64)) & 1;
  }
};

}  // namespace zp
