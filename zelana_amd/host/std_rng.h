// std_rng.h — rand 0.8 StdRng (ChaCha12, rand_chacha 0.3.1) seeded by
// rand_core 0.6.4 seed_from_u64 (PCG32 expansion), and ark-ff 0.5 Fp::rand
// for Fr: what Groth16Prover::prove draws r and s from
// (core/src/sequencer/settlement/prover.rs:354).
#pragma once
#include <stdint.h>

#include "fr.h"

namespace zp {

class StdRng {
 public:
  static StdRng seed_from_u64(uint64_t state) {
    StdRng r;
    const uint64_t mul = 6364136223846793005ULL, inc = 11634580027462260723ULL;
    for (int i = 0; i < 8; i++) {
      state = state * mul + inc;
      uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
      uint32_t rot = (uint32_t)(state >> 59);
      r.key_[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
    }
    return r;
  }
  uint32_t next_u32() {
    if (pos_ == 16) block();
    return buf_[pos_++];
  }
  uint64_t next_u64() {
    uint64_t lo = next_u32();
    return lo | ((uint64_t)next_u32() << 32);
  }
  // Fp::rand: 4 limbs, top masked to 254 bits, rejected if >= r; the limbs
  // are the MONTGOMERY representation (value = limbs * 2^-256 mod r)
  Fr fr_rand() {
    for (;;) {
      Fr x;
      for (int i = 0; i < 4; i++) x.l[i] = next_u64();
      x.l[3] &= (1ULL << 62) - 1;
      if (!Fr::geq_p(x.l)) return x;
    }
  }

 private:
  static uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
  static void qr(uint32_t* s, int a, int b, int c, int d) {
    s[a] += s[b];
    s[d] = rotl(s[d] ^ s[a], 16);
    s[c] += s[d];
    s[b] = rotl(s[b] ^ s[c], 12);
    s[a] += s[b];
    s[d] = rotl(s[d] ^ s[a], 8);
    s[c] += s[d];
    s[b] = rotl(s[b] ^ s[c], 7);
  }
  void block() {
    uint32_t in[16] = {0x61707865, 0x3320646E, 0x79622D32, 0x6B206574};
    for (int i = 0; i < 8; i++) in[4 + i] = key_[i];
    in[12] = (uint32_t)counter_;
    in[13] = (uint32_t)(counter_ >> 32);
    in[14] = in[15] = 0;
    uint32_t x[16];
    for (int i = 0; i < 16; i++) x[i] = in[i];
    for (int r = 0; r < 6; r++) {  // 12 rounds
      qr(x, 0, 4, 8, 12), qr(x, 1, 5, 9, 13), qr(x, 2, 6, 10, 14), qr(x, 3, 7, 11, 15);
      qr(x, 0, 5, 10, 15), qr(x, 1, 6, 11, 12), qr(x, 2, 7, 8, 13), qr(x, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; i++) buf_[i] = x[i] + in[i];
    counter_++;
    pos_ = 0;
  }
  uint32_t key_[8] = {0};
  uint64_t counter_ = 0;
  uint32_t buf_[16] = {0};
  int pos_ = 16;
};

}  // namespace zp
