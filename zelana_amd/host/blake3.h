// blake3.h — BLAKE3 hash mode, 32-byte output, for the host mirror:
// Groth16Prover::compute_vk_hash (prover.rs:289-294: blake3 of the compressed
// VK), MockProver (prover.rs:179-245) and compute_batch_hash (:525-558).  The
// blake3 crate is a third-party dependency absent here; this restates the
// published algorithm (chunks of 1024 B, 64-B blocks, binary chunk tree whose
// left subtree holds the largest power of two of chunks).
#pragma once
#include <stdint.h>
#include <string.h>

#include <array>
#include <vector>

namespace zp {

class Blake3 {
 public:
  void update(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    buf_.insert(buf_.end(), p, p + n);
  }
  std::array<uint8_t, 32> finalize() const {
    const size_t n = buf_.size();
    const size_t nchunks = n == 0 ? 1 : (n + 1023) / 1024;
    std::array<uint32_t, 8> cv;
    if (nchunks == 1) {
      cv = chunk_cv(buf_.data(), n, 0, true);
    } else {
      std::vector<std::array<uint32_t, 8>> cvs(nchunks);
      for (size_t i = 0; i < nchunks; i++)
        cvs[i] = chunk_cv(buf_.data() + i * 1024, std::min<size_t>(1024, n - i * 1024), i, false);
      cv = merge(cvs, 0, nchunks, true);
    }
    std::array<uint8_t, 32> out;
    for (int i = 0; i < 8; i++)
      for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(cv[i] >> (8 * b));
    return out;
  }
  static std::array<uint8_t, 32> hash(const void* data, size_t n) {
    Blake3 h;
    h.update(data, n);
    return h.finalize();
  }

 private:
  static constexpr uint32_t IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                     0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
  enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
  static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  static void g(uint32_t* s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    s[a] = s[a] + s[b] + x;
    s[d] = rotr(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + y;
    s[d] = rotr(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];
    s[b] = rotr(s[b] ^ s[c], 7);
  }
  static std::array<uint32_t, 8> compress(const uint32_t cv[8], const uint32_t mw[16], uint64_t counter,
                                          uint32_t len, uint32_t flags) {
    static const int PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
    uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7], IV[0], IV[1], IV[2], IV[3],
                      (uint32_t)counter, (uint32_t)(counter >> 32), len, flags};
    uint32_t m[16], t[16];
    memcpy(m, mw, 64);
    for (int r = 0; r < 7; r++) {
      g(s, 0, 4, 8, 12, m[0], m[1]), g(s, 1, 5, 9, 13, m[2], m[3]);
      g(s, 2, 6, 10, 14, m[4], m[5]), g(s, 3, 7, 11, 15, m[6], m[7]);
      g(s, 0, 5, 10, 15, m[8], m[9]), g(s, 1, 6, 11, 12, m[10], m[11]);
      g(s, 2, 7, 8, 13, m[12], m[13]), g(s, 3, 4, 9, 14, m[14], m[15]);
      for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
      memcpy(m, t, 64);
    }
    std::array<uint32_t, 8> o;
    for (int i = 0; i < 8; i++) o[i] = s[i] ^ s[i + 8];
    return o;
  }
  static std::array<uint32_t, 8> chunk_cv(const uint8_t* p, size_t n, uint64_t counter, bool root) {
    uint32_t cv[8];
    memcpy(cv, IV, 32);
    const size_t nblocks = n == 0 ? 1 : (n + 63) / 64;
    for (size_t i = 0; i < nblocks; i++) {
      uint8_t blk[64] = {0};
      const size_t len = std::min<size_t>(64, n - i * 64);
      if (n) memcpy(blk, p + i * 64, len);
      uint32_t mw[16];
      for (int k = 0; k < 16; k++) mw[k] = blk[4 * k] | blk[4 * k + 1] << 8 | blk[4 * k + 2] << 16 | (uint32_t)blk[4 * k + 3] << 24;
      uint32_t flags = (i == 0 ? CHUNK_START : 0) | (i == nblocks - 1 ? CHUNK_END : 0);
      if (root && i == nblocks - 1) flags |= ROOT;
      auto o = compress(cv, mw, counter, n ? (uint32_t)len : 0, flags);
      memcpy(cv, o.data(), 32);
    }
    std::array<uint32_t, 8> r;
    memcpy(r.data(), cv, 32);
    return r;
  }
  static std::array<uint32_t, 8> merge(const std::vector<std::array<uint32_t, 8>>& cvs, size_t lo, size_t hi,
                                       bool root) {
    const size_t n = hi - lo;
    if (n == 1) return cvs[lo];
    size_t left = 1;
    while (left * 2 < n) left *= 2;
    auto l = merge(cvs, lo, lo + left, false), r = merge(cvs, lo + left, hi, false);
    uint32_t mw[16];
    memcpy(mw, l.data(), 32);
    memcpy(mw + 8, r.data(), 32);
    return compress(IV, mw, 0, 64, PARENT | (root ? ROOT : 0));
  }
  std::vector<uint8_t> buf_;
};

}  // namespace zp
