// ff.h — BN254 Fq / Fr arithmetic for CDNA4 (gfx950), host+device.
//
// Representation (MI355X-first, not arkworks' 4x64):
//   * 9 limbs x 29 bits held in 32-bit VGPRs, Montgomery radix R = 2^261.
//   * Product-scanning Montgomery multiplication: every partial product is one
//     v_mad_u64_u32 into a single 64-bit column accumulator.  29-bit limbs leave
//     headroom for 18 products per column (< 2^64) so no carry chains are needed
//     inside a column (measured: v_mad_u64_u32 issues at the same rate as a
//     plain VALU op on gfx950, see tools/mb_modmul.hip / profiles/).
//   * Lazy reduction: mul accepts inputs < 8p with limbs < 1.5*2^30 and returns
//     a value < 2p with normalised limbs (R > 32p), so no final subtraction.
//     add/sub return normalised values in [0, 2p).
//   * Storage in HBM/LDS-less paths is the packed 8 x u32 (256-bit) form.
// The GPU's Montgomery radix differs from arkworks' (2^256); conversion happens
// only at the boundary (canonical <-> internal), never in the hot loops.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define ZK_HD __host__ __device__ __forceinline__
#else
#define ZK_HD inline
#endif

namespace zk {

constexpr int NL = 9;
constexpr uint32_t LMASK = (1u << 29) - 1;

struct Fe {
  uint32_t v[NL];
};

// Base field q (G1/G2 coordinates)
struct FqP {
  static constexpr bool ASM = true;
  static constexpr uint32_t P[NL] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                     0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  static constexpr uint32_t P2[NL] = {0x10f9fa8eu, 0x0208c16du, 0x18e5469eu, 0x05aa45a1u, 0x0b0bb2f0u,
                                      0x05b68181u, 0x014dc282u, 0x1cb84c68u, 0x0060c89cu};
  static constexpr uint32_t PINV = 0x04866389u;  // -p^-1 mod 2^29
  static constexpr uint32_t ONE[NL] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u,
                                       0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // R mod p
  static constexpr uint32_t R2[NL] = {0x059bac10u, 0x0d1503a3u, 0x018016b8u, 0x10ab0ca8u, 0x02632639u,
                                      0x02c0169fu, 0x169bfd53u, 0x11869d4cu, 0x002a11a6u};  // R^2 mod p
  // 4p, 6p, 8p in normalised limbs (biases of the lazy subtractions)
  static constexpr uint32_t P4[NL] = {0x01f3f51cu, 0x041182dbu, 0x11ca8d3cu, 0x0b548b43u, 0x161765e0u,
                                      0x0b6d0302u, 0x029b8504u, 0x197098d0u, 0x00c19139u};
  static constexpr uint32_t P6[NL] = {0x12edefaau, 0x061a4448u, 0x0aafd3dau, 0x10fed0e5u, 0x012318d0u,
                                      0x11238484u, 0x03e94786u, 0x1628e538u, 0x012259d6u};
  static constexpr uint32_t P8[NL] = {0x03e7ea38u, 0x082305b6u, 0x03951a78u, 0x16a91687u, 0x0c2ecbc0u,
                                      0x16da0605u, 0x05370a08u, 0x12e131a0u, 0x01832273u};
  // Borrow forms of K p: limbs 0..7 raised by m 2^29 (m borrowed from the next
  // limb), so that K p - a is limb-wise non-negative for any normalised a
  // (m = 1) or for a + 2b (m = 3) without a carry pass (BK_m, ec.h
  // xyzz_madd_g1f).  Same values as K p.
  static constexpr uint32_t B2_1[NL] = {0x30f9fa8eu, 0x2208c16cu, 0x38e5469du, 0x25aa45a0u, 0x2b0bb2efu,
                                        0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};
  static constexpr uint32_t B4_1[NL] = {0x21f3f51cu, 0x241182dau, 0x31ca8d3bu, 0x2b548b42u, 0x361765dfu,
                                        0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
  static constexpr uint32_t B8_1[NL] = {0x23e7ea38u, 0x282305b5u, 0x23951a77u, 0x36a91686u, 0x2c2ecbbfu,
                                        0x36da0604u, 0x25370a07u, 0x32e1319fu, 0x01832272u};
  static constexpr uint32_t B6_3[NL] = {0x72edefaau, 0x661a4445u, 0x6aafd3d7u, 0x70fed0e2u, 0x612318cdu,
                                        0x71238481u, 0x63e94783u, 0x7628e535u, 0x012259d3u};
  static constexpr uint32_t B10_1[NL] = {0x34e1e4c6u, 0x2a2bc722u, 0x3c7a6115u, 0x3c535c27u, 0x373a7eafu,
                                         0x3c908785u, 0x2684cc89u, 0x2f997e07u, 0x01e3eb0fu};
};
// Scalar field r (NTT domain)
struct FrP {
  static constexpr bool ASM = true;  // (compiler-scheduled products: 2^24 NTT+INTT 4.41 -> 5.30 ms)
  static constexpr uint32_t P[NL] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                                     0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  static constexpr uint32_t P2[NL] = {0x00000002u, 0x1e1f593fu, 0x1cb848a1u, 0x0fa121e6u, 0x0b0ba506u,
                                      0x05b68181u, 0x014dc282u, 0x1cb84c68u, 0x0060c89cu};
  // 4r, 6r, 8r (biases of the lazy subtractions, conditional subtractions)
  static constexpr uint32_t P4[NL] = {0x00000004u, 0x1c3eb27eu, 0x19709143u, 0x1f4243cdu, 0x16174a0cu,
                                      0x0b6d0302u, 0x029b8504u, 0x197098d0u, 0x00c19139u};
  static constexpr uint32_t P6[NL] = {0x00000006u, 0x1a5e0bbdu, 0x1628d9e5u, 0x0ee365b4u, 0x0122ef13u,
                                      0x11238484u, 0x03e94786u, 0x1628e538u, 0x012259d6u};
  static constexpr uint32_t P8[NL] = {0x00000008u, 0x187d64fcu, 0x12e12287u, 0x1e84879bu, 0x0c2e9419u,
                                      0x16da0605u, 0x05370a08u, 0x12e131a0u, 0x01832273u};
  static constexpr uint32_t P16[NL] = {0x00000010u, 0x10fac9f8u, 0x05c2450fu, 0x1d090f37u, 0x185d2833u,
                                       0x0db40c0au, 0x0a6e1411u, 0x05c26340u, 0x030644e7u};
  static constexpr uint32_t PINV = 0x0fffffffu;
  static constexpr uint32_t ONE[NL] = {0x0fffff57u, 0x1ea70ab4u, 0x052c068bu, 0x17504f49u, 0x0aa8075bu,
                                       0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};
  static constexpr uint32_t R2[NL] = {0x05b69bd4u, 0x06170a5au, 0x020cddceu, 0x1db6310bu, 0x0e54d0ffu,
                                      0x1cf855e3u, 0x1c15e103u, 0x07d09161u, 0x000a054au};
};

// Fq for G2 code: same constants, compiler-scheduled products (pmac)
struct FqPn : FqP {
  static constexpr bool ASM = false;
};

// ---------------------------------------------------------------- packing
// 256-bit little-endian (8 x u32) <-> 9 x 29-bit limbs.
ZK_HD Fe unpack(const uint32_t w[8]) {
  Fe r;
  r.v[0] = w[0] & LMASK;
  r.v[1] = ((w[0] >> 29) | (w[1] << 3)) & LMASK;
  r.v[2] = ((w[1] >> 26) | (w[2] << 6)) & LMASK;
  r.v[3] = ((w[2] >> 23) | (w[3] << 9)) & LMASK;
  r.v[4] = ((w[3] >> 20) | (w[4] << 12)) & LMASK;
  r.v[5] = ((w[4] >> 17) | (w[5] << 15)) & LMASK;
  r.v[6] = ((w[5] >> 14) | (w[6] << 18)) & LMASK;
  r.v[7] = ((w[6] >> 11) | (w[7] << 21)) & LMASK;
  r.v[8] = w[7] >> 8;
  return r;
}
ZK_HD void pack(uint32_t w[8], const Fe& a) {
  w[0] = a.v[0] | (a.v[1] << 29);
  w[1] = (a.v[1] >> 3) | (a.v[2] << 26);
  w[2] = (a.v[2] >> 6) | (a.v[3] << 23);
  w[3] = (a.v[3] >> 9) | (a.v[4] << 20);
  w[4] = (a.v[4] >> 12) | (a.v[5] << 17);
  w[5] = (a.v[5] >> 15) | (a.v[6] << 14);
  w[6] = (a.v[6] >> 18) | (a.v[7] << 11);
  w[7] = (a.v[7] >> 21) | (a.v[8] << 8);
}

template <class P>
ZK_HD Fe fe_const(const uint32_t (&c)[NL]) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c[i];
  return r;
}
ZK_HD Fe fe_zero() {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = 0;
  return r;
}

// ------------------------------------------------------- column accumulate
// acc += a * b as exactly one v_mad_u64_u32 on the device.  Written as inline
// asm so that every column stays ONE dependent chain: left to itself the
// compiler splits columns into parallel partial sums (to hide mad latency a
// single wave would see) and pays a 64-bit add per split, ~9% of a
// multiplication; with 3-4 waves per SIMD the latency is already hidden.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ZK_NO_ASM_MAD)
// The carry-out (unused) goes to a fresh SGPR pair ("=s").  (Writing VCC,
// declared clobbered, instead saves ~20 SGPR-spill reloads per G1
// accumulation step but makes hipcc 8x slower on these files.)
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cy) : "v"(a), "v"(b));
}
__device__ __forceinline__ void macs(uint64_t& acc, uint32_t a, uint32_t b_uniform) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cy) : "v"(a), "s"(b_uniform));
}
// acc += d (32-bit addend) as one v_mad_u64_u32 by the inline constant 1
__device__ __forceinline__ void mac1(uint64_t& acc, uint32_t d) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %2, 1, %0" : "+v"(acc), "=s"(cy) : "v"(d));
}
#else
ZK_HD void mac(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }
ZK_HD void macs(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }
ZK_HD void mac1(uint64_t& acc, uint32_t d) { acc += d; }
#endif

// Product accumulation by field: P::ASM picks the one-chain inline-asm mads
// (throughput kernels: G1, Fr) or plain C that the compiler may split into
// parallel partial sums.  G2 (Fq2) code uses FqPn (ASM = false): at its 2
// waves/SIMD the split chains win (2^20 G2 MSM, 2 lanes: 294 -> 308 Mpt/s),
// and its ~half as many instructions (no hazard nops) fit the code in the
// instruction cache.
template <class P>
ZK_HD void pmac(uint64_t& acc, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ZK_NO_ASM_MAD)
  if constexpr (P::ASM) {
    mac(acc, a, b);
    return;
  }
#endif
  acc += (uint64_t)a * b;
}
template <class P>
ZK_HD void pmacs(uint64_t& acc, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ZK_NO_ASM_MAD)
  if constexpr (P::ASM) {
    macs(acc, a, b);
    return;
  }
#endif
  acc += (uint64_t)a * b;
}
template <class P>
ZK_HD void pmac1(uint64_t& acc, uint32_t d) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ZK_NO_ASM_MAD)
  if constexpr (P::ASM) {
    mac1(acc, d);
    return;
  }
#endif
  acc += d;
}

// ------------------------------------------------------------ Montgomery mul
// r = a*b*2^-261 mod p (lazy: result < 2p, normalised limbs).
template <class P>
ZK_HD Fe mul(const Fe& a, const Fe& b) {
  uint32_t m[NL];
  Fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    pmac<P>(acc, a.v[k], b.v[0]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// r = a*b*2^-261 + d (mod p, lazy): the Montgomery product with d added into
// its upper columns, so the sum comes out normalised with no carry pass of its
// own (9 one-instruction adds instead of a 9-limb signed-carry subtraction
// when d is a borrow-form difference such as 8p - x, FqP::BK_m).  d: limbs
// 0..7 non-negative and < 2^31; limb 8 is added modulo 2^32 (a borrow there is
// harmless while the true sum is non-negative).  Value: < a b / R + p + d.
template <class P>
ZK_HD Fe mul_add(const Fe& a, const Fe& b, const Fe& d) {
  uint32_t m[NL];
  Fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    pmac<P>(acc, a.v[k], b.v[0]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    pmac1<P>(acc, d.v[k - NL]);
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc + d.v[NL - 1];
  return r;
}
// r = a^2 * 2^-261 + d, as mul_add
template <class P>
ZK_HD Fe sqr_add(const Fe& a, const Fe& d) {
  uint32_t m[NL], dd[NL];
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) dd[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < (k + 1) / 2; j++) pmac<P>(acc, dd[j], a.v[k - j]);
    if ((k & 1) == 0) pmac<P>(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
    for (int j = 0; j < k; j++) pmacs<P>(acc, m[j], P::P[k - j]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    pmac1<P>(acc, d.v[k - NL]);
#pragma unroll
    for (int j = k - (NL - 1); j < (k + 1) / 2; j++) pmac<P>(acc, dd[j], a.v[k - j]);
    if ((k & 1) == 0) pmac<P>(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) pmacs<P>(acc, m[j], P::P[k - j]);
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc + d.v[NL - 1];
  return r;
}
// limb-wise c - a (c a borrow-form constant, a normalised): no carry pass
ZK_HD Fe bsub(const uint32_t (&c)[NL], const Fe& a) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c[i] - a.v[i];
  return r;
}
// limb-wise c - a - 2b (c = BK_3)
ZK_HD Fe bsub2(const uint32_t (&c)[NL], const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c[i] - (a.v[i] + (b.v[i] << 1));
  return r;
}
// limb-wise c - a + b (c = BK_1, a and b normalised): limbs < 1.5 2^30
ZK_HD Fe bsubadd(const uint32_t (&c)[NL], const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c[i] - a.v[i] + b.v[i];
  return r;
}

// squaring: off-diagonal products once, doubled operand
template <class P>
ZK_HD Fe sqr(const Fe& a) {
  uint32_t m[NL], d[NL];
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) d[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < (k + 1) / 2; j++) pmac<P>(acc, d[j], a.v[k - j]);
    if ((k & 1) == 0) pmac<P>(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
    for (int j = 0; j < k; j++) pmacs<P>(acc, m[j], P::P[k - j]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < (k + 1) / 2; j++) pmac<P>(acc, d[j], a.v[k - j]);
    if ((k & 1) == 0) pmac<P>(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) pmacs<P>(acc, m[j], P::P[k - j]);
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// --------------------------------------------------------------- add / sub
// r = a - b mod p for a, b in [0, 2p) normalised -> [0, 2p) normalised.
template <class P>
ZK_HD Fe sub(const Fe& a, const Fe& b) {
  Fe r;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + br;
    r.v[i] = (uint32_t)t & LMASK;
    br = t >> 29;
  }
  // br is 0 or -1; add 2p under mask
  uint32_t mask = (uint32_t)br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint32_t t = r.v[i] + (P::P2[i] & mask) + c;
    r.v[i] = t & LMASK;
    c = t >> 29;
  }
  return r;
}
// r = a + b mod p for a, b in [0, 2p) -> [0, 2p)
template <class P>
ZK_HD Fe add(const Fe& a, const Fe& b) {
  Fe r;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int32_t t = (int32_t)(a.v[i] + b.v[i]) - (int32_t)P::P2[i] + br;
    r.v[i] = (uint32_t)t & LMASK;
    br = t >> 29;
  }
  uint32_t mask = (uint32_t)(br >> 31);  // top is negative -> add 2p back
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint32_t t = r.v[i] + (P::P2[i] & mask) + c;
    r.v[i] = t & LMASK;
    c = t >> 29;
  }
  return r;
}
template <class P>
ZK_HD Fe dbl(const Fe& a) {
  return add<P>(a, a);
}
template <class P>
ZK_HD Fe neg(const Fe& a) {
  return sub<P>(fe_zero(), a);
}
// lazy add: limbwise, no carry (limbs < 2^30, value < 4p).  Only as a mul input.
ZK_HD Fe add_lazy(const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// ---------------------------------------------------------- lazy forms
// Bounds used by the fast G1 mixed addition (R/p = 169.3, so a Montgomery
// product of values a, b with a*b < 169 p^2 still lands in [0, 2p); columns
// stay below 2^64 while one factor's limbs are < 2^30 and the other's < 2^29,
// or both < 2^30 for a single product).
//
// a - b + K p in one signed-carry pass: normalised limbs, value a - b + Kp.
// Caller guarantees 0 <= a - b + Kp < 2^261 (limbs of a, b may be up to 2^31).
template <class P, int K>
ZK_HD Fe subk(const Fe& a, const Fe& b) {
  static_assert(K == 2 || K == 4 || K == 6 || K == 8, "bias");
  const uint32_t* kp = K == 2 ? P::P2 : K == 4 ? P::P4 : K == 6 ? P::P6 : P::P8;
  Fe r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int32_t t = (int32_t)(a.v[i] + kp[i]) - (int32_t)b.v[i] + c;
    r.v[i] = (uint32_t)t & LMASK;
    c = t >> 29;
  }
  return r;
}
// (a*b + c*d) * 2^-261 mod p in one product-scanning pass (one reduction for
// two products).  a, c: limbs < 2^30; b, d: limbs < 2^29; a*b + c*d < 169 p^2.
template <class P>
ZK_HD Fe mul2(const Fe& a, const Fe& b, const Fe& c, const Fe& d) {
  uint32_t m[NL];
  Fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmac<P>(acc, c.v[j], d.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    pmac<P>(acc, a.v[k], b.v[0]);
    pmac<P>(acc, c.v[k], d.v[0]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmac<P>(acc, c.v[j], d.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}
// Two independent Montgomery products interleaved column by column: two
// accumulator chains in one instruction stream give each wave the ILP that a
// single dependent mad chain lacks.
template <class P>
ZK_HD void mul_x2(const Fe& a, const Fe& b, const Fe& c, const Fe& d, Fe& r0, Fe& r1) {
  uint32_t m[NL], n[NL];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      mac(x, a.v[j], b.v[k - j]);
      mac(y, c.v[j], d.v[k - j]);
      macs(x, m[j], P::P[k - j]);
      macs(y, n[j], P::P[k - j]);
    }
    mac(x, a.v[k], b.v[0]);
    mac(y, c.v[k], d.v[0]);
    m[k] = ((uint32_t)x * P::PINV) & LMASK;
    n[k] = ((uint32_t)y * P::PINV) & LMASK;
    macs(x, m[k], P::P[0]);
    macs(y, n[k], P::P[0]);
    x >>= 29;
    y >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      mac(x, a.v[j], b.v[k - j]);
      mac(y, c.v[j], d.v[k - j]);
      macs(x, m[j], P::P[k - j]);
      macs(y, n[j], P::P[k - j]);
    }
    r0.v[k - NL] = (uint32_t)x & LMASK;
    r1.v[k - NL] = (uint32_t)y & LMASK;
    x >>= 29;
    y >>= 29;
  }
  r0.v[NL - 1] = (uint32_t)x;
  r1.v[NL - 1] = (uint32_t)y;
}
template <class P>
ZK_HD void sqr_x2(const Fe& a, const Fe& c, Fe& r0, Fe& r1) {
  uint32_t m[NL], n[NL], da[NL], dc[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    da[i] = a.v[i] << 1;
    dc[i] = c.v[i] << 1;
  }
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < (k + 1) / 2; j++) {
      mac(x, da[j], a.v[k - j]);
      mac(y, dc[j], c.v[k - j]);
    }
    if ((k & 1) == 0) {
      mac(x, a.v[k / 2], a.v[k / 2]);
      mac(y, c.v[k / 2], c.v[k / 2]);
    }
#pragma unroll
    for (int j = 0; j < k; j++) {
      macs(x, m[j], P::P[k - j]);
      macs(y, n[j], P::P[k - j]);
    }
    m[k] = ((uint32_t)x * P::PINV) & LMASK;
    n[k] = ((uint32_t)y * P::PINV) & LMASK;
    macs(x, m[k], P::P[0]);
    macs(y, n[k], P::P[0]);
    x >>= 29;
    y >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < (k + 1) / 2; j++) {
      mac(x, da[j], a.v[k - j]);
      mac(y, dc[j], c.v[k - j]);
    }
    if ((k & 1) == 0) {
      mac(x, a.v[k / 2], a.v[k / 2]);
      mac(y, c.v[k / 2], c.v[k / 2]);
    }
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      macs(x, m[j], P::P[k - j]);
      macs(y, n[j], P::P[k - j]);
    }
    r0.v[k - NL] = (uint32_t)x & LMASK;
    r1.v[k - NL] = (uint32_t)y & LMASK;
    x >>= 29;
    y >>= 29;
  }
  r0.v[NL - 1] = (uint32_t)x;
  r1.v[NL - 1] = (uint32_t)y;
}

// (a*b + c*d + e*f + g*h) * 2^-261 mod p: four products, one reduction.
// All operand limbs < 2^29 (normalised); sum of products < 169 p^2.
template <class P>
ZK_HD Fe mul4(const Fe& a, const Fe& b, const Fe& c, const Fe& d, const Fe& e, const Fe& f, const Fe& g,
              const Fe& h) {
  uint32_t m[NL];
  Fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmac<P>(acc, c.v[j], d.v[k - j]);
      pmac<P>(acc, e.v[j], f.v[k - j]);
      pmac<P>(acc, g.v[j], h.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    pmac<P>(acc, a.v[k], b.v[0]);
    pmac<P>(acc, c.v[k], d.v[0]);
    pmac<P>(acc, e.v[k], f.v[0]);
    pmac<P>(acc, g.v[k], h.v[0]);
    m[k] = ((uint32_t)acc * P::PINV) & LMASK;
    pmacs<P>(acc, m[k], P::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      pmac<P>(acc, a.v[j], b.v[k - j]);
      pmac<P>(acc, c.v[j], d.v[k - j]);
      pmac<P>(acc, e.v[j], f.v[k - j]);
      pmac<P>(acc, g.v[j], h.v[k - j]);
      pmacs<P>(acc, m[j], P::P[k - j]);
    }
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// [0, 32p) -> [0, 2p), normalised limbs, in one pass (Fq and Fr share the
// top limb p8 = 0x30644e): q = floor(x8 M / 2^48), M = floor(2^48 / (p8 + 2)),
// satisfies x / p - 1 - 2^-14 < q <= x / p (x8 < 2^27), so x - q p is in
// [0, 2p).  One 9-limb signed-carry pass instead of conditional subtractions.
// The input's limbs 0..7 may be unnormalised (< 2^31, e.g. limb-wise sums):
// they move the value by < 4 units of the top limb, which only lowers q by a
// vanishing fraction, and the carry pass normalises the output.
template <class P>
ZK_HD Fe reduce_q32(const Fe& x) {
  static_assert(P::P[NL - 1] == 0x0030644eu, "top limb of the quotient estimate");
  constexpr uint32_t M = 88753946u;  // floor(2^48 / (0x30644e + 2))
  const uint32_t q = (uint32_t)(((uint64_t)x.v[NL - 1] * M) >> 48);
  Fe r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int64_t t = (int64_t)x.v[i] - (int64_t)((uint64_t)q * P::P[i]) + c;
    r.v[i] = (uint32_t)t & LMASK;
    c = t >> 29;
  }
  return r;
}
// [0, 8p) -> [0, 2p), normalised limbs
template <class P>
ZK_HD Fe reduce8(const Fe& a) {
  return reduce_q32<P>(a);
}

// fully reduce [0, 2p) -> [0, p)
template <class P>
ZK_HD Fe reduce(const Fe& a) {
  Fe d;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int32_t t = (int32_t)a.v[i] - (int32_t)P::P[i] + br;
    d.v[i] = (uint32_t)t & LMASK;
    br = t >> 29;
  }
  Fe r;
  bool neg_ = br < 0;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = neg_ ? a.v[i] : d.v[i];
  return r;
}
template <class P>
ZK_HD bool is_zero(const Fe& a) {
  Fe t = reduce<P>(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) o |= t.v[i];
  return o == 0;
}
template <class P>
ZK_HD bool eq(const Fe& a, const Fe& b) {
  Fe x = reduce<P>(a), y = reduce<P>(b);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) o |= x.v[i] ^ y.v[i];
  return o == 0;
}
template <class P>
ZK_HD Fe one() {
  return fe_const<P>(P::ONE);
}
// canonical (packed, < p) -> Montgomery internal
template <class P>
ZK_HD Fe to_mont(const Fe& a) {
  return mul<P>(a, fe_const<P>(P::R2));
}
// Montgomery internal -> canonical, fully reduced
template <class P>
ZK_HD Fe from_mont(const Fe& a) {
  Fe o = fe_zero();
  o.v[0] = 1;
  return reduce<P>(mul<P>(a, o));
}
// a^e for a small public exponent given as 4 x u64 (used off the hot path)
template <class P>
ZK_HD Fe pow(const Fe& a, const uint64_t e[4]) {
  Fe r = one<P>();
  for (int i = 255; i >= 0; i--) {
    r = sqr<P>(r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = mul<P>(r, a);
  }
  return r;
}

// ---------------------------------------------------------------- Fq2
// Fq2 = Fq[u]/(u^2 + 1)
struct Fe2 {
  Fe c0, c1;
};
ZK_HD Fe2 f2_add(const Fe2& a, const Fe2& b) { return {add<FqPn>(a.c0, b.c0), add<FqPn>(a.c1, b.c1)}; }
ZK_HD Fe2 f2_sub(const Fe2& a, const Fe2& b) { return {sub<FqPn>(a.c0, b.c0), sub<FqPn>(a.c1, b.c1)}; }
ZK_HD Fe2 f2_dbl(const Fe2& a) { return {dbl<FqPn>(a.c0), dbl<FqPn>(a.c1)}; }
ZK_HD Fe2 f2_neg(const Fe2& a) { return {neg<FqPn>(a.c0), neg<FqPn>(a.c1)}; }
ZK_HD Fe2 f2_mul(const Fe2& a, const Fe2& b) {
  Fe t0 = mul<FqPn>(a.c0, b.c0);
  Fe t1 = mul<FqPn>(a.c1, b.c1);
  Fe t2 = mul<FqPn>(add_lazy(a.c0, a.c1), add_lazy(b.c0, b.c1));
  return {sub<FqPn>(t0, t1), sub<FqPn>(sub<FqPn>(t2, t0), t1)};
}
ZK_HD Fe2 f2_sqr(const Fe2& a) {
  // (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u
  Fe s = add_lazy(a.c0, a.c1);
  Fe d = sub<FqPn>(a.c0, a.c1);
  Fe c0 = mul<FqPn>(s, d);
  Fe c1 = mul<FqPn>(a.c0, a.c1);
  return {c0, dbl<FqPn>(c1)};
}
ZK_HD bool f2_is_zero(const Fe2& a) { return is_zero<FqPn>(a.c0) && is_zero<FqPn>(a.c1); }
ZK_HD bool fe_is_zero_raw(const Fe& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) o |= a.v[i];
  return o == 0;
}
ZK_HD Fe2 f2_zero() { return {fe_zero(), fe_zero()}; }
ZK_HD Fe2 f2_one() { return {one<FqPn>(), fe_zero()}; }

// Fq2 products with one reduction per component (mul2): inputs normalised
// limbs, values < 4p; outputs < 2p.
ZK_HD Fe2 f2_mul_n(const Fe2& a, const Fe2& b) {
  Fe nb1 = subk<FqPn, 4>(fe_zero(), b.c1);
  return {mul2<FqPn>(a.c0, b.c0, a.c1, nb1), mul2<FqPn>(a.c0, b.c1, a.c1, b.c0)};
}
ZK_HD Fe2 f2_sqr_n(const Fe2& a) {
  return {mul<FqPn>(add_lazy(a.c0, a.c1), subk<FqPn, 4>(a.c0, a.c1)), mul<FqPn>(add_lazy(a.c0, a.c0), a.c1)};
}

// Uniform field interface used by the curve templates.
struct FqOps {
  using T = Fe;
  static ZK_HD T mul(const T& a, const T& b) { return zk::mul<FqP>(a, b); }
  static ZK_HD T sqr(const T& a) { return zk::sqr<FqP>(a); }
  static ZK_HD T add(const T& a, const T& b) { return zk::add<FqP>(a, b); }
  static ZK_HD T sub(const T& a, const T& b) { return zk::sub<FqP>(a, b); }
  static ZK_HD T dbl(const T& a) { return zk::dbl<FqP>(a); }
  static ZK_HD T neg(const T& a) { return zk::neg<FqP>(a); }
  static ZK_HD bool is_zero(const T& a) { return zk::is_zero<FqP>(a); }
  static ZK_HD bool is_zero_raw(const T& a) { return fe_is_zero_raw(a); }
  static ZK_HD T zero() { return fe_zero(); }
  static ZK_HD T one() { return zk::one<FqP>(); }
};
struct Fq2Ops {
  using T = Fe2;
  static ZK_HD T mul(const T& a, const T& b) { return f2_mul(a, b); }
  static ZK_HD T sqr(const T& a) { return f2_sqr(a); }
  static ZK_HD T add(const T& a, const T& b) { return f2_add(a, b); }
  static ZK_HD T sub(const T& a, const T& b) { return f2_sub(a, b); }
  static ZK_HD T dbl(const T& a) { return f2_dbl(a); }
  static ZK_HD T neg(const T& a) { return f2_neg(a); }
  static ZK_HD bool is_zero(const T& a) { return f2_is_zero(a); }
  static ZK_HD bool is_zero_raw(const T& a) { return fe_is_zero_raw(a.c0) && fe_is_zero_raw(a.c1); }
  static ZK_HD T zero() { return f2_zero(); }
  static ZK_HD T one() { return f2_one(); }
};

}  // namespace zk
