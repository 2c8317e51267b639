// wprog.hip — witness programs: per-batch witness generation on the GPU,
// writing the full assignment z straight into HBM.
//
// The zelana_batch circuit (forge/circuits/zelana_batch/src/main.nr) is 99%
// MiMC: ~3,900 permutations of 91 rounds x -> (x + c_i)^7 whose per-round
// values t^2, t^4, t^6, t^7 are the witness (host restatement
// prover-worker/src/mimc.rs:52-142; zelana_amd/zbatch.py).  Its proving key
// fits one circuit shape, so the witness is a FIXED straight-line program over
// Fr; only ~2,400 free inputs (Prover.toml values) change per batch.  The
// program is recorded once on the host (zelana_amd/wprog.py) as ops over
// linear combinations of z, grouped into dependency levels:
//   MUL    z[out] = <a, z> * <b, z>                (products, selects, Merkle d)
//   INV    z[out] = <a, z>^-1 or 0                 (signature != 0 witnesses)
//   BITS64 z[out + i] = bit i of <a, z>, i < 64    (u64 range checks)
//   PERM   z[out + 4 r + k] = (t_r^2, t_r^4, t_r^6, t_r^7), t_0 = <a, z> + c_0,
//          t_r = t_{r-1}^7 + c_r                   (one MiMC permutation)
// and, for L2BlockCircuit (prover/src/l2_circuit.rs:180-505, recorded by the
// C++ synthesizer, zelana_amd/host/l2_circuit.cpp):
//   BITS   z[out + i] = bit i of <a, z>, i < n     (to_non_unique_bits_le)
//   NZ     z[out] = (<a, z> != 0)                  (is_neq's flag)
//   INV1   z[out] = <a, z>^-1, or 1 for 0         (is_neq's multiplier)
//   POSEIDON  one permutation of the width-3 sponge (l2_circuit.rs:68-83:
//          x^5, 8 full + 56 partial rounds, Grain-LFSR constants): state in =
//          three combinations, out = every S-box's x^2, x^4, x^5 in round
//          order (round 0 skips constant elements, per the op's mask)
// and each level is one launch; a batch uploads only its inputs.
//
// The program is latency-bound, not throughput-bound: its critical path is
// ~70 dependent permutations (a depth-32 Merkle path is 64 of them) with ~57
// independent chains beside it, so one launch holds a wave or two.  A
// permutation is therefore worked by a QUAD of lanes: all four square t, two
// pairs form t^4 / t^3 and then t^6 / t^7 (DPP quad broadcasts exchange
// them), and each lane converts and stores one of the round's four values
// (the four stores of a round are one 128-byte run).  That keeps the
// dependent chain per round at three Montgomery products.  The witness stream
// runs beside the previous batch's proof (zkmi_wprog_run, async): it occupies
// a few CUs while the prover has the rest.
//
// Column chains are left to the compiler here (ZK_NO_ASM_MAD): with one wave
// per SIMD, the mad latency it hides by splitting columns matters more than
// the add it costs (the opposite trade of the throughput kernels).
#define ZK_NO_ASM_MAD 1
#include <string.h>

#include <algorithm>
#include <vector>

#include "dev_io.h"
#include "ff.h"

#include "zkmi_internal.h"

namespace zk {

constexpr int WP_MUL = 1, WP_INV = 2, WP_BITS64 = 3, WP_PERM = 4, WP_BITS = 5, WP_NZ = 6, WP_POSEIDON = 7,
              WP_INV1 = 8;
constexpr int MIMC_R = 91;
// Poseidon (get_poseidon_config): constants at coefficient ids 3 r + i (ark)
// and 192 + 3 i + j (MDS) of the program's table (zkmi.h)
constexpr int POS_ROUNDS = 64, POS_FULL_HALF = 4, POS_NCONST = 201;
__host__ __device__ constexpr uint32_t poseidon_trace_len(uint32_t mask) {
  return 3 * ((mask & 1) + ((mask >> 1) & 1) + ((mask >> 2) & 1)) + 231;
}

// a * 2^-261 mod r for a < 2^261 with normalised limbs: Montgomery reduction
// alone (a product with 1 without its 81 product mads)
__device__ __forceinline__ Fe redc_fr(const Fe& a) {
  uint32_t m[NL];
  Fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    acc += a.v[k];
#pragma unroll
    for (int j = 0; j < k; j++) acc += (uint64_t)m[j] * FrP::P[k - j];
    m[k] = ((uint32_t)acc * FrP::PINV) & LMASK;
    acc += (uint64_t)m[k] * FrP::P[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) acc += (uint64_t)m[j] * FrP::P[k - j];
    r.v[k - NL] = (uint32_t)acc & LMASK;
    acc >>= 29;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// Montgomery product (R = 2^261, lazy: < 2p out) with four independent
// accumulators per product-scanning column (even / odd j for the a*b and the
// m*p terms): one wave per SIMD exposes the mad latency of a single chain,
// and splitting it cuts the dependent chain per column to ~k/2 mads.
__device__ __forceinline__ Fe mul_ilp(const Fe& a, const Fe& b) {
  uint32_t m[NL];
  Fe r;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = 0; j < k; j++) {
      if (j & 1) {
        s1 += (uint64_t)a.v[j] * b.v[k - j];
        s3 += (uint64_t)m[j] * FrP::P[k - j];
      } else {
        s0 += (uint64_t)a.v[j] * b.v[k - j];
        s2 += (uint64_t)m[j] * FrP::P[k - j];
      }
    }
    if (k & 1) s1 += (uint64_t)a.v[k] * b.v[0];
    else s0 += (uint64_t)a.v[k] * b.v[0];
    uint64_t tot = (s0 + s1) + (s2 + s3);
    m[k] = ((uint32_t)tot * FrP::PINV) & LMASK;
    tot += (uint64_t)m[k] * FrP::P[0];
    c = tot >> 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      if (j & 1) {
        s1 += (uint64_t)a.v[j] * b.v[k - j];
        s3 += (uint64_t)m[j] * FrP::P[k - j];
      } else {
        s0 += (uint64_t)a.v[j] * b.v[k - j];
        s2 += (uint64_t)m[j] * FrP::P[k - j];
      }
    }
    const uint64_t tot = (s0 + s1) + (s2 + s3);
    r.v[k - NL] = (uint32_t)tot & LMASK;
    c = tot >> 29;
  }
  r.v[NL - 1] = (uint32_t)c;
  return r;
}

// squaring with the same split: off-diagonal products once (doubled operand)
__device__ __forceinline__ Fe sqr_ilp(const Fe& a) {
  uint32_t m[NL], d[NL];
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) d[i] = a.v[i] << 1;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = 0; j < (k + 1) / 2; j++) {
      if (j & 1) s1 += (uint64_t)d[j] * a.v[k - j];
      else s0 += (uint64_t)d[j] * a.v[k - j];
    }
    if ((k & 1) == 0) s1 += (uint64_t)a.v[k / 2] * a.v[k / 2];
#pragma unroll
    for (int j = 0; j < k; j++) {
      if (j & 1) s3 += (uint64_t)m[j] * FrP::P[k - j];
      else s2 += (uint64_t)m[j] * FrP::P[k - j];
    }
    uint64_t tot = (s0 + s1) + (s2 + s3);
    m[k] = ((uint32_t)tot * FrP::PINV) & LMASK;
    tot += (uint64_t)m[k] * FrP::P[0];
    c = tot >> 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = k - (NL - 1); j < (k + 1) / 2; j++) {
      if (j & 1) s1 += (uint64_t)d[j] * a.v[k - j];
      else s0 += (uint64_t)d[j] * a.v[k - j];
    }
    if ((k & 1) == 0) s1 += (uint64_t)a.v[k / 2] * a.v[k / 2];
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      if (j & 1) s3 += (uint64_t)m[j] * FrP::P[k - j];
      else s2 += (uint64_t)m[j] * FrP::P[k - j];
    }
    const uint64_t tot = (s0 + s1) + (s2 + s3);
    r.v[k - NL] = (uint32_t)tot & LMASK;
    c = tot >> 29;
  }
  r.v[NL - 1] = (uint32_t)c;
  return r;
}

// (a0 b0 + a1 b1 + a2 b2) R^-1 with ONE reduction (a Poseidon MDS row): the
// three products share the m digits and the m*p columns, ~160 mads fewer than
// three mul_ilp.  a_k < p (constants), b_k < 2p, normalised: the sum is
// < 6 p^2, inside the Montgomery bound (R / p = 169), so the output is < 2p;
// accumulator sums stay below 14 * 2^58 per column.
__device__ __forceinline__ Fe mul3_ilp(const Fe& a0, const Fe& b0, const Fe& a1, const Fe& b1, const Fe& a2,
                                       const Fe& b2) {
  uint32_t m[NL];
  Fe r;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = 0; j <= k; j++) {
      if (j & 1) {
        s1 += (uint64_t)a0.v[j] * b0.v[k - j];
        s1 += (uint64_t)a1.v[j] * b1.v[k - j];
        s3 += (uint64_t)a2.v[j] * b2.v[k - j];
      } else {
        s0 += (uint64_t)a0.v[j] * b0.v[k - j];
        s0 += (uint64_t)a1.v[j] * b1.v[k - j];
        s2 += (uint64_t)a2.v[j] * b2.v[k - j];
      }
      if (j < k) {
        if (j & 1) s3 += (uint64_t)m[j] * FrP::P[k - j];
        else s2 += (uint64_t)m[j] * FrP::P[k - j];
      }
    }
    uint64_t tot = (s0 + s1) + (s2 + s3);
    m[k] = ((uint32_t)tot * FrP::PINV) & LMASK;
    tot += (uint64_t)m[k] * FrP::P[0];
    c = tot >> 29;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    uint64_t s0 = c, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int j = k - (NL - 1); j < NL; j++) {
      if (j & 1) {
        s1 += (uint64_t)a0.v[j] * b0.v[k - j];
        s1 += (uint64_t)a1.v[j] * b1.v[k - j];
        s3 += (uint64_t)a2.v[j] * b2.v[k - j];
        s3 += (uint64_t)m[j] * FrP::P[k - j];
      } else {
        s0 += (uint64_t)a0.v[j] * b0.v[k - j];
        s0 += (uint64_t)a1.v[j] * b1.v[k - j];
        s2 += (uint64_t)a2.v[j] * b2.v[k - j];
        s2 += (uint64_t)m[j] * FrP::P[k - j];
      }
    }
    const uint64_t tot = (s0 + s1) + (s2 + s3);
    r.v[k - NL] = (uint32_t)tot & LMASK;
    c = tot >> 29;
  }
  r.v[NL - 1] = (uint32_t)c;
  return r;
}

__device__ __forceinline__ void st_canon(uint32_t* z, uint32_t var, const Fe& v) {
  uint32_t w[8];
  pack(w, reduce<FrP>(v));
  uint4* p = reinterpret_cast<uint4*>(z + (size_t)var * 8);
  p[0] = make_uint4(w[0], w[1], w[2], w[3]);
  p[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
__device__ __forceinline__ Fe ld_canon(const uint32_t* z, uint32_t var) {
  const uint4* p = reinterpret_cast<const uint4*>(z + (size_t)var * 8);
  uint4 a = p[0], b = p[1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return unpack(w);
}

// <terms, z>: coefficients held in Montgomery form, z canonical, so each
// product mul(c R, x) = c x lands in value form (< 2p), summed mod 2p
// (terms fetched four at a time so their loads are in flight together: a
// dependent load chain per term costs microseconds on the short levels)
__device__ __forceinline__ Fe eval_lc(const uint2* __restrict__ terms, uint32_t off, uint32_t len,
                                      const uint32_t* __restrict__ coeff_m, const uint32_t* __restrict__ z) {
  Fe acc = fe_zero();
  uint32_t i = 0;
  for (; i + 4 <= len; i += 4) {
    uint2 t[4];
#pragma unroll
    for (int k = 0; k < 4; k++) t[k] = terms[off + i + k];
    Fe c[4], x[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c[k] = ld_canon(coeff_m, t[k].y);  // packed Montgomery coefficient
      x[k] = ld_canon(z, t[k].x);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) acc = add<FrP>(acc, mul_ilp(c[k], x[k]));
  }
  for (; i < len; i++) {
    const uint2 t = terms[off + i];
    acc = add<FrP>(acc, mul_ilp(ld_canon(coeff_m, t.y), ld_canon(z, t.x)));
  }
  return acc;
}
__device__ __forceinline__ void st_raw(uint32_t* z, uint32_t var, const Fe& v) {
  uint32_t w[8];
  pack(w, v);
  uint4* p = reinterpret_cast<uint4*>(z + (size_t)var * 8);
  p[0] = make_uint4(w[0], w[1], w[2], w[3]);
  p[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

template <int LANE>
__device__ __forceinline__ Fe quad_bcast(const Fe& x) {
  constexpr int ctrl = LANE | (LANE << 2) | (LANE << 4) | (LANE << 6);  // quad_perm [L, L, L, L]
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.v[i], ctrl, 0xF, 0xF, false);
  return r;
}
__device__ __forceinline__ Fe sel(bool c, const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// One level: op = lo + thread / 4, q = lane in its quad.  The four lanes of a
// quad share an op, so a quad is either wholly active or wholly not (DPP
// reads stay inside active quads).
// One POSEIDON op on a quad: lane q < 3 holds state element q (Montgomery
// form); each round adds its constant, S-boxes (all lanes in full rounds,
// lane 0 in partial ones; the S-boxing lane stores x^2, x^4, x^5), then every
// lane forms its MDS row from the three elements (DPP quad broadcasts).
__device__ __forceinline__ void poseidon_quad(const Fe& in, uint32_t q, uint32_t out, uint32_t mask,
                                              const Fe* __restrict__ pc, uint32_t* __restrict__ z) {
  const uint32_t qq = q < 3 ? q : 2;
  Fe s = mul<FrP>(in, fe_const<FrP>(FrP::R2));
  const uint32_t m0 = 3 * __builtin_popcount(mask);  // trace values of round 0
  for (int r = 0; r < POS_ROUNDS; r++) {
    const Fe t = add<FrP>(s, pc[3 * r + qq]);
    const bool full = r < POS_FULL_HALF || r >= POS_ROUNDS - POS_FULL_HALF;
    Fe u = t;
    if (full || q == 0) {
      const Fe x2 = sqr_ilp(t), x4 = sqr_ilp(x2), x5 = mul_ilp(x4, t);
      u = x5;
      uint32_t at;
      bool st = q < 3;
      if (r == 0) {
        st = st && ((mask >> q) & 1);
        at = 3 * __builtin_popcount(mask & ((1u << q) - 1));
      } else if (r < POS_FULL_HALF) {
        at = m0 + 9 * (r - 1) + 3 * q;
      } else if (!full) {
        at = m0 + 27 + 3 * (r - POS_FULL_HALF);
      } else {
        at = m0 + 27 + 3 * (POS_ROUNDS - 2 * POS_FULL_HALF) + 9 * (r - (POS_ROUNDS - POS_FULL_HALF)) + 3 * q;
      }
      if (st) {  // Montgomery form (k_wprog_canon_vars converts them at the end of the run), except
                 // the last round's x^5, which the next permutations' state combinations read
        st_raw(z, out + at, x2);
        st_raw(z, out + at + 1, x4);
        if (r == POS_ROUNDS - 1) st_canon(z, out + at + 2, redc_fr(x5));
        else st_raw(z, out + at + 2, x5);
      }
    }
    const Fe b0 = quad_bcast<0>(u), b1 = quad_bcast<1>(u), b2 = quad_bcast<2>(u);
    const Fe* row = pc + 3 * POS_ROUNDS + 3 * qq;
    s = mul3_ilp(row[0], b0, row[1], b1, row[2], b2);
  }
}

// a^e (Montgomery form) for the Fermat inversion, on one lane: fixed 3-bit
// windows over e (86 digits, table a^1..a^7 selected without dynamic
// register indexing) with the latency-split products above -- ~74 products
// and 253 squarings instead of the binary ladder's ~127 and 255 asm-chain
// ones (the INV ops run alone on a lane, so latency is what counts).
__device__ Fe pow_w3(const Fe& a, const uint64_t e[4]) {
  Fe t[8];
  t[1] = a;
  t[2] = sqr_ilp(a);
#pragma unroll
  for (int k = 3; k < 8; k++) t[k] = mul_ilp(t[k - 1], a);
  Fe r = fe_zero();
  bool started = false;
  for (int j = 85; j >= 0; j--) {
    const int b0 = 3 * j;
    uint32_t d = 0;
#pragma unroll
    for (int u = 2; u >= 0; u--) {
      const int bit = b0 + u;
      d = (d << 1) | (bit < 256 ? (uint32_t)((e[bit >> 6] >> (bit & 63)) & 1) : 0u);
    }
    if (started) {
      r = sqr_ilp(r);
      r = sqr_ilp(r);
      r = sqr_ilp(r);
    }
    if (d) {
      Fe m = t[1];
#pragma unroll
      for (int k = 2; k < 8; k++) m = sel(d == (uint32_t)k, t[k], m);
      r = started ? mul_ilp(r, m) : m;
      started = true;
    }
  }
  return started ? r : one<FrP>();
}

// One op of a level, on the quad of lanes (op_i, q).
template <bool POS>
__device__ __forceinline__ void wprog_op(uint32_t op_i, uint32_t q, const uint4* __restrict__ ops,
                                         const uint2* __restrict__ terms, const uint32_t* __restrict__ coeff_m,
                                         const uint32_t* rc_s, const Fe* pc_s, uint32_t* __restrict__ z) {
  const uint4 op = ops[op_i];
  const int kind = op.x & 0xFF;
  const uint32_t alen = (op.x >> 8) & 0xFFF, blen = op.x >> 20, out = op.y;
  if constexpr (POS) {
    if (kind == WP_POSEIDON) {
      // lane q evaluates state combination q (stored contiguously at op.z)
      const uint32_t l2 = op.w & 0xFFFF;
      const uint32_t off = op.z + (q >= 1 ? alen : 0) + (q >= 2 ? blen : 0);
      const uint32_t len = q == 0 ? alen : q == 1 ? blen : q == 2 ? l2 : 0;
      poseidon_quad(eval_lc(terms, off, len, coeff_m, z), q, out, op.w >> 16, pc_s, z);
      return;
    }
  }
  const Fe a = eval_lc(terms, op.z, alen, coeff_m, z);
  if (kind == WP_PERM) {
    const Fe r2 = fe_const<FrP>(FrP::R2);
    Fe x = mul<FrP>(a, r2);  // Montgomery form
    const bool odd = q & 1;
    for (int r = 0; r < MIMC_R; r++) {
      const Fe tm = add<FrP>(x, unpack(rc_s + 8 * r));
      const Fe t2 = sqr_ilp(tm);
      const Fe p = mul_ilp(t2, sel(odd, tm, t2));  // even lanes: t^4, odd: t^3
      const Fe t4 = quad_bcast<0>(p), t3 = quad_bcast<1>(p);
      const Fe u = mul_ilp(t4, sel(odd, t3, t2));  // even lanes: t^6, odd: t^7
      x = quad_bcast<1>(u);                          // t^7 for the next round
      const Fe mine = q == 0 ? t2 : (q == 1 ? t4 : u);  // lanes store t^2, t^4, t^6, t^7
      // Montgomery form as is (k_wprog_canon converts them all afterwards in
      // one wide pass), except the permutation's output, which later ops read
      if (r == MIMC_R - 1 && q == 3) st_canon(z, out + 4 * (uint32_t)r + q, redc_fr(mine));
      else st_raw(z, out + 4 * (uint32_t)r + q, mine);
    }
    return;
  }
  if (kind == WP_BITS64 || kind == WP_BITS) {
    const uint32_t nbits = kind == WP_BITS ? op.w : 64;
    uint32_t w[8];
    pack(w, reduce<FrP>(a));
    for (uint32_t i = q; i < nbits; i += 4) {
      Fe b = fe_zero();
      b.v[0] = (w[i >> 5] >> (i & 31)) & 1;
      st_canon(z, out + i, b);
    }
    return;
  }
  if (q != 0) return;
  if (kind == WP_MUL) {
    const Fe b = eval_lc(terms, op.w, blen, coeff_m, z);
    st_canon(z, out, mul<FrP>(mul<FrP>(a, fe_const<FrP>(FrP::R2)), b));
  } else if (kind == WP_NZ) {
    const Fe ar = reduce<FrP>(a);
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) nz |= ar.v[i];
    Fe ne = fe_zero();
    ne.v[0] = nz != 0;
    st_canon(z, out, ne);
  } else if (kind == WP_INV || kind == WP_INV1) {
    // r - 2 (Fermat); 0 stays 0 (INV) or becomes 1 (INV1)
    const uint64_t e[4] = {0x43e1f593efffffffULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                           0x30644e72e131a029ULL};
    const Fe am = mul<FrP>(a, fe_const<FrP>(FrP::R2));
    Fe inv = redc_fr(reduce<FrP>(pow_w3(am, e)));
    if (kind == WP_INV1) {
      uint32_t nz = 0;
#pragma unroll
      for (int i = 0; i < NL; i++) nz |= inv.v[i];
      if (!nz) inv.v[0] = 1;
    }
    st_canon(z, out, inv);
  }
}

template <bool POS>
__global__ void __launch_bounds__(256) k_wprog_level(const uint4* __restrict__ ops, uint32_t lo, uint32_t hi,
                                                     const uint2* __restrict__ terms,
                                                     const uint32_t* __restrict__ coeff_m,
                                                     const uint32_t* __restrict__ rc_m, uint32_t* __restrict__ z,
                                                     size_t zstride) {
  z += blockIdx.y * zstride;  // batch blockIdx.y of a multi-batch run
  // Round constants in LDS: a global load inside the round loop would make
  // every round wait (vmcnt) for the previous round's stores to land.
  __shared__ uint32_t rc_s[MIMC_R * 8];
  __shared__ Fe pc_s[POS ? POS_NCONST : 1];  // Poseidon constants, unpacked Montgomery
  for (uint32_t i = threadIdx.x; i < MIMC_R * 8; i += blockDim.x) rc_s[i] = rc_m[i];
  if constexpr (POS)
    for (uint32_t i = threadIdx.x; i < POS_NCONST; i += blockDim.x) pc_s[i] = ld_canon(coeff_m, i);
  __syncthreads();
  // The program runs beside a proof whose MSM waves fill the same SIMDs:
  // top wave priority wins the VALU arbitration for this latency-critical
  // chain (a handful of waves against the proof's thousands)
  __builtin_amdgcn_s_setprio(3);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t op_i = lo + (t >> 2), q = t & 3;
  if (op_i >= hi) return;
  wprog_op<POS>(op_i, q, ops, terms, coeff_m, rc_s, pc_s, z);
}

// A run of consecutive small levels without permutations (the comparison
// gadgets' MUL / NZ chains: dozens of levels of a few ops each) in ONE
// launch: one 1024-thread workgroup per batch steps through the levels with a
// barrier between them (global stores of a level are visible to the whole
// workgroup after it), instead of one launch per level.
__global__ void __launch_bounds__(1024) k_wprog_chain(const uint4* __restrict__ ops,
                                                      const uint32_t* __restrict__ level_start, uint32_t l0,
                                                      uint32_t l1, const uint2* __restrict__ terms,
                                                      const uint32_t* __restrict__ coeff_m,
                                                      const uint32_t* __restrict__ rc_m, uint32_t* __restrict__ z,
                                                      size_t zstride) {
  z += blockIdx.y * zstride;
  __shared__ uint32_t rc_s[MIMC_R * 8];
  for (uint32_t i = threadIdx.x; i < MIMC_R * 8; i += blockDim.x) rc_s[i] = rc_m[i];
  __builtin_amdgcn_s_setprio(3);
  for (uint32_t l = l0; l < l1; l++) {
    __syncthreads();
    const uint32_t lo = level_start[l], hi = level_start[l + 1];
    for (uint32_t op_i = lo + (threadIdx.x >> 2); op_i < hi; op_i += blockDim.x >> 2)
      wprog_op<false>(op_i, threadIdx.x & 3, ops, terms, coeff_m, rc_s, nullptr, z);
  }
}

// Montgomery -> canonical for the first 4*91 - 1 trace values of every
// permutation (the last one, its output, is stored canonical)
__global__ void __launch_bounds__(256) k_wprog_canon(const uint32_t* __restrict__ perm_out, uint32_t nperm,
                                                     uint32_t* __restrict__ z, size_t zstride) {
  constexpr uint32_t PER = 4 * MIMC_R - 1;
  z += blockIdx.y * zstride;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nperm * PER) return;
  const uint32_t var = perm_out[i / PER] + i % PER;
  st_canon(z, var, redc_fr(ld_canon(z, var)));
}

// Montgomery -> canonical for a list of variables (Poseidon traces)
__global__ void __launch_bounds__(256) k_wprog_canon_vars(const uint32_t* __restrict__ vars, uint32_t n,
                                                          uint32_t* __restrict__ z, size_t zstride) {
  z += blockIdx.y * zstride;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_canon(z, vars[i], redc_fr(ld_canon(z, vars[i])));
}

__global__ void __launch_bounds__(256) k_wprog_inputs(const uint32_t* __restrict__ in, const uint32_t* __restrict__ var,
                                                      uint32_t n, uint32_t* __restrict__ z, size_t zstride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  z += blockIdx.y * zstride;
  in += (size_t)blockIdx.y * n * 8;
  if (i >= n) return;
  const uint4* s = reinterpret_cast<const uint4*>(in + (size_t)i * 8);
  uint4* d = reinterpret_cast<uint4*>(z + (size_t)var[i] * 8);
  d[0] = s[0];
  d[1] = s[1];
}

// canonical -> packed Montgomery (R = 2^261)
__global__ void __launch_bounds__(256) k_wprog_to_mont(uint32_t* __restrict__ v, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  for (int k = 0; k < 8; k++) w[k] = v[(size_t)i * 8 + k];
  pack(w, reduce<FrP>(mul<FrP>(unpack(w), fe_const<FrP>(FrP::R2))));
  for (int k = 0; k < 8; k++) v[(size_t)i * 8 + k] = w[k];
}

}  // namespace zk

struct zkmi_wprog {
  zkmi_ctx* ctx = nullptr;  // null once the context is destroyed (wprog_detach_all): the program is then only freed
  int device = 0;
  size_t num_vars = 0, num_inputs = 0;
  uint32_t *d_input_var = nullptr, *d_coeff = nullptr, *d_rc = nullptr, *d_in = nullptr;
  uint4* d_ops = nullptr;
  uint2* d_terms = nullptr;
  uint32_t* d_perm_out = nullptr;  // first trace variable of every permutation
  uint32_t* d_level_start = nullptr;
  uint32_t* d_raw = nullptr;  // Poseidon trace variables stored in Montgomery form
  uint32_t num_raw = 0;
  uint32_t num_perms = 0;
  std::vector<uint32_t> level_start;  // host: op ranges per level
  std::vector<uint32_t> op_kinds;     // host: kinds (level geometry)
  hipStream_t st = nullptr;           // the witness stream
  hipEvent_t done = nullptr, ctx_mark = nullptr;
  bool have_mark = false;
  uint64_t* h_in[2] = {nullptr, nullptr};  // pinned staging of the inputs (alternating)
  hipEvent_t in_done[2] = {nullptr, nullptr};
  int next_in = 0;
  size_t in_cap = 1;  // batches h_in / d_in hold
};

namespace zk {
// Release a program's own stream (after its work): called for every program
// of a context when a communicator is created (stream budget),
// so the context never holds a fifth stream beside context + 2 lanes + the
// RCCL stream; later runs go to the context stream (wprog_stream).
static void wprog_drop_stream(zkmi_wprog* p) {
  if (!p->st) return;
  (void)hipStreamSynchronize(p->st);
  (void)hipStreamDestroy(p->st);
  p->st = nullptr;
  if (p->ctx) p->ctx->nstreams--;
}
void wprog_release_streams(zkmi_ctx* ctx) {
  for (zkmi_wprog* p : ctx->wprogs) wprog_drop_stream(p);
}
// zkmi_ctx_destroy with programs still alive (a caller may free its context
// before its programs, e.g. a garbage collector's order): their streams go
// with the context and they forget it, so a later zkmi_wprog_destroy only
// frees the program's own buffers (on its device).
void wprog_detach_all(zkmi_ctx* ctx) {
  for (zkmi_wprog* p : ctx->wprogs) {
    wprog_drop_stream(p);
    p->ctx = nullptr;
  }
  ctx->wprogs.clear();
}
static void wprog_free(zkmi_wprog* p) {
  if (!p) return;
  // runs may sit on the program's stream and (beside a communicator, or after
  // its stream was released) on the context stream: both drain before the
  // buffers go
  if (p->st) (void)hipStreamSynchronize(p->st);
  if (p->ctx) {
    (void)hipStreamSynchronize(p->ctx->stream);
    auto& reg = p->ctx->wprogs;
    reg.erase(std::remove(reg.begin(), reg.end(), p), reg.end());
  }
  (void)hipFree(p->d_input_var);
  (void)hipFree(p->d_coeff);
  (void)hipFree(p->d_rc);
  (void)hipFree(p->d_in);
  (void)hipFree(p->d_ops);
  (void)hipFree(p->d_terms);
  (void)hipFree(p->d_perm_out);
  (void)hipFree(p->d_level_start);
  (void)hipFree(p->d_raw);
  for (int b = 0; b < 2; b++) {
    if (p->h_in[b]) (void)hipHostFree(p->h_in[b]);
    if (p->in_done[b]) (void)hipEventDestroy(p->in_done[b]);
  }
  if (p->done) (void)hipEventDestroy(p->done);
  if (p->ctx_mark) (void)hipEventDestroy(p->ctx_mark);
  wprog_drop_stream(p);
  delete p;
}

// The stream a run goes on: its own highest-priority stream (the program is a
// chain of ~140 small launches that must get onto CUs between the blocks of
// the proof running beside it), made at the first run -- or, while a
// communicator exists on the context, the context stream (stream budget,
// no fifth stream beside context + 2 lanes + the RCCL stream).
static int wprog_stream(zkmi_ctx* ctx, zkmi_wprog* p, hipStream_t* st) {
  if (ctx->ncomm > 0) {
    wprog_drop_stream(p);  // (released at zkmi_comm_init already; kept for safety)
    *st = ctx->stream;
    return 0;
  }
  if (!p->st) {
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithPriority(&p->st, hipStreamNonBlocking, prio_hi) != hipSuccess) {
      (void)hipGetLastError();
      p->st = nullptr;
      set_error("zkmi_wprog_run: cannot create the program's stream");
      return ZKMI_EHIP;
    }
    ctx->nstreams++;
  }
  *st = p->st;
  return 0;
}
}  // namespace zk

using namespace zk;

extern "C" {

int zkmi_wprog_create(zkmi_ctx* ctx, const zkmi_wprog_desc* d, zkmi_wprog** out) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !d || !out || !d->num_vars || !d->num_inputs || !d->input_var || (d->num_ops && !d->op) ||
      !d->level_start || !d->num_coeffs || !d->coeff) {
    set_error("zkmi_wprog_create: bad arguments");
    return ZKMI_EINVAL;
  }
  // validate on the host: every index in range, levels cover the ops
  if (d->level_start[0] != 0 || d->level_start[d->num_levels] != d->num_ops) {
    set_error("zkmi_wprog_create: levels do not cover the ops");
    return ZKMI_EINVAL;
  }
  for (size_t l = 0; l < d->num_levels; l++)
    if (d->level_start[l] > d->level_start[l + 1]) {
      set_error("zkmi_wprog_create: level starts not monotone");
      return ZKMI_EINVAL;
    }
  for (size_t i = 0; i < d->num_inputs; i++)
    if (d->input_var[i] >= d->num_vars) {
      set_error("zkmi_wprog_create: input %zu outside z", i);
      return ZKMI_EINVAL;
    }
  for (size_t i = 0; i < d->num_terms; i++)
    if (d->term[2 * i] >= d->num_vars || d->term[2 * i + 1] >= d->num_coeffs) {
      set_error("zkmi_wprog_create: term %zu out of range", i);
      return ZKMI_EINVAL;
    }
  std::vector<uint32_t> kinds(d->num_ops);
  for (size_t i = 0; i < d->num_ops; i++) {
    const uint32_t* o = d->op + 4 * i;
    const uint32_t kind = o[0] & 0xFF, alen = (o[0] >> 8) & 0xFFF, blen = o[0] >> 20;
    bool ok = kind >= WP_MUL && kind <= WP_INV1;
    uint64_t span = 1;
    if (kind == WP_POSEIDON) {
      const uint32_t l2 = o[3] & 0xFFFF, mask = o[3] >> 16;
      span = poseidon_trace_len(mask);
      ok = ok && kind != 0 && mask >= 1 && mask <= 7 && l2 < 4096 && (uint64_t)o[2] + alen + blen + l2 <= d->num_terms &&
           d->num_coeffs >= (size_t)POS_NCONST;
    } else {
      span = kind == WP_PERM ? 4 * MIMC_R : kind == WP_BITS64 ? 64 : kind == WP_BITS ? o[3] : 1;
      ok = ok && (uint64_t)o[2] + alen <= d->num_terms && (kind == WP_MUL ? (uint64_t)o[3] + blen <= d->num_terms : !blen) &&
           (kind != WP_BITS || (o[3] >= 1 && o[3] <= 256));
    }
    if (!ok || o[1] + span > d->num_vars) {
      set_error("zkmi_wprog_create: op %zu malformed", i);
      return ZKMI_EINVAL;
    }
    kinds[i] = kind;
  }
  for (size_t i = 0; i < d->num_coeffs; i++) {
    const uint64_t* c = d->coeff + 4 * i;
    // < r (canonical)
    const uint64_t R[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                           0x30644e72e131a029ULL};
    bool lt = false;
    for (int k = 3; k >= 0; k--)
      if (c[k] != R[k]) {
        lt = c[k] < R[k];
        break;
      }
    if (!lt) {
      set_error("zkmi_wprog_create: coefficient %zu not reduced", i);
      return ZKMI_EINVAL;
    }
  }
  zkmi_wprog* p = new zkmi_wprog;
  p->ctx = ctx;
  p->device = ctx->device;
  ctx->wprogs.push_back(p);
  p->num_vars = d->num_vars;
  p->num_inputs = d->num_inputs;
  p->level_start.assign(d->level_start, d->level_start + d->num_levels + 1);
  p->op_kinds = kinds;
  auto fail = [&](const char* what) {
    (void)hipGetLastError();
    set_error("zkmi_wprog_create: %s", what);
    wprog_free(p);
    return ZKMI_EHIP;
  };
  if (hipEventCreateWithFlags(&p->done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ctx_mark, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->in_done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->in_done[1], hipEventDisableTiming) != hipSuccess)
    return fail("stream / events");
  std::vector<uint32_t> perm_out;
  for (size_t i = 0; i < d->num_ops; i++)
    if (kinds[i] == WP_PERM) perm_out.push_back(d->op[4 * i + 1]);
  // Poseidon traces are stored in Montgomery form but for the last round's
  // x^5 values; no op may read the others
  std::vector<uint32_t> raw;
  {
    std::vector<uint8_t> is_raw(d->num_vars, 0);
    for (size_t i = 0; i < d->num_ops; i++) {
      if (kinds[i] != WP_POSEIDON) continue;
      const uint32_t out = d->op[4 * i + 1], len = poseidon_trace_len(d->op[4 * i + 3] >> 16);
      for (uint32_t k = 0; k < len; k++) {
        const bool final_x5 = k >= len - 9 && (k - (len - 9)) % 3 == 2;
        if (!final_x5) {
          is_raw[out + k] = 1;
          raw.push_back(out + k);
        }
      }
    }
    for (size_t i = 0; i < d->num_terms && !raw.empty(); i++)
      if (is_raw[d->term[2 * i]]) {
        set_error("zkmi_wprog_create: term %zu reads a Poseidon trace value other than the output round's x^5", i);
        wprog_free(p);
        return ZKMI_EINVAL;
      }
  }
  p->num_perms = (uint32_t)perm_out.size();
  const size_t ni = d->num_inputs, no = std::max<size_t>(1, d->num_ops), nt = std::max<size_t>(1, d->num_terms);
  if (hipMalloc(&p->d_perm_out, std::max<size_t>(1, perm_out.size()) * 4) != hipSuccess ||
      (!perm_out.empty() && hipMemcpy(p->d_perm_out, perm_out.data(), perm_out.size() * 4, hipMemcpyHostToDevice) !=
                                hipSuccess))
    return fail("permutation list");
  p->num_raw = (uint32_t)raw.size();
  if (hipMalloc(&p->d_raw, std::max<size_t>(1, raw.size()) * 4) != hipSuccess ||
      (!raw.empty() && hipMemcpy(p->d_raw, raw.data(), raw.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
    return fail("Poseidon trace list");
  if (hipMalloc(&p->d_level_start, (d->num_levels + 1) * 4) != hipSuccess ||
      hipMemcpy(p->d_level_start, d->level_start, (d->num_levels + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
    return fail("level list");
  if (hipMalloc(&p->d_input_var, ni * 4) != hipSuccess || hipMalloc(&p->d_in, ni * 32) != hipSuccess ||
      hipMalloc(&p->d_ops, no * 16) != hipSuccess || hipMalloc(&p->d_terms, nt * 8) != hipSuccess ||
      hipMalloc(&p->d_coeff, d->num_coeffs * 32) != hipSuccess || hipMalloc(&p->d_rc, MIMC_R * 32) != hipSuccess ||
      hipHostMalloc(&p->h_in[0], ni * 32, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&p->h_in[1], ni * 32, hipHostMallocDefault) != hipSuccess)
    return fail("allocation");
  // MiMC round constants c_i = (i+1)^3 + (i+1) (poseidon.nr:15-56)
  uint64_t rc[MIMC_R * 4] = {0};
  for (int i = 0; i < MIMC_R; i++) rc[4 * i] = (uint64_t)(i + 1) * (i + 1) * (i + 1) + (i + 1);
  hipStream_t st = ctx->stream;  // the run stream is made at the first run (wprog_stream)
  if (hipMemcpyAsync(p->d_input_var, d->input_var, ni * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      (d->num_ops && hipMemcpyAsync(p->d_ops, d->op, d->num_ops * 16, hipMemcpyHostToDevice, st) != hipSuccess) ||
      (d->num_terms && hipMemcpyAsync(p->d_terms, d->term, d->num_terms * 8, hipMemcpyHostToDevice, st) != hipSuccess) ||
      hipMemcpyAsync(p->d_coeff, d->coeff, d->num_coeffs * 32, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(p->d_rc, rc, sizeof(rc), hipMemcpyHostToDevice, st) != hipSuccess)
    return fail("upload");
  k_wprog_to_mont<<<(unsigned)((d->num_coeffs + 255) / 256), 256, 0, st>>>(p->d_coeff, (uint32_t)d->num_coeffs);
  k_wprog_to_mont<<<1, 256, 0, st>>>(p->d_rc, MIMC_R);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return fail("init kernels");
  *out = p;
  return 0;
}

void zkmi_wprog_destroy(zkmi_wprog* p) {
  if (!p) return;
  ::zk::DeviceGuard guard(p->device);  // (the context may be gone: wprog_detach_all)
  wprog_free(p);
}

int zkmi_wprog_run_many(zkmi_ctx* ctx, zkmi_wprog* p, size_t nb, const uint64_t* inputs, void* d_z,
                        size_t z_stride, int async) {
  ZK_DEVICE_GUARD(ctx);
  if (!ctx || !p || !inputs || !d_z || p->ctx != ctx || nb == 0 || nb > 65535 ||
      (nb > 1 && (z_stride < p->num_vars * 32 || z_stride % 32))) {
    set_error("zkmi_wprog_run: bad arguments");
    return ZKMI_EINVAL;
  }
  hipStream_t st;
  ZK_TRY(wprog_stream(ctx, p, &st));
  // The z this run writes was last read by context work enqueued before the
  // previous run (callers alternate two z buffers / buffer sets): wait for
  // exactly that, so this run overlaps the previous batches' proofs.
  // Synchronous runs wait for the whole context first.
  if (!async) ZK_TRY(ctx_sync_all(ctx));
  const size_t in_bytes = p->num_inputs * 32;
  if (nb > p->in_cap) {  // grow the input staging (both halves idle after these waits)
    ZK_HIP(hipEventSynchronize(p->in_done[0]));
    ZK_HIP(hipEventSynchronize(p->in_done[1]));
    ZK_HIP(hipStreamSynchronize(st));
    for (int b = 0; b < 2; b++) {
      ZK_HIP(hipHostFree(p->h_in[b]));
      p->h_in[b] = nullptr;
    }
    ZK_HIP(hipFree(p->d_in));
    p->d_in = nullptr;
    if (hipHostMalloc(&p->h_in[0], nb * in_bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&p->h_in[1], nb * in_bytes, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&p->d_in, nb * in_bytes) != hipSuccess) {
      (void)hipGetLastError();
      set_error("zkmi_wprog_run: cannot allocate input staging for %zu batches", nb);
      return ZKMI_ENOMEM;
    }
    p->in_cap = nb;
  }
  const int b = p->next_in;
  p->next_in ^= 1;
  ZK_HIP(hipEventSynchronize(p->in_done[b]));  // that staging buffer's last upload has landed
  memcpy(p->h_in[b], inputs, nb * in_bytes);
  if (p->have_mark) ZK_HIP(hipStreamWaitEvent(st, p->ctx_mark, 0));
  uint32_t* z = (uint32_t*)d_z;
  const size_t zs = nb > 1 ? z_stride / 4 : 0;  // words
  const unsigned nby = (unsigned)nb;
  ScopedKernelTimer tm(ctx, "wprog", st);
  ZK_HIP(hipMemcpyAsync(p->d_in, p->h_in[b], nb * in_bytes, hipMemcpyHostToDevice, st));
  ZK_HIP(hipEventRecord(p->in_done[b], st));
  k_wprog_inputs<<<dim3((unsigned)((p->num_inputs + 255) / 256), nby), 256, 0, st>>>(
      p->d_in, p->d_input_var, (uint32_t)p->num_inputs, z, zs);
  const size_t nl = p->level_start.size() - 1;
  // chainable: no permutation (they sort first in their level), one pass of
  // a 1024-thread workgroup
  auto chainable = [&](size_t l) {
    const uint32_t lo = p->level_start[l], hi = p->level_start[l + 1];
    return hi > lo && hi - lo <= 256 && p->op_kinds[lo] != WP_PERM && p->op_kinds[lo] != WP_POSEIDON;
  };
  for (size_t l = 0; l < nl;) {
    const uint32_t lo = p->level_start[l], hi = p->level_start[l + 1];
    if (hi == lo) {
      l++;
      continue;
    }
    size_t l1 = l;
    while (l1 < nl && chainable(l1)) l1++;
    if (l1 - l >= 2) {
      k_wprog_chain<<<dim3(1, nby), 1024, 0, st>>>(p->d_ops, p->d_level_start, (uint32_t)l, (uint32_t)l1, p->d_terms,
                                                   p->d_coeff, p->d_rc, z, zs);
      l = l1;
      continue;
    }
    const size_t threads = (size_t)(hi - lo) * 4;
    auto kern = p->op_kinds[lo] == WP_POSEIDON ? k_wprog_level<true> : k_wprog_level<false>;
    kern<<<dim3((unsigned)((threads + 255) / 256), nby), 256, 0, st>>>(p->d_ops, lo, hi, p->d_terms, p->d_coeff,
                                                                       p->d_rc, z, zs);
    l++;
  }
  if (p->num_perms) {
    const size_t nconv = (size_t)p->num_perms * (4 * MIMC_R - 1);
    k_wprog_canon<<<dim3((unsigned)((nconv + 255) / 256), nby), 256, 0, st>>>(p->d_perm_out, p->num_perms, z, zs);
  }
  if (p->num_raw)
    k_wprog_canon_vars<<<dim3((p->num_raw + 255) / 256, nby), 256, 0, st>>>(p->d_raw, p->num_raw, z, zs);
  ZK_HIP(hipGetLastError());
  ZK_HIP(hipEventRecord(p->done, st));
  // later context work (the proofs over these z) waits for the witness
  ZK_HIP(hipStreamWaitEvent(ctx->stream, p->done, 0));  // MSM lanes fork from the context stream
  // everything enqueued on the context so far (the previous proofs, which
  // read the other z buffers) must finish before the NEXT run writes them
  ZK_HIP(hipEventRecord(p->ctx_mark, ctx->stream));
  p->have_mark = true;
  if (!async) {
    ZK_HIP(hipStreamSynchronize(st));
    return timer_flush(ctx);
  }
  return 0;
}

int zkmi_wprog_run(zkmi_ctx* ctx, zkmi_wprog* p, const uint64_t* inputs, void* d_z, int async) {
  return zkmi_wprog_run_many(ctx, p, 1, inputs, d_z, 0, async);
}

}  // extern "C"
