// ntt.hip — radix-2 NTT over BN254 Fr for gfx950.  Replaces ark-poly 0.5.0
// Radix2EvaluationDomain::{fft,ifft}_in_place and the coset variants used by
// ark-groth16's witness map.  Semantics (natural order
// in and out, omega_n = 5^((r-1)/2^28)^(2^28/n), coset offset g = 5, ifft
// scaled by n^-1) are exactly arkworks'; field results are exact, so any
// correct schedule is bit-identical.
//
// Schedule: log2(n) butterfly stages are cut into groups of <= 8 stages.  One
// workgroup loads 2048 elements (8 independent 256-point sub-transforms whose
// columns are adjacent in memory -> 256-B coalesced bursts), runs its stages
// out of LDS (72 KB in the unpacked 9 x 29-bit form, two workgroups per CU),
// and writes back.  Twiddles come from a per-size table omega^e resident in
// HBM (n/2 entries) instead of being recomputed (1 mul saved per butterfly;
// the kernel is VALU-bound, bytes are cheap).  Forward = DIF (natural ->
// bit-reversed) + tiled LDS bit-reversal; the witness map chains DIF/DIT so it
// never needs the permutation.
#include <string.h>

#include <algorithm>

#include "dev_io.h"
#include "zkmi_internal.h"

namespace zk {

__constant__ uint32_t W28[8] = {0x725b19f0u, 0x9bd61b6eu, 0x41112ed4u, 0x402d111eu,
                                0x8ef62abcu, 0x00e0a7ebu, 0xa58a7e85u, 0x2a3c09f0u};
__constant__ uint32_t W28I[8] = {0x9d18157eu, 0x72394277u, 0xfd399d5du, 0xec9d51f8u,
                                 0x49d5387fu, 0x6117635du, 0x9c229cd5u, 0x01b77519u};

__device__ __forceinline__ Fe mont_from_canon(const uint32_t* c) { return to_mont<FrP>(ldc_fe(c)); }

// root of unity of order 2^logn (Montgomery), inverse if inv
__device__ Fe root_of_unity(uint32_t logn, bool inv) {
  Fe w = mont_from_canon(inv ? W28I : W28);
  for (uint32_t i = logn; i < 28; i++) w = sqr<FrP>(w);
  return w;
}
__device__ Fe fe_pow_u64(Fe base, uint64_t e) {
  Fe r = one<FrP>();
  while (e) {
    if (e & 1) r = mul<FrP>(r, base);
    base = sqr<FrP>(base);
    e >>= 1;
  }
  return r;
}

// Twiddle table omega^e, e < half, reduced, stored UNPACKED (9 x 29-bit limbs)
// in two planes so the butterflies skip the 8 -> 9 limb unpack: limbs 0..7
// at tw[8e..8e+8) (two 16-B loads), limb 8 at tw[8 half + e].
//
// ZK_NTT_STAGE_TW: the table is stage-major instead: 2 half slots, slot
// h + i (h a power of two <= half, i < h) = omega_{2h}^i, the twiddle of pair
// i of a stage with pair distance h; limbs 0..7 at tw[8 slot], limb 8 at
// tw[16 half + slot].  Slots [half, 2 half) are the plain table.  A stage
// with distance h then reads h contiguous slots instead of every (half/h)-th
// entry of the plain table, whose 36-B entries at strides >= 64 B pulled a
// whole line per twiddle: ~1.1 GB of twiddle fetch in the first pass of a
// 2^24 transform against ~0.6 GB stage-major.  Measured (round 6, one box,
// 3 interleaved repeats, tools/r06_ntt_ab.sh): 2^24 NTT+INTT 3.91-3.97 ->
// 3.74 ms, 2^22 1.00 -> 0.97-0.98 ms.  Twice the table memory (n x 36 B).
#ifndef ZK_NTT_STAGE_TW
#define ZK_NTT_STAGE_TW 1
#endif
__device__ __forceinline__ Fe ld_tw_slot(const uint32_t* __restrict__ tw, uint64_t l8, uint64_t slot) {
  const uint4* p = reinterpret_cast<const uint4*>(tw + slot * 8);
  const uint4 a = p[0], b = p[1];
  return Fe{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, tw[l8 + slot]}};
}
// (small transforms only: log n < 11, no limb-8 permutation)
__device__ __forceinline__ Fe ld_tw(const uint32_t* __restrict__ tw, uint64_t half, uint64_t e) {
  if (ZK_NTT_STAGE_TW) return ld_tw_slot(tw, 16 * half, half + e);
  return ld_tw_slot(tw, 8 * half, e);
}
static constexpr uint64_t ntt_tw_words(uint64_t half) { return (ZK_NTT_STAGE_TW ? 2 : 1) * half * 9; }
// ZK_NTT_TW_L8P: limb 8 of the outermost group's stages (pair distance h >=
// 2^cb0, cb0 = log n - k0, k0 = that group's stage count) is stored
// workgroup-major.  Such a stage's pair i = col + jj 2^cb0 (col < 2^cb0) is
// read by the workgroup of columns col >> L (L = 10 - k0, 2^L adjacent
// columns per 1024-element tile); its limb-8 word goes to slot position
// h + (((col >> L) (h >> cb0) + jj) << L) + (col mod 2^L), so one workgroup's
// limb-8 words of a stage are contiguous (2 KB) instead of 16 B per 128-B
// line.  Limbs 0..7 are 4 adjacent slots = one full line either way.
// Measured (round 6, one box, 3 interleaved repeats): first-pass fetch at
// 2^24 1.61 -> 1.14 GB (PMC, FETCH_SIZE x 2), 2^24 NTT+INTT 3.80-3.81 ->
// 3.79-3.80 ms, 2^22 0.978-0.987 -> 0.971-0.975 ms: the pass is issue-bound
// (0.84-0.86), so the bytes saved show little in its time.
#ifndef ZK_NTT_TW_L8P
#define ZK_NTT_TW_L8P 1
#endif
__host__ __device__ __forceinline__ uint64_t ntt_l8_pos(uint64_t h, uint64_t i, uint32_t cb0, uint32_t L) {
  if (!ZK_NTT_TW_L8P || !ZK_NTT_STAGE_TW || cb0 == 0 || h < (1ull << cb0)) return h + i;
  const uint64_t col = i & ((1ull << cb0) - 1), jj = i >> cb0;
  return h + ((((col >> L) * (h >> cb0)) + jj) << L) + (col & ((1ull << L) - 1));
}
// twiddle of pair i < h of a stage with pair distance h (= omega_n^(i half / h));
// l8: the slot of its limb 8 (ntt_l8_pos; h + i outside the outermost group)
__device__ __forceinline__ Fe ld_tw_stage(const uint32_t* __restrict__ tw, uint32_t half, uint32_t h, uint32_t i,
                                          uint32_t l8) {
  if (ZK_NTT_STAGE_TW) {
    const uint4* p = reinterpret_cast<const uint4*>(tw + (size_t)(h + i) * 8);
    const uint4 a = p[0], b = p[1];
    return Fe{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, tw[(size_t)16 * half + l8]}};
  }
  return ld_tw_slot(tw, 8 * (uint64_t)half, (uint64_t)i * (half / h));
}
// Each thread: one pow + 63 muls for a run of 64.
__global__ void __launch_bounds__(256) k_ntt_twiddles(uint32_t* __restrict__ tw, uint32_t logn, int inv, uint64_t half,
                                                      uint32_t cb0, uint32_t L) {
  uint64_t run = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t e0 = run * 64;
  if (e0 >= half) return;
  Fe w = root_of_unity(logn, inv != 0);
  Fe cur = fe_pow_u64(w, e0);
  const uint64_t s0 = ZK_NTT_STAGE_TW ? half : 0, l8 = ZK_NTT_STAGE_TW ? 16 * half : 8 * half;
  for (int k = 0; k < 64 && e0 + k < half; k++) {
    const Fe v = reduce<FrP>(cur);
#pragma unroll
    for (int l = 0; l < 8; l++) tw[(s0 + e0 + k) * 8 + l] = v.v[l];
    tw[l8 + (ZK_NTT_STAGE_TW ? ntt_l8_pos(half, e0 + k, cb0, L) : e0 + k)] = v.v[8];
    cur = mul<FrP>(cur, w);
  }
}
// stage-major slots [1, half) from the plain slots [half, 2 half)
__global__ void __launch_bounds__(256) k_ntt_tw_levels(uint32_t* __restrict__ tw, uint64_t half, uint32_t cb0,
                                                       uint32_t L) {
  const uint64_t slot = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (slot == 0 || slot >= half) return;
  const uint64_t h = 1ull << (63 - __clzll((long long)slot)), e = (slot - h) * (half / h);
#pragma unroll
  for (int l = 0; l < 8; l++) tw[slot * 8 + l] = tw[(half + e) * 8 + l];
  tw[16 * half + ntt_l8_pos(h, slot - h, cb0, L)] = tw[16 * half + ntt_l8_pos(half, e, cb0, L)];
}

// One group of `k` <= 8 stages over a tile of 2048 elements.  Sub-transform
// q -> (blk, col): col = q mod 2^(a-k), blk = q / 2^(a-k); its element j lives
// at blk*2^a + col + j*2^(a-k).  Tile index e = j*2^lsub + s (lsub = 11-k,
// s = sub-transform within the workgroup, q = blockIdx*2^lsub + s), so the 2^lsub
// adjacent columns of one j form a contiguous 2^lsub*32-B burst in HBM.
// DIT=false: DIF stages m = 2^a .. 2^(a-k+1); DIT=true: m = 2^(a-k+1) .. 2^a.
//
// Radix-8 rounds: every thread holds 8 elements in registers -- the tile
// indices base | t<<lo, t < 8 -- and runs up to three stages on them (12
// butterflies, 4 independent multiplies per stage for ILP).  Rounds meet in
// LDS (limb-major, XOR-swizzled so every wave's 64 lanes hit 64 banks), so a
// group of 8 stages costs 2 LDS exchanges instead of 8 read/write passes.  The
// first round loads straight from HBM and the last stores straight back.
constexpr int NTT_TILE = 2048;

__device__ __forceinline__ uint32_t ntt_slot(uint32_t e) {
  uint32_t h = (e >> 6) & 7;
  return e ^ h ^ (h << 3);
}

struct NttGroup {
  uint32_t logn, a, lsub, smask, colbits, colmask, q0, qsh;
  // sub-transform s of this workgroup is q = q0 + (s << qsh): qsh = 0 packs
  // adjacent columns (coalesced reads); the permuting last pass takes
  // sub-transforms 2^qsh blocks apart so that its natural-order writes land
  // on 2^lsub adjacent elements
  __device__ __forceinline__ size_t gidx(uint32_t e) const {
    uint32_t q = q0 + ((e & smask) << qsh), j = e >> lsub;
    return ((size_t)(q >> colbits) << a) + (q & colmask) + ((size_t)j << colbits);
  }
};

// Lazy DIF sums.  A DIF butterfly's sum x0 = u + v needs no reduction until
// the round's elements are stored: x0 is a limb-wise add (9 ops instead of two
// carry chains), and the difference takes a bias K r >= v in one signed-carry
// pass before its multiplication.  Every element carries a bound (value < b r,
// limbs < l 2^29) that is a compile-time constant per register slot (the
// stage loops are unrolled), so the bias choice and the end-of-round
// reduction to [0, 2r) fold away: slots above 2r take one quotient-estimate
// pass (fr_reduce_q32, which also normalises), the others at most a carry
// pass.  Bounds: b <= 16 (the sub output stays < 24 r, far inside the
// Montgomery product's 169 r^2), limbs < 2^31 wherever a signed-carry pass
// reads them.
//
// carry-propagate limbs < 2^31 into 29-bit limbs (the top limb keeps the rest)
__device__ __forceinline__ Fe fr_norm(const Fe& x) {
  Fe r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    const uint32_t t = x.v[i] + c;
    r.v[i] = t & LMASK;
    c = t >> 29;
  }
  r.v[NL - 1] = x.v[NL - 1] + c;
  return r;
}
// value < 32 r (limbs < 2^31) -> [0, 2r), normalised, in one pass (ff.h reduce_q32)
__device__ __forceinline__ Fe fr_reduce_q32(const Fe& x) { return reduce_q32<FrP>(x); }
__device__ __forceinline__ int fr_pow2_ceil(int b) { return b <= 2 ? 2 : b <= 4 ? 4 : b <= 8 ? 8 : 16; }

// Lazy DIT sums.  A DIT butterfly adds 2r to the bound of both outputs (x0 =
// u + t, x1 = u - t + 2r, with t = v w < 2r), so the growth over a pass is
// additive: values stay normalised at round ends (LDS) and are reduced once,
// on the pass's last round.  The omega^0 round (round 0 of the innermost
// group, inputs < 2r from HBM) doubles its bounds instead; with <= 8 stages a
// pass ends below 16 + 5 * 2 = 26 r, and one quotient-estimate subtraction
// (fr_reduce_q32) brings it to [0, 2r).  v enters the product < 32 r.
constexpr int NTT_DIT_BOUND = 32;

// TRIV: the round touches stages whose twiddles are omega^0 for every pair p
// with p mod 2^rb == 0 (the register round at tile bit lsub of a group with
// no column bits: the last DIF / first DIT round of the innermost group);
// those multiplications by one are skipped (value form: x * R * R^-1 = x).
template <bool DIT, int R, bool TRIV, int EPT>
__device__ __forceinline__ void ntt_r8_stages(Fe (&x)[EPT], uint32_t base, uint32_t lo, const uint32_t* __restrict__ tw,
                                              const NttGroup& g) {
  constexpr int NP = EPT / 2;  // butterflies per stage per thread
  int bd[EPT], lb[EPT];          // bounds per slot (see "Lazy DIF sums")
#pragma unroll
  for (int t = 0; t < EPT; t++) {
    bd[t] = 2;
    lb[t] = 1;
  }
#pragma unroll
  for (int si = 0; si < R; si++) {
    const int rb = DIT ? si : R - 1 - si;  // register bit of this stage
    const uint32_t lhl = lo + rb - g.lsub;  // j-bit of the pair distance
    const uint32_t sh = g.logn - (g.colbits + lhl + 1);
    const uint64_t half = 1ull << (g.logn - 1);
    // twiddles (unpacked planes).  The twiddle of pair p depends only on the
    // bits of p below rb (the higher ones select slot bits above the pair
    // distance), so a stage loads 2^rb of them, not NP: 3 instead of 4 per
    // radix-4 round.
    Fe w[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
      if (p >= (1 << rb)) continue;
      if (TRIV && (p & ((1 << rb) - 1)) == 0) continue;
      const int t0 = ((p >> rb) << (rb + 1)) | (p & ((1 << rb) - 1));
      const uint32_t e0 = base | ((uint32_t)t0 << lo);
      const uint32_t col = (g.q0 + ((e0 & g.smask) << g.qsh)) & g.colmask;
      const uint32_t jj = (e0 >> g.lsub) & ((1u << lhl) - 1);
      // omega_m^(i mod m/2) = omega_n^((i mod m/2) * n/m)
      const uint32_t h = (uint32_t)(half >> sh), i = col + (jj << g.colbits);
      // outermost group (ntt_l8_pos): pair i = col + jj 2^colbits, h = 2^(colbits + lhl)
      const uint32_t l8 = (ZK_NTT_TW_L8P && g.a == g.logn)
                              ? h + (((((col >> g.lsub) << lhl) | jj) << g.lsub) | (col & g.smask))
                              : h + i;
      w[p] = ld_tw_stage(tw, (uint32_t)half, h, i, l8);
    }
#pragma unroll
    for (int p = 0; p < NP; p++) {
      const int t0 = ((p >> rb) << (rb + 1)) | (p & ((1 << rb) - 1)), t1 = t0 | (1 << rb);
      Fe u = x[t0], v = x[t1];
      const bool one_w = TRIV && (p & ((1 << rb) - 1)) == 0;
      if (DIT) {
        if (lb[t0] > 3) {  // the signed-carry pass below reads u's limbs
          u = fr_norm(u);
          lb[t0] = 1;
        }
        if (one_w) {  // round 0 only: bd[] are the true bounds here
          const int bu = bd[t0], bvt = bd[t1], bv = fr_pow2_ceil(bvt);
          Fe dlt;
          if (bv == 2) dlt = subk<FrP, 2>(u, v);
          else if (bv == 4) dlt = subk<FrP, 4>(u, v);
          else dlt = subk<FrP, 8>(u, v);
          Fe sum = add_lazy(u, v);
          int ls = lb[t0] + lb[t1];
          if (ls > 4) {
            sum = fr_norm(sum);
            ls = 1;
          }
          x[t1] = dlt;
          bd[t1] = bu + bv;
          lb[t1] = 1;
          x[t0] = sum;
          bd[t0] = bu + bvt;
          lb[t0] = ls;
          continue;
        }
        if (lb[t1] > 2) v = fr_norm(v);  // product operand limbs < 2^30
        const Fe t = mul<FrP>(v, w[p & ((1 << rb) - 1)]);
        x[t1] = subk<FrP, 2>(u, t);
        bd[t1] = bd[t0] + 2;
        lb[t1] = 1;
        x[t0] = add_lazy(u, t);
        bd[t0] += 2;
        lb[t0] += 1;
      } else {
        if (lb[t0] > 3) {  // the signed-carry pass below reads u's limbs
          u = fr_norm(u);
          lb[t0] = 1;
        }
        const int bu = bd[t0], bv = fr_pow2_ceil(bd[t1]);
        Fe dlt;
        if (bv == 2) dlt = subk<FrP, 2>(u, v);
        else if (bv == 4) dlt = subk<FrP, 4>(u, v);
        else dlt = subk<FrP, 8>(u, v);
        Fe sum = add_lazy(u, v);
        int ls = lb[t0] + lb[t1];
        if (ls > 4) {
          sum = fr_norm(sum);
          ls = 1;
        }
        x[t0] = sum;
        bd[t0] = bu + bd[t1];
        lb[t0] = ls;
        x[t1] = one_w ? dlt : mul<FrP>(dlt, w[p & ((1 << rb) - 1)]);
        bd[t1] = one_w ? bu + bv : 2;
        lb[t1] = 1;
      }
    }
  }
  if (!DIT) {  // back to normalised [0, 2r) for LDS / HBM
#pragma unroll
    for (int t = 0; t < EPT; t++) {
      if (bd[t] > 2) x[t] = fr_reduce_q32(x[t]);  // also normalises limbs < 2^31
      else if (lb[t] > 1) x[t] = fr_norm(x[t]);
    }
  } else {  // normalised for LDS; k_ntt_group reduces on the pass's last round
#pragma unroll
    for (int t = 0; t < EPT; t++)
      if (lb[t] > 1) x[t] = fr_norm(x[t]);
  }
}

// Element-wise work folded into the first / last pass of a transform (these
// would otherwise be separate HBM-bound passes over the vector):
//   PRO 1: x_i *= g^i = lo[i mod 2^KB] * hi[i >> KB] at natural index i, on
//          the first loads (forward coset; DIF first group reads natural order)
//   EPI 1: x *= c;  EPI 2: x *= lo[i mod 2^KB] * hi[i >> KB], with i the
//          natural index of the element (bit reversal of its DIF position)
//   PERM:  the innermost DIF group writes natural order, out of place, so
//          natural -> natural needs no bit-reversal pass
// Outputs of EPI / PERM passes are fully reduced (canonical).
struct NttIo {
  const uint32_t *lo, *hi, *c;
};
__device__ __forceinline__ Fe ntt_tab_scale(Fe v, uint64_t i, const NttIo& io) {
  v = mul<FrP>(v, ld_fe(io.lo + (i & ((1u << COSET_KB) - 1)) * 8));
  return mul<FrP>(v, ld_fe(io.hi + (i >> COSET_KB) * 8));
}

// TB = log2(tile), RB = log2(elements per thread): (11, 3) = 2048-element
// tiles in radix-8 register rounds (72 KB LDS, 2 waves/SIMD); (10, 2) =
// 1024-element tiles in radix-4 rounds (36 KB LDS, <= 128 VGPRs: 4 waves/SIMD
// to hide the load and twiddle latency the 2-wave form exposes).

template <bool DIT, int PRO, int EPI, bool PERM, int TB, int RB>
__global__ void __launch_bounds__(1 << (TB - RB), (RB == 3 ? 2 : 4) * 256 / (1 << (TB - RB))) k_ntt_group(const uint32_t* src, uint32_t* dst,
                                                                          const uint32_t* __restrict__ tw, uint32_t logn,
                                                                          uint32_t a, uint32_t k, NttIo io) {
  constexpr int TILE = 1 << TB, EPT = 1 << RB;
  extern __shared__ __align__(16) uint32_t lds[];  // [limb][slot]
  NttGroup g;
  g.logn = logn;
  g.a = a;
  g.lsub = TB - k;
  g.smask = (1u << g.lsub) - 1;
  g.colbits = a - k;
  g.colmask = (1u << g.colbits) - 1;
  if (PERM) {  // innermost group: colbits == 0, one block per sub-transform
    g.q0 = blockIdx.x;
    g.qsh = logn - k - g.lsub;
  } else {
    g.q0 = blockIdx.x << g.lsub;
    g.qsh = 0;
  }
  const uint32_t tid = threadIdx.x;
  const uint32_t nr = (k + RB - 1) / RB, rem = k - RB * (nr - 1);
  const bool triv_group = g.colbits == 0;
  Fe x[EPT];
  for (uint32_t r = 0; r < nr; r++) {
    // DIF: stages run high j-bit -> low, the partial round last;
    // DIT: low -> high, the partial round first.
    uint32_t R, b0;
    if (!DIT) {
      R = r == nr - 1 ? rem : RB;
      b0 = TB - RB * r - R;
    } else {
      R = r == 0 ? rem : RB;
      b0 = g.lsub + (r == 0 ? 0 : rem + RB * (r - 1));
    }
    const uint32_t lo = b0;
    const uint32_t base = (tid & ((1u << lo) - 1)) | ((tid >> lo) << (lo + RB));
    if (r == 0) {
#pragma unroll
      for (int t = 0; t < EPT; t++) {
        const size_t gi = g.gidx(base | ((uint32_t)t << lo));
        x[t] = ld_fe(src + gi * 8);
        if (PRO == 1) x[t] = ntt_tab_scale(x[t], gi, io);
      }
    } else {
#pragma unroll
      for (int t = 0; t < EPT; t++) {
        const uint32_t sl = ntt_slot(base | ((uint32_t)t << lo));
#pragma unroll
        for (int l = 0; l < NL; l++) x[t].v[l] = lds[l * TILE + sl];
      }
      __syncthreads();  // every read of this round is done before the next write
    }
    // the round at tile bit lsub of the innermost group has omega^0 pairs
    const bool triv = triv_group && lo == g.lsub;
    if (R == 3) {
      if (triv) ntt_r8_stages<DIT, 3, true, EPT>(x, base, lo, tw, g);
      else ntt_r8_stages<DIT, 3, false, EPT>(x, base, lo, tw, g);
    } else if (R == 2) {
      if (triv) ntt_r8_stages<DIT, 2, true, EPT>(x, base, lo, tw, g);
      else ntt_r8_stages<DIT, 2, false, EPT>(x, base, lo, tw, g);
    } else {
      if (triv) ntt_r8_stages<DIT, 1, true, EPT>(x, base, lo, tw, g);
      else ntt_r8_stages<DIT, 1, false, EPT>(x, base, lo, tw, g);
    }
    if (r == nr - 1) {
#pragma unroll
      for (int t = 0; t < EPT; t++) {
        const size_t gi = g.gidx(base | ((uint32_t)t << lo));
        if (DIT) x[t] = fr_reduce_q32(x[t]);  // lazy DIT sums (< NTT_DIT_BOUND r) -> [0, 2r)
        if (EPI == 0 && !PERM) {
          st_fe(dst + gi * 8, x[t]);
        } else {
          const uint64_t ni = __brev((uint32_t)gi) >> (32 - logn);  // natural index (DIF output)
          Fe v = x[t];
          if (EPI == 1) v = mul<FrP>(v, ld_fe(io.c));
          if (EPI == 2) v = ntt_tab_scale(v, ni, io);
          st_fe(dst + (PERM ? ni : gi) * 8, reduce<FrP>(v));
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < EPT; t++) {
        const uint32_t sl = ntt_slot(base | ((uint32_t)t << lo));
#pragma unroll
        for (int l = 0; l < NL; l++) lds[l * TILE + sl] = x[t].v[l];
      }
      __syncthreads();
    }
  }
}

// small transforms (n < 2048): one workgroup, all stages in LDS
template <bool DIT>
__global__ void __launch_bounds__(256) k_ntt_small(uint32_t* __restrict__ data, const uint32_t* __restrict__ tw,
                                                   uint32_t logn) {
  extern __shared__ __align__(16) uint32_t lds[];
  const uint32_t n = 1u << logn;
  for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
    Fe v = ld_fe(data + (size_t)e * 8);
#pragma unroll
    for (int l = 0; l < NL; l++) lds[e * NL + l] = v.v[l];
  }
  __syncthreads();
  for (uint32_t st = 0; st < logn; st++) {
    uint32_t logm = DIT ? st + 1 : logn - st;
    uint32_t h = 1u << (logm - 1);
    for (uint32_t b = threadIdx.x; b < n / 2; b += blockDim.x) {
      uint32_t i0 = (b / h) * (2 * h) + (b % h), i1 = i0 + h;
      Fe u, v;
#pragma unroll
      for (int l = 0; l < NL; l++) {
        u.v[l] = lds[i0 * NL + l];
        v.v[l] = lds[i1 * NL + l];
      }
      uint32_t te = (i0 & (h - 1)) << (logn - logm);
      Fe w = ld_tw(tw, (uint64_t)n / 2, te);
      Fe x, y;
      if (DIT) {
        Fe t = mul<FrP>(v, w);
        x = add<FrP>(u, t);
        y = sub<FrP>(u, t);
      } else {
        x = add<FrP>(u, v);
        y = mul<FrP>(sub<FrP>(u, v), w);
      }
#pragma unroll
      for (int l = 0; l < NL; l++) {
        lds[i0 * NL + l] = x.v[l];
        lds[i1 * NL + l] = y.v[l];
      }
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
    Fe v;
#pragma unroll
    for (int l = 0; l < NL; l++) v.v[l] = lds[e * NL + l];
    st_fe(data + (size_t)e * 8, v);
  }
}

__device__ __forceinline__ uint32_t brev_bits(uint32_t x, uint32_t bits) { return __brev(x) >> (32 - bits); }

// In-place bit reversal, tiles of 2^(2b) elements through LDS:
// i = (hi:b | mid | lo:b) -> rev(i) = (rev(lo) | rev(mid) | rev(hi)).  The
// workgroup for `mid` swaps tile(mid) with tile(rev(mid)) (or permutes its own
// tile when mid is a palindrome); workgroups with mid > rev(mid) exit.
// Values are fully reduced to [0, r) on the way out.
// Optional scaling of the output element at natural index i (the inverse
// transform's n^-1 and coset factors, folded into this memory-bound pass):
// mode 1: * c; mode 2: * lo[i mod 2^KB] * hi[i >> KB] (Montgomery multipliers).
struct BitrevScale {
  int mode;
  const uint32_t *c, *lo, *hi;
};
__device__ __forceinline__ Fe bitrev_scale(Fe v, uint64_t i, const BitrevScale& sc) {
  if (sc.mode == 1) v = mul<FrP>(v, ld_fe(sc.c));
  else if (sc.mode == 2) {
    v = mul<FrP>(v, ld_fe(sc.lo + (i & ((1u << COSET_KB) - 1)) * 8));
    v = mul<FrP>(v, ld_fe(sc.hi + (i >> COSET_KB) * 8));
  }
  return v;
}
__global__ void __launch_bounds__(256) k_bitrev_tiled(uint32_t* __restrict__ data, uint32_t logn, uint32_t b,
                                                      BitrevScale sc) {
  extern __shared__ __align__(16) uint32_t lds[];  // two tiles [hi][lo][8]
  const uint32_t T = 1u << b, midbits = logn - 2 * b;
  const uint32_t mid = blockIdx.x;
  const uint32_t rmid = midbits ? brev_bits(mid, midbits) : 0;
  if (mid > rmid) return;
  const uint32_t mids[2] = {mid, rmid};
  const int ntile = mid == rmid ? 1 : 2;
  for (int t = 0; t < ntile; t++) {
    for (uint32_t e = threadIdx.x; e < T * T; e += blockDim.x) {
      uint32_t hi = e / T, lo = e % T;
      uint64_t idx = ((uint64_t)hi << (logn - b)) | ((uint64_t)mids[t] << b) | lo;
      const uint4* p = reinterpret_cast<const uint4*>(data + idx * 8);
      uint4 x = p[0], y = p[1];
      uint32_t* d = lds + ((size_t)t * T * T + e) * 8;
      d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
      d[4] = y.x; d[5] = y.y; d[6] = y.z; d[7] = y.w;
    }
  }
  __syncthreads();
  for (int t = 0; t < ntile; t++) {
    // tile t's elements land in tile (rev of mids[t]) = mids[ntile - 1 - t]
    const uint32_t omid = mids[ntile - 1 - t];
    for (uint32_t e = threadIdx.x; e < T * T; e += blockDim.x) {
      uint32_t rlo = e / T, rhi = e % T;  // output (rlo | omid | rhi), rhi contiguous
      uint32_t lo = brev_bits(rlo, b), hi = brev_bits(rhi, b);
      const uint32_t* src = lds + ((size_t)t * T * T + (size_t)hi * T + lo) * 8;
      uint32_t w[8];
#pragma unroll
      for (int l = 0; l < 8; l++) w[l] = src[l];
      uint64_t oidx = ((uint64_t)rlo << (logn - b)) | ((uint64_t)omid << b) | rhi;
      Fe v = reduce<FrP>(bitrev_scale(unpack(w), oidx, sc));
      st_fe(data + oidx * 8, v);
    }
  }
}
__global__ void __launch_bounds__(256) k_bitrev_naive(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      uint32_t logn, BitrevScale sc) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1u << logn)) return;
  uint32_t r = logn ? brev_bits(i, logn) : 0;
  st_fe(out + (size_t)r * 8, reduce<FrP>(bitrev_scale(ld_fe(in + (size_t)i * 8), r, sc)));
}

// data[i] *= g^i in natural order (forward coset), g^i = lo[i mod 2^KB] * hi[i >> KB]
__global__ void __launch_bounds__(256) k_ntt_coset_scale(uint32_t* __restrict__ data, uint32_t logn,
                                                         const uint32_t* __restrict__ lo,
                                                         const uint32_t* __restrict__ hi) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (1ull << logn)) return;
  Fe v = mul<FrP>(ld_fe(data + i * 8), ld_fe(lo + (i & ((1u << COSET_KB) - 1)) * 8));
  st_fe(data + i * 8, mul<FrP>(v, ld_fe(hi + (i >> COSET_KB) * 8)));
}

// x[p] *= lo[i] * hi[i] at natural index i = rev(p), canonical out (small n)
__global__ void __launch_bounds__(256) k_scale_rev_small(uint32_t* __restrict__ data, uint32_t logn,
                                                         const uint32_t* __restrict__ lo,
                                                         const uint32_t* __restrict__ hi) {
  size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (p >= (1ull << logn)) return;
  uint32_t e = logn ? (__brev((uint32_t)p) >> (32 - logn)) : 0;
  Fe v = mul<FrP>(ld_fe(data + p * 8), ld_fe(lo + (size_t)(e & ((1u << COSET_KB) - 1)) * 8));
  st_fe(data + p * 8, reduce<FrP>(mul<FrP>(v, ld_fe(hi + (size_t)(e >> COSET_KB) * 8))));
}

// ------------------------------------------------------------- host side
static int get_twiddles(zkmi_ctx* ctx, uint32_t logn, int inv, const uint32_t** out) {
  char name[64];
  snprintf(name, sizeof(name), "ntt_tw_%s_%u", inv ? "inv" : "fwd", logn);
  bool fresh = ctx->ws.bufs.find(name) == ctx->ws.bufs.end();
  uint64_t half = std::max<uint64_t>(1, (1ull << logn) / 2);
  uint32_t* tw;
  ZK_TRY(ctx->ws.get(name, ntt_tw_words(half) * 4, (void**)&tw));
  if (fresh) {
    uint64_t runs = (half + 63) / 64;
    // the outermost group of the 1024-element tile plan (ntt_groups)
    const uint32_t k0 = logn >= 11 ? (logn + ((logn + 7) / 8) - 1) / ((logn + 7) / 8) : 0;
    const uint32_t cb0 = logn >= 11 ? logn - k0 : 0, L = logn >= 11 ? 10 - k0 : 0;
    k_ntt_twiddles<<<(unsigned)((runs + 255) / 256), 256, 0, ctx->stream>>>(tw, logn, inv, half, cb0, L);
    if (ZK_NTT_STAGE_TW && half > 1)
      k_ntt_tw_levels<<<(unsigned)((half + 255) / 256), 256, 0, ctx->stream>>>(tw, half, cb0, L);
    ZK_HIP(hipGetLastError());
  }
  *out = tw;
  return 0;
}

// Group plan of a 2^logn transform: ceil(logn / 8) groups of <= 8 stages
// (tile = 2048 elements: 8 sub-transforms of 256, or fewer larger ones).
// (Measured, round 5: at most 6 stages per pass -- 16 adjacent columns, 512-B
// bursts in every strided pass, four passes at 2^24 instead of three -- 2^24
// NTT+INTT group time 4.28-4.30 -> 5.00-5.04 ms, 2^22 1.13-1.15 -> 1.21-1.23
// ms: the fourth pass's traffic and per-pass work cost more than the longer
// bursts save.)
static std::vector<uint32_t> ntt_groups(uint32_t logn) {
  int ng = (logn + 7) / 8;  // <= 8 stages per group for either tile shape
  std::vector<uint32_t> ks(ng, logn / ng);
  for (uint32_t r = 0; r < logn % ng; r++) ks[r]++;
  return ks;
}

// group kernel shape: radix-4 register rounds (4 elements per thread, <= 128
// VGPRs: 4 waves/SIMD; a 2048-element radix-8 form was 7% slower, dropped).
// Passes with column bits (every pass of a large transform but the innermost)
// read 2^(TB - k) adjacent columns per row of the tile: 1024-element tiles of
// 256 threads give 4 columns = 128-B bursts at 2^(a - k)-element strides (2 MB
// at 2^24).  ZK_NTT_TB_OUTER = 12 runs those passes on 4096-element tiles of
// 1024 threads (147 KB of LDS, one workgroup = 16 waves per CU, the same 4
// waves/SIMD): 16 columns = 512-B bursts.  Measured (round 5, one box, 3
// interleaved repeats, tools/gpu_r05e.sh): 2^24 NTT+INTT group time 4.25 ms
// with 1024-element tiles against 5.58-5.97 ms with 4096 (2^22: 1.13 vs 1.32
// ms) -- the 16-wave barriers of the big tile cost more than the longer bursts
// save -- so the default stays 10.
#ifndef ZK_NTT_TB_OUTER
#define ZK_NTT_TB_OUTER 10
#endif
static_assert(!ZK_NTT_TW_L8P || ZK_NTT_TB_OUTER == 10, "the limb-8 layout assumes 1024-element outer tiles");
template <bool DIT, int PRO, int EPI, bool PERM>
static void launch_group(hipStream_t st, const uint32_t* src, uint32_t* dst, const uint32_t* tw, uint32_t logn,
                         uint32_t a, uint32_t k, const NttIo& io) {
  constexpr int TBo = ZK_NTT_TB_OUTER;
  if (TBo != 10 && !PERM && a > k && logn >= (uint32_t)TBo && k <= (uint32_t)TBo - 2) {  // a pass with column bits
    const size_t sm = ((size_t)1 << TBo) * NL * 4;
    const unsigned grid = (unsigned)((1ull << logn) >> TBo);
    k_ntt_group<DIT, PRO, EPI, PERM, TBo, 2><<<grid, 1 << (TBo - 2), sm, st>>>(src, dst, tw, logn, a, k, io);
    return;
  }
  const size_t sm = (size_t)1024 * NL * 4;
  const unsigned grid = (unsigned)((1ull << logn) / 1024);
  k_ntt_group<DIT, PRO, EPI, PERM, 10, 2><<<grid, 256, sm, st>>>(src, dst, tw, logn, a, k, io);
}

// in-place transform in the requested order without scaling:
// dit=false: natural in -> bit-reversed out; dit=true: bit-reversed in -> natural out
// epi (DIF only): 0 none, 2 = x * lo[i] * hi[i] at natural index i, canonical out
int ntt_raw_epi(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inv, bool dit, int epi, const uint32_t* lo,
                const uint32_t* hi) {
  const uint32_t* tw;
  ZK_TRY(get_twiddles(ctx, logn, inv, &tw));
  hipStream_t st = ctx->stream;
  if (logn == 0) return 0;
  if ((1u << logn) < (uint32_t)NTT_TILE && logn < 11) {
    size_t sm = ((size_t)1 << logn) * NL * 4;
    ScopedKernelTimer tm(ctx, "ntt_small");
    if (dit) k_ntt_small<true><<<1, 256, sm, st>>>(d, tw, logn);
    else k_ntt_small<false><<<1, 256, sm, st>>>(d, tw, logn);
    ZK_HIP(hipGetLastError());
    if (epi) {
      ScopedKernelTimer tm2(ctx, "ntt_scale");
      k_scale_rev_small<<<(unsigned)(((1ull << logn) + 255) / 256), 256, 0, st>>>(d, logn, lo, hi);
      ZK_HIP(hipGetLastError());
    }
    return 0;
  }
  const std::vector<uint32_t> ks = ntt_groups(logn);
  const int ng = (int)ks.size();
  const NttIo io{lo, hi, nullptr};
  if (!dit) {
    uint32_t a = logn;
    for (int g = 0; g < ng; g++) {
      ScopedKernelTimer tm(ctx, "ntt_group");
      if (g == ng - 1 && epi == 2) launch_group<false, 0, 2, false>(st, d, d, tw, logn, a, ks[g], io);
      else launch_group<false, 0, 0, false>(st, d, d, tw, logn, a, ks[g], io);
      a -= ks[g];
    }
  } else {
    uint32_t a = 0;
    for (int g = ng - 1; g >= 0; g--) {
      a += ks[g];
      ScopedKernelTimer tm(ctx, "ntt_group");
      launch_group<true, 0, 0, false>(st, d, d, tw, logn, a, ks[g], io);
    }
  }
  ZK_HIP(hipGetLastError());
  return 0;
}
int ntt_raw(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inv, bool dit) {
  return ntt_raw_epi(ctx, d, logn, inv, dit, 0, nullptr, nullptr);
}

// in-place permutation natural <-> bit-reversed (+ optional scaling, + full reduction)
static int ntt_bitrev_scaled(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, BitrevScale sc) {
  hipStream_t st = ctx->stream;
  ScopedKernelTimer tm(ctx, "ntt_bitrev");
  if (logn >= 10) {
    uint32_t b = 5;
    unsigned grid = 1u << (logn - 2 * b);
    k_bitrev_tiled<<<grid, 256, 2 * (1u << (2 * b)) * 32, st>>>(d, logn, b, sc);
  } else {
    uint32_t* tmp;
    ZK_TRY(ctx->ws.get("ntt_tmp_small", ((size_t)1 << logn) * 32, (void**)&tmp));
    k_bitrev_naive<<<((1u << logn) + 255) / 256, 256, 0, st>>>(d, tmp, logn, sc);
    ZK_HIP(hipMemcpyAsync(d, tmp, ((size_t)1 << logn) * 32, hipMemcpyDeviceToDevice, st));
  }
  ZK_HIP(hipGetLastError());
  return 0;
}
int ntt_bitrev(zkmi_ctx* ctx, uint32_t* d, uint32_t logn) {
  return ntt_bitrev_scaled(ctx, d, logn, BitrevScale{0, nullptr, nullptr, nullptr});
}

// natural order in and out (arkworks semantics), DIF passes only:
//   forward: first pass reads d (x_i *= g^i folded in for the coset),
//            middle passes in place in a scratch vector, the innermost
//            group writes natural order back into d (PERM)
//   inverse: the same with omega^-1 and * n^-1 [g^-i] folded into the
//            permuting pass
// Small transforms (one tile or less) keep the single-workgroup kernel and
// a separate bit reversal.
int ntt_device(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inverse, int coset) {
  if (logn > 28) {
    set_error("ntt: log_n %u > 28 (two-adicity of Fr)", logn);
    return ZKMI_EINVAL;
  }
  DomainCache dc;
  ZK_TRY(domain_cache(ctx, logn, &dc));
  if (logn < 11) {
    if (!inverse) {
      if (coset) {
        ScopedKernelTimer tm(ctx, "ntt_scale");
        k_ntt_coset_scale<<<(unsigned)(((1ull << logn) + 255) / 256), 256, 0, ctx->stream>>>(d, logn, dc.lo_g,
                                                                                             dc.hi_gf);
        ZK_HIP(hipGetLastError());
      }
      ZK_TRY(ntt_raw(ctx, d, logn, 0, false));
      return ntt_bitrev(ctx, d, logn);
    }
    ZK_TRY(ntt_raw(ctx, d, logn, 1, false));
    BitrevScale sc = coset ? BitrevScale{2, nullptr, dc.lo_gi, dc.hi_gi} : BitrevScale{1, dc.ninv_m, nullptr, nullptr};
    return ntt_bitrev_scaled(ctx, d, logn, sc);
  }
  const uint32_t* tw;
  ZK_TRY(get_twiddles(ctx, logn, inverse, &tw));
  uint32_t* s;
  ZK_TRY(ctx->ws.get("ntt_scratch", ((size_t)1 << logn) * 32, (void**)&s));
  hipStream_t st = ctx->stream;
  const std::vector<uint32_t> ks = ntt_groups(logn);
  const int ng = (int)ks.size();
  const NttIo pro{dc.lo_g, dc.hi_gf, nullptr};
  NttIo epi{nullptr, nullptr, nullptr};
  if (inverse) epi = coset ? NttIo{dc.lo_gi, dc.hi_gi, nullptr} : NttIo{nullptr, nullptr, dc.ninv_m};
  uint32_t a = logn;
  for (int g = 0; g < ng; g++) {
    ScopedKernelTimer tm(ctx, "ntt_group");
    const uint32_t* src = g == 0 ? d : s;
    if (g < ng - 1) {
      if (g == 0 && coset && !inverse) launch_group<false, 1, 0, false>(st, src, s, tw, logn, a, ks[g], pro);
      else launch_group<false, 0, 0, false>(st, src, s, tw, logn, a, ks[g], pro);
    } else if (!inverse) {
      launch_group<false, 0, 0, true>(st, src, d, tw, logn, a, ks[g], epi);
    } else if (coset) {
      launch_group<false, 0, 2, true>(st, src, d, tw, logn, a, ks[g], epi);
    } else {
      launch_group<false, 0, 1, true>(st, src, d, tw, logn, a, ks[g], epi);
    }
    a -= ks[g];
  }
  ZK_HIP(hipGetLastError());
  return 0;
}

}  // namespace zk
