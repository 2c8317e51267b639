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
__constant__ uint32_t GINV[8] = {0xc6666667u, 0xe7f3fbd4u, 0xca4a2d06u, 0xa9ae5ce9u,
                                 0x33cd568bu, 0x49b9b57cu, 0x5a13d9aau, 0x135b5294u};

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

// tw[e] = omega^e, e < half.  Each thread: one pow + 63 muls for a run of 64.
__global__ void __launch_bounds__(256) k_ntt_twiddles(uint32_t* __restrict__ tw, uint32_t logn, int inv, uint64_t half) {
  uint64_t run = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t e0 = run * 64;
  if (e0 >= half) return;
  Fe w = root_of_unity(logn, inv != 0);
  Fe cur = fe_pow_u64(w, e0);
  for (int k = 0; k < 64 && e0 + k < half; k++) {
    st_fe(tw + (e0 + k) * 8, reduce<FrP>(cur));
    cur = mul<FrP>(cur, w);
  }
}

// One group of `k` stages.  Sub-transform q -> (blk, col): col = q mod 2^(a-k),
// blk = q / 2^(a-k); element j of it lives at blk*2^a + col + j*2^(a-k).
// DIT=false: DIF stages m = 2^a .. 2^(a-k+1); DIT=true: m = 2^(a-k+1) .. 2^a.
constexpr int NTT_TILE = 2048;
template <bool DIT>
__global__ void __launch_bounds__(256) k_ntt_group(uint32_t* __restrict__ data, const uint32_t* __restrict__ tw,
                                                   uint32_t logn, uint32_t a, uint32_t k) {
  extern __shared__ __align__(16) uint32_t lds[];  // [j][sub][9]
  const uint32_t sub_n = NTT_TILE >> k;            // sub-transforms per workgroup
  const uint32_t len = 1u << k;
  const uint32_t colbits = a - k;
  const uint64_t q0 = (uint64_t)blockIdx.x * sub_n;
  // load: element e = j*sub_n + s
  for (uint32_t e = threadIdx.x; e < NTT_TILE; e += blockDim.x) {
    uint32_t j = e / sub_n, s = e % sub_n;
    uint64_t q = q0 + s;
    uint64_t col = q & ((1ull << colbits) - 1), blk = q >> colbits;
    uint64_t idx = (blk << a) + col + ((uint64_t)j << colbits);
    Fe v = ld_fe(data + idx * 8);
#pragma unroll
    for (int l = 0; l < NL; l++) lds[e * NL + l] = v.v[l];
  }
  __syncthreads();
  const uint32_t nb = NTT_TILE / 2;
  for (uint32_t st = 0; st < k; st++) {
    // local half-distance (in j units) for this stage
    uint32_t hl = DIT ? (1u << st) : (len >> (st + 1));
    uint32_t logm = colbits + (DIT ? st + 1 : k - st);  // m = 2^logm
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
      uint32_t s = b % sub_n, pj = b / sub_n;  // pair index within sub-transform
      uint32_t j0 = (pj / hl) * (2 * hl) + (pj % hl);
      uint32_t e0 = j0 * sub_n + s, e1 = (j0 + hl) * sub_n + s;
      Fe u, v;
#pragma unroll
      for (int l = 0; l < NL; l++) {
        u.v[l] = lds[e0 * NL + l];
        v.v[l] = lds[e1 * NL + l];
      }
      // twiddle index: i mod (m/2) scaled by n/m
      uint64_t q = q0 + s;
      uint64_t col = q & ((1ull << colbits) - 1), blk = q >> colbits;
      uint64_t i = (blk << a) + col + ((uint64_t)j0 << colbits);
      uint64_t jm = i & ((1ull << (logm - 1)) - 1);
      uint64_t te = jm << (logn - logm);
      Fe w = ld_fe(tw + te * 8);
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
        lds[e0 * NL + l] = x.v[l];
        lds[e1 * NL + l] = y.v[l];
      }
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < NTT_TILE; e += blockDim.x) {
    uint32_t j = e / sub_n, s = e % sub_n;
    uint64_t q = q0 + s;
    uint64_t col = q & ((1ull << colbits) - 1), blk = q >> colbits;
    uint64_t idx = (blk << a) + col + ((uint64_t)j << colbits);
    Fe v;
#pragma unroll
    for (int l = 0; l < NL; l++) v.v[l] = lds[e * NL + l];
    st_fe(data + idx * 8, v);
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
      Fe w = ld_fe(tw + (size_t)te * 8);
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
__global__ void __launch_bounds__(256) k_bitrev_tiled(uint32_t* __restrict__ data, uint32_t logn, uint32_t b) {
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
      Fe v = reduce<FrP>(unpack(w));
      uint64_t oidx = ((uint64_t)rlo << (logn - b)) | ((uint64_t)omid << b) | rhi;
      st_fe(data + oidx * 8, v);
    }
  }
}
__global__ void __launch_bounds__(256) k_bitrev_naive(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      uint32_t logn) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1u << logn)) return;
  uint32_t r = logn ? brev_bits(i, logn) : 0;
  st_fe(out + (size_t)r * 8, reduce<FrP>(ld_fe(in + (size_t)i * 8)));
}

// data[i] = reduce(data[i] * c * g^(+-i)) in natural order; g^i by runs of 64.
// mode bit0: multiply by n^-1; bit1: coset powers; bit2: inverse coset (g^-i)
__global__ void __launch_bounds__(256) k_ntt_scale(uint32_t* __restrict__ data, uint32_t logn, int mode) {
  uint64_t n = 1ull << logn;
  uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 64;
  if (i0 >= n) return;
  Fe c = one<FrP>();
  if (mode & 1) {
    // n^-1 = (2^-1)^logn with 2^-1 = (r+1)/2
    const uint32_t half_c[8] = {0xf8000001u, 0xa1f0fac9u, 0x3cdcb848u, 0x9419f424u,
                                0x40c0ac2eu, 0xdc2822dbu, 0x7098d014u, 0x18322739u};
    Fe hinv = to_mont<FrP>(ldc_fe(half_c));
    for (uint32_t k = 0; k < logn; k++) c = mul<FrP>(c, hinv);
  }
  Fe g = one<FrP>(), cur = c;
  if (mode & 2) {
    if (mode & 4) g = mont_from_canon(GINV);
    else g = to_mont<FrP>(Fe{{5, 0, 0, 0, 0, 0, 0, 0, 0}});
    cur = mul<FrP>(c, fe_pow_u64(g, i0));
  }
  for (int k = 0; k < 64 && i0 + k < n; k++) {
    uint32_t* p = data + (i0 + k) * 8;
    st_fe(p, reduce<FrP>(mul<FrP>(ld_fe(p), cur)));
    if (mode & 2) cur = mul<FrP>(cur, g);
  }
}

// ------------------------------------------------------------- host side
static int get_twiddles(zkmi_ctx* ctx, uint32_t logn, int inv, const uint32_t** out) {
  char name[64];
  snprintf(name, sizeof(name), "ntt_tw_%s_%u", inv ? "inv" : "fwd", logn);
  bool fresh = ctx->ws.bufs.find(name) == ctx->ws.bufs.end();
  uint64_t half = std::max<uint64_t>(1, (1ull << logn) / 2);
  uint32_t* tw;
  ZK_TRY(ctx->ws.get(name, half * 32, (void**)&tw));
  if (fresh) {
    uint64_t runs = (half + 63) / 64;
    k_ntt_twiddles<<<(unsigned)((runs + 255) / 256), 256, 0, ctx->stream>>>(tw, logn, inv, half);
    ZK_HIP(hipGetLastError());
  }
  *out = tw;
  return 0;
}

// in-place transform in the requested order without scaling:
// dit=false: natural in -> bit-reversed out; dit=true: bit-reversed in -> natural out
int ntt_raw(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inv, bool dit) {
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
    return 0;
  }
  // groups of <= 8 stages (tile = 2048 elements: 8 sub-transforms of 256 or
  // fewer larger ones when k > 8); balance group sizes
  int ng = (logn + 7) / 8;
  std::vector<uint32_t> ks(ng, logn / ng);
  for (uint32_t r = 0; r < logn % ng; r++) ks[r]++;
  size_t sm = (size_t)NTT_TILE * NL * 4;
  unsigned grid = (unsigned)((1ull << logn) / NTT_TILE);
  if (!dit) {
    uint32_t a = logn;
    for (int g = 0; g < ng; g++) {
      ScopedKernelTimer tm(ctx, "ntt_group");
      k_ntt_group<false><<<grid, 256, sm, st>>>(d, tw, logn, a, ks[g]);
      a -= ks[g];
    }
  } else {
    uint32_t a = 0;
    for (int g = ng - 1; g >= 0; g--) {
      a += ks[g];
      ScopedKernelTimer tm(ctx, "ntt_group");
      k_ntt_group<true><<<grid, 256, sm, st>>>(d, tw, logn, a, ks[g]);
    }
  }
  ZK_HIP(hipGetLastError());
  return 0;
}

// in-place permutation natural <-> bit-reversed (+ full reduction)
int ntt_bitrev(zkmi_ctx* ctx, uint32_t* d, uint32_t logn) {
  hipStream_t st = ctx->stream;
  ScopedKernelTimer tm(ctx, "ntt_bitrev");
  if (logn >= 10) {
    uint32_t b = 5;
    unsigned grid = 1u << (logn - 2 * b);
    k_bitrev_tiled<<<grid, 256, 2 * (1u << (2 * b)) * 32, st>>>(d, logn, b);
  } else {
    uint32_t* tmp;
    ZK_TRY(ctx->ws.get("ntt_tmp_small", ((size_t)1 << logn) * 32, (void**)&tmp));
    k_bitrev_naive<<<((1u << logn) + 255) / 256, 256, 0, st>>>(d, tmp, logn);
    ZK_HIP(hipMemcpyAsync(d, tmp, ((size_t)1 << logn) * 32, hipMemcpyDeviceToDevice, st));
  }
  ZK_HIP(hipGetLastError());
  return 0;
}

int ntt_scale(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int mode) {
  uint64_t runs = ((1ull << logn) + 63) / 64;
  ScopedKernelTimer tm(ctx, "ntt_scale");
  k_ntt_scale<<<(unsigned)((runs + 255) / 256), 256, 0, ctx->stream>>>(d, logn, mode);
  ZK_HIP(hipGetLastError());
  return 0;
}

// natural order in and out (arkworks semantics)
int ntt_device(zkmi_ctx* ctx, uint32_t* d, uint32_t logn, int inverse, int coset) {
  if (logn > 28) {
    set_error("ntt: log_n %u > 28 (two-adicity of Fr)", logn);
    return ZKMI_EINVAL;
  }
  if (!inverse) {
    if (coset) ZK_TRY(ntt_scale(ctx, d, logn, 2));
    ZK_TRY(ntt_raw(ctx, d, logn, 0, false));
    ZK_TRY(ntt_bitrev(ctx, d, logn));
  } else {
    ZK_TRY(ntt_raw(ctx, d, logn, 1, false));
    ZK_TRY(ntt_bitrev(ctx, d, logn));
    ZK_TRY(ntt_scale(ctx, d, logn, coset ? (1 | 2 | 4) : 1));
  }
  return 0;
}

}  // namespace zk
