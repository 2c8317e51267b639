// mimc.cpp — native MiMC-x^7 for the zelana_batch witness (zelana_amd/zbatch.py).
//
// The permutation of forge/circuits/zelana_lib/src/poseidon.nr:15-56 (host
// restatement forge/crates/prover-worker/src/mimc.rs:52-122): 91 rounds of
// t = x + k + c_i, x <- t^7 with c_i = (i+1)^3 + (i+1), output x + k.
// zp_mimc_trace also writes the per-round witness values (t^2, t^4, t^6, t^7),
// in the order zbatch.Builder.permute allocates them, so the Python front-end
// spends no big-integer arithmetic on the ~1.4M MiMC trace variables of a
// batch.  All values are canonical little-endian 4 x u64.
// Pinned by the reference's batch-58 batch-hash KAT (mimc.rs:386-450) and the
// batch-70 Prover.toml roots, which tests/test_zbatch.py recomputes through
// this code, and by equality with the Python restatement (same file).
#include <stddef.h>
#include <stdint.h>

#include "fr.h"

using namespace zp;

namespace {
constexpr int kRounds = 91;

struct RoundConstants {
  Fr c[kRounds];
  RoundConstants() {
    for (int i = 0; i < kRounds; i++) {
      const uint64_t j = (uint64_t)i + 1;  // j^3 + j < 2^64 for j <= 91
      c[i] = Fr::from_u64(j * j * j + j);
    }
  }
};
const RoundConstants& rc() {
  static const RoundConstants k;
  return k;
}
}  // namespace

extern "C" {

int zp_mimc_rounds() { return kRounds; }

// y = permute(x, k)   (mimc.rs:52-122; zbatch.mimc_permute)
void zp_mimc_permute(const uint64_t x[4], const uint64_t k[4], uint64_t y[4]) {
  const RoundConstants& R = rc();
  const Fr kk = Fr::from_canon(k);
  Fr v = Fr::from_canon(x);
  for (int i = 0; i < kRounds; i++) {
    const Fr t = v + kk + R.c[i];
    const Fr t2 = t * t, t4 = t2 * t2, t6 = t4 * t2;
    v = t6 * t;
  }
  (v + kk).to_canon(y);
}

// trace[4 * 4 * r + 4 * j + limb] = canonical (t^2, t^4, t^6, t^7)[j] of round r
// for permute(x, 0); the last entry is the output.  (zbatch.Builder.permute)
void zp_mimc_trace(const uint64_t x[4], uint64_t* trace) {
  const RoundConstants& R = rc();
  Fr v = Fr::from_canon(x);
  for (int i = 0; i < kRounds; i++) {
    const Fr t = v + R.c[i];
    const Fr t2 = t * t, t4 = t2 * t2, t6 = t4 * t2;
    v = t6 * t;
    uint64_t* o = trace + 16 * (size_t)i;
    t2.to_canon(o);
    t4.to_canon(o + 4);
    t6.to_canon(o + 8);
    v.to_canon(o + 12);
  }
}

}  // extern "C"
