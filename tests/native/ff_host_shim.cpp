// Host build of zelana_amd/csrc/ff.h (the exact source the gfx950 kernels use)
// so the limb arithmetic can be unit-tested on CPU against Python integers.
#include "../../zelana_amd/csrc/ff.h"
using namespace zk;
template <class P> static Fe ld(const uint32_t* w) { return unpack(w); }
extern "C" {
// op: 0 mul (Montgomery, raw), 1 sqr, 2 add, 3 sub, 4 reduce, 5 to_mont, 6 from_mont, 7 neg
// field: 0 = Fq, 1 = Fr.  Inputs/outputs packed 8 x u32.
void ff_op(int field, int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  for (int i = 0; i < n; i++) {
    Fe x = unpack(a + 8 * i), y = unpack(b + 8 * i), r;
    if (field == 0) {
      switch (op) {
        case 0: r = mul<FqP>(x, y); break;
        case 1: r = sqr<FqP>(x); break;
        case 2: r = add<FqP>(x, y); break;
        case 3: r = sub<FqP>(x, y); break;
        case 4: r = reduce<FqP>(x); break;
        case 5: r = to_mont<FqP>(x); break;
        case 6: r = from_mont<FqP>(x); break;
        default: r = neg<FqP>(x); break;
      }
    } else {
      switch (op) {
        case 0: r = mul<FrP>(x, y); break;
        case 1: r = sqr<FrP>(x); break;
        case 2: r = add<FrP>(x, y); break;
        case 3: r = sub<FrP>(x, y); break;
        case 4: r = reduce<FrP>(x); break;
        case 5: r = to_mont<FrP>(x); break;
        case 6: r = from_mont<FrP>(x); break;
        default: r = neg<FrP>(x); break;
      }
    }
    pack(out + 8 * i, r);
  }
}
// lazy-add then mul: (a + b) * c with limbwise add (exercises the 2^30-limb path)
void ff_lazy_mul(int field, const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* out, int n) {
  for (int i = 0; i < n; i++) {
    Fe s = add_lazy(unpack(a + 8 * i), unpack(b + 8 * i));
    Fe s2 = add_lazy(unpack(c + 8 * i), unpack(c + 8 * i));
    Fe r = field == 0 ? mul<FqP>(s, s2) : mul<FrP>(s, s2);
    pack(out + 8 * i, r);
  }
}
}
