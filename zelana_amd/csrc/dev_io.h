// dev_io.h — HBM <-> register movement of packed 256-bit field elements
// (8 x u32, two 16-B loads/stores per element) and unpacking into the 9 x
// 29-bit limb form the arithmetic works on.
#pragma once
#include <hip/hip_runtime.h>

#include "ff.h"

namespace zk {

__device__ __forceinline__ Fe ld_fe(const uint32_t* p) {
  uint4 a = reinterpret_cast<const uint4*>(p)[0];
  uint4 b = reinterpret_cast<const uint4*>(p)[1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return unpack(w);
}
__device__ __forceinline__ void st_fe(uint32_t* p, const Fe& f) {
  uint32_t w[8];
  pack(w, f);
  reinterpret_cast<uint4*>(p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
  reinterpret_cast<uint4*>(p)[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
// element from a constant table (scalar loads)
__device__ __forceinline__ Fe ldc_fe(const uint32_t* c) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = c[i];
  return unpack(w);
}

}  // namespace zk
