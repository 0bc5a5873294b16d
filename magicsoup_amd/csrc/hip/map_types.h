// Molecule-map storage types: fp32 (default), bf16, fp16; kernels compute in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msd {

enum MapType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

struct bf16_t {
  uint16_t u;
};

template <class T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) {
  return *p;
}
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) {
  return __uint_as_float((uint32_t)p->u << 16);
}
template <>
__device__ __forceinline__ float ld<_Float16>(const _Float16* p) {
  return (float)*p;
}

template <class T>
__device__ __forceinline__ void st(T* p, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, float v) {
  *p = v;
}
template <>
__device__ __forceinline__ void st<bf16_t>(bf16_t* p, float v) {
  uint32_t u = __float_as_uint(v);
  if ((u & 0x7F800000u) == 0x7F800000u) {  // inf / nan: truncate, keep a quiet nan
    p->u = (uint16_t)((u >> 16) | ((u & 0xFFFFu) ? 0x40u : 0u));
    return;
  }
  u += 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even
  p->u = (uint16_t)(u >> 16);
}
template <>
__device__ __forceinline__ void st<_Float16>(_Float16* p, float v) {
  *p = (_Float16)v;
}

// 4 consecutive, 4-element-aligned values (one 16 B / 8 B vector access)
template <class T>
__device__ __forceinline__ void ld4(const T* p, float v[4]);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float v[4]) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
}
template <>
__device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float v[4]) {
  const uint2 q = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(q.x << 16), v[1] = __uint_as_float(q.x & 0xFFFF0000u);
  v[2] = __uint_as_float(q.y << 16), v[3] = __uint_as_float(q.y & 0xFFFF0000u);
}
template <>
__device__ __forceinline__ void ld4<_Float16>(const _Float16* p, float v[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 q = *reinterpret_cast<const h4*>(p);
  v[0] = (float)q[0], v[1] = (float)q[1], v[2] = (float)q[2], v[3] = (float)q[3];
}

template <class T>
__device__ __forceinline__ void st4(T* p, const float v[4]);
template <>
__device__ __forceinline__ void st4<float>(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <>
__device__ __forceinline__ void st4<bf16_t>(bf16_t* p, const float v[4]) {
  bf16_t h[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) st(h + j, v[j]);
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)h[0].u | ((uint32_t)h[1].u << 16),
                                            (uint32_t)h[2].u | ((uint32_t)h[3].u << 16));
}
template <>
__device__ __forceinline__ void st4<_Float16>(_Float16* p, const float v[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  h4 q;
  q[0] = (_Float16)v[0], q[1] = (_Float16)v[1], q[2] = (_Float16)v[2], q[3] = (_Float16)v[3];
  *reinterpret_cast<h4*>(p) = q;
}

// streaming store of 4 values (the stencil's output is not re-read before the next step): fp32
// with a nontemporal hint (-4 % on the 4096^2 x 14 fp32 stencil; nontemporal loads measured +6 %,
// the halo rows are re-read by the neighbouring band), the narrow types as st4
template <class T>
__device__ __forceinline__ void st4_stream(T* p, const float v[4]) {
  st4(p, v);
}
template <>
__device__ __forceinline__ void st4_stream<float>(float* p, const float v[4]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 q;
  q[0] = v[0], q[1] = v[1], q[2] = v[2], q[3] = v[3];
  __builtin_nontemporal_store(q, reinterpret_cast<f4*>(p));
}

// 8 consecutive, 8-element-aligned values: fp32 as two 16 B accesses, bf16 / fp16 as one 16 B
// access with the packed hardware conversions (gfx950 v_cvt_pk_bf16_f32: round to nearest even,
// as st<bf16_t>)
template <class T>
__device__ __forceinline__ void ld8(const T* p, float v[8]);
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float v[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
}
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float v[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
template <>
__device__ __forceinline__ void ld8<_Float16>(const _Float16* p, float v[8]) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const h8 q = *reinterpret_cast<const h8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)q[j];
}

// Raw bits of 8 consecutive values (fp32: two 16 B words, bf16 / fp16: one), loaded without
// converting: a prefetched row's load stays in flight until the row is used (a conversion right
// after the load would wait for it there)
template <class T>
struct Bits8 {
  uint4 q[sizeof(T) == 4 ? 2 : 1];
};
template <class T>
__device__ __forceinline__ void ld8_bits(const T* p, Bits8<T>& r) {
  const uint4* w = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(r.q) / sizeof(uint4)); ++i) r.q[i] = w[i];
}
template <class T>
__device__ __forceinline__ void zero8_bits(Bits8<T>& r) {
#pragma unroll
  for (int i = 0; i < (int)(sizeof(r.q) / sizeof(uint4)); ++i) r.q[i] = make_uint4(0u, 0u, 0u, 0u);
}
template <class T>
__device__ __forceinline__ void cvt8(const Bits8<T>& r, float v[8]);
template <>
__device__ __forceinline__ void cvt8<float>(const Bits8<float>& r, float v[8]) {
  const uint32_t w[8] = {r.q[0].x, r.q[0].y, r.q[0].z, r.q[0].w, r.q[1].x, r.q[1].y, r.q[1].z, r.q[1].w};
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(w[j]);
}
template <>
__device__ __forceinline__ void cvt8<bf16_t>(const Bits8<bf16_t>& r, float v[8]) {
  const uint32_t w[4] = {r.q[0].x, r.q[0].y, r.q[0].z, r.q[0].w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
template <>
__device__ __forceinline__ void cvt8<_Float16>(const Bits8<_Float16>& r, float v[8]) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const h8 q = __builtin_bit_cast(h8, r.q[0]);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)q[j];
}
// one value as raw bits (zero-extended) and back
template <class T>
__device__ __forceinline__ uint32_t ld_bits(const T* p) {
  if constexpr (sizeof(T) == 4) return *reinterpret_cast<const uint32_t*>(p);
  else return *reinterpret_cast<const uint16_t*>(p);
}
template <class T>
__device__ __forceinline__ float from_bits(uint32_t u) {
  if constexpr (sizeof(T) == 4) return __uint_as_float(u);
  else if constexpr (__is_same(T, bf16_t)) return __uint_as_float(u << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)u);
}

template <class T>
__device__ __forceinline__ void st8_stream(T* p, const float v[8]);
template <>
__device__ __forceinline__ void st8_stream<float>(float* p, const float v[8]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = v[j], b[j] = v[j + 4];
  __builtin_nontemporal_store(a, reinterpret_cast<f4*>(p));
  __builtin_nontemporal_store(b, reinterpret_cast<f4*>(p) + 1);
}
template <>
__device__ __forceinline__ void st8_stream<bf16_t>(bf16_t* p, const float v[8]) {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  b8 q;
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = (__bf16)v[j];
  *reinterpret_cast<b8*>(p) = q;
}
template <>
__device__ __forceinline__ void st8_stream<_Float16>(_Float16* p, const float v[8]) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  h8 q;
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = (_Float16)v[j];
  *reinterpret_cast<h8*>(p) = q;
}

// runtime-typed access (cold paths: a few pixels per cell)
__device__ __forceinline__ float ld_map(const void* base, size_t i, int dtype) {
  switch (dtype) {
    case kBF16: return ld(reinterpret_cast<const bf16_t*>(base) + i);
    case kF16: return ld(reinterpret_cast<const _Float16*>(base) + i);
    default: return ld(reinterpret_cast<const float*>(base) + i);
  }
}

__device__ __forceinline__ void st_map(void* base, size_t i, float v, int dtype) {
  switch (dtype) {
    case kBF16: st(reinterpret_cast<bf16_t*>(base) + i, v); break;
    case kF16: st(reinterpret_cast<_Float16*>(base) + i, v); break;
    default: st(reinterpret_cast<float*>(base) + i, v); break;
  }
}

}  // namespace msd

namespace msd {
// Deferred diffusion mass correction (see maps.hip): a map plane may hold raw values whose true
// value is max(raw + corr[mol], 0). corr == nullptr: raw values are true values.
__device__ __forceinline__ float corr_in(float raw, const float* corr, int mol) {
  return corr ? fmaxf(raw + corr[mol], 0.0f) : raw;
}
__device__ __forceinline__ float corr_out(float v, const float* corr, int mol) { return corr ? v - corr[mol] : v; }
}  // namespace msd

