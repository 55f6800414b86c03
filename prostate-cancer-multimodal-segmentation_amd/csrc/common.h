// Shared device helpers for the gfx950 (CDNA4) U-Net kernels.
//
// Storage types: activations are NDHWC in either fp32 (parity build) or bf16
// (performance build, raw bits in uint16_t).  All accumulation is fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

typedef uint16_t bf16_t;  // raw bf16 bits (same bytes as torch.bfloat16)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

#define LDS_AS __attribute__((address_space(3)))

// dtype codes.  Activations: 0 fp32, 1 bf16.  The 3x3x3 conv entry points also take 2: fp32
// data with the faster bf16x3 arithmetic (dtype 0 there means bf16x6, fp32-grade).
enum { PCMS_F32 = 0, PCMS_BF16 = 1, PCMS_F32X3 = 2 };
// conv epilogue flags (pcms_conv3_fwd, pcms_split_epilogue, pcms_stem_fwd)
enum { PCMS_CONV_ACCUMULATE = 1, PCMS_CONV_RELU = 2 };
// pcms_stem_fwd: the K-dense kernel (the pack's second form; weights with <= 5 input channels)
enum { PCMS_STEM_DENSE = 16 };
// gradient writer flags (pcms_conv3_wgrad): store instead of accumulating
enum { PCMS_GRAD_STORE = 1 };

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even via the hardware convert (v_cvt_pk_bf16_f32 on gfx950)
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// two floats -> packed bf16x2 (lo = a), one v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const f32x2_t f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}

// arithmetic tags of the fp32-data conv kernels (split-bf16: conv_common.h)
struct x3_t {};
struct x6_t {};

// three bf16 parts of 8 floats (h, m, l: 8 packed bf16 each)
__device__ __forceinline__ void split3x8(const float* f, u32x4_t& h, u32x4_t& m, u32x4_t& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = f[2 * i], b = f[2 * i + 1];
    const uint32_t hh = pack_bf16x2(a, b);
    const float ra = a - __uint_as_float(hh << 16), rb = b - __uint_as_float(hh & 0xffff0000u);
    const uint32_t mm = pack_bf16x2(ra, rb);
    h[i] = hh;
    m[i] = mm;
    l[i] = pack_bf16x2(ra - __uint_as_float(mm << 16), rb - __uint_as_float(mm & 0xffff0000u));
  }
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
  static __device__ __forceinline__ float cvt(float v) { return v; }
  static constexpr int kVec = 4;  // elements per 16-byte vector
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
  static __device__ __forceinline__ bf16_t cvt(float v) { return f2bf(v); }
  static constexpr int kVec = 8;
};

// 16-byte vector load/store of kVec elements as floats.
template <typename T> __device__ __forceinline__ void load16(const T* p, float* out);
template <> __device__ __forceinline__ void load16<float>(const float* p, float* out) {
  f32x4_t v = *reinterpret_cast<const f32x4_t*>(p);
  out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
}
template <> __device__ __forceinline__ void load16<bf16_t>(const bf16_t* p, float* out) {
  u32x4_t v = *reinterpret_cast<const u32x4_t*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = __uint_as_float(v[i] << 16);
    out[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
template <typename T> __device__ __forceinline__ void store16(T* p, const float* in);
template <> __device__ __forceinline__ void store16<float>(float* p, const float* in) {
  f32x4_t v = {in[0], in[1], in[2], in[3]};
  *reinterpret_cast<f32x4_t*>(p) = v;
}
template <> __device__ __forceinline__ void store16<bf16_t>(bf16_t* p, const float* in) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = (uint32_t)f2bf(in[2 * i]) | ((uint32_t)f2bf(in[2 * i + 1]) << 16);
  *reinterpret_cast<u32x4_t*>(p) = v;
}

// non-temporal forms (streams far larger than the 256 MB Infinity Cache: nothing to keep)
template <typename T> __device__ __forceinline__ void load16_nt(const T* p, float* out);
template <> __device__ __forceinline__ void load16_nt<float>(const float* p, float* out) {
  f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
  out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
}
template <> __device__ __forceinline__ void load16_nt<bf16_t>(const bf16_t* p, float* out) {
  u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = __uint_as_float(v[i] << 16);
    out[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
template <typename T> __device__ __forceinline__ void store16_nt(T* p, const float* in);
template <> __device__ __forceinline__ void store16_nt<float>(float* p, const float* in) {
  f32x4_t v = {in[0], in[1], in[2], in[3]};
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t*>(p));
}
template <> __device__ __forceinline__ void store16_nt<bf16_t>(bf16_t* p, const float* in) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = (uint32_t)f2bf(in[2 * i]) | ((uint32_t)f2bf(in[2 * i + 1]) << 16);
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
}
template <bool NT, typename T> __device__ __forceinline__ void ld16(const T* p, float* out) {
  if constexpr (NT) load16_nt<T>(p, out); else load16<T>(p, out);
}
template <bool NT, typename T> __device__ __forceinline__ void st16(T* p, const float* in) {
  if constexpr (NT) store16_nt<T>(p, in); else store16<T>(p, in);
}
// BatchNorm (train or eval coefficients) + ReLU of one element: the one expression every
// kernel that applies it uses (bn_relu pass and the fused consumers), so a recomputed
// activation equals the stored one bit for bit
__device__ __forceinline__ float bn_relu1(float y, float sc, float sh) { return fmaxf(__builtin_fmaf(y, sc, sh), 0.f); }
// ReLU of 8 packed bf16 values: negative ones (sign bit set) -> +0
__device__ __forceinline__ u32x4_t relu_bf16x8(u32x4_t v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] &= ~(((v[i] >> 15) & 0x00010001u) * 0xffffu);
  return v;
}
// a value as it reads back after a store in T (bf16: rounded to nearest even)
template <typename T> __device__ __forceinline__ float round_st(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v)); else return v;
}

// streams this large bypass the caches (non-temporal loads / stores)
#ifndef PCMS_NT_MB
#define PCMS_NT_MB 128  // A/B switch (build-time)
#endif
constexpr long kNtBytes = (long)PCMS_NT_MB << 20;
// the BatchNorm / ReLU / pool passes stream level-1-sized tensors (67 MB) past the caches too:
// their inputs were written a full conv earlier and their outputs are read a conv later
// (A/B: BN rows -12..-15 us per step, the ConvTranspose forward +3 us at 64 MB: kept at 128
// there, profiles/r4_nt_threshold_ab.txt)
#ifndef PCMS_BN_NT_MB
#define PCMS_BN_NT_MB 64
#endif
constexpr long kNtBytesBn = (long)PCMS_BN_NT_MB << 20;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Raw buffer descriptor (4 SGPRs): base, stride 0, num_records bytes (out-of-range offsets
// read 0), dword3 as __builtin_amdgcn_make_buffer_rsrc(..., 0x00020000) builds it.
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
__device__ __forceinline__ i32x4_t buffer_desc(const void* base, uint32_t num_bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4_t d;
  d[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  d[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xffff);
  d[2] = __builtin_amdgcn_readfirstlane((int)num_bytes);
  d[3] = 0x00020000;
  return d;
}

// 16-byte LDS-DMA (buffer_load_dwordx4 ... lds): lane l's 16 bytes from rsrc at
// voff + soff land at LDS byte lds_base + 16 l (lds_base wave-uniform).  Issued from inline
// asm so the compiler's waitcnt pass does not see it: it would otherwise wait vmcnt(0)
// before the next LDS read of ANY buffer (killing a multi-stage ring).  The caller retires
// these with explicit s_waitcnt vmcnt(N) + a barrier before reading the data.
// Wait states inside the string (the compiler pads nothing in it): s_nop 4 first, for an
// soffset / descriptor SGPR fresh from v_readfirstlane (VALU SGPR write -> VMEM read), and
// one state between the M0 write and the LDS-DMA that reads it.  M0 is compiler-reserved
// and not preserved around an asm statement, so the statement saves and restores it.
__device__ __forceinline__ void dma16(i32x4_t rsrc, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(lds_base), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory");
}
// the same with the non-temporal policy (data read once: streamed past the caches)
__device__ __forceinline__ void dma16_nt(i32x4_t rsrc, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(lds_base), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// One Adam element update (torch.optim.Adam, coupled weight decay): g_eff = g * s (written
// back when s != 1), shared by the flat Adam kernel and the fused Adam + weight-pack kernels
// so every path performs the identical fp32 operation sequence.
struct AdamCoef {
  float step_size, b1, b2, eps, wd, bc2_sqrt, gscale;
};
__device__ __forceinline__ float adam_update(float& p, float& g, float& m, float& v, const AdamCoef& c, float s) {
  float gi = g;
  if (s != 1.f) {
    gi *= s;
    g = gi;
  }
  const float pi = p;
  if (c.wd != 0.f) gi = gi + c.wd * pi;
  m = m + (1.f - c.b1) * (gi - m);                  // exp_avg.lerp_(grad, 1 - beta1)
  v = v * c.b2 + (1.f - c.b2) * gi * gi;            // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = sqrtf(v) / c.bc2_sqrt + c.eps;
  p = pi - c.step_size * (m / denom);
  return p;
}

// sum of n <= 16 values src[0], src[step], ... in that order, all loads issued before the
// first add (a load -> add chain per row was latency-bound); longer: 16 at a time
__device__ __forceinline__ float sum_rows16(const float* src, long step, int n) {
  float sum = 0.f;
  for (int base = 0; base < n; base += 16) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (base + r < n) v[r] = src[(long)(base + r) * step];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (base + r < n) sum += v[r];
  }
  return sum;
}

#define PCMS_CHECK_LAUNCH() return (int)hipGetLastError()

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
