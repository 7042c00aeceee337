// Device-side helpers (MFMA fragment types, bf16 conversion, LDS transpose reads, Philox RNG).
// Included only by the .hip kernel translation units.
#pragma once
#include "mnist_common.h"

namespace mnist {

// Zero StepState for kernels launched without one (module API): `st = a.state ? a.state : &g_zero_state`
// keeps the state load unconditional.  A load under a branch ends in vmcnt(0) at the join, which
// serialises every load issued before it.
static __device__ StepState g_zero_state;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float floatx4;
typedef __attribute__((ext_vector_type(2))) float float2v;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
  return __builtin_bit_cast(uint16_t, b);
}
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE, the same bits as two f2bf calls;
// the scalar form compiled to one conversion per value plus the packing)
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const b2_t b = __builtin_convertvector((f2_t){lo, hi}, b2_t);
  return __builtin_bit_cast(uint32_t, b);
}

__device__ __forceinline__ floatx4 mfma16x16x32(const bf16x8& a, const bf16x8& b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16-byte LDS / global fragment loads (8 bf16)
__device__ __forceinline__ bf16x8 ld16(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ bf16x8 zero_frag() {
  u32x4 z = {0u, 0u, 0u, 0u};
  return __builtin_bit_cast(bf16x8, z);
}

// gfx950 ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p passes the address of row q,
// columns 4p..4p+3; lane i receives column i of the 4 rows.  Two of them give an 8-deep k slice.
__device__ __forceinline__ short4_t lds_tr16(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
}
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* row_lo, const uint16_t* row_hi) {
  short4_t a = lds_tr16(row_lo), b = lds_tr16(row_hi);
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  short8_t v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// 16-byte WRITE-THROUGH store (buffer_store_dwordx4 ... sc1): the line leaves this XCD's L2 with
// the store instead of staying dirty there, so the kernel-end release has nothing of it to write
// back - a dependent kernel boundary costs ~B / 6 TB/s more when the predecessor leaves B bytes
// dirty (MI355X_MICROARCH.md 'boundary'; the step's wgrad slabs are 19 MB).  For data only a LATER
// kernel reads; same cost as a plain 16-B store.
__device__ __forceinline__ void store_wt16(const void* base, int64_t byte_off, u32x4 v) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)byte_off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void store_wt16(const void* base, int64_t byte_off, floatx4 v) {
  store_wt16(base, byte_off, __builtin_bit_cast(u32x4, v));
}
__device__ __forceinline__ void store_wt16(const void* base, int64_t byte_off, uint4 v) {
  store_wt16(base, byte_off, u32x4{v.x, v.y, v.z, v.w});
}
__device__ __forceinline__ floatx4 make_floatx4(const float4& v) { return floatx4{v.x, v.y, v.z, v.w}; }
// write-through only where it pays: small batches, whose kernels are short enough that the
// kernel-end write-back of their dirty lines shows up as a gap (B = 200: 600 steps 70.2 -> 67.8
// us/step); at B = 8192 the write-through stores cost more than the write-back they save (0.930 ->
// 0.952 ms/step, same box: profiles/r4/ab/), so large batches keep plain stores
template <class T>
__device__ __forceinline__ void store16(bool wt, const void* base, int64_t byte_off, T v) {
  if (wt) store_wt16(base, byte_off, v);
  else *reinterpret_cast<T*>(static_cast<char*>(const_cast<void*>(base)) + byte_off) = v;
}

// Workgroup barrier for LDS data only: waits for this wave's LDS operations, not for its global
// loads and stores.  __syncthreads() is a workgroup fence + s_barrier, and the fence drains every
// outstanding global access (vmcnt(0)) first - a prefetch issued before it lands before anyone
// passes.  Only where the barrier publishes LDS data (no global data passes between waves).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Philox-4x32-10 (Salmon et al. 2011), the counter-based generator family torch uses for dropout.
__device__ __forceinline__ u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  u32x4 r = {c0, c1, c2, c3};
  return r;
}
// Random bytes for elements [16*blk, 16*blk+16) of one dropout invocation (counter = offset):
// element k of the block uses byte (k & 3) of word (k >> 2).
__device__ __forceinline__ u32x4 dropout_block(uint64_t seed, uint64_t offset, uint64_t blk) {
  return philox4x32((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)offset,
                    (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
}
__device__ __forceinline__ uint32_t dropout_byte(const u32x4& w, int k) {
  return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// conv1 pre-activation at one output pixel/channel from an fp32 input tile with row stride 28.
// Shared by the forward kernel and the backward relu-mask recompute so both see identical bits.
__device__ __forceinline__ float conv1_preact(const float* x, int stride, const float* w9, float b) {
  float acc = b;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) acc = __builtin_fmaf(x[ky * stride + kx], w9[ky * 3 + kx], acc);
  return acc;
}

// torchvision ToTensor()+Normalize((0.1307,),(0.3081,)) of one uint8 pixel: (v/255 - mean)/std in fp32.
// The 256 possible results are folded at compile time (IEEE round-to-nearest, identical to the
// runtime fp32 divisions) into a constant table: no divisions in any kernel.
struct NormLut {
  float v[256];
  constexpr NormLut() : v() {
    for (int i = 0; i < 256; ++i) v[i] = ((float)i / 255.0f - MNIST_MEAN) / MNIST_STD;
  }
};
__constant__ constexpr NormLut kNormLut{};
__device__ __forceinline__ float normalize_u8(uint8_t v) { return kNormLut.v[v]; }
// The same value from IEEE fp32 arithmetic (correctly rounded division, contraction off: bitwise the
// table entry): for a pixel whose load should not grow a dependent table load in a latency chain.
__device__ __forceinline__ float normalize_u8_alu(uint32_t v) {
#pragma clang fp contract(off)
  return ((float)v / 255.0f - MNIST_MEAN) / MNIST_STD;
}

// ---- race-window widening (debug build `_C_rw`, -DMNIST_RACE_WIDEN=<us>; docs/DEBUGGING.md) ----
// Every kernel's workgroups sleep a pseudo-random 0..MNIST_RACE_WIDEN us before their first global
// read (RW_ENTRY, placed after a kernel's start signal), and every stream hand-off signal - start
// signals, signal launches, held completions - is preceded by such a sleep (RW_SIGNAL).  The delays
// are drawn from the real-time clock per workgroup, so each launch of each step explores another
// interleaving of the compute and comm streams: a buffer that a hand-off does not actually protect
// is read or overwritten out of order in some step, and the schedule stops being bitwise equal to
// SERIAL.  Compiled out of the product build (no cost there).
#ifdef MNIST_RACE_WIDEN
__device__ __forceinline__ void race_widen_sleep(uint32_t tag) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();               // 100 MHz
  uint32_t h = (uint32_t)t0 * 0x9e3779b9u ^ (blockIdx.x + 0x7f4a7c15u * tag);
  h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
  const uint64_t ticks = h % (uint32_t)(MNIST_RACE_WIDEN * 100);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}
#define RW_ENTRY() ::mnist::race_widen_sleep(__LINE__)
#define RW_SIGNAL() ::mnist::race_widen_sleep(__LINE__ * 7u + 1u)
#else
#define RW_ENTRY() ((void)0)
#define RW_SIGNAL() ((void)0)
#endif

// Spin (one lane) until *a >= target: relaxed agent-scope polls with s_sleep; after ~60 s sets *err
// and gives up (a protocol bug must not hang the GPU).  Used by the schedule-3 stream hand-offs.
__device__ __forceinline__ void spin_until_geq(const int* a, int target, int* err) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();               // 100 MHz
  while (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 6000000000ull) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  RW_SIGNAL();   // (debug build: the held kernel's completion - its hand-off - comes later)
}


// One Adadelta element update (torch/optim/adadelta.py, foreach order: mul_, addcmul_, add+sqrt,
// add+sqrt, div_, mul_, mul_, addcmul_, add_), every operation individually rounded (FMA
// contraction off), so the result is a pure function of the inputs - bitwise identical in every
// kernel that applies it (the optimizer kernels and the fused fc-backward epilogue).
struct Ada {
  float rho, eps, wd, lr;
  __device__ __forceinline__ float step(float& p, float g, float& sq, float& acc) const {
#pragma clang fp contract(off)
    if (wd != 0.0f) g = g + wd * p;
    const float c = 1.0f - rho;
    sq = sq * rho + (c * g) * g;
    const float sd = sqrtf(sq + eps);
    float d = sqrtf(acc + eps);
    d = (d / sd) * g;
    acc = acc * rho + (c * d) * d;
    p = p + (-lr) * d;
    return p;
  }
};

}  // namespace mnist
