// cram_fused.hip — fused elementwise kernels of the CrAM engine (gfx950).
//
// The IE sweep / decode run the model's non-attention elementwise work between
// hipBLASLt GEMMs.  As torch ops that is ~10 HBM passes per layer (RMSNorm:
// cast, pow, mean, rsqrt, mul, cast, mul; RoPE: mul, cat, neg, mul, add; MLP:
// silu, mul).  These kernels do each group in one pass and keep transformers'
// rounding points (LlamaRMSNorm, apply_rotary_pos_emb, LlamaMLP), so results
// equal the reference's op sequence up to the fp32 order of the RMS reduction (rnd = round to the
// model dtype, bf16 or fp16):
//   rmsnorm      y = rnd(w * rnd(x * rsqrt(mean(x^2) + eps)))      [+ fused residual add]
//   rope         x' = rnd(rnd(x * cos) + rnd(rotate_half(x) * sin))  in place on the QKV buffer
//   silu_mul     y = rnd(rnd(silu(g)) * u)
// All loads/stores are 16 B per lane (8 elements).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cram_attn.h"
#include "cram_silu.inc"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <typename T> struct Vec;
template <> struct Vec<__bf16> { typedef bf16x8 x8; };
template <> struct Vec<_Float16> { typedef f16x8 x8; };

// round-to-nearest-even to bf16 and back, by integer arithmetic: the compiler folds a
// (float)(__bf16)x pair away in some contexts (measured on ROCm 7.2: 1-ulp RoPE mismatches),
// which would skip the intermediate rounding transformers performs.  Inputs here are finite.
__device__ __forceinline__ float bfr(float x) {
  unsigned u = __float_as_uint(x);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
  return __uint_as_float(u);
}
// fp16: the hardware conversion (RNE, subnormals kept), its result pinned in a register so the
// round trip cannot be folded away either
__device__ __forceinline__ float hfr(float x) {
  unsigned short b = __builtin_bit_cast(unsigned short, (_Float16)x);
  asm volatile("" : "+v"(b));
  return (float)__builtin_bit_cast(_Float16, b);
}
template <typename T> __device__ __forceinline__ float rnd(float x);
template <> __device__ __forceinline__ float rnd<__bf16>(float x) { return bfr(x); }
template <> __device__ __forceinline__ float rnd<_Float16>(float x) { return hfr(x); }

template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) s += red[w];
  return s;
}

// one workgroup per row; VPT 8-element vectors per thread
template <typename T, int NT, int VPT>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(const T* __restrict__ x, int64_t x_rs,
                                                     const T* __restrict__ res, int64_t r_rs,
                                                     T* __restrict__ h_out, int64_t h_rs,
                                                     const T* __restrict__ w, T* __restrict__ y,
                                                     int64_t y_rs, int D, float eps) {
  using V8 = typename Vec<T>::x8;
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * x_rs;
  V8 v[VPT];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * NT) * 8;
    if (c < D) {
      v[i] = *reinterpret_cast<const V8*>(xr + c);
      if (res) {
        const V8 r = *reinterpret_cast<const V8*>(res + row * r_rs + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (T)((float)v[i][j] + (float)r[j]);
        *reinterpret_cast<V8*>(h_out + row * h_rs + c) = v[i];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)v[i][j];
        ss += f * f;
      }
    }
  }
  const float var = block_sum<NT>(ss, red) / (float)D;
  const float inv = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * NT) * 8;
    if (c < D) {
      const V8 ww = *reinterpret_cast<const V8*>(w + c);
      V8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (T)((float)ww[j] * rnd<T>((float)v[i][j] * inv));
      *reinterpret_cast<V8*>(y + row * y_rs + c) = o;
    }
  }
}

// one thread = 8 rotation pairs (i, i + d/2) of one head of one row.  SPLIT: the row's heads are q | k | v
// (hq, then (heads - hq) / 2 each); q rotates in place, k rotates into kout (and in place too if keep_k) and v is
// copied into vout.  Destination of buffer row r: sequence b = r / T, row kv_row0 + r % T, or, with dst_b,
// sequence dst_b[r], row kv_row0 + pos[r]; strides kv_bs (sequence), kv_hs (head), kv_rs (row).  The IE sweep's
// suffix K/V go straight behind their shared prefix, the packed decode prefill's K/V straight into the cache.
template <typename E, bool SPLIT>
__global__ __launch_bounds__(256) void rope_kernel(E* __restrict__ qkv, int64_t rs, int rows, int T, int heads,
                                                   int d, const E* __restrict__ cos_t,
                                                   const E* __restrict__ sin_t, int64_t tab_rs,
                                                   const int64_t* __restrict__ pos, int hq, E* __restrict__ kout,
                                                   E* __restrict__ vout, int64_t kv_bs, int64_t kv_hs, int64_t kv_rs,
                                                   int kv_row0, const int64_t* __restrict__ dst_b, int keep_k) {
  using V8 = typename Vec<E>::x8;
  const unsigned half = (unsigned)d >> 1, vpp = half >> 3;  // vectors per half-row
  const unsigned gid = blockIdx.x * 256u + threadIdx.x;      // host guarantees rows*heads*vpp < 2^31
  if (gid >= (unsigned)rows * (unsigned)heads * vpp) return;
  const unsigned vi = gid % vpp;
  const unsigned rh = gid / vpp;
  const unsigned h = rh % (unsigned)heads;
  const unsigned row32 = rh / (unsigned)heads;
  const int64_t row = row32;
  E* base = qkv + row * rs + (int64_t)h * d + vi * 8;
  const V8 x1 = *reinterpret_cast<const V8*>(base);
  const V8 x2 = *reinterpret_cast<const V8*>(base + half);
  E* dst = base;
  E* dst2 = nullptr;                                         // second destination of a rotated k (keep_k)
  if (SPLIT && h >= (unsigned)hq) {
    const unsigned hkv = ((unsigned)heads - (unsigned)hq) >> 1;
    const bool is_v = h >= (unsigned)hq + hkv;
    const unsigned hk = h - (unsigned)hq - (is_v ? hkv : 0u);
    const int64_t b = dst_b ? dst_b[row] : (int64_t)(row32 / (unsigned)T);
    const int64_t t = dst_b ? pos[row] : (int64_t)(row32 % (unsigned)T);
    E* o = (is_v ? vout : kout) + b * kv_bs + (kv_row0 + t) * kv_rs + (int64_t)hk * kv_hs + vi * 8;
    if (is_v) {                                              // v: copied, not rotated
      *reinterpret_cast<V8*>(o) = x1;
      *reinterpret_cast<V8*>(o + half) = x2;
      return;
    }
    if (keep_k) dst2 = o;
    else dst = o;
  }
  const int64_t p = pos ? pos[row] : (int64_t)(row32 % (unsigned)T);
  const E* ct = cos_t + p * tab_rs + vi * 8;
  const E* st = sin_t + p * tab_rs + vi * 8;
  const V8 c1 = *reinterpret_cast<const V8*>(ct), c2 = *reinterpret_cast<const V8*>(ct + half);
  const V8 s1 = *reinterpret_cast<const V8*>(st), s2 = *reinterpret_cast<const V8*>(st + half);
  V8 o1, o2;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float a = (float)x1[j], b = (float)x2[j];
    // first half: x1*cos - x2*sin ; second half: x2*cos + x1*sin   (rotate_half = cat(-x2, x1))
    o1[j] = (E)(rnd<E>(a * (float)c1[j]) + rnd<E>(-b * (float)s1[j]));
    o2[j] = (E)(rnd<E>(b * (float)c2[j]) + rnd<E>(a * (float)s2[j]));
  }
  *reinterpret_cast<V8*>(dst) = o1;
  *reinterpret_cast<V8*>(dst + half) = o2;
  if (SPLIT && dst2) {
    *reinterpret_cast<V8*>(dst2) = o1;
    *reinterpret_cast<V8*>(dst2 + half) = o2;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void silu_mul_kernel(const T* __restrict__ gu, int64_t gu_rs,
                                                       T* __restrict__ y, int64_t y_rs, int rows, int F) {
  using V8 = typename Vec<T>::x8;
  const unsigned vpr = (unsigned)F >> 3;
  const unsigned gid = blockIdx.x * 256u + threadIdx.x;      // host guarantees rows*vpr < 2^31
  if (gid >= (unsigned)rows * vpr) return;
  const int64_t row = gid / vpr;
  const int c = (int)(gid % vpr) * 8;
  const V8 g = *reinterpret_cast<const V8*>(gu + row * gu_rs + c);
  const V8 u = *reinterpret_cast<const V8*>(gu + row * gu_rs + F + c);
  V8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = (float)g[j];
    const float s = rnd<T>(cram_silu<T>(x));
    o[j] = (T)(s * (float)u[j]);
  }
  *reinterpret_cast<V8*>(y + row * y_rs + c) = o;
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool m8(int64_t s) { return (s & 7) == 0; }

inline bool dtype_ok(int dtype) { return dtype == CRAM_DTYPE_BF16 || dtype == CRAM_DTYPE_F16; }

template <typename T>
int launch_rms(int rows, hipStream_t st, const void* x, int64_t x_rs, const void* r, int64_t r_rs, void* h,
               int64_t h_rs, const void* w, void* y, int64_t y_rs, int D, float eps) {
  const int vec = D / 8;
  const dim3 g(rows);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, g, dim3(256), 0, st, (const T*)x, x_rs, (const T*)r, r_rs, (T*)h, h_rs, (const T*)w,
                       (T*)y, y_rs, D, eps);
  };
  if (vec <= 256) go(rmsnorm_kernel<T, 256, 1>);
  else if (vec <= 512) go(rmsnorm_kernel<T, 256, 2>);
  else if (vec <= 1024) go(rmsnorm_kernel<T, 256, 4>);
  else return CRAM_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

}  // namespace

extern "C" {

int cram_rmsnorm(const void* x, int64_t x_rs, const void* residual, int64_t r_rs, void* h_out, int64_t h_rs,
                 const void* w, void* y, int64_t y_rs, int rows, int D, float eps, int dtype, cram_stream_t stream) {
  if (!x || !w || !y || rows < 0 || D <= 0 || (residual && !h_out)) return CRAM_ERR_INVALID_ARG;
  if (!dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (rows == 0) return CRAM_OK;
  if ((D & 7) || !m8(x_rs) || !m8(y_rs) || !al16(x) || !al16(y) || !al16(w)) return CRAM_ERR_ALIGNMENT;
  if (residual && (!m8(r_rs) || !m8(h_rs) || !al16(residual) || !al16(h_out))) return CRAM_ERR_ALIGNMENT;
  const hipStream_t st = (hipStream_t)stream;
  return dtype == CRAM_DTYPE_BF16
             ? launch_rms<__bf16>(rows, st, x, x_rs, residual, r_rs, h_out, h_rs, w, y, y_rs, D, eps)
             : launch_rms<_Float16>(rows, st, x, x_rs, residual, r_rs, h_out, h_rs, w, y, y_rs, D, eps);
}

int cram_rope_inplace(void* qkv, int64_t row_stride, int rows, int T, int heads, int d, const void* cos_t,
                      const void* sin_t, int64_t tab_rs, const int64_t* pos, int dtype, cram_stream_t stream) {
  if (!qkv || !cos_t || !sin_t || rows < 0 || heads <= 0 || T <= 0) return CRAM_ERR_INVALID_ARG;
  if (!dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (rows == 0) return CRAM_OK;
  if ((d & 15) || !m8(row_stride) || !m8(tab_rs) || !al16(qkv) || !al16(cos_t) || !al16(sin_t))
    return CRAM_ERR_ALIGNMENT;
  const int64_t total = (int64_t)rows * heads * (d / 16);
  if (total >= (1ll << 31)) return CRAM_ERR_INVALID_ARG;
  const dim3 g((unsigned)((total + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == CRAM_DTYPE_BF16)
    hipLaunchKernelGGL((rope_kernel<__bf16, false>), g, dim3(256), 0, st, (__bf16*)qkv, row_stride, rows, T, heads,
                       d, (const __bf16*)cos_t, (const __bf16*)sin_t, tab_rs, pos, heads, nullptr, nullptr, 0, 0, 0, 0, nullptr, 0);
  else
    hipLaunchKernelGGL((rope_kernel<_Float16, false>), g, dim3(256), 0, st, (_Float16*)qkv, row_stride, rows, T,
                       heads, d, (const _Float16*)cos_t, (const _Float16*)sin_t, tab_rs, pos, heads, nullptr, nullptr,
                       0, 0, 0, 0, nullptr, 0);
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

int cram_rope_split(void* qkv, int64_t row_stride, int rows, int T, int hq, int hkv, int d, const void* cos_t,
                    const void* sin_t, int64_t tab_rs, const int64_t* pos, void* kout, void* vout, int64_t kv_bs,
                    int64_t kv_hs, int64_t kv_rs, int kv_row0, const int64_t* dst_b, int keep_k, int dtype,
                    cram_stream_t stream) {
  if (!qkv || !cos_t || !sin_t || !kout || !vout || rows < 0 || hq <= 0 || hkv <= 0 || T <= 0 || kv_row0 < 0 ||
      (dst_b ? !pos : rows % T != 0))
    return CRAM_ERR_INVALID_ARG;
  if (!dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (rows == 0) return CRAM_OK;
  if ((d & 15) || !m8(row_stride) || !m8(tab_rs) || !m8(kv_bs) || !m8(kv_hs) || !m8(kv_rs) || !al16(qkv) || !al16(cos_t) ||
      !al16(sin_t) || !al16(kout) || !al16(vout))
    return CRAM_ERR_ALIGNMENT;
  const int heads = hq + 2 * hkv;
  const int64_t total = (int64_t)rows * heads * (d / 16);
  if (total >= (1ll << 31)) return CRAM_ERR_INVALID_ARG;
  const dim3 g((unsigned)((total + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == CRAM_DTYPE_BF16)
    hipLaunchKernelGGL((rope_kernel<__bf16, true>), g, dim3(256), 0, st, (__bf16*)qkv, row_stride, rows, T, heads,
                       d, (const __bf16*)cos_t, (const __bf16*)sin_t, tab_rs, pos, hq, (__bf16*)kout, (__bf16*)vout,
                       kv_bs, kv_hs, kv_rs, kv_row0, dst_b, keep_k);
  else
    hipLaunchKernelGGL((rope_kernel<_Float16, true>), g, dim3(256), 0, st, (_Float16*)qkv, row_stride, rows, T,
                       heads, d, (const _Float16*)cos_t, (const _Float16*)sin_t, tab_rs, pos, hq, (_Float16*)kout,
                       (_Float16*)vout, kv_bs, kv_hs, kv_rs, kv_row0, dst_b, keep_k);
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

int cram_silu_mul(const void* gu, int64_t gu_rs, void* y, int64_t y_rs, int rows, int F, int dtype,
                  cram_stream_t stream) {
  if (!gu || !y || rows < 0 || F <= 0) return CRAM_ERR_INVALID_ARG;
  if (!dtype_ok(dtype)) return CRAM_ERR_UNSUPPORTED;
  if (rows == 0) return CRAM_OK;
  if ((F & 7) || !m8(gu_rs) || !m8(y_rs) || !al16(gu) || !al16(y)) return CRAM_ERR_ALIGNMENT;
  const int64_t total = (int64_t)rows * (F / 8);
  if (total >= (1ll << 31)) return CRAM_ERR_INVALID_ARG;
  const dim3 g((unsigned)((total + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == CRAM_DTYPE_BF16)
    hipLaunchKernelGGL(silu_mul_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)gu, gu_rs, (__bf16*)y, y_rs,
                       rows, F);
  else
    hipLaunchKernelGGL(silu_mul_kernel<_Float16>, g, dim3(256), 0, st, (const _Float16*)gu, gu_rs, (_Float16*)y,
                       y_rs, rows, F);
  return hipGetLastError() == hipSuccess ? CRAM_OK : CRAM_ERR_LAUNCH;
}

}  // extern "C"
