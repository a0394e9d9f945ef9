/*
 * abi_demo.c — the C-ABI of include/cram_attn.h driven from plain C (no Python, no torch): one
 * credibility-biased causal GQA prefill on the GPU checked against a double-precision CPU loop, plus the
 * error path.  Shows what a non-Python host (the reference's callers bind it via ctypes; a C/C++ or other
 * runtime links it directly) needs: device buffers from the HIP runtime, element strides, a stream.
 *
 * Build:  make -C examples          (gcc + /opt/rocm HIP runtime + ../cram_amd/libcram_attn.so)
 * Run:    examples/abi_demo         (exit status 0 when max |err| <= 3e-2, bf16 output tolerance)
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "cram_attn.h"

static uint16_t f2bf(float f) {                      /* round to nearest even */
  union { float f; uint32_t u; } x = {f};
  uint32_t lsb = (x.u >> 16) & 1u;
  return (uint16_t)((x.u + 0x7FFFu + lsb) >> 16);
}
static float bf2f(uint16_t h) {
  union { uint32_t u; float f; } x = {(uint32_t)h << 16};
  return x.f;
}
static float frand(unsigned* s) {                    /* uniform in [-1, 1) */
  *s = *s * 1664525u + 1013904223u;
  return (float)((*s >> 8) & 0xFFFFFF) / 8388608.0f - 1.0f;
}

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

int main(void) {
  const int B = 2, Hq = 8, Hkv = 2, T = 200, d = 128, W = 190, G = Hq / Hkv;
  const size_t nq = (size_t)B * T * Hq * d, nk = (size_t)B * Hkv * T * d;
  uint16_t* hq = malloc(nq * 2); uint16_t* hk = malloc(nk * 2); uint16_t* hv = malloc(nk * 2);
  uint16_t* ho = malloc(nq * 2);
  float* bias = malloc((size_t)B * T * 4);
  uint8_t en[2 * 8];
  unsigned seed = 7;
  for (size_t i = 0; i < nq; ++i) hq[i] = f2bf(frand(&seed));
  for (size_t i = 0; i < nk; ++i) { hk[i] = f2bf(frand(&seed)); hv[i] = f2bf(frand(&seed)); }
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < T; ++j)    /* the hook's values: log 0 -> -inf, log 0.1 (fp16 log, bf16) -> -2.296875 */
      bias[b * T + j] = (j >= 10 && j < 40) ? -INFINITY : (j >= 60 && j < 120) ? -2.296875f : 0.0f;
  for (int i = 0; i < B * Hq; ++i) en[i] = (uint8_t)(i % 2);

  /* q, o token-major [B][T][Hq][d]; k, v head-major [B][Hkv][T][d] -- any element strides work */
  void *dq, *dk, *dv, *dout, *dbias, *den;
  CHECK(hipMalloc(&dq, nq * 2)); CHECK(hipMalloc(&dk, nk * 2)); CHECK(hipMalloc(&dv, nk * 2));
  CHECK(hipMalloc(&dout, nq * 2)); CHECK(hipMalloc(&dbias, (size_t)B * T * 4)); CHECK(hipMalloc(&den, sizeof en));
  CHECK(hipMemcpy(dq, hq, nq * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dk, hk, nk * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dv, hv, nk * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dbias, bias, (size_t)B * T * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(den, en, sizeof en, hipMemcpyHostToDevice));
  const float scale = 1.0f / sqrtf((float)d);
  int rc = cram_attn_prefill(dq, (int64_t)T * Hq * d, d, (int64_t)Hq * d,
                             dk, (int64_t)Hkv * T * d, (int64_t)T * d, d,
                             dv, (int64_t)Hkv * T * d, (int64_t)T * d, d,
                             dout, (int64_t)T * Hq * d, d, (int64_t)Hq * d,
                             B, Hq, Hkv, T, T, d, 0, scale, dbias, T, den, Hq, W, CRAM_DTYPE_BF16, NULL);
  if (rc != CRAM_OK) { fprintf(stderr, "cram_attn_prefill: %s\n", cram_strerror(rc)); return 3; }
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(ho, dout, nq * 2, hipMemcpyDeviceToHost));

  double max_err = 0.0;
  double* s = malloc((size_t)T * sizeof(double));
  for (int b = 0; b < B; ++b)
    for (int h = 0; h < Hq; ++h)
      for (int i = 0; i < T; ++i) {
        const uint16_t* qi = hq + (((size_t)b * T + i) * Hq + h) * d;
        const size_t kvh = ((size_t)b * Hkv + h / G) * T * d;
        double mx = -INFINITY, den_ = 0.0;
        for (int j = 0; j <= i; ++j) {
          double acc = 0.0;
          for (int c = 0; c < d; ++c) acc += (double)bf2f(qi[c]) * bf2f(hk[kvh + (size_t)j * d + c]);
          s[j] = acc * scale + ((en[b * Hq + h] && j < W) ? bias[b * T + j] : 0.0);
          if (s[j] > mx) mx = s[j];
        }
        for (int j = 0; j <= i; ++j) { s[j] = exp(s[j] - mx); den_ += s[j]; }
        for (int c = 0; c < d; ++c) {
          double o = 0.0;
          for (int j = 0; j <= i; ++j) o += s[j] * bf2f(hv[kvh + (size_t)j * d + c]);
          const double err = fabs(o / den_ - bf2f(ho[(((size_t)b * T + i) * Hq + h) * d + c]));
          if (err > max_err) max_err = err;
        }
      }
  /* the error path: an unsupported head dim is rejected before any launch */
  rc = cram_attn_prefill(dq, 0, 0, 0, dk, 0, 0, 0, dv, 0, 0, 0, dout, 0, 0, 0,
                         1, 1, 1, 1, 1, 96, 0, 1.0f, NULL, 0, NULL, 0, 0, CRAM_DTYPE_BF16, NULL);
  printf("abi %d: prefill B=%d Hq=%d Hkv=%d T=%d d=%d max|err|=%.3e; d=96 -> %d (%s)\n", cram_abi_version(), B, Hq,
         Hkv, T, d, max_err, rc, cram_strerror(rc));
  hipFree(dq); hipFree(dk); hipFree(dv); hipFree(dout); hipFree(dbias); hipFree(den);
  free(hq); free(hk); free(hv); free(ho); free(bias); free(s);
  return (max_err <= 3e-2 && rc == CRAM_ERR_UNSUPPORTED) ? 0 : 1;
}
