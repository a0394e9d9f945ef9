// Host-side AddressSanitizer / UBSan driver for the C-ABI (include/cram_attn.h): no GPU, no launches.
//
// Built by tests/asan/Makefile from the product sources with the host pass sanitized (hipcc --cuda-host-only:
// the kernels' host stubs only, device code is irrelevant to the paths exercised here).  It drives
//   * every argument-validation path of every device entry point (null pointers, sizes, unsupported head dim
//     and element type, misaligned strides / pointers, missing split-S workspace, 32-bit extent limits), which
//     return before any HIP call;
//   * the kernel-selection knobs;
//   * cram_passage_weights (host C++) on random monotone and non-monotone offset maps, empty prompts and
//     prompts without passages, checked against a naive last-match scan (re_weighting.py:105-110).
// Exit status 0 = every expectation held and the sanitizers reported nothing.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "cram_attn.h"

static int g_fail = 0;
#define EXPECT(cond)                                                         \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

static void validation_paths() {
  void* f = reinterpret_cast<void*>(uintptr_t(1) << 20);   // 16-B aligned, never dereferenced
  void* mis = reinterpret_cast<void*>((uintptr_t(1) << 20) + 2);
  // prefill
  EXPECT(cram_attn_prefill(nullptr, 0, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, 0, 1.f, nullptr,
                           0, nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 3, 2, 1, 1, 128, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);     // Hq % Hkv
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 0, 1, 1, 1, 1, 128, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);     // B = 0
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, -1, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);     // q_pos0 < 0
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 96, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_UNSUPPORTED);     // d = 96
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, 5, nullptr) == CRAM_ERR_UNSUPPORTED);                    // dtype
  EXPECT(cram_attn_prefill(mis, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_ALIGNMENT);
  EXPECT(cram_attn_prefill(f, 0, 0, 12, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, 0, 1.f, nullptr, 0,
                           nullptr, 0, 0, CRAM_DTYPE_F16, nullptr) == CRAM_ERR_ALIGNMENT);
  float* fb = reinterpret_cast<float*>(f);
  uint8_t* fe = reinterpret_cast<uint8_t*>(f);
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 1, 128, 0, 1.f, fb, 8, fe, 8,
                           -1, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);                // W < 0
  EXPECT(cram_attn_prefill(f, 0, 0, 8, f, 0, 0, int64_t(1) << 20, f, 0, 0, 8, f, 0, 0, 8, 1, 1, 1, 1, 4096, 128, 0,
                           1.f, nullptr, 0, nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_UNSUPPORTED);  // 2^31 extent
  // varlen
  EXPECT(cram_attn_prefill_varlen(f, 8, 8, f, 8, 8, f, 8, 8, f, 8, 8, nullptr, 1, 4, 1, 1, 128, 1.f, nullptr, 0,
                                  nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_attn_prefill_varlen(f, 8, 8, f, 8, 8, f, 8, 8, f, 8, 8, reinterpret_cast<int32_t*>(f), 1, 4, 1, 1, 64,
                                  1.f, nullptr, 0, nullptr, 0, 0, 9, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_attn_prefill_varlen(f, 8, 4, f, 8, 8, f, 8, 8, f, 8, 8, reinterpret_cast<int32_t*>(f), 1, 4, 1, 1, 64,
                                  1.f, nullptr, 0, nullptr, 0, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_ALIGNMENT);
  // decode
  EXPECT(cram_attn_decode_workspace_size(2, 32, 128, 4) == size_t(2) * 32 * 4 * 130 * 4);
  EXPECT(cram_attn_decode_workspace_size(2, 32, 128, 1) == 0);
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 1, 1, 1, 4, nullptr, 128, 1.f, nullptr, 0,
                          nullptr, 0, 0, 4, nullptr, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_WORKSPACE);
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 1, 1, 1, 4, nullptr, 128, 1.f, nullptr, 0,
                          nullptr, 0, 0, 4, f, 16, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_WORKSPACE);   // too small
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 70000, 1, 1, 4, nullptr, 128, 1.f, nullptr, 0,
                          nullptr, 0, 0, 1, nullptr, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);  // B > 65535
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 1, 1, 1, 4, nullptr, 128, 1.f, nullptr, 0,
                          nullptr, 0, 0, 0, nullptr, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_INVALID_ARG);  // 0 splits
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 1, 3, 1, 4, nullptr, 32, 1.f, nullptr, 0,
                          nullptr, 0, 0, 1, nullptr, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_attn_decode(f, 0, 0, f, 0, 0, 8, f, 0, 0, 8, f, 0, 0, 1, 3, 1, 4, nullptr, 128, 1.f, nullptr, 0,
                          nullptr, 0, 0, 1, nullptr, 0, CRAM_DTYPE_BF16, nullptr) == CRAM_ERR_UNSUPPORTED);  // G = 3
  // answer logits
  EXPECT(cram_answer_logits(nullptr, 8, f, 8, reinterpret_cast<int32_t*>(f), 1, 8, 0, fb, 0, nullptr) ==
         CRAM_ERR_INVALID_ARG);
  EXPECT(cram_answer_logits(f, 8, f, 8, reinterpret_cast<int32_t*>(f), 0, 8, 0, fb, 0, nullptr) == CRAM_OK);  // n = 0
  EXPECT(cram_answer_logits(f, 8, f, 8, reinterpret_cast<int32_t*>(f), 1, 12, 0, fb, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  // fused elementwise
  EXPECT(cram_rmsnorm(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, 1, 8, 1e-5f, 0, nullptr) ==
         CRAM_ERR_INVALID_ARG);
  EXPECT(cram_rmsnorm(f, 8, f, 8, nullptr, 0, f, f, 8, 1, 8, 1e-5f, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_rmsnorm(f, 8, nullptr, 0, nullptr, 0, f, f, 8, 0, 8, 1e-5f, 0, nullptr) == CRAM_OK);   // rows = 0
  EXPECT(cram_rmsnorm(f, 8, nullptr, 0, nullptr, 0, f, f, 8, 1, 12, 1e-5f, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  EXPECT(cram_rope_inplace(nullptr, 8, 1, 1, 1, 128, f, f, 128, nullptr, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_rope_inplace(f, 8, 1, 1, 1, 128, f, f, 128, nullptr, 3, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_rope_split(f, 8, 1, 1, 1, 1, 128, f, f, 128, nullptr, nullptr, f, 8, 8, 8, 0, nullptr, 0, 0,
                         nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_silu_mul(f, 8, f, 8, 1, 16, 7, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_silu_mul(f, 8, f, 8, 1, 12, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  EXPECT(cram_silu_mul(f, 8, f, 8, 0, 16, 0, nullptr) == CRAM_OK);
  // projection GEMM: validated before any launch
  EXPECT(cram_gemm(nullptr, 64, f, 64, f, 256, 1, 256, 64, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm(f, 64, f, 64, f, 256, 0, 256, 64, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm(f, 64, f, 64, f, 256, 1, 256, 64, 2, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm(f, 64, f, 64, f, 256, 1, 256, 64, CRAM_GEMM_STORE, 5, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm(f, 64, f, 64, f, 256, 1, 200, 64, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm(f, 48, f, 48, f, 256, 1, 256, 48, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm(f, 68, f, 64, f, 256, 1, 256, 64, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  EXPECT(cram_gemm(f, 64, f, 64, f, 128, 1, 512, 64, CRAM_GEMM_STORE, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm(f, 64, f, 64, f, 255, 1, 512, 64, CRAM_GEMM_SILU_MUL, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  // residual and q/k/v + RoPE GEMMs: overlap, alignment, head dim, rows <= M
  char* const fc = static_cast<char*>(f);
  void* g = fc + (1 << 16);
  EXPECT(cram_gemm_residual(f, 64, f, 64, nullptr, 256, f, 256, 1, 256, 64, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm_residual(f, 64, f, 64, fc + 16, 256, f, 256, 1, 256, 64, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm_residual(f, 64, f, 64, g, 260, f, 256, 1, 256, 64, 0, nullptr) == CRAM_ERR_ALIGNMENT);
  EXPECT(cram_gemm_residual(f, 64, f, 64, g, 256, f, 256, 1, 200, 64, 0, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm_rope(f, 128, f, 128, nullptr, f, 6144, 256, 128, 257, 256, 32, 8, 128, f, f, 128, nullptr, 0, nullptr,
                        nullptr, 0, 0, 0, 0, nullptr, 0, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm_rope(f, 128, f, 128, nullptr, f, 6144, 256, 128, 256, 256, 32, 8, 64, f, f, 128, nullptr, 0, nullptr,
                        nullptr, 0, 0, 0, 0, nullptr, 0, 0, nullptr) == CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm_rope(f, 128, f, 128, nullptr, f, 6144, 256, 128, 256, 256, 32, 8, 128, f, f, 128, nullptr, 0, f,
                        nullptr, 0, 0, 0, 0, nullptr, 0, 0, nullptr) == CRAM_ERR_INVALID_ARG);
  // error strings and knobs
  for (int c = 1; c >= -7; --c) EXPECT(cram_strerror(c) != nullptr && std::strlen(cram_strerror(c)) > 0);
  EXPECT(cram_abi_version() == CRAM_ABI_VERSION);
  EXPECT(cram_set_knob(CRAM_KNOB_COUNT, 0) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_set_knob(-1, 0) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_set_knob(CRAM_KNOB_PREFILL_VARIANT, 5) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_U, 3) == CRAM_ERR_INVALID_ARG);
  int kv = 0;
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_U, 2) == CRAM_OK && cram_get_knob(CRAM_KNOB_DECODE_U, &kv) == CRAM_OK &&
         kv == 2);
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_U, -1) == CRAM_OK && cram_get_knob(CRAM_KNOB_DECODE_U, &kv) == CRAM_OK &&
         kv == -1);
  kv = 5;
  EXPECT(cram_get_knob(7, &kv) == CRAM_ERR_INVALID_ARG && kv == 5);
  EXPECT(cram_get_knob(CRAM_KNOB_DECODE_U, nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_MFMA, 2) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_MFMA, 0) == CRAM_OK && cram_get_knob(CRAM_KNOB_DECODE_MFMA, &kv) == CRAM_OK &&
         kv == 0);
  EXPECT(cram_set_knob(CRAM_KNOB_DECODE_MFMA, -1) == CRAM_OK);
  // knobs from several host threads at once (std::call_once + atomics): no data race for the sanitizer to see
  {
    std::vector<std::thread> th;
    for (int i = 0; i < 8; ++i)
      th.emplace_back([i] {
        int v = 0;
        for (int r = 0; r < 1000; ++r) {
          cram_set_knob(CRAM_KNOB_DECODE_U, (i & 1) ? 1 : 2);
          cram_get_knob(CRAM_KNOB_DECODE_U, &v);
        }
      });
    for (auto& t : th) t.join();
    EXPECT(cram_set_knob(CRAM_KNOB_DECODE_U, -1) == CRAM_OK);
  }
  // split-K GEMM argument validation
  const size_t ws = cram_gemm_splitk_workspace_size(16, 512, 4);
  EXPECT(ws == 4u * 16u * 512u * 4u && cram_gemm_splitk_workspace_size(0, 512, 4) == 0);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 3, CRAM_GEMM_STORE, nullptr, f, ws, 0, nullptr) ==
         CRAM_ERR_UNSUPPORTED);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 4, CRAM_GEMM_SILU_MUL, nullptr, f, ws, 0,
                          nullptr) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 4, CRAM_GEMM_SILU_MUL_CAT, f, f, ws, 0, nullptr) ==
         CRAM_ERR_INVALID_ARG);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 4, CRAM_GEMM_STORE, nullptr, nullptr, ws, 0,
                          nullptr) == CRAM_ERR_WORKSPACE);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 4, CRAM_GEMM_STORE, nullptr, f, ws - 1, 0,
                          nullptr) == CRAM_ERR_WORKSPACE);
  EXPECT(cram_gemm_splitk(f, 512, f, 512, f, 512, 16, 512, 512, 4, CRAM_GEMM_STORE, nullptr, f, ws, 7, nullptr) ==
         CRAM_ERR_UNSUPPORTED);
}

static uint16_t f16_bits(float x) {
  _Float16 h = static_cast<_Float16>(x);
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}

// naive restatement of re_weighting.py:105-110 over one prompt
static void naive(const std::vector<int64_t>& st, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi,
                  const std::vector<float>& sc, std::vector<int32_t>& slo, std::vector<int32_t>& shi,
                  std::vector<uint16_t>& w) {
  const int64_t T = (int64_t)st.size();
  w.assign(T, f16_bits(1.f));
  for (size_t p = 0; p < lo.size(); ++p) {
    int64_t a = -1, e = -1;
    for (int64_t t = 0; t < T; ++t) {
      if (st[t] <= lo[p]) a = t;
      if (st[t] <= hi[p]) e = t;
    }
    slo.push_back((int32_t)a);
    shi.push_back((int32_t)e);
    for (int64_t t = a; t <= e; ++t) w[t] = f16_bits(sc[p]);
  }
}

static void passage_weights() {
  std::mt19937_64 rng(12345);
  for (int trial = 0; trial < 200; ++trial) {
    const int B = 1 + (int)(rng() % 5);
    std::vector<int64_t> cu_tok{0}, cu_par{0}, st, lo, hi;
    std::vector<float> sc;
    std::vector<int32_t> exp_lo, exp_hi;
    std::vector<uint16_t> exp_w;
    for (int b = 0; b < B; ++b) {
      const int T = (int)(rng() % 300);                     // empty prompts included
      std::vector<int64_t> s(T);
      int64_t c = 0;
      for (int t = 0; t < T; ++t) {
        c += 1 + (int64_t)(rng() % 6);
        s[t] = c;
      }
      if (T > 4 && rng() % 3 == 0) s[T / 2] = 0;               // special token at (0, 0): non-monotone row
      if (T > 0) s[0] = 0;
      const int P = T > 0 ? (int)(rng() % 6) : 0;             // prompts without passages included
      std::vector<int64_t> l, h;
      std::vector<float> v;
      for (int p = 0; p < P; ++p) {
        const int64_t a = (int64_t)(rng() % (uint64_t)(c + 1));
        l.push_back(a);
        h.push_back(a + (int64_t)(rng() % 200));
        const float choices[4] = {0.f, 0.1f, 1.f, 0.37f};
        v.push_back(choices[rng() % 4]);
      }
      std::vector<int32_t> el, eh;
      std::vector<uint16_t> ew;
      naive(s, l, h, v, el, eh, ew);
      st.insert(st.end(), s.begin(), s.end());
      lo.insert(lo.end(), l.begin(), l.end());
      hi.insert(hi.end(), h.begin(), h.end());
      sc.insert(sc.end(), v.begin(), v.end());
      exp_lo.insert(exp_lo.end(), el.begin(), el.end());
      exp_hi.insert(exp_hi.end(), eh.begin(), eh.end());
      exp_w.insert(exp_w.end(), ew.begin(), ew.end());
      cu_tok.push_back((int64_t)st.size());
      cu_par.push_back((int64_t)lo.size());
    }
    // exact-size heap buffers so ASan sees any overrun
    auto* out_lo = new int32_t[lo.size() + 1];
    auto* out_hi = new int32_t[hi.size() + 1];
    auto* w = new uint16_t[st.size() + 1];
    const int rc = cram_passage_weights(B, cu_tok.data(), st.data(), cu_par.data(), lo.data(), hi.data(), sc.data(),
                                        out_lo, out_hi, w);
    EXPECT(rc == CRAM_OK);
    if (rc == CRAM_OK) {
      for (size_t p = 0; p < lo.size(); ++p) EXPECT(out_lo[p] == exp_lo[p] && out_hi[p] == exp_hi[p]);
      for (size_t t = 0; t < st.size(); ++t) EXPECT(w[t] == exp_w[t]);
    }
    delete[] out_lo;
    delete[] out_hi;
    delete[] w;
  }
  // error paths: passage not found, inverted range, precedes every token, null buffers, B = 0
  int64_t cu_t[2] = {0, 3}, cu_p[2] = {0, 1}, st[3] = {5, 6, 7}, lo[1] = {-1}, hi[1] = {4};
  float sc[1] = {0.1f};
  int32_t a[1], e[1];
  uint16_t w[3];
  EXPECT(cram_passage_weights(1, cu_t, st, cu_p, lo, hi, sc, a, e, w) == CRAM_ERR_INVALID_ARG);
  lo[0] = 6; hi[0] = 5;
  EXPECT(cram_passage_weights(1, cu_t, st, cu_p, lo, hi, sc, a, e, w) == CRAM_ERR_INVALID_ARG);
  lo[0] = 2; hi[0] = 4;
  EXPECT(cram_passage_weights(1, cu_t, st, cu_p, lo, hi, sc, a, e, w) == CRAM_ERR_INVALID_ARG);
  EXPECT(cram_passage_weights(1, cu_t, st, cu_p, lo, hi, sc, nullptr, e, w) == CRAM_ERR_INVALID_ARG);
  int64_t z[1] = {0};
  EXPECT(cram_passage_weights(0, z, nullptr, z, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == CRAM_OK);
  EXPECT(cram_passage_weights(-1, z, nullptr, z, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) ==
         CRAM_ERR_INVALID_ARG);
}

int main() {
  validation_paths();
  passage_weights();
  if (g_fail) {
    std::fprintf(stderr, "abi_asan: %d expectation(s) failed\n", g_fail);
    return 1;
  }
  std::printf("abi_asan: all expectations held\n");
  return 0;
}
