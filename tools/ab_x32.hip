// A/B and agreement check of prefill_x32_kernel (two workgroups per CU, 32 rows per wave) against the library's
// prefill_kernel on the same inputs, in one process (arm "x32b" launches x32 again: the run-to-run noise of the A/B;
// round 2's one-wave-per-SIMD x64 kernel held that arm until round 4 removed it):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ab_x32.hip -o tools/ab_x32 && tools/ab_x32
// Cases: the IE-sweep shape (B=33, T=962, Llama-3 GQA 32/8, d 128, fused QKV layout), a suffix-style call (queries at
// positions p0.., keys 0..p0+T), a biased call (some heads enabled, -inf and log 0.1 spans), the 8.3k-token prompt.
// Prints max |x - library| and the kernels' times (median of 5 rounds of 10 launches each, interleaved).
// -DCRAM_X32_STAMPS: per-phase cycle stamps of the kernel.
#include "../cram_amd/csrc/cram_attn.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Case {
  const char* name;
  int B, T, p0, Hq, Hkv, biased;
};

static double flops_of(const Case& c) {
  // causal visible keys: row i (0-based) at position p0 + i sees p0 + i + 1 keys
  double vis = 0;
  for (int i = 0; i < c.T; ++i) vis += c.p0 + i + 1;
  return 4.0 * 128 * c.Hq * c.B * vis;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  const char* only = argc > 2 ? argv[2] : nullptr;   // substring of the case names to run
  std::vector<Case> cases = {
      {"sweep B=33 T=962", 33, 962, 0, 32, 8, 0},
      {"suffix B=33 T=937 p0=25", 33, 937, 25, 32, 8, 0},
      {"biased B=3 T=517", 3, 517, 0, 32, 8, 1},
      {"ragged B=2 T=77", 2, 77, 0, 32, 8, 1},
      {"8k B=1 T=8300", 1, 8300, 0, 32, 8, 0},
      {"8k biased B=1 T=8300", 1, 8300, 0, 32, 8, 1},
  };
  const int d = 128;
  bool all_ok = true;
  for (const Case& c : cases) {
    if (only && !strstr(c.name, only)) continue;
    const int S = c.p0 + c.T;
    const int N = (c.Hq + 2 * c.Hkv) * d;   // fused QKV row for the queries; K/V in their own [B][S][Hkv][d] buffers
    const size_t nq = (size_t)c.B * c.T * N, nkv = (size_t)c.B * S * c.Hkv * d, no = (size_t)c.B * c.T * c.Hq * d;
    std::vector<__bf16> hq(nq), hk(nkv), hv(nkv);
    std::mt19937 rng(1234);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto& x : hq) x = (__bf16)(nd(rng) * 1.5f);
    for (auto& x : hk) x = (__bf16)(nd(rng) * 1.5f);
    for (auto& x : hv) x = (__bf16)nd(rng);
    std::vector<float> hb((size_t)c.B * S, 0.f);
    std::vector<uint8_t> he((size_t)c.B * c.Hq, 0);
    int W = 0;
    if (c.biased) {
      W = S - 3;
      for (int b = 0; b < c.B; ++b) {
        for (int j = 0; j < S; ++j) {
          const int seg = (j / 41) % 5;   // spans of 41 keys: 1.0, 0.1, 0, 1.0, 0.1 credibility weights
          hb[(size_t)b * S + j] = j == 0 ? 0.f : seg == 1 || seg == 4 ? logf(0.1f) : seg == 2 ? -INFINITY : 0.f;
        }
        for (int h = 0; h < c.Hq; ++h) he[(size_t)b * c.Hq + h] = ((h * 7 + b) % 3) != 0;
      }
    }
    __bf16 *q, *k, *v, *o1, *o2, *o3;
    float* bias;
    uint8_t* en;
    CK(hipMalloc(&q, nq * 2)); CK(hipMalloc(&k, nkv * 2)); CK(hipMalloc(&v, nkv * 2));
    CK(hipMalloc(&o1, no * 2)); CK(hipMalloc(&o2, no * 2)); CK(hipMalloc(&o3, no * 2));
    CK(hipMalloc(&bias, hb.size() * 4)); CK(hipMalloc(&en, he.size()));
    CK(hipMemcpy(q, hq.data(), nq * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(k, hk.data(), nkv * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv.data(), nkv * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(en, he.data(), he.size(), hipMemcpyHostToDevice));
    CK(hipMemset(o1, 0, no * 2));
    CK(hipMemset(o2, 0, no * 2));
    CK(hipMemset(o3, 0, no * 2));

    PrefillParams p{};
    p.q = q; p.q_sb = (int64_t)c.T * N; p.q_sh = d; p.q_st = N;
    p.k = k; p.k_sb = (int64_t)S * c.Hkv * d; p.k_sh = d; p.k_st = (int64_t)c.Hkv * d;
    p.v = v; p.v_sb = p.k_sb; p.v_sh = d; p.v_st = p.k_st;
    p.o_sb = (int64_t)c.T * c.Hq * d; p.o_sh = d; p.o_st = (int64_t)c.Hq * d;
    p.bias = c.biased ? bias : nullptr; p.bias_sb = S;
    p.enable = c.biased ? en : nullptr; p.en_sb = c.Hq;
    p.B = c.B; p.Hq = c.Hq; p.Hkv = c.Hkv; p.Tq = c.T; p.S = S; p.W = W; p.q_pos0 = c.p0;
    p.scale_log2 = kLog2e / sqrtf((float)d);
    p.cu = nullptr;
    PrefillParams p1 = p, p2 = p, p3 = p;
    p1.o = o1; p1.hp = 4; p1.nqb = (c.T + 31) / 32; p1.nblocks = p1.nqb * (c.Hq / 4) * c.B;
    p2.o = o2; p2.hp = 4; p2.nqb = (c.T + 31) / 32; p2.nblocks = p2.nqb * (c.Hq / 4) * c.B;
    p3.o = o3; p3.hp = 4; p3.nqb = (c.T + 31) / 32; p3.nblocks = p3.nqb * (c.Hq / 4) * c.B;
    auto run = [&](int which) {
      if (which == 0)
        hipLaunchKernelGGL((prefill_kernel<__bf16, 128, 64, 2>), dim3(p1.nblocks), dim3(256), 0, 0, p1);
      else if (which == 1)
        hipLaunchKernelGGL(prefill_x32_kernel, dim3(p3.nblocks), dim3(256), 0, 0, p2);
      else
        hipLaunchKernelGGL(prefill_x32_kernel, dim3(p3.nblocks), dim3(256), 0, 0, p3);
    };
    run(0);
    run(1);
    run(2);
    CK(hipDeviceSynchronize());
    std::vector<__bf16> a(no), bb(no);
    CK(hipMemcpy(a.data(), o1, no * 2, hipMemcpyDeviceToHost));
    double md[3] = {}, sd[3] = {};
    size_t nbad[3] = {}, nnan[3] = {};
    for (int w = 1; w < 3; ++w) {
      CK(hipMemcpy(bb.data(), w == 1 ? o2 : o3, no * 2, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < no; ++i) {
        const double x = (float)a[i], y = (float)bb[i];
        if (std::isnan(y) || std::isinf(y)) { ++nnan[w]; continue; }
        const double e = fabs(x - y);
        md[w] = std::max(md[w], e);
        sd[w] += e;
        if (e > 2e-2 + 2e-2 * fabs(x)) ++nbad[w];
      }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<float> t[3];
    for (int rnd = 0; rnd < 5; ++rnd)
      for (int w = 0; w < 3; ++w) {
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) run(w);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[w].push_back(ms / iters);
      }
    for (auto& x : t) std::sort(x.begin(), x.end());
#ifdef CRAM_X32_STAMPS
    {
      unsigned long long* st;
      const size_t ns = (size_t)p3.nblocks * 4 * 10;
      CK(hipMalloc(&st, ns * 8));
      CK(hipMemset(st, 0, ns * 8));
      // >= 2 s of back-to-back launches first, so the clock the stamps see is the one the chip holds under this load
      {
        hipEvent_t w0, w1;
        CK(hipEventCreate(&w0)); CK(hipEventCreate(&w1));
        float wms = 0.f;
        CK(hipEventRecord(w0));
        for (int i = 0; wms < 2000.f; ++i) {
          run(2);
          if ((i & 255) == 255) { CK(hipEventRecord(w1)); CK(hipEventSynchronize(w1)); CK(hipEventElapsedTime(&wms, w0, w1)); }
        }
      }
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_x32_stamps), &st, sizeof(st)));
      run(2);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> hs(ns);
      CK(hipMemcpy(hs.data(), st, ns * 8, hipMemcpyDeviceToHost));
      double sum[10] = {};
      for (size_t w = 0; w < (size_t)p3.nblocks * 4; ++w)
        for (int k = 0; k < 10; ++k) sum[k] += (double)hs[w * 10 + k];
      const double nw = (double)p3.nblocks * 4, steps = sum[4];
      printf("  x32 in-kernel clock %.3f GHz (wave cycles / 100-MHz ticks, after 2 s of launches)\n",
             sum[6] / sum[7] * 0.1);
      printf("  x32 stamps per wave: prologue %.0f, epilogue %.0f cycles; per step: A %.0f, B %.0f (R: vmcnt wait %.0f, "
             "barrier %.0f) (steps/wave %.1f)\n", sum[0] / nw, sum[5] / nw, sum[1] / steps, sum[2] / steps,
             sum[3] / steps, sum[8] / steps, steps / nw);
      unsigned long long* nul = nullptr;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_x32_stamps), &nul, sizeof(nul)));
      CK(hipFree(st));
    }
#endif
    const double fl = flops_of(c);
    const bool ok = nbad[1] == 0 && nnan[1] == 0 && nbad[2] == 0 && nnan[2] == 0;
    all_ok &= ok;
    printf("%-26s lib %.3f ms (%5.0f TF/s) | x32b %.3f ms (%5.0f) x%.3f max|d| %.2e mean %.2e bad %zu nan %zu | "
           "x32 %.3f ms (%5.0f) x%.3f max|d| %.2e mean %.2e bad %zu nan %zu %s\n",
           c.name, t[0][2], fl / t[0][2] / 1e9, t[1][2], fl / t[1][2] / 1e9, t[0][2] / t[1][2], md[1], sd[1] / no,
           nbad[1], nnan[1], t[2][2], fl / t[2][2] / 1e9, t[0][2] / t[2][2], md[2], sd[2] / no, nbad[2], nnan[2],
           ok ? "OK" : "MISMATCH");
    fflush(stdout);
    CK(hipFree(q)); CK(hipFree(k)); CK(hipFree(v)); CK(hipFree(o1)); CK(hipFree(o2)); CK(hipFree(o3)); CK(hipFree(bias)); CK(hipFree(en));
  }
  return all_ok ? 0 : 2;
}
