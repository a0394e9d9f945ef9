// Diagnostic: where a prefill_kernel tile's cycles go (s_memtime stamps, MI355X guide §7 idiom).
// Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCRAM_STAMPS tools/stamp_prefill.hip -o tools/stamp_prefill
// Run:    tools/stamp_prefill B T        (Llama-3 GQA 32/8, d 128, random bf16 q/k/v)
// Prints the mean / median shader cycles per tile phase over every (workgroup, wave, computed tile):
//   QK   loop top -> row max known (K reads + 16 MFMAs + max)     SM   -> exponentials + row sum
//   PV   -> rescale + P pack + V^T reads + 16 MFMAs issued       BAR  -> bias write + barrier
#include "../cram_amd/csrc/cram_attn.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 33, T = argc > 2 ? atoi(argv[2]) : 962;
  const int Hq = 32, Hkv = 8, d = 128;
  const size_t nq = (size_t)B * T * Hq * d, nk = (size_t)B * T * Hkv * d;
  std::vector<__bf16> hq(nq), hk(nk), hv(nk);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : hq) x = (__bf16)nd(rng);
  for (auto& x : hk) x = (__bf16)nd(rng);
  for (auto& x : hv) x = (__bf16)nd(rng);
  __bf16 *q, *k, *v, *o;
  hipMalloc(&q, nq * 2); hipMalloc(&k, nk * 2); hipMalloc(&v, nk * 2); hipMalloc(&o, nq * 2);
  hipMemcpy(q, hq.data(), nq * 2, hipMemcpyHostToDevice);
  hipMemcpy(k, hk.data(), nk * 2, hipMemcpyHostToDevice);
  hipMemcpy(v, hv.data(), nk * 2, hipMemcpyHostToDevice);
  const int tiles = (T + 63) / 64;
  PrefillParams p{};
  p.q = q; p.q_sb = (int64_t)T * Hq * d; p.q_sh = d; p.q_st = (int64_t)Hq * d;
  p.k = k; p.k_sb = (int64_t)Hkv * T * d; p.k_sh = (int64_t)T * d; p.k_st = d;
  p.v = v; p.v_sb = p.k_sb; p.v_sh = p.k_sh; p.v_st = d;
  p.o = o; p.o_sb = p.q_sb; p.o_sh = d; p.o_st = p.q_st;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = T; p.S = T; p.W = 0; p.q_pos0 = 0;
  p.scale_log2 = kLog2e / sqrtf((float)d);
  // same grid as launch_prefill<128>
  p.hp = 4;
  p.nqb = (T + 31) / 32;
  p.nblocks = p.nqb * (Hq / 4) * B;
  const size_t ns = (size_t)p.nblocks * 4 * tiles * 8;
  unsigned long long* st;
  hipMalloc(&st, ns * 8);
  hipMemset(st, 0, ns * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_tiles), &tiles, sizeof(int));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(prefill_kernel<128>, dim3(p.nblocks), dim3(256), 0, 0, p);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(ns);
  hipMemcpy(h.data(), st, ns * 8, hipMemcpyDeviceToHost);
  const char* names[4] = {"QK", "SM", "PV", "BAR"};
  std::vector<double> ph[4];
  std::vector<double> idle;
  for (size_t w = 0; w < (size_t)p.nblocks * 4; ++w)
    for (int t = 0; t < tiles; ++t) {
      const unsigned long long* s = &h[(w * tiles + t) * 8];
      if (!s[0] || !s[4]) continue;
      if (s[1] && s[2] && s[3]) {
        ph[0].push_back((double)(s[1] - s[0]));
        ph[1].push_back((double)(s[2] - s[1]));
        ph[2].push_back((double)(s[3] - s[2]));
        ph[3].push_back((double)(s[4] - s[3]));
      } else {
        idle.push_back((double)(s[4] - s[0]));
      }
    }
  printf("B=%d T=%d: %zu computed tiles (wave-tiles), %zu skipped\n", B, T, ph[0].size(), idle.size());
  double tot = 0;
  for (int k2 = 0; k2 < 4; ++k2) {
    auto& x = ph[k2];
    double mean = 0;
    for (double y : x) mean += y;
    mean /= std::max<size_t>(1, x.size());
    std::sort(x.begin(), x.end());
    tot += mean;
    printf("  %-4s mean %8.1f  median %8.1f  p90 %8.1f cycles\n", names[k2], mean, x.empty() ? 0 : x[x.size() / 2],
           x.empty() ? 0 : x[x.size() * 9 / 10]);
  }
  printf("  tile mean %.1f cycles (32 MFMA = 1024 issue-cycles per wave; 2 waves share a SIMD)\n", tot);
  return 0;
}
