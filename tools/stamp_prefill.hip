// Diagnostic: where a prefill_kernel tile's cycles go (s_memtime stamps, MI355X guide §7 idiom).
// Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCRAM_STAMPS tools/stamp_prefill.hip -o tools/stamp_prefill
// Run:    tools/stamp_prefill B T        (Llama-3 GQA 32/8, d 128, random bf16 q/k/v)
// Prints the mean shader cycles per tile phase over every (workgroup, wave, computed tile):
//   QK   loop top -> row max known (K reads + 16 MFMAs + max)     SM   -> exponentials + row sum
//   PV   -> rescale + P pack + V^T reads + 16 MFMAs issued       DMA  -> next tile's LDS-DMA landed
//   BAR  -> bias write + barrier (skew between the workgroup's waves)
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
  PrefillParams p{};
  p.q = q; p.q_sb = (int64_t)T * Hq * d; p.q_sh = d; p.q_st = (int64_t)Hq * d;
  p.k = k; p.k_sb = (int64_t)Hkv * T * d; p.k_sh = (int64_t)T * d; p.k_st = d;
  p.v = v; p.v_sb = p.k_sb; p.v_sh = p.k_sh; p.v_st = d;
  p.o = o; p.o_sb = p.q_sb; p.o_sh = d; p.o_st = p.q_st;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = T; p.S = T; p.W = 0; p.q_pos0 = 0;
  p.scale_log2 = kLog2e / sqrtf((float)d);
  p.hp = 4;                                      // same grid as launch_prefill<128>
  p.nqb = (T + 31) / 32;
  p.nblocks = p.nqb * (Hq / 4) * B;
  const size_t ns = (size_t)p.nblocks * 4 * 8;
  unsigned long long* st;
  hipMalloc(&st, ns * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((prefill_kernel<__bf16, 128, 64, 2>), dim3(p.nblocks), dim3(256), 0, 0, p);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(ns);
  hipMemcpy(h.data(), st, ns * 8, hipMemcpyDeviceToHost);
  const char* names[5] = {"QK", "SM", "PV", "DMA", "BAR"};
  double sum[5] = {}, tiles = 0;
  for (size_t w = 0; w < (size_t)p.nblocks * 4; ++w) {
    for (int k2 = 0; k2 < 5; ++k2) sum[k2] += (double)h[w * 8 + k2];
    tiles += (double)h[w * 8 + 6];
  }
  printf("B=%d T=%d: %.0f computed wave-tiles\n", B, T, tiles);
  double tot = 0;
  for (int k2 = 0; k2 < 5; ++k2) {
    tot += sum[k2] / tiles;
    printf("  %-4s mean %8.1f cycles\n", names[k2], sum[k2] / tiles);
  }
  printf("  tile mean %.1f cycles (32 MFMA x 32 cycles = 1024 per wave; two waves share a SIMD)\n", tot);
  return 0;
}
