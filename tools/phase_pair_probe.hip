// Does the phase alignment of the two waves that share a SIMD bound the prefill attention step?  The x32 kernel's
// step is two phases of 16 v_mfma_f32_32x32x16_bf16 each: A(t) = S(t) = K(t).Q^T beside the 32 exponentials / row
// sums / bf16 packs of tile t-1 (issue-heavy), B(t) = O += V(t-1)^T.P(t-1)^T beside the row max and exponent arguments
// of S(t) (matrix-heavy), one barrier per step.  Its two waves per SIMD come from two independent workgroups, so
// nothing decides whether partners sit in the same phase (A beside A: both issue-bound) or in opposite phases.  This
// probe runs that step, compiler-scheduled, operands from LDS, random bf16 data, in three arrangements:
//   mode 0: 4-wave workgroups, two per CU (x32's arrangement: partner phases uncontrolled)
//   mode 1: 8-wave workgroups, one per CU, waves w and w + 4 share a SIMD, both halves A,B | A,B | ... (in phase)
//   mode 2: the same, waves 4-7 rotated by one phase: A(0) | B(0),A(1) | B(1),A(2) | ... (opposite phases)
// and prints TFLOP/s, the in-kernel clock and cycles per wave-step.  Timing probe only: its outputs are not checked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/phase_pair_probe.hip -o tools/phase_pair_probe && tools/phase_pair_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
  } while (0)

constexpr int LDS = 64 * 1024;

struct WaveState {
  f32x16 s[2];      // S(t)
  float x[32];      // exponent arguments of the pending tile
  bf16x8 pk[4];     // P of the tile awaiting PV
  f32x16 o[4];
  float m, l, alpha;
};

__device__ __forceinline__ void phase_a(WaveState& w, const bf16x8* sm, int base, int lane, const bf16x8 (&q)[8]) {
  w.s[0] = f32x16{};
  w.s[1] = f32x16{};
  float rs = 0.f;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      w.s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sm[(base + lane + 64 * (ks * 2 + kb)) & 4095], q[ks], w.s[kb], 0,
                                                         0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // 4 of the pending tile's 32 exponentials per QK MFMA pair
      const int e = 4 * ks + j;
      const float p = __builtin_amdgcn_exp2f(w.x[e]);
      rs += p;
      w.pk[e >> 3][e & 7] = (__bf16)p;
    }
  }
  w.l = w.l * w.alpha + rs;
}

__device__ __forceinline__ void phase_b(WaveState& w, const bf16x8* sm, int base, int lane) {
  float mx = w.s[0][0];
  const float c = 0.0883883f * 1.442695f;
#pragma unroll
  for (int ss = 0; ss < 4; ++ss) {
#pragma unroll
    for (int db = 0; db < 4; ++db)
      w.o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sm[(base + 2048 + lane + 64 * (ss * 4 + db)) & 4095], w.pk[ss],
                                                         w.o[db], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = 8 * ss + j;
      mx = fmaxf(mx, w.s[e >> 4][e & 15]);
    }
  }
  const float mn = fmaxf(w.m, mx * c);
  w.alpha = __builtin_amdgcn_exp2f(w.m - mn);
  w.m = mn;
#pragma unroll
  for (int e = 0; e < 32; ++e) w.x[e] = fmaf(w.s[e >> 4][e & 15], c, -mn);
}

template <int MODE>
__global__ __launch_bounds__(MODE == 0 ? 256 : 512, MODE == 0 ? 2 : 1) void pair_probe(
    const bf16x8* __restrict__ src, float* __restrict__ out, int steps, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) bf16x8 sm[LDS / 16];
  constexpr int NT = MODE == 0 ? 256 : 512;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < LDS / 16; i += NT) sm[i] = src[(blockIdx.x * 97 + i) % (1 << 16)];
  bf16x8 q[8];
  for (int i = 0; i < 8; ++i) q[i] = src[(blockIdx.x * 131 + tid * 8 + i) % (1 << 16)];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  WaveState w;
  w.m = 0.f;
  w.l = 0.f;
  w.alpha = 1.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) w.x[e] = -1.f;
#pragma unroll
  for (int db = 0; db < 4; ++db) w.o[db] = f32x16{};
#pragma unroll
  for (int i = 0; i < 4; ++i) w.pk[i] = bf16x8{};
  // rotated half: the barrier after phase A instead of after B (one code path, wave-uniform branches): between two
  // barriers the other half runs A(t+1), B(t+1) while this one runs B(t), A(t+1)
  const bool rotated = MODE == 2 && __builtin_amdgcn_readfirstlane(wave) >= 4;
  for (int st = 0; st < steps; ++st) {
    const int base = (st & 7) * 512 + (wave & 3) * 64;
    phase_a(w, sm, base, lane, q);
    __builtin_amdgcn_sched_barrier(0);
    if (rotated) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    phase_b(w, sm, base, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (!rotated) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }
  float acc = w.l;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc += w.o[db][e];
  out[blockIdx.x * NT + tid] = acc;
  if (tid == 0 && clk) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 400;
  std::vector<__bf16> h((size_t)8 << 16);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : h) x = (__bf16)nd(rng);
  bf16x8* src;
  float* out;
  unsigned long long* clk;
  const int waves_total = 2048 * 4;   // the same wave count in every mode
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMalloc(&out, (size_t)waves_total * 64 * 4));
  CK(hipMalloc(&clk, (size_t)waves_total * 16));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const double flop = 2.0 * 2 * 64 * 32 * 128 * (double)waves_total * steps;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 3; ++round)
    for (int mode : {0, 1, 2}) {
      const int grid = mode == 0 ? waves_total / 4 : waves_total / 8;
      auto run = [&](unsigned long long* c) {
        if (mode == 0) hipLaunchKernelGGL(pair_probe<0>, dim3(grid), dim3(256), 0, 0, src, out, steps, c);
        else if (mode == 1) hipLaunchKernelGGL(pair_probe<1>, dim3(grid), dim3(512), 0, 0, src, out, steps, c);
        else hipLaunchKernelGGL(pair_probe<2>, dim3(grid), dim3(512), 0, 0, src, out, steps, c);
      };
      float ms = 0.f;
      CK(hipEventRecord(e0));
      while (ms < 1500.f) {
        for (int i = 0; i < 8; ++i) run(nullptr);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
      }
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) run(nullptr);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      run(clk);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> hc((size_t)grid * 2);
      CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, tick = 0;
      for (int b = 0; b < grid; ++b) { cyc += hc[2 * b]; tick += hc[2 * b + 1]; }
      printf("round %d mode %d: %.3f ms/launch, %.1f TFLOP/s, in-kernel clock %.3f GHz, %.0f cycles per wave-step\n",
             round, mode, ms / 10, flop / (ms / 10) / 1e9, cyc / tick * 0.1, cyc / grid / steps);
      fflush(stdout);
    }
  return 0;
}
