// Does the MFMA shape change what an attention-shaped step delivers on MI355X?  (MI355X_MICROARCH.md 'DVFS give-back'
// item 7: bare bf16 loops on random data ran 1.12-1.15x the FLOP/s with v_mfma_f32_16x16x32_bf16 as with 32x32x16 at
// about equal cycles per FLOP, because the chip holds a higher clock.)  This probe runs the same per-wave step as the
// prefill kernels — S^T = K.Q^T for 64 keys x 32 query rows x d 128, the exponentials / row sums / bf16 packing of
// those 2048 scores (32 per lane), O^T += V^T.P^T — with either MFMA shape, operands re-read from LDS by ds_read_b128,
// two 4-wave workgroups per CU, one barrier per step, random bf16 data; it prints TFLOP/s and the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_shape_probe.hip -o tools/mfma_shape_probe && tools/mfma_shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } \
  } while (0)

constexpr int LDS = 64 * 1024;

template <int SHAPE>   // 32: v_mfma_f32_32x32x16_bf16, 16: v_mfma_f32_16x16x32_bf16
__global__ __launch_bounds__(256, 2) void step_probe(const bf16x8* __restrict__ src, float* __restrict__ out, int steps,
                                                     unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) bf16x8 sm[LDS / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < LDS / 16; i += 256) sm[i] = src[(blockIdx.x * 97 + i) % (1 << 16)];
  bf16x8 q[8];
  for (int i = 0; i < 8; ++i) q[i] = src[(blockIdx.x * 131 + tid * 8 + i) % (1 << 16)];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float m = 0.f, l = 0.f;
  const float c = 0.0883883f * 1.442695f;
  if constexpr (SHAPE == 32) {
    f32x16 o[4] = {};
    for (int st = 0; st < steps; ++st) {
      const int base = (st & 7) * 512 + (tid >> 6) * 64;
      f32x16 s[2] = {};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sm[(base + lane + 64 * (ks * 2 + kb)) & 4095], q[ks], s[kb], 0, 0, 0);
      float mx = s[0][0];
#pragma unroll
      for (int e = 1; e < 32; ++e) mx = fmaxf(mx, s[e >> 4][e & 15]);
      const float mn = fmaxf(m, mx * c);
      const float al = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      bf16x8 pk[4];
      float rs = 0.f;
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[e >> 4][e & 15], c, -m));
        rs += p;
        pk[e >> 3][e & 7] = (__bf16)p;
      }
      l = l * al + rs;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= al;
#pragma unroll
      for (int ss = 0; ss < 4; ++ss)
#pragma unroll
        for (int db = 0; db < 4; ++db)
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sm[(base + 2048 + lane + 64 * (ss * 4 + db)) & 4095], pk[ss], o[db], 0, 0, 0);
      __syncthreads();
    }
    float acc = l;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc += o[db][e];
    out[blockIdx.x * 256 + tid] = acc;
  } else {
    f32x4 o[8][2] = {};
    for (int st = 0; st < steps; ++st) {
      const int base = (st & 7) * 512 + (tid >> 6) * 64;
      f32x4 s[4][2] = {};
#pragma unroll
      for (int ds = 0; ds < 4; ++ds)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const bf16x8 a = sm[(base + lane + 64 * (ds * 4 + kb)) & 4095];
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) s[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, q[ds * 2 + qb], s[kb][qb], 0, 0, 0);
        }
      float mx = s[0][0][0];
#pragma unroll
      for (int e = 1; e < 32; ++e) mx = fmaxf(mx, s[(e >> 2) & 3][e >> 4][e & 3]);
      const float mn = fmaxf(m, mx * c);
      const float al = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      bf16x8 pk[2][2];
      float rs = 0.f;
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[(e >> 2) & 3][e >> 4][e & 3], c, -m));
        rs += p;
        pk[(e >> 3) & 1][e >> 4][e & 7] = (__bf16)p;
      }
      l = l * al + rs;
#pragma unroll
      for (int db = 0; db < 8; ++db) { o[db][0] *= al; o[db][1] *= al; }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int db = 0; db < 8; ++db) {
          const bf16x8 a = sm[(base + 2048 + lane + 64 * (ks * 8 + db)) & 4095];
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pk[ks][qb], o[db][qb], 0, 0, 0);
        }
      __syncthreads();
    }
    float acc = l;
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += o[db][0][e] + o[db][1][e];
    out[blockIdx.x * 256 + tid] = acc;
  }
  if (tid == 0 && clk) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 400;
  const int grid = 512 * 4;
  std::vector<__bf16> h((size_t)8 << 16);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : h) x = (__bf16)nd(rng);
  bf16x8* src;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMalloc(&out, (size_t)grid * 256 * 4));
  CK(hipMalloc(&clk, (size_t)grid * 16));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const double flop = 2.0 * 2 * 64 * 32 * 128 * 4.0 * steps * grid;   // 4 waves per block
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 3; ++round)
    for (int shape : {32, 16}) {
      auto run = [&](unsigned long long* c) {
        if (shape == 32) hipLaunchKernelGGL(step_probe<32>, dim3(grid), dim3(256), 0, 0, src, out, steps, c);
        else hipLaunchKernelGGL(step_probe<16>, dim3(grid), dim3(256), 0, 0, src, out, steps, c);
      };
      // ~2 s of back-to-back launches, then the timed launches and one stamped launch
      float ms = 0.f;
      CK(hipEventRecord(e0));
      int n = 0;
      while (ms < 2000.f) {
        for (int i = 0; i < 8; ++i, ++n) run(nullptr);
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
      printf("round %d shape %dx%d: %.3f ms/launch, %.1f TFLOP/s, in-kernel clock %.3f GHz, %.0f cycles per wave-step\n",
             round, shape, shape, ms / 10, flop / (ms / 10) / 1e9, cyc / tick * 0.1, cyc / grid / steps);
      fflush(stdout);
    }
  return 0;
}
